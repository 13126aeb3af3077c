"""Stratum V2 client session against scripted loopback pools: handshake outcomes, the job / prev-hash activation
state machine, SetTarget re-issue, submit sequencing and verdicts, reconnect / close handling, malformed input.

Mirrors the reference's engine run_test.go fakePool + stratumv2 dialer_test.go cases (TestEngine_Handshake*,
TestEngine_SubmittedShareEchoesJobVersion, future-job / prev-hash activation, TestDialer_*), driven through the
production V2Dialer over real sockets.
"""
from __future__ import annotations

import asyncio
import struct

import pytest

from otedama_amd.poolproto import base as B
from otedama_amd.poolproto import stratumv2 as V2
from otedama_amd.stratum import frame as F
from otedama_amd.stratum import messages as M

PREV = bytes(range(32))
ROOT = bytes(range(32, 64))
T1 = b"\x00" * 28 + b"\xff" * 4
T2 = b"\x00" * 29 + b"\xff" * 3


class Pool:
    """One-connection scripted SV2 pool. ``script(pool)`` runs after the handshake and can send / expect frames."""

    def __init__(self, setup_reply=None, open_reply=None, script=None, dialect=M.REFERENCE):
        self.setup_reply = setup_reply or M.SetupConnectionSuccess(2, M.FLAG_REQUIRES_VERSION_ROLLING)
        self.open_reply = open_reply or M.OpenMiningChannelSuccess(1, 7, T1, b"\x01\x02", 4)
        self.script = script
        self.dialect = dialect
        self.got: list[M.Message] = []
        self.done = asyncio.Event()

    async def start(self):
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return self.server.sockets[0].getsockname()[1]

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()

    async def send(self, m):
        self.w.write(M.encode_message(m, self.dialect))
        await self.w.drain()

    async def recv(self):
        f = await asyncio.wait_for(F.read_frame_async(self.r), 5)
        m = M.dispatch_frame(f, self.dialect)
        self.got.append(m)
        return m

    async def _handle(self, r, w):
        self.r, self.w = r, w
        try:
            await self.recv()  # SetupConnection
            await self.send(self.setup_reply)
            if isinstance(self.setup_reply, M.SetupConnectionSuccess):
                await self.recv()  # OpenMiningChannel
                await self.send(self.open_reply)
                if self.script:
                    await self.script(self)
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.TimeoutError):
            pass
        finally:
            self.done.set()


async def _dial(pool: Pool, **creds_kw):
    port = await pool.start()
    creds = B.Credentials(user="bc1q.rig", **creds_kw)
    return await V2.V2Dialer(False, dialect=pool.dialect).dial(f"stratum+v2://127.0.0.1:{port}", creds, timeout=5)


async def _next_job(s, timeout=5):
    return await asyncio.wait_for(s.jobs.get(), timeout)


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 20))


# ------------------------------------------------------------------ handshake
def test_handshake_sends_reference_setup_and_open_channel():
    async def go():
        pool = Pool()
        s = await _dial(pool, nominal_hashrate=18.8e9)
        setup, open_ = pool.got[:2]
        assert isinstance(setup, M.SetupConnection) and setup.min_version == setup.max_version == 2
        assert setup.flags == M.FLAG_REQUIRES_VERSION_ROLLING and setup.endpoint.startswith("127.0.0.1:")
        assert (setup.vendor, setup.hardware_version, setup.firmware, setup.device_id) == \
            ("Otedama", "v3.0.0", "main", "gfx950")
        assert isinstance(open_, M.OpenMiningChannel) and open_.req_id == 1 and open_.user == "bc1q.rig"
        assert open_.nominal_hashrate == pytest.approx(18.8e9, rel=1e-6)
        assert s.channel_id == 7 and s.share_target == T1 and s.extranonce_prefix == b"\x01\x02"
        assert s.version_mask == V2.BIP320_MASK and s.protocol == B.ProtocolID.STRATUM_V2
        await s.close()
        await pool.stop()
    run(go())


def test_version_rolling_needs_both_sides():
    async def go():
        pool = Pool(setup_reply=M.SetupConnectionSuccess(2, 0))
        s = await _dial(pool)
        assert s.version_mask == 0
        await s.close()
        await pool.stop()
        pool = Pool()
        s = await _dial(pool, version_rolling=False)
        assert pool.got[0].flags == 0 and s.version_mask == 0
        await s.close()
        await pool.stop()
    run(go())


def test_setup_connection_error_is_fatal():
    async def go():
        pool = Pool(setup_reply=M.SetupConnectionError(0, "unsupported-protocol"))
        with pytest.raises(B.FatalPoolError, match="unsupported-protocol"):
            await _dial(pool)
        await pool.stop()
    run(go())


@pytest.mark.parametrize("reply,exc", [(M.OpenMiningChannelError(1, "unknown-user"), B.HandshakeFailed),
                                       (M.SetTarget(1, T1), B.HandshakeFailed)])
def test_open_channel_failures(reply, exc):
    async def go():
        pool = Pool(open_reply=reply)
        with pytest.raises(exc):
            await _dial(pool)
        await pool.stop()
    run(go())


def test_unexpected_setup_reply_is_handshake_failure():
    async def go():
        pool = Pool(setup_reply=M.Reconnect("x", 1))
        with pytest.raises(B.HandshakeFailed):
            await _dial(pool)
        await pool.stop()
    run(go())


def test_spec_dialect_handshake():
    async def go():
        pool = Pool(dialect=M.SPEC, open_reply=M.OpenMiningChannelSuccess(1, 9, T1, b"\x05", group_channel_id=3))
        s = await _dial(pool)
        assert pool.got[0].endpoint_port > 0 and s.channel_id == 9 and s.extranonce_prefix == b"\x05"
        await s.close()
        await pool.stop()
    run(go())


# ------------------------------------------------------------------ activation state machine
def _script(*steps):
    async def script(pool):
        for st in steps:
            if st == "recv":
                await pool.recv()
            elif isinstance(st, float):
                await asyncio.sleep(st)
            else:
                await pool.send(st)
        await asyncio.sleep(0.3)
    return script


def test_future_job_activates_on_set_new_prev_hash():
    async def go():
        pool = Pool(script=_script(M.NewMiningJob(7, 100, False, 0, 0x20000000, ROOT),
                                   M.SetNewPrevHash(7, 100, PREV, 1_700_000_000, 0x1703A30C)))
        s = await _dial(pool)
        j = await _next_job(s)
        assert (j.job_id, j.version, j.prev_hash, j.merkle_root, j.ntime, j.nbits) == \
            ("100", 0x20000000, PREV, ROOT, 1_700_000_000, 0x1703A30C)
        assert j.clean_jobs and j.target == T1 and j.channel_id == 7 and j.version_mask == V2.BIP320_MASK
        assert s.jobs.empty()  # the future job was not mined before its prev-hash
        await s.close()
        await pool.stop()
    run(go())


def test_job_with_min_ntime_after_prev_hash_is_active_immediately():
    async def go():
        pool = Pool(script=_script(M.NewMiningJob(7, 1, False, 0, 0x20000000, ROOT),
                                   M.SetNewPrevHash(7, 1, PREV, 100, 0x1d00ffff),
                                   M.NewMiningJob(7, 2, True, 150, 0x20000004, ROOT[::-1])))
        s = await _dial(pool)
        a = await _next_job(s)
        b = await _next_job(s)
        assert (a.job_id, b.job_id) == ("1", "2") and b.ntime == 150 and b.version == 0x20000004
        assert b.prev_hash == PREV and b.merkle_root == ROOT[::-1]
        await s.close()
        await pool.stop()
    run(go())


def test_job_with_min_ntime_before_any_prev_hash_is_held():
    async def go():
        pool = Pool(script=_script(M.NewMiningJob(7, 5, True, 500, 0x20000000, ROOT), 0.1,
                                   M.SetNewPrevHash(7, 5, PREV, 400, 0x1d00ffff)))
        s = await _dial(pool)
        j = await _next_job(s)
        assert j.job_id == "5" and j.ntime == 500  # max(prev-hash min_ntime, job min_ntime)
        await s.close()
        await pool.stop()
    run(go())


def test_prev_hash_drops_every_other_job_and_unknown_job_pauses():
    async def go():
        pool = Pool(script=_script(M.NewMiningJob(7, 1, False, 0, 1, ROOT), M.NewMiningJob(7, 2, False, 0, 2, ROOT),
                                   M.SetNewPrevHash(7, 2, PREV, 10, 0x1d00ffff), 0.05,
                                   M.SetNewPrevHash(7, 1, PREV[::-1], 20, 0x1d00ffff)))
        s = await _dial(pool)
        j = await _next_job(s)
        assert j.job_id == "2"
        paused = await _next_job(s)
        assert paused is None  # job 1 was dropped by the first prev-hash: nothing valid to mine
        assert s._active is None and s._jobs == {}
        await s.close()
        await pool.stop()
    run(go())


def test_set_target_reissues_the_active_job_with_the_new_target():
    async def go():
        pool = Pool(script=_script(M.NewMiningJob(7, 1, False, 0, 1, ROOT), M.SetNewPrevHash(7, 1, PREV, 10, 0x1d00ffff),
                                   0.05, M.SetTarget(7, T2)))
        s = await _dial(pool)
        a = await _next_job(s)
        b = await _next_job(s)
        assert a.target == T1 and b.target == T2 and b.job_id == a.job_id and b.ntime == a.ntime
        from otedama_amd.models.header import difficulty_from_target

        assert s.share_target == T2 and s.suggested_difficulty() == difficulty_from_target(T2)
        await s.close()
        await pool.stop()
    run(go())


def test_set_target_before_any_job_only_updates_the_channel_target():
    async def go():
        pool = Pool(script=_script(M.SetTarget(7, T2), M.NewMiningJob(7, 1, False, 0, 1, ROOT),
                                   M.SetNewPrevHash(7, 1, PREV, 10, 0x1d00ffff)))
        s = await _dial(pool)
        j = await _next_job(s)
        assert j.target == T2
        await s.close()
        await pool.stop()
    run(go())


# ------------------------------------------------------------------ submits
def test_submit_sequence_numbers_and_verdicts():
    async def script(pool):
        a = await pool.recv()
        b = await pool.recv()
        c = await pool.recv()
        assert [m.sequence_number for m in (a, b, c)] == [1, 2, 3]
        await pool.send(M.SubmitSharesError(7, 2, "difficulty-too-low"))
        await pool.send(M.SubmitSharesSuccess(7, 3, 2, 2))
        await asyncio.sleep(0.3)

    async def go():
        pool = Pool(script=script)
        s = await _dial(pool)
        subs = [B.ShareSubmission("100", 0xDEADBEEF + i, 0x60000000, 0x20000004) for i in range(3)]
        r = await asyncio.gather(*(s.submit(x, timeout=5) for x in subs))
        assert [x.accepted for x in r] == [True, False, True] and r[1].reason == "difficulty-too-low"
        assert all(x.latency_ms >= 0 for x in r)
        first = pool.got[2]
        assert isinstance(first, M.SubmitSharesStandard)
        assert (first.channel_id, first.job_id, first.nonce, first.ntime, first.nversion) == \
            (7, 100, 0xDEADBEEF, 0x60000000, 0x20000004)  # NVersion echo
        await s.close()
        await pool.stop()
    run(go())


def test_submit_with_a_non_numeric_job_id_is_rejected_locally():
    async def go():
        pool = Pool(script=_script(0.5))
        s = await _dial(pool)
        r = await s.submit(B.ShareSubmission("v1-job", 1, 2, 3))
        assert not r.accepted and "stale-job" in r.reason and len(pool.got) == 2
        await s.close()
        await pool.stop()
    run(go())


def test_submit_timeout_and_close_before_verdict():
    async def go():
        pool = Pool(script=_script("recv", "recv", 1.0))
        s = await _dial(pool)
        r = await s.submit(B.ShareSubmission("1", 1, 2, 3), timeout=0.2)
        assert not r.accepted and "timeout" in r.reason
        task = asyncio.ensure_future(s.submit(B.ShareSubmission("1", 2, 2, 3), timeout=5))
        await asyncio.sleep(0.1)
        await s.close()
        with pytest.raises(B.PoolProtoError, match="closed"):
            await task
        with pytest.raises(B.PoolProtoError, match="closed"):
            await s.submit(B.ShareSubmission("1", 3, 2, 3))
        await pool.stop()
    run(go())


def test_submit_map_is_bounded():
    async def go():
        pool = Pool(script=_script(60.0))  # the pool never answers while the test runs
        s = await _dial(pool)
        tasks = [asyncio.ensure_future(s.submit(B.ShareSubmission("1", i, 2, 3), timeout=60))
                 for i in range(V2.SUBMIT_MAP_CAP + 10)]
        for _ in range(600):  # every submit issued (a loaded host runs the tasks late)
            await asyncio.sleep(0.05)
            if s._seq >= V2.SUBMIT_MAP_CAP + 10:
                break
        await asyncio.sleep(0.05)
        assert len(s._pending) <= V2.SUBMIT_MAP_CAP
        dropped = [t.result() for t in tasks if t.done()]
        assert dropped and all("overflow" in r.reason for r in dropped)
        pending = [t for t in tasks if not t.done()]
        await s.close()
        # every submit still waiting ends with "closed": gathered, so no task's exception goes unretrieved
        results = await asyncio.gather(*pending, return_exceptions=True)
        # each ends on the close: "closed before verdict" while waiting for it, "Connection lost" while still
        # writing (a loaded host), or dropped by the map's bound meanwhile; none hangs, none is accepted
        bad = [r for r in results if not ((isinstance(r, B.PoolProtoError) and ("closed" in str(r)
                                                                               or "Connection lost" in str(r)))
                                           or (isinstance(r, B.ShareResult) and "overflow" in r.reason))]
        assert results and not bad, bad[:3]
        await pool.stop()
    run(go())


def test_extended_channel_submit_carries_the_extranonce():
    async def script(pool):
        await pool.send(M.NewExtendedMiningJob(7, 3, False, 0, 0x20000000, True, [ROOT], b"\x01" * 10, b"\x02" * 10))
        await pool.send(M.SetNewPrevHash(7, 3, PREV, 10, 0x1d00ffff))
        m = await pool.recv()
        assert isinstance(m, M.SubmitSharesExtended) and m.extranonce == b"\xaa\xbb\xcc\xdd"
        await pool.send(M.SubmitSharesSuccess(7, m.sequence_number, 1, 1))
        await asyncio.sleep(0.3)

    async def go():
        pool = Pool(open_reply=M.OpenExtendedMiningChannelSuccess(1, 7, T1, 4, b"\x09\x09"), script=script)
        s = await _dial(pool, extended_channel=True)
        assert isinstance(pool.got[1], M.OpenExtendedMiningChannel) and pool.got[1].min_extranonce_size == 4
        j = await _next_job(s)
        assert j.coinb1 == b"\x01" * 10 and j.extranonce1 == b"\x09\x09" and j.extranonce2_size == 4
        assert j.merkle_root is None and j.merkle_branches == [ROOT]
        r = await s.submit(B.ShareSubmission("3", 1, 10, 0x20000000, b"\xaa\xbb\xcc\xdd"))
        assert r.accepted
        await s.close()
        await pool.stop()
    run(go())


def test_set_extranonce_prefix_reissues_the_extended_job():
    async def script(pool):
        await pool.send(M.NewExtendedMiningJob(7, 3, False, 0, 0x20000000, True, [ROOT], b"\x01" * 10, b"\x02" * 10))
        await pool.send(M.SetNewPrevHash(7, 3, PREV, 10, 0x1d00ffff))
        await asyncio.sleep(0.1)
        await pool.send(M.SetExtranoncePrefix(99, b"\xee"))           # another channel: ignored
        await pool.send(M.SetExtranoncePrefix(7, b"\x0a\x0b\x0c"))
        await asyncio.sleep(0.3)

    async def go():
        pool = Pool(open_reply=M.OpenExtendedMiningChannelSuccess(1, 7, T1, 4, b"\x09\x09"), script=script)
        s = await _dial(pool, extended_channel=True)
        first = await _next_job(s)
        again = await _next_job(s)
        assert first.extranonce1 == b"\x09\x09"
        # total extranonce = 2 + 4 = 6 bytes; a 3-byte prefix leaves 3 rollable, and the re-issued job carries the
        # new prefix epoch in its id so a share found under the old prefix is dropped instead of being rejected
        assert again.job_id == "3~1" and again.clean_jobs and again.extranonce1 == b"\x0a\x0b\x0c"
        assert again.extranonce2_size == 3 and s.extranonce_size == 3
        assert s.extranonce_prefix == b"\x0a\x0b\x0c" and s.jobs.empty()
        n_sent = len(pool.got)
        r = await s.submit(B.ShareSubmission(first.job_id, 1, 10, 0x20000000, b"\xaa\xbb\xcc\xdd"))
        assert not r.accepted and "stale-prefix" in r.reason
        await asyncio.sleep(0.05)
        assert len(pool.got) == n_sent  # nothing went to the pool
        await s.close()
        await pool.stop()
    run(go())


def test_set_extranonce_prefix_leaving_no_rollable_bytes_closes_the_session():
    async def script(pool):
        await pool.send(M.NewExtendedMiningJob(7, 3, False, 0, 0x20000000, True, [ROOT], b"\x01" * 10, b"\x02" * 10))
        await pool.send(M.SetNewPrevHash(7, 3, PREV, 10, 0x1d00ffff))
        await asyncio.sleep(0.1)
        await pool.send(M.SetExtranoncePrefix(7, b"\x0a" * 6))  # 6 of 6 bytes: nothing left to roll
        await asyncio.sleep(0.5)

    async def go():
        pool = Pool(open_reply=M.OpenExtendedMiningChannelSuccess(1, 7, T1, 4, b"\x09\x09"), script=script)
        s = await _dial(pool, extended_channel=True)
        await _next_job(s)
        for _ in range(50):
            if s.closed:
                break
            await asyncio.sleep(0.02)
        assert s.closed and s.extranonce_prefix == b"\x09\x09"
        await pool.stop()
    run(go())


def test_set_extranonce_prefix_on_a_standard_channel_only_records_it():
    async def go():
        pool = Pool(script=_script(M.NewMiningJob(7, 3, False, 0, 0x20000000, ROOT), M.SetNewPrevHash(7, 3, PREV, 10,
                    0x1d00ffff), 0.1, M.SetExtranoncePrefix(7, b"\x05" * 8)))
        s = await _dial(pool)
        await _next_job(s)
        await asyncio.sleep(0.3)
        assert s.jobs.empty() and s.extranonce_prefix == b"\x05" * 8
        await s.close()
        await pool.stop()
    run(go())


@pytest.mark.parametrize("size", [0, 9])
def test_extended_channel_rejects_unsupported_extranonce_sizes(size):
    async def go():
        pool = Pool(open_reply=M.OpenExtendedMiningChannelSuccess(1, 7, T1, size, b""))
        with pytest.raises(B.HandshakeFailed, match="extranonce size"):
            await _dial(pool, extended_channel=True)
        await pool.stop()
    run(go())


# ------------------------------------------------------------------ session end
@pytest.mark.parametrize("msg", [M.Reconnect("evil.example", 3336), M.CloseChannel(7, "maintenance")])
def test_pool_initiated_reconnect_or_close_ends_the_session(msg):
    async def go():
        pool = Pool(script=_script(msg, 0.5))
        s = await _dial(pool)
        await asyncio.wait_for(s.wait_closed(), 5)
        if isinstance(msg, M.Reconnect):
            note = s.notices.get_nowait()
            assert "evil.example:3336" in note and "not followed" in note
        await pool.stop()
    run(go())


def test_oversized_frame_ends_the_session_cleanly():
    async def script(pool):
        pool.w.write(F.Header(0, 0x15, F.MAX_MESSAGE_LENGTH).encode())  # 16 MiB claim, no payload
        await pool.w.drain()
        await asyncio.sleep(0.5)

    async def go():
        pool = Pool(script=script)
        s = await _dial(pool)
        await asyncio.wait_for(s.wait_closed(), 5)
        assert s._task.done() and s._task.exception() is None
        await pool.stop()
    run(go())


def test_undecodable_message_ends_the_session_cleanly():
    async def script(pool):
        pool.w.write(F.Header(F.CHANNEL_MSG_BIT, M.MSG_SET_TARGET, 8).encode() + b"\x07\x00\x00\x00abcd")
        await pool.w.drain()
        await asyncio.sleep(0.5)

    async def go():
        pool = Pool(script=script)
        s = await _dial(pool)
        await asyncio.wait_for(s.wait_closed(), 5)
        assert s._task.exception() is None
        await pool.stop()
    run(go())


def test_unknown_message_types_are_ignored():
    async def script(pool):
        pool.w.write(F.encode_frame(F.Frame(F.Header(0, 0x70, 3), b"xyz")))
        await pool.w.drain()
        await pool.send(M.NewMiningJob(7, 1, False, 0, 1, ROOT))
        await pool.send(M.SetNewPrevHash(7, 1, PREV, 10, 0x1d00ffff))
        await asyncio.sleep(0.3)

    async def go():
        pool = Pool(script=script)
        s = await _dial(pool)
        assert (await _next_job(s)).job_id == "1" and not s.closed
        await s.close()
        await pool.stop()
    run(go())


def test_pool_disconnect_closes_the_session():
    async def go():
        pool = Pool(script=_script())
        s = await _dial(pool)
        await asyncio.wait_for(pool.done.wait(), 5)
        pool.w.close()
        await asyncio.wait_for(s.wait_closed(), 5)
        await pool.stop()
    run(go())


def test_dial_unreachable_pool():
    async def go():
        with pytest.raises(OSError):
            await V2.V2Dialer(False).dial("stratum+v2://127.0.0.1:1", B.Credentials(user="u"), timeout=2)
    run(go())


def test_dialer_registry_has_v2():
    assert isinstance(B.lookup(B.ProtocolID.STRATUM_V2), V2.V2Dialer)
    assert B.lookup(B.ProtocolID.STRATUM_V2_TLS).use_tls
    assert struct.calcsize("<I") == 4
