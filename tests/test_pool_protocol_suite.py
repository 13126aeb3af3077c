"""Local pool server, wire level: raw Stratum V1 JSON lines and raw SV2 frames against `PoolServer`.

[NO REFERENCE CODE] for the server side: these tests pin the protocol contract the pool offers the
reference client and ours — handshake answers, error codes and strings, job broadcast, share verdicts (the reject
strings land in the engine's taxonomy, engine/stats.go:263-277), vardiff re-targets — and that malformed input from
one miner is answered, never crashes the listener. Shares are mined on the CPU through the native scanner.
"""
import asyncio
import json
import struct
import time

import pytest

from otedama_amd.models.header import hash_to_int, sha256d
from otedama_amd.ops.native import require_native
from otedama_amd.pool.server import BIP320_MASK, EN1_SIZE, EN2_SIZE, PoolOptions, PoolServer
from otedama_amd.stratum import messages as M
from otedama_amd.stratum.frame import FrameReader

N = require_native()
ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


async def with_pool(body, **kw):
    kw.setdefault("initial_difficulty", 2e-5)
    pool = PoolServer(PoolOptions(payout_address=ADDR, job_interval=3600, block_interval=3600, **kw))
    await pool.start()
    try:
        return await body(pool)
    finally:
        await pool.stop()


def mine(pool, job_id, extranonce, version=None, ntime=None, want_valid=True):
    """(nonce, ntime, version, header) of a share for `job_id` (or a nonce that misses the share target)."""
    job = pool.jobs[job_id]
    version = job.version if version is None else version
    ntime = job.ntime if ntime is None else ntime
    target = pool.share_target(2e-5)
    hdr = pool.header_for(job, extranonce, version, ntime, 0)
    if want_valid:
        hits = N.cpu_scan_sha256d(hdr, target, 0, 1 << 20)
        assert hits, "no share in 2^20 nonces"
        return hits[0], ntime, version, hdr
    for n in range(1 << 16):
        if hash_to_int(sha256d(hdr[:76] + struct.pack("<I", n))) > hash_to_int(target):
            return n, ntime, version, hdr
    raise AssertionError("no miss found")


# ---------------------------------------------------------------------------------------------- raw V1 client

class V1Raw:
    def __init__(self, reader, writer):
        self.r, self.w = reader, writer
        self.next_id = 0
        self.notes: list[dict] = []

    @classmethod
    async def connect(cls, pool):
        h, p = pool.addr_v1.rsplit(":", 1)
        return cls(*await asyncio.open_connection(h, int(p)))

    async def send_raw(self, data: bytes):
        self.w.write(data)
        await self.w.drain()

    async def call(self, method, params, mid=None):
        self.next_id += 1
        mid = self.next_id if mid is None else mid
        await self.send_raw(json.dumps({"id": mid, "method": method, "params": params}).encode() + b"\n")
        while True:
            msg = await self.read()
            if msg.get("id") == mid and msg.get("method") is None:
                return msg
            self.notes.append(msg)

    async def read(self, timeout=5.0):
        return json.loads(await asyncio.wait_for(self.r.readline(), timeout))

    async def note(self, method, timeout=5.0):
        for i, n in enumerate(self.notes):
            if n.get("method") == method:
                return self.notes.pop(i)
        while True:
            msg = await self.read(timeout)
            if msg.get("method") == method:
                return msg
            self.notes.append(msg)

    async def handshake(self, user=ADDR + ".w1", mask="1fffe000"):
        if mask is not None:
            await self.call("mining.configure", [["version-rolling"], {"version-rolling.mask": mask}])
        sub = await self.call("mining.subscribe", ["test/1"])
        self.en1 = bytes.fromhex(sub["result"][1])
        auth = await self.call("mining.authorize", [user, "x"])
        assert auth["result"] is True
        return await self.note("mining.notify")

    def close(self):
        self.w.close()


def test_v1_configure_version_rolling_mask_negotiation():
    async def body(pool):
        c = await V1Raw.connect(pool)
        r = await c.call("mining.configure", [["version-rolling"], {"version-rolling.mask": "ffffffff"}])
        assert r["result"] == {"version-rolling": True, "version-rolling.mask": f"{BIP320_MASK:08x}"}
        r = await c.call("mining.configure", [["version-rolling"], {"version-rolling.mask": "00006000"}])
        assert r["result"]["version-rolling.mask"] == "00006000"
        r = await c.call("mining.configure", [["minimum-difficulty"], {}])
        assert r["result"] == {} and r["error"] is None
        c.close()
    run(with_pool(body))


def test_v1_configure_refused_when_pool_disallows_rolling():
    async def body(pool):
        c = await V1Raw.connect(pool)
        r = await c.call("mining.configure", [["version-rolling"], {"version-rolling.mask": "1fffe000"}])
        assert r["result"] == {}
        c.close()
    run(with_pool(body, allow_version_rolling=False))


def test_v1_malformed_configure_is_answered_and_connection_survives():
    async def body(pool):
        c = await V1Raw.connect(pool)
        r = await c.call("mining.configure", [["version-rolling"], {"version-rolling.mask": 12345}])
        assert r["error"][:2] == [20, "invalid parameters"]
        r = await c.call("mining.configure", [["version-rolling"], {"version-rolling.mask": "xyz"}])
        assert r["error"][0] == 20
        sub = await c.call("mining.subscribe", [])
        assert sub["error"] is None
        c.close()
    run(with_pool(body))


def test_v1_subscribe_result_shape_and_unique_extranonce1():
    async def body(pool):
        a, b = await V1Raw.connect(pool), await V1Raw.connect(pool)
        ra, rb = await a.call("mining.subscribe", ["x"]), await b.call("mining.subscribe", ["x"])
        subs, en1, size = ra["result"]
        assert subs[0][0] == "mining.notify" and len(bytes.fromhex(en1)) == EN1_SIZE and size == EN2_SIZE
        assert rb["result"][1] != en1
        a.close()
        b.close()
    run(with_pool(body))


@pytest.mark.parametrize("params", [[], [""], [42]])
def test_v1_authorize_requires_a_user(params):
    async def body(pool):
        c = await V1Raw.connect(pool)
        await c.call("mining.subscribe", [])
        r = await c.call("mining.authorize", params)
        assert r["result"] is False and r["error"][:2] == [24, "unauthorized worker"]
        c.close()
    run(with_pool(body))


def test_v1_authorize_sends_difficulty_then_current_job():
    async def body(pool):
        c = await V1Raw.connect(pool)
        await c.call("mining.subscribe", [])
        await c.call("mining.authorize", [ADDR, "x"])
        d = await c.note("mining.set_difficulty")
        n = await c.note("mining.notify")
        assert d["params"] == [2e-5]
        job = next(reversed(pool.jobs.values()))
        p = n["params"]
        assert p[0] == job.job_id and p[2] == job.coinb1.hex() and p[3] == job.coinb2.hex()
        assert p[5] == f"{job.version:08x}" and p[6] == f"{job.block.nbits:08x}" and p[8] is True
        c.close()
    run(with_pool(body))


def test_v1_submit_before_authorize_is_refused():
    async def body(pool):
        c = await V1Raw.connect(pool)
        await c.call("mining.subscribe", [])
        r = await c.call("mining.submit", ["w", "1", "00000000", "00000000", "00000000"])
        assert r["error"][:2] == [24, "unauthorized worker"]
        c.close()
    run(with_pool(body))


@pytest.mark.parametrize("params", [["w", "1"], ["w", "1", "zz", "00000000", "00000000"],
                                    ["w", "1", "0000", "00000000", "00000000"],
                                    ["w", "1", "00000000", "nothex", "00000000"], {"bad": 1}])
def test_v1_malformed_submit_is_answered(params):
    async def body(pool):
        c = await V1Raw.connect(pool)
        await c.handshake()
        r = await c.call("mining.submit", params)
        assert r["result"] is None and r["error"][0] == 20
        ping = await c.call("mining.extranonce.subscribe", [])
        assert ping["result"] is True  # connection still serving
        c.close()
    run(with_pool(body))


def test_v1_share_verdicts_and_error_codes():
    async def body(pool):
        c = await V1Raw.connect(pool)
        n = await c.handshake()
        jid, en2 = n["params"][0], bytes.fromhex("00000001")
        nonce, ntime, _, _ = mine(pool, jid, c.en1 + en2)
        args = ["w1", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}"]
        ok = await c.call("mining.submit", args)
        assert ok["result"] is True and ok["error"] is None
        dup = await c.call("mining.submit", args)
        assert dup["error"][:2] == [22, "duplicate-share"]
        stale = await c.call("mining.submit", ["w1", "ffff", en2.hex(), f"{ntime:08x}", f"{nonce:08x}"])
        assert stale["error"][:2] == [21, "stale-job"]
        miss, _, _, _ = mine(pool, jid, c.en1 + en2, want_valid=False)
        low = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime:08x}", f"{miss:08x}"])
        assert low["error"][:2] == [23, "low-difficulty-share"]
        old = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime - 1:08x}", f"{nonce:08x}"])
        assert old["error"][:2] == [20, "invalid-ntime"]
        future = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{int(time.time()) + 3 * 3600:08x}",
                                                f"{nonce:08x}"])
        assert future["error"][:2] == [20, "invalid-ntime"]
        assert pool.accepted == 1 and pool.reject_reasons == {"duplicate-share": 1, "stale-job": 1,
                                                              "low-difficulty-share": 1, "invalid-ntime": 2}
        c.close()
    run(with_pool(body))


def test_v1_version_rolling_share_and_out_of_mask_bits():
    async def body(pool):
        c = await V1Raw.connect(pool)
        n = await c.handshake()
        jid, en2 = n["params"][0], bytes.fromhex("00000002")
        job = pool.jobs[jid]
        rolled = (job.version & ~BIP320_MASK) | 0x00006000
        nonce, ntime, _, _ = mine(pool, jid, c.en1 + en2, version=rolled)
        ok = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}", "00006000"])
        assert ok["result"] is True
        bad = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}", "80006000"])
        assert bad["error"][:2] == [20, "invalid-version-bits"]
        c.close()
    run(with_pool(body))


def test_v1_rolling_without_negotiation_is_rejected():
    async def body(pool):
        c = await V1Raw.connect(pool)
        n = await c.handshake(mask=None)
        jid, en2 = n["params"][0], bytes(4)
        r = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{pool.jobs[jid].ntime:08x}", "00000000",
                                           "00002000"])
        assert r["error"][1] == "invalid-version-bits"
        c.close()
    run(with_pool(body))


def test_v1_unknown_method_and_garbage_lines():
    async def body(pool):
        c = await V1Raw.connect(pool)
        await c.send_raw(b"not json\n[1,2]\n\"str\"\n\xff\xfe\n")
        await c.send_raw(json.dumps({"id": None, "method": "mining.suggest_difficulty", "params": [8]}).encode()
                         + b"\n")  # notification: no answer
        r = await c.call("mining.get_transactions", ["1"])
        assert r["error"][0] == 20 and "unknown method" in r["error"][1]
        c.close()
    run(with_pool(body))


def test_v1_job_broadcast_only_to_authorized_and_new_block_stales_old_jobs():
    async def body(pool):
        authed, idle = await V1Raw.connect(pool), await V1Raw.connect(pool)
        first = await authed.handshake()
        await idle.call("mining.subscribe", [])
        j = pool.new_job(clean=False)
        n = await authed.note("mining.notify")
        assert n["params"][0] == j.job_id and n["params"][8] is False
        with pytest.raises(asyncio.TimeoutError):
            await idle.read(timeout=0.3)
        pool.new_block()
        n2 = await authed.note("mining.notify")
        assert n2["params"][8] is True and n2["params"][1] != first["params"][1]   # new prevhash
        en2 = bytes(4)
        r = await authed.call("mining.submit", ["w1", first["params"][0], en2.hex(), first["params"][7], "00000000"])
        assert r["error"][1] == "stale-job"
        authed.close()
        idle.close()
    run(with_pool(body))


def test_v1_vardiff_retarget_sends_set_difficulty():
    async def body(pool):
        c = await V1Raw.connect(pool)
        n = await c.handshake()
        await c.note("mining.set_difficulty")
        jid = n["params"][0]
        for i in range(64):
            en2 = struct.pack(">I", 100 + i)
            nonce, ntime, _, _ = mine(pool, jid, c.en1 + en2)
            r = await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}"])
            assert r["result"] is True, r
            if any(x.get("method") == "mining.set_difficulty" for x in c.notes):
                break
        d = await c.note("mining.set_difficulty")
        assert d["params"][0] > 2e-5   # shares arrived far faster than the target interval
        c.close()
    run(with_pool(body, retarget_seconds=0.0, target_share_seconds=60.0))


# ---------------------------------------------------------------------------------------------- raw SV2 client

class V2Raw:
    def __init__(self, reader, writer, dialect=M.REFERENCE):
        self.r, self.w = reader, writer
        self.frames = FrameReader(reader)
        self.dialect = dialect

    @classmethod
    async def connect(cls, pool):
        h, p = pool.addr_sv2.rsplit(":", 1)
        return cls(*await asyncio.open_connection(h, int(p)))

    async def send(self, msg):
        self.w.write(M.encode_message(msg, self.dialect))
        await self.w.drain()

    async def recv(self, timeout=5.0):
        return M.dispatch_frame(await asyncio.wait_for(self.frames.read_frame(), timeout), self.dialect)

    async def expect(self, cls, timeout=5.0):
        while True:
            m = await self.recv(timeout)
            if isinstance(m, cls):
                return m

    async def setup(self, flags=M.FLAG_REQUIRES_VERSION_ROLLING):
        await self.send(M.SetupConnection(flags=flags, vendor="t"))
        return await self.recv()

    async def open(self, user=ADDR, hashrate=0.0, extended=False, min_en=0):
        if extended:
            await self.send(M.OpenExtendedMiningChannel(req_id=7, user=user, nominal_hashrate=hashrate,
                                                        min_extranonce_size=min_en))
        else:
            await self.send(M.OpenMiningChannel(req_id=7, user=user, nominal_hashrate=hashrate))
        return await self.expect((M.OpenMiningChannelSuccess, M.OpenExtendedMiningChannelSuccess,
                                  M.OpenMiningChannelError))

    def close(self):
        self.w.close()


def test_v2_setup_connection_success_echoes_version_rolling():
    async def body(pool):
        c = await V2Raw.connect(pool)
        r = await c.setup()
        assert isinstance(r, M.SetupConnectionSuccess) and r.used_version == 2
        assert r.flags == M.FLAG_REQUIRES_VERSION_ROLLING
        c2 = await V2Raw.connect(pool)
        r2 = await c2.setup(flags=0)
        assert r2.flags == 0
        c.close()
        c2.close()
    run(with_pool(body))


def test_v2_version_rolling_refused_when_pool_disallows():
    async def body(pool):
        c = await V2Raw.connect(pool)
        r = await c.setup()
        assert isinstance(r, M.SetupConnectionSuccess) and r.flags == 0
        c.close()
    run(with_pool(body, allow_version_rolling=False))


@pytest.mark.parametrize("kw,err", [({"min_version": 3, "max_version": 4}, "unsupported-protocol-version"),
                                    ({"min_version": 1, "max_version": 1}, "unsupported-protocol-version")])
def test_v2_setup_connection_error(kw, err):
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.send(M.SetupConnection(**kw))
        r = await c.recv()
        assert isinstance(r, M.SetupConnectionError) and err in r.error
        c.close()
    run(with_pool(body))


def test_v2_open_channel_before_setup_or_without_user():
    async def body(pool):
        c = await V2Raw.connect(pool)
        r = await c.open()
        assert isinstance(r, M.OpenMiningChannelError) and r.error == "setup-required" and r.req_id == 7
        await c.setup()
        r = await c.open(user="")
        assert isinstance(r, M.OpenMiningChannelError) and r.error == "unknown-user"
        c.close()
    run(with_pool(body))


def test_v2_standard_channel_open_sends_target_prefix_and_future_job():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        ok = await c.open()
        assert isinstance(ok, M.OpenMiningChannelSuccess) and ok.req_id == 7 and ok.channel_id >= 1
        assert len(ok.extranonce) == EN1_SIZE + EN2_SIZE
        assert ok.target == pool.share_target(2e-5)
        job = await c.expect(M.NewMiningJob)
        ph = await c.expect(M.SetNewPrevHash)
        pj = next(reversed(pool.jobs.values()))
        assert job.channel_id == ok.channel_id and not job.has_min_ntime and job.job_id == pj.job_int
        assert job.merkle_root == pool.merkle_root_for(pj, ok.extranonce)
        assert ph.job_id == job.job_id and ph.prev_hash == pj.block.prev_hash and ph.nbits == pj.block.nbits
        c.close()
    run(with_pool(body))


def test_v2_nominal_hashrate_sets_initial_difficulty():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        ok = await c.open(hashrate=1.8e10)
        want = pool.vardiff.difficulty_for_hashrate(f32(1.8e10))  # nominal_hashrate travels as an f32
        assert ok.target == pool.share_target(want) and want > 1
        c.close()
    run(with_pool(body))


def test_v2_extended_channel_min_extranonce_too_large():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        r = await c.open(extended=True, min_en=EN2_SIZE + 1)
        assert isinstance(r, M.OpenMiningChannelError) and r.error == "min-extranonce-size-too-large"
        ok = await c.open(extended=True, min_en=EN2_SIZE)
        assert isinstance(ok, M.OpenExtendedMiningChannelSuccess) and ok.extranonce_size == EN2_SIZE
        assert len(ok.extranonce_prefix) == EN1_SIZE
        j = await c.expect(M.NewExtendedMiningJob)
        pj = next(reversed(pool.jobs.values()))
        assert j.coinbase_prefix == pj.coinb1 and j.coinbase_suffix == pj.coinb2 and j.merkle_path == pj.branches
        c.close()
    run(with_pool(body))


def test_v2_standard_share_success_then_duplicate_and_stale():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        ok = await c.open()
        job = await c.expect(M.NewMiningJob)
        jid = f"{job.job_id:x}"
        nonce, ntime, ver, _ = mine(pool, jid, ok.extranonce)
        sub = M.SubmitSharesStandard(channel_id=ok.channel_id, sequence_number=1, job_id=job.job_id, nonce=nonce,
                                     ntime=ntime, nversion=ver)
        await c.send(sub)
        r = await c.expect(M.SubmitSharesSuccess)
        assert r.last_sequence_number == 1 and r.new_submits_accepted == 1
        sub.sequence_number = 2
        await c.send(sub)
        r = await c.expect(M.SubmitSharesError)
        assert r.error == "duplicate-share" and r.sequence_number == 2
        pool.new_block()
        await c.expect(M.SetNewPrevHash)
        sub.sequence_number = 3
        await c.send(sub)
        r = await c.expect(M.SubmitSharesError)
        assert r.error == "stale-job"
        c.close()
    run(with_pool(body))


def test_v2_submit_channel_checks():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        std = await c.open()
        ext = await c.open(extended=True)
        await c.send(M.SubmitSharesStandard(channel_id=99, sequence_number=1, job_id=1))
        assert (await c.expect(M.SubmitSharesError)).error == "invalid-channel-id"
        await c.send(M.SubmitSharesStandard(channel_id=ext.channel_id, sequence_number=2, job_id=1))
        assert (await c.expect(M.SubmitSharesError)).error == "invalid-channel-id"   # standard on extended
        await c.send(M.SubmitSharesExtended(channel_id=std.channel_id, sequence_number=3, job_id=1, extranonce=bytes(4)))
        assert (await c.expect(M.SubmitSharesError)).error == "invalid-channel-id"   # extended on standard
        await c.send(M.SubmitSharesExtended(channel_id=ext.channel_id, sequence_number=4, job_id=1, extranonce=bytes(3)))
        assert (await c.expect(M.SubmitSharesError)).error == "invalid-extranonce-size"
        c.close()
    run(with_pool(body))


def test_v2_extended_share_accepted_with_rolled_extranonce():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        ok = await c.open(extended=True)
        job = await c.expect(M.NewExtendedMiningJob)
        jid = f"{job.job_id:x}"
        en = bytes.fromhex("0000abcd")
        nonce, ntime, ver, _ = mine(pool, jid, ok.extranonce_prefix + en)
        await c.send(M.SubmitSharesExtended(channel_id=ok.channel_id, sequence_number=5, job_id=job.job_id,
                                            nonce=nonce, ntime=ntime, nversion=ver, extranonce=en))
        r = await c.expect(M.SubmitSharesSuccess)
        assert r.last_sequence_number == 5
        c.close()
    run(with_pool(body))


def test_v2_update_channel_sends_set_target():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        ok = await c.open()
        await c.send(M.UpdateChannel(channel_id=ok.channel_id, nominal_hashrate=4e12))
        st = await c.expect(M.SetTarget)
        assert st.channel_id == ok.channel_id
        assert st.max_target == pool.share_target(pool.vardiff.difficulty_for_hashrate(f32(4e12)))
        c.close()
    run(with_pool(body))


def test_v2_close_channel_invalidates_it():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        ok = await c.open()
        await c.send(M.CloseChannel(channel_id=ok.channel_id, reason="bye"))
        await c.send(M.SubmitSharesStandard(channel_id=ok.channel_id, sequence_number=1, job_id=1))
        assert (await c.expect(M.SubmitSharesError)).error == "invalid-channel-id"
        c.close()
    run(with_pool(body))


def test_v2_new_job_broadcast_to_every_channel():
    async def body(pool):
        c = await V2Raw.connect(pool)
        await c.setup()
        a = await c.open()
        b = await c.open(user=ADDR + ".b")
        await c.expect(M.SetNewPrevHash)   # b's initial (job, prevhash) pair; a's was skipped by open()
        j = pool.new_job(clean=False)
        got = {(await c.expect(M.NewMiningJob)).channel_id for _ in range(2)}
        assert got == {a.channel_id, b.channel_id}
        assert j.job_int > 0
        c.close()
    run(with_pool(body))


def test_v2_garbage_frame_ends_only_that_connection():
    async def body(pool):
        bad = await V2Raw.connect(pool)
        bad.w.write(b"\x00\x00\x00\xff\xff\xff" + b"\x00" * 10)   # claims a 16 MiB payload, then stalls
        bad.w.write_eof()
        good = await V2Raw.connect(pool)
        r = await good.setup()
        assert isinstance(r, M.SetupConnectionSuccess)
        bad.close()
        good.close()
    run(with_pool(body))


def test_pool_metrics_track_clients_and_verdicts():
    async def body(pool):
        c = await V1Raw.connect(pool)
        n = await c.handshake()
        jid, en2 = n["params"][0], bytes(4)
        nonce, ntime, _, _ = mine(pool, jid, c.en1 + en2)
        await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}"])
        await c.call("mining.submit", ["w1", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}"])
        text = pool.registry.render()
        assert 'otedama_pool_shares_total{algo="sha256d",status="accepted"} 1' in text
        assert 'otedama_pool_shares_total{algo="sha256d",status="rejected"} 1' in text
        assert 'otedama_pool_connected_clients{algo="sha256d"} 1' in text
        st = pool.stats()
        assert st["clients_v1"] == 1 and st["accepted"] == 1 and st["rejected"] == 1
        c.close()
    run(with_pool(body))


def test_pool_workers_and_blocks_api():
    """GET /api/v1/workers and /api/v1/blocks payloads: journal totals merged with the live vardiff state, and the
    blocks found with their payout split."""
    async def body(pool):
        c = await V1Raw.connect(pool)
        n = await c.handshake(user=ADDR + ".rigA")
        jid, en2 = n["params"][0], bytes(4)
        nonce, ntime, _, _ = mine(pool, jid, c.en1 + en2)
        await c.call("mining.submit", ["w", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}"])
        await c.call("mining.submit", ["w", jid, en2.hex(), f"{ntime:08x}", f"{nonce:08x}"])  # duplicate
        ws = pool.workers()
        assert len(ws) == 1
        w = ws[0]
        assert w["worker"] == ADDR + ".rigA" and w["accepted"] == 1 and w["rejected"] == 1 and w["connected"] == 1
        assert w["difficulty"] == pytest.approx(2e-5) and w["accepted_work"] == pytest.approx(2e-5)
        assert w["algorithm"] == "sha256d"
        assert pool.blocks() == []
        pool.journal.record_block(840000, "00" * 32, ADDR + ".rigA", 312_500_000, "pplns")
        b = pool.blocks()
        assert b[0]["height"] == 840000 and b[0]["payouts"] == [{"worker": ADDR + ".rigA", "amount": 312_500_000}]
        c.close()
        await asyncio.sleep(0.1)
        assert pool.workers()[0]["connected"] == 0   # journal totals outlive the session
    run(with_pool(body))
