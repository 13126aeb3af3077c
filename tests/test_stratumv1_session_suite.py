"""Stratum V1 client session, case by case: mirrors internal/poolproto/stratumv1/{stratumv1,dialer,coverage}_test.go.

Every case runs the real client against a loopback pool whose replies are scripted per method (the reference's
runFakeServer / net.Pipe pattern, stratumv1_test.go:288-325,1438-1500). Reference behaviour (file:line in
/root/reference/internal/poolproto/stratumv1):
  * Negotiate: subscribe -> authorize (must be true) -> extranonce.subscribe (errors tolerated) ... dialer.go:109-174
  * dispatch: responses by id (int / float / numeric string), notify (drop-oldest, clean purges),
    set_difficulty, set_extranonce, show_message, reconnect (closes, host NOT followed),
    unknown methods and malformed lines ignored .................................... stratumv1.go:209-325
  * call(): id-correlated pending map; close fails pending calls; submit after close fails  :330-458
  * 64 KiB line cap ends the session ............................................... :73,183-194
Additions here: BIP310 mining.configure (version mask), the 6th submit parameter computed against the share's own
job version, extranonce2 / worker / hex formatting of mining.submit.
"""
import asyncio
import json
import math

import pytest

from otedama_amd.models.header import hash_to_int, target_from_difficulty
from otedama_amd.poolproto import base as PB
from otedama_amd.poolproto.base import Credentials, FatalPoolError, HandshakeFailed, PoolProtoError, ProtocolID, \
    ShareSubmission
from otedama_amd.poolproto.stratumv1 import BIP320_MASK, MAX_LINE_BYTES, V1Dialer, V1Session, prevhash_to_stratum

PREV = prevhash_to_stratum(bytes(range(32)))


def notify(job_id="1a", clean=True, version="20000000", ntime="5f5e1000", coinb1="01000000", branches=()):
    return {"id": None, "method": "mining.notify",
            "params": [job_id, PREV, coinb1, "ffffffff", list(branches), version, "1d00ffff", ntime, clean]}


def note(method, *params):
    return {"id": None, "method": method, "params": list(params)}


class Pool:
    """Loopback V1 pool: `replies[method]` is a result value, ("error", err) or a callable(msg) -> reply dict|None.
    `after_auth` items (dicts or raw bytes) are sent right after a successful authorize."""

    def __init__(self, replies=None, after_auth=(), configure=True):
        self.replies = {
            "mining.configure": {"version-rolling": True, "version-rolling.mask": "1fffe000"} if configure
            else ("error", [20, "Unknown method", None]),
            "mining.subscribe": [[["mining.notify", "s1"]], "abcd0001", 4],
            "mining.authorize": True,
            "mining.extranonce.subscribe": True,
            "mining.submit": True,
        }
        self.replies.update(replies or {})
        self.after_auth = list(after_auth)
        self.received: list[dict] = []
        self.writers = []
        self.server = None

    async def start(self):
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return f"stratum+tcp://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"

    async def push(self, *items):
        for w in self.writers:
            for it in items:
                w.write(it if isinstance(it, bytes) else json.dumps(it).encode() + b"\n")
            await w.drain()

    async def stop(self):
        for w in self.writers:
            w.close()
        self.server.close()
        await self.server.wait_closed()

    async def _handle(self, reader, writer):
        self.writers.append(writer)
        while True:
            line = await reader.readline()
            if not line:
                return
            msg = json.loads(line)
            self.received.append(msg)
            rep = self.replies.get(msg["method"], ("error", [20, "Unknown method", None]))
            if callable(rep):
                rep = rep(msg)
                if rep is None:
                    continue
                out = rep
            elif isinstance(rep, tuple) and rep and rep[0] == "error":
                out = {"id": msg["id"], "result": None, "error": rep[1]}
            elif isinstance(rep, tuple) and rep and rep[0] == "close":
                writer.close()
                return
            else:
                out = {"id": msg["id"], "result": rep, "error": None}
            writer.write(json.dumps(out).encode() + b"\n")
            if msg["method"] == "mining.authorize" and out.get("result") is True:
                for it in self.after_auth:
                    writer.write(it if isinstance(it, bytes) else json.dumps(it).encode() + b"\n")
            await writer.drain()

    def methods(self):
        return [m["method"] for m in self.received]

    def submits(self):
        return [m["params"] for m in self.received if m["method"] == "mining.submit"]


def creds(**kw):
    c = dict(user="bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq.rig7", worker="rig7", version_rolling=True)
    c.update(kw)
    return Credentials(**c)


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


async def session(pool, **kw):
    url = await pool.start()
    return await V1Dialer().dial(url, creds(**kw))


async def until(cond, timeout=5.0):
    end = asyncio.get_running_loop().time() + timeout
    while not cond():
        if asyncio.get_running_loop().time() > end:
            raise AssertionError("condition not reached")
        await asyncio.sleep(0.01)


async def next_job(s, timeout=5.0):
    return await asyncio.wait_for(s.jobs.get(), timeout)


# ---------------------------------------------------------------------------------------------- dialer / registry

def test_dialer_protocols_and_registration():
    assert V1Dialer().protocol is ProtocolID.STRATUM_V1
    assert V1Dialer(True).protocol is ProtocolID.STRATUM_V1_TLS
    assert isinstance(PB.lookup(ProtocolID.STRATUM_V1), V1Dialer) and not PB.lookup(ProtocolID.STRATUM_V1).use_tls
    assert PB.lookup(ProtocolID.STRATUM_V1_TLS).use_tls
    assert {ProtocolID.STRATUM_V1, ProtocolID.STRATUM_V1_TLS} <= set(PB.available())


@pytest.mark.parametrize("url", ["stratum+tcp://", "stratum+tcp:///"])
def test_dialer_empty_host_is_an_error(url):
    async def main():
        with pytest.raises(PoolProtoError):
            await V1Dialer().dial(url, creds())
    run(main())


def test_dialer_unreachable_host_fails():
    async def main():
        srv = await asyncio.start_server(lambda r, w: None, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        srv.close()
        await srv.wait_closed()
        with pytest.raises(OSError):
            await V1Dialer().dial(f"stratum+tcp://127.0.0.1:{port}", creds(), timeout=2)
    run(main())


def test_dialer_dial_fn_seam_success_and_error():
    async def main():
        pool = Pool()
        url = await pool.start()
        port = int(url.rsplit(":", 1)[1])
        seen = []

        async def dial_fn(host, p):
            seen.append((host, p))
            return await asyncio.open_connection("127.0.0.1", port)
        s = await V1Dialer(dial_fn=dial_fn).dial("stratum+tcp://pool.example:4444", creds())
        assert seen == [("pool.example", 4444)] and not s.closed
        await s.close()

        async def failing(host, p):
            raise ConnectionRefusedError("nope")
        with pytest.raises(ConnectionRefusedError):
            await V1Dialer(dial_fn=failing).dial("stratum+tcp://pool.example:4444", creds())
        await pool.stop()
    run(main())


def test_dialer_default_port_is_3333():
    async def main():
        seen = []

        async def dial_fn(host, p):
            seen.append((host, p))
            raise ConnectionRefusedError("stop here")
        with pytest.raises(ConnectionRefusedError):
            await V1Dialer(dial_fn=dial_fn).dial("stratum+tcp://pool.example", creds())
        assert seen == [("pool.example", 3333)]
    run(main())


def test_tls_dialer_rejects_garbage_ca_pem():
    async def main():
        pool = Pool()
        url = await pool.start()
        with pytest.raises(Exception):
            await V1Dialer(True).dial(url.replace("stratum+tcp", "stratum+tls"),
                                      creds(tls_root_cas_pem=b"-----BEGIN CERTIFICATE-----\ngarbage\n"), timeout=3)
        await pool.stop()
    run(main())


# ---------------------------------------------------------------------------------------------- negotiate

def test_negotiate_success_extranonce_parsed():
    async def main():
        pool = Pool()
        s = await session(pool)
        assert pool.methods() == ["mining.configure", "mining.subscribe", "mining.authorize",
                                  "mining.extranonce.subscribe"]
        assert s.extranonce1 == bytes.fromhex("abcd0001") and s.extranonce2_size == 4
        assert s.version_mask == BIP320_MASK and s.protocol is ProtocolID.STRATUM_V1
        assert s.remote_addr.startswith("127.0.0.1:")
        auth = pool.received[2]["params"]
        assert auth == ["bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq.rig7", "x"]  # empty password defaults to "x"
        assert pool.received[1]["params"][0].startswith("Otedama/")
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_sends_configured_password():
    async def main():
        pool = Pool()
        s = await session(pool, password="d=1024")
        assert pool.received[2]["params"][1] == "d=1024"
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_configure_request_shape():
    async def main():
        pool = Pool()
        s = await session(pool)
        exts, opts = pool.received[0]["params"]
        assert exts == ["version-rolling"] and opts["version-rolling.mask"] == "1fffe000"
        assert opts["version-rolling.min-bit-count"] == 2
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_without_version_rolling_skips_configure():
    async def main():
        pool = Pool()
        s = await session(pool, version_rolling=False)
        assert "mining.configure" not in pool.methods() and s.version_mask == 0
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_configure_unsupported_leaves_mask_zero():
    async def main():
        pool = Pool(configure=False)
        s = await session(pool)
        assert s.version_mask == 0 and "mining.subscribe" in pool.methods()
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_configure_mask_is_clamped_to_bip320():
    async def main():
        pool = Pool({"mining.configure": {"version-rolling": True, "version-rolling.mask": "ffffffff"}})
        s = await session(pool)
        assert s.version_mask == BIP320_MASK
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_subscribe_error_is_handshake_failed():
    async def main():
        pool = Pool({"mining.subscribe": ("error", [25, "not subscribed", None])})
        with pytest.raises(HandshakeFailed, match="subscribe failed"):
            await session(pool)
        await pool.stop()
    run(main())


@pytest.mark.parametrize("result,match", [
    ("nope", "unexpected subscribe result"),
    ([[], "ab"], "unexpected subscribe result"),
    ([[], 7, 4], "extranonce1 not a string"),
    ([[], "ab", "4"], "extranonce2_size not a number"),
    ([[], "ab", 99], "out of range"),
    ([[], "zz", 4], "not hex"),
])
def test_negotiate_subscribe_result_unparseable(result, match):
    async def main():
        pool = Pool({"mining.subscribe": result})
        with pytest.raises(HandshakeFailed, match=match):
            await session(pool)
        await pool.stop()
    run(main())


def test_negotiate_empty_subscriptions_array_is_fine():
    async def main():
        pool = Pool({"mining.subscribe": [[], "", 8]})
        s = await session(pool)
        assert s.extranonce1 == b"" and s.extranonce2_size == 8
        await s.close()
        await pool.stop()
    run(main())


@pytest.mark.parametrize("reply", [False, None, ("error", [24, "unauthorized worker", None])])
def test_negotiate_authorize_rejected_is_fatal(reply):
    async def main():
        pool = Pool({"mining.authorize": reply})
        with pytest.raises(FatalPoolError, match="authorize rejected"):
            await session(pool)
        await pool.stop()
    run(main())


@pytest.mark.parametrize("reply", [("error", [20, "Method not found", None]), False, True])
def test_negotiate_extranonce_subscribe_outcome_never_fails_handshake(reply):
    async def main():
        pool = Pool({"mining.extranonce.subscribe": reply})
        s = await session(pool)
        assert not s.closed
        await s.close()
        await pool.stop()
    run(main())


def test_negotiate_pool_closes_during_subscribe():
    async def main():
        pool = Pool({"mining.subscribe": ("close",)})
        with pytest.raises(PoolProtoError):
            await session(pool)
        await pool.stop()
    run(main())


# ---------------------------------------------------------------------------------------------- dispatch

def test_notify_delivers_job_with_session_fields():
    async def main():
        pool = Pool(after_auth=[note("mining.set_difficulty", 2), notify(branches=["11" * 32])])
        s = await session(pool)
        job = await next_job(s)
        assert job.job_id == "1a" and job.prev_hash == bytes(range(32)) and job.nbits == 0x1D00FFFF
        assert job.version == 0x20000000 and job.ntime == 0x5F5E1000 and job.clean_jobs
        assert job.coinb1 == bytes.fromhex("01000000") and job.merkle_branches == [bytes.fromhex("11" * 32)]
        assert job.extranonce1 == bytes.fromhex("abcd0001") and job.extranonce2_size == 4
        assert job.version_mask == BIP320_MASK and job.algorithm == "sha256d"
        assert hash_to_int(job.target) == hash_to_int(target_from_difficulty(2.0))
        await s.close()
        await pool.stop()
    run(main())


def test_dispatch_empty_and_malformed_lines_are_ignored():
    async def main():
        pool = Pool(after_auth=[b"\n", b"\r\n", b"{not json\n", b"[1,2,3]\n", b"\xff\xfe\n", b"42\n",
                                notify(job_id="after")])
        s = await session(pool)
        assert (await next_job(s)).job_id == "after" and not s.closed
        await s.close()
        await pool.stop()
    run(main())


def test_dispatch_notify_parse_error_is_ignored():
    async def main():
        bad = [note("mining.notify", "x", PREV), note("mining.notify", "y", "zz", "", "", [], "2", "1", "1", True),
               note("mining.notify", "z", PREV, "01", "ff", [], "20000000", "1d00ffff", "5f5e1000", "yes")]
        pool = Pool(after_auth=bad + [notify(job_id="good")])
        s = await session(pool)
        assert (await next_job(s)).job_id == "good" and s.jobs.empty()
        await s.close()
        await pool.stop()
    run(main())


def test_notify_clean_jobs_as_int():
    async def main():
        n = notify(job_id="c0")
        n["params"][8] = 0
        pool = Pool(after_auth=[n])
        s = await session(pool)
        assert not (await next_job(s)).clean_jobs
        await s.close()
        await pool.stop()
    run(main())


def test_notify_numeric_job_id_stays_an_opaque_string():
    async def main():
        n = notify()
        n["params"][0] = 1234
        pool = Pool(after_auth=[n])
        s = await session(pool)
        assert (await next_job(s)).job_id == "1234"
        await s.close()
        await pool.stop()
    run(main())


def test_full_job_channel_drops_oldest():
    async def main():
        pool = Pool(after_auth=[notify(job_id=f"j{i}", clean=False) for i in range(12)])
        s = await session(pool)
        await until(lambda: s.last_job is not None and s.last_job.job_id == "j11")
        ids = [s.jobs.get_nowait().job_id for _ in range(s.jobs.qsize())]
        assert ids == [f"j{i}" for i in range(4, 12)]  # capacity 8, newest kept
        await s.close()
        await pool.stop()
    run(main())


def test_clean_jobs_purges_pending_jobs():
    async def main():
        pool = Pool(after_auth=[notify(job_id="a", clean=False), notify(job_id="b", clean=False),
                                notify(job_id="c", clean=True)])
        s = await session(pool)
        await until(lambda: s.last_job is not None and s.last_job.job_id == "c")
        assert s.jobs.qsize() == 1 and s.jobs.get_nowait().job_id == "c"
        await s.close()
        await pool.stop()
    run(main())


def test_set_extranonce_updates_fields_for_next_job():
    async def main():
        pool = Pool(after_auth=[note("mining.set_extranonce", "beef", 6), notify()])
        s = await session(pool)
        job = await next_job(s)
        assert s.extranonce1 == b"\xbe\xef" and s.extranonce2_size == 6
        assert job.extranonce1 == b"\xbe\xef" and job.extranonce2_size == 6
        await s.close()
        await pool.stop()
    run(main())


@pytest.mark.parametrize("params", [["beef"], [7, 4], ["beef", "4"], ["beef", 99], ["beef", -1], ["xyz", 4]])
def test_set_extranonce_malformed_is_ignored(params):
    async def main():
        pool = Pool(after_auth=[note("mining.set_extranonce", *params), notify()])
        s = await session(pool)
        await next_job(s)
        assert s.extranonce1 == bytes.fromhex("abcd0001") and s.extranonce2_size == 4 and not s.closed
        await s.close()
        await pool.stop()
    run(main())


@pytest.mark.parametrize("value", [0, -3, "8", None, True, math.inf])
def test_set_difficulty_invalid_values_are_ignored(value):
    async def main():
        pool = Pool(after_auth=[note("mining.set_difficulty", 4), notify(),
                                note("mining.set_difficulty", value if value is not math.inf else 1e400)])
        s = await session(pool)
        await next_job(s)
        await asyncio.sleep(0.1)
        assert s.suggested_difficulty() == 4.0 and s.jobs.empty()
        await s.close()
        await pool.stop()
    run(main())


def test_set_difficulty_before_first_job_applies_to_it():
    async def main():
        pool = Pool(after_auth=[note("mining.set_difficulty", 0.5)])
        s = await session(pool)
        await until(lambda: s.suggested_difficulty() == 0.5)
        assert s.jobs.empty()  # nothing to re-issue yet
        await pool.push(notify())
        job = await next_job(s)
        assert hash_to_int(job.target) == hash_to_int(target_from_difficulty(0.5))
        await s.close()
        await pool.stop()
    run(main())


def test_suggested_difficulty_initial_default_is_zero():
    async def main():
        pool = Pool()
        s = await session(pool)
        assert s.suggested_difficulty() == 0.0
        await pool.push(notify())
        job = await next_job(s)
        assert hash_to_int(job.target) == hash_to_int(target_from_difficulty(1.0))  # difficulty 1 until told
        await s.close()
        await pool.stop()
    run(main())


def test_set_version_mask_updates_and_clamps():
    async def main():
        pool = Pool(after_auth=[note("mining.set_version_mask", "ffffffff"), notify()])
        s = await session(pool)
        assert (await next_job(s)).version_mask == BIP320_MASK
        await pool.push(note("mining.set_version_mask", "00006000"), notify(job_id="b"))
        assert (await next_job(s)).version_mask == 0x6000
        await s.close()
        await pool.stop()
    run(main())


def test_show_message_delivered_on_notice_channel():
    async def main():
        pool = Pool(after_auth=[note("client.show_message", "maintenance at 12:00")])
        s = await session(pool)
        assert await asyncio.wait_for(s.notices.get(), 5) == "maintenance at 12:00"
        await s.close()
        await pool.stop()
    run(main())


@pytest.mark.parametrize("params", [[""], [], [42]])
def test_show_message_empty_or_malformed_not_delivered(params):
    async def main():
        pool = Pool(after_auth=[note("client.show_message", *params), notify()])
        s = await session(pool)
        await next_job(s)
        assert s.notices.empty()
        await s.close()
        await pool.stop()
    run(main())


def test_show_message_full_channel_drops_oldest():
    async def main():
        pool = Pool(after_auth=[note("client.show_message", f"m{i}") for i in range(10)] + [notify()])
        s = await session(pool)
        await next_job(s)
        got = [s.notices.get_nowait() for _ in range(s.notices.qsize())]
        assert got == [f"m{i}" for i in range(2, 10)]
        await s.close()
        await pool.stop()
    run(main())


def test_unknown_notification_silently_ignored():
    async def main():
        pool = Pool(after_auth=[note("mining.fancy_new_thing", 1, 2), note("client.get_version"), notify()])
        s = await session(pool)
        assert (await next_job(s)).job_id == "1a" and not s.closed
        await s.close()
        await pool.stop()
    run(main())


@pytest.mark.parametrize("method", ["client.reconnect", "mining.reconnect"])
def test_reconnect_closes_session_and_is_not_followed(method):
    async def main():
        pool = Pool(after_auth=[note(method, "evil.example", "4444", 9)])
        s = await session(pool)
        await until(lambda: s.closed)
        assert s.last_reconnect == {"host": "evil.example", "port": 4444, "wait": 9}
        await pool.stop()
    run(main())


def test_pool_closed_mid_session_closes_the_session():
    async def main():
        pool = Pool()
        s = await session(pool)
        for w in pool.writers:
            w.close()
        await asyncio.wait_for(s.wait_closed(), 5)
        assert s.closed
        with pytest.raises(PoolProtoError, match="session closed"):
            await s.submit(ShareSubmission("1a", 1, 1))
        await pool.stop()
    run(main())


def test_oversized_line_terminates_session():
    async def main():
        pool = Pool(after_auth=[b'{"id":null,"method":"client.show_message","params":["' + b"x" * MAX_LINE_BYTES
                                + b'"]}\n'])
        s = await session(pool)
        await asyncio.wait_for(s.wait_closed(), 5)
        assert s.notices.empty()
        await pool.stop()
    run(main())


def test_line_just_under_the_cap_is_accepted():
    async def main():
        body = b'{"id":null,"method":"client.show_message","params":["'
        tail = b'"]}\n'
        msg = b"y" * (MAX_LINE_BYTES - len(body) - len(tail) - 1)
        pool = Pool(after_auth=[body + msg + tail])
        s = await session(pool)
        assert await asyncio.wait_for(s.notices.get(), 5) == msg.decode()
        await s.close()
        await pool.stop()
    run(main())


# ---------------------------------------------------------------------------------------------- calls / submit

@pytest.mark.parametrize("rid", [2, 2.0, "2"])
def test_response_id_forms_resolve_pending_call(rid):
    async def main():
        pool = Pool({"mining.ping": lambda msg: None})  # the test answers by hand
        s = await session(pool)
        fut = asyncio.ensure_future(s._call("mining.ping", []))
        await until(lambda: pool.methods()[-1:] == ["mining.ping"])
        mid = s._next_id
        await pool.push({"id": str(mid) if isinstance(rid, str) else (float(mid) if isinstance(rid, float) else mid),
                         "result": "pong", "error": None})
        assert await asyncio.wait_for(fut, 5) == ("pong", None)
        await s.close()
        await pool.stop()
    run(main())


def test_response_for_unknown_id_is_ignored():
    async def main():
        pool = Pool(after_auth=[{"id": 999, "result": True, "error": None}, {"id": "abc", "result": 1, "error": None},
                                notify()])
        s = await session(pool)
        assert (await next_job(s)).job_id == "1a" and not s.closed
        await s.close()
        await pool.stop()
    run(main())


def test_call_timeout_clears_pending():
    async def main():
        pool = Pool({"mining.slow": lambda msg: None})
        s = await session(pool)
        with pytest.raises(asyncio.TimeoutError):
            await s._call("mining.slow", [], timeout=0.2)
        assert not s._pending
        await s.close()
        await pool.stop()
    run(main())


def test_close_cancels_pending_calls():
    async def main():
        pool = Pool({"mining.slow": lambda msg: None})
        s = await session(pool)
        fut = asyncio.ensure_future(s._call("mining.slow", []))
        await until(lambda: "mining.slow" in pool.methods())
        await s.close()
        with pytest.raises(PoolProtoError, match="closed before response"):
            await asyncio.wait_for(fut, 5)
        await pool.stop()
    run(main())


def test_close_is_idempotent_and_submit_after_close_fails():
    async def main():
        pool = Pool()
        s = await session(pool)
        await s.close()
        await s.close()
        assert s.closed
        with pytest.raises(PoolProtoError, match="session closed"):
            await s.submit(ShareSubmission("1a", 1, 1))
        await pool.stop()
    run(main())


def test_submit_wire_format():
    async def main():
        pool = Pool(after_auth=[notify()])
        s = await session(pool)
        job = await next_job(s)
        r = await s.submit(ShareSubmission("1a", 0xABC, 0x5F5E10FF, job.version, b"\x00\x00\x00\x07", worker="w2"))
        assert r.accepted and r.latency_ms > 0
        assert pool.submits()[0] == ["w2", "1a", "00000007", "5f5e10ff", "00000abc"]
        await s.close()
        await pool.stop()
    run(main())


def test_submit_worker_precedence_and_default_extranonce2():
    async def main():
        pool = Pool(after_auth=[notify()])
        s = await session(pool)
        await next_job(s)
        await s.submit(ShareSubmission("1a", 1, 2))                        # creds.worker
        s.creds.worker = ""
        await s.submit(ShareSubmission("1a", 1, 3))                        # creds.user
        first, second = pool.submits()
        assert first[0] == "rig7" and second[0] == "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq.rig7"
        assert first[2] == "00000000"  # zero extranonce2 of the negotiated size
        await s.close()
        await pool.stop()
    run(main())


def test_submit_version_bits_only_when_rolled():
    async def main():
        pool = Pool(after_auth=[notify(version="20000000")])
        s = await session(pool)
        job = await next_job(s)
        await s.submit(ShareSubmission("1a", 1, 1, job.version))
        await s.submit(ShareSubmission("1a", 2, 1, job.version | 0x00006000))
        await s.submit(ShareSubmission("1a", 3, 1, job.version | 0x40000000 | 0x2000))  # bits outside mask dropped
        a, b, c = pool.submits()
        assert len(a) == 5 and b[5] == "00006000" and c[5] == "00002000"
        await s.close()
        await pool.stop()
    run(main())


def test_submit_version_param_compares_against_the_shares_own_job():
    """Two live non-clean jobs with different versions: a share for job A rolled to job B's version still needs
    the 6th parameter, or the pool rebuilds job A's version and rejects it."""
    async def main():
        pool = Pool(after_auth=[notify(job_id="A", version="20000000"),
                                notify(job_id="B", version="20004000", clean=False)])
        s = await session(pool)
        await until(lambda: s.last_job is not None and s.last_job.job_id == "B")
        await s.submit(ShareSubmission("A", 1, 1, 0x20004000))
        await s.submit(ShareSubmission("B", 1, 1, 0x20004000))
        a, b = pool.submits()
        assert a[5] == "00004000" and len(b) == 5
        await s.close()
        await pool.stop()
    run(main())


def test_submit_without_negotiated_mask_never_sends_version():
    async def main():
        pool = Pool(after_auth=[notify()], configure=False)
        s = await session(pool)
        job = await next_job(s)
        await s.submit(ShareSubmission("1a", 1, 1, job.version | 0x2000))
        assert len(pool.submits()[0]) == 5
        await s.close()
        await pool.stop()
    run(main())


@pytest.mark.parametrize("error,reason", [([23, "low difficulty share", None], "low difficulty share"),
                                          ({"code": 21, "message": "job not found"}, "job not found"),
                                          ("stale", "stale")])
def test_submit_pool_error_reports_reason(error, reason):
    async def main():
        pool = Pool({"mining.submit": ("error", error)}, after_auth=[notify()])
        s = await session(pool)
        await next_job(s)
        r = await s.submit(ShareSubmission("1a", 1, 1))
        assert not r.accepted and r.reason == reason
        await s.close()
        await pool.stop()
    run(main())


def test_submit_false_result_is_rejected():
    async def main():
        pool = Pool({"mining.submit": False}, after_auth=[notify()])
        s = await session(pool)
        await next_job(s)
        r = await s.submit(ShareSubmission("1a", 1, 1))
        assert not r.accepted and r.reason == "rejected"
        await s.close()
        await pool.stop()
    run(main())


def test_submit_accepted_reports_current_difficulty():
    async def main():
        pool = Pool(after_auth=[note("mining.set_difficulty", 64), notify()])
        s = await session(pool)
        await next_job(s)
        r = await s.submit(ShareSubmission("1a", 1, 1))
        assert r.accepted and r.difficulty == 64.0
        await s.close()
        await pool.stop()
    run(main())


def test_submit_pool_closes_mid_submit_raises():
    async def main():
        pool = Pool({"mining.submit": ("close",)}, after_auth=[notify()])
        s = await session(pool)
        await next_job(s)
        with pytest.raises(PoolProtoError):
            await s.submit(ShareSubmission("1a", 1, 1))
        await pool.stop()
    run(main())


def test_concurrent_submits_are_correlated_by_id():
    async def main():
        def reply(msg):
            nonce = msg["params"][4]
            if int(nonce, 16) % 2:
                return {"id": msg["id"], "result": True, "error": None}
            return {"id": msg["id"], "result": None, "error": [23, f"odd-{nonce}", None]}
        pool = Pool({"mining.submit": reply}, after_auth=[notify()])
        s = await session(pool)
        await next_job(s)
        rs = await asyncio.gather(*(s.submit(ShareSubmission("1a", n, 1)) for n in range(20)))
        for n, r in enumerate(rs):
            assert r.accepted == bool(n % 2)
            if not r.accepted:
                assert r.reason == f"odd-{n:08x}"
        await s.close()
        await pool.stop()
    run(main())


def test_session_is_a_v1session():
    async def main():
        pool = Pool()
        s = await session(pool)
        assert isinstance(s, V1Session) and isinstance(s, PB.Session)
        await s.close()
        await pool.stop()
    run(main())
