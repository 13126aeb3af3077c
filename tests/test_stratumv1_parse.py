"""Stratum V1 parsers and the client's notification dispatcher, table-driven.

Mirrors internal/poolproto/stratumv1/parse_test.go and the dispatch cases of stratumv1_test.go
(TestParseNotify_*, TestParseDifficulty_*, TestParseSetExtranonce_*, TestParseShowMessage_*,
TestParseReconnect_*, TestParseSubscribeResult_*, TestSendJob_CleanJobsPurges, TestSendJob_DropOldest), plus
the fixes this client makes over the reference (prevhash word order, hex job ids, malformed notifications
never end the session).
"""
from __future__ import annotations

import asyncio
import json
import math

import pytest

from otedama_amd.models.header import DIFF1_TARGET_INT, hash_to_int, target_from_difficulty
from otedama_amd.poolproto import base as B
from otedama_amd.poolproto import stratumv1 as V1

PREV_HDR = bytes(range(32))
PREV = V1.prevhash_to_stratum(PREV_HDR)


def _notify(**kw):
    d = dict(job_id="1a", prev=PREV, coinb1="01000000", coinb2="ffffffff", branches=[], version="20000000",
             nbits="1d00ffff", ntime="5f5e1000", clean=True)
    d.update(kw)
    return [d["job_id"], d["prev"], d["coinb1"], d["coinb2"], d["branches"], d["version"], d["nbits"], d["ntime"],
            d["clean"]]


# ------------------------------------------------------------------ prevhash word order
def test_prevhash_round_trip_and_word_swap():
    s = V1.prevhash_to_stratum(PREV_HDR)
    assert V1.prevhash_from_stratum(s) == PREV_HDR
    # each 4-byte word is reversed, word order kept
    assert bytes.fromhex(s)[:4] == PREV_HDR[:4][::-1] and bytes.fromhex(s)[28:] == PREV_HDR[28:][::-1]


@pytest.mark.parametrize("bad", ["00" * 31, "00" * 33, "zz" * 32, ""])
def test_prevhash_rejects_bad_input(bad):
    with pytest.raises(ValueError):
        V1.prevhash_from_stratum(bad)


# ------------------------------------------------------------------ mining.notify
def test_parse_notify_fields():
    br = ["11" * 32, "22" * 32]
    j = V1.parse_notify(_notify(branches=br, coinb1="aabb", coinb2="ccdd"))
    assert j.job_id == "1a" and j.prev_hash == PREV_HDR
    assert (j.version, j.nbits, j.ntime) == (0x20000000, 0x1D00FFFF, 0x5F5E1000)
    assert j.coinb1 == b"\xaa\xbb" and j.coinb2 == b"\xcc\xdd" and j.merkle_branches == [b"\x11" * 32, b"\x22" * 32]
    assert j.clean_jobs is True and j.merkle_root is None


@pytest.mark.parametrize("jid,want", [("1a", "1a"), ("00ff", "00ff"), (17, "17"), ("job-7", "job-7")])
def test_parse_notify_job_id_is_opaque(jid, want):
    assert V1.parse_notify(_notify(job_id=jid)).job_id == want


@pytest.mark.parametrize("clean,want", [(True, True), (False, False), (1, True), (0, False), (1.0, True), (0.0, False)])
def test_parse_notify_clean_jobs_bool_or_number(clean, want):
    assert V1.parse_notify(_notify(clean=clean)).clean_jobs is want


@pytest.mark.parametrize("params", [
    None, {}, "x", [], _notify()[:8],
    _notify(clean="yes"), _notify(clean=None),
    _notify(version="zz"), _notify(nbits="1d00fffg"), _notify(ntime=""),
    _notify(prev="00" * 31), _notify(coinb1="abc"), _notify(branches=["0"]),
])
def test_parse_notify_rejects_malformed(params):
    with pytest.raises((ValueError, TypeError)):
        V1.parse_notify(params)


def test_parse_notify_ignores_extra_params():
    assert V1.parse_notify(_notify() + ["extra", 1]).job_id == "1a"


def test_parse_notify_masks_fields_to_u32():
    j = V1.parse_notify(_notify(version="1ffffffff", ntime="100000001"))
    assert j.version == 0xFFFFFFFF and j.ntime == 1


# ------------------------------------------------------------------ other notifications
@pytest.mark.parametrize("params,want", [([1], 1.0), ([0.5], 0.5), ([1024, "x"], 1024.0), ([], None), (None, None),
                                         (["2"], None), ([True], None), ({"d": 1}, None)])
def test_parse_difficulty(params, want):
    assert V1.parse_difficulty(params) == want


@pytest.mark.parametrize("params,want", [(["abcd", 4], ("abcd", 4)), (["", 8], ("", 8)), (["abcd"], None),
                                         ([1, 4], None), (["ab", "4"], None), (None, None)])
def test_parse_set_extranonce(params, want):
    assert V1.parse_set_extranonce(params) == want


@pytest.mark.parametrize("params,want", [(["hello"], "hello"), ([""], ""), ([5], None), ([], None), (None, None)])
def test_parse_show_message(params, want):
    assert V1.parse_show_message(params) == want


@pytest.mark.parametrize("params,want", [
    (["pool2.example", 3334, 5], {"host": "pool2.example", "port": 3334, "wait": 5}),
    (["pool2.example", "3334"], {"host": "pool2.example", "port": 3334, "wait": 0}),
    (["h", "x"], {"host": "h", "port": 0, "wait": 0}),
    ([], {"host": "", "port": 0, "wait": 0}),
    (None, {"host": "", "port": 0, "wait": 0}),
    ([5, 6, "7"], {"host": "", "port": 6, "wait": 0}),
])
def test_parse_reconnect(params, want):
    assert V1.parse_reconnect(params) == want


@pytest.mark.parametrize("result,want", [
    ([[["mining.notify", "s"]], "abcd0001", 4], ("abcd0001", 4)),
    ([[], "", 8], ("", 8)),
    ([None, "00", 4.0], ("00", 4)),
])
def test_parse_subscribe_result(result, want):
    assert V1.parse_subscribe_result(result) == want


@pytest.mark.parametrize("result", [None, [], [[], "ab"], [[], 5, 4], [[], "ab", "4"], [[], "ab", True],
                                    [[], "ab", -1], [[], "ab", 33], [[], "ab", 4.5], [[], "xyz", 4]])
def test_parse_subscribe_result_rejects(result):
    with pytest.raises(B.HandshakeFailed):
        V1.parse_subscribe_result(result)


# ------------------------------------------------------------------ dispatcher (no sockets)
class _W:
    def __init__(self):
        self.buf = bytearray()
        self.closed = False

    def write(self, b):
        self.buf += b

    async def drain(self):
        pass

    def close(self):
        self.closed = True

    def get_extra_info(self, k):
        return ("127.0.0.1", 3333) if k == "peername" else None


def _session(algo="sha256d"):
    return V1.V1Session(asyncio.StreamReader(), _W(), B.Credentials(user="u.w"), B.ProtocolID.STRATUM_V1, algo)


def _line(method, params, mid=None):
    return (json.dumps({"id": mid, "method": method, "params": params}) + "\n").encode()


def _jobs(s):
    out = []
    while not s.jobs.empty():
        out.append(s.jobs.get_nowait())
    return out


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 10))


def test_notify_job_carries_session_state():
    async def go():
        s = _session()
        s.extranonce1, s.extranonce2_size, s.version_mask = b"\xab\xcd", 4, V1.BIP320_MASK
        s._dispatch(_line("mining.set_difficulty", [2]))
        s._dispatch(_line("mining.notify", _notify()))
        (j,) = _jobs(s)
        assert j.extranonce1 == b"\xab\xcd" and j.extranonce2_size == 4 and j.version_mask == V1.BIP320_MASK
        assert j.target == target_from_difficulty(2)
    run(go())


def test_default_share_target_is_difficulty_1():
    async def go():
        s = _session()
        s._dispatch(_line("mining.notify", _notify()))
        (j,) = _jobs(s)
        assert hash_to_int(j.target) == DIFF1_TARGET_INT
    run(go())


def test_scrypt_session_uses_the_scrypt_diff1():
    async def go():
        s = _session("scrypt")
        s._dispatch(_line("mining.notify", _notify()))
        (j,) = _jobs(s)
        assert hash_to_int(j.target) > DIFF1_TARGET_INT and j.algorithm == "scrypt"
    run(go())


def test_clean_jobs_purges_queued_jobs_and_non_clean_appends():
    async def go():
        s = _session()
        for i in range(3):
            s._dispatch(_line("mining.notify", _notify(job_id=f"a{i}", clean=False)))
        s._dispatch(_line("mining.notify", _notify(job_id="b0", clean=True)))
        s._dispatch(_line("mining.notify", _notify(job_id="b1", clean=False)))
        assert [j.job_id for j in _jobs(s)] == ["b0", "b1"]
    run(go())


def test_job_queue_drops_the_oldest_when_full():
    async def go():
        s = _session()
        for i in range(s.jobs.maxsize + 5):
            s._dispatch(_line("mining.notify", _notify(job_id=str(i), clean=False)))
        ids = [j.job_id for j in _jobs(s)]
        assert len(ids) == s.jobs.maxsize and ids[-1] == str(s.jobs.maxsize + 4) and ids[0] == "5"
    run(go())


def test_set_difficulty_reissues_a_copy_keeping_the_queued_clean_job():
    async def go():
        s = _session()
        s._dispatch(_line("mining.notify", _notify(clean=True)))
        s._dispatch(_line("mining.set_difficulty", [8]))
        first, second = _jobs(s)
        assert first.clean_jobs is True and first.target == target_from_difficulty(1)
        assert second.clean_jobs is False and second.target == target_from_difficulty(8)
        assert s.suggested_difficulty() == 8
    run(go())


@pytest.mark.parametrize("bad", [[0], [-1], ["8"], [], None])
def test_invalid_difficulty_is_ignored(bad):
    async def go():
        s = _session()
        s._dispatch(_line("mining.set_difficulty", [4]))
        s._dispatch(_line("mining.set_difficulty", bad))
        assert s.suggested_difficulty() == 4
    run(go())


def test_non_finite_difficulty_is_ignored():
    async def go():
        s = _session()
        s._dispatch(_line("mining.set_difficulty", [4]))
        s._dispatch(b'{"id": null, "method": "mining.set_difficulty", "params": [Infinity]}\n')
        s._dispatch(b'{"id": null, "method": "mining.set_difficulty", "params": [NaN]}\n')
        assert s.suggested_difficulty() == 4 and math.isfinite(s.suggested_difficulty())
    run(go())


def test_set_extranonce_updates_later_jobs():
    async def go():
        s = _session()
        s._dispatch(_line("mining.set_extranonce", ["f00d", 6]))
        s._dispatch(_line("mining.notify", _notify()))
        (j,) = _jobs(s)
        assert (s.extranonce1, s.extranonce2_size) == (b"\xf0\x0d", 6) and j.extranonce2_size == 6
    run(go())


@pytest.mark.parametrize("params", [["nothex", 4], ["abcd", -1], ["abcd", 64], ["abc", 4]])
def test_malformed_set_extranonce_keeps_the_previous_values(params):
    async def go():
        s = _session()
        s.extranonce1, s.extranonce2_size = b"\x01", 4
        s._dispatch(_line("mining.set_extranonce", params))
        assert (s.extranonce1, s.extranonce2_size) == (b"\x01", 4) and not s.closed
    run(go())


@pytest.mark.parametrize("mask,want", [("1fffe000", 0x1FFFE000), ("ffffffff", 0x1FFFE000), ("00006000", 0x6000),
                                       ("zz", 0)])
def test_set_version_mask_is_clamped_to_bip320(mask, want):
    async def go():
        s = _session()
        s._dispatch(_line("mining.set_version_mask", [mask]))
        assert s.version_mask == want
    run(go())


def test_show_message_goes_to_notices():
    async def go():
        s = _session()
        s._dispatch(_line("client.show_message", ["maintenance at 12:00"]))
        s._dispatch(_line("client.show_message", [""]))
        assert s.notices.get_nowait() == "maintenance at 12:00" and s.notices.empty()
    run(go())


@pytest.mark.parametrize("method", ["client.reconnect", "mining.reconnect"])
def test_reconnect_records_and_closes_without_following(method):
    async def go():
        s = _session()
        s._dispatch(_line(method, ["evil.example", 4444, 0]))
        await asyncio.sleep(0.01)
        assert s.closed and s.writer.closed and s.last_reconnect["host"] == "evil.example"
    run(go())


@pytest.mark.parametrize("line", [b"", b"\n", b"not json\n", b"[1,2]\n", b"\xff\xfe\n", b'{"id": "x"}\n',
                                  b'{"id": 99, "result": true}\n', b'{"method": "mining.unknown", "params": []}\n',
                                  b'{"method": "mining.notify", "params": [1]}\n'])
def test_garbage_lines_are_ignored(line):
    async def go():
        s = _session()
        s._dispatch(line)
        assert s.jobs.empty() and not s.closed
    run(go())


def test_responses_resolve_pending_calls_by_id():
    async def go():
        s = _session()
        fut = asyncio.get_running_loop().create_future()
        s._pending[7] = fut
        s._dispatch(b'{"id": "7", "result": true, "error": null}\n')
        assert fut.result() == (True, None) and 7 not in s._pending
    run(go())


def test_submit_params_and_version_bits():
    async def go():
        s = _session()
        s.extranonce2_size, s.version_mask = 4, V1.BIP320_MASK
        s._dispatch(_line("mining.notify", _notify()))
        s.last_job = _jobs(s)[0]
        task = asyncio.ensure_future(s.submit(B.ShareSubmission("1a", 0xDEADBEEF, 0x5F5E1001, 0x20002000,
                                                                b"\x01\x00\x00\x00", worker="rig7")))
        await asyncio.sleep(0)
        sent = json.loads(bytes(s.writer.buf).decode().splitlines()[-1])
        assert sent["method"] == "mining.submit"
        assert sent["params"] == ["rig7", "1a", "01000000", "5f5e1001", "deadbeef", "00002000"]
        s._dispatch(json.dumps({"id": sent["id"], "result": None, "error": [23, "Low difficulty share", None]})
                    .encode() + b"\n")
        r = await task
        assert not r.accepted and r.reason == "Low difficulty share"
    run(go())


def test_submit_without_rolled_version_omits_the_version_param():
    async def go():
        s = _session()
        s.extranonce2_size = 2
        s._dispatch(_line("mining.notify", _notify()))
        task = asyncio.ensure_future(s.submit(B.ShareSubmission("1a", 1, 2, 0x20000000)))
        await asyncio.sleep(0)
        sent = json.loads(bytes(s.writer.buf).decode().splitlines()[-1])
        assert sent["params"] == ["u.w", "1a", "0000", "00000002", "00000001"]
        s._dispatch(json.dumps({"id": sent["id"], "result": True, "error": None}).encode() + b"\n")
        assert (await task).accepted
    run(go())


@pytest.mark.parametrize("err,want", [([21, "Job not found", None], "Job not found"), ({"message": "stale"}, "stale"),
                                      ("boom", "boom"), ([1], "[1]")])
def test_error_text(err, want):
    assert V1._error_text(err) == want


# ------------------------------------------------------------------ poolproto helpers
@pytest.mark.parametrize("url,pid", [
    ("stratum+tcp://h:1", B.ProtocolID.STRATUM_V1), ("stratum+tls://h:1", B.ProtocolID.STRATUM_V1_TLS),
    ("stratum+v2://h:1", B.ProtocolID.STRATUM_V2), ("stratum+v2tls://h:1", B.ProtocolID.STRATUM_V2_TLS),
    ("datum://h:1", B.ProtocolID.DATUM), ("http://h", B.ProtocolID.UNKNOWN), ("", B.ProtocolID.UNKNOWN),
])
def test_from_url(url, pid):
    assert B.from_url(url) == pid


def test_protocol_tls_flags():
    assert [p for p in B.ProtocolID if p.uses_tls] == [B.ProtocolID.STRATUM_V1_TLS, B.ProtocolID.STRATUM_V2_TLS]
    assert not any(p.post_quantum_ready() for p in B.ProtocolID)


@pytest.mark.parametrize("url,want", [("stratum+tcp://pool:3333", "pool:3333"), ("stratum+v2tls://a.b/x", "a.b/x")])
def test_strip_scheme(url, want):
    assert B.strip_scheme(url) == want


@pytest.mark.parametrize("url", ["stratum+tcp://", "http://x", "pool:3333"])
def test_strip_scheme_unknown(url):
    with pytest.raises(B.UnknownProtocol):
        B.strip_scheme(url)


@pytest.mark.parametrize("hp,want", [("pool:3333", ("pool", 3333)), ("pool", ("pool", 9)), ("[::1]:10", ("::1", 10)),
                                     ("[::1]", ("::1", 9)), ("pool:3333/path", ("pool", 3333))])
def test_split_host_port(hp, want):
    assert B.split_host_port(hp, 9) == want


@pytest.mark.parametrize("v,size,want", [(1, 4, "01000000"), (0x0102, 2, "0201"), (1, 0, ""), (1, 10, "01" + "00" * 9),
                                         ((1 << 64) + 5, 8, "05" + "00" * 7)])
def test_extranonce2_bytes(v, size, want):
    assert B.extranonce2_bytes(v, size).hex() == want


def test_dialer_registry():
    assert {B.ProtocolID.STRATUM_V1, B.ProtocolID.STRATUM_V1_TLS} <= set(B.available())
    with pytest.raises(B.PoolProtoError, match="already registered"):
        B.register(V1.V1Dialer(False))
    with pytest.raises(B.UnknownProtocol):
        B.lookup(B.ProtocolID.DATUM)

    class Unknown(B.Dialer):
        protocol = B.ProtocolID.UNKNOWN

        async def dial(self, url, creds, timeout=10.0):
            raise AssertionError

    with pytest.raises(B.PoolProtoError, match="ProtocolUnknown"):
        B.register(Unknown())
    with pytest.raises(B.PoolProtoError, match="nil"):
        B.register(None)


def test_dial_url_unknown_scheme():
    with pytest.raises(B.UnknownProtocol):
        run(B.dial_url("ftp://x", B.Credentials()))


def test_job_template_for_the_native_runtime():
    j = V1.parse_notify(_notify(coinb1="aa", coinb2="bb", branches=["11" * 32]))
    j.extranonce1, j.extranonce2_size, j.version_mask = b"\x01", 4, 0x6000
    t = j.template()
    assert len(t["header"]) == 80 and t["header"][4:36] == PREV_HDR and t["header"][36:68] == bytes(32)
    assert t["coinb1"] == b"\xaa" and t["extranonce2_size"] == 4 and t["merkle_branches"] == [b"\x11" * 32]
    assert t["version_mask"] == 0x6000 and t["target"] == b"\xff" * 32
    j2 = B.Job("x", merkle_root=b"\x07" * 32)
    assert "coinb1" not in j2.template() and j2.template()["header"][36:68] == b"\x07" * 32


def test_put_drop_oldest():
    q = asyncio.Queue(maxsize=2)
    for i in range(5):
        B.put_drop_oldest(q, i)
    assert [q.get_nowait(), q.get_nowait()] == [3, 4]
