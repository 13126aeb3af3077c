"""Protocol / economics units with property tests (hypothesis).

Mirrors stratum/{frame,messages}_fuzz_test.go, poolproto/stratumv1/parse_test.go,
arbitration/engine_property_test.go, rates/fetcher_test.go, i18n/*_test.go,
daemon/service_test.go, and adds vardiff + merkle checks for the pool.
"""
import asyncio
import http.server
import threading

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from otedama_amd import arbitration as A
from otedama_amd import daemon, i18n
from otedama_amd.hal import Capabilities, Family, Identity
from otedama_amd.pool import template as T
from otedama_amd.pool.vardiff import Vardiff, VardiffConfig
from otedama_amd.poolproto.stratumv1 import parse_notify, prevhash_from_stratum, prevhash_to_stratum
from otedama_amd.provider import sats_per_second
from otedama_amd.rates import Fetcher, Source
from otedama_amd.stratum import messages as M
from otedama_amd.stratum.frame import (Frame, FrameError, FrameReader, FrameScanner, Header, decode_header,
                                       encode_frame, iter_frames)


# ------------------------------------------------------------------ frames / messages
@settings(max_examples=300, deadline=None)
@given(st.binary(min_size=0, max_size=200))
def test_frame_and_dispatch_fuzz_never_crash(data):
    try:
        frames = list(iter_frames(data))
    except (FrameError, EOFError):  # malformed header / truncated frame (io.ErrUnexpectedEOF)
        return
    for f in frames:
        for dialect in (M.REFERENCE, M.SPEC):
            try:
                msg = M.dispatch_frame(f, dialect)
            except FrameError:
                continue
            assert isinstance(msg, M.Message)


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 2 ** 32 - 1), st.integers(0, 2 ** 32 - 1), st.integers(0, 2 ** 32 - 1),
       st.integers(0, 2 ** 32 - 1), st.integers(0, 2 ** 32 - 1), st.binary(min_size=32, max_size=32))
def test_message_roundtrips(ch, job, nonce, ntime, ver, h32):
    msgs = [M.NewMiningJob(ch, job, True, ntime, ver, h32), M.NewMiningJob(ch, job, False, 0, ver, h32),
            M.SetNewPrevHash(ch, job, h32, ntime, nonce), M.SetTarget(ch, h32),
            M.SubmitSharesStandard(ch, job & 0xFFFF, job, nonce, ntime, ver)]
    for m in msgs:
        for dialect in (M.REFERENCE, M.SPEC):
            raw = M.encode_message(m, dialect)
            (f,) = list(iter_frames(raw))
            assert f.header.channel_msg == m.CHANNEL_MSG
            assert M.dispatch_frame(f, dialect) == m


@settings(max_examples=60, deadline=None)
@given(ch=st.integers(0, 2 ** 32 - 1), job=st.integers(0, 2 ** 32 - 1), ntime=st.integers(0, 2 ** 32 - 1),
       path=st.lists(st.binary(min_size=32, max_size=32), max_size=12), pre=st.binary(max_size=300),
       suf=st.binary(max_size=300), en=st.binary(max_size=32), opt=st.booleans())
def test_extended_channel_messages_roundtrip(ch, job, ntime, path, pre, suf, en, opt):
    msgs = [M.OpenExtendedMiningChannel(ch, "u.w", 2.0 ** 40, bytes(range(32)), len(en)),
            M.OpenExtendedMiningChannelSuccess(ch, job, bytes(32), len(en), en),
            M.NewExtendedMiningJob(ch, job, opt, ntime if opt else 0, 0x20000000, opt, path, pre, suf),
            M.SubmitSharesExtended(ch, job, job, ntime, ntime, 0x20002000, en)]
    for m in msgs:
        for dialect in (M.REFERENCE, M.SPEC):
            (f,) = list(iter_frames(M.encode_message(m, dialect)))
            assert f.header.channel_msg == m.CHANNEL_MSG
            assert M.dispatch_frame(f, dialect) == m


def test_frame_header_u24_and_unknown():
    f = Frame(Header(0, 0x7F, 3), b"abc")
    raw = encode_frame(f)
    assert decode_header(raw).msg_length == 3
    msg = M.dispatch_frame(list(iter_frames(raw))[0])
    assert isinstance(msg, M.UnknownMessage)
    with pytest.raises(FrameError):
        decode_header(b"\x00\x00")


_frame = st.builds(lambda ext, t, p: Frame(Header(ext, t, len(p)), p),
                   st.integers(0, 0xFFFF), st.integers(0, 255), st.binary(min_size=4, max_size=300))


@settings(max_examples=150, deadline=None)
@given(frames=st.lists(_frame, max_size=12), cuts=st.lists(st.integers(0, 4000), max_size=8), native=st.booleans())
def test_frame_scanner_matches_iter_frames_under_any_chunking(frames, cuts, native):
    raw = b"".join(encode_frame(f) for f in frames)
    pos = sorted({c % (len(raw) + 1) for c in cuts} | {0, len(raw)})
    sc = FrameScanner(native=native)
    got = []
    for a, b in zip(pos, pos[1:]):
        got += sc.feed(raw[a:b])
    assert got == frames == list(iter_frames(raw)) and sc.pending == 0


@settings(max_examples=300, deadline=None)
@given(st.binary(min_size=0, max_size=120), st.integers(7, 64))
def test_native_and_python_scanners_agree(data, max_frame):
    from otedama_amd.ops.native import load
    from otedama_amd.stratum.frame import _scan_py

    mod = load(build_if_missing=False)
    if mod is None:
        pytest.skip("native extension not built")
    recs, consumed, status = mod.sv2_scan(data, max_frame)
    assert (recs, consumed, status) == _scan_py(data, max_frame)


def test_frame_scanner_errors_after_the_good_frames():
    good = encode_frame(Frame(Header(0, 1, 2), b"ok"))
    bad_channel = bytes([0, 0x80, 0x20, 2, 0, 0]) + b"xy"      # channel bit, 2-byte payload
    sc = FrameScanner()
    assert [f.payload for f in sc.feed(good + bad_channel)] == [b"ok"]
    with pytest.raises(FrameError, match="channel message requires payload"):
        sc.feed(b"")
    huge = bytes([0, 0, 1, 0xFF, 0xFF, 0xFF])                  # 16 MiB + 5 > max frame, rejected on the header
    with pytest.raises(FrameError, match="exceeds MaxFrameSize"):
        FrameScanner(max_frame_size=1 << 20).feed(huge)
    with pytest.raises(FrameError):
        FrameScanner(max_frame_size=0)


def test_frame_reader_chunks_and_eof():
    async def main():
        r = asyncio.StreamReader()
        frames = [Frame(Header(0, 0x20, n), bytes([n & 0xFF]) * n) for n in (0, 5, 1000, 70000)]
        r.feed_data(b"".join(encode_frame(f) for f in frames) + encode_frame(frames[1])[:4])
        r.feed_eof()
        fr = FrameReader(r, chunk=4096)
        assert [await fr.read_frame() for _ in frames] == frames
        with pytest.raises(asyncio.IncompleteReadError):
            await fr.read_frame()

    asyncio.run(main())


# ------------------------------------------------------------------ V1 parsing
def test_prevhash_word_swap_roundtrip():
    header_prev = bytes(range(32))
    s = prevhash_to_stratum(header_prev)
    assert s[:8] == "03020100" and prevhash_from_stratum(s) == header_prev


def test_parse_notify():
    prev = prevhash_to_stratum(bytes(range(32)))
    job = parse_notify(["j1", prev, "01000000", "ffffffff", ["aa" * 32], "20000000", "1d00ffff", "5f5e1000", True])
    assert job.job_id == "j1" and job.version == 0x20000000 and job.nbits == 0x1D00FFFF and job.clean_jobs
    assert job.prev_hash == bytes(range(32)) and job.merkle_branches == [bytes.fromhex("aa" * 32)]
    with pytest.raises(ValueError):
        parse_notify(["j1"])


# ------------------------------------------------------------------ merkle / template
def test_merkle_block_100000():
    txids = [bytes.fromhex(h)[::-1] for h in (
        "8c14f0db3df150123e6f3dbbf30f8b955a8249b62ac1d1ff16284aefa3d06d87",
        "fff2525b8931402dd09222c50775608f75787bd2b87e56995a7bdd30f79702c4",
        "6359f0868171b1d194cbee1af2f16ea598ae8fad666d9b012c8ed2b79a236ec4",
        "e9a66845e05d5abc0ad04ec80f774a7e585c6e8db975962d069a522137b80c1d")]
    root = "f3e94742aca4b5ef85488dc37c06c3282295ffec960994b2c0d5ac2a25a95766"
    assert T.merkle_root_full(txids)[::-1].hex() == root
    assert T.merkle_root_from_branches(txids[0], T.merkle_branches(txids[1:]))[::-1].hex() == root


def test_varint_scriptnum():
    assert T.varint(0xFC) == b"\xfc" and T.varint(0xFD) == b"\xfd\xfd\x00"
    assert T.varint(0x10000) == b"\xfe\x00\x00\x01\x00"
    assert T.script_num(0) == b"\x00" and T.script_num(1) == b"\x01\x01"
    assert T.script_num(128) == b"\x02\x80\x00" and T.script_num(840000) == b"\x03\x40\xd1\x0c"


# ------------------------------------------------------------------ vardiff
def test_vardiff_converges_and_bounds():
    now = [0.0]
    vd = Vardiff(VardiffConfig(target_share_seconds=10, retarget_seconds=30), clock=lambda: now[0])
    s = vd.new_state(1.0)
    # shares every 1 s at difficulty 1 -> should raise difficulty (bounded x4 per step) once min_shares arrived
    new = None
    for _ in range(16):
        now[0] += 1.0
        new = vd.on_share(s) or new
    assert new == 4.0 and s.difficulty == 4.0
    # no shares for a long time -> lower difficulty
    now[0] += 70
    assert vd.maybe_retarget(s) == 1.0
    assert vd.difficulty_for_hashrate(2 ** 32 / 10) == pytest.approx(1.0)
    assert vd.clamp(1e30) == vd.cfg.max_difficulty


# ------------------------------------------------------------------ arbitration
def _dev(i, fam=Family.GPU):
    return A.DeviceRef(Identity(f"d{i}", fam, "amd", "mi355x"), Capabilities(sha256d=True, general_compute=True))


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(st.floats(0, 100), st.floats(0, 1)), min_size=1, max_size=5),
       st.floats(0, 0.5), st.integers(1, 4))
def test_arbitration_properties(yields, hyst, ndev):
    streams = [A.Stream(f"s{i}", [Family.GPU], default_yield=A.Yield(y, c)) for i, (y, c) in enumerate(yields)]
    devs = [_dev(i) for i in range(ndev)]
    a1 = A.decide(A.Input(devs, streams, hysteresis_margin=hyst))
    a2 = A.decide(A.Input(list(reversed(devs)), streams, hysteresis_margin=hyst))
    assert [(x.device_id, x.stream) for x in a1.assignments] == [(x.device_id, x.stream) for x in a2.assignments]
    best = max((s.default_yield.effective() for s in streams), default=0)
    for a in a1.assignments:
        assert a.expected_yield <= best + 1e-12
        if best > 0:
            assert a.expected_yield == best  # no previous allocation: always the best
    # with the previous allocation, a hold never loses more than the hysteresis margin
    a3 = A.decide(A.Input(devs, streams, previous=a1, hysteresis_margin=hyst))
    for a in a3.assignments:
        if a.held:
            assert best <= a.expected_yield * (1 + hyst) + 1e-9


def test_arbitration_errors_and_floor():
    s = [A.Stream("m", [Family.GPU], default_yield=A.Yield(1.0, 1.0))]
    with pytest.raises(A.ArbitrationError):
        A.decide(A.Input([_dev(0), _dev(0)], s))
    with pytest.raises(A.ArbitrationError):
        A.decide(A.Input([_dev(0)], s, hysteresis_margin=-1))
    a = A.decide(A.Input([_dev(0)], s, min_yield_sats_per_sec=2.0))
    assert a.assignments[0].idle() and "floor" in a.assignments[0].reason and a.skipped_device == 1
    assert A.Policy.parse("stack_btc") is A.Policy.STACK_BTC


def test_sats_per_second():
    assert sats_per_second(0.36, 100_000) == pytest.approx(0.36 / 3600 / 100_000 * 1e8)
    assert sats_per_second(1, 0) == 0


# ------------------------------------------------------------------ rates
def test_rates_median_fallback_and_plausibility():
    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            body = self.path.strip("/").encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    try:
        f = Fetcher(95000, sources=[Source(n, f"{base}/{v}", float) for n, v in
                                    (("a", "100000"), ("b", "102000"), ("c", "5"), ("d", "101000"))])
        assert f.btc_usd_rate() == (95000, False)
        f.fetch()
        assert f.btc_usd_rate() == (101000, True)
        assert f.source_health()[:2] == (3, 4)
        bad = Fetcher(95000, sources=[Source("x", "http://127.0.0.1:1/", float)], timeout=1)
        with pytest.raises(RuntimeError, match="all sources failed"):
            bad.fetch()
        assert bad.btc_usd_rate() == (95000, False)
    finally:
        srv.shutdown()


# ------------------------------------------------------------------ i18n
def test_i18n_catalog_complete_and_detection():
    b = i18n.new_bundle()
    assert len(b.languages()) >= 10
    for lang in b.languages():
        assert b.missing_translations(lang) == []
    assert i18n.detect_lang("ja-JP") == "ja" and i18n.detect_lang("xx") == "en" and i18n.detect_lang("") == "en"
    assert i18n.detect_lang_from_env({"LANG": "de_DE.UTF-8"}.get) == "de"
    assert i18n.detect_lang_from_env({"LC_ALL": "C"}.get) == "en"
    assert "{{" not in b.render_with("en", i18n.STARTUP_POOL_CONNECTING, {"url": "x"})


# ------------------------------------------------------------------ daemon
def test_daemon_unit_generation(tmp_path, monkeypatch):
    calls = []
    monkeypatch.setattr(daemon, "run_cmd", lambda *a: calls.append(a))
    monkeypatch.setattr(daemon, "platform", "linux")
    m = daemon.Manager("/etc/o t/config.yaml", str(tmp_path / "data"),
                       daemon.ServiceFlags(bitcoin_address="bc1qx", log_level="debug"), executable="/usr/bin/python3",
                       home=str(tmp_path))
    unit = m.systemd_unit()
    assert f'ExecStart={m.executable} -m otedama_amd run --config "/etc/o t/config.yaml"' in unit
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in unit and f"ReadWritePaths={tmp_path}/data" in unit
    m.install()
    assert m.systemd_unit_path().exists() and calls[-1][:3] == ("systemctl", "--user", "enable")
    plist = m.launchd_plist()
    assert "<string>otedama_amd</string>" in plist and "&" not in plist.replace("&amp;", "")
    monkeypatch.setattr(daemon, "platform", "plan9")
    with pytest.raises(daemon.DaemonError):
        m.install()
    assert daemon.quote_token('a"b c') == '"a\\"b c"'


# ------------------------------------------------------------------ HAL
def test_hal_drm_driver_filters(tmp_path):
    """gpu_linux.go parity: render nodes are reported once, AMD nodes are left to the HIP driver, and a node
    whose vendor cannot be read (another partition's node in a container) is not reported at all."""
    from otedama_amd import hal

    def node(name, vendor, pci="PCI_ID=10DE:2684"):
        dev = tmp_path / "devices" / name
        dev.mkdir(parents=True)
        if vendor is not None:
            (dev / "vendor").write_text(vendor + "\n")
        (dev / "uevent").write_text(pci + "\n")
        (tmp_path / "drm" / name).mkdir(parents=True)
        (tmp_path / "drm" / name / "device").symlink_to(dev)

    node("renderD128", "0x10de")
    node("renderD129", "0x1002", "PCI_ID=1002:75A3")
    node("renderD130", None)
    drv = hal.GPULinuxDriver(str(tmp_path / "drm"), skip_vendors=("0x1002",))
    devs = drv.enumerate()
    assert [d.identity().id for d in devs] == ["gpu-renderD128"]
    assert devs[0].identity().vendor == "NVIDIA" and not devs[0].capabilities().sha256d
    assert devs[0].capabilities().general_compute


def test_hal_capabilities_match_kernels():
    from otedama_amd import hal
    from otedama_amd.models import algorithms

    cpu = hal.CPUDriver(2).enumerate()[0]
    # CpuMiner: SHA-256d through SHA-NI, scrypt / X11 through the host reference chains
    assert cpu.capabilities().sha256d and cpu.capabilities().scrypt and cpu.capabilities().x11
    gfx950 = hal.KERNEL_ISAS["gfx950"]
    assert gfx950.sha256d and gfx950.scrypt and gfx950.x11
    assert set(algorithms.ALGORITHMS) == {"sha256d", "scrypt", "x11"}
    with pytest.raises(ValueError, match="unknown algorithm"):
        algorithms.get("x17")


def test_extranonce2_bytes_matches_the_native_coinbase_for_every_size():
    """The submitted extranonce2 must be the bytes the native runtime put in the coinbase (low 8 bytes rolled,
    the rest zero), including extranonce2_size > 8 (the old serialisation sent only 8 bytes there)."""
    from otedama_amd.ops.native import load
    from otedama_amd.poolproto.base import extranonce2_bytes

    assert extranonce2_bytes(0x1234, 0) == b""
    assert extranonce2_bytes(0x0102030405060708, 4) == bytes([8, 7, 6, 5])
    assert extranonce2_bytes(0x0102030405060708, 12) == bytes([8, 7, 6, 5, 4, 3, 2, 1, 0, 0, 0, 0])
    N = load()
    if N is None:
        return
    import hashlib

    def sha256d(b):
        return hashlib.sha256(hashlib.sha256(b).digest()).digest()

    coinb1, coinb2, en1 = b"\x01" * 41, b"\x02" * 30, b"\xaa\xbb\xcc\xdd"
    for size in (1, 4, 8, 12, 16):
        j = {"header": bytes(80), "target": b"\xff" * 32, "epoch": 1, "job_id": "1", "coinb1": coinb1,
             "coinb2": coinb2, "extranonce1": en1, "extranonce2_size": size, "merkle_branches": []}
        en2 = 0xA1B2C3D4E5F60718 & ((1 << (8 * min(size, 8))) - 1)
        assert N.merkle_root(j, en2) == sha256d(coinb1 + en1 + extranonce2_bytes(en2, size) + coinb2)
