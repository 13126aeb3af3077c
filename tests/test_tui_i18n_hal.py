"""TUI dashboard rendering, i18n catalogs and the hardware abstraction layer.

Mirrors internal/tui/dashboard_test.go (TestFormat*, TestVisibleLen_*, TestTruncateVisible_*, TestPadRight_*,
TestShortenURL_*, TestDashboard_*), internal/i18n(+/messages)/*_test.go (catalog completeness, placeholder
rendering, locale detection) and internal/hal/*_test.go (Identity validation, registry, detector partial
failure, fake-sysfs DRM enumeration).
"""
from __future__ import annotations

import io
import os
import threading
import time

import pytest

from otedama_amd import hal
from otedama_amd import i18n as I
from otedama_amd import tui as T


# ================================================================== TUI
@pytest.mark.parametrize("hps,want", [(0, "0 H/s"), (999, "999 H/s"), (1000, "1.00 kH/s"), (999_999, "1000.00 kH/s"),
                                      (1e6, "1.00 MH/s"), (1e9, "1.00 GH/s"), (18.8e9, "18.80 GH/s"),
                                      (1e12, "1.00 TH/s"), (150.4e12, "150.40 TH/s"), (2e15, "2.00 PH/s"),
                                      (-5, "-5 H/s")])
def test_format_hash_rate(hps, want):
    assert T.format_hash_rate(hps) == want


@pytest.mark.parametrize("sec,want", [(0, "0s"), (0.9, "0s"), (59, "59s"), (60, "1m 0s"), (3599, "59m 59s"),
                                      (3600, "1h 0m 0s"), (90061, "25h 1m 1s")])
def test_format_duration(sec, want):
    assert T.format_duration(sec) == want


@pytest.mark.parametrize("sats,want", [(0, "0 sats"), (999, "999 sats"), (1000, "1000 sats (0.00001 BTC)"),
                                       (99_999_999, "99999999 sats (1.00000 BTC)"), (100_000_000, "1.0000 BTC"),
                                       (250_000_000, "2.5000 BTC")])
def test_sats_to_display(sats, want):
    assert T.sats_to_display(sats) == want


def test_default_sats_per_hash_is_tiny_and_positive():
    v = T.default_sats_per_hash()
    assert 0 < v < 1e-10 and v == pytest.approx(3.125e8 / 6e23)


@pytest.mark.parametrize("s,n", [("", 0), ("plain", 5), ("\x1b[1m\x1b[36mbold cyan\x1b[0m", 9),
                                 ("a\x1b[2Kb", 2), ("x\x1b[", 1), ("\x1b[38;5;208morange\x1b[0m", 6), ("日本", 2)])
def test_visible_len(s, n):
    assert T.visible_len(s) == n


def test_truncate_visible():
    assert T.truncate_visible("hello world", 5) == "hello" + T.RESET
    assert T.truncate_visible("hi", 5) == "hi" + T.RESET
    out = T.truncate_visible(T.GREEN + "abcdef" + T.RESET, 3)
    assert out.startswith(T.GREEN + "abc") and out.endswith(T.RESET) and T.visible_len(out) == 3
    assert T.truncate_visible("abc", 0) == "" and T.truncate_visible("abc", -2) == ""


@pytest.mark.parametrize("s,w,want_len", [("abc", 6, 6), ("abcdef", 3, 6), ("", 4, 4), (T.RED + "ab" + T.RESET, 5, 5)])
def test_pad_right(s, w, want_len):
    assert T.visible_len(T.pad_right(s, w)) == want_len


@pytest.mark.parametrize("url,n,want", [("stratum+tcp://a.b:1", 19, "stratum+tcp://a.b:1"),
                                        ("stratum+tcp://a.b:12", 19, "stratum+tcp://a...."),
                                        ("abcdef", 3, "abcdef"), ("abcdefgh", 4, "a...")])
def test_shorten_url(url, n, want):
    got = T.shorten_url(url, n)
    assert got == want and (len(got) <= n or n < 4)


@pytest.mark.parametrize("s,b,want", [("abcdef", 10, "abcdef"), ("abcdef", 5, "ab..."), ("abcdef", 3, "abc"),
                                      ("abc", 0, "")])
def test_truncate_to_budget(s, b, want):
    assert T.truncate_to_budget(s, b) == want


def _dash(cols=80):
    d = T.Dashboard(io.StringIO(), interval=0.01)
    d.set_width(cols)
    return d


@pytest.mark.parametrize("cols", [40, 60, 80, 120, 200])
def test_every_frame_line_is_exactly_the_width(cols):
    d = _dash(cols)
    s = T.Stats(hash_rate=18.8e9, shares_found=10, shares_sent=9, pool_url="stratum+v2://" + "x" * 200 + ":3336",
                connected=True, pool_latency_ms=3, providers=[T.ProviderStats("AI Inference (simulated)", 2.5, True),
                                                              T.ProviderStats("Bitcoin Mining", 0.001, False)],
                wallet_fingerprint="abcd1234", est_sats_earned=5, uptime=3725, devices=8, devices_idle=1)
    frame = d.render(s)
    assert frame.startswith(T.HOME)
    for ln in frame[len(T.HOME):].split("\r\n")[:-1]:
        assert ln.startswith(T.CLEAR_LINE) and T.visible_len(ln) == cols


def test_zero_state_renders():
    frame = _dash().render(T.Stats())
    for needle in ("MINING", "EARNINGS", "WALLET", "0 H/s", "disconnected", "not initialized", "uptime: 0s"):
        assert needle in frame
    assert "ARBITRATION" not in frame


def test_set_width_minimum():
    d = _dash()
    d.set_width(10)
    assert d.cols == 80
    d.set_width(40)
    assert d.cols == 40


def test_mining_line_states():
    d = _dash()
    base = dict(hash_rate=1e9, devices=2)
    normal = d.mining_line(T.Stats(**base))
    assert "1.00 GH/s" in normal and "2 device(s)" in normal and "stalled" not in normal and "idle" not in normal
    assert "1 idle" in d.mining_line(T.Stats(**base, devices_idle=1))
    assert "⚠ stalled" in d.mining_line(T.Stats(**base, stalled=True))
    paused = d.mining_line(T.Stats(**base, stalled=True, curtailed=True))
    assert "⏸ paused" in paused and "stalled" not in paused  # curtailment takes priority


def test_pool_line_status_survives_a_narrow_width():
    d = _dash(40)
    line = d.pool_line(T.Stats(pool_url="stratum+v2://a-very-long-pool-hostname.example.com:3336", connected=True,
                               pool_latency_ms=12))
    assert "✓ connected" in line and "(12ms)" in line and T.visible_len(line) <= 40
    assert "✗ disconnected" in d.pool_line(T.Stats(pool_url="x"))


def test_earnings_line_adds_active_providers_only():
    d = _dash()
    s = T.Stats(hash_rate=0, providers=[T.ProviderStats("a", 1.0, True), T.ProviderStats("b", 100.0, False)])
    assert "86400 sats/day" in d.earnings_line(s)


def test_provider_line_active_vs_idle():
    assert "● active" in T.Dashboard.provider_line(T.ProviderStats("x", 1, True))
    assert "○ idle" in T.Dashboard.provider_line(T.ProviderStats("x", 1, False))


def test_wallet_line_and_footer():
    assert "abcd1234" in T.Dashboard.wallet_line(T.Stats(wallet_fingerprint="abcd1234"))
    d = _dash(40)
    f = d.footer(T.Stats(uptime=61, algorithm="x11"))
    assert "uptime: 1m 1s" in f and "algo: x11" in f and "Ctrl+C" in f
    narrow = _dash(40).footer(T.Stats(uptime=10 ** 7))  # left part wider than the budget
    assert " " + T.DIM + "Ctrl+C" in narrow  # the gap clamps at one space


def test_header_mentions_otedama():
    assert "Otedama" in _dash().render(T.Stats())


def test_stats_from_engine_dict():
    s = T.Stats.from_engine({"hashrate": 5.0, "shares_found": 3, "shares_submitted": 2, "pool": "p",
                             "latency_p50_ms": None, "connected": 1, "providers": [{"name": "n", "active": True}],
                             "devices": {"gpu-0": {}, "gpu-1": {}}, "stalled": 0, "algorithm": "scrypt"})
    assert (s.hash_rate, s.shares_found, s.shares_sent, s.devices, s.algorithm) == (5.0, 3, 2, 2, "scrypt")
    assert s.connected and s.pool_latency_ms == 0 and s.providers[0].name == "n"


def test_update_is_non_blocking_and_latest_wins():
    d = _dash()
    for i in range(1000):
        d.update(T.Stats(shares_found=i))
    d.update({"shares_found": 7})
    assert d._last.shares_found == 7


def test_render_loop_paints_updates_and_stops_cleanly():
    w = io.StringIO()
    d = T.Dashboard(w, interval=0.01)
    d.start()
    d.start()  # second start is a no-op
    d.update(T.Stats(hash_rate=2e9))
    deadline = time.time() + 5
    while "2.00 GH/s" not in w.getvalue() and time.time() < deadline:
        time.sleep(0.01)
    d.stop()
    d.stop()  # double stop is safe
    out = w.getvalue()
    assert out.startswith("\x1b[?25l") and "2.00 GH/s" in out and out.endswith("\x1b[?25h\n")
    n = len(out)
    time.sleep(0.05)
    assert len(w.getvalue()) == n  # nothing is written after stop returns


def test_stop_without_start_is_safe():
    T.Dashboard(io.StringIO()).stop()


def test_loop_exits_when_the_writer_breaks():
    class Broken(io.StringIO):
        def write(self, s):
            if "\x1b[H" in s and "MINING" in s:
                raise OSError("EPIPE")
            return super().write(s)

    d = T.Dashboard(Broken(), interval=0.01)
    d.start()
    d._thread.join(2)
    assert not d._thread.is_alive()
    d._thread = None


# ================================================================== i18n
def _all_placeholders() -> dict:
    import re

    names = set()
    for msg in I.new_bundle().catalogs["en"].messages.values():
        names |= set(re.findall(r"\{\{\s*\.(\w+)\s*\}\}", msg))
    return {k: "X" for k in names}


def test_every_language_translates_every_message():
    b = I.new_bundle()
    assert b.languages() == list(I.PRIORITY_LANGUAGES)
    for lang in I.PRIORITY_LANGUAGES:
        assert b.missing_translations(lang) == [], lang
        for mid in I.ALL_IDS:
            out = b.render_with(lang, mid, _all_placeholders())
            assert out and "<no value>" not in out and "{{" not in out


@pytest.mark.parametrize("mid", I.ALL_IDS)
def test_ids_are_valid_and_english_has_no_dangling_placeholders(mid):
    assert I.valid_id(mid)
    out = I.new_bundle().render_with("en", mid, _all_placeholders())
    assert "{{" not in out and "<no value>" not in out


def test_placeholders_are_consistent_across_languages():
    import re

    b = I.new_bundle()
    ph = re.compile(r"\{\{\s*\.(\w+)\s*\}\}")
    for mid in I.ALL_IDS:
        want = set(ph.findall(b.catalogs["en"].messages[mid]))
        for lang in I.PRIORITY_LANGUAGES:
            assert set(ph.findall(b.catalogs[lang].messages[mid])) == want, (lang, mid)


def test_render_with_missing_data_uses_no_value():
    b = I.new_bundle()
    assert "<no value>" in b.render_with("en", I.STARTUP_POOL_CONNECTING, {})
    assert "stratum+tcp://x" in b.render_with("ja", I.STARTUP_POOL_CONNECTING, {"url": "stratum+tcp://x"})


def test_unknown_language_falls_back_to_english_and_unknown_id_raises():
    b = I.new_bundle()
    assert b.render("xx", I.STATUS_MINING) == b.render("en", I.STATUS_MINING)
    with pytest.raises(I.I18nError):
        b.render("en", "no.such.id")


def test_catalog_validation():
    with pytest.raises(I.I18nError, match="unsupported language"):
        I.Catalog("tlh", {})
    with pytest.raises(I.I18nError, match="invalid message id"):
        I.Catalog("en", {"Bad ID!": "x"})
    with pytest.raises(I.I18nError, match="English"):
        I.Bundle([I.Catalog("ja", {})])


def test_missing_translations_for_a_partial_catalog():
    b = I.Bundle([I.Catalog("en", {"a.b": "x", "c.d": "y"}), I.Catalog("ja", {"a.b": "ｘ"})])
    assert b.missing_translations("ja") == ["c.d"] and b.missing_translations("ko") == ["a.b", "c.d"]
    assert b.languages() == ["en", "ja"]


@pytest.mark.parametrize("tag,want", [("", "en"), ("ja", "ja"), ("JA", "ja"), ("zh-CN", "zh"), ("pt_BR", "pt"),
                                      ("es-419", "es"), ("xx", "en"), ("tlh-KX", "en"), ("ar", "ar")])
def test_detect_lang(tag, want):
    assert I.detect_lang(tag) == want


@pytest.mark.parametrize("env,want", [({}, "en"), ({"LANG": "ja_JP.UTF-8"}, "ja"), ({"LANG": "C"}, "en"),
                                      ({"LANG": "POSIX"}, "en"), ({"LC_ALL": "de_DE@euro", "LANG": "ja_JP"}, "de"),
                                      ({"LC_MESSAGES": "ko_KR.UTF-8", "LANG": "fr_FR"}, "ko"),
                                      ({"LC_ALL": "", "LANG": "ru_RU.UTF-8"}, "ru"), ({"LANG": "C.UTF-8"}, "en")])
def test_detect_lang_from_env(env, want):
    assert I.detect_lang_from_env(env.get) == want


# ================================================================== HAL
@pytest.mark.parametrize("ident,ok", [
    (hal.Identity("gpu-0", hal.Family.GPU), True), (hal.Identity("cpu-0", hal.Family.CPU, "x", "y"), True),
    (hal.Identity("", hal.Family.GPU), False), (hal.Identity("a b", hal.Family.GPU), False),
    (hal.Identity("a/b", hal.Family.GPU), False), (hal.Identity("a\tb", hal.Family.GPU), False),
    (hal.Identity("ok", "gpu"), False),
])
def test_identity_validate(ident, ok):
    if ok:
        ident.validate()
    else:
        with pytest.raises(hal.HalError):
            ident.validate()


def test_identity_str():
    assert str(hal.Identity("gpu-0", hal.Family.GPU)) == "gpu[gpu-0: unknown]"
    assert str(hal.Identity("gpu-0", hal.Family.GPU, "AMD", "MI355X")) == "gpu[gpu-0: MI355X]"


@pytest.mark.parametrize("algo,want", [("sha256d", True), ("scrypt", True), ("x11", True), ("ethash", False)])
def test_gfx950_capabilities(algo, want):
    assert hal.KERNEL_ISAS["gfx950"].supports(algo) is want


def test_registry_rules():
    r = hal.Registry()
    r.register(hal.CPUDriver(2))
    with pytest.raises(hal.HalError, match="already registered"):
        r.register(hal.CPUDriver(2))
    with pytest.raises(hal.HalError, match="nil"):
        r.register(None)

    class Nameless:
        def name(self):
            return ""

    with pytest.raises(hal.HalError, match="non-empty"):
        r.register(Nameless())
    assert len(r) == 1 and r.lookup("cpu") is not None and r.lookup("nope") is None


def test_cpu_driver_device():
    (d,) = hal.CPUDriver(3).enumerate()
    assert d.identity().id == "cpu-0" and d.identity().family == hal.Family.CPU and d.threads == 3
    assert d.capabilities().sha256d and d.capabilities().general_compute and d.capabilities().scrypt  # host chains


class _Drv:
    def __init__(self, name, devs=(), exc=None, delay=0.0):
        self._name, self.devs, self.exc, self.delay = name, list(devs), exc, delay

    def name(self):
        return self._name

    def enumerate(self):
        time.sleep(self.delay)
        if self.exc:
            raise self.exc
        return self.devs


def _dev(did, fam=hal.Family.GPU):
    return hal.SimpleDevice(hal.Identity(did, fam), hal.Capabilities())


def test_detector_merges_sorts_and_tolerates_partial_failure():
    r = hal.Registry()
    r.register(_Drv("b", [_dev("gpu-1"), _dev("gpu-0")]))
    r.register(_Drv("a", exc=RuntimeError("driver exploded")))
    r.register(_Drv("c", [_dev("bad id"), _dev("cpu-0", hal.Family.CPU)]))
    logs = []
    got = hal.Detector(r, logger=lambda n, m, e: logs.append((n, m))).detect()
    assert [d.identity().id for d in got] == ["cpu-0", "gpu-0", "gpu-1"]
    assert ("a", "enumerate failed") in logs and ("c", "device rejected due to invalid identity") in logs


def test_detector_runs_drivers_concurrently_and_abandons_a_hung_one():
    r = hal.Registry()
    r.register(_Drv("slow1", [_dev("gpu-0")], delay=0.3))
    r.register(_Drv("slow2", [_dev("gpu-1")], delay=0.3))
    r.register(_Drv("hung", [_dev("gpu-9")], delay=30))
    logs = []
    t0 = time.perf_counter()
    got = hal.Detector(r, logger=lambda n, m, e: logs.append((n, m)), timeout=1.0).detect()
    dt = time.perf_counter() - t0
    assert [d.identity().id for d in got] == ["gpu-0", "gpu-1"] and dt < 2.0
    assert ("hung", "enumerate timed out") in logs


def test_detector_with_no_drivers():
    assert hal.Detector(hal.Registry()).detect() == []


@pytest.mark.parametrize("vid,want", [("0x1002", "AMD"), ("0x10de", "NVIDIA"), ("0x8086", "Intel"),
                                      (" 0x1002\n", "AMD"), ("0xffff", "Unknown GPU vendor")])
def test_infer_vendor_name(vid, want):
    assert hal.infer_vendor_name(vid) == want


def _fake_sysfs(tmp_path, nodes):
    base = tmp_path / "drm"
    base.mkdir()
    for name, vendor, pci in nodes:
        dev = tmp_path / "devices" / name
        dev.mkdir(parents=True)
        if vendor is not None:
            (dev / "vendor").write_text(vendor + "\n")
        (dev / "uevent").write_text(f"DRIVER=amdgpu\nPCI_ID={pci}\n" if pci else "DRIVER=x\n")
        (base / name).mkdir()
        os.symlink(dev, base / name / "device")
    (base / "card0").mkdir()  # non-render nodes are skipped
    return str(base)


def test_drm_driver_enumerates_render_nodes(tmp_path):
    base = _fake_sysfs(tmp_path, [("renderD128", "0x1002", "1002:75A3"), ("renderD129", "0x10de", None),
                                  ("renderD130", None, None)])
    devs = hal.GPULinuxDriver(base).enumerate()
    assert [d.identity().id for d in devs] == ["gpu-renderD128", "gpu-renderD129"]
    assert devs[0].identity().model == "AMD GPU (1002:75A3)" and devs[1].identity().model == "NVIDIA GPU"
    assert not devs[0].capabilities().sha256d and devs[0].capabilities().general_compute


def test_drm_driver_skips_vendors_and_dedupes_shared_devices(tmp_path):
    base = _fake_sysfs(tmp_path, [("renderD128", "0x1002", None), ("renderD129", "0x8086", None)])
    os.symlink(tmp_path / "devices" / "renderD129", tmp_path / "drm" / "renderD129b")
    (tmp_path / "drm" / "renderD129b").rename(tmp_path / "drm" / "renderD131")
    devs = hal.GPULinuxDriver(base, skip_vendors=("0x1002",)).enumerate()
    assert [d.identity().vendor for d in devs] == ["Intel"]


def test_drm_driver_missing_base_path(tmp_path):
    assert hal.GPULinuxDriver(str(tmp_path / "nope")).enumerate() == []


def test_hip_driver_with_a_fake_runtime():
    class N:
        def gpu_device_count(self):
            return 2

        def gpu_arch_name(self, i):
            return "gfx950:sramecc+:xnack-" if i == 0 else "gfx942"

        def gpu_cu_count(self, i):
            return 256 if i == 0 else 304

    devs = hal.HIPDriver(lambda: N()).enumerate()
    assert [d.identity().id for d in devs] == ["gpu-0", "gpu-1"]
    assert devs[0].capabilities().sha256d and devs[0].capabilities().scrypt and devs[0].index == 0
    assert "MI355X" in devs[0].identity().model and devs[0].extra == {"arch": "gfx950", "cus": 256}
    assert not devs[1].capabilities().sha256d and devs[1].capabilities().general_compute


@pytest.mark.parametrize("loader", [lambda: None, lambda: (_ for _ in ()).throw(RuntimeError("no hip"))])
def test_hip_driver_without_a_runtime(loader):
    assert hal.HIPDriver(loader).enumerate() == []


def test_default_registry_drivers():
    names = [d.name() for d in hal.default_registry(1).drivers()]
    assert names == ["cpu", "gpu_linux", "hip"]
    assert [d.name() for d in hal.default_registry(1, include_drm=False).drivers()] == ["cpu", "hip"]


def test_simple_device_shutdown_is_a_noop():
    assert _dev("gpu-0").shutdown() is None


def test_detector_is_thread_safe_under_concurrent_calls():
    r = hal.Registry()
    r.register(_Drv("a", [_dev("gpu-0")], delay=0.05))
    out = []
    ts = [threading.Thread(target=lambda: out.append(len(hal.Detector(r).detect()))) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(5)
    assert out == [1] * 8


def test_kfd_topology_reads_gpu_to_gpu_links(tmp_path, monkeypatch):
    """hal.kfd_topology: GPU nodes in HIP ordinal order (CPU nodes skipped), their hive ids, and the directed
    GPU-to-GPU io_links with their type named (11 = xgmi, 2 = pcie); links to CPU nodes are left out."""
    from otedama_amd import hal

    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)

    def node(n, props, links=()):
        d = tmp_path / str(n)
        d.mkdir()
        (d / "properties").write_text("\n".join(f"{k} {v}" for k, v in props.items()) + "\n")
        for i, lp in enumerate(links):
            ld = d / "io_links" / str(i)
            ld.mkdir(parents=True)
            (ld / "properties").write_text("\n".join(f"{k} {v}" for k, v in lp.items()) + "\n")

    gpu = {"simd_count": 1024, "simd_per_cu": 4, "gfx_target_version": 90500, "hive_id": 77,
           "num_sdma_xgmi_engines": 14}
    node(0, {"simd_count": 0, "cpu_cores_count": 64})
    node(1, gpu, [{"type": 2, "node_from": 1, "node_to": 0, "weight": 20},
                  {"type": 11, "node_from": 1, "node_to": 2, "weight": 15, "max_bandwidth": 50000}])
    node(2, gpu, [{"type": 11, "node_from": 2, "node_to": 1, "weight": 15, "max_bandwidth": 50000}])
    t = hal.kfd_topology(str(tmp_path))
    assert [g["node"] for g in t["gpus"]] == [1, 2] and t["gpus"][0]["hive_id"] == 77
    assert t["links"] == [{"from": 0, "to": 1, "type": "xgmi", "weight": 15, "max_bandwidth": 50000},
                          {"from": 1, "to": 0, "type": "xgmi", "weight": 15, "max_bandwidth": 50000}]
    assert hal.kfd_topology(str(tmp_path / "missing")) == {"gpus": [], "links": []}
