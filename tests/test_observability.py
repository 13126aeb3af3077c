"""Metrics registry, HTTP management server, structured logger, clock and build metadata.

Mirrors internal/metrics/metrics_test.go + runtime_test.go, internal/httpserver/server_test.go,
internal/logger/logger_test.go, internal/clock/clock_test.go and internal/version/version_test.go.
"""
from __future__ import annotations

import base64
import hashlib
import http.client
import io
import json
import math
import socket
import struct
import threading
import time

import pytest

from otedama_amd import httpserver as H
from otedama_amd import metrics as MT
from otedama_amd import version as V
from otedama_amd.utils import clock as CK
from otedama_amd.utils import logger as L


# ------------------------------------------------------------------ counters / gauges
def test_counter_semantics():
    r = MT.Registry()
    c = r.new_counter("otd_x_total", "x")
    assert c.value() == 0
    c.inc()
    c.add(41)
    assert c.value() == 42
    with pytest.raises(MT.MetricsError):
        c.add(-1)
    assert r.new_counter("otd_x_total", "other help") is c  # duplicate name returns the existing series
    c2 = r.new_counter("otd_x_total", "x", {"status": "ok"})
    assert c2 is not c and c2.value() == 0


def test_counter_concurrent_inc_is_atomic():
    c = MT.Registry().new_counter("otd_c_total", "c")
    ts = [threading.Thread(target=lambda: [c.inc() for _ in range(5000)]) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert c.value() == 40000


def test_counter_add_wraps_at_u64():
    c = MT.Registry().new_counter("otd_w_total", "w")
    c.add((1 << 64) - 1)
    c.add(2)
    assert c.value() == 1


def test_gauge_semantics():
    r = MT.Registry()
    g = r.new_gauge("otd_g", "g")
    g.set(3.5)
    g.set(1.25)
    assert g.value() == 1.25
    g.add(0.75)
    assert g.value() == 2.0 and r.new_gauge("otd_g", "g") is g


@pytest.mark.parametrize("name", ["otd_ok", "a", "_x", "ns:sub_total", "A1"])
def test_valid_metric_names(name):
    MT.Registry().new_counter(name, "h")


@pytest.mark.parametrize("name", ["", "1abc", "has-dash", "sp ace", "ünï", "a.b"])
def test_invalid_metric_names(name):
    with pytest.raises(MT.MetricsError, match="invalid metric name"):
        MT.Registry().new_counter(name, "h")
    with pytest.raises(MT.MetricsError, match="invalid metric name"):
        MT.Registry().new_gauge(name, "h")


@pytest.mark.parametrize("label,ok", [("status", True), ("_x", True), ("a1", True), ("1a", False), ("a:b", False),
                                      ("a-b", False), ("", False)])
def test_label_names(label, ok):
    r = MT.Registry()
    if ok:
        r.new_gauge("otd_l", "h", {label: "v"})
    else:
        with pytest.raises(MT.MetricsError, match="invalid label name"):
            r.new_gauge("otd_l", "h", {label: "v"})


def test_cross_type_name_clash_across_label_sets():
    r = MT.Registry()
    r.new_counter("otd_clash", "h", {"a": "1"})
    with pytest.raises(MT.MetricsError, match="already registered as a counter"):
        r.new_gauge("otd_clash", "h", {"b": "2"})
    r.new_gauge("otd_g2", "h")
    with pytest.raises(MT.MetricsError, match="already registered as a gauge"):
        r.new_counter("otd_g2", "h", {"x": "y"})


# ------------------------------------------------------------------ exposition
def test_write_text_format_ordering_and_help_once():
    r = MT.Registry()
    r.new_gauge("otd_b", "B help").set(2)
    c = r.new_counter("otd_a_total", "A help", {"status": "rejected"})
    c.add(3)
    r.new_counter("otd_a_total", "A help", {"status": "accepted"}).inc()
    assert r.render() == (
        "# HELP otd_a_total A help\n# TYPE otd_a_total counter\n"
        'otd_a_total{status="accepted"} 1\notd_a_total{status="rejected"} 3\n'
        "# HELP otd_b B help\n# TYPE otd_b gauge\notd_b 2\n")


def test_empty_registry_renders_nothing():
    assert MT.Registry().render() == ""


def test_label_values_and_help_are_escaped():
    r = MT.Registry()
    r.new_gauge("otd_e", 'line1\nline2 \\ "q"', {"v": 'a"b\\c\nd'}).set(1)
    out = r.render()
    assert '# HELP otd_e line1\\nline2 \\\\ "q"\n' in out
    assert 'otd_e{v="a\\"b\\\\c\\nd"} 1\n' in out


def test_labels_render_sorted_by_key():
    r = MT.Registry()
    r.new_gauge("otd_m", "h", {"z": "1", "a": "2", "m": "3"}).set(0)
    assert 'otd_m{a="2",m="3",z="1"} 0' in r.render()


@pytest.mark.parametrize("v,want", [(math.nan, "NaN"), (math.inf, "+Inf"), (-math.inf, "-Inf"), (0.0, "0"),
                                    (-0.0, "-0"), (1.0, "1"), (0.5, "0.5"), (123456.0, "123456"),
                                    (1234567.0, "1.234567e+06"), (1e21, "1e+21"), (0.0001, "0.0001"),
                                    (0.00001, "1e-05"), (-2.5e-7, "-2.5e-07"), (18756971599.625828, "1.8756971599625828e+10"),
                                    (100.0, "100"), (1e6, "1e+06"), (999999.0, "999999"), (3.14159, "3.14159")])
def test_format_float_matches_go_percent_g(v, want):
    assert MT.format_float(v) == want


def test_gauge_text_cache_tracks_sign_and_nan():
    g = MT.Registry().new_gauge("otd_n", "n")
    g.set(0.0)
    assert g.text() == "0"
    g.set(-0.0)
    assert g.text() == "-0"
    g.set(math.nan)
    assert g.text() == "NaN"
    g.set(2)
    assert g.text() == "2"


def test_collectors_run_after_static_metrics_in_order():
    r = MT.Registry()
    r.new_gauge("otd_z", "z").set(1)
    r.register_collector(lambda w: w.write("# c1\n"))
    r.register_collector(lambda w: w.write("# c2\n"))
    out = r.render()
    assert out.index("otd_z 1") < out.index("# c1") < out.index("# c2")


def test_collector_errors_propagate():
    r = MT.Registry()

    def boom(w):
        raise OSError("disk full")

    r.register_collector(boom)
    with pytest.raises(OSError):
        r.render()


def test_writer_errors_propagate():
    class Bad(io.StringIO):
        def write(self, s):
            raise OSError("broken pipe")

    r = MT.Registry()
    r.new_gauge("otd_x", "x")
    with pytest.raises(OSError):
        r.write_text(Bad())


def test_names():
    r = MT.Registry()
    r.new_gauge("otd_a", "a")
    r.new_counter("otd_b_total", "b", {"k": "v"})
    assert r.names() == {"otd_a", "otd_b_total"}


def test_runtime_collector_series():
    r = MT.Registry()
    r.register_collector(MT.runtime_collector())
    out = r.render()
    for name in ("python_threads", "python_info", "process_resident_memory_bytes", "process_cpu_seconds_total",
                 "process_start_time_seconds", "python_gc_collections_total"):
        assert f"# HELP {name} " in out and f"# TYPE {name} " in out
    threads = int(next(ln.split()[1] for ln in out.splitlines() if ln.startswith("python_threads ")))
    assert threads >= 1
    assert 'python_info{version="' in out


def test_full_mining_scenario_scrape_is_parseable():
    r = MT.Registry()
    r.new_counter("otedama_shares_total", "Shares", {"status": "accepted"}).add(10)
    r.new_counter("otedama_shares_total", "Shares", {"status": "rejected"}).add(1)
    r.new_gauge("otedama_hashrate_hashes_per_second", "H/s").set(18.8e9)
    for q in ("0.5", "0.95", "0.99"):
        r.new_gauge("otedama_submit_latency_milliseconds", "ms", {"quantile": q}).set(0.2)
    for line in r.render().splitlines():
        if line.startswith("#"):
            assert line.split()[1] in ("HELP", "TYPE")
            continue
        name_labels, value = line.rsplit(" ", 1)
        float(value.replace("+Inf", "inf"))
        assert name_labels.startswith("otedama_")


# ------------------------------------------------------------------ HTTP server
@pytest.fixture
def server():
    r = MT.Registry()
    r.new_gauge("otd_up", "up").set(1)
    s = H.HTTPServer("127.0.0.1:0", r, api={"stats": lambda: {"hashrate": 1.5, "raw": b"\x01\x02"},
                                             "devices": lambda: [{"id": "gpu-0"}],
                                             "boom": lambda: 1 / 0,
                                             "debug_stats": lambda: {"gpu-0": {"launches": 3}}})
    s.start()
    yield s
    s.stop()


def _get(s, path, method="GET", headers=None):
    host, port = s.addr.rsplit(":", 1)
    c = http.client.HTTPConnection(host, int(port), timeout=5)
    c.request(method, path, headers=headers or {})
    r = c.getresponse()
    body = r.read()
    c.close()
    return r.status, dict(r.getheaders()), body


def test_healthz(server):
    st, h, b = _get(server, "/healthz")
    assert (st, b) == (200, b"ok\n") and h["Content-Type"].startswith("text/plain")


def test_readyz_flips(server):
    assert _get(server, "/readyz")[::2] == (503, b"not ready\n")
    server.set_ready(True)
    assert _get(server, "/readyz")[::2] == (200, b"ready\n")
    server.set_ready(False)
    assert _get(server, "/readyz")[0] == 503


def test_metrics_endpoint(server):
    st, h, b = _get(server, "/metrics")
    assert st == 200 and h["Content-Type"] == "text/plain; version=0.0.4; charset=utf-8" and b"otd_up 1\n" in b


def test_metrics_without_registry_is_500():
    s = H.HTTPServer("127.0.0.1:0", None)
    s.start()
    try:
        assert _get(s, "/metrics")[0] == 500
    finally:
        s.stop()


def test_index_and_404(server):
    st, h, b = _get(server, "/")
    assert st == 200 and b"<html>" in b and h["Content-Type"].startswith("text/html")
    assert _get(server, "/nope")[0] == 404
    assert _get(server, "/metricsx")[0] == 404


def test_head_has_no_body(server):
    st, h, b = _get(server, "/healthz", "HEAD")
    assert st == 200 and b == b"" and h["Content-Length"] == "3"


def test_query_string_is_ignored_for_routing(server):
    assert _get(server, "/healthz?x=1")[0] == 200


def test_rest_api(server):
    st, h, b = _get(server, "/api/v1/stats")
    assert st == 200 and h["Content-Type"] == "application/json"
    assert json.loads(b) == {"hashrate": 1.5, "raw": "0102"}
    assert json.loads(_get(server, "/api/v1/devices/")[2]) == [{"id": "gpu-0"}]
    st, _, b = _get(server, "/api/v1/boom")
    assert st == 500 and "division" in json.loads(b)["error"]
    assert _get(server, "/api/v1/missing")[0] == 404


def test_debug_stats(server):
    st, _, b = _get(server, "/debug/stats")
    assert st == 200 and json.loads(b)["gpu-0"]["launches"] == 3


def test_pprof_disabled_by_default(server):
    assert _get(server, "/debug/pprof/")[0] == 404


def test_pprof_enabled_serves_index_and_profiles():
    s = H.HTTPServer("127.0.0.1:0", MT.Registry(), enable_pprof=True)
    s.start()
    try:
        assert b"goroutine" in _get(s, "/debug/pprof/")[2]
        st, _, b = _get(s, "/debug/pprof/goroutine")
        assert st == 200 and b"otedama-http" in b
        assert json.loads(_get(s, "/debug/pprof/heap")[2])["objects"] > 0
        assert _get(s, "/debug/pprof/cmdline")[0] == 200
        st, _, b = _get(s, "/debug/pprof/profile?seconds=0.1")
        assert st == 200 and b"function calls" in b
        assert _get(s, "/debug/pprof/bogus")[0] == 404
    finally:
        s.stop()


def test_concurrent_requests(server):
    errs = []

    def hit():
        try:
            for _ in range(20):
                assert _get(server, "/metrics")[0] == 200
        except Exception as exc:  # noqa: BLE001
            errs.append(exc)

    ts = [threading.Thread(target=hit) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert not errs


def test_start_on_a_bad_address_raises():
    s = H.HTTPServer("256.0.0.1:99999", MT.Registry())
    with pytest.raises((OSError, OverflowError)):
        s.start()


def test_addr_before_and_after_start_and_clean_stop():
    s = H.HTTPServer("127.0.0.1:0", MT.Registry())
    assert s.addr == "127.0.0.1:0"
    s.start()
    assert s.addr.startswith("127.0.0.1:") and not s.addr.endswith(":0")
    s.stop()
    assert s.serve_error() is None


def test_websocket_streams_stats(server):
    host, port = server.addr.rsplit(":", 1)
    sock = socket.create_connection((host, int(port)), timeout=5)
    key = base64.b64encode(b"0123456789abcdef").decode()
    sock.sendall((f"GET /ws HTTP/1.1\r\nHost: x\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                  f"Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\n\r\n").encode())
    buf = b""
    while b"\r\n\r\n" not in buf:
        buf += sock.recv(4096)
    head, rest = buf.split(b"\r\n\r\n", 1)
    assert head.startswith(b"HTTP/1.1 101")
    want = base64.b64encode(hashlib.sha1((key + H.WS_GUID).encode()).digest())
    assert b"Sec-WebSocket-Accept: " + want in head
    while len(rest) < 2:
        rest += sock.recv(4096)
    assert rest[0] == 0x81
    n = rest[1] & 0x7F
    while len(rest) < 2 + n:
        rest += sock.recv(4096)
    assert json.loads(rest[2:2 + n]) == {"hashrate": 1.5, "raw": "0102"}
    sock.sendall(bytes([0x88, 0x80]) + b"\x00" * 4)  # masked close
    sock.close()


def test_websocket_without_upgrade_is_400(server):
    assert _get(server, "/ws")[0] == 400


@pytest.mark.parametrize("n,hdr_len", [(5, 2), (125, 2), (126, 4), (65535, 4), (65536, 10)])
def test_ws_frame_lengths(n, hdr_len):
    f = H.ws_frame(b"x" * n)
    assert len(f) == n + hdr_len and f[0] == 0x81
    if hdr_len == 4:
        assert f[1] == 126 and struct.unpack("!H", f[2:4])[0] == n
    if hdr_len == 10:
        assert f[1] == 127 and struct.unpack("!Q", f[2:10])[0] == n


# ------------------------------------------------------------------ logger
@pytest.mark.parametrize("s,lvl", [("debug", L.DEBUG), ("INFO", L.INFO), ("warn", L.WARN), ("warning", L.WARN),
                                   ("error", L.ERROR), ("", L.INFO), ("bogus", L.INFO), (" Debug ", L.DEBUG)])
def test_parse_level(s, lvl):
    assert L.parse_level(s) == lvl


def test_text_format_quotes_like_slog():
    w = io.StringIO()
    L.new(L.DEBUG, "text", w).info("hello world", k="v", sp="a b", empty="", n=3)
    line = w.getvalue().strip()
    assert line.startswith("time=") and ' level=INFO msg="hello world" k=v sp="a b" empty="" n=3' in line


def test_json_format():
    w = io.StringIO()
    L.new(L.INFO, "json", w).warn("careful", device="gpu-0", rate=1.5)
    d = json.loads(w.getvalue())
    assert d["level"] == "WARN" and d["msg"] == "careful" and d["device"] == "gpu-0" and d["rate"] == 1.5
    assert "time" in d


def test_level_filter():
    w = io.StringIO()
    lg = L.new(L.WARN, "text", w)
    lg.debug("d")
    lg.info("i")
    lg.warn("w")
    lg.error("e")
    assert [ln.split("msg=")[1] for ln in w.getvalue().splitlines()] == ["w", "e"]


def test_discard_writes_nothing(capsys):
    L.discard().error("x")
    assert capsys.readouterr() == ("", "")


def test_adapter_routes_by_level_and_unknown_to_info():
    w = io.StringIO()
    fn = L.new(L.DEBUG, "json", w).adapter()
    for lvl in ("debug", "info", "warn", "error", "weird", ""):
        fn(lvl, lvl or "empty")
    got = [json.loads(x)["level"] for x in w.getvalue().splitlines()]
    assert got == ["DEBUG", "INFO", "WARN", "ERROR", "INFO", "INFO"]


def test_with_attrs_adds_to_every_record():
    w = io.StringIO()
    lg = L.new(L.INFO, "json", w).with_attrs(rank=3)
    lg.info("a")
    lg.info("b", rank=4)
    recs = [json.loads(x) for x in w.getvalue().splitlines()]
    assert recs[0]["rank"] == 3 and recs[1]["rank"] == 4


def test_default_singleton_and_set_default():
    d = L.default()
    assert L.default() is d
    new = L.new()
    L.set_default(new)
    try:
        assert L.default() is new
        L.set_default(None)  # nil does not clobber
        assert L.default() is new
    finally:
        L.set_default(d)


def test_context_round_trip():
    import contextvars

    def inner():
        assert L.from_context() is L.default()
        lg = L.new()
        L.into_context(lg)
        assert L.from_context() is lg
        L.into_context(None)
        assert L.from_context() is lg

    contextvars.copy_context().run(inner)


def test_concurrent_default_access():
    seen = []
    ts = [threading.Thread(target=lambda: seen.append(L.default())) for _ in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all(x is seen[0] for x in seen)


def test_closed_writer_does_not_raise():
    w = io.StringIO()
    lg = L.new(L.INFO, "text", w)
    w.close()
    lg.info("after close")


# ------------------------------------------------------------------ clock / version
def test_system_clock_tracks_time():
    c = CK.SystemClock()
    assert abs(c.now() - time.time()) < 1 and c.monotonic() <= time.monotonic()


def test_fake_clock_set_and_advance():
    c = CK.FakeClock(100)
    assert c.now() == 100 and c.monotonic() == 100
    c.advance(2.5)
    assert c.now() == 102.5
    c.set(7)
    assert c.now() == 7


def test_fake_clock_concurrent_advance():
    c = CK.FakeClock()
    ts = [threading.Thread(target=lambda: [c.advance(1) for _ in range(1000)]) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert c.now() == 8000


def test_version_info(monkeypatch):
    monkeypatch.setattr(V, "_cached", None)
    monkeypatch.setenv("OTEDAMA_VERSION", "v9.9.9")
    monkeypatch.setenv("OTEDAMA_COMMIT", "abc1234")
    monkeypatch.setenv("OTEDAMA_BUILD_DATE", "2026-01-01")
    info = V.get()
    assert (info.version, info.commit, info.build_date, info.gpu_arch) == ("v9.9.9", "abc1234", "2026-01-01", "gfx950")
    assert str(info).startswith("otedama v9.9.9 (abc1234) built 2026-01-01")
    assert set(info.to_dict()) == {"version", "commit", "build_date", "python_version", "platform", "gpu_arch"}
    assert V.get() is info
    monkeypatch.setattr(V, "_cached", None)


def test_version_defaults(monkeypatch):
    monkeypatch.setattr(V, "_cached", None)
    for k in ("OTEDAMA_VERSION", "OTEDAMA_COMMIT", "OTEDAMA_BUILD_DATE"):
        monkeypatch.delenv(k, raising=False)
    info = V.get()
    assert info.version == V.VERSION and info.commit and info.build_date == "unknown"
    monkeypatch.setattr(V, "_cached", None)
