"""Control-plane units: metrics text format, HTTP server, logger, clock, config, CLI, docs sync.

Mirrors internal/metrics/*_test.go, internal/httpserver/server_test.go,
internal/logger/logger_test.go, internal/clock/clock_test.go,
internal/config/config_test.go and cmd/otedama/*_test.go.
"""
import io
import json
import socket
import urllib.error
import urllib.request
from pathlib import Path

import pytest

from otedama_amd import config as C
from otedama_amd.cli import main as cli
from otedama_amd.httpserver import HTTPServer
from otedama_amd.metrics import MetricsError, Registry, format_float
from otedama_amd.utils import logger as L
from otedama_amd.utils.clock import FakeClock

ROOT = Path(__file__).resolve().parent.parent
ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


# ------------------------------------------------------------------ metrics
@pytest.mark.parametrize("v,want", [
    (0.0, "0"), (1.0, "1"), (0.5, "0.5"), (123456.0, "123456"), (1234567.0, "1.234567e+06"),
    (1e21, "1e+21"), (0.0001, "0.0001"), (0.00001, "1e-05"), (-2.5, "-2.5"), (16.36e9, "1.636e+10"),
    (float("inf"), "+Inf"), (float("-inf"), "-Inf"), (float("nan"), "NaN"), (3.125e8, "3.125e+08"),
    (100000.0, "100000"), (0.1 + 0.2, "0.30000000000000004"),
])
def test_format_float_matches_go_g(v, want):
    assert format_float(v) == want


def test_registry_text_format():
    r = Registry()
    c = r.new_counter("otedama_x_total", "X count.")
    c.add(3)
    g = r.new_gauge("otedama_dev", "Per device.", {"device": 'gpu"0'})
    g.set(2.5)
    r.new_gauge("otedama_dev", "Per device.", {"device": "gpu1"}).set(1e7)
    assert r.new_counter("otedama_x_total", "dup") is c  # dedupe
    out = r.render()
    assert out.count("# HELP otedama_dev") == 1 and "# TYPE otedama_dev gauge" in out
    assert 'otedama_dev{device="gpu\\"0"} 2.5' in out and 'otedama_dev{device="gpu1"} 1e+07' in out
    assert "otedama_x_total 3" in out
    assert out.index("otedama_dev") < out.index("otedama_x_total")
    with pytest.raises(MetricsError):
        r.new_gauge("otedama_x_total", "cross-type")
    with pytest.raises(MetricsError):
        r.new_counter("bad-name", "x")
    with pytest.raises(MetricsError):
        r.new_counter("ok_name", "x", {"bad-label": "v"})


# ------------------------------------------------------------------ http
def _get(url):
    try:
        with urllib.request.urlopen(url, timeout=5) as r:
            return r.status, r.read().decode(), r.headers.get("Content-Type")
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode(), e.headers.get("Content-Type")


def test_http_endpoints():
    reg = Registry()
    reg.new_gauge("otedama_hashrate", "H/s").set(5.0)
    srv = HTTPServer("127.0.0.1:0", reg, api={"stats": lambda: {"hashrate": 5.0},
                                               "debug_stats": lambda: {"devices": {"gpu-0": {"faulted": False}}}})
    srv.start()
    base = f"http://{srv.addr}"
    try:
        assert _get(base + "/healthz")[:2] == (200, "ok\n")
        assert _get(base + "/readyz")[0] == 503
        srv.set_ready(True)
        assert _get(base + "/readyz")[0] == 200
        code, body, ctype = _get(base + "/metrics")
        assert code == 200 and "otedama_hashrate 5" in body and "version=0.0.4" in ctype
        code, body, _ = _get(base + "/api/v1/stats")
        assert code == 200 and json.loads(body) == {"hashrate": 5.0}
        assert _get(base + "/api/v1/nope")[0] == 404
        assert _get(base + "/debug/pprof/")[0] == 404  # pprof off by default
        code, body, ctype = _get(base + "/debug/stats")     # debug stats are not behind the pprof opt-in
        assert code == 200 and json.loads(body)["devices"]["gpu-0"] == {"faulted": False} and "json" in ctype
        assert _get(base + "/nothing")[0] == 404
        # websocket upgrade handshake
        host, port = srv.addr.rsplit(":", 1)
        s = socket.create_connection((host, int(port)), timeout=5)
        s.sendall(b"GET /ws HTTP/1.1\r\nHost: x\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                  b"Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nSec-WebSocket-Version: 13\r\n\r\n")
        resp = s.recv(4096)
        s.close()
        assert b"101" in resp.split(b"\r\n")[0] and b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo=" in resp
    finally:
        srv.stop()


def test_http_listen_error():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(1)
    try:
        with pytest.raises(OSError, match="listen"):
            HTTPServer(f"127.0.0.1:{s.getsockname()[1]}", Registry()).start()
    finally:
        s.close()


# ------------------------------------------------------------------ logger / clock
def test_logger_text_and_json():
    w = io.StringIO()
    lg = L.new(L.parse_level("debug"), "text", w).with_attrs(component="engine")
    lg.info("hello world", n=1)
    line = w.getvalue()
    assert "level=INFO" in line and 'msg="hello world"' in line and "component=engine" in line and "n=1" in line
    w = io.StringIO()
    L.new(L.parse_level("warn"), "json", w).info("dropped")
    assert w.getvalue() == ""
    L.new(L.parse_level("info"), "json", w).error("boom", code=7)
    d = json.loads(w.getvalue())
    assert d["level"] == "ERROR" and d["msg"] == "boom" and d["code"] == 7
    assert L.parse_level("loud") == L.parse_level("info")  # unknown -> info (logger.go:75-86)
    assert L.parse_level(" WARNING ") == L.parse_level("warn")
    L.discard().error("nothing")


def test_fake_clock():
    c = FakeClock(100.0)
    c.advance(2.5)
    assert c.now() == 102.5 and c.monotonic() == 102.5
    c.set(5)
    assert c.now() == 5.0


# ------------------------------------------------------------------ config
def test_config_layering_and_validation(tmp_path, monkeypatch):
    p = tmp_path / "c.yaml"
    p.write_text(f"bitcoin_address: {ADDR}\nlog_level: debug\nmining:\n  algorithm: scrypt\n")
    f, warn = C.load_config_file(str(p))
    assert warn is None and f.mining.algorithm == "scrypt"
    monkeypatch.setenv("OTEDAMA_LOG_LEVEL", "warn")
    cfg, origins = C.resolve_with_origins(f, None, C.FlagValues())
    assert cfg.log_level == "warn" and origins["log_level"] == C.ValueOrigin.ENV
    assert origins["bitcoin_address"] == C.ValueOrigin.FILE
    cfg = C.resolve(f, None, C.FlagValues(log_level="error"))
    assert cfg.log_level == "error"
    cfg.validate()
    p.write_text("bitcoin_addres: typo\n")
    f, warn = C.load_config_file(str(p))
    assert warn and "bitcoin_addres" in warn
    with pytest.raises(C.ConfigError):
        C.Config(bitcoin_address="not-an-address").validate()
    assert C.validate_pool_url("http://x") is not None
    assert C.validate_pool_url("stratum+tcp://pool.example:3333") is None


def test_config_pool_noise_fields_validate():
    good = "ab" * 32
    C.Config(bitcoin_address=ADDR, pools=[C.PoolConfig(url="stratum+v2://p:3336", pool_pubkey=good)]).validate()
    C.Config(bitcoin_address=ADDR, pools=[C.PoolConfig(url="stratum+v2tls://p:3336", noise=True)]).validate()
    C.Config(bitcoin_address=ADDR, pools=[C.PoolConfig(url="stratum+v2://p:3336", noise=True,
                                                       noise_suite="legacy")]).validate()
    for bad in (C.PoolConfig(url="stratum+v2://p:3336", noise=True, noise_suite="p256"),
                C.PoolConfig(url="stratum+v2://p:3336", pool_pubkey="xyz"),
                C.PoolConfig(url="stratum+v2://p:3336", pool_pubkey="ab" * 31),
                C.PoolConfig(url="stratum+tcp://p:3333", noise=True)):
        with pytest.raises(C.ConfigError):
            C.Config(bitcoin_address=ADDR, pools=[bad]).validate()


def test_config_example_loads():
    cfg, warn = C.load_config_file(str(ROOT / "config.yaml.example"))
    assert warn is None
    cfg.validate()
    assert len(cfg.pools) == 2 and cfg.pools[0].payout_scheme == "pplns"


# ------------------------------------------------------------------ CLI
def _cli(*args):
    out, err = io.StringIO(), io.StringIO()
    rc = cli.run(list(args), out, err)
    return rc, out.getvalue(), err.getvalue()


def test_cli_basics(monkeypatch, tmp_path):
    monkeypatch.setenv("HOME", str(tmp_path))
    assert _cli()[0] == cli.EXIT_USAGE
    rc, out, _ = _cli("help")
    assert rc == 0 and "Usage:" in out
    rc, out, _ = _cli("version")
    assert rc == 0 and "otedama" in out
    rc, out, _ = _cli("version", "--json")
    assert json.loads(out)["version"]
    assert _cli("frobnicate")[0] == cli.EXIT_USAGE
    assert _cli("run", "--no-such-flag")[0] == cli.EXIT_USAGE
    rc, out, _ = _cli("run", "--help")
    assert rc == 0
    assert _cli("run", "--dry-run")[0] == cli.EXIT_CONFIG  # no address
    rc, out, _ = _cli("run", "--dry-run", "--bitcoin-address", ADDR)
    assert rc == 0 and "dry-run" in out
    rc, out, _ = _cli("config", "validate", "--bitcoin-address", ADDR)
    assert rc == 0 and "valid" in out
    rc, out, _ = _cli("config", "show", "--bitcoin-address", ADDR, "--origin")
    assert rc == 0 and "[flag]" in out and "log_level:       info [default]" in out
    rc, out, _ = _cli("config", "show", "--bitcoin-address", ADDR, "--json")
    assert json.loads(out)["bitcoin_address"] == ADDR
    for shell in ("bash", "zsh", "fish"):
        rc, out, _ = _cli("completion", shell)
        assert rc == 0 and "otedama" in out and "doctor" in out
    assert _cli("completion", "tcsh")[0] == cli.EXIT_USAGE
    assert _cli("service")[0] == cli.EXIT_USAGE


def test_cli_doctor_json(monkeypatch, tmp_path):
    from otedama_amd import doctor

    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.setattr(doctor, "network_check_endpoint", ("127.0.0.1", 1))
    monkeypatch.setattr(doctor, "clock_skew_probe_url", "http://127.0.0.1:1/")
    monkeypatch.setattr(doctor, "dial_timeout", 0.5)
    rc, out, _ = _cli("doctor", "--json", "--bitcoin-address", ADDR, "--data-dir", str(tmp_path / "d"))
    doc = json.loads(out)
    assert rc == doc["exit_code"] and rc in (1, 2)
    names = {c["name"]: c["status"] for c in doc["checks"]}
    assert names["Bitcoin address"] == "pass" and names["Native extension"] == "pass"


# ------------------------------------------------------------------ docs
def test_metrics_doc_in_sync():
    import importlib.util

    spec = importlib.util.spec_from_file_location("gen", ROOT / "tools" / "gen_metrics_doc.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert (ROOT / "docs" / "METRICS.md").read_text() == mod.render(), "run `make docs`"
