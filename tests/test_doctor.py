"""doctor: report format, exit codes, individual checks (internal/doctor/*_test.go)."""
import io
import json
import socket
import threading

import pytest

from otedama_amd import config as C
from otedama_amd import doctor as D

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


def _report(*statuses):
    return D.Report([D.Result(f"c{i}", s, "d", "f" if s == D.Status.FAIL else "") for i, s in enumerate(statuses)],
                    0.012)


def test_exit_codes_and_print():
    assert _report(D.Status.PASS, D.Status.SKIP).exit_code() == 0
    assert _report(D.Status.PASS, D.Status.WARN).exit_code() == 1
    assert _report(D.Status.WARN, D.Status.FAIL).exit_code() == 2
    w = io.StringIO()
    _report(D.Status.PASS, D.Status.FAIL, D.Status.WARN, D.Status.SKIP).print(w)
    out = w.getvalue()
    assert "[✓] c0: d" in out and "[✗] c1: d\n    → fix: f" in out and "[!] c2" in out and "[-] c3" in out
    assert "Summary: 1 passed, 1 failed, 1 warning, 1 skipped (completed in 12ms)" in out


def test_json():
    w = io.StringIO()
    _report(D.Status.PASS, D.Status.WARN, D.Status.WARN).write_json(w)
    doc = json.loads(w.getvalue())
    assert doc["summary"] == {"passed": 1, "failed": 0, "warnings": 2, "skipped": 0}
    assert doc["exit_code"] == 1 and doc["checks"][1]["status"] == "warn"


def test_runner_parallel_timeout_and_crash():
    ev = threading.Event()

    def slow():
        ev.wait(2)
        return D.Result()

    def boom():
        raise RuntimeError("x")

    rep = D.Runner([D.Check("ok", lambda: D.Result(detail="fine")), D.Check("slow", slow),
                    D.Check("boom", boom)], timeout=0.2).run()
    ev.set()
    by = {r.name: r for r in rep.results}
    assert [r.name for r in rep.results] == ["ok", "slow", "boom"]
    assert by["ok"].status == D.Status.PASS and by["slow"].status == D.Status.FAIL
    assert "crashed" in by["boom"].detail


def _cfg(**kw):
    c = C.Config(bitcoin_address=ADDR)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_address_checks():
    assert D.check_bitcoin_address(_cfg()).run().status == D.Status.PASS
    assert D.check_bitcoin_address(_cfg(bitcoin_address="")).run().status == D.Status.FAIL
    assert D.check_bitcoin_address(_cfg(bitcoin_address=ADDR[:-1] + "x")).run().status == D.Status.FAIL
    assert D.check_failover_addresses(_cfg()).run().status == D.Status.SKIP
    assert D.check_failover_addresses(_cfg(bitcoin_addresses=[ADDR])).run().status == D.Status.WARN


def test_pool_checks(monkeypatch):
    one = [C.PoolConfig(url="stratum+tcp://127.0.0.1:1")]
    assert D.check_pool_diversity(_cfg()).run().status == D.Status.WARN
    assert D.check_pool_diversity(_cfg(pools=one)).run().status == D.Status.WARN
    two = one + [C.PoolConfig(url="stratum+tls://127.0.0.1:2", payout_scheme="pplns")]
    assert D.check_pool_diversity(_cfg(pools=two)).run().status == D.Status.PASS
    assert D.check_pool_encryption(_cfg(pools=two)).run().status == D.Status.WARN
    r = D.check_pool_endpoint_diversity(_cfg(pools=two)).run()
    assert r.status == D.Status.WARN and "same endpoint" in r.detail
    r = D.check_payout_scheme(_cfg(pools=two)).run()
    assert "PPLNS" in r.detail and r.fix
    # reachability against a real loopback listener
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(4)
    port = srv.getsockname()[1]
    try:
        good = [C.PoolConfig(url=f"stratum+tcp://127.0.0.1:{port}")]
        assert D.check_pool_reachability(_cfg(pools=good)).run().status == D.Status.PASS
        monkeypatch.setattr(D, "dial_timeout", 0.5)
        mixed = good + [C.PoolConfig(url="stratum+tcp://127.0.0.1:1")]
        assert D.check_pool_reachability(_cfg(pools=mixed)).run().status == D.Status.WARN
    finally:
        srv.close()


def test_tls_ca_and_data_dir(tmp_path):
    bad = tmp_path / "ca.pem"
    bad.write_text("not pem")
    p = [C.PoolConfig(url="stratum+tls://x:1", tls_ca_file=str(bad))]
    assert D.check_pool_tls_ca(_cfg(pools=p)).run().status == D.Status.FAIL
    p = [C.PoolConfig(url="stratum+tls://x:1", tls_ca_file=str(tmp_path / "missing"))]
    assert D.check_pool_tls_ca(_cfg(pools=p)).run().status == D.Status.FAIL
    d = tmp_path / "dd"
    assert D.check_data_dir(_cfg(data_dir=str(d))).run().status == D.Status.WARN  # created on first run
    d.mkdir(mode=0o755)
    d.chmod(0o755)
    assert D.check_data_dir(_cfg(data_dir=str(d))).run().status == D.Status.WARN
    d.chmod(0o700)
    assert D.check_data_dir(_cfg(data_dir=str(d))).run().status == D.Status.PASS
    assert D.check_wallet(_cfg(data_dir=str(d))).run().status == D.Status.WARN
    (d / "wallet.dat").write_bytes(b"\x01short")
    assert D.check_wallet(_cfg(data_dir=str(d))).run().status == D.Status.FAIL


def test_misc_checks(monkeypatch):
    assert D.check_power_cost(_cfg()).run().status == D.Status.SKIP
    assert D.check_power_cost(_cfg(power_watts=1400)).run().status == D.Status.WARN
    r = D.check_power_cost(_cfg(power_watts=1400, electricity_price_per_kwh=0.1)).run()
    assert r.status == D.Status.PASS and "$0.1400/h" in r.detail
    assert D.check_profitability_floor(_cfg()).run().status == D.Status.SKIP
    monkeypatch.setenv("OTEDAMA_POWER_WATTS", "abc")
    assert D.check_env_vars().run().status == D.Status.WARN
    monkeypatch.setattr(D, "clock_skew_probe_url", "http://127.0.0.1:1/")
    monkeypatch.setattr(D, "dial_timeout", 0.5)
    assert D.check_clock().run().status == D.Status.WARN
    assert D.check_native().run().status == D.Status.PASS
    assert D.check_collectives().run().status in (D.Status.PASS, D.Status.WARN)


def test_default_checks_names():
    names = [c.name for c in D.default_checks(_cfg())]
    for want in ("Configuration", "Bitcoin address", "Failover payout addresses", "Data directory",
                 "Lightning wallet", "Pool reachability", "Pool diversity", "Pool endpoint diversity",
                 "Pool connection encryption", "Pool TLS CA files", "Power & cost config", "Environment variables",
                 "Profitability floor", "Pool payout schemes", "Hardware", "Network", "System clock accuracy",
                 "Native extension", "GPU runtime", "Collectives"):
        assert want in names


@pytest.mark.parametrize("algo", ["sha256d", "scrypt", "x11"])
def test_pow_self_test_check(algo):
    from otedama_amd import config as C

    cfg = C.Config()
    cfg.mining.algorithm = algo
    r = D.check_pow_self_test(cfg).run()
    assert r.status == D.Status.PASS, r.detail
    assert algo in r.detail


def test_pow_self_test_detects_a_wrong_oracle(monkeypatch):
    from otedama_amd import config as C
    from otedama_amd.models import algorithms

    bad = algorithms.PowAlgorithm("x11", algorithms.ALGORITHMS["x11"].diff1, lambda h: bytes(32), True, "broken")
    monkeypatch.setitem(algorithms.ALGORITHMS, "x11", bad)
    cfg = C.Config()
    cfg.mining.algorithm = "x11"
    r = D.check_pow_self_test(cfg).run()
    assert r.status == D.Status.FAIL and "genesis" in r.detail
