"""Doctor: every check's pass / warn / fail / skip branch, the report formats and the parallel runner.

Mirrors internal/doctor/{doctor,checks,extras}_test.go (TestStatus_*, TestReport_*, TestRunner_*,
TestCheck<Name>_* with the injectable pool dialer, DNS resolver, network endpoint and clock-probe seams).
"""
from __future__ import annotations

import email.utils
import http.server
import io
import json
import os
import ssl
import threading
import time

import pytest

from otedama_amd import config as C
from otedama_amd import doctor as D

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"
ADDR2 = "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa"


def run(check) -> D.Result:
    return check.run()


def cfg(**kw) -> C.Config:
    c = C.Config(bitcoin_address=ADDR)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def pools(*urls, **kw):
    return [C.PoolConfig(url=u, **kw) for u in urls]


# ------------------------------------------------------------------ status / report / runner
def test_status_strings_and_symbols():
    assert [str(s) for s in D.Status] == ["pass", "warn", "fail", "skip"]
    assert [s.symbol for s in D.Status] == ["✓", "!", "✗", "-"]


@pytest.mark.parametrize("statuses,code", [([], 0), ([D.Status.PASS], 0), ([D.Status.SKIP], 0),
                                           ([D.Status.PASS, D.Status.WARN], 1), ([D.Status.WARN, D.Status.FAIL], 2),
                                           ([D.Status.FAIL], 2)])
def test_exit_code(statuses, code):
    assert D.Report([D.Result("x", s) for s in statuses]).exit_code() == code


def test_report_print_summary_and_fix_lines():
    r = D.Report([D.Result("A", D.Status.PASS, "fine"), D.Result("B", D.Status.WARN, "meh", "do this"),
                  D.Result("C", D.Status.SKIP, "n/a")], 0.0123)
    w = io.StringIO()
    r.print(w)
    out = w.getvalue()
    assert "[✓] A: fine\n" in out and "[!] B: meh\n    → fix: do this\n" in out and "[-] C: n/a" in out
    assert out.rstrip().endswith("Summary: 1 passed, 0 failed, 1 warning, 1 skipped (completed in 12ms)")


def test_report_warning_plural():
    w = io.StringIO()
    D.Report([D.Result("a", D.Status.WARN), D.Result("b", D.Status.WARN)]).print(w)
    assert "2 warnings" in w.getvalue()


def test_report_json():
    w = io.StringIO()
    D.Report([D.Result("A", D.Status.FAIL, "bad", "fix it", 0.5), D.Result("B")], 1.0).write_json(w)
    doc = json.loads(w.getvalue())
    assert doc["summary"] == {"passed": 1, "failed": 1, "warnings": 0, "skipped": 0}
    assert doc["exit_code"] == 2 and doc["duration_ms"] == 1000
    assert doc["checks"][0] == {"name": "A", "status": "fail", "detail": "bad", "fix": "fix it", "elapsed_ms": 500}
    assert "fix" not in doc["checks"][1]


def test_runner_runs_checks_in_parallel_keeps_order_and_names():
    def slow(tag):
        def f():
            time.sleep(0.3)
            return D.Result(detail=tag)
        return f

    checks = [D.Check(f"c{i}", slow(str(i))) for i in range(6)]
    t0 = time.monotonic()
    rep = D.Runner(checks).run()
    assert time.monotonic() - t0 < 1.5
    assert [r.name for r in rep.results] == [f"c{i}" for i in range(6)] and [r.detail for r in rep.results] == list("012345")
    assert all(r.elapsed >= 0.29 for r in rep.results)


def test_runner_crash_becomes_fail():
    rep = D.Runner([D.Check("boom", lambda: 1 / 0)]).run()
    assert rep.results[0].status == D.Status.FAIL and "check crashed" in rep.results[0].detail


def test_runner_timeout_does_not_wait_for_a_hung_check():
    rep_t0 = time.monotonic()
    rep = D.Runner([D.Check("hung", lambda: time.sleep(30) or D.Result()), D.Check("ok", lambda: D.Result())],
                   timeout=0.5).run()
    assert time.monotonic() - rep_t0 < 2
    assert rep.results[0].status == D.Status.FAIL and rep.results[0].detail == "check timed out"
    assert rep.results[1].status == D.Status.PASS


def test_runner_with_no_checks():
    rep = D.Runner([]).run()
    assert rep.results == [] and rep.exit_code() == 0


# ------------------------------------------------------------------ configuration / address
def test_configuration_check(tmp_path):
    r = run(D.check_configuration(cfg(), ""))
    assert r.status == D.Status.WARN and "no config file found" in r.detail and "config.yaml.example" in r.fix
    r = run(D.check_configuration(cfg(), str(tmp_path / "absent.yaml")))
    assert r.status == D.Status.WARN and "not found" in r.detail and "--config" in r.fix
    p = tmp_path / "c.yaml"
    p.write_text("")
    r = run(D.check_configuration(cfg(), str(p)))
    assert r.status == D.Status.PASS and r.detail == f"loaded from {p}"
    r = run(D.check_configuration(C.Config(), str(p)))
    assert r.status == D.Status.FAIL and "bitcoin_address is required" in r.detail and "\n" not in r.detail
    assert r.fix
    # without a file the validation errors ride along on the warning
    r = run(D.check_configuration(C.Config(), ""))
    assert r.status == D.Status.WARN and "bitcoin_address is required" in r.detail


@pytest.mark.parametrize("c,status,needle", [
    (cfg(), D.Status.PASS, "likely valid"),
    (C.Config(bitcoin_address=ADDR2), D.Status.PASS, "P2PKH legacy"),
    (C.Config(), D.Status.FAIL, "no address configured"),
    (C.Config(bitcoin_addresses=[ADDR]), D.Status.WARN, "failover list only"),
    (C.Config(bitcoin_address=ADDR[:-1] + "x"), D.Status.FAIL, "checksum"),
])
def test_bitcoin_address_check(c, status, needle):
    r = run(D.check_bitcoin_address(c))
    assert r.status == status and needle.lower() in r.detail.lower()


@pytest.mark.parametrize("lst,status", [([], D.Status.SKIP), ([ADDR2], D.Status.PASS), ([ADDR2, ADDR2], D.Status.WARN),
                                        ([ADDR], D.Status.WARN), ([ADDR2, "bogus"], D.Status.FAIL)])
def test_failover_addresses_check(lst, status):
    assert run(D.check_failover_addresses(cfg(bitcoin_addresses=lst))).status == status


# ------------------------------------------------------------------ data dir / wallet
def test_data_dir_check(tmp_path):
    d = tmp_path / "d"
    r = run(D.check_data_dir(cfg(data_dir=str(d))))
    assert r.status == D.Status.WARN and "will be created on first run" in r.detail
    d.mkdir(mode=0o700)
    r = run(D.check_data_dir(cfg(data_dir=str(d))))
    assert r.status == D.Status.PASS and "(exists, writable)" in r.detail
    os.chmod(d, 0o755)
    r = run(D.check_data_dir(cfg(data_dir=str(d))))
    assert r.status == D.Status.WARN and "0755" in r.detail and "chmod 0700" in r.fix
    f = tmp_path / "file"
    f.write_text("")
    r = run(D.check_data_dir(cfg(data_dir=str(f))))
    assert r.status == D.Status.FAIL and "not a directory" in r.detail and r.fix
    assert run(D.check_data_dir(cfg(data_dir=""))).status in (D.Status.WARN, D.Status.SKIP, D.Status.PASS)


@pytest.mark.skipif(os.geteuid() == 0, reason="root bypasses permission bits")
def test_data_dir_not_writable(tmp_path):
    d = tmp_path / "ro"
    d.mkdir(mode=0o500)
    assert run(D.check_data_dir(cfg(data_dir=str(d)))).status == D.Status.FAIL


def test_wallet_check(tmp_path):
    from otedama_amd.lightning import seedstore

    r = run(D.check_wallet(cfg(data_dir=str(tmp_path))))
    assert r.status == D.Status.WARN and "no wallet found" in r.detail and "wallet-passphrase" in r.fix
    w = tmp_path / "wallet.dat"
    w.write_bytes(b"garbage")
    os.chmod(w, 0o600)
    assert run(D.check_wallet(cfg(data_dir=str(tmp_path)))).status == D.Status.FAIL
    # format check only (no KDF): version 0x01 | salt 16 | nonce 12 | ciphertext+tag
    w.write_bytes(seedstore.EncryptedSeed(seedstore.VERSION, os.urandom(16), os.urandom(12), os.urandom(80)).marshal())
    assert run(D.check_wallet(cfg(data_dir=str(tmp_path)))).status == D.Status.PASS
    os.chmod(w, 0o644)
    assert run(D.check_wallet(cfg(data_dir=str(tmp_path)))).status == D.Status.WARN


# ------------------------------------------------------------------ pools
def test_pool_targets_default_ports():
    c = cfg(pools=pools("stratum+tcp://a.example", "stratum+v2://b.example", "stratum+tls://c.example:443",
                        "junk://x"))
    assert D._pool_targets(c) == [("stratum+tcp://a.example", "a.example", 3333),
                                  ("stratum+v2://b.example", "b.example", 3336),
                                  ("stratum+tls://c.example:443", "c.example", 443)]
    assert D._pool_targets(cfg())[0][0] == C.DEFAULT_POOL_URL


def test_pool_reachability(monkeypatch):
    up = {"a.example"}

    def dial(host, port, timeout):
        if host not in up:
            raise ConnectionRefusedError("refused")

    monkeypatch.setattr(D, "pool_dial", dial)
    c = cfg(pools=pools("stratum+tcp://a.example:1", "stratum+tcp://b.example:2"))
    r = run(D.check_pool_reachability(c))
    assert r.status == D.Status.WARN and "b.example" in r.detail
    up.add("b.example")
    assert run(D.check_pool_reachability(c)).status == D.Status.PASS
    up.clear()
    assert run(D.check_pool_reachability(c)).status == D.Status.FAIL


def test_pool_reachability_real_loopback_dial():
    import socket

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    try:
        assert run(D.check_pool_reachability(cfg(pools=pools(f"stratum+tcp://127.0.0.1:{port}")))).status == D.Status.PASS
    finally:
        srv.close()


@pytest.mark.parametrize("n,status", [(0, D.Status.WARN), (1, D.Status.WARN), (2, D.Status.PASS), (3, D.Status.PASS)])
def test_pool_diversity(n, status):
    c = cfg(pools=pools(*[f"stratum+tcp://p{i}.example:3333" for i in range(n)]))
    assert run(D.check_pool_diversity(c)).status == status


def test_pool_endpoint_diversity(monkeypatch):
    table = {"a.example": ["10.0.0.1"], "b.example": ["10.0.0.2"], "c.example": ["10.0.0.1", "10.0.0.9"]}

    def resolve(host):
        if host not in table:
            raise OSError("nxdomain")
        return table[host]

    monkeypatch.setattr(D, "resolve_host", resolve)
    two = lambda a, b: cfg(pools=pools(f"stratum+tcp://{a}:1", f"stratum+tcp://{b}:1"))  # noqa: E731
    assert run(D.check_pool_endpoint_diversity(two("a.example", "b.example"))).status == D.Status.PASS
    r = run(D.check_pool_endpoint_diversity(two("a.example", "c.example")))
    assert r.status == D.Status.WARN and "10.0.0.1" in r.detail and "illusory" in r.detail
    assert run(D.check_pool_endpoint_diversity(two("a.example", "nx.example"))).status == D.Status.SKIP
    assert run(D.check_pool_endpoint_diversity(cfg(pools=pools("stratum+tcp://a.example")))).status == D.Status.SKIP


@pytest.mark.parametrize("urls,status", [((), D.Status.SKIP), (("stratum+tls://a:1", "stratum+v2tls://b:1"), D.Status.PASS),
                                         (("stratum+tls://a:1", "stratum+tcp://b:1"), D.Status.WARN),
                                         (("stratum+v2://a:1",), D.Status.WARN)])
def test_pool_encryption(urls, status):
    assert run(D.check_pool_encryption(cfg(pools=pools(*urls)))).status == status


def _self_signed_pem(tmp_path) -> str:
    # a syntactically valid CA bundle: the system bundle if present, else skip
    for cand in (ssl.get_default_verify_paths().cafile, "/etc/ssl/certs/ca-certificates.crt"):
        if cand and os.path.exists(cand):
            return cand
    pytest.skip("no PEM CA bundle on this host")


def test_pool_tls_ca(tmp_path):
    assert run(D.check_pool_tls_ca(cfg(pools=pools("stratum+tls://a:1")))).status == D.Status.SKIP
    missing = cfg(pools=pools("stratum+tls://a:1", tls_ca_file=str(tmp_path / "nope.pem")))
    assert run(D.check_pool_tls_ca(missing)).status == D.Status.FAIL
    bad = tmp_path / "bad.pem"
    bad.write_text("-----BEGIN CERTIFICATE-----\nnot base64\n-----END CERTIFICATE-----\n")
    assert run(D.check_pool_tls_ca(cfg(pools=pools("stratum+tls://a:1", tls_ca_file=str(bad))))).status == D.Status.FAIL
    good = _self_signed_pem(tmp_path)
    assert run(D.check_pool_tls_ca(cfg(pools=pools("stratum+tls://a:1", tls_ca_file=good)))).status == D.Status.PASS


def test_payout_scheme_check():
    assert run(D.check_payout_scheme(cfg())).status == D.Status.SKIP
    r = run(D.check_payout_scheme(cfg(pools=pools("stratum+tcp://a:1", payout_scheme="pplns"))))
    assert "PPLNS" in r.detail and r.fix == ""
    r = run(D.check_payout_scheme(cfg(pools=pools("stratum+tcp://a:1", "stratum+tcp://"))))
    assert "scheme not set" in r.detail and r.fix and "stratum+tcp://" in r.detail


# ------------------------------------------------------------------ economics / env
@pytest.mark.parametrize("w,p,status", [(0, 0, D.Status.SKIP), (1000, 0, D.Status.WARN), (0, 0.1, D.Status.WARN),
                                        (1000, 0.1, D.Status.PASS)])
def test_power_cost(w, p, status):
    r = run(D.check_power_cost(cfg(power_watts=w, electricity_price_per_kwh=p)))
    assert r.status == status
    if status == D.Status.PASS:
        assert "$0.1000/h" in r.detail


def test_env_vars(monkeypatch):
    for k in list(os.environ):
        if k.startswith("OTEDAMA_"):
            monkeypatch.delenv(k)
    assert run(D.check_env_vars()).status == D.Status.PASS
    monkeypatch.setenv("OTEDAMA_POWER_WATTS", "many")
    r = run(D.check_env_vars())
    assert r.status == D.Status.WARN and "OTEDAMA_POWER_WATTS" in r.detail


def test_profitability_floor():
    assert run(D.check_profitability_floor(cfg())).status == D.Status.SKIP
    assert "2.5" in run(D.check_profitability_floor(cfg(min_yield_sats_per_sec=2.5))).detail


# ------------------------------------------------------------------ network / clock
def test_network_check(monkeypatch):
    monkeypatch.setattr(D, "pool_dial", lambda h, p, t: None)
    assert run(D.check_network()).status == D.Status.PASS
    monkeypatch.setattr(D, "network_check_endpoint", ("127.0.0.1", 1))
    monkeypatch.setattr(D, "pool_dial", lambda h, p, t: (_ for _ in ()).throw(OSError("unreachable")))
    r = run(D.check_network())
    assert r.status == D.Status.FAIL and "127.0.0.1:1" in r.detail and r.fix


class _DateServer:
    def __init__(self, date):
        outer = self
        self.date = date

        class H(http.server.BaseHTTPRequestHandler):
            def do_GET(self):
                self.log_request(200)
                self.send_response_only(200)
                if outer.date is not None:
                    self.send_header("Date", outer.date)
                self.send_header("Content-Length", "0")
                self.end_headers()

            def log_message(self, *a):
                pass

        self.httpd = http.server.HTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}/"

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


@pytest.mark.parametrize("offset,status", [(0, D.Status.PASS), (200, D.Status.WARN), (-200, D.Status.WARN),
                                           (600, D.Status.FAIL), (-600, D.Status.FAIL)])
def test_clock_check(monkeypatch, offset, status):
    s = _DateServer(email.utils.formatdate(time.time() + offset, usegmt=True))
    try:
        monkeypatch.setattr(D, "clock_skew_probe_url", s.url)
        assert run(D.check_clock()).status == status
    finally:
        s.close()


@pytest.mark.parametrize("date", [None, "not a date"])
def test_clock_check_without_a_usable_date(monkeypatch, date):
    s = _DateServer(date)
    try:
        monkeypatch.setattr(D, "clock_skew_probe_url", s.url)
        r = run(D.check_clock())
        assert r.status == D.Status.WARN and r.fix
    finally:
        s.close()


def test_clock_check_probe_unreachable(monkeypatch):
    monkeypatch.setattr(D, "clock_skew_probe_url", "http://127.0.0.1:1/")
    monkeypatch.setattr(D, "dial_timeout", 0.5)
    r = run(D.check_clock())
    assert r.status == D.Status.WARN and "cannot reach clock probe endpoint" in r.detail and r.fix


# ------------------------------------------------------------------ hardware / native / collectives
def test_hardware_check_drm_without_hip(monkeypatch, tmp_path):
    import otedama_amd.ops.native as native

    monkeypatch.setattr(native, "load", lambda build_if_missing=False: None)
    (tmp_path / "renderD128").mkdir()
    monkeypatch.setattr(D, "gpu_drm_path", str(tmp_path))
    r = run(D.check_hardware())
    assert r.status == D.Status.WARN and "render node" in r.detail
    monkeypatch.setattr(D, "gpu_drm_path", str(tmp_path / "none"))
    assert "no GPU detected" in run(D.check_hardware()).detail


def test_native_and_gpu_runtime_checks(monkeypatch):
    import otedama_amd.ops.native as native

    class N:
        def __init__(self, archs):
            self.archs = archs

        def cpu_has_sha_ni(self):
            return True

        def gpu_device_count(self):
            return len(self.archs)

        def gpu_arch_name(self, i):
            return self.archs[i] + ":sramecc+"

        def gpu_cu_count(self, i):
            return 256

    monkeypatch.setattr(native, "load", lambda build_if_missing=False: None)
    assert run(D.check_native()).status == D.Status.FAIL
    assert run(D.check_gpu_runtime()).status == D.Status.SKIP
    monkeypatch.setattr(native, "load", lambda build_if_missing=False: N(["gfx950"] * 8))
    assert "SHA-NI=yes" in run(D.check_native()).detail
    r = run(D.check_gpu_runtime())
    assert r.status == D.Status.PASS and "8 x gfx950 (256 CUs each)" in r.detail
    monkeypatch.setattr(native, "load", lambda build_if_missing=False: N(["gfx950", "gfx942"]))
    assert run(D.check_gpu_runtime()).status == D.Status.WARN


def test_collectives_check(monkeypatch):
    monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = run(D.check_collectives())
    assert r.status == D.Status.PASS and "gloo=yes" in r.detail
    import torch.distributed as dist

    if dist.is_nccl_available():
        monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "1")
        assert run(D.check_collectives()).status == D.Status.WARN


def test_default_checks_cover_the_reference_and_mi355x_set():
    names = [c.name for c in D.default_checks(cfg())]
    assert len(names) == len(set(names)) == 21
    for n in ("Configuration", "Bitcoin address", "Data directory", "Lightning wallet", "Pool reachability",
              "Pool diversity", "Pool endpoint diversity", "Pool connection encryption", "Pool TLS CA files",
              "Network", "System clock accuracy", "Hardware", "Native extension", "GPU runtime", "Collectives",
              "PoW self-test"):
        assert n in names


def test_collectives_check_reports_the_native_module_and_xgmi_pairs(monkeypatch):
    """The Collectives check names the node's data plane (the native RCCL module), and on a multi-GPU host counts
    the xGMI-linked GPU pairs from the KFD topology: all pairs linked passes, a pair without xGMI warns."""
    from otedama_amd import doctor, hal

    monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    gpus = [{"index": i, "node": i + 2, "hive_id": 7, "sdma_xgmi_engines": 14} for i in range(3)]
    full = [{"from": a, "to": b, "type": "xgmi", "weight": 15, "max_bandwidth": 76000}
            for a in range(3) for b in range(3) if a != b]
    monkeypatch.setattr(hal, "kfd_topology", lambda base_path=None: {"gpus": gpus, "links": full})
    r = doctor.check_collectives().run()
    assert "native RCCL module" in r.detail and "3 GPUs: 6/6 directed pairs on xGMI, 1 hive(s)" in r.detail
    monkeypatch.setattr(hal, "kfd_topology", lambda base_path=None: {"gpus": gpus, "links": full[:4]})
    r = doctor.check_collectives().run()
    assert r.status == doctor.Status.WARN and "4/6" in r.detail and "PCIe" in r.fix
