"""internal/doctor/{doctor,extras}_test.go, case by case, for the behaviours not already pinned by
test_doctor_checks.py / test_doctor.py: the address helpers, the data-dir / wallet branches (no home, stat
errors, fingerprint display), the pool-reachability URL handling, the network and hardware checks against
local fixtures, and the clock probe's request/response edge cases."""
from __future__ import annotations

import http.server
import os
import socket
import threading

import pytest

from otedama_amd import config as C
from otedama_amd import doctor as D

BECH32 = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"
TAPROOT = "bc1p5d7rjq7g6rdk2yhzks9smlaqtedr4dekq08ge8ztwac72sfr9rusxg3297"
P2WSH = "bc1qrp33g0q5c5txsp9arysrx4k6zdkfs4nce4xj0gdcccefvpysxf3qccfmv3"
P2PKH = "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa"
P2SH = "3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy"


def run(check: D.Check) -> D.Result:
    return check.run()


# ------------------------------------------------------------------ helpers (checks.go:856-916)
@pytest.mark.parametrize("addr,want", [
    (BECH32, True), (P2PKH, True), (P2SH, True), (TAPROOT, True),
    ("", False), ("bc1", False), ("2NotAnAddress000000000000000", False),
    ("1" + "0" * 25, False),  # '0' is not base58
    ("3" + "O" * 25, False),  # 'O' is not base58
    ("bc1" + "q" * 22 + "B", False),  # uppercase is outside the bech32 charset
    ("  " + BECH32 + "\n", True),  # trimmed
])
def test_is_likely_bitcoin_address(addr, want):
    assert D.is_likely_bitcoin_address(addr) is want


def test_is_likely_bitcoin_address_length_boundaries():
    assert not D.is_likely_bitcoin_address("1" + "a" * 24)  # 25
    assert D.is_likely_bitcoin_address("1" + "a" * 25)  # 26
    assert D.is_likely_bitcoin_address("bc1" + "q" * 87)  # 90
    assert not D.is_likely_bitcoin_address("bc1" + "q" * 88)  # 91


def test_is_likely_bitcoin_address_one_char_off_prefix():
    for bad in ("bc2" + BECH32[3:], "tb1" + BECH32[3:], "2" + P2PKH[1:], "4" + P2SH[1:]):
        assert not D.is_likely_bitcoin_address(bad)


def test_bech32_char_set():
    for c in "qpzry9x8gf2tvdw0s3jn54khce6mua7l":
        assert D.is_bech32_char(c)
    for c in "bio1BQP!":
        assert not D.is_bech32_char(c)


def test_base58_char_set():
    for c in "0OIl":
        assert not D.is_base58_char(c)
    for c in "123456789":
        assert D.is_base58_char(c)
    for c in "ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz":
        assert D.is_base58_char(c)


def test_mask_address():
    assert D.mask_address(BECH32) == "bc1qar···5mdq"
    assert D.mask_address("short") == "short"
    assert D.mask_address("0123456789") == "0123456789"  # length 10: unchanged
    assert D.mask_address("0123456789a") == "012345···789a"  # length 11: masked
    m = D.mask_address(P2PKH)
    assert m.startswith(P2PKH[:6]) and m.endswith(P2PKH[-4:]) and "···" in m


@pytest.mark.parametrize("addr,kind", [
    (BECH32, "P2WPKH SegWit v0"), (P2WSH, "P2WSH SegWit v0"), (TAPROOT, "P2TR Taproot"),
    (P2PKH, "P2PKH legacy"), (P2SH, "P2SH"), ("zzz", "unrecognised type"),
])
def test_address_kind(addr, kind):
    assert D.address_kind(addr) == kind


def test_append_unique():
    xs = ["a"]
    assert D.append_unique(xs, "a") == ["a"]
    assert D.append_unique(xs, "b") == ["a", "b"]


# ------------------------------------------------------------------ bitcoin address check
@pytest.mark.parametrize("addr", [BECH32, TAPROOT, P2PKH, P2SH])
def test_bitcoin_address_valid_passes_and_surfaces_type(addr):
    r = run(D.check_bitcoin_address(C.Config(bitcoin_address=addr)))
    assert r.status == D.Status.PASS and D.address_kind(addr) in r.detail
    assert addr not in r.detail and D.mask_address(addr) in r.detail  # never the full address


@pytest.mark.parametrize("addr", [BECH32[:-1] + ("q" if BECH32[-1] != "q" else "p"), P2PKH[:-1] + "b"])
def test_bitcoin_address_typo_fails_checksum(addr):
    r = run(D.check_bitcoin_address(C.Config(bitcoin_address=addr)))
    assert r.status == D.Status.FAIL and "checksum" in r.fix


def test_bitcoin_address_invalid_shape():
    r = run(D.check_bitcoin_address(C.Config(bitcoin_address="not-an-address")))
    assert r.status == D.Status.FAIL and "does not look like a valid address" in r.detail and r.fix


def test_failover_addresses_typo_fails_checksum_with_index():
    r = run(D.check_failover_addresses(C.Config(bitcoin_addresses=[BECH32, P2PKH[:-1] + "b"])))
    assert r.status == D.Status.FAIL and "bitcoin_addresses[1]" in r.detail
    r = run(D.check_failover_addresses(C.Config(bitcoin_addresses=[BECH32, "not-a-valid-address"])))
    assert r.status == D.Status.FAIL and "bitcoin_addresses[1]" in r.detail
    r = run(D.check_failover_addresses(C.Config(bitcoin_addresses=[BECH32, P2SH])))
    assert r.status == D.Status.PASS and "2 failover address(es)" in r.detail


# ------------------------------------------------------------------ data dir / wallet
def test_data_dir_no_home_skips(monkeypatch):
    monkeypatch.setattr(C, "default_data_dir", lambda *a, **k: "")
    r = run(D.check_data_dir(C.Config(data_dir="")))
    assert r.status == D.Status.SKIP and "no home directory" in r.detail


def test_data_dir_empty_uses_default(monkeypatch, tmp_path):
    monkeypatch.setattr(C, "default_data_dir", lambda *a, **k: str(tmp_path / "default-dd"))
    r = run(D.check_data_dir(C.Config(data_dir="")))
    assert r.status == D.Status.WARN and "default-dd" in r.detail


def test_data_dir_stat_error_not_not_exist_fails(tmp_path):
    f = tmp_path / "file"
    f.write_text("")
    r = run(D.check_data_dir(C.Config(data_dir=str(f / "sub"))))  # ENOTDIR, not ENOENT
    assert r.status == D.Status.FAIL and "cannot stat" in r.detail and r.fix


def test_data_dir_creates_on_first_run_is_only_a_warning(tmp_path):
    r = run(D.check_data_dir(C.Config(data_dir=str(tmp_path / "a" / "b"))))
    assert r.status == D.Status.WARN and "will be created on first run" in r.detail


def _wallet_dir(tmp_path, fingerprint: str | None):
    from otedama_amd.lightning import seedstore

    w = tmp_path / "wallet.dat"
    w.write_bytes(seedstore.EncryptedSeed(seedstore.VERSION, os.urandom(16), os.urandom(12), os.urandom(80)).marshal())
    os.chmod(w, 0o600)
    if fingerprint is not None:
        (tmp_path / "wallet.fingerprint").write_text(fingerprint)
    return C.Config(data_dir=str(tmp_path))


def test_wallet_with_fingerprint_shows_it(tmp_path):
    r = run(D.check_wallet(_wallet_dir(tmp_path, "a1b2c3d4")))
    assert r.status == D.Status.PASS and "a1b2c3d4" in r.detail


def test_wallet_without_fingerprint_file_passes_with_note(tmp_path):
    r = run(D.check_wallet(_wallet_dir(tmp_path, None)))
    assert r.status == D.Status.PASS and "fingerprint file missing" in r.detail


def test_wallet_fingerprint_trimmed_of_whitespace(tmp_path):
    r = run(D.check_wallet(_wallet_dir(tmp_path, "deadbeef\n")))
    assert "deadbeef" in r.detail and "deadbeef\n" not in r.detail


def test_wallet_no_home_skips(monkeypatch):
    monkeypatch.setattr(C, "default_data_dir", lambda *a, **k: "")
    r = run(D.check_wallet(C.Config(data_dir="")))
    assert r.status == D.Status.SKIP and "no home directory" in r.detail


def test_wallet_empty_data_dir_uses_default(monkeypatch, tmp_path):
    monkeypatch.setattr(C, "default_data_dir", lambda *a, **k: str(tmp_path))
    r = run(D.check_wallet(C.Config(data_dir="")))
    assert r.status == D.Status.WARN and str(tmp_path) in r.detail


def test_wallet_stat_error_not_not_exist_fails(tmp_path):
    f = tmp_path / "file"
    f.write_text("")
    r = run(D.check_wallet(C.Config(data_dir=str(f))))  # <file>/wallet.dat: ENOTDIR
    assert r.status == D.Status.FAIL and "cannot stat" in r.detail and r.fix


# ------------------------------------------------------------------ pools
def test_pool_reachability_malformed_url_fails(monkeypatch):
    monkeypatch.setattr(D, "pool_dial", lambda h, p, t: None)
    r = run(D.check_pool_reachability(C.Config(pools=[C.PoolConfig(url="not-a-valid-url")])))
    assert r.status == D.Status.FAIL and "cannot parse pool URL" in r.detail and r.fix


def test_pool_reachability_malformed_among_good_warns(monkeypatch):
    monkeypatch.setattr(D, "pool_dial", lambda h, p, t: None)
    c = C.Config(pools=[C.PoolConfig(url="stratum+tcp://a.example:1"), C.PoolConfig(url="junk")])
    r = run(D.check_pool_reachability(c))
    assert r.status == D.Status.WARN and "junk" in r.detail


def test_pool_reachability_no_pools_uses_default(monkeypatch):
    seen = []

    def dial(host, port, timeout):
        seen.append((host, port))
        raise OSError("offline")

    monkeypatch.setattr(D, "pool_dial", dial)
    r = run(D.check_pool_reachability(C.Config()))
    assert r.status == D.Status.FAIL and r.fix
    assert seen and seen[0][0] in C.DEFAULT_POOL_URL


def test_pool_reachability_pass_reports_latency():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    try:
        r = run(D.check_pool_reachability(C.Config(pools=[C.PoolConfig(url=f"stratum+v2://127.0.0.1:{port}")])))
        assert r.status == D.Status.PASS and f"127.0.0.1:{port}" in r.detail and "ms)" in r.detail
    finally:
        srv.close()


def test_payout_scheme_empty_host_uses_url():
    r = run(D.check_payout_scheme(C.Config(pools=[C.PoolConfig(url="stratum+tcp://", payout_scheme="pplns")])))
    assert "stratum+tcp://" in r.detail


# ------------------------------------------------------------------ network / hardware
def test_network_local_listener_passes(monkeypatch):
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    try:
        monkeypatch.setattr(D, "network_check_endpoint", ("127.0.0.1", srv.getsockname()[1]))
        r = run(D.check_network())
        assert r.status == D.Status.PASS and r.detail == "IPv4 OK"
    finally:
        srv.close()


def test_network_unreachable_fails_with_fix(monkeypatch):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()  # nothing listens there now
    monkeypatch.setattr(D, "network_check_endpoint", ("127.0.0.1", port))
    r = run(D.check_network())
    assert r.status == D.Status.FAIL and "firewall" in r.fix


def _no_hip(monkeypatch):
    import otedama_amd.ops.native as native

    monkeypatch.setattr(native, "load", lambda build_if_missing=False: None)


def test_hardware_gpu_detected_from_drm(monkeypatch, tmp_path):
    _no_hip(monkeypatch)
    for name in ("renderD128", "renderD129", "card0"):
        (tmp_path / name).mkdir()
    monkeypatch.setattr(D, "gpu_drm_path", str(tmp_path))
    r = run(D.check_hardware())
    assert "2 GPU(s) detected" in r.detail and "-core CPU" in r.detail


def test_hardware_empty_drm_dir_no_gpu_passes(monkeypatch, tmp_path):
    _no_hip(monkeypatch)
    monkeypatch.setattr(D, "gpu_drm_path", str(tmp_path))
    r = run(D.check_hardware())
    assert r.status == D.Status.PASS and "no GPU" in r.detail


# ------------------------------------------------------------------ clock probe
class _Probe:
    """Loopback HTTP server: GET returns an optional Date header and a body; records whether the client read
    the whole body before closing."""

    def __init__(self, date: str | None, body: bytes = b'{"data":{"epoch":0}}'):
        outer = self
        self.requests = []

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def do_GET(self):
                outer.requests.append(dict(self.headers))
                self.send_response_only(200)
                if date is not None:
                    self.send_header("Date", date)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        self.httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}/v2/time"

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


def test_clock_accurate_date_passes_and_sends_user_agent(monkeypatch):
    import email.utils

    p = _Probe(email.utils.formatdate(usegmt=True), body=b"x" * 20000)  # body larger than the 8 KiB drain
    try:
        monkeypatch.setattr(D, "clock_skew_probe_url", p.url)
        r = run(D.check_clock())
        assert r.status == D.Status.PASS and "within 120 s" in r.detail
        assert p.requests and p.requests[0].get("User-Agent", "").startswith("Otedama/")
    finally:
        p.close()


def test_clock_malformed_date_warns(monkeypatch):
    p = _Probe("yesterday-ish")
    try:
        monkeypatch.setattr(D, "clock_skew_probe_url", p.url)
        r = run(D.check_clock())
        assert r.status == D.Status.WARN and "cannot parse server Date header" in r.detail
    finally:
        p.close()


def test_clock_request_build_error_warns(monkeypatch):
    monkeypatch.setattr(D, "clock_skew_probe_url", "::not a url::")
    r = run(D.check_clock())
    assert r.status == D.Status.WARN and "could not build request" in r.detail and r.fix


def test_clock_thresholds_match_reference():
    assert D.CLOCK_SKEW_WARN_SECS == 120.0 and D.CLOCK_SKEW_FAIL_SECS == 300.0


# ------------------------------------------------------------------ default set
def test_default_checks_all_have_name_and_run_and_unique_names():
    checks = D.default_checks(C.Config())
    names = [c.name for c in checks]
    assert all(names) and all(callable(c.run) for c in checks)
    assert len(names) == len(set(names))
    for want in ("Lightning wallet", "Pool connection encryption", "Power & cost config", "Profitability floor",
                 "Pool payout schemes", "System clock accuracy", "Environment variables"):
        assert want in names
