"""BTC/USD rate fetcher: extractors, median consensus, plausibility band, fallback / staleness, clock-skew
sensor, source health, single-flight, body cap, background loop — against loopback HTTP servers.

Mirrors internal/rates/fetcher_test.go (Test*Extractor_*, TestFetchOne_*, TestFetcher_*, TestStartBackground_*).
"""
from __future__ import annotations

import email.utils
import http.server
import json
import threading
import time

import pytest

from otedama_amd import rates as R


# ------------------------------------------------------------------ extractors
@pytest.mark.parametrize("body,want", [(b'{"data":{"amount":"95123.45","currency":"USD"}}', 95123.45),
                                       (b'{"data":{"amount":"1"}}', 1.0)])
def test_coinbase_extractor(body, want):
    assert R._coinbase(body) == want


@pytest.mark.parametrize("body", [b"not json", b'{"data":{}}', b'{"data":{"amount":"abc"}}', b'{}',
                                  b'{"data":{"amount":"95000x"}}'])
def test_coinbase_extractor_rejects(body):
    with pytest.raises((ValueError, KeyError, TypeError)):
        R._coinbase(body)


@pytest.mark.parametrize("body,want", [(b'{"error":[],"result":{"XXBTZUSD":{"c":["96000.1","0.01"]}}}', 96000.1)])
def test_kraken_extractor(body, want):
    assert R._kraken(body) == want


@pytest.mark.parametrize("body", [b'{"result":{}}', b'{"result":{"X":{"c":[]}}}', b"{bad", b'{"result":null}',
                                  b'{"result":{"X":{"c":["96000z"]}}}'])
def test_kraken_extractor_rejects(body):
    with pytest.raises((ValueError, KeyError, TypeError, AttributeError)):
        R._kraken(body)


def test_coingecko_extractor():
    assert R._coingecko(b'{"bitcoin":{"usd":97000}}') == 97000.0


@pytest.mark.parametrize("body", [b'{"ethereum":{"usd":1}}', b'{"bitcoin":{}}', b"{}", b"[", b'{"bitcoin":5}'])
def test_coingecko_extractor_rejects(body):
    with pytest.raises(ValueError):
        R._coingecko(body)


def test_default_sources():
    assert len(R.DEFAULT_SOURCES) >= 2
    for s in R.DEFAULT_SOURCES:
        assert s.name and s.url.startswith("https://") and callable(s.extract)
    assert [s.name for s in R.DEFAULT_SOURCES] == ["Coinbase", "Kraken", "CoinGecko"]
    assert 60 <= R.CACHE_DURATION <= 3600


# ------------------------------------------------------------------ loopback servers
class _Srv:
    """One HTTP server; routes map path -> (status, body, date header or None, delay)."""

    def __init__(self):
        self.routes: dict[str, tuple] = {}
        self.hits: dict[str, int] = {}
        self.agents: list[str] = []
        outer = self

        class H(http.server.BaseHTTPRequestHandler):
            def do_GET(self):
                outer.hits[self.path] = outer.hits.get(self.path, 0) + 1
                outer.agents.append(self.headers.get("User-Agent", ""))
                status, body, date, delay = outer.routes.get(self.path, (404, b"", None, 0))
                if delay:
                    time.sleep(delay)
                self.send_response(status)
                if date is not None:
                    self.send_header("Date", date)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def send_response(self, code, message=None):
                # no automatic Date header: the tests control it
                self.log_request(code)
                self.send_response_only(code, message)

            def log_message(self, *a):
                pass

        self.httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.t = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.t.start()

    def url(self, path):
        return f"http://127.0.0.1:{self.httpd.server_address[1]}{path}"

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


@pytest.fixture
def srv():
    s = _Srv()
    yield s
    s.close()


def _now_date(offset=0.0):
    return email.utils.formatdate(time.time() + offset, usegmt=True)


def _cb(v):
    return json.dumps({"data": {"amount": str(v)}}).encode()


def _src(srv, path, status=200, body=b"", date=None, delay=0.0, extract=R._coinbase):
    srv.routes[path] = (status, body, date, delay)
    return R.Source(path.strip("/"), srv.url(path), extract)


# ------------------------------------------------------------------ fetcher
def test_before_any_fetch_reports_fallback_and_no_age():
    f = R.Fetcher(95_000, sources=[])
    assert f.btc_usd_rate() == (95_000, False)
    assert f.rate_age() == (0.0, False)
    assert f.clock_skew_seconds() == 0.0
    assert f.source_health() == (0, 0, False)


def test_fetch_from_one_source(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(91234.5))])
    f.fetch()
    rate, fresh = f.btc_usd_rate()
    assert rate == 91234.5 and fresh
    age, ok = f.rate_age()
    assert ok and 0 <= age < 5
    assert f.source_health() == (1, 1, True)
    assert srv.agents and srv.agents[0].startswith("Otedama/")


def test_median_of_three_and_of_two(srv):
    srcs = [_src(srv, "/a", body=_cb(90000)), _src(srv, "/b", body=_cb(100000)), _src(srv, "/c", body=_cb(91000))]
    f = R.Fetcher(sources=srcs)
    f.fetch()
    assert f.btc_usd_rate()[0] == 91000
    f = R.Fetcher(sources=srcs[:2])
    f.fetch()
    assert f.btc_usd_rate()[0] == 95000  # median of two = mean


@pytest.mark.parametrize("bad", [50, 2e8, 0, "nan", "inf"])
def test_implausible_readings_are_excluded(srv, bad):
    logs = []
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(bad)), _src(srv, "/b", body=_cb(93000))], log=logs.append)
    f.fetch()
    assert f.btc_usd_rate()[0] == 93000 and f.source_health() == (1, 2, True)
    if bad not in (0,):
        assert any("implausible" in m for m in logs)


def test_all_sources_fail_keeps_fallback_and_joins_causes(srv):
    f = R.Fetcher(80_000, sources=[_src(srv, "/a", status=500, body=b"oops"), _src(srv, "/b", body=b"{}"),
                                   R.Source("dead", "http://127.0.0.1:1/x", R._coinbase)], timeout=2)
    with pytest.raises(RuntimeError) as ei:
        f.fetch()
    msg = str(ei.value)
    assert "all sources failed" in msg and "a:" in msg and "b:" in msg and "dead:" in msg
    assert f.btc_usd_rate() == (80_000, False)
    assert f.source_health() == (0, 3, True)


def test_all_readings_implausible(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(1))])
    with pytest.raises(RuntimeError, match="implausible"):
        f.fetch()


def test_last_good_rate_survives_a_failed_fetch(srv):
    s = _src(srv, "/a", body=_cb(90500))
    f = R.Fetcher(sources=[s])
    f.fetch()
    srv.routes["/a"] = (500, b"", None, 0)
    with pytest.raises(RuntimeError):
        f.fetch()
    assert f.btc_usd_rate() == (90500, True) and f.source_health() == (0, 1, True)


def test_rate_goes_stale_after_the_cache_duration(srv, monkeypatch):
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(90000))])
    f.fetch()
    real = time.time
    monkeypatch.setattr(R.time, "time", lambda: real() + R.CACHE_DURATION + 1)
    rate, fresh = f.btc_usd_rate()
    assert rate == 90000 and not fresh
    assert f.rate_age()[0] > R.CACHE_DURATION


def test_non_200_is_an_error(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", status=503, body=_cb(90000))])
    with pytest.raises(RuntimeError):
        f.fetch()


def test_response_body_is_capped(srv):
    big = b'{"data":{"amount":"90000"},"pad":"' + b"x" * (R.BODY_CAP + 10) + b'"}'
    f = R.Fetcher(sources=[_src(srv, "/a", body=big)])
    with pytest.raises(RuntimeError):
        f.fetch()  # truncated at 64 KiB -> invalid JSON, never buffered whole


def test_timeout_is_honoured(srv):
    f = R.Fetcher(sources=[_src(srv, "/slow", body=_cb(90000), delay=1.5)], timeout=0.3)
    t0 = time.perf_counter()
    with pytest.raises(RuntimeError):
        f.fetch()
    assert time.perf_counter() - t0 < 1.4


@pytest.mark.parametrize("offset,warn", [(0, False), (-3600, True), (500, True)])
def test_clock_skew_sensor(srv, offset, warn):
    logs = []
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(90000), date=_now_date(offset))], log=logs.append)
    f.fetch()
    assert abs(f.clock_skew_seconds() - abs(offset)) < 5
    assert any("clock is" in m for m in logs) is warn


def test_missing_or_bad_date_header_gives_zero_skew(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(90000)), _src(srv, "/b", body=_cb(90000), date="garbage")])
    f.fetch()
    assert f.clock_skew_seconds() == 0.0


def test_fetch_is_single_flight(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(90000), delay=0.3)])
    errs = []

    def go():
        try:
            f.fetch()
        except Exception as exc:  # noqa: BLE001
            errs.append(exc)

    ts = [threading.Thread(target=go) for _ in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert not errs and srv.hits["/a"] == 1 and f.btc_usd_rate()[0] == 90000


def test_single_flight_followers_see_the_leaders_error(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", status=500, delay=0.3)])
    errs = []

    def go():
        try:
            f.fetch()
        except Exception as exc:  # noqa: BLE001
            errs.append(exc)

    ts = [threading.Thread(target=go) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert len(errs) == 4 and srv.hits["/a"] == 1


def test_concurrent_reads_are_safe(srv):
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(90000))])
    stop = threading.Event()
    seen = set()

    def reader():
        while not stop.is_set():
            seen.add(f.btc_usd_rate()[0])

    ts = [threading.Thread(target=reader) for _ in range(4)]
    for t in ts:
        t.start()
    for _ in range(5):
        f.fetch()
    stop.set()
    for t in ts:
        t.join(5)
    assert seen <= {95_000.0, 90000.0}


def test_background_fetches_immediately_and_stops(srv):
    logs = []
    f = R.Fetcher(sources=[_src(srv, "/a", body=_cb(90000))], log=logs.append)
    t = f.start_background(interval=0.05)
    deadline = time.time() + 5
    while f.btc_usd_rate()[0] != 90000 and time.time() < deadline:
        time.sleep(0.01)
    assert f.btc_usd_rate()[0] == 90000
    time.sleep(0.2)
    assert srv.hits["/a"] >= 2  # periodic
    f.stop()
    t.join(2)
    assert not t.is_alive() and not logs


def test_background_logs_initial_then_periodic_failures(srv):
    logs = []
    f = R.Fetcher(sources=[_src(srv, "/a", status=500)], log=logs.append)
    t = f.start_background(interval=0.05)
    deadline = time.time() + 5
    while len(logs) < 2 and time.time() < deadline:
        time.sleep(0.01)
    f.stop()
    t.join(2)
    assert logs[0].startswith("rates: initial fetch failed") and logs[1].startswith("rates: periodic fetch failed")


def test_background_zero_interval_uses_the_default():
    f = R.Fetcher(sources=[])
    t = f.start_background(interval=0)
    time.sleep(0.05)
    f.stop()
    t.join(2)
    assert not t.is_alive()


def test_default_logger_is_silent():
    R.Fetcher(sources=[]).log("anything")


def test_failed_fetches_leave_no_cyclic_garbage():
    """On a host with no route to the rate APIs every fetch fails. A failure must not leave reference cycles
    (raised error -> traceback -> frame -> error; the futures' exceptions -> worker frames -> opener, socket): only a
    full GC frees those, and in a long-running process they piled up as ~2.5 MB of RSS per 5-minute fetch
    (profiles/r5/n_rss). Before the fix, 10 failed fetches left 2,882 unreachable objects."""
    import gc

    from otedama_amd import rates

    dead = [rates.Source("Dead", "http://127.0.0.1:1/x", lambda b: 0.0)] * 3
    f = rates.Fetcher(sources=dead, timeout=2)
    try:
        f.fetch()  # the pool's threads and the resolver set-up, once
    except Exception:  # noqa: BLE001
        pass
    gc.collect()
    gc.disable()
    try:
        for _ in range(10):
            with pytest.raises(RuntimeError, match="all sources failed"):
                f.fetch()
        assert gc.collect() == 0
    finally:
        gc.enable()
        f.stop()
