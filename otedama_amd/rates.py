"""BTC/USD rate fetcher: median of Coinbase / Kraken / CoinGecko.

Parity: internal/rates/fetcher.go
  * default sources + extractors ................................. :38-97
  * CacheDuration 5 min; plausibility band [100, 1e8] ............ :100-113
  * BTCUSDRate (fallback 95000 when never fetched; fresh < 5 min)  :200-207
  * Fetch single-flight; doFetch parallel, median, per-source
    health, HTTP Date -> clock-skew sensor (warn > 120 s) ......... :235-370
  * fetchOne: 10 s timeout, 64 KiB body cap, non-200 = error ...... :375-411
  * StartBackground(interval) .................................... :416-437
Offline-safe: with no egress every source fails fast and the fallback rate is
reported as stale, exactly as the reference does. Sources are injectable
(test seam, rates/fetcher_test.go:35).
"""
from __future__ import annotations

import concurrent.futures as cf
import email.utils
import json
import statistics
import threading
import time
import urllib.request
from dataclasses import dataclass
from typing import Callable

CACHE_DURATION = 300.0
MIN_PLAUSIBLE = 100.0
MAX_PLAUSIBLE = 100_000_000.0
CLOCK_SKEW_WARN = 120.0
BODY_CAP = 64 * 1024
USER_AGENT = "Otedama/3.0.0-mi355x (non-custodial mining)"


def _coinbase(b: bytes) -> float:
    return float(json.loads(b)["data"]["amount"])


def _kraken(b: bytes) -> float:
    res = json.loads(b).get("result") or {}
    for t in res.values():
        c = t.get("c") or []
        if c:
            return float(c[0])
    raise ValueError("rates: kraken: no ticker data")


def _coingecko(b: bytes) -> float:
    v = json.loads(b)
    try:
        return float(v["bitcoin"]["usd"])
    except (KeyError, TypeError):
        raise ValueError("rates: coingecko: missing bitcoin.usd field") from None


@dataclass(frozen=True)
class Source:
    name: str
    url: str
    extract: Callable[[bytes], float]


DEFAULT_SOURCES = (
    Source("Coinbase", "https://api.coinbase.com/v2/prices/BTC-USD/spot", _coinbase),
    Source("Kraken", "https://api.kraken.com/0/public/Ticker?pair=XBTUSD", _kraken),
    Source("CoinGecko", "https://api.coingecko.com/api/v3/simple/price?ids=bitcoin&vs_currencies=usd", _coingecko),
)


class Fetcher:
    def __init__(self, fallback: float = 95_000.0, sources=DEFAULT_SOURCES, timeout: float = 10.0, log=None):
        self.fallback = fallback
        self.sources = list(sources)
        self.timeout = timeout
        self.log = log or (lambda msg: None)
        self._lock = threading.Lock()
        self._rate = 0.0
        self._fetched_at = 0.0
        self._skew = 0.0
        self._last_ok = 0
        self._attempts = 0
        self._inflight: threading.Event | None = None
        self._inflight_err: Exception | None = None
        self._flight_lock = threading.Lock()
        self._stop = threading.Event()
        # one pool of source threads for the fetcher's life: a new executor per fetch started new threads every 5
        # minutes, and each new thread's malloc arena showed as ~2.5 MB of RSS per fetch in a long soak
        self._pool: cf.ThreadPoolExecutor | None = None

    def btc_usd_rate(self) -> tuple[float, bool]:
        with self._lock:
            if self._rate <= 0:
                return self.fallback, False
            return self._rate, time.time() - self._fetched_at < CACHE_DURATION

    def rate_age(self) -> tuple[float, bool]:
        with self._lock:
            if not self._fetched_at:
                return 0.0, False
            return time.time() - self._fetched_at, True

    def clock_skew_seconds(self) -> float:
        with self._lock:
            return self._skew

    def source_health(self) -> tuple[int, int, bool]:
        with self._lock:
            return self._last_ok, len(self.sources), self._attempts > 0

    def fetch(self) -> None:
        """Single-flight: concurrent callers wait for the in-progress fetch."""
        with self._flight_lock:
            ev = self._inflight
            if ev is None:
                ev = self._inflight = threading.Event()
                leader = True
            else:
                leader = False
        if not leader:
            ev.wait()
            if self._inflight_err:
                raise self._inflight_err
            return
        err = None
        try:
            self._do_fetch()
        except Exception as exc:  # noqa: BLE001
            err = exc.with_traceback(None)  # the waiters re-raise it; its old frames are not kept alive
        with self._flight_lock:
            self._inflight_err = err
            self._inflight = None
        ev.set()
        if err:
            try:
                raise err
            finally:
                del err  # no frame -> exception -> traceback -> frame cycle for the cyclic GC to find later

    def _fetch_one(self, src: Source) -> tuple[float, float]:
        req = urllib.request.Request(src.url, headers={"User-Agent": USER_AGENT})
        skew = 0.0
        with urllib.request.urlopen(req, timeout=self.timeout) as resp:  # noqa: S310 - fixed https URLs
            date = resp.headers.get("Date")
            if date:
                try:
                    skew = abs(time.time() - email.utils.parsedate_to_datetime(date).timestamp())
                except (TypeError, ValueError):
                    pass
            body = resp.read(BODY_CAP)
            if resp.status != 200:
                raise RuntimeError(f"rates: {src.name}: HTTP {resp.status}")
        return src.extract(body), skew

    def _do_fetch(self) -> None:
        rates, errs, max_skew, skew_seen = [], [], 0.0, False
        with self._lock:
            if self._pool is None:
                self._pool = cf.ThreadPoolExecutor(max_workers=max(len(self.sources), 1),
                                                   thread_name_prefix="otedama-rates-src")
            ex = self._pool
        futs = [ex.submit(self._fetch_one, s) for s in self.sources]
        for s, fut in zip(self.sources, futs):
            try:
                r, sk = fut.result()
            except Exception as exc:  # noqa: BLE001
                errs.append(f"{s.name}: {exc}")
                # A failed request's traceback holds the worker's frames (opener, handlers, the socket). Kept by
                # the future, it joins a reference cycle that only a full GC frees. In a process with torch's
                # millions of objects, full collections are rare, and every 5-minute fetch that failed (no route
                # to the rate APIs) showed as ~2.5 MB of RSS growth of the leader in a long soak.
                exc.__traceback__ = None
                continue
            if sk > 0:
                skew_seen, max_skew = True, max(max_skew, sk)
            if not MIN_PLAUSIBLE <= r <= MAX_PLAUSIBLE:
                if r != 0:
                    self.log(f"rates: ignoring implausible reading {r:.2f} (outside [{MIN_PLAUSIBLE:.0f}, "
                             f"{MAX_PLAUSIBLE:.0f}])")
                continue
            rates.append(r)
        if skew_seen:
            with self._lock:
                self._skew = max_skew
            if max_skew > CLOCK_SKEW_WARN:
                self.log(f"rates: WARNING: local clock is {max_skew:.0f} s off server time (threshold "
                         f"{CLOCK_SKEW_WARN:.0f} s)")
        with self._lock:
            self._last_ok = len(rates)
            self._attempts += 1
        del futs
        if not rates:
            raise RuntimeError("rates: all sources failed: " + ("; ".join(errs) or "all readings implausible"))
        med = statistics.median(rates)
        with self._lock:
            self._rate, self._fetched_at = med, time.time()

    def start_background(self, interval: float = CACHE_DURATION) -> threading.Thread:
        interval = interval if interval > 0 else CACHE_DURATION

        def loop():
            first = True
            while not self._stop.is_set():
                try:
                    self.fetch()
                except Exception as exc:  # noqa: BLE001
                    self.log(("rates: initial fetch failed: " if first else "rates: periodic fetch failed: ")
                             + str(exc))
                first = False
                self._stop.wait(interval)

        t = threading.Thread(target=loop, name="otedama-rates", daemon=True)
        t.start()
        return t

    def stop(self) -> None:
        self._stop.set()
        with self._lock:
            pool, self._pool = self._pool, None
        if pool is not None:
            pool.shutdown(wait=False)
