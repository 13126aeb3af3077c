"""Engine health / statistics helpers.

Parity: internal/engine/stats.go
  * hashrateWindow (counter-reset saturation: no negative/NaN rates) .. :151-175
  * uptimeAccountant / satsAccountant ................................ :185-245
  * rejectClass taxonomy (stale/duplicate/difficulty/hardware/other) . :263-277
  * acceptanceRate / effectiveYield .................................. :286-325
  * LatencyTracker (ring 256, nearest-rank quantiles) ................ :337-400
  * HashrateMonitor (3 samples <= floor -> stalled) .................. :412-457
  * publishBTCRate / publishDifficulty (interval = D*2^32/H) ......... :476-513
  * HashRateString (miner/worker.go:285-298)
"""
from __future__ import annotations

import threading


def hashrate_string(hps: float) -> str:
    units = (("EH/s", 1e18), ("PH/s", 1e15), ("TH/s", 1e12), ("GH/s", 1e9), ("MH/s", 1e6), ("kH/s", 1e3))
    for name, scale in units:
        if hps >= scale:
            return f"{hps / scale:.2f} {name}"
    return f"{hps:.0f} H/s"  # worker.go:296: whole hashes below 1 kH/s


class HashrateWindow:
    def __init__(self) -> None:
        self.last_total = 0
        self.last_time = 0.0
        self.primed = False

    def observe(self, total: int, now: float) -> float:
        if not self.primed:
            self.primed, self.last_total, self.last_time = True, total, now
            return 0.0
        dt = now - self.last_time
        rate = (total - self.last_total) / dt if dt > 0 and total >= self.last_total else 0.0
        self.last_total, self.last_time = total, now
        return rate


class UptimeAccountant:
    def __init__(self) -> None:
        self.last_tick: float | None = None
        self.accum = 0.0

    def observe(self, now: float, productive: bool, counter) -> None:
        if self.last_tick is None:
            self.last_tick = now
            return
        elapsed = now - self.last_tick
        self.last_tick = now
        if elapsed <= 0 or not productive or counter is None:
            return
        self.accum += elapsed
        whole = int(self.accum)
        if whole > 0:
            counter.add(whole)
            self.accum -= whole


class SatsAccountant:
    def __init__(self) -> None:
        self.last_tick: float | None = None
        self.total = 0.0

    def observe(self, now: float, rate_per_sec: float, productive: bool) -> float:
        if self.last_tick is None:
            self.last_tick = now
            return self.total
        elapsed = now - self.last_tick
        self.last_tick = now
        if elapsed > 0 and productive and rate_per_sec > 0:
            self.total += rate_per_sec * elapsed
        return self.total


def reject_class(reason: str) -> tuple[str, str]:
    r = reason.lower()
    if "stale" in r or "job not found" in r or "unknown job" in r:
        return "stale", "likely cause: network latency / stale work"
    if "duplicate" in r:
        return "duplicate", "likely cause: firmware or connectivity (duplicate submission)"
    if "above" in r or "target" in r or "low difficulty" in r or "low-difficulty" in r or "high-hash" in r:
        return "difficulty", "likely cause: difficulty configuration or hardware error"
    if "invalid" in r or "bad" in r:
        return "hardware", "likely cause: hardware error (failing chip / overheating)"
    return "other", "cause unclassified — check pool documentation"


REJECT_CATEGORIES = ("stale", "duplicate", "difficulty", "hardware", "other")


def acceptance_rate(accepted: int, rejected: int) -> float:
    total = accepted + rejected
    return 1.0 if total == 0 else accepted / total


def effective_yield(expected: float, productive_seconds: float, uptime_seconds: float) -> float:
    if uptime_seconds <= 0:
        return 0.0
    frac = min(max(productive_seconds / uptime_seconds, 0.0), 1.0)
    return expected * frac


class LatencyTracker:
    def __init__(self, size: int = 256):
        if size < 1:
            size = 256
        self._samples = [0.0] * size
        self._next = 0
        self._filled = False
        self._lock = threading.Lock()

    def record(self, ms: float) -> None:
        if ms < 0:
            return
        with self._lock:
            self._samples[self._next] = ms
            self._next = (self._next + 1) % len(self._samples)
            if self._next == 0:
                self._filled = True

    def count(self) -> int:
        with self._lock:
            return len(self._samples) if self._filled else self._next

    def quantile(self, q: float) -> float:
        with self._lock:
            n = len(self._samples) if self._filled else self._next
            if n == 0:
                return 0.0
            cp = sorted(self._samples[:n])
        idx = int(q * n + 0.5) - 1
        return cp[min(max(idx, 0), n - 1)]


class HashrateMonitor:
    def __init__(self, floor: float = 0.0, max_stall: int = 3, log=None):
        self.floor = floor
        self.max_stall = max_stall if max_stall >= 1 else 3
        self.stall_count = 0
        self.warned = False
        self.log = log

    def observe(self, hashrate: float) -> None:
        if hashrate <= self.floor:
            self.stall_count += 1
            if self.stall_count >= self.max_stall and not self.warned:
                self.warned = True
                if self.log:
                    self.log("warn", f"engine: hashrate stalled at {hashrate_string(hashrate)} for "
                                     f"{self.stall_count} consecutive samples — check device health, cooling, "
                                     "and pool connection")
            return
        if self.warned and self.log:
            self.log("info", "engine: hashrate recovered")
        self.stall_count = 0
        self.warned = False

    def stalled(self) -> bool:
        return self.warned


def publish_btc_rate(m, fetcher) -> None:
    rate, _fresh = fetcher.btc_usd_rate()
    if rate > 0:
        m.btc_usd_rate.set(rate)
    skew = fetcher.clock_skew_seconds()
    if skew > 0:
        m.clock_skew_seconds.set(skew)
    age, ever = fetcher.rate_age()
    if ever:
        m.btc_rate_age_seconds.set(age)
    ok, total, fetched = fetcher.source_health()
    if fetched:
        m.rate_sources_ok.set(ok)
        m.rate_sources_total.set(total)


def publish_difficulty(m, diff: float, hashrate: float, hashes_per_diff1: float = 4294967296.0) -> None:
    if diff <= 0:
        return
    m.pool_difficulty.set(diff)
    m.estimated_share_interval_seconds.set(diff * hashes_per_diff1 / hashrate if hashrate > 0 else 0)
