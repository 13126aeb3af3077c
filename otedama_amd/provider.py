"""Revenue-stream providers publishing periodic yield quotes.

Parity: internal/provider
  * Yield (gross / net sats/s, confidence; Effective uses NET) ..... provider.go:92-114
  * Quote / Provider / RateSource / SatsPerSecond ................... provider.go:117-175
  * pollingProvider: publish now + every interval, drop-oldest send  polling.go:38-119
  * MiningProvider "mining.stratum": sats/s = H/1e21 x 3.125 BTC /
    600 s x 1e8, 1% pool fee, confidence 0.95 fresh / 0.7 stale,
    static per-family fallback hashrates ............................ mining.go:44-144
  * AkashProvider "ai.akash" (simulated, GPU-only): midpoint of
    $0.30-0.60/h, 20% fee, confidence 0.85 / 0.6 .................... ai_inference.go:55-142
  * StaticRateSource ................................................. ai_inference.go:150-156
The live HashrateFunc feeds the measured per-device rate (the gfx950 kernels
run ~16 GH/s per GPU), so the fallback table is only used before the first
stats tick.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field
from typing import Callable

from otedama_amd.hal import Family

MIN_QUOTE_INTERVAL = 30.0
NETWORK_HASHRATE = 1e21
BLOCK_REWARD_BTC = 3.125
BLOCK_TIME_SEC = 600.0
FALLBACK_BTC_USD = 95_000.0
DEFAULT_HASHRATES = {Family.ASIC: 100e12, Family.GPU: 1.5e9, Family.CPU: 10e6}


@dataclass(frozen=True)
class Yield:
    sats_per_second: float = 0.0
    net_sats_per_second: float = 0.0
    confidence: float = 0.0

    def effective(self) -> float:
        if self.net_sats_per_second <= 0 or self.confidence <= 0:
            return 0.0
        return self.net_sats_per_second * self.confidence


@dataclass
class Quote:
    provider_id: str
    device_id: str = ""
    yield_: Yield = field(default_factory=Yield)
    accepted_families: list[Family] = field(default_factory=list)
    at: float = field(default_factory=time.time)


def sats_per_second(usd_per_hour: float, btc_usd: float) -> float:
    if btc_usd <= 0 or usd_per_hour <= 0:
        return 0.0
    return usd_per_hour / btc_usd * 1e8 / 3600


class StaticRateSource:
    def __init__(self, rate: float):
        self.rate = rate

    def btc_usd_rate(self) -> tuple[float, bool]:
        return self.rate, True


class PollingProvider:
    id = ""
    queue_size = 16

    def __init__(self, interval: float):
        self.interval = interval
        self.quotes: asyncio.Queue = asyncio.Queue(maxsize=self.queue_size)
        self._task: asyncio.Task | None = None
        self.devices: list = []

    def name(self) -> str:
        return self.id

    def prepare(self, devices: list) -> None:
        self.devices = list(devices)

    def start(self, devices: list) -> None:
        if self._task is not None:
            raise RuntimeError(f"provider: {self.id} already started")
        self.prepare(devices)
        self._task = asyncio.ensure_future(self._loop())

    async def _loop(self) -> None:
        while True:
            self.publish()
            await asyncio.sleep(self.interval)

    def send_quote(self, q: Quote) -> None:
        try:
            self.quotes.put_nowait(q)
        except asyncio.QueueFull:
            try:
                self.quotes.get_nowait()
            except asyncio.QueueEmpty:
                pass
            self.quotes.put_nowait(q)

    def publish(self) -> None:
        raise NotImplementedError

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._task = None
            self.quotes = asyncio.Queue(maxsize=self.queue_size)


class MiningProvider(PollingProvider):
    id = "mining.stratum"
    queue_size = 16

    def __init__(self, pool_url: str, rates, interval: float = 30.0,
                 hashrate_func: Callable[[str], float] | None = None, algorithm: str = "sha256d"):
        super().__init__(interval)
        self.pool_url = pool_url
        self.rates = rates
        self.hashrate_func = hashrate_func
        self.algorithm = algorithm

    def name(self) -> str:
        return f"Bitcoin Mining ({self.pool_url})"

    def publish(self) -> None:
        rate, fresh = self.rates.btc_usd_rate()
        confidence = 0.95 if fresh else 0.7
        fams = [Family.ASIC, Family.GPU, Family.CPU]
        for dev in self.devices:
            if not dev.capabilities().supports(self.algorithm):
                continue
            h = self.hashrate_func(dev.identity().id) if self.hashrate_func else 0.0
            if h <= 0:
                h = DEFAULT_HASHRATES.get(dev.identity().family, 10e6)
            sats = h / NETWORK_HASHRATE * BLOCK_REWARD_BTC / BLOCK_TIME_SEC * 1e8
            self.send_quote(Quote(self.id, dev.identity().id, Yield(sats, sats * 0.99, confidence), fams))


class AkashProvider(PollingProvider):
    id = "ai.akash"
    queue_size = 32

    def __init__(self, rates, interval: float = 60.0, min_usd_per_hour: float = 0.30, max_usd_per_hour: float = 0.60):
        super().__init__(interval)
        self.rates = rates
        self.min_usd_per_hour = min_usd_per_hour
        self.max_usd_per_hour = max_usd_per_hour

    def name(self) -> str:
        return "AI Inference (Akash Network, simulated)"

    def prepare(self, devices: list) -> None:
        self.devices = [d for d in devices if d.identity().family == Family.GPU and d.capabilities().general_compute]

    def publish(self) -> None:
        if not self.devices:
            self.send_quote(Quote(self.id, "", Yield(confidence=0.0), [Family.GPU]))
            return
        rate, fresh = self.rates.btc_usd_rate()
        if rate <= 0:
            rate = FALLBACK_BTC_USD
        confidence = 0.85 if fresh else 0.6
        usd = (self.min_usd_per_hour + self.max_usd_per_hour) / 2.0
        for dev in self.devices:
            self.send_quote(Quote(self.id, dev.identity().id,
                                  Yield(sats_per_second(usd, rate), sats_per_second(usd * 0.80, rate), confidence),
                                  [Family.GPU]))
