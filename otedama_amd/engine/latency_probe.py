"""End-to-end share-latency probe (BASELINE metric "p50 share latency").

Runs the real engine on one GPU against the in-process local pool over a
loopback Stratum V2 connection for a few seconds and reports:
  * submit -> accept quantiles (the reference's definition:
    otedama_submit_latency_milliseconds, internal/engine/run.go:813-821), and
  * hit -> accept quantiles: from the moment the host runtime verified the
    kernel's candidate to the pool's SubmitSharesSuccess (native share queue +
    asyncio submit + pool-side re-hash / validation).
The reference never published a number for this.
"""
from __future__ import annotations

import asyncio

from otedama_amd import hal
from otedama_amd.config import Config, MiningConfig, PoolConfig
from otedama_amd.engine.run import Engine, Options
from otedama_amd.pool.server import PoolOptions, PoolServer
from otedama_amd.provider import StaticRateSource

PROBE_ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


async def _probe(device_index: int, seconds: float, algorithm: str, shares_per_sec: float, batch_nonces: int,
                 expected_hashrate: float) -> dict:
    devs = [d for d in hal.HIPDriver().enumerate() if d.index == device_index]
    if not devs:
        raise RuntimeError(f"no HIP device {device_index}")
    hashes_per_diff1 = 2.0 ** 16 if algorithm == "scrypt" else 2.0 ** 32  # scrypt pools: diff1 = 0xFFFF << 224
    diff = expected_hashrate / (shares_per_sec * hashes_per_diff1)
    pool = PoolServer(PoolOptions(algorithm=algorithm, initial_difficulty=diff, retarget_seconds=3600,
                                  payout_address=PROBE_ADDR, listen_v1=""))
    await pool.start()
    cfg = Config(bitcoin_address=PROBE_ADDR, pools=[PoolConfig(url=f"stratum+v2://{pool.addr_sv2}")],
                 mining=MiningConfig(algorithm=algorithm, batch_nonces=batch_nonces))
    eng = Engine(Options(config=cfg, devices=devs, rate_fetcher=StaticRateSource(95000), stats_interval=1.0))
    task = asyncio.ensure_future(eng.run())
    await asyncio.sleep(seconds)
    task.cancel()
    try:
        await task
    except (asyncio.CancelledError, Exception):  # noqa: BLE001
        pass
    await pool.stop()
    lat, pipe = eng.latency, eng.pipeline_latency
    return {
        "p50_ms": lat.quantile(0.5), "p95_ms": lat.quantile(0.95), "p99_ms": lat.quantile(0.99),
        "hit_to_accept_p50_ms": pipe.quantile(0.5), "hit_to_accept_p95_ms": pipe.quantile(0.95),
        "accepted": eng.m.shares_accepted.value(), "rejected": eng.m.shares_rejected.value(),
        "pool_accepted": pool.accepted, "pool_rejected": pool.rejected, "share_difficulty": diff,
        "batch_nonces": batch_nonces, "seconds": seconds, "protocol": "stratum-v2 (loopback)",
        "engine_hashrate": eng.current_hashrate,
    }


def measure_share_latency(device_index: int = 0, seconds: float = 6.0, algorithm: str = "sha256d",
                          shares_per_sec: float = 40.0, batch_nonces: int = 1 << 27,
                          expected_hashrate: float = 16e9) -> dict:
    return asyncio.run(_probe(device_index, seconds, algorithm, shares_per_sec, batch_nonces, expected_hashrate))
