"""Local-pool throughput: BASELINE.json config 5 ("Full Stratum pool: mixed SHA-256d + scrypt workers,
share validation + vardiff").

N simulated SV2 miners (the production V2 client, `poolproto.stratumv2`) connect to an in-process
PoolServer per algorithm and submit shares as fast as the pool acknowledges them, `--inflight` per miner.
Difficulty is pinned at the minimum, so every nonce is a valid share. The pool still rebuilds the header
(coinbase + merkle), checks stale/duplicate/ntime/version rules, recomputes the PoW hash (SHA-256d
inline, scrypt on its native thread pool), journals the share and runs vardiff.

Output: one JSON line per pool with validated shares/s and submit->ack latency quantiles (the pool section of
bench.py reports it as the pool's flood capacity; tools/bench_pool.py is the command-line wrapper).
Usage: python -m otedama_amd.pool.load [--algo sha256d|scrypt|x11|mixed|a,b] [--miners 16] [--seconds 10]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import statistics
import sys
import time

from otedama_amd.pool.server import PoolOptions, PoolServer
from otedama_amd.poolproto.base import Credentials, ShareSubmission
from otedama_amd.poolproto.stratumv2 import V2Dialer

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


async def _miner(url: str, algo: str, idx: int, deadline: float, inflight: int, lat: list, counts: dict):
    s = await V2Dialer().dial(url, Credentials(user=f"{ADDR}.m{idx}", worker=f"m{idx}"), algorithm=algo)
    job = await asyncio.wait_for(s.jobs.get(), 30)
    nonce = idx << 24

    async def one():
        nonlocal nonce
        while time.perf_counter() < deadline:
            nonce += 1
            r = await s.submit(ShareSubmission(job.job_id, nonce & 0xFFFFFFFF, job.ntime, job.version))
            counts["ok" if r.accepted else r.reason] = counts.get("ok" if r.accepted else r.reason, 0) + 1
            if r.accepted:
                lat.append(r.latency_ms)

    try:
        await asyncio.gather(*(one() for _ in range(inflight)))
    finally:
        await s.close()


async def _run_pool(algo: str, miners: int, seconds: float, inflight: int) -> dict:
    # difficulty 1e-12: the share target overflows and is clamped to 2^256-1 for both algorithms
    pool = PoolServer(PoolOptions(algorithm=algo, initial_difficulty=1e-12, min_difficulty=1e-12,
                                  payout_address=ADDR, retarget_seconds=1e9, target_share_seconds=1e-12))
    pool.vardiff.cfg.min_shares = 1 << 62  # keep every share valid: vardiff still runs, never retargets
    await pool.start()
    url = f"stratum+v2://{pool.addr_sv2}"
    lat: list[float] = []
    counts: dict[str, int] = {}
    t0 = time.perf_counter()
    await asyncio.gather(*(_miner(url, algo, i, t0 + seconds, inflight, lat, counts) for i in range(miners)))
    dt = time.perf_counter() - t0
    await pool.stop()
    lat.sort()
    q = (lambda p: lat[min(len(lat) - 1, int(p * len(lat)))] if lat else None)
    return {"pool": algo, "miners": miners, "inflight_per_miner": inflight, "seconds": round(dt, 2),
            "validated_shares_per_sec": pool.accepted / dt, "accepted": pool.accepted,
            "rejected": pool.rejected, "client_verdicts": counts,
            "ack_latency_ms": {"p50": q(0.5), "p95": q(0.95), "p99": q(0.99),
                               "mean": statistics.fmean(lat) if lat else None}}


async def main_async(args) -> list[dict]:
    algos = ["sha256d", "scrypt", "x11"] if args.algo == "mixed" else [a for a in args.algo.split(",") if a]
    per = max(1, args.miners // len(algos))
    return list(await asyncio.gather(*(_run_pool(a, per, args.seconds, args.inflight) for a in algos)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="mixed", help="sha256d, scrypt, x11, mixed (all three) or a comma list")
    ap.add_argument("--miners", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--inflight", type=int, default=8)
    args = ap.parse_args()
    for r in asyncio.run(main_async(args)):
        print(json.dumps(r))
    return 0


if __name__ == "__main__":
    sys.exit(main())
