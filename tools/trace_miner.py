#!/usr/bin/env python3
"""Drive the production native miner (MinerSet -> GpuMiner thread) for a few seconds per algorithm,
for `rocprofv3 --marker-trace --kernel-trace` (tools/gpu_trace.sh): the roctx ranges
otd.{sha256d,scrypt}.batch (enqueue -> host verification) and otd.verify_candidates line up with the
kernels they cover. Prints one JSON line per algorithm with the miner's own counters."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from otedama_amd.engine.miners import MinerSet  # noqa: E402
from otedama_amd.hal import HIPDriver  # noqa: E402
from otedama_amd.models.header import int_to_hash  # noqa: E402


def run(algo: str, seconds: float, target_bits: int) -> dict:
    gpus = HIPDriver().enumerate()
    ms = MinerSet(gpus[:1], algorithm=algo)
    ms.start()
    t0 = time.perf_counter()
    ms.set_job({"header": os.urandom(76) + bytes(4), "target": int_to_hash((1 << target_bits) - 1), "job_id": algo,
                "algo": algo, "version_mask": 0x1FFFE000})
    shares = 0
    while time.perf_counter() - t0 < seconds:
        shares += len(ms.poll(4096))
        time.sleep(0.01)
    st = ms.device_stats()
    ms.stop()
    dt = time.perf_counter() - t0
    s = next(iter(st.values()))
    return {"algo": algo, "seconds": round(dt, 3), "hashes_per_sec": s["hashes"] / dt, "launches": s["launches"],
            "shares": shares, "faulted": s["faulted"], "busy_ratio": s["busy_seconds"] / dt}


if __name__ == "__main__":
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    print(json.dumps(run("sha256d", secs, 230)), flush=True)
    print(json.dumps(run("scrypt", secs, 236)), flush=True)
