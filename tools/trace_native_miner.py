#!/usr/bin/env python3
"""The production native miner (GpuMiner) in this one process, for `rocprofv3 --kernel-trace --stats`: a few seconds
of SHA-256d, scrypt and X11 each, so the kernel statistics show the per-launch clock probes and the search kernels
side by side, with no child process (a profiled process must not start other programs).

Usage: python3 tools/trace_native_miner.py [seconds_per_algorithm] [algo,algo,...]   (one JSON line per algorithm)"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["OTEDAMA_NO_TORCH"] = "1"

from otedama_amd.models.header import int_to_hash  # noqa: E402
from otedama_amd.ops.native import require_native  # noqa: E402

TARGET_BITS = {"sha256d": 226, "scrypt": 240, "x11": 236}


def run(N, algo: str, seconds: float) -> dict:
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, grid=N.gpu_cu_count(0) * 6, queue_cap=65536, sha_variants=128)
    m.set_job({"header": os.urandom(76) + bytes(4), "target": int_to_hash((1 << TARGET_BITS[algo]) - 1),
               "job_id": algo, "epoch": 1, "algo": algo, "version_mask": 0x1FFFE000})
    m.start()
    shares = 0
    t0 = time.monotonic()
    s0 = None
    while time.monotonic() - t0 < seconds:
        shares += len(m.poll(65536))
        if s0 is None and time.monotonic() - t0 > 1.0:
            s0 = m.stats()
        time.sleep(0.05)
    s1 = m.stats()
    m.stop()
    span = s1["hashes_done_at_s"] - s0["hashes_done_at_s"] if s0 else 0.0
    return {"algo": algo, "hashes_per_sec": (s1["hashes"] - s0["hashes"]) / span if span > 0 else None,
            "launches": s1["launches"], "shares": shares, "rejected_candidates": s1["rejected_candidates"],
            "clock_samples": s1.get("clock_samples"), "host_abort": s1.get("host_abort"), "faulted": s1["faulted"]}


def main() -> int:
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    N = require_native()
    algos = sys.argv[2].split(",") if len(sys.argv) > 2 else ("sha256d", "scrypt", "x11")
    for algo in algos:
        print(json.dumps(run(N, algo, secs)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
