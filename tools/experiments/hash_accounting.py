#!/usr/bin/env python3
"""Does the production miner's hash counter match the work its hits prove? (round 6)

The pool probe saw ~4% fewer accepted scrypt shares than the miner's counted hashes imply, on three boxes. Here the
native GpuMiner (in this process, no torch) runs one algorithm against a target whose top word alone decides a hit
(target = (top + 1) * 2^224 - 1), so the kernel's candidate count is an exact Poisson count with mean
hashes * (top + 1) / 2^32, independent of the host verifier. Reported per mode: counted hashes, candidates, their
expectation and the z-score. Modes: scrypt with the two staggered halves (the default) and OTEDAMA_SCRYPT_HALVES=0
(read at miner construction), SHA-256d and X11 as controls.

Usage: python tools/experiments/hash_accounting.py [seconds]   (one JSON line per mode)
"""
from __future__ import annotations

import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["OTEDAMA_NO_TORCH"] = "1"

from otedama_amd.models.header import int_to_hash  # noqa: E402
from otedama_amd.ops.native import require_native  # noqa: E402

TOP = {"sha256d": (1 << 8) - 1, "scrypt": (1 << 17) - 1, "x11": (1 << 14) - 1}  # 2^-24, 2^-15, 2^-18 per hash


def run(N, algo: str, seconds: float) -> dict:
    top = TOP[algo]
    target = ((top + 1) << 224) - 1
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, grid=N.gpu_cu_count(0) * 6, queue_cap=1 << 20, sha_variants=128)
    m.set_job({"header": os.urandom(76) + bytes(4), "target": int_to_hash(target), "job_id": algo, "epoch": 1,
               "algo": algo, "version_mask": 0x1FFFE000})
    m.start()
    time.sleep(2.0)
    s0 = m.stats()
    t0 = time.monotonic()
    while time.monotonic() - t0 < seconds:
        m.poll(1 << 20)
        time.sleep(0.02)
    s1 = m.stats()
    m.stop()
    hashes = s1["hashes"] - s0["hashes"]
    cand = s1["candidates"] - s0["candidates"]
    exp = hashes * (top + 1) / 2.0 ** 32
    span = s1["hashes_done_at_s"] - s0["hashes_done_at_s"]
    return {"algo": algo, "halves": os.environ.get("OTEDAMA_SCRYPT_HALVES", "1") != "0", "hashes": hashes,
            "hashes_per_sec": hashes / span if span > 0 else None, "candidates": cand, "expected": exp,
            "ratio_found_over_expected": cand / exp if exp else None,
            "z": (cand - exp) / math.sqrt(exp) if exp else None,
            "launches": s1["launches"] - s0["launches"], "aborted": s1["aborted_launches"] - s0["aborted_launches"],
            "ring_overflow": s1.get("ring_overflow")}


def main() -> int:
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    algos = sys.argv[2].split(",") if len(sys.argv) > 2 else ["scrypt", "sha256d", "x11"]
    N = require_native()
    for algo in algos:
        print(json.dumps(run(N, algo, secs)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
