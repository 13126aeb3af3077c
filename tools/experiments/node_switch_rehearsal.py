#!/usr/bin/env python3
"""Node-wide job switch and per-algorithm node runs, rehearsed on the one-GPU box.

With OTEDAMA_DIST_BACKEND=gloo, ``otedama node --gpus N`` runs N ranks that share GPU 0 (one device process each,
the same op log / doorbell / job-preview control plane as the RCCL node). For each (world, algorithm) this runs
parallel/node_probe.measure_node with forced new blocks at the pool and prints one JSON line: the node hashrate, the
per-rank switch latency (pool send -> each rank's device running the new work) and the stale rejects.

Usage: OTEDAMA_DIST_BACKEND=gloo python tools/node_switch_rehearsal.py [--worlds 2,4] [--algorithms sha256d]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    from otedama_amd.parallel.node_probe import EXPECTED_RATE, measure_node

    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4")
    ap.add_argument("--algorithms", default="sha256d")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--switches", type=int, default=8)
    ap.add_argument("--cpu", action="store_true", help="CPU miners instead of the GPU (container rehearsal)")
    a = ap.parse_args()
    for algo in [x for x in a.algorithms.split(",") if x]:
        for world in [int(x) for x in a.worlds.split(",") if x]:
            print(f"[rehearsal] {algo} world {world}", file=sys.stderr, flush=True)
            # the ranks share one GPU: size the pinned difficulty for 1/world of its rate per rank
            per = EXPECTED_RATE["cpu" if a.cpu else "gpu"][algo] / (1 if a.cpu else world)
            try:
                r = measure_node(world, seconds=a.seconds, warmup=3.0, cpu=a.cpu, algorithm=algo,
                                 switches=a.switches, expected_per_gpu=per, shares_per_gpu=25.0 / world)
            except Exception as exc:  # noqa: BLE001 - one failed configuration must not hide the others
                r = {"error": f"{type(exc).__name__}: {exc}"}
            r.pop("per_device_hashes_per_sec", None)
            print(json.dumps({"algorithm": algo, "world": world, "backend": os.environ.get("OTEDAMA_DIST_BACKEND"),
                              **r}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
