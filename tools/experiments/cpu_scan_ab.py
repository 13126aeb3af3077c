"""CPU SHA-256d (BASELINE config 1): the SHA-NI scan (OTEDAMA_CPU_LANES=4 / 2) against the 16-lane AVX-512 scan
(=16; "16g2" = two 16-lane groups in flight, OTEDAMA_CPU_SCAN_GROUPS=2), single thread and on this process's CPU share through the production CpuMiner (otedama_amd/cli/bench_cmd.py
``bench_cpu``). Each variant runs in a fresh process (the lane choice is read once), rounds interleaved. One JSON line
per run, then the medians."""
from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = ("import json, sys; sys.path.insert(0, sys.argv[1]); from otedama_amd.cli.bench_cmd import bench_cpu, cpu_share; "
         "r = bench_cpu(seconds=3.0, threads=cpu_share(), single_seconds=2.0); "
         "print(json.dumps({k: r[k] for k in ('sha256d_single_thread_hps', 'sha256d_all_threads_hps', 'threads')}))")


def main() -> int:
    variants = sys.argv[1:] or ["4", "16"]
    res: dict[str, list[dict]] = {v: [] for v in variants}
    for _ in range(2):
        for v in variants:
            lanes, _, groups = v.partition("g")
            env = dict(os.environ, OTEDAMA_CPU_LANES=lanes, OTEDAMA_CPU_SCAN_GROUPS=groups or "1")
            out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True,
                                 timeout=120)
            rec = json.loads(out.stdout.strip().splitlines()[-1])
            res[v].append(rec)
            print(json.dumps({"lanes": v, **rec}), flush=True)
    print(json.dumps({"median_single_mhs": {v: round(statistics.median(r["sha256d_single_thread_hps"] for r in rs) / 1e6, 2)
                                            for v, rs in res.items()},
                      "median_all_mhs": {v: round(statistics.median(r["sha256d_all_threads_hps"] for r in rs) / 1e6, 1)
                                         for v, rs in res.items()},
                      "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
