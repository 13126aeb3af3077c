"""Where a device process's ~1 GB of host memory goes, and which knobs move it.

Each variant is a fresh torch-free child (the device process's own import path) that records, at every start-up
phase, its RSS and an smaps breakdown grouped by mapping (anonymous private memory, the ROCm / HIP libraries, the
extension, /dev/kfd and render-node mappings), and finally the production miner's SHA-256d rate over an exact
device-timeline window. Variants: the default, the HIP queue ring buffers / context-save areas in device memory
(HSA_ALLOCATE_QUEUE_DEV_MEM=1), one search stream instead of two (OTEDAMA_SEARCH_STREAMS=1), both, and the two
search streams sharing one hardware queue (GPU_MAX_HW_QUEUES=1).

Usage: python tools/rss_breakdown.py [--seconds 6]   (one JSON line per variant)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
os.environ["OTEDAMA_NO_TORCH"] = "1"
secs = float(sys.argv[2])

def rss():
    with open("/proc/self/statm") as f:
        return round(int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20, 1)

def smaps():
    """Rss (MiB) by mapping: anonymous mappings bucketed by size, files by basename, devices by path."""
    groups, name, size_kb = {}, "?", 0
    big = []
    with open("/proc/self/smaps") as f:
        for line in f:
            parts = line.split()
            if parts and "-" in parts[0] and len(parts) >= 5 and not parts[0].endswith(":"):
                lo, hi = (int(x, 16) for x in parts[0].split("-"))
                size_kb = (hi - lo) // 1024
                path = parts[5] if len(parts) >= 6 else ""
                if not path:
                    name = "anon"
                elif path.startswith("/dev/"):
                    name = path
                elif path.startswith("["):
                    name = path
                else:
                    name = os.path.basename(path)
            elif parts and parts[0] == "Rss:":
                kb = int(parts[1])
                groups[name] = groups.get(name, 0) + kb
                if name == "anon" and kb >= 16 * 1024:
                    big.append([round(size_kb / 1024, 1), round(kb / 1024, 1)])
    top = sorted(((k, round(v / 1024, 1)) for k, v in groups.items() if v >= 1024), key=lambda kv: -kv[1])
    return {"by_mapping_mib": dict(top[:14]), "anon_mappings_ge_16mib": sorted(big, key=lambda x: -x[1])[:24]}

out = {"start_mib": rss()}
from otedama_amd.models.header import int_to_hash
from otedama_amd.ops.native import require_native
N = require_native()
out["native_imported_mib"] = rss()
cus = N.gpu_cu_count(0)
out["hip_runtime_up_mib"] = rss()
m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, grid=cus * 6, queue_cap=4096, sha_variants=128)
m.start()
hdr = bytes(range(76)) + bytes(4)
m.set_job({"header": hdr, "target": int_to_hash((1 << 200) - 1), "job_id": "r", "epoch": 1, "algo": "sha256d",
           "version_mask": 0x1FFFE000})
time.sleep(2.0)
out["sha_running_mib"] = rss()
out["smaps_sha_running"] = smaps()
st = m.stats()
out["miner_phase_rss_mib"] = st.get("startup_rss_mb")
h0, d0 = st["hashes"], st["hashes_done_at_s"]
time.sleep(secs)
st = m.stats()
out["sha256d_hps"] = (st["hashes"] - h0) / max(st["hashes_done_at_s"] - d0, 1e-9)
out["faulted"] = st["faulted"]
out["host_abort"] = st.get("host_abort")
out["clock_samples"] = st.get("clock_samples")
m.stop()
print(json.dumps(out))
'''

VARIANTS = [
    ("default", {}),
    # the round-3 layout: the abort word stored through a high-priority control stream (one more hardware queue)
    ("control_stream", {"OTEDAMA_HOST_ABORT": "0"}),
    ("queue_dev_mem", {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1"}),
    ("one_search_stream", {"OTEDAMA_SEARCH_STREAMS": "1"}),
    ("queue_dev_mem+one_search_stream", {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1", "OTEDAMA_SEARCH_STREAMS": "1"}),
    # both search streams multiplexed onto one normal-priority hardware queue (the control stream keeps its own)
    ("hw_queues_1", {"GPU_MAX_HW_QUEUES": "1"}),
    # ... and ROCr's host-memory fragment allocator off (the /dev/zero mappings, ~55 MiB)
    ("hw_queues_1+no_fragments", {"GPU_MAX_HW_QUEUES": "1", "HSA_DISABLE_FRAGMENT_ALLOCATOR": "1"}),
]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--only", default="", help="comma list of variant names")
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))
    for name, extra in VARIANTS:
        if only and name not in only:
            continue
        env = dict(os.environ, **extra)
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(a.seconds)], capture_output=True, text=True,
                             timeout=120, env=env)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if out.returncode != 0 or not line:
            print(json.dumps({"variant": name, "error": out.returncode, "stderr": out.stderr[-1500:]}), flush=True)
            return 1
        print(json.dumps({"variant": name, "env": extra, **json.loads(line[0])}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
