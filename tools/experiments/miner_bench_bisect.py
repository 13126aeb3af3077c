"""Bisect bench.py's preamble for the production miner's lower scrypt rate inside bench.py (16.2 vs 17.3 MH/s in a
fresh process, profiles/r4/e_miner_ctx). Each variant is a fresh child that replays a prefix of what bench.py does
before its miner section, then runs engine/miner_probe.measure_miner on scrypt. One JSON line per variant.

Usage: python tools/miner_bench_bisect.py [--seconds 6]"""
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
stage, secs = int(sys.argv[2]), float(sys.argv[3])
import torch
from otedama_amd.ops.native import require_native
from otedama_amd.engine.miner_probe import measure_miner
from otedama_amd.models.header import int_to_hash
N = require_native()
torch.zeros(1, device="cuda:0")
if stage >= 1:  # bench.py's rank set-up: process info, NodeComm buffers and its comm stream
    from otedama_amd.parallel import NodeComm, init_from_env
    info = init_from_env(use_gpu=True)
    comm = NodeComm(info)
if stage >= 2:  # the SHA-256d section: version-parallel launches alternating over the current stream and s1
    from otedama_amd.ops.search import SHA256D_V2_BLOCKS_PER_CU, Sha256dSearchV, default_grid
    dev = torch.device("cuda:0")
    s1 = torch.cuda.Stream(dev)
    search = Sha256dSearchV(dev, grid=default_grid(dev, SHA256D_V2_BLOCKS_PER_CU), chains=2, occupancy8=False)
    hdrs = [bytes([v]) + bytes(79) for v in range(128)]
    prep = search.prepare(hdrs, int_to_hash((1 << 200) - 1))
    out = torch.zeros(1 + 2 * search.cap, dtype=torch.int32, device=dev)
    s0 = torch.cuda.current_stream(dev)
    for j in range(8):
        search.launch_into(prep, j << 25, 1 << 25, out, s0 if j % 2 == 0 else s1)
    torch.cuda.synchronize()
if stage >= 3:  # the scrypt kernel section (ops API, its own 128 GiB pad), then freed
    from otedama_amd.ops.search import ScryptSearch
    sc = ScryptSearch("cuda:0")
    prm = N.scrypt_prepare(bytes(80), int_to_hash(0xFFFF << 224))
    for i in range(4):
        sc.launch(prm, i * sc.batch)
    torch.cuda.synchronize()
    del sc
    torch.cuda.empty_cache()
r = measure_miner(N, 0, "scrypt", 0xFFFF << 224, seconds=secs, warmup=2.0, recheck=8)
print(json.dumps({k: r[k] for k in ("hashes_per_sec", "launches", "window_device_seconds", "window_wall_seconds")}))
'''
STAGES = ["torch_only", "+rank_setup", "+sha_section", "+scrypt_kernel_section"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    a = ap.parse_args()
    for stage, name in enumerate(STAGES):
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(stage), str(a.seconds)], capture_output=True,
                             text=True, timeout=200)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        rec = json.loads(line[0]) if line else {"error": out.returncode, "stderr": out.stderr[-800:]}
        print(json.dumps({"variant": name, **rec}), flush=True)
        if not line:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
