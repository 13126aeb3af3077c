"""Interleaved A/B of the hot kernels between two source trees on one GPU (each measurement a fresh process).

python tools/ab_kernels.py --a . --b ab_old [--rounds 3]
Prints one JSON line: per workload, the A and B rates of every round and their medians. Workloads: SHA-256d
two-chain version-parallel (2^35 hashes per launch), scrypt lane-cooperative ROMix (1 Mi hashes per launch),
X11 chain (2^23 nonces per launch); the ops API launches (no abort word), timed with a synchronize around N
launches after two warm-up launches.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

CHILD = r'''
import sys, time, json
sys.path.insert(0, sys.argv[1])
import torch
from otedama_amd.ops import search as S
N = S.require_native()
w = sys.argv[2]
dev = "cuda:0"
hdr = bytes(range(76)) + bytes(4)
if w == "sha256d":
    s = S.Sha256dSearchV(dev, grid=S.default_grid(dev, S.SHA256D_V2_BLOCKS_PER_CU), chains=2, occupancy8=False)
    hs = [((0x20000000 | (v << 13)) & 0xFFFFFFFF).to_bytes(4, "little") + hdr[4:] for v in range(128)]
    prep = s.prepare(hs, (1 << 200).to_bytes(32, "little"))
    run = lambda i: s.launch(prep, (i * (1 << 28)) & 0xFFFFFFFF, 1 << 28)
    per, n = 128 * (1 << 28), 6
elif w == "scrypt":
    s = S.ScryptSearch(dev)
    p = s.prepare(hdr, bytes(32))
    run = lambda i: s.launch(p, i * s.batch)
    per, n = s.batch, 8
else:
    s = S.X11Search(dev)
    p = s.prepare(hdr, bytes(32))
    run = lambda i: s.launch(p, i * s.batch)
    per, n = s.batch, 12
run(0); run(1); torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(n):
    run(i + 2)
torch.cuda.synchronize()
print(json.dumps({"rate": per * n / (time.perf_counter() - t0)}))
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default=".")
    ap.add_argument("--b", default="ab_old")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workloads", default="sha256d,scrypt,x11")
    a = ap.parse_args()
    out = {}
    for w in a.workloads.split(","):
        rows = {"a": [], "b": []}
        for _ in range(a.rounds):
            for tag, tree in (("a", a.a), ("b", a.b)):
                r = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(tree), w], capture_output=True,
                                   text=True, timeout=300)
                if r.returncode != 0:
                    print(json.dumps({"error": w, "tree": tree, "stderr": r.stderr[-2000:]}))
                    return 1
                rows[tag].append(json.loads(r.stdout.strip().splitlines()[-1])["rate"])
        ma, mb = statistics.median(rows["a"]), statistics.median(rows["b"])
        out[w] = {"a": rows["a"], "b": rows["b"], "median_a": ma, "median_b": mb, "a_over_b": ma / mb}
        print(json.dumps({w: out[w]}), flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
