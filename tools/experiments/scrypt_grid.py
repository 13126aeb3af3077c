"""scrypt ROMix pad size sweep through the ops API (one process per grid so each pad is freed): MH/s at
16 / 20 / 24 / 28 blocks per CU (128 / 160 / 192 / 224 GiB of pad), interleaved rounds.
python tools/scrypt_grid.py [--rounds 2]  -> one JSON line."""
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
bpc = int(sys.argv[2])
dev = "cuda:0"
s = S.ScryptSearch(dev, grid=S.default_grid(dev, bpc))
p = s.prepare(bytes(range(76)) + bytes(4), bytes(32))
for i in range(2):
    s.launch(p, i * s.batch)
torch.cuda.synchronize()
n = max(3, int(3.0 * 16.5e6 / s.batch))
t0 = time.perf_counter()
for i in range(n):
    s.launch(p, (i + 2) * s.batch)
torch.cuda.synchronize()
print(json.dumps({"rate": s.batch * n / (time.perf_counter() - t0), "batch": s.batch}))
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--bpc", default="16,20,24,28")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    res: dict = {}
    for _ in range(a.rounds):
        for b in a.bpc.split(","):
            out = subprocess.run([sys.executable, "-c", CHILD, root, b], capture_output=True, text=True, timeout=300)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if out.returncode != 0 or not line:
                print(json.dumps({"error": b, "stderr": out.stderr[-1500:]}))
                return 1
            res.setdefault(b, []).append(json.loads(line[0])["rate"])
    print(json.dumps({b: {"rates": v, "median": statistics.median(v)} for b, v in res.items()}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
