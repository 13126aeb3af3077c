"""SHA-256d: single-midstate kernel vs the K-variant shared-schedule kernel over K and the grid.

python tools/bench_sha_k.py [--count LOG2] [--ks 4,8,16] [--bpc 4,8]
  -> one JSON line per (kernel, grid): GH/s per GPU (hashes = K x count per launch)
"""
from __future__ import annotations

import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=32, help="log2 nonces per variant per launch")
    ap.add_argument("--ks", default="2,3,4,6,8,12,16")
    ap.add_argument("--bpc", default="4,6,8", help="blocks of 256 per CU")
    a = ap.parse_args()
    count = 1 << a.count

    from otedama_amd.ops.search import Sha256dSearch, Sha256dSearchK

    tail = bytes(range(4, 76)) + bytes(4)
    headers = [struct.pack("<I", 0x20000000 | (v << 13)) + tail for v in range(16)]
    target = bytes(32)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(launch, hashes, reps=3):
        launch()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(reps):
            launch()
        ev1.record()
        torch.cuda.synchronize()
        return hashes * reps / (ev0.elapsed_time(ev1) * 1e-3)

    s1 = Sha256dSearch("cuda:0")
    p1 = s1.prepare(headers[0], target)
    print(json.dumps({"kernel": "k1", "grid": s1.grid, "ghs": round(run(lambda: s1.launch(p1, 0, count), count) / 1e9, 3)}),
          flush=True)
    for k in map(int, a.ks.split(",")):
        for bpc in map(int, a.bpc.split(",")):
            s = Sha256dSearchK("cuda:0", k=k, grid=cus * bpc)
            p = s.prepare(headers[:k], target)
            rate = run(lambda: s.launch(p, 0, count), k * count)
            print(json.dumps({"kernel": f"k{k}", "grid": s.grid, "ghs": round(rate / 1e9, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
