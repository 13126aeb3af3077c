"""X11 per-stage timing and chain hashrate on one MI355X.

python tools/bench_x11.py [--batch 2^23] [--iters 5]
Prints one JSON line: chain MH/s and the per-stage ms / share of the chain.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAGES = ["blake", "bmw", "groestl", "skein", "jh", "keccak", "luffa", "cubehash", "shavite", "simd", "echo"]


def main() -> int:
    import torch

    from otedama_amd.ops.search import X11Search

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 23)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    s = X11Search("cuda:0", batch=a.batch)
    hdr = bytes(range(80))
    params = s.prepare(hdr, bytes(32))  # target 0: no hits
    stream = torch.cuda.current_stream()
    for _ in range(2):
        s.launch(params, 0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(12)]
    per = [0.0] * 11
    for _ in range(a.iters):
        for st in range(11):
            ev[st].record(stream)
            s.native.launch_x11_stage(params, st, 0, s.H.data_ptr(), s.batch, s.batch,
                                      s.out.data_ptr() if st == 10 else 0, s.cap if st == 10 else 0,
                                      stream.cuda_stream)
        ev[11].record(stream)
        torch.cuda.synchronize()
        for st in range(11):
            per[st] += ev[st].elapsed_time(ev[st + 1]) / a.iters
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(stream)
    base = 0
    for _ in range(a.iters):
        s.launch(params, base)
        base += s.batch
    t1.record(stream)
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / a.iters
    tot = sum(per)
    print(json.dumps({
        "metric": "x11_hashrate", "mhs": round(s.batch / ms / 1e3, 2), "ms_per_batch": round(ms, 3), "batch": s.batch,
        "stages_ms": {n: round(v, 3) for n, v in zip(STAGES, per)},
        "stages_pct": {n: round(100 * v / tot, 1) for n, v in zip(STAGES, per)},
    }))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
