"""scrypt ROMix: one launch per batch (both phases in each wave) vs split phases (pad writes, then lookups, as two
launches). Checks that both report the same nonces as hashlib on an easy target first, then times each over grids.

python tools/bench_scrypt_split.py [--grids 2048,4096,5120] [--reps 4]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    import torch

    from otedama_amd.ops.search import ScryptSearch

    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="2048,4096,5120")
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    hdr = bytes(range(76)) + bytes(4)
    easy = (((1 << 256) - 1) >> 6).to_bytes(32, "little")  # ~1 in 64
    want = sorted(n for n in range(2048) if int.from_bytes(
        hashlib.scrypt(hdr[:76] + n.to_bytes(4, "little"), salt=hdr[:76] + n.to_bytes(4, "little"), n=1024, r=1,
                       p=1, dklen=32), "little") <= int.from_bytes(easy, "little"))
    for kernel in ("coop", "split"):
        got = sorted(ScryptSearch("cuda:0", grid=64, kernel=kernel).search(hdr, easy, 0, 2048))
        r = {"check": kernel, "hits": len(got), "expected": len(want), "ok": got == want}
        print(json.dumps(r), flush=True)
        if not r["ok"]:
            return 1
    tgt = bytes(32)
    for grid in [int(x) for x in a.grids.split(",") if x]:
        for kernel in ("coop", "split"):
            s = ScryptSearch("cuda:0", grid=grid, kernel=kernel)
            p = s.prepare(hdr, tgt)
            s.launch(p, 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.reps):
                s.launch(p, i * s.batch)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"kernel": kernel, "grid": grid, "pad_gib": round(s.scratch_bytes / 2**30, 1),
                              "mhs": round(a.reps * s.batch / dt / 1e6, 3)}), flush=True)
            del s
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
