#!/usr/bin/env python3
"""Interleaved in-process sweeps of the search kernels' launch geometry.

Per §5.4 rule 24 of the CDNA guide, variants are timed in interleaved rounds in
ONE process and the median/min reported. Output: one JSON line per variant.
"""
from __future__ import annotations

import argparse
import json
import statistics
import time

import torch


def time_launch(fn, reps: int) -> list[float]:
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="sha256d", choices=["sha256d", "scrypt"])
    ap.add_argument("--grids", default="")
    ap.add_argument("--gaps", default="1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--count", type=int, default=1 << 32)
    args = ap.parse_args()

    from otedama_amd.ops.native import require_native
    from otedama_amd.ops.search import ScryptSearch, Sha256dSearch

    N = require_native()
    cus = N.gpu_cu_count(0)
    hdr = bytes(range(76)) + bytes(4)
    tgt = bytes(28) + b"\xff\xff\x00\x00"
    results: dict[str, list[float]] = {}
    if args.algo == "sha256d":
        grids = [int(g) for g in args.grids.split(",")] if args.grids else [cus * k for k in (4, 5, 6, 7, 8, 12, 16)]
        searchers = {g: Sha256dSearch("cuda:0", grid=g) for g in grids}
        params = N.sha256d_prepare(hdr, tgt)
        for s in searchers.values():
            s.launch(params, 0, 1 << 28)
        for _ in range(args.rounds):
            for g, s in searchers.items():
                results.setdefault(f"grid={g}", []).extend(
                    time_launch(lambda: s.launch(params, 0, args.count), args.reps))
        for k, v in results.items():
            print(json.dumps({"algo": "sha256d", "variant": k, "count": args.count,
                              "median_s": statistics.median(v), "min_s": min(v),
                              "ghs_median": args.count / statistics.median(v) / 1e9,
                              "ghs_best": args.count / min(v) / 1e9}), flush=True)
    else:
        grids = [int(g) for g in args.grids.split(",")] if args.grids else [cus * k for k in (4, 8)]
        gaps = [int(x) for x in args.gaps.split(",")]
        params = N.scrypt_prepare(hdr, bytes(28) + b"\xff\xff\x00\x00")
        for g in grids:
            for gap in gaps:
                sc = ScryptSearch("cuda:0", grid=g, gap=gap, kernel="lane" if gap in (2, 4, 9) else "coop")
                sc.launch(params, 0)
                ts = []
                for _ in range(args.rounds * args.reps):
                    ts += time_launch(lambda: sc.launch(params, 0), 1)
                print(json.dumps({"algo": "scrypt", "grid": g, "gap": gap, "lanes": sc.batch,
                                  "scratch_gib": round(sc.scratch_bytes / 2**30, 2),
                                  "median_s": statistics.median(ts), "min_s": min(ts),
                                  "mhs_median": sc.batch / statistics.median(ts) / 1e6,
                                  "mhs_best": sc.batch / min(ts) / 1e6}), flush=True)
                del sc
                torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
