"""SHA-256d: K-variant kernel (K=8, schedule per lane on the VALU) vs the version-parallel kernels (64 x NC variants
per wave, NC per lane, schedule on the scalar unit), with bit-exactness checks against the CPU / the one-chain kernel.

python tools/bench_sha_v.py [--count LOG2] [--groups 1,2] [--bpc ...] [--bpc8 ...] [--block64-bpc ...]
                            [--chains2-bpc ...] [--chains2-block64-bpc ...] [--chainsn "3:bpc,..;4:bpc,.."]
  -> one JSON line per (kernel, grid, groups): GH/s per GPU
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def headers_for(n: int) -> list[bytes]:
    tail = bytes(range(4, 76)) + bytes(4)
    return [struct.pack("<I", 0x20000000 | ((v & 0xFFFF) << 13)) + tail for v in range(n)]


def check(dev: str, block: int = 256) -> dict:
    """Easy target: every hit of a small W3 window must be a true share, and every true share must be hit."""
    from otedama_amd.ops.search import Sha256dSearchV

    s = Sha256dSearchV(dev, block=block)
    hs = headers_for(64)
    target = (((1 << 248) - 1)).to_bytes(32, "little")  # ~1 in 256
    base, count = 0x12345600, 2048
    got = sorted(s.search(hs, target, base, count))
    want = []
    for vi, h in enumerate(hs):
        for w3 in range(base, base + count):
            nonce = int.from_bytes(w3.to_bytes(4, "big"), "little")
            d = hashlib.sha256(hashlib.sha256(h[:76] + nonce.to_bytes(4, "little")).digest()).digest()
            if int.from_bytes(d, "little") <= int.from_bytes(target, "little"):
                want.append((nonce, vi))
    return {"check": "sha256d_v_vs_cpu", "block": block, "hits": len(got), "expected": len(sorted(want)), "ok": got == sorted(want)}


def main() -> int:
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=29, help="log2 nonces (W3 values) per variant per launch")
    ap.add_argument("--groups", default="1,2")
    ap.add_argument("--bpc", default="7,14,21,24,28")
    ap.add_argument("--bpc8", default="8,16,24,32")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--block64-bpc", default="", help="also time 64-thread blocks at these 64-thread blocks per CU")
    ap.add_argument("--chains2-bpc", default="", help="also time the two-variants-per-lane kernel at these blocks per CU")
    ap.add_argument("--chainsn", default="", help="also time 3/4 variants per lane: 'NC:bpc,bpc;NC:bpc'")
    ap.add_argument("--chains2-block64-bpc", default="", help="two chains with one-wave blocks, these blocks per CU")
    a = ap.parse_args()
    count = 1 << a.count
    if not a.no_check:
        r = check("cuda:0")
        print(json.dumps(r), flush=True)
        if not r["ok"]:
            return 1

    from otedama_amd.ops.search import Sha256dSearchK, Sha256dSearchV

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

    sk = Sha256dSearchK("cuda:0", k=8)
    pk = sk.prepare(headers_for(8), target)
    kcount = 1 << 32
    print(json.dumps({"kernel": "k8", "grid": sk.grid, "ghs": round(run(lambda: sk.launch(pk, 0, kcount), 8 * kcount) / 1e9, 3)}),
          flush=True)
    for occ8 in (False, True):
        for g in map(int, a.groups.split(",")):
            for bpc in [int(x) for x in (a.bpc8 if occ8 else a.bpc).split(",") if x]:
                s = Sha256dSearchV("cuda:0", grid=cus * bpc, occupancy8=occ8)
                p = s.prepare(headers_for(64 * g), target)
                rate = run(lambda: s.launch(p, 0, count), 64 * g * count)
                print(json.dumps({"kernel": "v8" if occ8 else "v", "groups": g, "grid": s.grid,
                                  "ghs": round(rate / 1e9, 3)}), flush=True)
    if a.block64_bpc and not a.no_check:
        r = check("cuda:0", block=64)
        print(json.dumps(r), flush=True)
        if not r["ok"]:
            return 1
    for bpc in [int(x) for x in a.block64_bpc.split(",") if x]:
        s = Sha256dSearchV("cuda:0", grid=cus * bpc, block=64)
        p = s.prepare(headers_for(64), target)
        rate = run(lambda: s.launch(p, 0, count), 64 * count)
        print(json.dumps({"kernel": "v8", "block": 64, "grid": s.grid, "ghs": round(rate / 1e9, 3)}), flush=True)
    if a.chains2_bpc and not a.no_check:
        ref = sorted(Sha256dSearchV("cuda:0").search(headers_for(128), (((1 << 248) - 1)).to_bytes(32, "little"),
                                                     0x12345600, 1024))
        for occ in (False, True):
            got = sorted(Sha256dSearchV("cuda:0", chains=2, occupancy8=occ).search(
                headers_for(128), (((1 << 248) - 1)).to_bytes(32, "little"), 0x12345600, 1024))
            r = {"check": "sha256d_v2_vs_v", "occ5": occ, "hits": len(got), "expected": len(ref), "ok": got == ref}
            print(json.dumps(r), flush=True)
            if not r["ok"]:
                return 1
    for occ in (False, True):
        for bpc in [int(x) for x in a.chains2_bpc.split(",") if x]:
            s = Sha256dSearchV("cuda:0", grid=cus * bpc, chains=2, occupancy8=occ)
            p = s.prepare(headers_for(128), target)
            rate = run(lambda: s.launch(p, 0, count // 2), 128 * (count // 2))
            print(json.dumps({"kernel": "v2_5w" if occ else "v2_4w", "grid": s.grid, "ghs": round(rate / 1e9, 3)}),
                  flush=True)
    for bpc in [int(x) for x in a.chains2_block64_bpc.split(",") if x]:
        s = Sha256dSearchV("cuda:0", grid=cus * bpc, chains=2, occupancy8=False, block=64)
        p = s.prepare(headers_for(128), target)
        rate = run(lambda: s.launch(p, 0, count // 2), 128 * (count // 2))
        print(json.dumps({"kernel": "v2_4w", "block": 64, "grid": s.grid, "ghs": round(rate / 1e9, 3)}), flush=True)
    for spec in [x for x in a.chainsn.split(";") if x]:
        nc, bpcs = spec.split(":")
        nc = int(nc)
        hs = headers_for(64 * nc)
        if not a.no_check:
            t248 = ((1 << 248) - 1).to_bytes(32, "little")
            ref = sorted(Sha256dSearchV("cuda:0", cap=4096, grid=768).search(hs, t248, 0x12345600, 1024))  # 3072 waves
            got = sorted(Sha256dSearchV("cuda:0", cap=4096, chains=nc).search(hs, t248, 0x12345600, 1024))
            r = {"check": f"sha256d_v{nc}_vs_v", "hits": len(got), "expected": len(ref), "ok": got == ref}
            print(json.dumps(r), flush=True)
            if not r["ok"]:
                return 1
        for bpc in [int(x) for x in bpcs.split(",") if x]:
            s = Sha256dSearchV("cuda:0", grid=cus * bpc, chains=nc, occupancy8=False)
            p = s.prepare(hs, target)
            n = (1 << 35) // (64 * nc)
            rate = run(lambda: s.launch(p, 0, n), 64 * nc * n)
            print(json.dumps({"kernel": f"v{nc}", "grid": s.grid, "ghs": round(rate / 1e9, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
