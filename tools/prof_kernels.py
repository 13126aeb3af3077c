#!/usr/bin/env python3
"""Fixed workload for rocprofv3: SHA-256d full-range launches, scrypt batches, the version-parallel kernel, X11."""
import sys

import torch

from otedama_amd.ops.native import require_native
from otedama_amd.ops.search import ScryptSearch, Sha256dSearch

algo = sys.argv[1] if len(sys.argv) > 1 else "both"
N = require_native()
hdr = bytes(range(76)) + bytes(4)
tgt = bytes(28) + b"\xff\xff\x00\x00"
if algo in ("both", "sha256d"):
    s = Sha256dSearch("cuda:0")
    p = N.sha256d_prepare(hdr, tgt)
    for _ in range(3):
        s.launch(p, 0, 1 << 32)
    torch.cuda.synchronize()
if algo in ("both", "scrypt"):
    gap = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    sc = ScryptSearch("cuda:0", gap=gap)
    sp = N.scrypt_prepare(hdr, tgt)
    for i in range(4):
        sc.launch(sp, i * sc.batch)
    torch.cuda.synchronize()
if algo == "sha_v":  # K=8 vs version-parallel, equal work: 4 x 2^35 hashes each
    from otedama_amd.ops.search import Sha256dSearchK, Sha256dSearchV

    tail = bytes(range(4, 76)) + bytes(4)
    hs = [(0x20000000 | (v << 13)).to_bytes(4, "little") + tail for v in range(64)]
    sk = Sha256dSearchK("cuda:0", k=8)
    pk = sk.prepare(hs[:8], tgt)
    for _ in range(4):
        sk.launch(pk, 0, 1 << 32)
    sv = Sha256dSearchV("cuda:0")
    pv = sv.prepare(hs, tgt)
    for i in range(4):
        sv.launch(pv, i << 29, 1 << 29)
    torch.cuda.synchronize()
if algo == "sha_v2":  # one chain (64 variants) vs two chains per lane (128 variants), equal work: 4 x 2^35 hashes
    from otedama_amd.ops.search import SHA256D_V2_BLOCKS_PER_CU, Sha256dSearchV, default_grid

    tail = bytes(range(4, 76)) + bytes(4)
    hs = [(0x20000000 | (v << 13)).to_bytes(4, "little") + tail for v in range(128)]
    sv = Sha256dSearchV("cuda:0")
    pv = sv.prepare(hs[:64], tgt)
    for i in range(4):
        sv.launch(pv, i << 29, 1 << 29)
    s2 = Sha256dSearchV("cuda:0", grid=default_grid("cuda:0", SHA256D_V2_BLOCKS_PER_CU), chains=2, occupancy8=False)
    p2 = s2.prepare(hs, tgt)
    for i in range(4):
        s2.launch(p2, i << 28, 1 << 28)
    torch.cuda.synchronize()
if algo == "x11":  # the 11-stage chain, 4 batches of 2^23 nonces
    from otedama_amd.ops.search import X11Search

    xs = X11Search("cuda:0")
    xp = xs.prepare(hdr, tgt)
    for i in range(4):
        xs.launch(xp, i * xs.batch)
    torch.cuda.synchronize()
print("done")
