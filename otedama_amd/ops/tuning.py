"""Launch geometry of the search kernels, shared by the torch ops (ops/search.py) and the torch-free native-miner
call sites (engine/miners.py, engine/devproc.py, engine/latency_probe.py), so the engine never imports torch to
size a grid. Values are blocks of 256 lanes per CU; every number cites the sweep that picked it.
"""
from __future__ import annotations

# Single-midstate kernel (51 VGPRs, 7 waves/SIMD resident): an oversubscribed grid-stride grid wins over a resident
# one, a little more with every doubling (peek poll, one process per sweep): 6/7/8/14/28/64 per CU ->
# 16.18/16.23/16.24/16.35/16.43/16.50 GH/s (profiles/r3/ad_single/peek_prod), 32/64/128/256 per CU ->
# 16.42/16.48/16.52/16.55 (profiles/r3/af_single). A 2^32-nonce launch still gives every lane 256 trips.
SHA256D_BLOCKS_PER_CU = 256
SHA256D_K_BLOCKS_PER_CU = 16  # K-variant kernel: K=8 121 VGPRs (4 waves/SIMD); 4/8/12/16 per CU: 18.05/18.48/18.72/18.80 GH/s
# Version-parallel kernel, 8-waves/SIMD build: 64 blocks of 256 per CU (tools/bench_sha_v.py sweep, profiles/r2/sha_v:
# 8/16/32/64/96/128 per CU -> 18.37/18.73/19.00/19.61/19.58/19.61 GH/s; more resident-block rounds keep the waves'
# scalar/vector phases apart).
SHA256D_V_BLOCKS_PER_CU = 64
# Two-chain version-parallel kernel (two variants per lane), 4-waves/SIMD build: 128 blocks per CU (profiles/r2/sha_v2:
# 16/32/64/128/256 per CU -> 19.12/19.29/19.32/19.36-19.40/19.37-19.42 GH/s, against 19.21-19.30 for the one-chain
# kernel in the same runs).
SHA256D_V2_BLOCKS_PER_CU = 128
SCRYPT_BLOCKS_PER_CU = 16  # 128 GiB pad at gap 1 (grid sweep: 2048 16.4, 4096 16.75, 5120 16.95 MH/s)


def sha256d_grid(cus: int) -> int:
    """Grid of the single-midstate kernel (the native miner's ``grid`` argument) for a GPU with ``cus`` CUs."""
    return max(1, int(cus)) * SHA256D_BLOCKS_PER_CU
