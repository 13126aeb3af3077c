#!/usr/bin/env python3
"""Headline benchmark: whole-node SHA-256d hashes/sec (+ scrypt) on N MI355X.

BASELINE.json metric: "hashes/sec (whole node) SHA-256d + scrypt at 1/2/4/8
MI355X; p50 share latency". Reference headline: ~75 MH/s SHA-256d on a whole
Ryzen 9 7950X (BENCHMARKS.md:46, CPU only).

One rank per GPU (torchrun). One timed step =
  R1  broadcast of the job blob from rank 0 (torch.distributed / RCCL),
  K1  SHA-256d search over this rank's next 128 BIP320 header variants (two per
      lane of the version-parallel kernel, fixed midstate per variant, variants
      striped across ranks) x 2^28 nonces; 16 consecutive steps tile the full
      2^32 nonce space of each variant (--sha-chains 1: 64 variants x 2^29;
      --sha-kernel k: K variants x 2^32),
  R2  all_gather of every rank's on-device hit buffer,
  R3  all_reduce of the hash counters.
Data: synthetic 80-byte block headers (random prev-hash / merkle root), share
target = difficulty 1. Every hit found in the timed region is re-verified on
the CPU after timing. Weak scaling: per-GPU work is fixed as N grows.

Then scrypt(1024,1,1) is timed the same way (HBM-resident scratchpads), then
X11 (eleven chained 512-bit hashes, nonce ranges partitioned across ranks), and
p50 share latency is measured end-to-end (GPU hit -> SV2 SubmitSharesStandard
-> pool validation -> SubmitSharesSuccess) against the in-process local pool.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import torch

BASELINE_HPS = 75e6  # BENCHMARKS.md:46 (whole 7950X, SHA-256d)
METRIC = "hashes/sec (whole node) SHA-256d + scrypt at 1/2/4/8 MI355X; p50 share latency"


def synthetic_job(seed: int = 1) -> dict:
    from otedama_amd.models.header import DIFF1_TARGET_INT, int_to_hash

    h = hashlib.sha256(f"otedama-bench-{seed}".encode()).digest()
    prev = hashlib.sha256(h).digest()
    header = (0x20000000).to_bytes(4, "little") + prev + h + (1_700_000_000).to_bytes(4, "little") \
        + (0x1703A30C).to_bytes(4, "little") + bytes(4)
    return {
        "header": header,
        "target": int_to_hash(DIFF1_TARGET_INT),
        "epoch": 1,
        "job_id": "bench",
        "version_mask": 0x1FFFE000,  # BIP320 version rolling: 2^16 variants
        "ntime_roll": 0,
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--grid", type=int, default=0, help="SHA-256d blocks (0 = CUs x resident blocks)")
    ap.add_argument("--sha-kernel", choices=("v", "k"), default="v",
                    help="v: 64 x --sha-chains version variants per wave, block-2 schedule on the scalar unit (default); "
                         "k: --sha-variants variants per lane")
    ap.add_argument("--sha-chains", type=int, choices=(1, 2), default=2,
                    help="v kernel: variants per lane (2: 128 variants per wave-group, 4 waves/SIMD; 1: 64, 8 waves)")
    ap.add_argument("--sha-variants", type=int, default=8,
                    help="k kernel: BIP320 version variants per launch sharing the block-2 schedule (1 = single midstate)")
    ap.add_argument("--scrypt-steps", type=int, default=-1, help="-1 = same as --steps; 0 = skip")
    ap.add_argument("--scrypt-gap", type=int, default=1)
    ap.add_argument("--scrypt-kernel", choices=("coop", "lane"), default="coop")
    ap.add_argument("--x11-steps", type=int, default=-1, help="-1 = same as --steps; 0 = skip")
    ap.add_argument("--no-latency", action="store_true")
    args = ap.parse_args()

    from otedama_amd.ops import native
    from otedama_amd.ops.search import ScryptSearch, Sha256dSearch, Sha256dSearchK, Sha256dSearchV
    from otedama_amd.parallel import NodeComm, barrier, init_from_env, shutdown, stripe_for
    from otedama_amd.utils.trace import span

    if not torch.cuda.is_available():
        print("bench.py requires a GPU (HIP); run `python -m otedama_amd.cli bench-cpu` for the CPU config",
              file=sys.stderr)
        return 2
    N = native.require_native()
    info = init_from_env()
    comm = NodeComm(info)
    dev = info.device

    job = comm.broadcast_job(synthetic_job() if info.is_primary else None)  # R1
    stripe = stripe_for(info.rank, info.world_size)
    world = info.world_size
    use_v = args.sha_kernel == "v"
    if use_v:
        # One step = 64 x chains version variants (chains per lane of a wave) x 2^35 / that many nonces = 2^35
        # hashes, the same work as the K=8 step (8 x 2^32); 8 x chains consecutive steps tile the full 2^32 nonces
        # of one variant group. Two chains run the 4-waves/SIMD build at 128 blocks/CU (profiles/r2/sha_v2).
        K = N.SHA256D_V_GROUP * args.sha_chains
        V_COUNT = (1 << 35) // K
        steps_per_group = (1 << 32) // V_COUNT
        if args.sha_chains == 2:
            from otedama_amd.ops.search import SHA256D_V2_BLOCKS_PER_CU, default_grid

            search = Sha256dSearchV(dev, grid=args.grid or default_grid(dev, SHA256D_V2_BLOCKS_PER_CU), chains=2,
                                    occupancy8=False)
        else:
            search = Sha256dSearchV(dev, grid=args.grid or None)
    else:
        V_COUNT, steps_per_group = 1 << 32, 1
        K = max(k for k in (1, *N.SHA256D_K_VALUES) if k <= max(1, args.sha_variants))
        search = Sha256dSearchK(dev, k=K, grid=args.grid or None) if K > 1 else Sha256dSearch(dev, grid=args.grid or None)
    slot_words = 1 + (2 if K > 1 else 1) * search.cap
    gathered = torch.zeros(world, slot_words, dtype=torch.int32, device=dev)
    counters_hashes = 0

    def variant_params(step: int) -> tuple[list[bytes], bytes]:
        # step i of this rank: stripe positions K*i .. K*i + K-1 (version-rolled headers, identical block 2)
        hdrs = [N.variant_header(job, stripe.start + (step * K + j) * stripe.stride)[0] for j in range(K)]
        if K > 1:
            return hdrs, N.sha256d_prepare_k(hdrs, job["target"])
        return hdrs, N.sha256d_prepare(hdrs[0], job["target"])

    v_groups: dict[int, tuple[list[bytes], object]] = {}

    def v_group(q: int):
        # variant group q of this rank: stripe positions Kq .. Kq+K-1; the table is uploaded once, before timing
        if q not in v_groups:
            hdrs = [N.variant_header(job, stripe.start + (q * K + j) * stripe.stride)[0] for j in range(K)]
            v_groups[q] = (hdrs, search.prepare(hdrs, job["target"]))
        return v_groups[q]

    hits_log: list[tuple[list[bytes], torch.Tensor]] = []

    def step(i: int, record: bool) -> None:
        with span("otd.bench.sha256d_step"):
            _step(i, record)

    def _step(i: int, record: bool) -> None:
        nonlocal counters_hashes
        if world > 1:  # R1: job blob fan-out (kept on device; decoded only on job change)
            comm._run(lambda: torch.distributed.broadcast(comm._job, src=0))
        if use_v:  # K1: 64 variants x one eighth of the nonce space (W3 window)
            hdr, prep = v_group(i // steps_per_group)
            r = search.launch(prep, (i % steps_per_group) * V_COUNT, V_COUNT)
        else:
            hdr, params = variant_params(i)
            r = search.launch(params, 0, 1 << 32)  # K1: full 2^32 nonce space
        if world > 1:  # R2: on-device hit buffers, gathered on the comm stream
            comm._run(lambda: torch.distributed.all_gather_into_tensor(gathered.view(-1), r.buf.view(-1)))
        else:
            gathered[0].copy_(r.buf)
        counters_hashes += K * (V_COUNT if use_v else 1 << 32)
        if record:
            hits_log.append((hdr, gathered[info.rank].clone()))

    # Warmup steps take the stripe positions right after the timed ones (steps .. steps+W-1), so every position
    # used stays inside the 2^16 BIP320 variant space: (steps + W) * K * world <= 65536.
    positions = ((args.steps + args.warmup + steps_per_group - 1) // steps_per_group + 1) * K if use_v \
        else (args.steps + args.warmup) * K
    if positions * world > 1 << 16:
        raise SystemExit("bench.py: (steps + warmup) x variants x GPUs exceeds the 2^16 version-rolling space")
    if use_v:  # variant tables for every step, timed and warmup, built and uploaded before the timed region
        for i in range(args.steps + args.warmup):
            v_group(i // steps_per_group)
    for i in range(args.warmup):
        step(args.steps + i, False)
    torch.cuda.synchronize(dev)
    barrier(info)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    step_hashes = K * (V_COUNT if use_v else 1 << 32)
    total = comm.allreduce_counters(args.steps * step_hashes)[0] if world > 1 else args.steps * step_hashes  # R3
    torch.cuda.synchronize(dev)
    barrier(info)
    torch.cuda.synchronize(dev)
    elapsed = comm.allreduce_max(time.perf_counter() - t0)
    sha_hps = total / elapsed

    # Re-verify every hit of the timed region on the CPU (full 256-bit compare).
    found = verified = 0
    for hdrs, buf in hits_log:
        host = buf.cpu().tolist()
        n = min(host[0] & 0xFFFFFFFF, search.cap)
        pairs = [(host[1 + 2 * i], host[2 + 2 * i]) for i in range(n)] if K > 1 else [(x, 0) for x in host[1 : 1 + n]]
        for nonce, vi in pairs:
            nonce &= 0xFFFFFFFF
            found += 1
            if not 0 <= vi < K:
                continue
            hdr = hdrs[vi]
            h = hashlib.sha256(hashlib.sha256(hdr[:76] + nonce.to_bytes(4, "little")).digest()).digest()
            if int.from_bytes(h, "little") <= int.from_bytes(job["target"], "little"):
                verified += 1
    found, verified, _, _ = comm.allreduce_counters(found, verified)

    # ---------------------------------------------------------------- scrypt
    scrypt_hps = None
    ssteps = args.steps if args.scrypt_steps < 0 else args.scrypt_steps
    scrypt_info = {}
    if ssteps > 0:
        from otedama_amd.models.algorithms import ALGORITHMS
        from otedama_amd.models.header import int_to_hash

        sc = ScryptSearch(dev, gap=args.scrypt_gap, kernel=args.scrypt_kernel)
        starget = int_to_hash(ALGORITHMS["scrypt"].diff1)
        hdr, _, _, _ = N.variant_header(job, stripe.start)
        sparams = N.scrypt_prepare(hdr, starget)
        sc.launch(sparams, 0)
        torch.cuda.synchronize(dev)
        barrier(info)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(ssteps):
            sc.launch(sparams, (i * sc.batch) & 0xFFFFFFFF)
        torch.cuda.synchronize(dev)
        barrier(info)
        torch.cuda.synchronize(dev)
        selapsed = comm.allreduce_max(time.perf_counter() - t0)
        stotal = comm.allreduce_counters(ssteps * sc.batch)[0] if world > 1 else ssteps * sc.batch
        scrypt_hps = stotal / selapsed
        scrypt_info = {"kernel": sc.kernel, "lookup_gap": 1 if sc.kernel == "coop" else sc.gap, "lanes": sc.batch, "scratch_gib_per_gpu": round(sc.scratch_bytes / 2**30, 2)}
        del sc
        torch.cuda.empty_cache()

    # ------------------------------------------------------------------ X11
    # BASELINE config 4: X11 with the nonce range partitioned across ranks (rank r takes batches
    # r, r + N, r + 2N, ...). Target 2^-20 so every step yields hits that are re-verified on the CPU.
    x11_hps = None
    x11_info = {}
    xsteps = args.steps if args.x11_steps < 0 else args.x11_steps
    if xsteps > 0:
        from otedama_amd.models.header import int_to_hash
        from otedama_amd.ops.search import X11Search

        xs = X11Search(dev, cap=4096)
        xtarget_int = (1 << 236) - 1
        hdr, _, _, _ = N.variant_header(job, stripe.start)
        xparams = N.x11_prepare(hdr, int_to_hash(xtarget_int))
        xs.launch(xparams, 0)
        torch.cuda.synchronize(dev)
        barrier(info)
        torch.cuda.synchronize(dev)
        xhits: list[list[int]] = []
        t0 = time.perf_counter()
        for i in range(xsteps):
            base = ((i * world + info.rank) * xs.batch) & 0xFFFFFFFF
            r = xs.launch(xparams, base)
            xhits.append(r.buf.clone())
        torch.cuda.synchronize(dev)
        barrier(info)
        torch.cuda.synchronize(dev)
        xelapsed = comm.allreduce_max(time.perf_counter() - t0)
        xtotal = comm.allreduce_counters(xsteps * xs.batch)[0] if world > 1 else xsteps * xs.batch
        x11_hps = xtotal / xelapsed
        xfound = xver = 0
        for buf in xhits:
            host = buf.cpu().tolist()
            for nonce in host[1 : 1 + min(host[0] & 0xFFFFFFFF, xs.cap)]:
                xfound += 1
                h = N.x11(hdr[:76] + (nonce & 0xFFFFFFFF).to_bytes(4, "little"))
                xver += int.from_bytes(h, "little") <= xtarget_int
        xfound, xver, _, _ = comm.allreduce_counters(xfound, xver)
        x11_info = {"batch_per_launch": xs.batch, "kernels": "11 stage kernels per batch (tools/bench_x11.py)",
                    "hits_found": xfound, "hits_verified": xver, "hit_target": "2^-20"}
        del xs
        torch.cuda.empty_cache()

    # ---------------------------------------------------------- share latency
    latency = None
    if not args.no_latency and info.is_primary:
        try:
            from otedama_amd.engine.latency_probe import measure_share_latency

            latency = measure_share_latency(device_index=dev.index or 0, seconds=6.0)
        except Exception as exc:  # noqa: BLE001 - latency is auxiliary; never fail the headline
            latency = {"error": f"{type(exc).__name__}: {exc}"}

    if info.is_primary:
        out = {
            "metric": METRIC,
            "value": sha_hps,
            "unit": "hashes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": sha_hps / BASELINE_HPS,
            "dtype": "u32",
            "data": "synthetic 80-byte block headers (random prev-hash/merkle root), share target = difficulty 1",
            "config": {
                "model": "sha256d",
                "global_batch": step_hashes * world,
                "seq_len": 80,
                "parallelism": (f"dp{world} (nonce-space: per-rank variant stripe; "
                                + (f"{K} variants x 2^{(V_COUNT).bit_length() - 1} nonces per step, {steps_per_group} "
                                   "steps tile 2^32 per variant)" if use_v
                                   else "full 2^32 nonces per variant per step)")),
                "algorithm": ("SHA-256d nonce search, fixed midstate per variant; " + (
                    f"{K} BIP320 version variants per wave ({K // 64} per lane) share the block-2 message schedule, "
                    "computed on the scalar unit" if use_v else
                    f"{K} BIP320 version variants per launch share the block-2 message schedule")),
                "sha_kernel": (("otd_sha256d_search_v2<0>" if K == 128 else "otd_sha256d_search_v<8>") if use_v
                               else (f"otd_sha256d_search_k<{K}>" if K > 1 else "otd_sha256d_search")),
                "variants_per_step": K,
                "grid": search.grid,
            },
            "sha256d_hashes_per_sec": sha_hps,
            "sha256d_per_gpu_hashes_per_sec": sha_hps / world,
            "hits_found": found,
            "hits_verified": verified,
            "scrypt_hashes_per_sec": scrypt_hps,
            "scrypt": scrypt_info,
            "x11_hashes_per_sec": x11_hps,
            "x11": x11_info,
            "p50_share_latency_ms": (latency or {}).get("p50_ms") if isinstance(latency, dict) else None,
            "share_latency": latency,
        }
        print(json.dumps(out))
    shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
