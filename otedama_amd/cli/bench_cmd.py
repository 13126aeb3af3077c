"""``otedama bench`` / ``otedama devices``.

bench reproduces the reference's benchmark configurations on this machine
(BENCHMARKS.md:25-54 — single-thread and all-core SHA-256d) and adds the
gfx950 kernels (SHA-256d full 2^32 nonce space, scrypt N=1024). The headline
multi-GPU number is ``bench.py`` at the repo root (torchrun, RCCL).
"""
from __future__ import annotations

import json
import os
import struct
import time
from typing import TextIO

from otedama_amd.cli.flags import FlagSet
from otedama_amd.cli.main import EXIT_OK, EXIT_RUNTIME, parse_subcommand


def cpu_share() -> int:
    """CPUs this process may use: its affinity mask, capped by OMP_NUM_THREADS when set (a GPU box exposes the
    whole machine in os.cpu_count() but gives a job a share of it)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else max(1, n)


def bench_cpu(seconds: float = 2.0, threads: int = 0, single_seconds: float = 0.0) -> dict:
    """BASELINE config 1 on this host: the CPU SHA-256d scan (16-lane AVX-512 where the CPU has it, else SHA-NI) on
    one thread over a synthetic 80-byte header, then the production CpuMiner on ``threads`` threads
    (BENCHMARKS.md:25-28 single thread, :44-49 whole CPU)."""
    from otedama_amd.models.header import GENESIS_HEADER_HEX
    from otedama_amd.ops.native import require_native

    N = require_native()
    hdr = bytes.fromhex(GENESIS_HEADER_HEX)
    # single thread: 2^20-nonce scans until single_seconds (at least one), timed
    n, done = 1 << 21, 0
    t0 = time.perf_counter()
    while True:
        N.cpu_scan_sha256d(hdr, bytes(32), done & 0xFFFFFFFF, n)
        done += n
        if time.perf_counter() - t0 >= single_seconds:
            break
    single_s = time.perf_counter() - t0
    single = done / single_s
    threads = threads or (os.cpu_count() or 1)
    m = N.CpuMiner(threads, "cpu-0")
    m.set_job({"header": hdr, "target": bytes(32), "version_mask": 0x1FFFE000})
    m.start()
    time.sleep(0.3)
    h0, t0 = m.stats()["hashes"], time.perf_counter()
    time.sleep(seconds)
    h1, t1 = m.stats()["hashes"], time.perf_counter()
    m.stop()
    allc = (h1 - h0) / (t1 - t0)
    return {"sha256d_single_thread_hps": single, "sha256d_all_threads_hps": allc, "threads": threads,
            "scaling": allc / (single * threads), "sha_ni": bool(N.cpu_has_sha_ni()),
            "scan": N.cpu_scan_method(),
            "single_thread_seconds": round(single_s, 3), "single_thread_nonces": done,
            "all_threads_seconds": seconds, "header": "synthetic 80-byte header (Bitcoin genesis)",
            "reference": "~2.5 MH/s / ~75 MH/s on a Ryzen 9 7950X (BENCHMARKS.md:25,46)"}


def bench_gpu(device: int = 0, reps: int = 3, scrypt_batches: int = 4) -> dict:
    import torch

    from otedama_amd.ops.native import require_native
    from otedama_amd.ops.search import ScryptSearch, Sha256dSearch, Sha256dSearchV

    N = require_native()
    hdr = os.urandom(76) + bytes(4)
    s = Sha256dSearch(f"cuda:{device}")
    p = N.sha256d_prepare(hdr, bytes(32))
    s.launch(p, 0, 1 << 28)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        s.launch(p, 0, 1 << 32)
    torch.cuda.synchronize()
    sha = reps * (1 << 32) / (time.perf_counter() - t0)
    # version rolling (BIP320): 128 variants per wave-group, two per lane, block-2 schedule on the scalar unit
    from otedama_amd.ops.search import SHA256D_V2_BLOCKS_PER_CU, default_grid

    sv = Sha256dSearchV(f"cuda:{device}", grid=default_grid(f"cuda:{device}", SHA256D_V2_BLOCKS_PER_CU), chains=2,
                        occupancy8=False)
    pv = sv.prepare([struct.pack("<I", 0x20000000 | (v << 13)) + hdr[4:] for v in range(128)], bytes(32))
    sv.launch(pv, 0, 1 << 22)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        sv.launch(pv, i << 28, 1 << 28)
    torch.cuda.synchronize()
    sha_v = reps * 128 * (1 << 28) / (time.perf_counter() - t0)
    sc = ScryptSearch(f"cuda:{device}")
    sp = N.scrypt_prepare(hdr, bytes(32))
    sc.launch(sp, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(scrypt_batches):
        sc.launch(sp, i * sc.batch)
    torch.cuda.synchronize()
    scr = scrypt_batches * sc.batch / (time.perf_counter() - t0)
    return {"device": device, "arch": N.gpu_arch_name(device), "sha256d_hps": sha,
            "sha256d_version_rolling_hps": sha_v, "scrypt_hps": scr,
            "scrypt_scratch_gib": sc.scratch_bytes / 2 ** 30}


def cmd_bench(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    fs = FlagSet("bench", stderr)
    fs.string("device", "auto", "cpu | gpu | auto (gpu when present, plus cpu).")
    fs.float("seconds", 2.0, "CPU all-thread measurement window.")
    fs.int("threads", 0, "CPU threads (0 = all).")
    fs.int("gpu", 0, "HIP device ordinal.")
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    out = {}
    try:
        if fs["device"] in ("cpu", "auto"):
            out["cpu"] = bench_cpu(fs["seconds"], fs["threads"])
        if fs["device"] in ("gpu", "auto"):
            from otedama_amd.ops.native import gpu_count

            if gpu_count() > 0:
                out["gpu"] = bench_gpu(fs["gpu"])
            elif fs["device"] == "gpu":
                stderr.write("bench: no HIP device visible\n")
                return EXIT_RUNTIME
    except Exception as exc:  # noqa: BLE001
        stderr.write(f"bench: {exc}\n")
        return EXIT_RUNTIME
    stdout.write(json.dumps(out, indent=2) + "\n")
    return EXIT_OK


def cmd_devices(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    from otedama_amd import hal

    fs = FlagSet("devices", stderr)
    fs.bool("json", False, "Emit JSON.")
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    devs = hal.Detector(hal.default_registry()).detect()
    if fs["json"]:
        stdout.write(json.dumps([{"id": d.identity().id, "family": d.identity().family.value,
                                  "vendor": d.identity().vendor, "model": d.identity().model,
                                  "capabilities": d.capabilities().__dict__} for d in devs], indent=2) + "\n")
    else:
        for d in devs:
            caps = ",".join(k for k, v in d.capabilities().__dict__.items() if v) or "none"
            stdout.write(f"{d.identity()}  vendor={d.identity().vendor or '-'}  caps={caps}\n")
    return EXIT_OK
