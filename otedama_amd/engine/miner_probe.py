"""The production GPU miner's rate for one algorithm, measured the way it runs under the engine (bench.py).

``otedama run`` hashes through the native GpuMiner of a device process: two batches in flight on two streams (scrypt:
two half-grid batches, half a hash apart, each on its own half of the 128 GiB pad; X11: a digest plane per slot),
hits published from the running launch, every candidate re-verified on the host. The ops-API kernel sections of
bench.py time the kernels one launch after another instead, so the production layout is measured here, on the rank's
GPU, either in a device process exactly as the engine runs it (``process=True``, what bench.py uses: a torch-free
child, its own HIP context) or in this process:

  * the rate is exact over whole launches: hashes counted between two samples over the device-timeline span in
    which those launches completed (``hashes_done_at_s``), after a warm-up;
  * every share the miner queued was re-verified by the miner against the full 256-bit target; on top of that the
    shares are re-hashed here, independently of the native verifier (X11: all of them through the CPU chain; scrypt:
    up to ``recheck`` through hashlib.scrypt, ~1 ms each), and the candidate accounting (shares + rejected + lost)
    is reported.

Each rank of a node takes its own residue class of the variant space (``variant_start = rank``,
``variant_stride = world``), so ranks never hash the same header.
"""
from __future__ import annotations

import hashlib
import time

from otedama_amd.models.header import int_to_hash


def _header(base: bytes, share: dict) -> bytes:
    """The 80-byte header a share of a header-only job was found on (version rolled, nonce set)."""
    return (share["version"] & 0xFFFFFFFF).to_bytes(4, "little") + base[4:68] + \
        (share["ntime"] & 0xFFFFFFFF).to_bytes(4, "little") + base[72:76] + \
        (share["nonce"] & 0xFFFFFFFF).to_bytes(4, "little")


def measure_miner(N, device_index: int, algo: str, target_int: int, seconds: float = 8.0, warmup: float = 3.0,
                  rank: int = 0, world: int = 1, recheck: int = 64, seed: int = 1, process: bool = False) -> dict:
    """Run the GPU miner on ``algo`` for ``warmup + seconds`` and return its exact rate and share checks.
    ``process``: in a device process (engine/devproc.py), as ``otedama run`` does; else the native GpuMiner here."""
    base = hashlib.sha256(f"otedama-miner-probe-{algo}-{seed}".encode()).digest()
    hdr = (0x20000000).to_bytes(4, "little") + base + hashlib.sha256(base).digest() + \
        (1_700_000_000).to_bytes(4, "little") + (0x1D00FFFF).to_bytes(4, "little") + bytes(4)
    cus = N.gpu_cu_count(device_index)
    if process:
        from otedama_amd.engine.devproc import DeviceProcess

        m = DeviceProcess(device_index, f"gpu-{device_index}", batch_nonces=1 << 32, grid=cus * 6, queue_cap=65536,
                          sha_variants=128)
    else:
        m = N.GpuMiner(device_index, f"gpu-{device_index}", batch_nonces=1 << 32, grid=cus * 6, queue_cap=65536,
                       sha_variants=128)
    m.set_job({"header": hdr, "target": int_to_hash(target_int), "job_id": f"probe-{algo}", "epoch": 1, "algo": algo,
               "version_mask": 0x1FFFE000, "variant_start": rank, "variant_stride": world})
    shares: list[dict] = []
    m.start()

    def edge(after: dict, limit: float) -> dict:
        """The first stats whose completed-hash counter moved past ``after``'s: its device-timeline time is then
        that of a launch that has just completed, not a stale one (a window must start and end on such edges)."""
        nonlocal shares
        end = time.monotonic() + limit
        st = m.stats()
        while st["hashes"] == after["hashes"] and time.monotonic() < end:
            shares += m.poll(65536)
            time.sleep(0.002)
            st = m.stats()
        return st

    def launches() -> int:
        return int(m.stats().get("launches", 0))

    try:
        # warm-up: the time given, and at least 4 launches (the first scrypt job allocates a 128 GiB pad, which takes
        # seconds right after another process or allocator released one)
        end, cap = time.monotonic() + warmup, time.monotonic() + warmup + 60.0
        while time.monotonic() < end or (launches() < 4 and time.monotonic() < cap):
            shares += m.poll(65536)
            time.sleep(0.05)
        s0 = edge(m.stats(), 10.0)
        w0 = time.monotonic()
        end = w0 + seconds
        while time.monotonic() < end:
            shares += m.poll(65536)
            time.sleep(0.1)
        s1 = edge(m.stats(), 10.0)  # the first completion past the window
        w1 = time.monotonic()
    finally:
        m.stop()
    shares += m.poll(65536)
    st = s1 if process else m.stats()  # a stopped device process reports no more stats frames
    span = s1["hashes_done_at_s"] - s0["hashes_done_at_s"]
    hps = (s1["hashes"] - s0["hashes"]) / span if span > 0 else 0.0
    # independent re-hash of the shares the miner queued
    checked = ok = 0
    for s in shares:
        if algo == "scrypt" and checked >= recheck:
            break
        h80 = _header(hdr, s)
        if algo == "scrypt":
            d = hashlib.scrypt(h80, salt=h80, n=1024, r=1, p=1, dklen=32)
        elif algo == "x11":
            d = N.x11(h80)
        else:
            d = hashlib.sha256(hashlib.sha256(h80).digest()).digest()
        checked += 1
        ok += int.from_bytes(d, "little") <= target_int
    return {
        "hashes_per_sec": hps,
        "window_hashes": s1["hashes"] - s0["hashes"], "window_device_seconds": span, "window_wall_seconds": w1 - w0,
        "launches": st.get("launches", 0), "aborted_launches": st.get("aborted_launches", 0),
        "candidates": st.get("candidates", 0), "shares": max(int(st.get("shares", 0)), len(shares)),
        "rejected_candidates": st.get("rejected_candidates", 0), "dropped": st.get("dropped", 0),
        "ring_overflow": st.get("ring_overflow", 0), "verify_dropped": st.get("verify_dropped", 0),
        "shares_rechecked": checked, "shares_recheck_ok": ok, "faulted": bool(st.get("faulted")),
        "host_abort": st.get("host_abort"), "path": "device process" if process else "in-process GpuMiner",
        "definition": ("the production GPU miner (two batches in flight, hit ring, abort word, host re-verification)"
                       + (" in a device process, as `otedama run` runs it" if process else "")
                       + "; exact rate over the launches completed in the window, device timeline"),
    }
