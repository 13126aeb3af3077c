"""End-to-end share-latency and job-switch probes (BASELINE metric "p50 share latency").

Share latency: the real engine mines on one GPU (default 2^32-hash launches) against the local validating pool
running in a SEPARATE process (``otedama pool``), over loopback Stratum V2. Reported quantiles:
  * submit -> accept (the reference's definition: otedama_submit_latency_milliseconds,
    internal/engine/run.go:813-821);
  * device hit -> accept: from the kernel's own hit time (s_memrealtime stamped in the hit record, mapped to the
    host clock) through the host-coherent hit ring, CPU re-verification, the share queue's eventfd, the asyncio
    submit, the pool process's re-hash / validation and its SubmitSharesSuccess;
  * host verify -> accept (the part after the miner thread picked the hit up).
The reference never published a number for this.

Job switch: the native GpuMiner is handed new work every few hundred ms; each switch is timed from set_job() to
the first batch of the new work running on the device (obsolete batches stop at the device abort word).
"""
from __future__ import annotations

import asyncio
import os
import signal
import statistics
import subprocess
import sys
import time

from otedama_amd.ops.tuning import sha256d_grid

PROBE_ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spawn_pool(algorithm: str, difficulty: float, timeout: float = 120.0, fixed: bool = True,
               extra: list[str] | None = None) -> tuple[subprocess.Popen, str]:
    """Start ``otedama pool`` in its own process on an ephemeral loopback port; returns (process, sv2 address).
    ``fixed``: every connection is pinned at ``difficulty`` (no vardiff, no nominal-hashrate start)."""
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = [sys.executable, "-m", "otedama_amd", "pool", "--algorithms", algorithm, "--listen-sv2", "127.0.0.1:0",
           "--listen-v1=", "--difficulty", repr(difficulty), "--retarget-seconds", "3600", "--share-seconds", "1",
           "--job-interval", "3600", "--block-interval", "3600", "--payout-address", PROBE_ADDR,
           *(["--fixed-difficulty"] if fixed else []), *(extra or [])]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
    deadline = time.monotonic() + timeout
    seen = []
    while time.monotonic() < deadline:
        line = proc.stdout.readline()
        if not line:
            break
        seen.append(line)
        if "listening sv2=" in line:
            addr = line.split("listening sv2=", 1)[1].split()[0]
            return proc, addr
    proc.kill()
    raise RuntimeError("pool process did not start: " + "".join(seen[-5:]))


def stop_pool(proc: subprocess.Popen) -> dict:
    """SIGTERM the pool; it prints its stats as one JSON line per algorithm on the way out."""
    import json

    proc.send_signal(signal.SIGTERM)
    try:
        out, _ = proc.communicate(timeout=30)
    except subprocess.TimeoutExpired:
        proc.kill()
        out, _ = proc.communicate()
    for line in reversed((out or "").splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                pass
    return {}


async def _probe(device_index: int, seconds: float, algorithm: str, addr: str, batch_nonces: int,
                 warmup: float = 3.0, min_samples: int = 0, max_seconds: float = 30.0) -> dict:
    from otedama_amd import hal
    from otedama_amd.config import Config, MiningConfig, PoolConfig
    from otedama_amd.engine.run import Engine, Options
    from otedama_amd.provider import StaticRateSource

    devs = [d for d in hal.HIPDriver().enumerate() if d.index == device_index]
    if not devs:
        raise RuntimeError(f"no HIP device {device_index}")
    cfg = Config(bitcoin_address=PROBE_ADDR, pools=[PoolConfig(url=f"stratum+v2://{addr}")],
                 mining=MiningConfig(algorithm=algorithm, batch_nonces=batch_nonces))
    eng = Engine(Options(config=cfg, devices=devs, rate_fetcher=StaticRateSource(95000), stats_interval=1.0))
    task = asyncio.ensure_future(eng.run())
    # Warm-up: the first shares of a fresh engine / pool pair take the cold paths (first submit and validation in
    # each process; 1.0 ms device hit -> accept vs 0.5 ms for the next probes on the same box, profiles/r3/au_latency)
    # and are not recorded.
    await asyncio.sleep(warmup)
    from otedama_amd.engine.stats import LatencyTracker

    eng.latency, eng.pipeline_latency, eng.device_latency = LatencyTracker(4096), LatencyTracker(4096), \
        LatencyTracker(4096)
    t0 = time.monotonic()
    trace, end, cap = [], t0 + seconds, t0 + max(seconds, max_seconds)
    # the engine's hashrate at each stats tick of the recorded window; the window runs at least `seconds` and until
    # `min_samples` shares were accepted (bounded by max_seconds)
    while time.monotonic() < end or (eng.device_latency.count() < min_samples and time.monotonic() < cap):
        await asyncio.sleep(0.5)
        trace.append(round(eng.current_hashrate / 1e9, 3))
    eng.hashrate_trace_ghs = trace
    eng.recorded_seconds = time.monotonic() - t0
    eng.enforced_difficulty = eng.enforced_share_difficulty()
    task.cancel()
    try:
        await task
    except (asyncio.CancelledError, Exception):  # noqa: BLE001
        pass
    return {"eng": eng}


def measure_share_latency(device_index: int = 0, seconds: float = 6.0, algorithm: str = "sha256d",
                          shares_per_sec: float = 40.0, batch_nonces: int = 1 << 32,
                          expected_hashrate: float = 19e9, min_samples: int = 200) -> dict:
    hashes_per_diff1 = 2.0 ** 16 if algorithm == "scrypt" else 2.0 ** 32  # scrypt pools: diff1 = 0xFFFF << 224
    diff = expected_hashrate / (shares_per_sec * hashes_per_diff1)
    proc, addr = spawn_pool(algorithm, diff, fixed=True)
    try:
        eng = asyncio.run(_probe(device_index, seconds, algorithm, addr, batch_nonces, min_samples=min_samples))["eng"]
    finally:
        pool = stop_pool(proc)
    lat, pipe, dev = eng.latency, eng.pipeline_latency, eng.device_latency
    return {
        "p50_ms": lat.quantile(0.5), "p95_ms": lat.quantile(0.95), "p99_ms": lat.quantile(0.99),
        "samples": lat.count(),
        "device_hit_to_accept_p50_ms": dev.quantile(0.5), "device_hit_to_accept_p95_ms": dev.quantile(0.95),
        "device_hit_to_accept_p99_ms": dev.quantile(0.99), "device_hit_to_accept_samples": dev.count(),
        "hit_to_accept_p50_ms": pipe.quantile(0.5), "hit_to_accept_p95_ms": pipe.quantile(0.95),
        "hit_to_accept_samples": pipe.count(),
        "accepted": eng.m.shares_accepted.value(), "rejected": eng.m.shares_rejected.value(),
        "pool_accepted": pool.get("accepted"), "pool_rejected": pool.get("rejected"),
        # the difficulty the pool enforced (from the share target it sent, SetTarget / OpenMiningChannelSuccess),
        # next to the one the probe asked for; the pool pins it (--fixed-difficulty)
        "share_difficulty": getattr(eng, "enforced_difficulty", None), "requested_difficulty": diff,
        "pool_fixed_difficulty": pool.get("fixed_difficulty"),
        "pool_validate_ms": pool.get("validate_ms"),
        "batch_nonces": batch_nonces, "seconds": round(getattr(eng, "recorded_seconds", seconds), 2),
        "warmup_seconds": 3.0,
        "protocol": "stratum-v2 over loopback TCP; pool in a separate process (otedama pool)",
        # median over the recorded window's stats ticks (a single tick can catch a launch boundary)
        "engine_hashrate": (statistics.median(getattr(eng, "hashrate_trace_ghs", [])) * 1e9
                            if getattr(eng, "hashrate_trace_ghs", []) else eng.current_hashrate),
        "engine_hashrate_trace_ghs": getattr(eng, "hashrate_trace_ghs", []),
    }


def _switch_job(seed: int, algorithm: str) -> dict:
    import hashlib

    from otedama_amd.models.algorithms import ALGORITHMS
    from otedama_amd.models.header import int_to_hash

    h = hashlib.sha256(f"otedama-switch-{algorithm}-{seed}".encode()).digest()
    header = (0x20000000).to_bytes(4, "little") + h + hashlib.sha256(h).digest() + \
        (1_700_000_000).to_bytes(4, "little") + (0x1703A30C).to_bytes(4, "little") + bytes(4)
    return {"header": header, "target": int_to_hash(ALGORITHMS[algorithm].diff1), "job_id": f"s{seed}",
            "epoch": seed + 1, "algo": algorithm, "version_mask": 0x1FFFE000}


def measure_job_switch(device_index: int = 0, algorithm: str = "sha256d", switches: int = 8,
                       dwell: float | None = None, batch_nonces: int = 1 << 32) -> dict:
    """Job switch on the production path: the engine's MinerSet hands new work to the GPU's device process
    (msgpack frame over the socketpair, engine/devproc.py) ``switches`` times; each sample is engine set_job -> the
    first batch of the new work running on the GPU = the frame hop (parent send -> child's native set_job, on the
    shared CLOCK_MONOTONIC) + the native switch (set_job -> new batch running, measured by the miner thread). The
    in-process miner's own number is kept as ``in_process``."""
    from otedama_amd import hal
    from otedama_amd.engine.miners import MinerSet

    dwell = dwell if dwell is not None else (0.6 if algorithm == "scrypt" else 0.25)
    devs = [d for d in hal.KFDDriver().enumerate() if d.index == device_index]
    if not devs:
        raise RuntimeError(f"no KFD GPU node for device {device_index}")
    ms = MinerSet(devs, algorithm, batch_nonces, 0, isolation="process")
    dp = ms.miners[0].native
    ms.start()
    try:
        end = time.monotonic() + 60
        while not dp.ready_at and dp.alive and time.monotonic() < end:
            time.sleep(0.01)
        ms.set_job(_switch_job(0, algorithm))
        time.sleep(max(dwell, 2.0 if algorithm == "scrypt" else 0.5))  # first job: allocations, warm-up
        for i in range(1, switches + 1):
            ms.set_job(_switch_job(i, algorithm))
            time.sleep(dwell)
        time.sleep(0.6)  # one more stats frame from the child
        st = dp.stats()
    finally:
        ms.stop()
    if st.get("faulted"):
        raise RuntimeError(st.get("error"))
    native = list(st.get("job_switch_ms", []))
    hops = list(st.get("job_hop_ms", []))
    n = min(len(native), len(hops))
    pairs = list(zip(hops[:n], native[:n]))[1:]  # drop the cold first job
    total = [h + s for h, s in pairs]
    return {"path": "devproc", "p50_ms": statistics.median(total) if total else None,
            "max_ms": max(total) if total else None, "samples_ms": [round(x, 3) for x in total],
            "hop_p50_ms": statistics.median([h for h, _ in pairs]) if pairs else None,
            "native_p50_ms": statistics.median([s for _, s in pairs]) if pairs else None,
            "aborted_launches": st.get("aborted_launches"), "batch_nonces": batch_nonces,
            "definition": "engine MinerSet.set_job(new work) -> device process -> first batch of the new work "
                          "running on the GPU",
            "in_process": measure_job_switch_inprocess(device_index, algorithm, switches, dwell, batch_nonces)}


def measure_job_switch_inprocess(device_index: int = 0, algorithm: str = "sha256d", switches: int = 8,
                                 dwell: float | None = None, batch_nonces: int = 1 << 32) -> dict:
    """Hand an in-process native miner new work ``switches`` times and report set_job -> new batch running."""
    from otedama_amd.ops.native import require_native

    N = require_native()
    cus = N.gpu_cu_count(device_index) or 256
    dwell = dwell if dwell is not None else (0.6 if algorithm == "scrypt" else 0.25)
    m = N.GpuMiner(device_index, f"gpu-{device_index}", batch_nonces=batch_nonces, grid=sha256d_grid(cus), queue_cap=4096,
                   sha_variants=128)
    m.start()
    try:
        m.set_job(_switch_job(0, algorithm))
        time.sleep(max(dwell, 2.0 if algorithm == "scrypt" else 0.5))  # first job: allocations, warm-up
        for i in range(1, switches + 1):
            m.set_job(_switch_job(i, algorithm))
            time.sleep(dwell)
        st = m.stats()
    finally:
        m.stop()
    samples = list(st["job_switch_ms"])[1:]  # drop the cold first job
    if st["faulted"]:
        raise RuntimeError(st["error"])
    return {"p50_ms": statistics.median(samples) if samples else None, "max_ms": max(samples) if samples else None,
            "samples_ms": samples, "aborted_launches": st["aborted_launches"], "batch_nonces": batch_nonces,
            "definition": "set_job(new work) -> first batch of the new work running on the GPU"}


def measure_device_startup(device_index: int = 0, timeout: float = 60.0) -> dict:
    """Start-up of one production device process (engine/devproc.py: torch-free, its own HIP context): process
    spawn -> the first batch of a SHA-256d job running on the GPU, the child's phases, and its resident set."""
    from otedama_amd import hal
    from otedama_amd.engine.devproc import DeviceProcess

    devs = [d for d in hal.KFDDriver().enumerate() if d.index == device_index]
    cus = int(devs[0].extra.get("cus", 256)) if devs else 256
    dp = DeviceProcess(device_index, f"gpu-{device_index}", grid=sha256d_grid(cus))
    dp.set_job(_switch_job(0, "sha256d"))  # sent as soon as the child is up
    t0 = time.time()
    dp.start()
    try:
        end = time.monotonic() + timeout
        while time.monotonic() < end and not dp.first_hash_wall:
            time.sleep(0.005)
        if not dp.first_hash_wall:
            raise RuntimeError(f"device process reported no running batch within {timeout:.0f} s")
        rss = None
        try:
            import psutil

            rss = round(psutil.Process(dp.pid).memory_info().rss / 2**20, 1)
        except Exception:  # noqa: BLE001 - psutil missing / child gone
            pass
        return {"spawn_to_first_batch_s": dp.first_hash_wall - t0,
                "child_phases_s": {k: (v - t0) if v else None for k, v in dp.child_timing.items()},
                "native_phases_ms": dict(dp.native_startup_ms), "rss_mib": rss,
                "definition": "Popen of the device process -> its first SHA-256d batch running on the GPU"}
    finally:
        dp.stop()
