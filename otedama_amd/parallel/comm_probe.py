"""The node's data plane under a saturating miner, measured on one GPU.

In the node every rank process issues R1 / R2 / R3 on its comm stream while its sibling device process keeps every
CU of the same GPU busy with an oversubscribed grid (128 blocks per CU for SHA-256d; the scrypt kernel at full HBM
load). Two questions, each answered with numbers:

1. Do the data-plane operations wait behind that grid? Each op is timed from the rank's call to its result on the
   host (what the node's op loop sees: the H2D staging copy, the collective on the comm stream, the D2H read), idle
   and with the miner running, at node cadence (R2 share gathers at ``cadence_hz``, an R1 64 KiB job blob every 10th
   op, R3 counters every 25th). A one-rank RCCL group is forced (``NodeComm(force=True)``): RCCL runs its one-rank
   path (copies), so the collective itself is cheap and what is measured is whether any GPU work of this process
   is scheduled promptly. A tiny elementwise kernel on the comm stream (``kernel_probe``) measures the scheduling of
   a KERNEL from another process directly: at world > 1, RCCL's collectives are kernels that need CU slots too.
2. Does the data plane cost hash rate? The miner's exact device-timeline rate (the device process's counter pairs)
   over alternating windows without and with the ops.

Each configuration is run with the comm stream at normal and at high priority. The reference's rule is that the
fan-in never stalls a producer (internal/engine/fanin.go:22-58); SURVEY §5.8 puts RCCL on a dedicated stream so the
kernels keep running while R2/R3 move.
"""
from __future__ import annotations

import contextlib
import statistics
import sys
import time


def _say(msg: str) -> None:
    print(f"[comm_probe] {msg}", file=sys.stderr, flush=True)


def _q(xs: list[float]) -> dict:
    xs = sorted(xs)
    n = len(xs)

    def at(p):
        return xs[min(max(int(p * n + 0.5) - 1, 0), n - 1)] if n else None

    return {"p50_ms": at(0.5), "p99_ms": at(0.99), "max_ms": xs[-1] if n else None, "samples": n}


def _miner_rate(dp, t0: tuple[int, float], t1: tuple[int, float]) -> float | None:
    (h0, d0), (h1, d1) = t0, t1
    return (h1 - h0) / (d1 - d0) if d1 > d0 > 0 and h1 > h0 else None


def _counter(dp) -> tuple[int, float]:
    st = dp.stats()
    return int(st.get("hashes", 0)), float(st.get("hashes_done_at_s", 0.0) or 0.0)


def run_ops(comm, seconds: float, cadence_hz: float = 50.0, probe_kernel: bool = True) -> dict:
    """Issue R2 gathers at ``cadence_hz`` (an R1 job blob every 10th op, R3 counters every 25th) for ``seconds``;
    return per-op latency quantiles and the comm-stream kernel probe's."""
    import torch

    lat: dict[str, list[float]] = {"R1_job": [], "R2_gather": [], "R3_counters": [], "kernel": []}
    job = {"job_id": "probe", "header": bytes(80), "coinb1": bytes(2000), "coinb2": bytes(2000),
           "merkle_branches": [bytes(32)] * 12, "epoch": 1}
    shares = [{"epoch": 1, "nonce": i, "ntime": 1, "version": 2, "extranonce2": 3, "found_at": time.monotonic()}
              for i in range(4)]
    x = torch.zeros(1 << 12, dtype=torch.float32, device=comm.dev) if comm.stream is not None else None
    period = 1.0 / cadence_hz
    end = time.monotonic() + seconds
    k = 0
    nxt = time.monotonic()
    while time.monotonic() < end:
        k += 1
        t = time.perf_counter()
        if k % 10 == 0:
            comm.broadcast_job(job)
            lat["R1_job"].append((time.perf_counter() - t) * 1e3)
        elif k % 25 == 0:
            comm.gather_counters([1, 2, 3, 4])
            lat["R3_counters"].append((time.perf_counter() - t) * 1e3)
        else:
            comm.gather_shares(shares)
            lat["R2_gather"].append((time.perf_counter() - t) * 1e3)
        if probe_kernel and x is not None and k % 5 == 0:
            t = time.perf_counter()
            with torch.cuda.stream(comm.stream):
                x.add_(1.0)
            comm.stream.synchronize()
            lat["kernel"].append((time.perf_counter() - t) * 1e3)
        nxt += period
        time.sleep(max(0.0, nxt - time.monotonic()))
    return {k: _q(v) for k, v in lat.items() if v}


# The A/B: "legacy" is the round-4 layout (staging copies on the caller's stream, RCCL's streams and the comm stream
# at normal priority); "node" is the node's layout now (every copy on a high-priority comm stream through pinned
# buffers, RCCL's streams at high priority: comm.rccl_pg_options).
CONFIGS = {"legacy": {"pg_high": False, "staging": "legacy", "stream_priority": None},
           "node": {"pg_high": True, "staging": "stream", "stream_priority": "high"},
           # the node's data plane on GPUs from round 5 on: the native RCCL module (parallel/rcclcomm.py), the whole
           # op one chain on its own high-priority stream, no torch in the rank
           "native": {"native": True}}


def _one_rank_group(device, high: bool) -> None:
    """A one-rank RCCL group as the default group (the probe's own: it is destroyed after each window)."""
    import torch.distributed as dist

    opts = None
    if high:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=device,
                            pg_options=opts)


def _with_config(dev, device_index: int, name: str, fn):
    """Run ``fn(comm)`` with config ``name``'s process group and NodeComm, then tear the group down."""
    import torch.distributed as dist

    from otedama_amd.parallel.comm import DistInfo, NodeComm

    cfg = CONFIGS[name]
    if cfg.get("native"):
        return _with_native(device_index, fn)
    _one_rank_group(dev, cfg["pg_high"])
    try:
        comm = NodeComm(DistInfo(0, 1, device_index, "nccl", dev), bounded=True, deadline=10.0, force=True,
                        stream_priority=cfg["stream_priority"], staging=cfg["staging"])
        run_ops(comm, 0.3)  # warm: RCCL communicator, allocator, kernels
        return fn(comm)
    finally:
        dist.destroy_process_group()


_NATIVE_GEN = [0]


def _with_native(device_index: int, fn):
    from otedama_amd.parallel.commbase import Device, DistInfo
    from otedama_amd.parallel.kvclient import StoreClient
    from otedama_amd.parallel.kvstore import StoreServer
    from otedama_amd.parallel.rcclcomm import NativeNodeComm

    with StoreServer() as srv:
        info = DistInfo(0, 1, device_index, "rccl", Device("cuda", device_index),
                        store=StoreClient("127.0.0.1", srv.port, timeout=30))
        comm = NativeNodeComm(info, bounded=True, deadline=10.0, force=True)
        _NATIVE_GEN[0] += 1
        comm.reform([0], _NATIVE_GEN[0])
        try:
            run_ops(comm, 0.3)
            return fn(comm)
        finally:
            comm.close()


def measure_comm_under_load(device_index: int = 0, algorithms=("sha256d", "scrypt"), seconds: float = 4.0,
                            cadence_hz: float = 50.0, windows: int = 2, reserves=("",), variants=()) -> dict:
    """See the module docstring. Per configuration (CONFIGS) and algorithm: op latency idle / loaded, and the
    miner's rate over alternating windows without / with the ops. ``reserves``: OTEDAMA_RESERVE_CUS specs to run
    the miner with ("" = none; e.g. "0" keeps CU 0 out of the mining kernels' CU mask); each non-empty one is
    reported under "<algo>@reserve:<spec>" with the native configuration only. ``variants``: further miner
    environments ("NAME=VALUE[&NAME=VALUE]", e.g. "OTEDAMA_SCRYPT_SEGMENTS=8"), reported as "<algo>@<variant>" with
    the native configuration only."""
    import torch
    import torch.distributed as dist

    from otedama_amd import hal
    from otedama_amd.engine.latency_probe import _switch_job
    from otedama_amd.engine.miners import MinerSet

    if dist.is_initialized():
        raise RuntimeError("the comm probe needs the default process group to itself")
    dev = torch.device(f"cuda:{device_index}")
    torch.cuda.set_device(dev)
    _say("idle phase")
    out: dict = {"idle": {c: _with_config(dev, device_index, c, lambda comm: run_ops(comm, seconds, cadence_hz))
                          for c in CONFIGS},
                 "configs": CONFIGS, "rccl_world": 1, "cadence_hz": cadence_hz,
                 "definition": ("rank-process call -> result on the host for R1 (64 KiB job blob), R2 (share slots "
                                "all_gather) and R3 (counters all_gather) of a forced one-rank RCCL group; 'kernel' = "
                                "a 16 KiB elementwise kernel on the comm stream, enqueue -> done")}
    devs = [d for d in hal.KFDDriver().enumerate() if d.index == device_index]
    if not devs:
        raise RuntimeError(f"no KFD GPU node for device {device_index}")
    import os

    runs = [(algo, f"reserve:{spec}" if spec else "", {"OTEDAMA_RESERVE_CUS": spec} if spec else {})
            for spec in reserves for algo in algorithms]
    runs += [(algo, v, dict(kv.split("=", 1) for kv in v.split("&"))) for v in variants for algo in algorithms]
    for algo, tag, env in runs:
        key = algo if not tag else f"{algo}@{tag}"
        configs = list(CONFIGS) if not tag else ["native"]
        _say(f"{key}: miner up, alternating windows")
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)  # inherited by the device process
        ms = MinerSet(devs, algo, 1 << 32, 0, isolation="process")
        dp = ms.miners[0].native
        ms.start()
        try:
            end = time.monotonic() + 60
            while not dp.ready_at and dp.alive and time.monotonic() < end:
                time.sleep(0.01)
            ms.set_job(_switch_job(0, algo))
            time.sleep(3.0 if algo == "scrypt" else 1.5)  # allocations, first launches
            res: dict = {"loaded": {}, "rate_alone": [], "rate_with_ops": {c: [] for c in configs}}
            for w in range(windows):
                a = _counter(dp)
                time.sleep(seconds)
                res["rate_alone"].append(_miner_rate(dp, a, _counter(dp)))
                for c in configs:
                    def window(comm, c=c, w=w):
                        a = _counter(dp)
                        r = run_ops(comm, seconds, cadence_hz)
                        res["rate_with_ops"][c].append(_miner_rate(dp, a, _counter(dp)))
                        if w == 0:
                            res["loaded"][c] = r

                    _with_config(dev, device_index, c, window)
            st = dp.stats()
            if st.get("faulted"):
                raise RuntimeError(st.get("error"))
            res["reserved_cus"] = st.get("reserved_cus", 0)
        finally:
            ms.stop()
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        alone = [r for r in res["rate_alone"] if r]
        base = statistics.fmean(alone) if alone else None
        res["rate_alone_hps"] = base
        res["rate_loss_pct"] = {c: (100.0 * (1.0 - statistics.fmean([r for r in v if r]) / base)
                                    if base and any(v) else None) for c, v in res["rate_with_ops"].items()}
        out[key] = res
    return out


# ---------------------------------------------------------------------------------------------------------------------
# bench.py's comm section: the node's collectives measured across every rank of the run
NODE_COMM_DEFINITION = (
    "every rank in lockstep on the run's data plane (bench.py preflight.data_plane): R1 = the node's 64 KiB job-blob "
    "broadcast, R2 = its share-slot all_gather (64 x 10 int64 per rank), R3 = its counter all_reduce, each host call -> "
    "result on the host; R2_dev = bench.py's device-resident hit-slot gather, enqueue -> stream done. Ops interleaved "
    "R1,R2,R3,R2_dev at `cadence_hz` from a common barrier. Phases: idle, then with every rank's device process mining "
    "the named algorithm (the production miner, one per GPU). miner_rate_change_pct = node-wide miner rate with the ops "
    "against an equal window without them. busbw: one all_gather of `busbw_bytes` in total (device buffers), "
    "busbw = bytes/time x (N-1)/N as nccl-tests defines it")


def _lockstep_ops(comm, ops: int, cadence_hz: float, dev) -> dict:
    """``ops`` of each of R1 / R2 / R3 / R2_dev, interleaved, every rank on the same schedule from a barrier."""
    import torch

    from otedama_amd.parallel.commbase import SHARE_SLOTS

    job = {"job_id": "comm", "header": bytes(80), "coinb1": bytes(2000), "coinb2": bytes(2000),
           "merkle_branches": [bytes(32)] * 12, "epoch": 1}
    shares = [{"epoch": 1, "nonce": i, "ntime": 1, "version": 2, "extranonce2": 3, "found_at": time.monotonic()}
              for i in range(4)]
    world = comm.info.world_size
    slot = torch.zeros(1 + 2 * SHARE_SLOTS, dtype=torch.int32, device=dev)
    gathered = torch.zeros(world, slot.numel(), dtype=torch.int32, device=dev)
    cuda = dev.type == "cuda"
    lat: dict[str, list[float]] = {"R1": [], "R2": [], "R3": [], "R2_dev": []}
    names = list(lat)
    comm.barrier()
    t0 = time.monotonic()
    period = 1.0 / cadence_hz
    for k in range(4 * ops):
        time.sleep(max(0.0, t0 + k * period - time.monotonic()))
        op = names[k % 4]
        t = time.perf_counter()
        if op == "R1":
            comm.broadcast_job(job)
        elif op == "R2":
            comm.gather_shares(shares)
        elif op == "R3":
            comm.allreduce_counters(1, 2, 3, 4)
        else:
            stream = comm.stream if cuda else None
            with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
                comm.gather_tensor(gathered, slot)
            if stream is not None:
                stream.synchronize()
            elif cuda:
                torch.cuda.synchronize(dev)
        lat[op].append((time.perf_counter() - t) * 1e3)
    return {k: _q(v) for k, v in lat.items()}


def _busbw(comm, dev, total_bytes: int, iters: int = 5) -> dict:
    """One all_gather of ``total_bytes`` in total (each rank contributes total/N), timed over ``iters`` after a warm
    one; every rank's block is checked."""
    import torch

    world, rank = comm.info.world_size, comm.info.rank
    per = max(4096, (total_bytes // world) // 4096 * 4096)
    send = torch.full((per,), (rank + 1) & 0xFF, dtype=torch.uint8, device=dev)
    recv = torch.zeros(world, per, dtype=torch.uint8, device=dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    comm.gather_tensor(recv, send)
    sync()
    ok = all(int(recv[r, 0]) == (r + 1) & 0xFF and int(recv[r, -1]) == (r + 1) & 0xFF for r in range(world))
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        comm.gather_tensor(recv, send)
    sync()
    t = comm.allreduce_max((time.perf_counter() - t0) / iters)
    ok = comm.allreduce_counters(int(ok))[0] == world
    algbw = per * world / t / 1e9
    return {"bytes": per * world, "iters": iters, "ms": t * 1e3, "algbw_gbps": algbw,
            "busbw_gbps": algbw * (world - 1) / world, "blocks_ok": ok, "device": dev.type}


def _start_miner(device_index: int, algo: str):
    from otedama_amd import hal
    from otedama_amd.engine.latency_probe import _switch_job
    from otedama_amd.engine.miners import MinerSet

    devs = [d for d in hal.KFDDriver().enumerate() if d.index == device_index]
    if not devs:
        raise RuntimeError(f"no KFD GPU node for device {device_index}")
    ms = MinerSet(devs, algo, 1 << 32, 0, isolation="process")
    dp = ms.miners[0].native
    ms.start()
    end = time.monotonic() + 60
    while not dp.ready_at and dp.alive and time.monotonic() < end:
        time.sleep(0.01)
    if not dp.ready_at:
        ms.stop()
        raise RuntimeError(f"{algo} device process not ready")
    ms.set_job(_switch_job(0, algo))
    return ms, dp


def measure_node_comm(comm, dev, phases=("idle", "sha256d", "scrypt"), ops: int = 200, cadence_hz: float = 100.0,
                      busbw_bytes: int = 256 << 20, rate_window_s: float = 3.0, warm_s: dict | None = None,
                      say=None) -> dict:
    """bench.py's comm section (NODE_COMM_DEFINITION). Every rank calls this with the same arguments; each step that
    could fail on one rank (a miner that does not start) is agreed on through R3 first, so no rank is left alone in
    a collective."""
    say = say or (lambda m: None)
    world = comm.info.world_size
    warm_s = warm_s or {"sha256d": 1.5, "scrypt": 3.0}
    out: dict = {"world": world, "ops_per_type": ops, "cadence_hz": cadence_hz, "definition": NODE_COMM_DEFINITION}
    rates: dict = {}
    for ph in phases:
        if ph == "idle":
            say("comm: idle ops")
            out["idle"] = _lockstep_ops(comm, ops, cadence_hz, dev)
            continue
        say(f"comm: {ph} miner up")
        ms = dp = None
        err = ""
        try:
            ms, dp = _start_miner(dev.index or 0, ph)
            time.sleep(warm_s.get(ph, 2.0))
        except Exception as exc:  # noqa: BLE001 - agreed below
            err = f"{type(exc).__name__}: {exc}"[:200]
        try:
            if comm.allreduce_counters(int(ms is not None))[0] != world:
                out[ph] = {"skipped": err or "a peer's miner did not start"}
                continue
            comm.barrier()
            a = _counter(dp)
            time.sleep(rate_window_s)
            alone = _miner_rate(dp, a, _counter(dp)) or 0.0
            a = _counter(dp)
            res = _lockstep_ops(comm, ops, cadence_hz, dev)
            with_ops = _miner_rate(dp, a, _counter(dp)) or 0.0
            st = dp.stats()
            res["miner_rate_alone_hps"], res["miner_rate_with_ops_hps"] = alone, with_ops
            res["miner_faulted"] = bool(st.get("faulted"))
            out[ph] = res
            rates[ph] = (alone, with_ops)
        finally:
            if ms is not None:
                ms.stop()
    if rates:
        change = {}
        for ph, (alone, with_ops) in rates.items():
            tot_alone, tot_with, _, _ = comm.allreduce_counters(int(alone), int(with_ops))
            change[ph] = round(100.0 * (tot_with / tot_alone - 1.0), 2) if tot_alone > 0 else None
        out["miner_rate_change_pct"] = change
    if busbw_bytes > 0:
        say("comm: bus bandwidth")
        out["busbw"] = _busbw(comm, dev, busbw_bytes)
    return out


def main(argv=None) -> int:
    import argparse
    import json

    ap = argparse.ArgumentParser(prog="otedama_amd.parallel.comm_probe")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--algorithms", default="sha256d,scrypt")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--cadence", type=float, default=50.0)
    ap.add_argument("--windows", type=int, default=2)
    ap.add_argument("--reserves", default="", help="';'-separated OTEDAMA_RESERVE_CUS specs besides none, e.g. '0;0,32'")
    ap.add_argument("--variants", default="",
                    help="';'-separated miner environments, e.g. 'OTEDAMA_SCRYPT_SEGMENTS=8;OTEDAMA_SCRYPT_SEGMENTS=16'")
    a = ap.parse_args(argv)
    reserves = [""] + [x for x in a.reserves.split(";") if x]
    r = measure_comm_under_load(a.device, [x for x in a.algorithms.split(",") if x], a.seconds, a.cadence, a.windows,
                                reserves, [x for x in a.variants.split(";") if x])
    print(json.dumps(r))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
