"""The production node, measured the way an operator runs it (bench.py ``node`` object).

``otedama node --gpus N`` (the GPU-free supervisor, N ranks over RCCL, every rank's GPU miner in a device process of
its own, rank 0 holding the Stratum V2 session) mines against ``otedama pool`` in a separate process whose share
difficulty is pinned. Rank 0 writes its view of the node every 0.5 s (OTEDAMA_NODE_REPORT, engine/run.py
``node_report``); this module reads it over a recorded window after a warm-up and reports:

  * the node total hashrate and per-rank rates, each from one rank's device-timeline counter pairs
    (cumulative hashes, the device time at which they had completed) at the window's ends, so the rate is exact,
    not quantized by launch boundaries;
  * accepted / rejected shares (the engine's verdicts and the pool's own count, with reject reasons);
  * the RCCL ranks seen (the process group's members), the backend, and the device collectives every rank issued;
  * device hit -> pool accept quantiles with sample counts, separately for rank 0's own shares and for shares found
    by the other ranks (which cross the R2 gather), over the window.

The reference's whole-node figure is its production worker's rate (BENCHMARKS.md:44-49) and its latency metric covers
every share (internal/engine/run.go:813-821).
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import tempfile
import time

from otedama_amd.engine.latency_probe import PROBE_ADDR, ROOT, spawn_pool, stop_pool

_DROP_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
             "MASTER_PORT", "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
             "TORCHELASTIC_MAX_RESTARTS", "OTEDAMA_NODE_JOIN", "OTEDAMA_STORE_HOSTED", "OTEDAMA_PG_TIMEOUT")


def _read(path: str) -> dict:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _quantiles(xs: list[float]) -> dict:
    xs = sorted(xs)
    n = len(xs)

    def q(p: float):
        if not n:
            return None
        return xs[min(max(int(p * n + 0.5) - 1, 0), n - 1)]  # nearest rank (engine/stats.py LatencyTracker)

    return {"p50_ms": q(0.5), "p95_ms": q(0.95), "p99_ms": q(0.99), "samples": n}


def _rank_of(key: str) -> int:
    return int(key[4:]) if key.startswith("rank") else 0


def window_rates(samples: list, t0: float, t1: float) -> dict[str, float]:
    """Per counter key: (hashes_last - hashes_first) / (done_last - done_first) over the samples taken in
    [t0, t1] (device-timeline span); a key without a device timeline (CPU miners) falls back to the wall span."""
    inside = [(t, c) for t, c in samples if t0 <= t <= t1]
    out: dict[str, float] = {}
    if len(inside) < 2:
        return out
    keys = set(inside[0][1]) | set(inside[-1][1])
    for k in keys:
        pts = [(t, c[k]) for t, c in inside if k in c]
        if len(pts) < 2:
            continue
        (ta, (ha, da)), (tb, (hb, db)) = pts[0], pts[-1]
        if db > da > 0:
            out[k] = (hb - ha) / (db - da)
        elif tb > ta:
            out[k] = (hb - ha) / (tb - ta)
    return out


def process_rss(sup_pid: int) -> dict:
    """Resident set (MiB) of the node's processes by role: the supervisor, each rank (torch + the RCCL communicator),
    and each rank's device process (the GPU miner)."""
    try:
        import psutil
    except ImportError:
        return {}
    out: dict = {}
    try:
        sup = psutil.Process(sup_pid)
        out["supervisor"] = round(sup.memory_info().rss / 2**20, 1)
        for rank in sup.children():
            try:
                r = rank.environ().get("RANK", "?")
                out[f"rank{r}"] = round(rank.memory_info().rss / 2**20, 1)
                for c in rank.children():
                    if "otedama_amd.engine.devproc" in " ".join(c.cmdline()):
                        out[f"rank{r}_device_process"] = round(c.memory_info().rss / 2**20, 1)
            except (psutil.NoSuchProcess, psutil.AccessDenied):
                pass
    except (psutil.NoSuchProcess, psutil.AccessDenied):
        pass
    return out


# Expected per-GPU (per-rank CPU thread in the rehearsal) rates: the pinned share difficulty gives ~shares_per_gpu
# accepted shares per second per rank at these rates (MI355X: BASELINE.md; CPU: one native miner thread).
EXPECTED_RATE = {"gpu": {"sha256d": 19e9, "x11": 3.9e8, "scrypt": 1.7e7},
                 "cpu": {"sha256d": 8e6, "x11": 4e3, "scrypt": 1.2e4}}
HASHES_PER_DIFF1 = {"sha256d": 2.0 ** 32, "x11": 2.0 ** 32, "scrypt": 2.0 ** 16}  # scrypt diff1 = 0xFFFF << 224


def job_switch_stats(block_at: list[float], work_started: dict[str, list], ranks: int,
                     job_set_at: list | None = None, window: float = 2.0, job_bcast_at: list | None = None,
                     job_applied: dict[str, list] | None = None) -> dict:
    """Node-wide job switch from the pool's forced new blocks: for each block sent at t_b (CLOCK_MONOTONIC, which
    every process of the host shares) and each rank, the first (epoch, t) in that rank's work-start record with
    t_b < t <= t_b + window is the moment the rank's device was running the new block's work. Reported per rank and
    for the worst rank: p50 / max in ms, and how many block x rank pairs never showed a start (``missing``)."""
    per_rank: dict[str, list[float]] = {f"rank{r}": [] for r in range(ranks)}
    missing = 0
    worst_each: list[float] = []
    leader_each: list[float] = []
    bcast_each: list[float] = []
    applied_each: dict[str, list[float]] = {}
    blocks = sorted(block_at)
    for bi, tb in enumerate(blocks):
        # a start belongs to this block only before the next block was sent
        end = min(tb + window, blocks[bi + 1]) if bi + 1 < len(blocks) else tb + window
        worst = None
        for r in range(ranks):
            ts = sorted(t for _e, t in (work_started.get(f"rank{r}") or []) if tb < t <= end)
            if not ts:
                missing += 1
                continue
            ms = (ts[0] - tb) * 1e3
            per_rank[f"rank{r}"].append(ms)
            worst = ms if worst is None else max(worst, ms)
        if worst is not None:
            worst_each.append(worst)
        sets = sorted(t for _e, t in (job_set_at or []) if tb < t <= end)
        if sets:
            leader_each.append((sets[0] - tb) * 1e3)
        bc = sorted(t for _e, t in (job_bcast_at or []) if tb < t <= end)
        if bc:
            bcast_each.append((bc[0] - tb) * 1e3)
        for r in range(1, ranks):
            ap = sorted(t for _e, t in ((job_applied or {}).get(f"rank{r}") or []) if tb < t <= end)
            if ap:
                applied_each.setdefault(f"rank{r}", []).append((ap[0] - tb) * 1e3)

    def med(xs):
        xs = sorted(xs)
        return xs[len(xs) // 2] if xs else None

    rows = {r: {"p50_ms": med(v), "max_ms": max(v) if v else None, "samples": len(v)} for r, v in per_rank.items()}
    p50s = [v["p50_ms"] for v in rows.values() if v["p50_ms"] is not None]
    maxs = [v["max_ms"] for v in rows.values() if v["max_ms"] is not None]
    return {"blocks": len(blocks), "per_rank": rows,
            "worst_rank_p50_ms": max(p50s) if p50s else None, "worst_rank_max_ms": max(maxs) if maxs else None,
            "node_p50_ms": med(worst_each), "missing": missing,
            "pool_to_leader_p50_ms": med(leader_each),
            # where the time goes (medians, ms after the pool's send): the leader's R1 broadcast completing, and each
            # follower handing the job to its device process
            "pool_to_r1_done_p50_ms": med(bcast_each),
            "pool_to_follower_apply_p50_ms": {r: med(v) for r, v in applied_each.items()} or None,
            "definition": ("pool's new block (forced SetNewPrevHash, CLOCK_MONOTONIC at send) -> each rank's device "
                           "process running the first batch of the new work; node_p50 = median over blocks of the "
                           "slowest rank")}


def _switch_gap(algorithm: str, cpu: bool) -> float:
    """Seconds between forced blocks: a rank's first batch of block k must start before block k+1 is sent to count.
    CPU rehearsals run N ranks + their miners + the pool on a few shared cores, where a follower's apply can lag a
    second behind (a tests/test_bench_launcher.py world-4 run missed 4 of 32 starts at 1 s, and 1 of 32 at 2 s with
    other node tests running beside it)."""
    return (1.5 if algorithm == "scrypt" else 1.0) * (3.0 if cpu else 1.0)


def measure_node(gpus: int, seconds: float = 10.0, warmup: float = 3.0, shares_per_gpu: float = 25.0,
                 expected_per_gpu: float | None = None, startup_timeout: float = 150.0, cpu: bool = False,
                 log_path: str | None = None, algorithm: str = "sha256d", switches: int = 0,
                 switch_interval: float | None = None) -> dict:
    """Run ``otedama node --gpus N`` mining ``algorithm`` against a pinned-difficulty pool for ``warmup`` + ``seconds``
    and measure it; then force ``switches`` new blocks at the pool (SIGUSR1) and time how fast each rank's device
    runs the new work (``job_switch``). ``cpu``: a CPU rehearsal (gloo ranks, one CPU miner thread per rank) of the
    same processes."""
    kind = "cpu" if cpu else "gpu"
    if expected_per_gpu is None:
        expected_per_gpu = EXPECTED_RATE[kind][algorithm]
        shares_per_gpu = 4.0 if cpu else shares_per_gpu
    diff = expected_per_gpu / (shares_per_gpu * HASHES_PER_DIFF1[algorithm])
    tmp = tempfile.mkdtemp(prefix="otedama-node-")
    report = os.path.join(tmp, "report.json")
    log_path = log_path or os.path.join(tmp, "node.log")
    pool, addr = spawn_pool(algorithm, diff, fixed=True)
    cfg = os.path.join(tmp, "config.yaml")
    with open(cfg, "w") as f:
        f.write(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addr}\n"
                f"mining:\n  algorithm: {algorithm}\n" + ("  cpu_threads: 1\n" if cpu else ""))
    env = {k: v for k, v in os.environ.items() if k not in _DROP_ENV}
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env["OTEDAMA_NODE_REPORT"] = report
    env["OTEDAMA_PG_TIMEOUT"] = "60"
    if cpu:
        env.update(OTEDAMA_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    t_spawn, t_spawn_wall = time.monotonic(), time.time()
    out = open(log_path, "w")
    sup = subprocess.Popen([sys.executable, "-m", "otedama_amd", "node", "--gpus", str(gpus), "--config", cfg,
                            "--no-tui"], env=env, cwd=ROOT, stdout=out, stderr=subprocess.STDOUT)
    res: dict = {"algorithm": algorithm, "n_ranks": gpus, "share_difficulty_requested": diff,
                 "recorded_seconds": seconds, "warmup_seconds": warmup, "log": log_path}
    rep: dict = {}
    forced: list[float] = []
    pst: dict = {}
    try:
        # ready: every rank of the node is a member and has counted hashes on its device timeline
        end = time.monotonic() + startup_timeout
        while time.monotonic() < end:
            rep = _read(report)
            c = rep.get("counters", {})
            ranks = {_rank_of(k) for k, (h, _d) in c.items() if h > 0}
            if rep.get("connected") and rep.get("accepted", 0) > 0 and ranks >= set(range(gpus)) \
                    and len(rep.get("members", [])) == gpus:
                break
            if sup.poll() is not None:
                raise RuntimeError(f"otedama node exited with code {sup.returncode}")
            time.sleep(0.25)
        else:
            raise RuntimeError(f"node not ready within {startup_timeout:.0f} s")
        res["startup_s"] = time.monotonic() - t_spawn
        # where the start-up goes: seconds after rank 0's process started (torch import, rendezvous, engine phases,
        # the device process's first batch), and the supervisor's spawn -> rank 0's process start
        res["startup_phases_s"] = rep.get("startup_phases_s")
        if rep.get("process_start_wall"):
            res["supervisor_to_rank0_start_s"] = round(rep["process_start_wall"] - t_spawn_wall, 3)
            # `otedama node` launched -> rank 0's device process running its first batch (the reference's "reaches
            # hashing" figure, BENCHMARKS.md:105-118); startup_s above also waits for the first accepted share
            first = (res["startup_phases_s"] or {}).get("first_batch_running")
            if first is not None:
                res["time_to_hashing_s"] = round(res["supervisor_to_rank0_start_s"] + first, 3)
        time.sleep(warmup)
        t0 = time.monotonic()
        time.sleep(seconds)
        t1 = time.monotonic()
        while _read(report).get("mono", 0.0) < t1 + 0.5 and time.monotonic() < t1 + 5:  # a sample past the window
            time.sleep(0.1)
        rep = _read(report)
        res["rss_mib"] = process_rss(sup.pid)
        # node-wide job switch: new blocks forced at the pool, spaced so every rank's heartbeat (2 Hz, the last 8
        # starts) carries each one
        gap = switch_interval or _switch_gap(algorithm, cpu)
        rej0 = int(rep.get("rejected", 0) or 0)
        for _ in range(max(0, switches)):
            pool.send_signal(signal.SIGUSR1)
            forced.append(time.monotonic())
            time.sleep(gap)
        if switches > 0:
            time.sleep(1.2)  # the last start reaches the report through a heartbeat and a report tick
            rep_sw = _read(report)
            res["_switch_report"] = rep_sw
            res["_rej_during_switches"] = int(rep_sw.get("rejected", 0) or 0) - rej0
    finally:
        sup.send_signal(signal.SIGTERM)
        try:
            res["exit_code"] = sup.wait(timeout=60)
        except subprocess.TimeoutExpired:
            sup.kill()
            res["exit_code"] = sup.wait()
        out.close()
        pst = stop_pool(pool)
    rates = window_rates(rep.get("samples", []), t0, t1 + 0.75)
    per_rank = [0.0] * gpus
    for k, r in rates.items():
        if _rank_of(k) < gpus:
            per_rank[_rank_of(k)] += r
    acc = [a for a in rep.get("accept_log", []) if t0 <= a[0] <= t1]
    lat = {o: _quantiles([a[1] for a in acc if a[2] == o and a[1] is not None]) for o in ("local", "remote")}
    host = {o: _quantiles([a[4] for a in acc if a[2] == o and len(a) > 4 and a[4] is not None])
            for o in ("local", "remote")}
    follower_coll = rep.get("follower_collectives", {})
    res.update({
        "total_hashes_per_sec": sum(per_rank),
        "per_rank_hashes_per_sec": per_rank,
        "per_device_hashes_per_sec": rates,
        "rate_source": "device-timeline counter pairs at the window ends (one per rank's device process)",
        "accepted_in_window": len(acc),
        "accepted_remote_in_window": sum(1 for a in acc if a[2] == "remote"),
        "accepted": rep.get("accepted"), "rejected": rep.get("rejected"),
        "pool_accepted": pst.get("accepted"), "pool_rejected": pst.get("rejected"),
        "pool_reject_reasons": pst.get("reject_reasons"), "pool_validate_ms": pst.get("validate_ms"),
        "share_difficulty": rep.get("share_difficulty"),
        "dist_backend": rep.get("backend"), "ranks_seen": sorted(rep.get("members", [])),
        "generation": rep.get("generation"), "reforms": rep.get("reforms", 0), "lost_ranks": rep.get("lost_ranks", []),
        "collectives": {"rank0": rep.get("leader_collectives", 0), **follower_coll},
        "collectives_total": rep.get("leader_collectives", 0) + sum(follower_coll.values()),
        "node_ops": rep.get("ops", 0), "op_p50_ms": rep.get("op_p50_ms"), "op_p99_ms": rep.get("op_p99_ms"),
        "remote_stale": rep.get("remote_stale", 0),
        "share_previews": rep.get("share_previews", 0),
        "share_gathered_first": rep.get("share_gathered_first", 0),
        "hit_to_accept_rank0": lat["local"], "hit_to_accept_remote": lat["remote"],
        "host_verify_to_accept_rank0": host["local"], "host_verify_to_accept_remote": host["remote"],
        "definition": ("otedama node --gpus N (supervisor + N ranks, RCCL between them, each rank's GPU miner in its "
                       "own device process, rank 0 holding the SV2 session) against otedama pool (separate process, "
                       "pinned difficulty); rates and latencies over the recorded window after the warm-up"),
    })
    rep_sw = res.pop("_switch_report", None)
    rej_sw = res.pop("_rej_during_switches", None)
    if rep_sw is not None:
        # the pool's own send times of the forced blocks (its first block is the one the node started on)
        sent = [t for t in pst.get("new_block_at", []) if t >= (forced[0] - 0.5 if forced else 0)]
        js = job_switch_stats(sent or forced, rep_sw.get("work_started", {}), gpus, rep_sw.get("job_set_at"),
                              job_bcast_at=rep_sw.get("job_bcast_at"), job_applied=rep_sw.get("job_applied"))
        stale = (pst.get("reject_reasons") or {}).get("stale-job", 0)
        js.update({"forced_blocks": len(forced), "stale_rejects": stale, "engine_rejects_during_switches": rej_sw,
                   "interval_s": switch_interval or _switch_gap(algorithm, cpu)})
        res["job_switch"] = js
    return res
