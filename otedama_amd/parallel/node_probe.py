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


def measure_node(gpus: int, seconds: float = 10.0, warmup: float = 3.0, shares_per_gpu: float = 25.0,
                 expected_per_gpu: float = 19e9, startup_timeout: float = 150.0, cpu: bool = False,
                 log_path: str | None = None) -> dict:
    """Run ``otedama node --gpus N`` against a pinned-difficulty pool for ``warmup`` + ``seconds`` and measure it.
    ``cpu``: a CPU rehearsal (gloo ranks, one CPU miner thread per rank) of the same processes."""
    hashes_per_diff1 = 2.0 ** 32
    diff = expected_per_gpu / (shares_per_gpu * hashes_per_diff1)
    tmp = tempfile.mkdtemp(prefix="otedama-node-")
    report = os.path.join(tmp, "report.json")
    log_path = log_path or os.path.join(tmp, "node.log")
    pool, addr = spawn_pool("sha256d", diff, fixed=True)
    cfg = os.path.join(tmp, "config.yaml")
    with open(cfg, "w") as f:
        f.write(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addr}\n"
                + ("mining:\n  cpu_threads: 1\n" if cpu else ""))
    env = {k: v for k, v in os.environ.items() if k not in _DROP_ENV}
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env["OTEDAMA_NODE_REPORT"] = report
    env["OTEDAMA_PG_TIMEOUT"] = "60"
    if cpu:
        env.update(OTEDAMA_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    t_spawn = time.monotonic()
    out = open(log_path, "w")
    sup = subprocess.Popen([sys.executable, "-m", "otedama_amd", "node", "--gpus", str(gpus), "--config", cfg,
                            "--no-tui"], env=env, cwd=ROOT, stdout=out, stderr=subprocess.STDOUT)
    res: dict = {"n_ranks": gpus, "share_difficulty_requested": diff, "recorded_seconds": seconds,
                 "warmup_seconds": warmup, "log": log_path}
    rep: dict = {}
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
        time.sleep(warmup)
        t0 = time.monotonic()
        time.sleep(seconds)
        t1 = time.monotonic()
        while _read(report).get("mono", 0.0) < t1 + 0.5 and time.monotonic() < t1 + 5:  # a sample past the window
            time.sleep(0.1)
        rep = _read(report)
        res["rss_mib"] = process_rss(sup.pid)
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
        "hit_to_accept_rank0": lat["local"], "hit_to_accept_remote": lat["remote"],
        "host_verify_to_accept_rank0": host["local"], "host_verify_to_accept_remote": host["remote"],
        "definition": ("otedama node --gpus N (supervisor + N ranks, RCCL between them, each rank's GPU miner in its "
                       "own device process, rank 0 holding the SV2 session) against otedama pool (separate process, "
                       "pinned difficulty); rates and latencies over the recorded window after the warm-up"),
    })
    return res
