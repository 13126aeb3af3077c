"""BASELINE config 5, measured: the full Stratum pool with mixed SHA-256d + scrypt workers (bench.py ``pool``).

``otedama pool --algorithms sha256d,scrypt`` (one process, one SV2 listener, vardiff state, journal and validator per
algorithm) serves production miners: one ``otedama run`` per (GPU, algorithm) stream, each with its GPU's miner in a
device process. At one GPU both streams share GPU 0 (a SHA-256d and a scrypt device process); at N GPUs the first
ceil(N/2) GPUs mine SHA-256d and the rest scrypt. Vardiff is ON and every connection starts at the same initial
difficulty, so the record shows the pool converging each worker to its own rate. Reported per algorithm, over the
recorded window: validated shares/s (every accepted share was re-hashed by the pool: SHA-256d inline, scrypt on the
pool's native hash workers), rejects by reason, the pool's validation time (submit received -> verdict) quantiles,
each worker's difficulty in force / retarget count / time from channel open to its last retarget, and the miners'
device-timeline hashrates.

Steady state: the recorded window opens only once every worker's vardiff has settled (its
difficulty rests on most of a full estimator window, no refinement is left and none is pending; pool/vardiff.py) and
its estimate points within 10% of the difficulty in force; convergence time is reported on its own, and so is each
worker's retarget count inside the window (0 when the window really was steady). The vardiff target is a 0.05 s
share interval, so every algorithm collects several hundred validations in the window. Each worker's share
interval over the window is reported against that target (the reference's relation interval = D * 2^32 / H,
internal/engine/stats.go:502-513), and validation quantiles are computed from the pool's timed log over the window
only. A short flood (pool/load.py: SV2 clients submitting valid shares as fast as the pool acknowledges) gives the
pool's validated-shares-per-second ceiling per algorithm.

[NO REFERENCE CODE]: v3 removed the pool; BASELINE.json names this config without a number.
"""
from __future__ import annotations

import json
import math
import os
import signal
import subprocess
import sys
import tempfile
import time
import urllib.request

from otedama_amd.engine.latency_probe import PROBE_ADDR, ROOT
from otedama_amd.parallel.launch import free_port
from otedama_amd.parallel.node_probe import _DROP_ENV, _read, window_rates


def spawn_mixed_pool(algorithms: list[str], difficulty: float, share_seconds: float, retarget_seconds: float,
                     http: str, timeout: float = 120.0) -> tuple[subprocess.Popen, dict[str, str]]:
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = [sys.executable, "-m", "otedama_amd", "pool", "--algorithms", ",".join(algorithms),
           "--listen-sv2", "127.0.0.1:0", "--listen-v1=", "--difficulty", repr(difficulty),
           "--share-seconds", repr(share_seconds), "--retarget-seconds", repr(retarget_seconds),
           "--job-interval", "3600", "--block-interval", "3600", "--payout-address", PROBE_ADDR, "--http-addr", http]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
    addrs: dict[str, str] = {}
    deadline = time.monotonic() + timeout
    seen = []
    while time.monotonic() < deadline and len(addrs) < len(algorithms):
        line = proc.stdout.readline()
        if not line:
            break
        seen.append(line)
        if "listening sv2=" in line and "pool[" in line:
            algo = line.split("pool[", 1)[1].split("]", 1)[0]
            addrs[algo] = line.split("listening sv2=", 1)[1].split()[0]
    if len(addrs) < len(algorithms):
        proc.kill()
        raise RuntimeError("pool process did not start: " + "".join(seen[-5:]))
    return proc, addrs


def stop_pool_all(proc: subprocess.Popen) -> list[dict]:
    """SIGTERM the pool; it prints one JSON stats line per algorithm on the way out."""
    proc.send_signal(signal.SIGTERM)
    try:
        out, _ = proc.communicate(timeout=30)
    except subprocess.TimeoutExpired:
        proc.kill()
        out, _ = proc.communicate()
    res = []
    for line in (out or "").splitlines():
        if line.startswith("{"):
            try:
                res.append(json.loads(line))
            except ValueError:
                pass
    return res


def _pool_api(http: str) -> list[dict]:
    with urllib.request.urlopen(f"http://{http}/api/v1/pool", timeout=5) as r:
        return json.loads(r.read())


def layout(gpus: int) -> list[tuple[int, str]]:
    """(GPU, algorithm) streams: both algorithms on GPU 0 at one GPU, else the first ceil(N/2) GPUs SHA-256d."""
    if gpus <= 1:
        return [(0, "sha256d"), (0, "scrypt")]
    half = math.ceil(gpus / 2)
    return [(i, "sha256d" if i < half else "scrypt") for i in range(gpus)]


def _window_quantiles(log: list, t0: float, t1: float) -> dict:
    xs = sorted(ms for t, ms in log if t0 <= t <= t1)
    n = len(xs)

    def q(p: float):
        return xs[min(max(int(p * n + 0.5) - 1, 0), n - 1)] if n else None  # nearest rank

    return {"p50": q(0.5), "p95": q(0.95), "p99": q(0.99), "max": xs[-1] if n else None, "samples": n}


def flood(algorithms: list[str], seconds: float = 3.0, miners: int = 8, timeout: float = 90.0) -> dict:
    """The pool's validated-shares/s ceiling per algorithm: pool/load.py in its own process (the pool and SV2 flood
    clients, every share valid at the clamped minimum difficulty, fully validated and journaled)."""
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    out = subprocess.run([sys.executable, "-m", "otedama_amd.pool.load", "--algo", ",".join(algorithms),
                          "--miners", str(miners * len(algorithms)), "--seconds", repr(seconds)],
                         capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    res = {}
    for line in out.stdout.splitlines():
        if line.startswith("{"):
            r = json.loads(line)
            res[r["pool"]] = {"validated_shares_per_sec": r["validated_shares_per_sec"], "rejected": r["rejected"],
                              "ack_p50_ms": r["ack_latency_ms"]["p50"], "ack_p99_ms": r["ack_latency_ms"]["p99"],
                              "miners": r["miners"], "seconds": r["seconds"]}
    if not res:
        raise RuntimeError(f"flood produced no result: {out.stderr[-500:]}")
    return res


def _wait_hashing(miners: list, timeout: float) -> None:
    """Until every started miner's report shows device hashes (or ``timeout``): its GPU work is running."""
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        reps = [_read(m["report"]) for m in miners]
        if all(any(int((c or [0])[0]) > 0 for c in (r.get("counters") or {}).values()) for r in reps):
            return
        if any(m["proc"].poll() is not None for m in miners):
            raise RuntimeError(f"miner(s) exited: {[m['name'] for m in miners if m['proc'].poll() is not None]}")
        time.sleep(0.2)


def _hashes_per_diff1(algo: str) -> float:
    """Expected hashes per difficulty-1 share: 2^256 / the algorithm's difficulty-1 target."""
    from otedama_amd.models.algorithms import ALGORITHMS

    return float(2 ** 256) / ALGORITHMS[algo].diff1


def measure_pool(gpus: int = 1, seconds: float = 30.0, share_seconds: float = 0.05, retarget_seconds: float = 5.0,
                 difficulty: float = 1.0, cpu: bool = False, startup_timeout: float = 180.0,
                 settle_timeout: float = 120.0, flood_seconds: float = 3.0) -> dict:
    streams = layout(gpus)
    algos = sorted({a for _, a in streams}, key=["sha256d", "scrypt"].index)
    http = f"127.0.0.1:{free_port()}"
    pool, addrs = spawn_mixed_pool(algos, difficulty, share_seconds, retarget_seconds, http)
    tmp = tempfile.mkdtemp(prefix="otedama-pool-")
    env = {k: v for k, v in os.environ.items() if k not in _DROP_ENV}
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    if cpu:
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    miners = []
    final: dict = {}
    t_open = time.monotonic()
    shared = len({g for g, _ in streams}) < len(streams)  # a GPU hosts two streams (one GPU: both algorithms)
    try:
        # On a shared GPU the scrypt stream starts first and the SHA-256d one once scrypt is hashing: started
        # together, SHA-256d has the GPU to itself for its first seconds (19.3 GH/s against ~13.9 shared), and those
        # shares sat in its vardiff estimate at settling, ~4% high (profiles/r6/i_pool_flow/). scrypt's own drop when
        # SHA-256d joins is 3.5x, which vardiff's rate-change test catches at its next look.
        order = sorted(streams, key=lambda s: s[1] != "scrypt") if shared else streams
        for i, (gpu, algo) in enumerate(order):
            if shared and i > 0 and algo != order[i - 1][1]:
                _wait_hashing(miners, 60.0)
            name = f"{'cpu' if cpu else 'gpu'}{gpu}-{algo}"
            cfg = os.path.join(tmp, f"{name}.yaml")
            with open(cfg, "w") as f:
                f.write(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addrs[algo]}\n"
                        "    target_grace: 10\n"  # otedama pool credits in-flight shares for RETARGET_GRACE
                        f"workers:\n  name: {name}\nmining:\n  algorithm: {algo}\n"
                        + ("  cpu_threads: 1\n  gpus: none\n" if cpu else f"  gpus: '{gpu}'\n"))
            rep = os.path.join(tmp, f"{name}.json")
            log = open(os.path.join(tmp, f"{name}.log"), "w")
            p = subprocess.Popen([sys.executable, "-m", "otedama_amd", "run", "--config", cfg, "--no-tui"],
                                 env=dict(env, OTEDAMA_NODE_REPORT=rep), cwd=ROOT, stdout=log,
                                 stderr=subprocess.STDOUT)
            miners.append({"name": name, "gpu": gpu, "algorithm": algo, "proc": p, "report": rep, "logf": log})
        end = time.monotonic() + startup_timeout
        while time.monotonic() < end:
            reps = [_read(m["report"]) for m in miners]
            if all(r.get("accepted", 0) > 0 for r in reps):
                break
            dead = [m["name"] for m in miners if m["proc"].poll() is not None]
            if dead:
                raise RuntimeError(f"miner(s) exited: {dead}")
            time.sleep(0.25)
        else:
            raise RuntimeError(f"miners not accepted within {startup_timeout:.0f} s")
        t_first = time.monotonic()
        # steady state: every worker connected and its vardiff settled (pool/vardiff.py: the
        # difficulty rests on most of a full estimator window, no refinement is left and no retarget is pending), and
        # the estimate it holds points within 10% of the difficulty in force
        def calm(w: dict) -> bool:
            r = w.get("window_ratio")
            return bool(w.get("settled")) and r is not None and abs(math.log(max(r, 1e-12))) < math.log(1.10)

        # CPU miners (the rehearsal) are too slow to fill vardiff's window: their settle wait is short, the window is
        # recorded with steady_state false
        end = time.monotonic() + (min(settle_timeout, 30.0) if cpu else settle_timeout)
        settled = False
        while time.monotonic() < end:
            ws = [w for s in _pool_api(http) for w in s.get("workers", [])]
            if len(ws) >= len(miners) and all(w["accepted"] > 0 and calm(w) for w in ws):
                settled = True
                break
            time.sleep(0.25)
        t_settled = time.monotonic()
        a0, t0 = {s["algorithm"]: s for s in _pool_api(http)}, time.monotonic()
        reps0 = {m["name"]: _read(m["report"]) for m in miners}
        time.sleep(seconds)
        a1, t1 = {s["algorithm"]: s for s in _pool_api(http)}, time.monotonic()
        reps1 = {m["name"]: _read(m["report"]) for m in miners}
        time.sleep(0.6)
        reps = {m["name"]: _read(m["report"]) for m in miners}
    finally:
        for m in miners:
            if m["proc"].poll() is None:
                m["proc"].send_signal(signal.SIGTERM)
        for m in miners:
            try:
                m["exit_code"] = m["proc"].wait(timeout=60)
            except subprocess.TimeoutExpired:
                m["proc"].kill()
                m["exit_code"] = m["proc"].wait()
            m["logf"].close()
        final = {s["algorithm"]: s for s in stop_pool_all(pool)}
    dt = t1 - t0
    out: dict = {}
    for algo in algos:
        s0, s1, fin = a0.get(algo, {}), a1.get(algo, {}), final.get(algo, {})
        acc = s1.get("accepted", 0) - s0.get("accepted", 0)
        rej = s1.get("rejected", 0) - s0.get("rejected", 0)
        ms = [m for m in miners if m["algorithm"] == algo]
        rates = {}
        for m in ms:
            r = window_rates(reps[m["name"]].get("samples", []), t0, t1 + 0.75)
            rates[m["name"]] = sum(r.values())
        # the miners' own share accounting over the window (found on the device, skipped by the engine, submitted,
        # accepted): where a gap between the hash rate's expected shares and the pool's accepted ones would come from
        flow = {}
        for m in ms:
            r0, r1 = reps0.get(m["name"], {}), reps1.get(m["name"], {})
            flow[m["name"]] = {k: (r1.get(k) or 0) - (r0.get(k) or 0)
                               for k in ("shares_found", "submitted", "accepted", "rejected", "stale_skipped",
                                         "below_target_skipped")}
        workers = []
        for w in s1.get("workers", []):
            got = sum(1 for v in s1.get("workers", []) if v["name"] == w["name"])
            prev = next((v for v in s0.get("workers", []) if v["name"] == w["name"]), {})
            n = w["accepted"] - prev.get("accepted", 0)
            interval = dt / n if n else None
            miner = next((k for k in flow if w["name"].endswith("." + k)), None)
            rate = rates.get(miner) if miner else None
            workers.append({"name": w["name"], "difficulty": w["difficulty"], "retargets": w["retargets"],
                            "miner_flow_in_window": flow.get(miner),
                            "shares_expected_from_rate": (rate * dt / (w["difficulty"] * _hashes_per_diff1(algo))
                                                          if rate and w["difficulty"] else None),
                            "retargets_in_window": w["retargets"] - prev.get("retargets", w["retargets"]),
                            "estimate_ratio_at_open": prev.get("window_ratio"),
                            "estimate_shares_at_open": prev.get("window_shares"),
                            "converged_after_s": w["converged_after_s"], "settled_after_s": w["settled_after_s"],
                            "window_opened_after_s": w.get("age_s", 0.0) - (t1 - t0),
                            "connections": got, "accepted_in_window": n,
                            "share_interval_s": interval,
                            "interval_vs_target": interval / share_seconds if interval else None})
        out[algo] = {
            "validated_shares_per_sec": acc / dt, "accepted": acc, "rejected": rej,
            "reject_reasons": fin.get("reject_reasons", {}), "accepted_total": fin.get("accepted"),
            "rejected_total": fin.get("rejected"),
            "validate_ms": _window_quantiles(fin.get("validate_log", []), t0, t1),
            "validate_ms_whole_run": fin.get("validate_ms"),
            "target_share_seconds": share_seconds, "workers": workers,
            "miner_hashes_per_sec": rates, "miners": [{"name": m["name"], "gpu": m["gpu"], "exit_code": m["exit_code"]}
                                                      for m in ms],
        }
    res = {"algorithms": out, "layout": [f"{'cpu' if cpu else 'gpu'}{g}:{a}" for g, a in streams],
           "recorded_seconds": dt, "initial_difficulty": difficulty, "retarget_seconds": retarget_seconds,
           "vardiff": True, "steady_state": settled, "time_to_first_accept_s": t_first - t_open,
           "time_to_steady_s": t_settled - t_open,
           "steady_rule": "every worker's vardiff settled (no refinement left, none pending) and its estimate within "
                          "10% of the difficulty in force",
           "definition": ("otedama pool --algorithms sha256d,scrypt (one process) + one `otedama run` per "
                          "(GPU, algorithm) stream over SV2; every accepted share re-hashed by the pool; window opened "
                          "once every worker's vardiff converged; validation quantiles over the window only")}
    if flood_seconds > 0:
        try:
            res["flood"] = flood(algos, seconds=flood_seconds)
        except Exception as exc:  # noqa: BLE001 - the flood figure is auxiliary
            res["flood"] = {"error": f"{type(exc).__name__}: {exc}"}
    return res
