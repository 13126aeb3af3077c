"""GPU-box rehearsal of the production entry points on one MI355X.

1. ``otedama run`` (one device process per GPU, the engine GPU-free) against ``otedama pool`` in another process:
   process start -> first completed GPU batch, resident set of the engine and of the device process, hashrate.
2. ``otedama node --gpus 2`` with ``OTEDAMA_DIST_BACKEND=gloo``: two ranks sharing the one GPU, the same op-log /
   heartbeat control plane as the RCCL node: node hashrate vs 1., and the device collectives per second.

Prints one JSON line; every number is read from the running processes (/debug/stats, /api/v1/stats, psutil).
Usage: python tools/gpu_node_rehearsal.py [--seconds 25]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _get(url: str):
    with urllib.request.urlopen(url, timeout=5) as r:
        return json.loads(r.read())


def _wait(pred, timeout, step=0.02):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            v = pred()
            if v:
                return v
        except Exception:  # noqa: BLE001 - the HTTP server is not up yet
            pass
        time.sleep(step)
    return None


def _hashes(http: str) -> int:
    st = _get(f"http://{http}/debug/stats")
    return sum(int(d.get("hashes", 0)) for d in st["devices"].values())


def _sample(http: str) -> dict:
    """{device: (hashes, when counted)}: a remote rank's counters carry the time its heartbeat was written, so the
    rate over a window is exact instead of off by up to one heartbeat period at each end."""
    now = time.time()
    st = _get(f"http://{http}/debug/stats")
    # the device-timeline completion time of the counted launches makes the window exact (counter moves come in
    # whole 2^32-hash launches); else when the counters were taken
    return {k: (int(d.get("hashes", 0)), float(d.get("hashes_done_at_s") or d.get("counted_at") or now))
            for k, d in st["devices"].items()}


def _rate(a: dict, b: dict) -> float:
    total = 0.0
    for k, (h1, t1) in b.items():
        h0, t0 = a.get(k, (0, t1))
        if t1 > t0:
            total += (h1 - h0) / (t1 - t0)
    return total


def _rss_top(pid: int, n: int = 8) -> list:
    """The process's largest resident mappings (MiB, path or [anon]) from /proc/<pid>/smaps."""
    sizes: dict[str, float] = {}
    name = "?"
    try:
        with open(f"/proc/{pid}/smaps") as f:
            for line in f:
                parts = line.split()
                if parts and "-" in parts[0] and len(parts) >= 5:
                    name = parts[5] if len(parts) >= 6 else "[anon]"
                elif parts and parts[0] == "Rss:":
                    sizes[name] = sizes.get(name, 0.0) + int(parts[1]) / 1024
    except OSError as exc:
        return [str(exc)]
    return [(k, round(v, 1)) for k, v in sorted(sizes.items(), key=lambda kv: -kv[1])[:n]]


def _measure_pair(cmds: list[list[str]], https: list[str], env: dict, seconds: float, log_dir: str) -> dict:
    """Two independent `otedama run` processes sharing the one GPU: the fair baseline for a 2-rank node on this
    1-GPU box (two processes' hardware queues time-share the GPU either way); their rates are summed."""
    procs = [subprocess.Popen(c, env=env, cwd=ROOT, stdout=open(os.path.join(log_dir, f"pair{i}.log"), "w"),
                              stderr=subprocess.STDOUT) for i, c in enumerate(cmds)]
    out: dict = {}
    try:
        for h in https:
            _wait(lambda h=h: _hashes(h) > 0, 120)
        time.sleep(5.0)
        s0 = [_sample(h) for h in https]
        time.sleep(seconds)
        s1 = [_sample(h) for h in https]
        out["hashrates"] = [_rate(a, b) for a, b in zip(s0, s1)]
        out["hashrate"] = sum(out["hashrates"])
    finally:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()
    return out


def _measure(cmd: list[str], http: str, env: dict, seconds: float, log_path: str) -> dict:
    t_spawn = time.time()
    p = subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=open(log_path, "w"), stderr=subprocess.STDOUT)
    out: dict = {}
    try:
        first = _wait(lambda: _hashes(http) > 0 and time.time(), 120)
        out["spawn_to_first_hash_s"] = (first - t_spawn) if first else None
        st = _wait(lambda: _get(f"http://{http}/debug/stats"), 10)
        out["startup"] = (st or {}).get("startup")
        time.sleep(5.0)  # past the first job's start-up transients
        s0 = _sample(http)
        time.sleep(seconds)
        out["hashrate"] = _rate(s0, _sample(http))
        dbg = _get(f"http://{http}/debug/stats")
        out["node"] = dbg.get("node")
        out["startup"] = dbg.get("startup") or out["startup"]
        try:
            import psutil

            pp = psutil.Process(p.pid)
            out["rss_mib"] = {str(c.pid): round(c.memory_info().rss / 2**20, 1)
                              for c in [pp, *pp.children(recursive=True)]}
            out["rss_top_mappings"] = {str(c.pid): _rss_top(c.pid) for c in [pp, *pp.children(recursive=True)]}
        except Exception as exc:  # noqa: BLE001
            out["rss_mib"] = str(exc)
    finally:
        p.send_signal(signal.SIGTERM)
        try:
            out["exit_code"] = p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            out["exit_code"] = "killed"
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--out-dir", default=os.path.join(ROOT, "gpurun_out", "node_rehearsal"))
    ap.add_argument("--run-only", action="store_true", help="measure `otedama run` only (no node rehearsal)")
    a = ap.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    from otedama_amd.engine.latency_probe import PROBE_ADDR
    from otedama_amd.parallel.launch import free_port

    env = dict(os.environ, PYTHONPATH=ROOT)
    pool_http = f"127.0.0.1:{free_port()}"
    pool = subprocess.Popen([sys.executable, "-m", "otedama_amd", "pool", "--algorithms", "sha256d",
                             "--listen-sv2", "127.0.0.1:0", "--listen-v1=", "--difficulty", "4",
                             "--share-seconds", "1000", "--retarget-seconds", "3600", "--job-interval", "3600",
                             "--block-interval", "3600", "--http-addr", pool_http, "--payout-address", PROBE_ADDR],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
    addr = None
    for _ in range(400):
        line = pool.stdout.readline()
        if "listening sv2=" in line:
            addr = line.split("listening sv2=", 1)[1].split()[0]
            break
    if not addr:
        print(json.dumps({"error": "pool did not start"}))
        return 1
    cfg = os.path.join(a.out_dir, "config.yaml")
    with open(cfg, "w") as f:
        f.write(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addr}\n")
    res = {}
    try:
        http1 = f"127.0.0.1:{free_port()}"
        res["run"] = _measure([sys.executable, "-m", "otedama_amd", "run", "--config", cfg, "--no-tui",
                               "--http-addr", http1], http1, env, a.seconds, os.path.join(a.out_dir, "run.log"))
        if a.run_only:
            print(json.dumps(res))
            return 0
        http2 = f"127.0.0.1:{free_port()}"
        res["node_gloo_2ranks_shared_gpu"] = _measure(
            [sys.executable, "-m", "otedama_amd", "node", "--gpus", "2", "--config", cfg, "--no-tui", "--http-addr",
             http2], http2, dict(env, OTEDAMA_DIST_BACKEND="gloo"), a.seconds, os.path.join(a.out_dir, "node.log"))
        r, n = res["run"].get("hashrate"), res["node_gloo_2ranks_shared_gpu"].get("hashrate")
        res["node_vs_run"] = (n / r) if r and n else None
        https = [f"127.0.0.1:{free_port()}" for _ in range(2)]
        res["two_runs_shared_gpu"] = _measure_pair(
            [[sys.executable, "-m", "otedama_amd", "run", "--config", cfg, "--no-tui", "--http-addr", h] for h in https],
            https, env, a.seconds, a.out_dir)
        p2 = res["two_runs_shared_gpu"].get("hashrate")
        # the control plane's own cost: node vs the same two processes sharing the GPU without it
        res["node_vs_two_runs"] = (n / p2) if p2 and n else None
        res["pool"] = _get(f"http://{pool_http}/api/v1/pool")
    finally:
        pool.send_signal(signal.SIGTERM)
        try:
            pool.wait(timeout=30)
        except subprocess.TimeoutExpired:
            pool.kill()
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
