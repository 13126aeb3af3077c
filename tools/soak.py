"""Soak run of the production path on one GPU: the local validating pool (in this process) and `otedama run`
(a child process, native GPU miner) for a fixed time, with job refreshes and new blocks much more often than a
real pool sends them. Samples /metrics and the miner's RSS every --every seconds and prints one JSON line per
sample, then a summary line. Exits 1 if any share is rejected, a sample's hashrate falls below 90% of the
median after warm-up, or the miner's RSS (the engine alone, and the engine with its device processes) grows by
more than --max-rss-growth-mb.

python tools/soak.py [--seconds 180] [--protocol sv2|v1] [--algorithm sha256d]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import re
import signal
import statistics
import subprocess
import sys
import threading
import time
import urllib.request
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


def metric(body: str, name: str, labels: str = "") -> float:
    m = re.search(rf"^{re.escape(name)}{re.escape(labels)} (\S+)$", body, re.M)
    return float(m.group(1)) if m else 0.0


def rss_mb(pid: int) -> float:
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return int(line.split()[1]) / 1024.0
    except OSError:
        pass
    return 0.0


def proc_roles(pid: int) -> dict[int, tuple[str, float]]:
    """pid -> (role, RSS MB) for ``pid`` and its descendants: "supervisor"/"engine", "rank<r>", "devproc<r>"."""
    kids: dict[int, list[int]] = {}
    for d in os.listdir("/proc"):
        if d.isdigit():
            try:
                with open(f"/proc/{d}/stat") as f:
                    kids.setdefault(int(f.read().rsplit(")", 1)[1].split()[1]), []).append(int(d))
            except (OSError, IndexError, ValueError):
                continue
    out, todo = {}, [(pid, None)]
    while todo:
        p, parent_role = todo.pop()
        try:
            with open(f"/proc/{p}/cmdline", "rb") as f:
                cmd = f.read().replace(b"\0", b" ").decode(errors="replace")
            with open(f"/proc/{p}/environ", "rb") as f:
                env = dict(kv.split(b"=", 1) for kv in f.read().split(b"\0") if b"=" in kv)
        except OSError:
            continue
        rank = env.get(b"RANK", b"").decode()
        if "devproc" in cmd:
            role = "devproc" + (parent_role[4:] if parent_role and parent_role.startswith("rank") else "")
        elif parent_role is None:
            role = "top"
        elif " run " in cmd + " " and rank:
            role = f"rank{rank}"
        else:
            role = "other"
        out[p] = (role, rss_mb(p))
        todo += [(c, role) for c in kids.get(p, [])]
    return out


def tree_rss_mb(pid: int) -> tuple[float, float]:
    """(RSS of pid and all its descendants, RSS of the descendants): the engine keeps its GPUs in device processes."""
    kids: dict[int, list[int]] = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                ppid = int(f.read().rsplit(")", 1)[1].split()[1])
        except (OSError, IndexError, ValueError):
            continue
        kids.setdefault(ppid, []).append(int(d))
    todo, desc = list(kids.get(pid, [])), []
    while todo:
        c = todo.pop()
        desc.append(c)
        todo += kids.get(c, [])
    child = sum(rss_mb(c) for c in desc)
    return rss_mb(pid) + child, child


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--every", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=30.0)
    ap.add_argument("--protocol", choices=("sv2", "v1"), default="sv2")
    ap.add_argument("--algorithm", default="sha256d")
    ap.add_argument("--difficulty", type=float, default=2.0)
    ap.add_argument("--job-interval", type=float, default=5.0)
    ap.add_argument("--block-interval", type=float, default=45.0)
    ap.add_argument("--share-seconds", type=float, default=1.0, help="the pool's vardiff target share interval")
    ap.add_argument("--max-rss-growth-mb", type=float, default=64.0)
    ap.add_argument("--workdir", default="gpurun_out/soak")
    ap.add_argument("--bounce-at", type=float, default=0.0,
                    help="stop the pool this many seconds in, restart it on the same ports after --bounce-down s "
                         "(the engine must reconnect and resume; samples within 20 s after it skip the rate check)")
    ap.add_argument("--bounce-down", type=float, default=3.0)
    ap.add_argument("--node", type=int, default=0,
                    help="run `otedama node --gpus N` over gloo (ranks share the GPU) instead of `otedama run`")
    ap.add_argument("--extended", action="store_true", help="SV2 extended channel (miner-side extranonce rolling)")
    ap.add_argument("--noise", choices=("", "ellswift", "legacy"), default="",
                    help="SV2 Noise NX with this suite, pinned to the pool's authority key")
    a = ap.parse_args()

    from otedama_amd.pool.server import PoolOptions, PoolServer

    work = Path(a.workdir)
    work.mkdir(parents=True, exist_ok=True)
    if a.bounce_at and a.noise:
        raise SystemExit("soak: --bounce-at with --noise is not supported (a restarted pool has a new authority key)")

    def make_pool(sv2="127.0.0.1:0", v1="127.0.0.1:0"):
        return PoolServer(PoolOptions(algorithm=a.algorithm, initial_difficulty=a.difficulty, payout_address=ADDR,
                                      target_share_seconds=a.share_seconds, retarget_seconds=15.0, job_interval=a.job_interval,
                                      block_interval=a.block_interval, noise=bool(a.noise), noise_suite=a.noise,
                                      listen_sv2=sv2, listen_v1=v1))

    pool = make_pool()
    loop = asyncio.new_event_loop()
    ready = threading.Event()

    def serve():
        asyncio.set_event_loop(loop)
        loop.run_until_complete(pool.start())
        ready.set()
        loop.run_forever()

    threading.Thread(target=serve, daemon=True).start()
    if not ready.wait(30):
        print(json.dumps({"error": "pool did not start"}))
        return 1
    url = f"stratum+v2://{pool.addr_sv2}" if a.protocol == "sv2" else f"stratum+tcp://{pool.addr_v1}"
    cfg = work / "config.yaml"
    extra = ""
    if a.extended:
        extra += "    sv2_extended_channel: true\n"
    if a.noise:
        extra += f"    noise_suite: {a.noise}\n    pool_pubkey: \"{pool.noise_authority_pub.hex()}\"\n"
    cfg.write_text(f"bitcoin_address: {ADDR}\npools:\n  - url: {url}\n{extra}mining:\n  algorithm: {a.algorithm}\n")
    env = dict(os.environ, HOME=str(work), PYTHONPATH=str(ROOT), OTEDAMA_DATA_DIR=str(work / "data"))
    log = open(work / "miner.log", "w")
    if a.node:
        env["OTEDAMA_DIST_BACKEND"] = "gloo"
        cmd = [sys.executable, "-u", "-m", "otedama_amd", "node", "--gpus", str(a.node), "--config", str(cfg),
               "--no-tui", "--http-addr", "127.0.0.1:0"]
    else:
        cmd = [sys.executable, "-u", "-m", "otedama_amd", "run", "--config", str(cfg), "--no-tui",
               "--http-addr", "127.0.0.1:0", "--gpus", "0"]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
    http = None
    t_start = time.time()
    while time.time() - t_start < 120 and http is None:
        line = proc.stdout.readline()
        if not line:
            break
        log.write(line)
        m = re.search(r"http: listening on (\S+)", line)
        if m:
            http = m.group(1)
    threading.Thread(target=lambda: [log.write(x) for x in proc.stdout], daemon=True).start()
    samples, rc = [], 0
    bounce = None
    try:
        if http is None:
            print(json.dumps({"error": "miner did not start", "log": str(work / "miner.log")}))
            return 1
        t0 = time.time()
        base_acc = base_rej = 0.0  # pool counters of the pools before a bounce
        first_roles = last_roles = None  # per-process RSS at the first steady sample and at the end
        while time.time() - t0 < a.seconds:
            time.sleep(a.every)
            if a.bounce_at and bounce is None and time.time() - t0 >= a.bounce_at:
                acc_before = metric(urllib.request.urlopen(f"http://{http}/metrics", timeout=5).read().decode(),
                                    "otedama_shares_total", '{status="accepted"}')
                base_acc, base_rej = base_acc + pool.m_accepted.value(), base_rej + pool.m_rejected.value()
                addrs = (pool.addr_sv2, pool.addr_v1)
                asyncio.run_coroutine_threadsafe(pool.stop(), loop).result(30)
                t_down = time.time()
                time.sleep(a.bounce_down)
                pool = make_pool(*addrs)
                asyncio.run_coroutine_threadsafe(pool.start(), loop).result(30)
                t_up = time.time()
                first = None
                while time.time() - t_up < 90 and first is None:
                    time.sleep(0.2)
                    if pool.m_accepted.value() > 0:
                        first = time.time() - t_up
                bounce = {"t": round(t_down - t0, 1), "down_s": round(t_up - t_down, 2), "accepted_before": acc_before,
                          "first_accept_after_restart_s": round(first, 2) if first is not None else None}
                print(json.dumps({"bounce": bounce}), flush=True)
            if proc.poll() is not None:
                print(json.dumps({"error": f"miner exited with {proc.returncode}"}), flush=True)
                return 1
            with urllib.request.urlopen(f"http://{http}/metrics", timeout=5) as r:
                body = r.read().decode()
            s = {"t": round(time.time() - t0, 1),
                 "hashrate_ghs": round(metric(body, "otedama_hashrate_hashes_per_second") / 1e9, 6),
                 "accepted": metric(body, "otedama_shares_total", '{status="accepted"}'),
                 "rejected": metric(body, "otedama_shares_total", '{status="rejected"}'),
                 "p50_submit_ms": metric(body, "otedama_submit_latency_milliseconds", '{quantile="0.5"}'),
                 "pool_accepted": base_acc + pool.m_accepted.value(), "pool_rejected": base_rej + pool.m_rejected.value(),
                 "blocks": pool.m_blocks.value() if hasattr(pool, "m_blocks") else None,
                 "rss_mb": round(rss_mb(proc.pid), 1)}
            tree, child = tree_rss_mb(proc.pid)
            s["tree_rss_mb"], s["device_procs_rss_mb"] = round(tree, 1), round(child, 1)
            roles = proc_roles(proc.pid)
            s["rss_by_process_mb"] = {f"{r}:{p}": round(m, 1) for p, (r, m) in sorted(roles.items())}
            if first_roles is None and s["t"] >= a.warmup:
                first_roles = roles
            last_roles = roles
            samples.append(s)
            print(json.dumps(s), flush=True)
    finally:
        proc.send_signal(signal.SIGTERM)
        try:
            exit_code = proc.wait(60)
        except subprocess.TimeoutExpired:
            proc.kill()
            exit_code = proc.wait(10)
        asyncio.run_coroutine_threadsafe(pool.stop(), loop).result(30)
        loop.call_soon_threadsafe(loop.stop)
        log.close()
    steady = [s for s in samples if s["t"] >= a.warmup
              and not (bounce is not None and bounce["t"] <= s["t"] <= bounce["t"] + a.bounce_down + 20.0)] or samples
    rates = [s["hashrate_ghs"] for s in steady]
    med = statistics.median(rates) if rates else 0.0
    rss0 = steady[0]["rss_mb"] if steady else 0.0
    last = samples[-1] if samples else {}
    summary = {"summary": True, "seconds": a.seconds, "protocol": a.protocol, "algorithm": a.algorithm,
               "extended_channel": a.extended, "noise": a.noise or None, "bounce": bounce, "node_ranks": a.node or None,
               "median_hashrate_ghs": med, "min_hashrate_ghs": min(rates) if rates else 0.0,
               "accepted": last.get("accepted"), "rejected": last.get("rejected"),
               "pool_accepted": last.get("pool_accepted"), "pool_rejected": last.get("pool_rejected"),
               "blocks": last.get("blocks"), "rss_growth_mb": round((last.get("rss_mb") or 0.0) - rss0, 1),
               "tree_rss_growth_mb": round((last.get("tree_rss_mb") or 0.0) - (steady[0].get("tree_rss_mb") or 0.0
                                                                                if steady else 0.0), 1),
               "miner_exit_code": exit_code}
    if first_roles and last_roles:  # RSS growth per process over the steady window, by role
        summary["rss_growth_by_process_mb"] = {
            f"{last_roles[p][0]}:{p}": round(last_roles[p][1] - first_roles[p][1], 1)
            for p in sorted(last_roles, key=lambda q: last_roles[q][0]) if p in first_roles}
    ok = (rates and min(rates) >= 0.9 * med and (not a.bounce_at or (bounce or {}).get("first_accept_after_restart_s")) and not last.get("rejected") and not last.get("pool_rejected")
          and summary["rss_growth_mb"] <= a.max_rss_growth_mb and summary["tree_rss_growth_mb"] <= a.max_rss_growth_mb
          and exit_code == 0)
    summary["ok"] = bool(ok)
    print(json.dumps(summary), flush=True)
    return 0 if ok and rc == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
