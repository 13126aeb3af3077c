"""``otedama node`` mining X11 and scrypt (BASELINE config 4: "X11 ... nonce ranges partitioned").

The same production processes as the GPU node, rehearsed on the CPU: the supervisor, N gloo ranks, each rank's miner
in a device process of its own (the native CPU miner running the host X11 / scrypt chains), rank 0 holding the SV2
session with `otedama pool --algorithms <algo>` in its own process. Every rank must get shares accepted (its variant
stripe is searched and its shares cross R2), a follower SIGKILLed mid-run must be re-split around (the pool keeps
accepting with no duplicate: nothing is searched twice) and rejoin after the supervisor restarts it, and every share
the pool validates is re-hashed with that algorithm. Reference: every device worker gets the same set-up path whatever
its device (internal/engine/setup.go:59-77).
"""
import json
import os
import signal
import subprocess
import sys
import time

import psutil
import pytest

from otedama_amd.engine.latency_probe import PROBE_ADDR, stop_pool
from otedama_amd.parallel.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# difficulty for ~3 shares/s per rank on one CPU thread (node_probe.EXPECTED_RATE["cpu"]; x11 diff1 = 2^32 hashes,
# scrypt diff1 = 2^16 hashes)
DIFFICULTY = {"x11": 4e3 / (3 * 2.0 ** 32), "scrypt": 1.2e4 / (3 * 2.0 ** 16)}


def _pool_stats(http):
    import urllib.request

    with urllib.request.urlopen(f"http://{http}/api/v1/pool", timeout=5) as r:
        return json.loads(r.read())[0]


def _ranks(sup_pid):
    out = {}
    for c in psutil.Process(sup_pid).children():
        try:
            out[int(c.environ().get("RANK", "-1"))] = c
        except (psutil.NoSuchProcess, psutil.AccessDenied, ValueError):
            pass
    return out


def _wait(pred, timeout, step=0.25):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            if pred():
                return True
        except Exception:  # noqa: BLE001 - files / HTTP not up yet
            pass
        time.sleep(step)
    return False


def _accepted_by_rank(report) -> dict:
    try:
        with open(report) as f:
            rep = json.load(f)
    except (OSError, ValueError):
        return {}
    out: dict = {}
    for a in rep.get("accept_log", []):
        dev = a[3] if len(a) > 3 else ""
        key = dev if str(dev).startswith("rank") else "rank0"
        out[key] = out.get(key, 0) + 1
    return out


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("algo", ["x11", "scrypt"])
def test_node_mines_the_algorithm_on_every_rank_through_a_follower_loss(tmp_path, algo, world):
    http = f"127.0.0.1:{free_port()}"
    env = dict(os.environ, PYTHONPATH=ROOT)
    pool = subprocess.Popen([sys.executable, "-m", "otedama_amd", "pool", "--algorithms", algo,
                             "--listen-sv2", "127.0.0.1:0", "--listen-v1=", "--difficulty", repr(DIFFICULTY[algo]),
                             "--fixed-difficulty", "--job-interval", "3600", "--block-interval", "3600",
                             "--http-addr", http, "--payout-address", PROBE_ADDR],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
    addr = None
    for _ in range(200):
        line = pool.stdout.readline()
        if "listening sv2=" in line:
            addr = line.split("listening sv2=", 1)[1].split()[0]
            break
    assert addr, "pool did not start"
    cfg = tmp_path / "config.yaml"
    cfg.write_text(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addr}\n"
                   f"mining:\n  algorithm: {algo}\n  cpu_threads: 1\n")
    report = str(tmp_path / "report.json")
    nenv = dict(env, OTEDAMA_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
                OTEDAMA_PG_TIMEOUT="20", OTEDAMA_NODE_REPORT=report)
    log = tmp_path / "node.out"
    sup = subprocess.Popen([sys.executable, "-m", "otedama_amd", "node", "--gpus", str(world), "--config", str(cfg),
                            "--no-tui"], env=nenv, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT)
    try:
        # every rank's shares accepted: its stripe of the variant space is mined and its shares cross R2
        assert _wait(lambda: len(_accepted_by_rank(report)) == world, 180), (
            _accepted_by_rank(report), log.read_text()[-3000:])
        ranks = _ranks(sup.pid)
        assert set(ranks) == set(range(world))
        victim = world - 1
        victim_pid = ranks[victim].pid
        ranks[victim].send_signal(signal.SIGKILL)
        a0 = _pool_stats(http)["accepted"]
        assert _wait(lambda: _pool_stats(http)["accepted"] >= a0 + 3 * world, 90), log.read_text()[-3000:]
        assert _wait(lambda: f"rank {victim} joins" in log.read_text(), 90), log.read_text()[-3000:]
        st = _pool_stats(http)
        assert st["algorithm"] == algo and st["rejected"] == 0, st  # no duplicate or stale share through the loss
    finally:
        sup.send_signal(signal.SIGTERM)
        try:
            rc = sup.wait(timeout=60)
        except subprocess.TimeoutExpired:
            for c in psutil.Process(sup.pid).children(recursive=True):
                c.kill()
            sup.kill()
            rc = "timeout"
        pst = stop_pool(pool)
    assert rc == 0, (rc, log.read_text()[-3000:])
    assert pst["accepted"] > 0 and pst["rejected"] == 0, pst
    assert not [p for p in psutil.pids() if p == victim_pid and psutil.Process(p).status() != psutil.STATUS_ZOMBIE]
