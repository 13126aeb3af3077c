"""``otedama node`` end to end on the CPU (gloo ranks, one CPU miner each) against ``otedama pool`` in its own
process: the supervisor starts 3 ranks, rank 0 holds the SV2 session; a rank is SIGKILLed mid-job and the pool
keeps accepting shares from the survivors (no duplicate or stale rejects: the re-split never re-searches a
variant); the supervisor restarts the rank, which joins again; SIGTERM stops everything."""
import json
import os
import signal
import subprocess
import sys
import time
import urllib.request

import psutil
import pytest

from otedama_amd.engine.latency_probe import PROBE_ADDR, spawn_pool, stop_pool
from otedama_amd.parallel.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pool_stats(http):
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


def _wait(pred, timeout, step=0.2):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            if pred():
                return True
        except Exception:  # noqa: BLE001 - the pool's HTTP server may not be up yet
            pass
        time.sleep(step)
    return False


@pytest.mark.timeout(240)
def test_otedama_node_keeps_mining_through_a_rank_loss(tmp_path):
    http = f"127.0.0.1:{free_port()}"
    env = dict(os.environ, PYTHONPATH=ROOT)
    pool = subprocess.Popen([sys.executable, "-m", "otedama_amd", "pool", "--algorithms", "sha256d",
                             "--listen-sv2", "127.0.0.1:0", "--listen-v1=", "--difficulty", "0.0002", "--share-seconds", "0.05",
                             "--retarget-seconds", "3600", "--job-interval", "3600", "--block-interval", "3600",
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
    cfg.write_text(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addr}\nmining:\n  cpu_threads: 1\n")
    nenv = dict(env, OTEDAMA_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
                OTEDAMA_PG_TIMEOUT="20")
    sup = subprocess.Popen([sys.executable, "-m", "otedama_amd", "node", "--gpus", "3", "--config", str(cfg),
                            "--no-tui"], env=nenv, cwd=ROOT, stdout=open(tmp_path / "node.out", "w"),
                           stderr=subprocess.STDOUT)
    try:
        assert _wait(lambda: _pool_stats(http)["accepted"] >= 30, 120), (tmp_path / "node.out").read_text()[-4000:]
        ranks = _ranks(sup.pid)
        assert set(ranks) == {0, 1, 2}
        victim_pid = ranks[2].pid
        ranks[2].send_signal(signal.SIGKILL)
        a0 = _pool_stats(http)["accepted"]
        assert _wait(lambda: _pool_stats(http)["accepted"] >= a0 + 30, 30), (tmp_path / "node.out").read_text()[-4000:]
        # the supervisor restarts rank 2 and it is mining again
        assert _wait(lambda: 2 in _ranks(sup.pid) and _ranks(sup.pid)[2].pid != victim_pid, 30)
        assert _wait(lambda: "rank 2 joins" in (tmp_path / "node.out").read_text(), 40)
        a1 = _pool_stats(http)["accepted"]
        assert _wait(lambda: _pool_stats(http)["accepted"] >= a1 + 20, 40)
        st = _pool_stats(http)
        assert st["rejected"] == 0, st  # no duplicate / stale shares through the loss and the re-join
    finally:
        sup.send_signal(signal.SIGTERM)
        try:
            rc = sup.wait(timeout=40)
            assert rc == 0, (rc, (tmp_path / "node.out").read_text()[-3000:])  # a clean stop, like `otedama run`
            tail = (tmp_path / "node.out").read_text().split("stopping the node", 1)[-1]
            assert "lost" not in tail, tail[-3000:]  # followers leaving during the shutdown are not rank losses
        except subprocess.TimeoutExpired:
            for c in psutil.Process(sup.pid).children(recursive=True):
                c.kill()
            sup.kill()
            raise AssertionError("node did not stop within 40 s")
        finally:
            stop_pool(pool)
    assert not [p for p in psutil.pids() if p == victim_pid and psutil.Process(p).status() != psutil.STATUS_ZOMBIE]
