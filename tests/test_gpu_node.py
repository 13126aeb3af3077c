"""The production node on a real MI355X: ``otedama node --gpus 2`` (two gloo ranks sharing GPU 0, each with its miner
in a device process of its own) against ``otedama pool`` in its own process.

A GPU fault kills a device process, not the rank that owns the RCCL communicator and (rank 0) the pool session:
SIGKILLing rank 0's device child leaves rank 0 and its SV2 channel up (same process, same channel, no reconnect),
the follower keeps submitting through R2 meanwhile, and rank 0's own shares come back after the device process is
respawned. Shares from both ranks carry the kernel's hit time across the R2 gather."""
import json
import os
import signal
import subprocess
import sys
import time
import urllib.request

import psutil
import pytest

from otedama_amd.engine.latency_probe import PROBE_ADDR, stop_pool
from otedama_amd.parallel.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pool_stats(http):
    with urllib.request.urlopen(f"http://{http}/api/v1/pool", timeout=5) as r:
        return json.loads(r.read())[0]


def _report(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _wait(pred, timeout, step=0.1):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            v = pred()
            if v:
                return v
        except Exception:  # noqa: BLE001
            pass
        time.sleep(step)
    return None


def _rank(sup_pid, r):
    for c in psutil.Process(sup_pid).children():
        try:
            if c.environ().get("RANK") == str(r):
                return c
        except (psutil.NoSuchProcess, psutil.AccessDenied):
            pass
    return None


def _devproc(rank_proc):
    for c in rank_proc.children():
        try:
            if "otedama_amd.engine.devproc" in " ".join(c.cmdline()):
                return c
        except (psutil.NoSuchProcess, psutil.AccessDenied):
            pass
    return None


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_rank0_device_fault_keeps_the_pool_session(tmp_path):
    _device_fault_keeps_session(tmp_path, cpu=False)


@pytest.mark.timeout(240)
def test_rank0_device_fault_keeps_the_pool_session_cpu(tmp_path):
    """The same processes on a CPU host (gloo ranks, a CPU miner in each rank's device process)."""
    _device_fault_keeps_session(tmp_path, cpu=True)


def _device_fault_keeps_session(tmp_path, cpu: bool):
    http = f"127.0.0.1:{free_port()}"
    env = dict(os.environ, PYTHONPATH=ROOT)
    pool = subprocess.Popen([sys.executable, "-m", "otedama_amd", "pool", "--algorithms", "sha256d",
                             "--listen-sv2", "127.0.0.1:0", "--listen-v1=", "--difficulty", "0.002" if cpu else "0.5",
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
                   + ("mining:\n  cpu_threads: 1\n" if cpu else ""))
    report = tmp_path / "report.json"
    log = tmp_path / "node.out"
    nenv = dict(env, OTEDAMA_DIST_BACKEND="gloo", OTEDAMA_NODE_REPORT=str(report))
    if cpu:
        nenv.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    sup = subprocess.Popen([sys.executable, "-m", "otedama_amd", "node", "--gpus", "2", "--config", str(cfg),
                            "--no-tui"], env=nenv, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT)

    def accepts(rep, origin, since=0.0):
        return [a for a in rep.get("accept_log", []) if a[2] == origin and a[0] >= since]

    try:
        rep = _wait(lambda: (lambda r: r if len(accepts(r, "local")) >= 3 and len(accepts(r, "remote")) >= 3
                             else None)(_report(report)), 150)
        assert rep, log.read_text()[-5000:]
        if not cpu:  # remote shares carry the kernel's hit time across R2: device hit -> accept for both origins
            assert all(a[1] is not None for a in accepts(rep, "remote")), accepts(rep, "remote")[:5]
        r0 = _rank(sup.pid, 0)
        child = _devproc(r0)
        assert child is not None, [c.cmdline() for c in r0.children()]
        w0 = _pool_stats(http)["workers"]
        assert len(w0) == 1
        child.send_signal(signal.SIGKILL)
        t_kill = time.monotonic()
        # the follower keeps submitting through rank 0 while rank 0's device is down
        assert _wait(lambda: len(accepts(_report(report), "remote", t_kill)) >= 2, 30), log.read_text()[-4000:]
        # rank 0's device process is respawned and its shares flow again
        assert _wait(lambda: len(accepts(_report(report), "local", t_kill + 0.5)) >= 2, 60), log.read_text()[-4000:]
        new_child = _devproc(r0)
        assert new_child is not None and new_child.pid != child.pid
        # same rank-0 process, same pool channel: the session was never re-established
        assert _rank(sup.pid, 0).pid == r0.pid
        st = _pool_stats(http)
        assert len(st["workers"]) == 1 and st["workers"][0]["age_s"] > w0[0]["age_s"], (w0, st["workers"])
        assert st["clients_v2"] == 1 and st["rejected"] == 0, st
        assert _report(report).get("connected") is True
    finally:
        sup.send_signal(signal.SIGTERM)
        try:
            rc = sup.wait(timeout=60)
            assert rc == 0, (rc, log.read_text()[-3000:])
        except subprocess.TimeoutExpired:
            for c in psutil.Process(sup.pid).children(recursive=True):
                c.kill()
            sup.kill()
            raise AssertionError("node did not stop within 60 s")
        finally:
            stop_pool(pool)
