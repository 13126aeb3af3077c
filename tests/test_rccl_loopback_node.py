"""``otedama node`` on the native data plane's code path at world 4 and 8, rehearsed on CPUs.

On GPUs every rank runs parallel/rcclcomm.py over ``otedama_amd._rccl``. RCCL refuses two ranks on one GPU, so the
one-GPU box can run that path only at world 1. Here the ranks load tests/loopback_rccl.py instead
(``OTEDAMA_RCCL_MODULE``): the same module API, the collectives carried by the node's store. Everything else is the
production code of a GPU node: the unique id published per generation through the store, the all-ranks-together
choice recorded at ``otd/comm``, torch never imported by a rank, timeouts turned into CollectiveTimeout, ``abort`` and
a new generation after a follower is SIGKILLed, and the leader's take-over after rank 0 is SIGKILLed. The pool
re-hashes every share and must reject none (nothing searched twice, nothing stale).
Reference: the engine restarts a failed worker without stopping the others (internal/engine/run.go:368-521).
"""
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


def _ranks(sup_pid):
    out = {}
    for c in psutil.Process(sup_pid).children():
        try:
            out[int(c.environ().get("RANK", "-1"))] = c
        except (psutil.NoSuchProcess, psutil.AccessDenied, ValueError):
            pass
    return out


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
        except Exception:  # noqa: BLE001 - files / HTTP not up yet
            pass
        time.sleep(step)
    return None


def _remote(rep, since=0.0):
    return sum(1 for t, _ms, origin, *_ in rep.get("accept_log", []) if origin == "remote" and t >= since)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [4, 8])
def test_native_path_node_survives_a_follower_and_a_leader_loss(tmp_path, world):
    http = f"127.0.0.1:{free_port()}"
    env = dict(os.environ, PYTHONPATH=ROOT)
    pool = subprocess.Popen([sys.executable, "-m", "otedama_amd", "pool", "--algorithms", "sha256d",
                             "--listen-sv2", "127.0.0.1:0", "--listen-v1=", "--difficulty", "0.001",
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
    cfg.write_text(f"bitcoin_address: {PROBE_ADDR}\npools:\n  - url: stratum+v2://{addr}\nmining:\n  cpu_threads: 1\n")
    report = tmp_path / "report.json"
    nenv = dict(env, PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]), OTEDAMA_NODE_COMM="native",
                OTEDAMA_RCCL_MODULE="loopback_rccl", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
                OTEDAMA_PG_TIMEOUT="20", OTEDAMA_NODE_REPORT=str(report))
    nenv.pop("OTEDAMA_DIST_BACKEND", None)
    log = tmp_path / "node.out"
    api = f"127.0.0.1:{free_port()}"
    sup = subprocess.Popen([sys.executable, "-m", "otedama_amd", "node", "--gpus", str(world), "--config", str(cfg),
                            "--no-tui", "--http-addr", api], env=nenv, cwd=ROOT, stdout=open(log, "w"),
                           stderr=subprocess.STDOUT)
    try:
        # every follower's shares cross R2 on the native path's collectives
        first = _wait(lambda: (lambda r: r if _remote(r) >= world and r.get("world") == world else None)(
            _report(report)), 150)
        assert first, log.read_text()[-4000:]
        out = log.read_text()
        assert "native RCCL unavailable" not in out, out[-4000:]
        assert f"{world} ranks over rccl" in out, out[-4000:]
        ranks = _ranks(sup.pid)
        assert set(ranks) == set(range(world))
        for r, p in ranks.items():  # a native rank never loads torch (start-up and RSS)
            maps = open(f"/proc/{p.pid}/maps").read()
            assert "libtorch" not in maps, f"rank {r} mapped libtorch"
        # the leader's view over HTTP: every rank a member of generation 0 on the native data plane, heartbeating
        with urllib.request.urlopen(f"http://{api}/api/v1/node", timeout=5) as resp:
            st = json.loads(resp.read())
        assert st["world"] == world and st["backend"] == "rccl" and st["members"] == list(range(world)), st
        assert set(st["ranks"]) == {f"rank{r}" for r in range(world)}, st
        assert all(v["heartbeat_age_s"] < 2.0 and v["member"] for k, v in st["ranks"].items() if k != "rank0"), st
        assert st["share_previews"] > 0 and st["remote_stale"] == 0, st
        res = subprocess.run([sys.executable, "-m", "otedama_amd", "node", "status", "--http-addr", api],
                             capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
        assert res.returncode == 0, res.stderr
        assert f"node: {world} ranks over rccl, generation 0" in res.stdout, res.stdout
        assert all(f"rank{r}" in res.stdout for r in range(world)) and "total" in res.stdout, res.stdout

        # a follower lost: the leader's collective times out, it aborts and re-forms (without it, or with the
        # supervisor's replacement when that is already back); the replacement is a member of a later generation
        victim = world - 1
        gen0 = _report(report).get("generation", 0)
        ranks[victim].send_signal(signal.SIGKILL)
        t_kill = time.monotonic()  # the accept log's clock (CLOCK_MONOTONIC is system-wide)
        a0 = _pool_stats(http)["accepted"]
        rep = _wait(lambda: (lambda r: r if r.get("generation", 0) > gen0 and sorted(r.get("members", [])) ==
                             list(range(world)) and _remote(r, t_kill) >= 3 else None)(_report(report)), 120)
        assert rep, log.read_text()[-4000:]
        new_victim = _ranks(sup.pid).get(victim)
        assert new_victim is not None and new_victim.pid != ranks[victim].pid
        # seen by a native op's deadline (CollectiveTimeout) or first by the supervisor's mark, whichever won
        out = log.read_text()
        assert "collective failed (CollectiveTimeout" in out or f"rank {victim} lost" in out, out[-4000:]
        assert _wait(lambda: _pool_stats(http)["accepted"] >= a0 + 3 * world, 90), log.read_text()[-4000:]

        # the leader lost: the supervisor restarts rank 0, which takes the node over (next generation, every live
        # follower) and the followers' shares flow again
        old = _ranks(sup.pid)[0]
        old.send_signal(signal.SIGKILL)
        new = _wait(lambda: (lambda p: p if p is not None and p.pid != old.pid else None)(_ranks(sup.pid).get(0)), 30)
        assert new, log.read_text()[-4000:]
        rep = _wait(lambda: (lambda r: r if r.get("pid") == new.pid and r.get("world") == world
                             and _remote(r) >= 3 else None)(_report(report)), 120)
        assert rep, log.read_text()[-6000:]
        assert rep["leader_incarnation"] == 2 and sorted(rep["members"]) == list(range(world)), rep
        st = _pool_stats(http)
        assert st["rejected"] == 0, st  # no duplicate or stale share through either loss
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


def test_loopback_module_collectives_and_timeouts(monkeypatch):
    """The stand-in itself: RCCL's results for every op at world 3, a deadline when a member never enters the op,
    and an aborted communicator refusing further ops."""
    import threading

    import numpy as np

    import loopback_rccl as lb
    from otedama_amd.parallel.kvstore import StoreServer

    with StoreServer() as srv:
        monkeypatch.setenv("MASTER_PORT", str(srv.port))
        uid = lb.unique_id()
        comms, errs = [None] * 3, []

        def make(r):
            try:
                comms[r] = lb.RcclComm(0, 3, r, uid, 10.0)
            except Exception as exc:  # noqa: BLE001
                errs.append(exc)

        ts = [threading.Thread(target=make, args=(r,)) for r in range(3)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert not errs and all(comms)
        res = [None] * 3

        def ops(r):
            c = comms[r]
            b = c.broadcast(b"job!" if r == 0 else b"", 4, 0, 5.0)
            g = c.all_gather(np.array([r, 10 * r], dtype=np.int64).tobytes(), 5.0)
            s = c.all_reduce(np.array([r + 1], dtype=np.int64).tobytes(), "i64", "sum", 5.0)
            m = c.all_reduce(np.array([r * 0.5], dtype=np.float64).tobytes(), "f64", "max", 5.0)
            res[r] = (b, np.frombuffer(g, dtype=np.int64).tolist(), np.frombuffer(s, dtype=np.int64)[0],
                      np.frombuffer(m, dtype=np.float64)[0])

        ts = [threading.Thread(target=ops, args=(r,)) for r in range(3)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert all(x == (b"job!", [0, 0, 1, 10, 2, 20], 6, 1.0) for x in res), res
        assert comms[0].ops == 4
        t0 = time.monotonic()
        with pytest.raises(TimeoutError):  # ranks 1 and 2 never enter: a dead peer
            comms[0].all_gather(b"x" * 8, 0.3)
        assert time.monotonic() - t0 < 2.0
        with pytest.raises(RuntimeError, match="timed out"):  # broken until aborted, as the native module
            comms[0].all_gather(b"x" * 8, 0.3)
        comms[0].abort()
        assert not comms[0].alive
        with pytest.raises(RuntimeError):
            comms[0].broadcast(b"1234", 4, 0, 1.0)
        for c in comms[1:]:
            c.abort()
