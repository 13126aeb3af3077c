"""The node's native RCCL data plane (parallel/rcclcomm.py, csrc/runtime/rccl_comm.cpp).

GPU tests (one MI355X): the module's collectives at world 1, NativeNodeComm through a store over generations, and
a rank process that never imports torch. CPU tests: the choice of implementation and the all-ranks-together
fallback to torch.distributed when the native group cannot form (here: no GPU, OTEDAMA_NODE_COMM=native forces the
attempt), through `otedama node` end to end.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_wanted_rules(monkeypatch):
    from otedama_amd.parallel import rcclcomm

    monkeypatch.setenv("OTEDAMA_NODE_COMM", "torch")
    assert not rcclcomm.native_wanted()
    monkeypatch.setenv("OTEDAMA_NODE_COMM", "native")
    assert rcclcomm.native_wanted()
    monkeypatch.delenv("OTEDAMA_NODE_COMM")
    monkeypatch.setenv("OTEDAMA_DIST_BACKEND", "gloo")
    assert not rcclcomm.native_wanted()  # a gloo rehearsal stays on torch.distributed
    monkeypatch.delenv("OTEDAMA_DIST_BACKEND")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert not rcclcomm.native_wanted()  # no visible GPU


@pytest.mark.timeout(300)
def test_node_falls_back_to_torch_together_when_native_cannot_form():
    """Every rank attempts the native group (forced on a CPU host, where it cannot form), reports, and all of them
    continue on torch.distributed: the node mines, remote shares are accepted, and the choice is logged."""
    from otedama_amd.parallel.node_probe import measure_node

    os.environ["OTEDAMA_NODE_COMM"] = "native"
    try:
        r = measure_node(2, seconds=2, warmup=1, cpu=True, algorithm="sha256d", switches=0)
    finally:
        del os.environ["OTEDAMA_NODE_COMM"]
    log = open(r["log"]).read()
    assert "native RCCL unavailable on rank(s) [0, 1]" in log, log[-3000:]
    assert r["dist_backend"] == "gloo" and r["ranks_seen"] == [0, 1] and r["exit_code"] == 0
    assert all(x > 0 for x in r["per_rank_hashes_per_sec"]) and r["pool_rejected"] == 0


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_rccl_module_collectives_at_world_one():
    from otedama_amd import _rccl

    uid = _rccl.unique_id()
    assert len(uid) == 128
    c = _rccl.RcclComm(0, 1, 0, uid, 30.0)
    assert c.alive and c.nranks == 1 and c.rank == 0
    blob = bytes(range(256)) * 256
    assert c.broadcast(blob, len(blob), 0, 5.0) == blob
    mine = np.arange(640, dtype=np.int64).tobytes()
    assert c.all_gather(mine, 5.0) == mine
    v = np.array([3, -4, 5, 1 << 40], dtype=np.int64)
    assert np.frombuffer(c.all_reduce(v.tobytes(), "i64", "sum", 5.0), dtype=np.int64).tolist() == v.tolist()
    f = np.array([2.5], dtype=np.float64)
    assert np.frombuffer(c.all_reduce(f.tobytes(), "f64", "max", 5.0), dtype=np.float64)[0] == 2.5
    assert c.ops == 4
    c.abort()
    assert not c.alive
    with pytest.raises(RuntimeError):
        c.broadcast(blob, len(blob), 0, 5.0)


@pytest.mark.gpu
def test_native_node_comm_generations_through_the_store():
    from otedama_amd.parallel.commbase import Device, DistInfo
    from otedama_amd.parallel.kvclient import StoreClient
    from otedama_amd.parallel.kvstore import StoreServer
    from otedama_amd.parallel.rcclcomm import NativeNodeComm

    with StoreServer() as srv:
        info = DistInfo(0, 1, 0, "rccl", Device("cuda", 0), store=StoreClient("127.0.0.1", srv.port, timeout=10))
        comm = NativeNodeComm(info, force=True)
        comm.reform([0], 0)
        assert srv.get("otd-g0/rcclid") is not None and len(srv.get("otd-g0/rcclid")) == 128
        job = {"job_id": "j", "header": bytes(range(80)), "epoch": 7, "branches": [bytes(32)] * 3}
        assert comm.broadcast_job(job) == job
        got = comm.gather_shares([{"epoch": 7, "nonce": 5, "ntime": 1, "version": 2, "extranonce2": 3,
                                   "found_at": 1.5, "device_found_at": 1.25}])
        assert [(s["nonce"], s["epoch"], s["found_at"], s["device_found_at"]) for s in got] == [(5, 7, 1.5, 1.25)]
        assert comm.allreduce_counters(10, 2, 1, 0) == (10, 2, 1, 0)
        assert comm.gather_counters([1, 2, 3, 4]) == [[1, 2, 3, 4]]
        assert comm.broadcast_control([9, 8]) == [9, 8, 0, 0] and comm.allreduce_max(3.5) == 3.5
        comm.reform([0], 1)  # the next generation: a fresh id and communicator
        assert info.generation == 1 and srv.get("otd-g1/rcclid") != srv.get("otd-g0/rcclid")
        assert comm.allreduce_counters(1)[0] == 1 and comm.collectives == 7
        comm.close()


@pytest.mark.gpu
def test_a_native_rank_process_never_imports_torch():
    code = (
        "import sys, os\n"
        "os.environ['OTEDAMA_NO_TORCH'] = '1'\n"
        "from otedama_amd.parallel.commbase import Device, DistInfo\n"
        "from otedama_amd.parallel.kvstore import StoreServer\n"
        "from otedama_amd.parallel.kvclient import StoreClient\n"
        "from otedama_amd.parallel.rcclcomm import NativeNodeComm\n"
        "from otedama_amd.parallel.node import NodeMinerSet, NodeWorker\n"
        "from otedama_amd.ops.native import require_native\n"
        "require_native()\n"
        "srv = StoreServer()\n"
        "info = DistInfo(0, 1, 0, 'rccl', Device('cuda', 0), store=StoreClient('127.0.0.1', srv.port))\n"
        "c = NativeNodeComm(info, force=True); c.reform([0], 0)\n"
        "assert c.allreduce_counters(5)[0] == 5\n"
        "c.close(); srv.close()\n"
        "print('TORCH' if 'torch' in sys.modules else 'NO-TORCH')\n")
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                         env=dict(os.environ, PYTHONPATH=ROOT))
    assert res.returncode == 0, res.stderr[-3000:]
    assert res.stdout.strip().splitlines()[-1] == "NO-TORCH", res.stdout


@pytest.mark.gpu
def test_an_op_past_its_deadline_leaves_the_communicator_broken_until_aborted():
    """A timed-out op may still sit in the comm stream (at world > 1: its peer never came), so the next op must not
    stage into the buffers it uses: the communicator refuses every op until it is aborted, and a new one works."""
    from otedama_amd import _rccl

    c = _rccl.RcclComm(0, 1, 0, _rccl.unique_id(), 30.0)
    big = bytes(64 << 20)  # ~ms of staging copies: still in flight at a zero deadline
    with pytest.raises(TimeoutError):
        c.all_gather(big, 0.0)
    with pytest.raises(RuntimeError, match="timed out"):
        c.all_gather(b"x" * 8, 5.0)
    c.abort()
    d = _rccl.RcclComm(0, 1, 0, _rccl.unique_id(), 30.0)
    assert d.all_gather(b"y" * 8, 5.0) == b"y" * 8
    d.abort()


@pytest.mark.gpu
def test_device_resident_ops_at_world_one_and_their_stream_order():
    """The device-pointer forms bench.py's R1 / R2 and the comm section use (RcclComm.*_dev through NativeNodeComm):
    the all_gather reads and writes device memory on the caller's stream, nothing staged through the host; a host-
    staged op issued right after is ordered behind it on the device (the comm's event hand-off between streams)."""
    import torch

    from otedama_amd.parallel.commbase import DistInfo
    from otedama_amd.parallel.rcclcomm import NativeNodeComm

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    comm = NativeNodeComm(DistInfo(0, 1, 0, "rccl", dev), bounded=False, force=True, device_stream=True)
    comm.reform([0], 7)
    try:
        assert comm.stream is not None
        inp = torch.arange(1 << 20, dtype=torch.int32, device=dev)
        out = torch.zeros(1, 1 << 20, dtype=torch.int32, device=dev)
        ev = comm.run_async(lambda: comm.gather_tensor(out, inp))
        ev.synchronize()
        assert torch.equal(out[0], inp)
        t = torch.full((16,), 5, dtype=torch.uint8, device=dev)
        comm.broadcast_tensor(t)
        torch.cuda.synchronize()
        assert int(t.min()) == 5
        # a long producer on the current stream, the gather on the comm stream after it, then a host-staged R3
        big = torch.randn(4096, 4096, device=dev)
        for _ in range(8):
            big = big @ big.T / 4096.0
        inp2 = (big[0, :16] * 0 + 3).to(torch.int32).contiguous()
        out2 = torch.zeros(1, 16, dtype=torch.int32, device=dev)
        comm.run_async(lambda: comm.gather_tensor(out2, inp2))
        assert comm.allreduce_counters(5)[0] == 5
        torch.cuda.synchronize()
        assert out2.cpu().tolist()[0] == [3] * 16
        assert comm._rc.ops >= 4
    finally:
        comm.close()
