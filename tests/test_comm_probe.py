"""The comm-under-load probe (parallel/comm_probe.py): NodeComm's forced one-rank collectives and
the op loop that times them. The GPU measurement (RCCL + a saturating device process) is in the gpu-marked test; the
op loop and the forced world-1 path are checked on CPU over a one-rank gloo group."""
import pytest
import torch
import torch.distributed as dist

from otedama_amd.parallel.comm import DistInfo, NodeComm
from otedama_amd.parallel.comm_probe import _q, run_ops


@pytest.fixture
def one_rank_gloo():
    dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
    yield DistInfo(0, 1, 0, "gloo", torch.device("cpu"))
    dist.destroy_process_group()


def test_forced_world1_collectives_round_trip(one_rank_gloo):
    comm = NodeComm(one_rank_gloo, bounded=True, deadline=5.0, force=True)
    assert comm._job_h is comm._job  # CPU: the host mirror is the buffer itself
    assert comm.multi
    job = {"job_id": "j", "header": bytes(range(80)), "epoch": 7}
    assert comm.broadcast_job(job) == job
    got = comm.gather_shares([{"epoch": 7, "nonce": 5, "ntime": 1, "version": 2, "extranonce2": 3}])
    assert [(s["nonce"], s["epoch"]) for s in got] == [(5, 7)]
    assert comm.gather_counters([1, 2, 3, 4]) == [[1, 2, 3, 4]]
    assert comm.collectives == 3  # all three went through the process group


def test_unforced_world1_skips_collectives(one_rank_gloo):
    comm = NodeComm(one_rank_gloo)
    assert not comm.multi
    comm.gather_counters([1, 2, 3, 4])
    assert comm.collectives == 0


def test_run_ops_times_every_op_kind(one_rank_gloo):
    comm = NodeComm(one_rank_gloo, bounded=True, deadline=5.0, force=True)
    r = run_ops(comm, 0.6, cadence_hz=100.0)
    assert r["R2_gather"]["samples"] > 20 and r["R1_job"]["samples"] > 0 and r["R3_counters"]["samples"] > 0
    assert "kernel" not in r  # no comm stream on CPU
    assert all(v["p50_ms"] <= v["p99_ms"] <= v["max_ms"] for v in r.values())


def test_quantiles():
    q = _q([float(i) for i in range(1, 101)])
    assert q["p50_ms"] == 50.0 and q["p99_ms"] == 99.0 and q["max_ms"] == 100.0 and q["samples"] == 100


@pytest.mark.gpu
def test_comm_under_load_on_the_gpu():
    """One GPU: R1/R2/R3 through a forced one-rank RCCL group while a device process mines SHA-256d at full rate."""
    from otedama_amd.parallel.comm_probe import measure_comm_under_load

    r = measure_comm_under_load(0, ["sha256d"], seconds=1.0, cadence_hz=50.0, windows=1)
    assert r["idle"]["node"]["R2_gather"]["samples"] > 20 and r["idle"]["legacy"]["R2_gather"]["samples"] > 20
    assert r["idle"]["native"]["R2_gather"]["samples"] > 20 and r["sha256d"]["loaded"]["native"]["R1_job"]["samples"]
    s = r["sha256d"]
    assert s["rate_alone_hps"] > 1e10
    assert s["loaded"]["node"]["R2_gather"]["samples"] > 20 and s["loaded"]["legacy"]["kernel"]["samples"] > 0
    # the node's layout (everything on high-priority streams) is not slower than the legacy one under load
    assert s["loaded"]["node"]["R2_gather"]["p50_ms"] <= s["loaded"]["legacy"]["R2_gather"]["p50_ms"] * 1.2
