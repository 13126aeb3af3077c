"""The RCCL (torch.distributed "nccl") calls of the node path on a real MI355X, at world size 1: the exact
R1 broadcast, R2 all_gather_into_tensor, R3 all_reduce (int64 SUM, float64 MAX) and device barrier that
parallel/comm.py issues on its comm stream. NodeComm skips collectives at world size 1, so the calls are made
here directly on its buffers; the 2..8-rank runs are the driver's node benchmarks (RCCL refuses two ranks on
one GPU)."""
import socket

import pytest
import torch


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_rccl_collectives_on_the_comm_stream():
    import torch.distributed as dist

    from otedama_amd.parallel.comm import COUNTER_WORDS, SHARE_SLOTS, SHARE_WORDS, DistInfo, NodeComm

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        info = DistInfo(0, 1, 0, "nccl", dev)
        comm = NodeComm(info)
        assert comm.stream is not None
        # R1: job blob broadcast (rank 0 is the source)
        comm._job.copy_(torch.arange(comm._job.numel(), dtype=torch.int64).remainder(251).to(torch.uint8))
        want = comm._job.clone()
        comm._run(lambda: dist.broadcast(comm._job, src=0))
        torch.cuda.synchronize()
        assert torch.equal(comm._job, want)
        # R2: share slots all-gathered into the [world, slots, words] buffer
        comm._slots.copy_(torch.arange(SHARE_SLOTS * SHARE_WORDS, dtype=torch.int64).view(SHARE_SLOTS, SHARE_WORDS))
        comm._run(lambda: dist.all_gather_into_tensor(comm._gathered.view(-1, SHARE_WORDS), comm._slots))
        torch.cuda.synchronize()
        assert torch.equal(comm._gathered[0], comm._slots)
        # R3: int64 counters (values above 2^32 must survive) and the float64 max used for timing
        comm._counters.copy_(torch.tensor([1 << 40, 3, 0, 7], dtype=torch.int64)[:COUNTER_WORDS])
        comm._run(lambda: dist.all_reduce(comm._counters, op=dist.ReduceOp.SUM))
        assert comm._counters.cpu().tolist()[:4] == [1 << 40, 3, 0, 7]
        t = torch.tensor([1.25], dtype=torch.float64, device=dev)
        comm._run(lambda: dist.all_reduce(t, op=dist.ReduceOp.MAX))
        assert float(t.item()) == 1.25
        # the comm stream is ordered after the producer: a kernel on the current stream feeds the broadcast
        comm._job.fill_(9)
        comm._run(lambda: dist.broadcast(comm._job, src=0))
        torch.cuda.synchronize()
        assert int(comm._job.min()) == 9
        dist.barrier(device_ids=[0])  # the form barrier() uses for the nccl backend
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_group_rendezvous_through_the_supervisors_store():
    """`otedama node` ranks form their RCCL groups through the supervisor's torch-free store (parallel/kvstore.py),
    one PrefixStore per group generation as parallel/comm.py does. At world 1 on the real MI355X: RCCL's bootstrap
    uses only query types the server implements (none refused), and the group runs a collective."""
    import datetime

    import torch.distributed as dist

    from otedama_amd.parallel.kvstore import StoreServer

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    with StoreServer() as srv:
        client = dist.TCPStore("127.0.0.1", srv.port, None, False, datetime.timedelta(seconds=60),
                               wait_for_workers=False)
        for gen in range(2):
            dist.init_process_group("nccl", store=dist.PrefixStore(f"otd-g{gen}", client), rank=0, world_size=1,
                                    device_id=dev)
            try:
                t = torch.full((4,), 3, dtype=torch.int64, device=dev)
                dist.all_reduce(t)
                torch.cuda.synchronize()
                assert t.tolist() == [3, 3, 3, 3]
            finally:
                dist.destroy_process_group()
        assert srv.refused == 0
        assert srv.num_keys() > 0


@pytest.mark.gpu
def test_data_plane_probe_forms_an_rccl_group_at_world_one(monkeypatch):
    """bench.py's data-plane pre-flight (parallel/rccl_probe.py) on the GPU: the child forms a native RCCL group
    (otedama_amd._rccl, the bench's and the node's data plane) through the job's store, runs its all_reduce, meets
    its peers at the done barrier and reports ok; an injected hang is killed at the deadline and reported as such."""
    import datetime

    import torch.distributed as dist

    from otedama_amd.parallel.launch import free_port
    from otedama_amd.parallel.rccl_probe import run_probe

    port = free_port()
    store = dist.TCPStore("127.0.0.1", port, is_master=True, timeout=datetime.timedelta(seconds=60),
                          wait_for_workers=False)
    for k, v in {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(port), "TORCHELASTIC_RUN_ID": "probe-ok"}.items():
        monkeypatch.setenv(k, v)
    r = run_probe(store, 0, 1, timeout=60)
    assert r["ok"] and r["ranks"]["0"]["ok"] and r["impl"] == "rccl-native", r
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "probe-hang")
    r = run_probe(store, 0, 1, timeout=3, fault="hang")
    assert not r["ok"] and "killed" in r["ranks"]["0"]["reason"], r
