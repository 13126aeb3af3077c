"""Multi-process node (world_size 2, gloo on CPU): R1 job fan-out, R2 share fan-in,
R3 counters, disjoint stripes, remote pause and clean stop.

Same code path as the RCCL node on MI355X (parallel/node.py); only the
backend and the miner (native CpuMiner instead of GpuMiner) differ.
"""
import json
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from otedama_amd import hal
from otedama_amd.models.header import int_to_hash, sha256d

WORLD = 2


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job() -> dict:
    hdr = bytes([1, 0, 0, 0]) + bytes(range(32)) + bytes(range(32, 64)) + (1700000000).to_bytes(4, "little") + \
        bytes.fromhex("ffff001d") + bytes(4)
    return {"header": hdr, "target": int_to_hash(1 << 240), "job_id": "job-A", "algo": "sha256d",
            "version_mask": 0x1FFFE000}


def _worker(rank: int, port: int, out_path: str, world: int = WORLD) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from otedama_amd.engine.miners import MinerSet
    from otedama_amd.parallel.comm import NodeComm, init_from_env, shutdown
    from otedama_amd.parallel.node import NodeMinerSet, NodeWorker

    info = init_from_env(backend="gloo", use_gpu=False)
    dev = [hal.SimpleDevice(hal.Identity(f"cpu-{rank}", hal.Family.CPU, "t", "cpu"),
                            hal.Capabilities(sha256d=True, general_compute=True), threads=1)]
    local = MinerSet(dev, "sha256d", rank=info.rank, world_size=info.world_size)
    comm = NodeComm(info)
    if rank > 0:
        NodeWorker(local, comm, tick=0.005).run()
        shutdown(info)
        return
    node = NodeMinerSet(local, comm, tick=0.005)
    node.start()
    ep = node.set_job(_job())
    shares, deadline = [], time.monotonic() + 20
    while time.monotonic() < deadline:
        shares += node.poll(256)
        per_rank = [sum(1 for s in shares if s["device_id"] == f"rank{r}") for r in range(1, world)]
        if min(per_rank) >= 3 and len(shares) >= 2 * world:
            break
        time.sleep(0.02)
    end = time.monotonic() + 10  # remote counters arrive with the 2 Hz heartbeats (and R3 every stats interval)
    while time.monotonic() < end and not all(node.device_stats()[f"rank{r}"]["hashes"] > 0 for r in range(1, world)):
        time.sleep(0.05)
    node.update_hashrates()
    stats = node.device_stats()
    total = node.total_hashes()
    # pause the remote rank, wait for its counter to freeze
    node.pause_device("rank1", True)
    time.sleep(1.2)  # the pause reaches rank 1 (R1) and its counter reaches rank 0 (2 Hz heartbeat)
    h1 = node.device_stats()["rank1"]["hashes"]
    time.sleep(1.2)
    h2 = node.device_stats()["rank1"]["hashes"]
    node.stop()
    shutdown(info)
    with open(out_path, "w") as f:
        json.dump({"epoch": ep, "shares": shares, "stats": stats, "total": total, "paused_delta": h2 - h1,
               "len": len(node)}, f, default=str)


def test_node_two_ranks(tmp_path):
    out = tmp_path / "out.json"
    mp.start_processes(_worker, args=(_port(), str(out)), nprocs=WORLD, join=True, start_method="spawn")
    res = json.loads(out.read_text())
    shares = res["shares"]
    remote = [s for s in shares if s["device_id"] == "rank1"]
    local = [s for s in shares if s["device_id"] != "rank1"]
    assert len(remote) >= 3 and local
    assert res["len"] == 2 and "rank1" in res["stats"] and res["stats"]["rank1"]["hashes"] > 0
    assert res["total"] >= res["stats"]["rank1"]["hashes"]
    job = _job()
    for s in shares:
        assert s["job_id"] == "job-A" and int(s["epoch"]) == res["epoch"]
        hdr = bytearray(job["header"])
        hdr[0:4] = int(s["version"]).to_bytes(4, "little")
        hdr[68:72] = int(s["ntime"]).to_bytes(4, "little")
        hdr[76:80] = int(s["nonce"]).to_bytes(4, "little")
        assert int.from_bytes(sha256d(bytes(hdr)), "little") <= 1 << 240
        # disjoint stripes: variant parity (lowest rolled version bit 13) == rank
        rank = 1 if s["device_id"] == "rank1" else 0
        assert (int(s["version"]) >> 13) & 1 == rank
    assert res["paused_delta"] == 0
    if dist.is_initialized():
        dist.destroy_process_group()


def test_node_four_ranks_stripes_and_fan_in(tmp_path):
    """World size 4 (the 8-GPU node's code path at half the ranks): every remote rank's shares reach rank 0
    through R2, each rank hashes only its own stripe (variant index = rank mod 4, i.e. the two lowest rolled
    version bits), and the R3 counters cover all four ranks."""
    world = 4
    out = tmp_path / "out4.json"
    mp.start_processes(_worker, args=(_port(), str(out), world), nprocs=world, join=True, start_method="spawn")
    res = json.loads(out.read_text())
    assert res["len"] == world
    for r in range(1, world):
        assert res["stats"][f"rank{r}"]["hashes"] > 0
    job = _job()
    seen = set()
    for s in res["shares"]:
        rank = int(s["device_id"][4:]) if s["device_id"].startswith("rank") else 0
        seen.add(rank)
        assert (int(s["version"]) >> 13) & 3 == rank
        hdr = bytearray(job["header"])
        hdr[0:4] = int(s["version"]).to_bytes(4, "little")
        hdr[68:72] = int(s["ntime"]).to_bytes(4, "little")
        hdr[76:80] = int(s["nonce"]).to_bytes(4, "little")
        assert int.from_bytes(sha256d(bytes(hdr)), "little") <= 1 << 240
    assert seen == set(range(world))


@pytest.mark.parametrize("n", [1])
def test_nodecomm_single_rank_paths(n):
    from otedama_amd.parallel.comm import DistInfo, NodeComm

    c = NodeComm(DistInfo())
    assert c.broadcast_control([5, 0, 9]) == [5, 0, 9, 0]
    assert c.gather_counters([1, 2, 3, 4]) == [[1, 2, 3, 4]]
    got = c.gather_shares([{"epoch": 3, "nonce": 7, "ntime": 1, "version": 2, "extranonce2": 1 << 40,
                            "found_at": 12.5}])
    assert got[0]["extranonce2"] == 1 << 40 and got[0]["found_at"] == 12.5 and got[0]["epoch"] == 3


def test_host_buffers_keep_node_collectives_off_the_device():
    """Over gloo the node's buffers live in host memory (no comm stream); records round-trip in rank/slot order
    with every field, and empty slots are skipped."""
    import torch

    from otedama_amd.parallel.comm import SHARE_SLOTS, DistInfo, NodeComm

    c = NodeComm(DistInfo(backend="gloo"), host_buffers=True)
    assert c.dev == torch.device("cpu") and c.stream is None and c._slots.device.type == "cpu"
    shares = [{"epoch": (5 << 32) | 9, "nonce": 0xFFFFFFFF - i, "ntime": 100 + i, "version": 0x20000000 | i,
               "extranonce2": i << 33, "found_at": 1.25 + i, "device_found_at": 1.0 + i} for i in range(SHARE_SLOTS + 3)]
    got = c.gather_shares(shares)
    assert len(got) == SHARE_SLOTS  # one gather carries at most SHARE_SLOTS per rank
    for i, g in enumerate(got):
        s = shares[i]
        assert (g["epoch"], g["nonce"], g["ntime"], g["version"], g["extranonce2"]) == \
            (s["epoch"], s["nonce"], s["ntime"], s["version"], s["extranonce2"])
        assert g["found_at"] == s["found_at"] and g["device_found_at"] == s["device_found_at"] and g["orig_rank"] == 0
    assert c.gather_shares([]) == []


def test_ops_ride_the_doorbell_datagram():
    """The leader's op travels inline in the follower's doorbell datagram (no store round trip on the share path);
    bare wake-ups and share rings parse as no op."""
    from otedama_amd.parallel.node import _Bell, op_msg, parse_op_msg

    raw = json.dumps({"op": "gather", "gen": 3})
    assert parse_op_msg(op_msg(17, raw)) == (17, {"op": "gather", "gen": 3})
    assert parse_op_msg(b"o") is None and parse_op_msg(b"s") is None and parse_op_msg(b"o" + bytes(8) + b"{") is None
    a, b = _Bell(None, 0), _Bell(None, 1)
    try:
        a._ports[1] = (b.port, time.monotonic())
        a.ring(1, op_msg(4, raw))
        a.ring(1, b"s")
        got = []
        end = time.monotonic() + 2
        while len(got) < 2 and time.monotonic() < end:
            got += b.wait(0.1)
        assert [parse_op_msg(m) for m in got] == [(4, {"op": "gather", "gen": 3}), None]
    finally:
        a.close()
        b.close()


def _blob_worker(rank: int, port: int, out_path: str) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from otedama_amd.parallel.comm import NodeComm, init_from_env, shutdown

    info = init_from_env(backend="gloo", use_gpu=False)
    comm = NodeComm(info)
    big = dict(_job(), coinb1=bytes(range(150)), coinb2=bytes(i % 251 for i in range(2000)), extranonce1=b"\x01\x02",
               extranonce2_size=8, merkle_branches=[bytes([i]) * 32 for i in range(13)])
    got = comm.broadcast_job(big if rank == 0 else None)
    shutdown(info)
    if rank == 1:
        with open(out_path, "w") as f:
            json.dump({"same": got == big, "keys": sorted(got)}, f)


def test_node_broadcasts_a_large_v1_job(tmp_path):
    """R1 carries a full Stratum V1 job (2 KB coinb2, 13 merkle branches): well past the old 4 KiB blob once
    hex-encoded in JSON."""
    out = tmp_path / "blob.json"
    mp.start_processes(_blob_worker, args=(_port(), str(out)), nprocs=WORLD, join=True, start_method="spawn")
    r = json.loads(out.read_text())
    assert r["same"], r
