"""The node's native RCCL data plane: NodeComm's API over ``otedama_amd._rccl`` (csrc/runtime/rccl_comm.cpp).

On GPUs the node's rank processes use this instead of torch.distributed (SURVEY §7.1 puts "the RCCL comm layer
(R1-R3)" in C++): no ``import torch`` in a rank (it was ~1.45 s of the 1.8 s a rank took to its process group,
profiles/r5/c_node_rehearsal), every op one chain on a high-priority HIP stream (profiles/r5/d_comm_ab), and
``ncclCommAbort`` for a broken group. The store, op log, doorbells, heartbeats and re-form protocol of
parallel/node.py are unchanged; only the collectives move. A generation's RCCL unique id travels through the node's
store (``otd-g<gen>/rcclid``, posted by the group's rank 0, which is always the leader).

``open_node_comm`` picks the implementation for a rank. Generation 0 is formed natively when every rank manages to;
if any rank fails (the RCCL bootstrap, a missing library, a deadline), every rank falls back to torch.distributed
(RCCL through ProcessGroupNCCL) together, and the choice is recorded at ``otd/comm`` for replacement ranks. CPU hosts
and rehearsals (``OTEDAMA_DIST_BACKEND=gloo``) use torch.distributed over gloo as before; ``OTEDAMA_NODE_COMM=torch``
forces torch.distributed on GPUs too.

``OTEDAMA_RCCL_MODULE`` names a module with ``_rccl``'s API to load instead (tests/loopback_rccl.py: the collectives
over the store, so this protocol runs at world 4 / 8 on CPUs, where the one-GPU box cannot run RCCL at world > 1).
"""
from __future__ import annotations

import importlib
import os
import time

import numpy as np

from otedama_amd.parallel.commbase import (COUNTER_WORDS, JOB_BLOB_BYTES, PG_TIMEOUT_S, SHARE_SLOTS, SHARE_WORDS,
                                           CollectiveTimeout, Device, DistInfo, job_from_payload, job_payload,
                                           pack_shares, unpack_shares)

COMM_KEY = "otd/comm"  # "rccl" or "torch": the implementation the node's generation 0 settled on
FAILED_ID = b"!"       # published in place of a unique id that rank 0 could not create
_HOSTED_SERVER = None  # a store this process hosts (rank 0 without a supervisor / torchrun agent)


class NativeNodeComm:
    """R1 / R2 / R3 over the native RCCL module, one communicator per process-group generation. Same interface as
    parallel/comm.py NodeComm (the node uses nothing else)."""

    def __init__(self, info: DistInfo, bounded: bool = True, deadline: float = 3.0, force: bool = False,
                 device_stream: bool = False):
        """``device_stream``: give the comm a high-priority torch stream for the device-resident forms' overlapped
        use (``run_async``; bench.py). The node's ranks leave it off and never import torch."""
        self._rccl = rccl_module()
        self.info = info
        self.bounded = bounded
        self.deadline = deadline
        self.force = force
        self.collectives = 0
        self.stream = None
        self.dev = info.device
        if device_stream and getattr(info.device, "type", "cpu") == "cuda":
            import torch

            if not isinstance(info.device, torch.device):
                info.device = torch.device(info.device.type, info.device.index)
            self.dev = info.device
            lo, hi = torch.cuda.Stream.priority_range()
            self.stream = torch.cuda.Stream(self.dev, priority=min(lo, hi))
        self._rc = None  # the current generation's RcclComm
        self._job_h = np.zeros(JOB_BLOB_BYTES, dtype=np.uint8)  # rank 0's last blob

    @property
    def multi(self) -> bool:
        return self.info.world_size > 1 or self.force

    def bind_thread(self) -> None:
        """Nothing to do: every native op selects the comm's device itself."""

    def close(self) -> None:
        self.abort()

    # ---------------------------------------------------------------- generations
    def abort(self) -> None:
        """Tear the current communicator down at once (ncclCommAbort never waits for the peers)."""
        rc, self._rc = self._rc, None
        if rc is not None:
            try:
                rc.abort()
            except Exception:  # noqa: BLE001 - the group is unusable either way
                pass

    def reform(self, members: list[int], generation: int, timeout: float | None = None) -> None:
        """Leave the current group and form generation ``generation`` of ``members`` (orig ranks; group rank =
        position). The group's rank 0 publishes the RCCL unique id under otd-g<gen>/rcclid; the others wait for it
        (bounded by OTEDAMA_PG_TIMEOUT), then every member initialises its communicator (same bound)."""
        info = self.info
        if info.orig_rank not in members:
            raise ValueError(f"rank {info.orig_rank} is not a member of generation {generation}")
        self.abort()
        timeout = PG_TIMEOUT_S if timeout is None else timeout
        rank, world = members.index(info.orig_rank), len(members)
        if world > 1 or self.force:
            key = f"otd-g{generation}/rcclid"
            if rank == 0:
                try:
                    uid = self._rccl.unique_id()
                except Exception:
                    if info.store is not None:
                        info.store.set(key, FAILED_ID)  # the other members fail at once instead of at their deadline
                    raise
                if info.store is not None:  # a forced one-rank group may have no store (bench.py at N=1)
                    info.store.set(key, uid)
            else:
                uid = _wait_get(info.store, key, timeout)
                if uid == FAILED_ID:
                    raise RuntimeError(f"generation {generation}: the group's rank 0 could not create an RCCL id")
            self._rc = self._rccl.RcclComm(int(info.device.index or 0), world, rank, uid, timeout)
        info.rank, info.world_size, info.generation, info.members = rank, world, generation, list(members)

    # ---------------------------------------------------------------- ops
    def _timeout(self) -> float:
        return self.deadline if self.bounded else PG_TIMEOUT_S

    def _call(self, fn, *args):
        if self._rc is None:
            raise RuntimeError("rccl: no communicator for this generation")
        self.collectives += 1
        try:
            return fn(*args, self._timeout())
        except TimeoutError as exc:  # _rccl.RcclTimeout
            raise CollectiveTimeout(str(exc)) from None

    def broadcast_job(self, job: dict | None) -> dict | None:
        if self.info.is_primary:
            buf = job_payload(job)
        else:
            buf = b""
        if self.multi:
            buf = self._call(self._rc.broadcast, buf, JOB_BLOB_BYTES, 0)
        return job_from_payload(buf)

    def gather_shares(self, shares: list[dict], device_index: int = 0) -> list[dict]:
        rows = pack_shares(shares, self.info.rank, device_index)
        if self.multi:
            raw = self._call(self._rc.all_gather, rows.tobytes())
            g = np.frombuffer(raw, dtype=np.int64).reshape(-1, SHARE_SLOTS, SHARE_WORDS)
        else:
            g = rows[None]
        return unpack_shares(g, self.info.members)

    def allreduce_counters(self, hashes: int, shares: int = 0, dropped: int = 0, faults: int = 0) -> tuple:
        v = np.array([hashes, shares, dropped, faults], dtype=np.int64)
        if self.multi:
            v = np.frombuffer(self._call(self._rc.all_reduce, v.tobytes(), "i64", "sum"), dtype=np.int64)
        return tuple(int(x) for x in v)

    def gather_counters(self, values: list[int]) -> list[list[int]]:
        v = np.array(list(values)[:COUNTER_WORDS] + [0] * (COUNTER_WORDS - len(values)), dtype=np.int64)
        if self.multi:
            raw = self._call(self._rc.all_gather, v.tobytes())
            return np.frombuffer(raw, dtype=np.int64).reshape(-1, COUNTER_WORDS).tolist()
        return [v.tolist()]

    def broadcast_control(self, words: list[int]) -> list[int]:
        v = np.array(list(words)[:4] + [0] * (4 - len(words)), dtype=np.int64)
        if self.multi:
            raw = self._call(self._rc.broadcast, v.tobytes() if self.info.is_primary else b"", 32, 0)
            v = np.frombuffer(raw, dtype=np.int64)
        return v.tolist()

    def allreduce_max(self, value: float) -> float:
        v = np.array([value], dtype=np.float64)
        if self.multi:
            v = np.frombuffer(self._call(self._rc.all_reduce, v.tobytes(), "f64", "max"), dtype=np.float64)
        return float(v[0])

    def barrier(self) -> None:
        """Every rank reached this point (one R3 word)."""
        if self.multi:
            self.allreduce_counters(0)

    # ---------------------------------------------------------------- device-resident forms (bench.py)
    # torch tensors on this comm's device (CPU tensors under a CPU stand-in module); the op is enqueued on the current
    # torch stream and nothing goes through the host (RcclComm.*_dev). Same signatures as parallel/comm.py NodeComm.
    def _cur_stream(self) -> int:
        if getattr(self.dev, "type", "cpu") != "cuda":
            return 0
        import torch

        return torch.cuda.current_stream(self.dev).cuda_stream

    def gather_tensor(self, out, inp) -> None:
        """``out`` (world x inp.shape) gets every rank's contiguous ``inp``, in rank order."""
        if not self.multi or (self.info.world_size == 1 and os.environ.get("OTEDAMA_RCCL_LOCAL_R2") == "1"):
            out[0].copy_(inp)
            return
        if self._rc is None:
            raise RuntimeError("rccl: no communicator for this generation")
        self.collectives += 1
        self._rc.all_gather_dev(inp.data_ptr(), out.data_ptr(), inp.numel() * inp.element_size(), self._cur_stream(),
                                self._timeout())

    def broadcast_tensor(self, t, src: int = 0) -> None:
        if not self.multi:
            return
        if self._rc is None:
            raise RuntimeError("rccl: no communicator for this generation")
        self.collectives += 1
        self._rc.broadcast_dev(t.data_ptr(), t.numel() * t.element_size(), src, self._cur_stream(), self._timeout())

    def run_async(self, fn):
        """As parallel/comm.py NodeComm.run_async: ``fn``'s ops go on the comm stream, ordered after the current
        stream's queued work; returns an event on the comm stream (None without one: the op completed inline)."""
        if self.stream is None:
            fn()
            return None
        import torch

        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev


def rccl_module():
    """``otedama_amd._rccl``, or the stand-in OTEDAMA_RCCL_MODULE names (see the module docstring)."""
    name = os.environ.get("OTEDAMA_RCCL_MODULE")
    if name:
        return importlib.import_module(name)
    from otedama_amd import _rccl

    return _rccl


def cpu_standin() -> bool:
    """OTEDAMA_RCCL_MODULE names a stand-in that runs on CPUs (DEVICE_TYPE = "cpu"): the ranks mine on CPUs."""
    return bool(os.environ.get("OTEDAMA_RCCL_MODULE")) and getattr(rccl_module(), "DEVICE_TYPE", "cuda") == "cpu"


def _rank_device(local: int) -> Device:
    """The rank's device: its GPU, or a CPU under a CPU stand-in module."""
    return Device("cpu", None) if cpu_standin() else Device("cuda", local)


def _wait_get(store, key: str, timeout: float) -> bytes:
    """The key's value once it is set, within ``timeout`` s (TimeoutError otherwise)."""
    end = time.monotonic() + timeout
    while not store.check([key]):
        if time.monotonic() > end:
            raise TimeoutError(f"{key} not published within {timeout:.0f} s")
        time.sleep(0.01)
    return store.get(key)


# ---------------------------------------------------------------------------- choosing the implementation
def native_wanted() -> bool:
    """The native RCCL path applies: GPU ranks (not a gloo rehearsal), unless OTEDAMA_NODE_COMM says otherwise
    ("torch": never; "native": always try it, e.g. to exercise the fallback on a CPU host)."""
    mode = os.environ.get("OTEDAMA_NODE_COMM", "").lower()
    if mode == "torch":
        return False
    if mode == "native":
        return True
    if os.environ.get("OTEDAMA_DIST_BACKEND", "") == "gloo":
        return False
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        if os.environ.get(var) == "":
            return False
    from otedama_amd.parallel.launch import visible_gpus_kfd

    return visible_gpus_kfd() > 0


def _store_client(rank: int, world: int):
    """The node's store without torch: joined when a supervisor or torchrun's agent hosts it, else hosted here by
    rank 0 (our TCPStore-protocol server) and joined by the others."""
    global _HOSTED_SERVER
    from otedama_amd.parallel.kvclient import StoreClient

    addr = os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    hosted = os.environ.get("OTEDAMA_STORE_HOSTED") == "1" or os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    if rank == 0 and not hosted and _HOSTED_SERVER is None:
        from otedama_amd.parallel.kvstore import StoreServer

        _HOSTED_SERVER = StoreServer(addr, port)
        os.environ["OTEDAMA_STORE_HOSTED"] = "1"  # a torch fallback in this process joins it instead of hosting
    return StoreClient(addr, port, timeout=max(PG_TIMEOUT_S, 60.0))


def open_node_comm(joining: bool, host_buffers: bool = False, log=None):
    """(DistInfo, comm) for this rank of a node. See the module docstring for the choice and the fallback."""
    log = log or (lambda msg: None)
    if not native_wanted():
        return _torch_comm(joining, host_buffers)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    store = _store_client(rank, world)
    if joining:
        mode = _wait_get(store, COMM_KEY, PG_TIMEOUT_S).decode()
        if mode != "rccl":
            store.close()
            return _torch_comm(joining, host_buffers)
        info = DistInfo(-1, 0, local, "rccl", _rank_device(local), orig_rank=rank, generation=-1, members=[],
                        store=store, capacity=world)
        return info, NativeNodeComm(info)
    info = DistInfo(rank, world, local, "rccl", _rank_device(local), store=store, capacity=world)
    comm = None
    err = ""
    try:
        comm = NativeNodeComm(info)
        comm.reform(list(range(world)), 0)
        ok = True
    except Exception as exc:  # noqa: BLE001 - decided together below
        ok, err = False, f"{type(exc).__name__}: {exc}"
    store.set(f"otd/g0native/{rank}", "1" if ok else "0")
    flags = [_wait_get(store, f"otd/g0native/{r}", PG_TIMEOUT_S + 10.0) for r in range(world)]
    if all(f == b"1" for f in flags):
        if rank == 0:
            store.set(COMM_KEY, "rccl")
        return info, comm
    # some rank could not form the native group: every rank falls back to torch.distributed together
    log(f"node: native RCCL unavailable on rank(s) {[r for r, f in enumerate(flags) if f != b'1']}"
        + (f" ({err})" if err else "") + "; using torch.distributed")
    if comm is not None:
        comm.abort()
    if rank == 0:
        store.set(COMM_KEY, "torch")
    store.close()
    return _torch_comm(joining, host_buffers)


def _torch_comm(joining: bool, host_buffers: bool):
    from otedama_amd.parallel.comm import NodeComm, init_from_env, join_from_env

    info = join_from_env() if joining else init_from_env()
    if not joining and info.store is not None and info.rank == 0:
        try:
            info.store.set(COMM_KEY, "torch")
        except Exception:  # noqa: BLE001 - joiners then default to torch anyway
            pass
    return info, NodeComm(info, host_buffers=host_buffers)
