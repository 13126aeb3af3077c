"""Node-level collectives for multi-GPU mining: one process per GPU.

The reference has no collective layer at all ("Multi-node /
multi-GPU collectives: None"); its only parallelism is nonce-space DP over CPU
goroutines (internal/miner/worker.go:51-60,279) and a channel fan-in of shares
(internal/engine/fanin.go:61-68). Here the node is one rank per GPU over
``torch.distributed`` — backend ``nccl`` (= RCCL over xGMI on MI355X) on GPUs,
``gloo`` on CPU — and the three collectives of SURVEY §2.3 are:

  R1 broadcast  job fan-out from rank 0 (the pool-facing rank), fixed 4 KiB blob
  R2 all_gather share slots (fixed-size records, so the collective is static)
  R3 all_reduce hash / share / drop counters for the node hashrate

Payloads are bytes to a few KiB, so the budget is latency, not xGMI bandwidth:
collectives run on a dedicated comm stream so they overlap the search kernels
running on the miners' own HIP streams. ``run_async`` is the overlapped form
(nothing on the compute stream waits for the collective; bench.py double-buffers
the hit slots it gathers), ``_run`` the blocking one for results read at once.

Fault tolerance (parallel/node.py): the rendezvous TCPStore is created here (or
joined, when a GPU-free supervisor or torchrun's agent hosts it) and kept in
``DistInfo.store`` for the node's control plane and heartbeats; the process
group has a bounded timeout and lives under a per-generation store prefix, so
``NodeComm.reform`` can abort a group that lost a rank and form the next one
from the survivors. ``bounded`` collectives never wait past a deadline.
"""
from __future__ import annotations

import datetime
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from otedama_amd.parallel.commbase import (COUNTER_WORDS, JOB_BLOB_BYTES, PG_TIMEOUT_S, SHARE_SLOTS,  # noqa: F401
                                           SHARE_WORDS, CollectiveTimeout, DistInfo, _decode, _encode,
                                           job_from_payload, job_payload, pack_shares, unpack_shares)


def _connect_store(rank: int, world: int):
    """The rendezvous store: joined when a supervisor (OTEDAMA_STORE_HOSTED=1) or torchrun's agent hosts it, else
    hosted by rank 0."""
    addr = os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    hosted = os.environ.get("OTEDAMA_STORE_HOSTED") == "1" or os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    master = rank == 0 and not hosted
    kw = {"multi_tenant": True} if master else {}  # as torch's own env:// rendezvous hosts it
    return dist.TCPStore(addr, port, world_size=None if hosted else world, is_master=master,
                         timeout=datetime.timedelta(seconds=max(PG_TIMEOUT_S, 60.0)), wait_for_workers=False, **kw)


def connect_store_from_env():
    """This rank's connection to the job's rendezvous store (torchrun's agent, the supervisor, or hosted here by
    rank 0), before any process group: the bench's data-plane pre-flight (parallel/rccl_probe.py) uses it first."""
    return _connect_store(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")))


def init_from_env(backend: str | None = None, use_gpu: bool | None = None, store=None) -> DistInfo:
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun).

    One rank per GPU (LOCAL_RANK = HIP ordinal) over RCCL. ``OTEDAMA_DIST_BACKEND=gloo`` rehearses the
    N-rank control flow on fewer GPUs than ranks (ranks share ordinals modulo the device count; RCCL
    itself refuses two ranks on one GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = backend or os.environ.get("OTEDAMA_DIST_BACKEND") or None
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    ordinal = local % max(1, torch.cuda.device_count()) if (use_gpu and backend == "gloo") else local
    device = torch.device(f"cuda:{ordinal}") if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if world <= 1:
        return DistInfo(rank, 1, local, "none", device)
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    # RCCL: no watchdog that tears the process down on a peer's death; node.py aborts and re-forms instead
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
    if not dist.is_initialized():
        store = store if store is not None else _connect_store(rank, world)
        kw = {"device_id": device, "pg_options": rccl_pg_options()} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                store=dist.PrefixStore("otd-g0", store),
                                timeout=datetime.timedelta(seconds=PG_TIMEOUT_S), **kw)
    return DistInfo(rank, world, local, backend, device, store=store)


def join_from_env(backend: str | None = None, use_gpu: bool | None = None) -> DistInfo:
    """A replacement rank (the supervisor re-spawned a dead one): connect to the store only; the node leader adds
    it to the next process-group generation (parallel/node.py)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = backend or os.environ.get("OTEDAMA_DIST_BACKEND") or None
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    ordinal = local % max(1, torch.cuda.device_count()) if (use_gpu and backend == "gloo") else local
    device = torch.device(f"cuda:{ordinal}") if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
    store = _connect_store(rank, world)
    return DistInfo(-1, 0, local, backend or ("nccl" if use_gpu else "gloo"), device, orig_rank=rank,
                    generation=-1, members=[], store=store, capacity=world)


def barrier(info: DistInfo) -> None:
    if info.world_size > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def shutdown(info: DistInfo) -> None:
    if info.world_size > 1 and dist.is_initialized():
        dist.destroy_process_group()


class NodeComm:
    """R1/R2/R3 over torch.distributed with preallocated fixed-size buffers.

    ``bounded=True`` (the node): every collective is issued async and polled against ``deadline`` seconds; a
    collective that fails or times out raises (CollectiveTimeout / RuntimeError) instead of blocking forever.

    ``host_buffers=True``: the buffers live in host memory and there is no comm stream. That is the node's layout
    over gloo, a CPU transport: with device buffers every gloo collective adds device<->host staging and stream
    syncs (a 2-rank R2 gather took 4.7 ms p50 on the MI355X that way).

    On a GPU every op keeps ALL of its device work on the comm stream, a high-priority stream: the staged inputs
    (pinned host -> device), the collective (RCCL's own stream waits on it; the process group is created with
    high-priority RCCL streams, ``rccl_pg_options``) and the results (device -> pinned host). The GPU is saturated by
    the sibling device process's mining grid, and any kernel or blit of this process on a normal-priority queue waits
    behind it for a CU slot: an R2 gather with its copies on the default stream took 5.3 ms p50 under a SHA-256d miner
    against 0.16 ms idle (profiles/r5/c_comm_load). ``staging="legacy"`` keeps that old layout for the A/B."""

    def __init__(self, info: DistInfo, bounded: bool = False, deadline: float = 3.0, host_buffers: bool = False,
                 force: bool = False, stream_priority: int | str | None = "high", staging: str = "stream"):
        """``force``: issue the collectives at world 1 too (a one-rank process group must exist): the comm-under-load
        probe (parallel/comm_probe.py) measures the data plane's own path on a single GPU that way.
        ``stream_priority``: "high" (default), None (normal) or a HIP priority (lower = higher).
        ``staging``: "stream" (copies on the comm stream through pinned host buffers) or "legacy"."""
        if staging not in ("stream", "legacy"):
            raise ValueError("staging must be 'stream' or 'legacy'")
        self.info = info
        self.bounded = bounded
        self.deadline = deadline
        self.force = force
        self.staging = staging
        self.collectives = 0  # device collectives issued by this rank (node tick accounting)
        if not isinstance(info.device, torch.device):  # a torch-free Device (commbase): its torch twin
            info.device = torch.device(info.device.type, info.device.index)
        dev = torch.device("cpu") if host_buffers else info.device
        self.dev = dev
        self.cuda = dev.type == "cuda"
        self._job, self._job_h = self._pair(JOB_BLOB_BYTES, dtype=torch.uint8)
        self._slots, self._slots_h = self._pair(SHARE_SLOTS, SHARE_WORDS, dtype=torch.int64)
        self._counters, self._counters_h = self._pair(COUNTER_WORDS, dtype=torch.int64)
        self._ctl, self._ctl_h = self._pair(4, dtype=torch.int64)
        self._max, self._max_h = self._pair(1, dtype=torch.float64)
        self._alloc_world(max(info.world_size, 1))
        if not self.cuda:
            self.stream = None
        else:
            if stream_priority == "high":
                lo, hi = torch.cuda.Stream.priority_range()
                stream_priority = min(lo, hi)
            self.stream = torch.cuda.Stream(dev) if stream_priority is None else \
                torch.cuda.Stream(dev, priority=int(stream_priority))

    def _pair(self, *shape, dtype):
        """(device buffer, host mirror): the mirror is pinned on a GPU (async copies on the comm stream) and is the
        buffer itself on the CPU."""
        d = torch.zeros(*shape, dtype=dtype, device=self.dev)
        if not self.cuda:
            return d, d
        return d, torch.zeros(*shape, dtype=dtype, pin_memory=True)

    @property
    def multi(self) -> bool:
        """Collectives are issued: more than one rank, or forced at world 1."""
        return self.info.world_size > 1 or self.force

    def close(self) -> None:
        """Leave the process group at the end of the rank's life."""
        shutdown(self.info)

    def bind_thread(self) -> None:
        """Make the comm's GPU the calling thread's current device (the node's leader loop runs in a thread)."""
        if self.cuda:
            torch.cuda.set_device(self.info.device)

    def _alloc_world(self, world: int) -> None:
        self._gathered, self._gathered_h = self._pair(world, SHARE_SLOTS, SHARE_WORDS, dtype=torch.int64)
        self._counter_rows, self._counter_rows_h = self._pair(world, COUNTER_WORDS, dtype=torch.int64)

    # ---------------------------------------------------------------- group generations
    def abort(self) -> None:
        """Drop the current process group without waiting on it (a peer died)."""
        if not dist.is_initialized():
            return
        try:
            if self.info.backend == "nccl":
                from torch.distributed.distributed_c10d import _abort_process_group

                _abort_process_group()
            else:
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001 - the group is unusable either way
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001
                pass

    def reform(self, members: list[int], generation: int) -> None:
        """Leave the current group and form generation ``generation`` of the given orig ranks (this one included):
        group rank = position in ``members``. Every member calls this with the same arguments."""
        info = self.info
        if info.orig_rank not in members:
            raise ValueError(f"rank {info.orig_rank} is not a member of generation {generation}")
        self.abort()
        rank, world = members.index(info.orig_rank), len(members)
        if world > 1:
            kw = {"device_id": info.device, "pg_options": rccl_pg_options()} if info.backend == "nccl" else {}
            dist.init_process_group(backend=info.backend, rank=rank, world_size=world,
                                    store=dist.PrefixStore(f"otd-g{generation}", info.store),
                                    timeout=datetime.timedelta(seconds=PG_TIMEOUT_S), **kw)
        info.rank, info.world_size, info.generation, info.members = rank, world, generation, list(members)
        self._alloc_world(world)

    # ---------------------------------------------------------------- one op
    def _poll(self, done) -> None:
        """Wait for ``done()`` against the deadline: yield-only for the first 2 ms (a gather of the share slots
        completes in ~0.2 ms once every rank is in it), then 0.2 ms sleeps."""
        now = time.monotonic()
        end, spin_until = now + self.deadline, now + 0.002
        while not done():
            now = time.monotonic()
            if now > end:
                raise CollectiveTimeout(f"collective did not finish in {self.deadline:.1f} s")
            time.sleep(0.0 if now < spin_until else 0.0002)

    def _op(self, h2d: list, start, d2h: list) -> None:
        """One data-plane op: inputs staged host -> device, the collective ``start(async_op)``, results device ->
        host. ``h2d`` / ``d2h`` are (destination, source) pairs. Without a collective (world 1) the result is the
        input, copied on the host."""
        if not self.cuda:
            if self.multi:
                self._collect(start)
            return
        if self.staging == "legacy":  # copies on the caller's stream, the collective on the comm stream
            for d, h in h2d:
                d.copy_(h)
            if self.multi:
                self._collect(start)
            for h, d in d2h:
                h.copy_(d)
            return
        s = self.stream
        with torch.cuda.stream(s):
            for d, h in h2d:
                d.copy_(h, non_blocking=True)
            if self.multi:
                self.collectives += 1
                if self.bounded:
                    work = start(True)
                    self._poll(work.is_completed)
                    work.wait()  # re-raises a failed collective; the comm stream waits on RCCL's
                else:
                    start(False)
            for h, d in d2h:
                h.copy_(d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s)
        if self.bounded:
            self._poll(ev.query)
        else:
            ev.synchronize()

    def _collect(self, start) -> None:
        """Run one collective (CPU buffers, or the legacy staging). ``start(async_op)`` issues it; bounded mode polls
        the Work against the deadline."""
        self.collectives += 1
        if not self.bounded:
            self._run(lambda: start(False))
            return
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.info.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                work = start(True)
        else:
            work = start(True)
        self._poll(work.is_completed)
        work.wait()  # re-raises a failed collective (gloo: a peer's connection closed)
        if self.stream is not None:
            self.stream.synchronize()

    # ---------------------------------------------------------------- R1
    def broadcast_job(self, job: dict | None) -> dict | None:
        """Rank 0 passes the job dict (bytes values hex-encoded); all ranks get it back."""
        if self.info.is_primary:
            self._job_h.copy_(torch.frombuffer(bytearray(job_payload(job)), dtype=torch.uint8))
        if self.multi:
            self._op([(self._job, self._job_h)], lambda a: dist.broadcast(self._job, src=0, async_op=a),
                     [(self._job_h, self._job)])
        return job_from_payload(self._job_h.numpy().tobytes())

    # ---------------------------------------------------------------- R2
    def gather_shares(self, shares: list[dict], device_index: int = 0) -> list[dict]:
        """All-gather up to SHARE_SLOTS share records per rank; returns every rank's shares."""
        self._slots_h.copy_(torch.from_numpy(pack_shares(shares, self.info.rank, device_index)))
        if self.multi:
            self._op([(self._slots, self._slots_h)],
                     lambda a: dist.all_gather_into_tensor(self._gathered.view(-1, SHARE_WORDS), self._slots,
                                                           async_op=a),
                     [(self._gathered_h, self._gathered)])
        else:
            self._gathered_h[0].copy_(self._slots_h)
        return unpack_shares(self._gathered_h.numpy(), self.info.members)

    # ---------------------------------------------------------------- R3
    def allreduce_counters(self, hashes: int, shares: int = 0, dropped: int = 0, faults: int = 0) -> tuple:
        self._counters_h.copy_(torch.tensor([hashes, shares, dropped, faults], dtype=torch.int64))
        if self.multi:
            self._op([(self._counters, self._counters_h)],
                     lambda a: dist.all_reduce(self._counters, op=dist.ReduceOp.SUM, async_op=a),
                     [(self._counters_h, self._counters)])
        return tuple(int(x) for x in self._counters_h.tolist())

    def gather_counters(self, values: list[int]) -> list[list[int]]:
        """R3 variant for per-device stats: every rank's COUNTER_WORDS counters (all_gather, 32 B/rank)."""
        mine = torch.tensor(list(values)[:COUNTER_WORDS] + [0] * (COUNTER_WORDS - len(values)), dtype=torch.int64)
        self._counters_h.copy_(mine)
        if self.multi:
            self._op([(self._counters, self._counters_h)],
                     lambda a: dist.all_gather_into_tensor(self._counter_rows.view(-1), self._counters, async_op=a),
                     [(self._counter_rows_h, self._counter_rows)])
        else:
            self._counter_rows_h[0].copy_(self._counters_h)
        return self._counter_rows_h.tolist()

    def broadcast_control(self, words: list[int]) -> list[int]:
        """R1 control word (seq, stop, ...): 4 int64, every tick; the job blob follows only on change."""
        if self.info.is_primary:
            self._ctl_h.copy_(torch.tensor(list(words)[:4] + [0] * (4 - len(words)), dtype=torch.int64))
        if self.multi:
            self._op([(self._ctl, self._ctl_h)], lambda a: dist.broadcast(self._ctl, src=0, async_op=a),
                     [(self._ctl_h, self._ctl)])
        return self._ctl_h.tolist()

    def allreduce_max(self, value: float) -> float:
        self._max_h.fill_(value)
        if self.multi:
            self._op([(self._max, self._max_h)],
                     lambda a: dist.all_reduce(self._max, op=dist.ReduceOp.MAX, async_op=a),
                     [(self._max_h, self._max)])
        return float(self._max_h.item())

    def barrier(self) -> None:
        if self.bounded and self.info.world_size > 1 and self.info.backend != "nccl":
            self._bounded(dist.barrier(async_op=True))
        else:
            barrier(self.info)

    def _bounded(self, work) -> None:
        """Wait for an async collective against the deadline (CollectiveTimeout), re-raising its failure."""
        self._poll(work.is_completed)
        work.wait()

    # ---------------------------------------------------------------- device-resident forms (bench.py)
    def gather_tensor(self, out, inp) -> None:
        """``out`` (world x inp.shape) gets every rank's contiguous ``inp`` (parallel/rcclcomm.py has the same).
        ``bounded``: the collective is polled against the deadline instead of blocking."""
        if self.info.world_size > 1:
            self.collectives += 1
            if self.bounded:
                self._bounded(dist.all_gather_into_tensor(out.view(-1), inp.view(-1), async_op=True))
            else:
                dist.all_gather_into_tensor(out.view(-1), inp.view(-1))
        else:
            out[0].copy_(inp)

    def broadcast_tensor(self, t, src: int = 0) -> None:
        if self.info.world_size > 1:
            self.collectives += 1
            if self.bounded:
                self._bounded(dist.broadcast(t, src=src, async_op=True))
            else:
                dist.broadcast(t, src=src)

    def _run(self, fn) -> None:
        """Blocking form: the collective runs on the comm stream and the current stream waits for it (used where
        the caller reads the result right away)."""
        if self.stream is None:
            fn()
            return
        cur = torch.cuda.current_stream(self.info.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
        cur.wait_stream(self.stream)

    def run_async(self, fn):
        """Overlapped form: the collective is ordered after the work already queued on the current stream (its
        producer) but nothing on the current stream waits for it. Returns an event recorded on the comm stream
        (``None`` on CPU, where gloo collectives complete inline); a consumer, or the producer that reuses the
        collective's buffers, waits on that event only when it needs to."""
        if self.stream is None:
            fn()
            return None
        cur = torch.cuda.current_stream(self.info.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev


def rccl_pg_options():
    """ProcessGroupNCCL options for the node's groups: RCCL's internal streams at high priority, so a collective's
    kernel is dispatched ahead of the mining grid of the sibling device process (OTEDAMA_RCCL_HIGH_PRIORITY=0 turns
    it off)."""
    if os.environ.get("OTEDAMA_RCCL_HIGH_PRIORITY", "1") == "0":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except Exception:  # noqa: BLE001 - a torch without the NCCL backend
        return None
