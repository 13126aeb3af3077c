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
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

JOB_BLOB_BYTES = 64 << 10  # a real V1 job (coinbase parts + 12 merkle branches, hex in JSON) can pass 4 KiB
SHARE_SLOTS = 64
SHARE_WORDS = 9  # epoch_lo, epoch_hi|valid, nonce, ntime, version, en2_lo, en2_hi, rank|device, found_at_us
COUNTER_WORDS = 4  # hashes, shares, dropped, faulted


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_primary(self) -> bool:
        return self.rank == 0


def init_from_env(backend: str | None = None, use_gpu: bool | None = None) -> DistInfo:
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
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return DistInfo(rank, world, local, backend, device)


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
    """R1/R2/R3 over torch.distributed with preallocated fixed-size buffers."""

    def __init__(self, info: DistInfo):
        self.info = info
        dev = info.device
        self._job = torch.zeros(JOB_BLOB_BYTES, dtype=torch.uint8, device=dev)
        self._slots = torch.zeros(SHARE_SLOTS, SHARE_WORDS, dtype=torch.int64, device=dev)
        self._gathered = torch.zeros(info.world_size, SHARE_SLOTS, SHARE_WORDS, dtype=torch.int64, device=dev)
        self._counters = torch.zeros(COUNTER_WORDS, dtype=torch.int64, device=dev)
        self._counter_rows = torch.zeros(info.world_size, COUNTER_WORDS, dtype=torch.int64, device=dev)
        self._ctl = torch.zeros(4, dtype=torch.int64, device=dev)
        self.stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None

    # ---------------------------------------------------------------- R1
    def broadcast_job(self, job: dict | None) -> dict | None:
        """Rank 0 passes the job dict (bytes values hex-encoded); all ranks get it back."""
        if self.info.is_primary:
            payload = json.dumps(_encode(job)).encode() if job is not None else b""
            if len(payload) + 4 > JOB_BLOB_BYTES:
                raise ValueError(f"job blob too large for broadcast ({len(payload)} bytes)")
            buf = len(payload).to_bytes(4, "little") + payload
            host = torch.zeros(JOB_BLOB_BYTES, dtype=torch.uint8)
            host[: len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
            self._job.copy_(host)
        if self.info.world_size > 1:
            self._run(lambda: dist.broadcast(self._job, src=0))
        host = self._job.cpu().numpy().tobytes()
        n = int.from_bytes(host[:4], "little")
        if n == 0:
            return None
        return _decode(json.loads(host[4 : 4 + n].decode()))

    # ---------------------------------------------------------------- R2
    def gather_shares(self, shares: list[dict], device_index: int = 0) -> list[dict]:
        """All-gather up to SHARE_SLOTS share records per rank; returns every rank's shares."""
        host = torch.zeros(SHARE_SLOTS, SHARE_WORDS, dtype=torch.int64)
        for i, s in enumerate(shares[:SHARE_SLOTS]):
            e = int(s.get("epoch", 0))
            en2 = int(s.get("extranonce2", 0))
            host[i] = torch.tensor([
                e & 0xFFFFFFFF, (e >> 32) | (1 << 31), s["nonce"], s.get("ntime", 0), s.get("version", 0),
                en2 & 0xFFFFFFFF, en2 >> 32, (self.info.rank << 16) | device_index,
                int(s.get("found_at", 0.0) * 1e6),
            ], dtype=torch.int64)
        self._slots.copy_(host)
        if self.info.world_size > 1:
            self._run(lambda: dist.all_gather_into_tensor(self._gathered.view(-1, SHARE_WORDS), self._slots))
        else:
            self._gathered[0].copy_(self._slots)
        out = []
        g = self._gathered.cpu().tolist()
        for r in range(self.info.world_size):
            for rec in g[r]:
                if not rec[1] >> 31:
                    continue
                out.append({
                    "epoch": rec[0] | ((rec[1] & 0x7FFFFFFF) << 32), "nonce": rec[2] & 0xFFFFFFFF,
                    "ntime": rec[3] & 0xFFFFFFFF, "version": rec[4] & 0xFFFFFFFF,
                    "extranonce2": (rec[5] & 0xFFFFFFFF) | (rec[6] << 32), "rank": rec[7] >> 16,
                    "device_index": rec[7] & 0xFFFF, "found_at": rec[8] / 1e6,
                })
        return out

    # ---------------------------------------------------------------- R3
    def allreduce_counters(self, hashes: int, shares: int = 0, dropped: int = 0, faults: int = 0) -> tuple:
        self._counters.copy_(torch.tensor([hashes, shares, dropped, faults], dtype=torch.int64))
        if self.info.world_size > 1:
            self._run(lambda: dist.all_reduce(self._counters, op=dist.ReduceOp.SUM))
        return tuple(int(x) for x in self._counters.cpu().tolist())

    def gather_counters(self, values: list[int]) -> list[list[int]]:
        """R3 variant for per-device stats: every rank's COUNTER_WORDS counters (all_gather, 32 B/rank)."""
        mine = torch.tensor(list(values)[:COUNTER_WORDS] + [0] * (COUNTER_WORDS - len(values)), dtype=torch.int64)
        self._counters.copy_(mine)
        if self.info.world_size > 1:
            self._run(lambda: dist.all_gather_into_tensor(self._counter_rows.view(-1), self._counters))
        else:
            self._counter_rows[0].copy_(self._counters)
        return self._counter_rows.cpu().tolist()

    def broadcast_control(self, words: list[int]) -> list[int]:
        """R1 control word (seq, stop, ...): 4 int64, every tick; the job blob follows only on change."""
        if self.info.is_primary:
            self._ctl.copy_(torch.tensor(list(words)[:4] + [0] * (4 - len(words)), dtype=torch.int64))
        if self.info.world_size > 1:
            self._run(lambda: dist.broadcast(self._ctl, src=0))
        return self._ctl.cpu().tolist()

    def allreduce_max(self, value: float) -> float:
        t = torch.tensor([value], dtype=torch.float64, device=self.info.device)
        if self.info.world_size > 1:
            self._run(lambda: dist.all_reduce(t, op=dist.ReduceOp.MAX))
        return float(t.item())

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


def _encode(obj):
    if isinstance(obj, bytes):
        return {"__b": obj.hex()}
    if isinstance(obj, dict):
        return {k: _encode(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_encode(v) for v in obj]
    return obj


def _decode(obj):
    if isinstance(obj, dict):
        if set(obj) == {"__b"}:
            return bytes.fromhex(obj["__b"])
        return {k: _decode(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_decode(v) for v in obj]
    return obj
