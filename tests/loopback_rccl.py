"""A stand-in for ``otedama_amd._rccl`` that runs on CPUs: the same module API (``unique_id``, ``RcclComm`` with
``broadcast`` / ``all_gather`` / ``all_reduce`` / ``abort``), its collectives carried by the node's store.

The native data plane's Python side (parallel/rcclcomm.py: the unique-id exchange per generation, the all-ranks-together
choice, timeouts turned into CollectiveTimeout, aborts and re-forms after a lost rank) cannot run at world > 1 on the
one-GPU box: RCCL refuses two ranks on one device ("Duplicate GPU detected"). With ``OTEDAMA_RCCL_MODULE=loopback_rccl``
the node's ranks load this module instead, so that protocol runs end to end at world 4 and 8 on CPUs
(tests/test_rccl_loopback_node.py). The semantics that matter are kept:
  * init waits for all ``nranks`` members of the id (RCCL's bootstrap) and fails after ``timeout_s``;
  * an op completes only when every member has entered it; a dead peer makes it raise TimeoutError after its
    deadline (what ``RcclTimeout`` is on the native module);
  * an op that failed (a timeout) leaves the communicator broken: every later op raises RuntimeError until an abort;
  * ``abort`` is immediate and every later op raises RuntimeError.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np

from otedama_amd.parallel.kvclient import StoreClient

DEVICE_TYPE = "cpu"  # rcclcomm gives the rank a CPU device: its miners are the host chains
UNIQUE_ID_BYTES = 128


def unique_id() -> bytes:
    return os.urandom(UNIQUE_ID_BYTES)


def version() -> str:
    return "loopback"


class RcclComm:
    def __init__(self, device: int, nranks: int, rank: int, unique_id: bytes, timeout_s: float):
        if len(unique_id) != UNIQUE_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        if nranks < 1 or not 0 <= rank < nranks:
            raise ValueError("bad rank / nranks")
        self.nranks, self.rank = nranks, rank
        self._p = "lb/" + unique_id[:8].hex()
        self._store = StoreClient(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                                  timeout=30.0)
        self._seq = 0
        self._ops = 0
        self._alive = True
        self._broken = False
        self._store.set(f"{self._p}/join/{rank}", b"1")
        try:
            self._wait([f"{self._p}/join/{r}" for r in range(nranks)], timeout_s, "init")
        except Exception:
            self.abort()
            raise

    @property
    def alive(self) -> bool:
        return self._alive

    @property
    def ops(self) -> int:
        return self._ops

    def abort(self) -> None:
        if self._alive:
            self._alive = False
            try:
                self._store.close()
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------------------------------------------ internals
    def _wait(self, keys: list[str], timeout_s: float, what: str) -> None:
        end = time.monotonic() + timeout_s
        while not self._store.check(keys):
            if not self._alive:
                raise RuntimeError("rccl: communicator aborted")
            if time.monotonic() > end:
                raise TimeoutError(f"{what} did not finish in {timeout_s} s")
            time.sleep(0.0005)

    def _exchange(self, mine: bytes | None, senders: list[int], timeout_s: float, what: str) -> list[bytes]:
        if not self._alive:
            raise RuntimeError("rccl: communicator aborted")
        if self._broken:
            raise RuntimeError("rccl: an earlier op timed out; abort this communicator and re-form")
        s = self._seq
        self._seq += 1
        # every member has set its op s-1 key before anyone reaches op s+1, so op s-1's keys are read by now
        if s >= 2 and self.rank in senders:
            self._store.delete_key(f"{self._p}/{s - 2}/{self.rank}")
        self._store.set(f"{self._p}/{s}/{self.rank}", mine if mine is not None else b"")
        keys = [f"{self._p}/{s}/{r}" for r in range(self.nranks)]
        try:
            self._wait(keys, timeout_s, what)  # every member entered the op (a barrier, as a collective is)
        except TimeoutError:
            self._broken = True
            raise
        self._ops += 1
        return [self._store.get(f"{self._p}/{s}/{r}") for r in senders]

    # ------------------------------------------------------------------------------------------------ ops
    def broadcast(self, data: bytes, nbytes: int, root: int, timeout_s: float) -> bytes:
        if self.rank == root and len(data) != nbytes:
            raise ValueError("root's data must be nbytes long")
        got = self._exchange(bytes(data) if self.rank == root else b"", list(range(self.nranks)), timeout_s,
                             "broadcast")
        return got[root]

    def all_gather(self, mine: bytes, timeout_s: float) -> bytes:
        got = self._exchange(bytes(mine), list(range(self.nranks)), timeout_s, "all_gather")
        if len({len(g) for g in got}) != 1:
            raise RuntimeError("all_gather: contributions differ in length")
        return b"".join(got)

    def all_reduce(self, data: bytes, dtype: str, op: str, timeout_s: float) -> bytes:
        if dtype not in ("i64", "f64") or op not in ("sum", "max"):
            raise ValueError("dtype must be i64/f64 and op sum/max")
        got = self._exchange(bytes(data), list(range(self.nranks)), timeout_s, "all_reduce")
        a = np.stack([np.frombuffer(g, dtype=np.int64 if dtype == "i64" else np.float64) for g in got])
        return (a.sum(axis=0) if op == "sum" else a.max(axis=0)).tobytes()

    # "device" forms: here the pointers are host memory (CPU tensors' data_ptr()); the stream is ignored and the op
    # completes before it returns (a CPU rehearsal of bench.py's device-resident R1 / R2 / R3)
    def all_gather_dev(self, send: int, recv: int, nbytes: int, stream: int, timeout_s: float) -> None:
        out = self.all_gather(ctypes.string_at(send, nbytes), timeout_s)
        ctypes.memmove(recv, out, len(out))

    def broadcast_dev(self, buf: int, nbytes: int, root: int, stream: int, timeout_s: float) -> None:
        out = self.broadcast(ctypes.string_at(buf, nbytes) if self.rank == root else b"", nbytes, root, timeout_s)
        ctypes.memmove(buf, out, nbytes)

    def all_reduce_dev(self, buf: int, count: int, dtype: str, op: str, stream: int, timeout_s: float) -> None:
        out = self.all_reduce(ctypes.string_at(buf, 8 * count), dtype, op, timeout_s)
        ctypes.memmove(buf, out, 8 * count)
