"""The node data plane's torch-free pieces: record layouts, the rank/generation descriptor and the job-blob codec.

Shared by the two data-plane implementations: ``parallel/comm.py`` (torch.distributed: gloo on CPU hosts and
rehearsals, the bench's own collectives) and ``parallel/rcclcomm.py`` (the node's native RCCL path on GPUs, which
keeps torch out of the rank processes). SURVEY §2.3 names the three collectives: R1 job broadcast, R2 share gather,
R3 counters.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

JOB_BLOB_BYTES = 64 << 10  # a real V1 job (coinbase parts + 12 merkle branches, hex in JSON) can pass 4 KiB
SHARE_SLOTS = 64
# epoch_lo, epoch_hi|valid, nonce, ntime, version, en2_lo, en2_hi, rank|device, found_at_us, device_found_at_us
# (both times CLOCK_MONOTONIC, which every process of the host shares: the leader computes the kernel-hit -> accept
# latency of a remote rank's share directly)
SHARE_WORDS = 10
COUNTER_WORDS = 4  # hashes, shares, dropped, faulted

PG_TIMEOUT_S = float(os.environ.get("OTEDAMA_PG_TIMEOUT", "30"))


class CollectiveTimeout(RuntimeError):
    """A bounded collective did not finish in time (a peer is dead or stuck)."""


@dataclass
class Device:
    """torch.device's two fields, for processes without torch (the native RCCL node ranks)."""
    type: str = "cpu"
    index: int | None = None


@dataclass
class DistInfo:
    rank: int = 0            # rank in the current process group
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"    # "nccl" / "gloo" (torch.distributed), "rccl" (native), "none"
    device: object = field(default_factory=Device)  # torch.device or Device
    orig_rank: int = -1      # launcher-assigned identity (RANK at start); stable across re-forms
    generation: int = 0      # process-group generation (store prefix otd-g<gen>)
    members: list = field(default_factory=list)  # orig ranks of the current group, in group-rank order
    store: object = None     # the rendezvous TCPStore (node control plane)
    capacity: int = 0        # ranks the node was launched with (WORLD_SIZE at start; orig ranks 0..capacity-1)

    def __post_init__(self):
        if self.orig_rank < 0:
            self.orig_rank = self.rank
        if not self.members:
            self.members = list(range(self.world_size))
        if self.capacity <= 0:
            self.capacity = max(self.world_size, 1)

    @property
    def is_primary(self) -> bool:
        return self.rank == 0


def pack_shares(shares: list[dict], rank: int, device_index: int = 0) -> np.ndarray:
    """R2 record array of up to SHARE_SLOTS shares (SHARE_SLOTS x SHARE_WORDS int64; unused rows are all zero)."""
    rows = np.zeros((SHARE_SLOTS, SHARE_WORDS), dtype=np.int64)
    for i, s in enumerate(shares[:SHARE_SLOTS]):
        e = int(s.get("epoch", 0))
        en2 = int(s.get("extranonce2", 0))
        rows[i] = (e & 0xFFFFFFFF, (e >> 32) | (1 << 31), s["nonce"], s.get("ntime", 0), s.get("version", 0),
                   en2 & 0xFFFFFFFF, en2 >> 32, (rank << 16) | device_index,
                   int(s.get("found_at", 0.0) * 1e6), int((s.get("device_found_at", 0.0) or 0.0) * 1e6))
    return rows


def unpack_shares(g: np.ndarray, members: list) -> list[dict]:
    """Every valid record of a gathered (world x SHARE_SLOTS x SHARE_WORDS) array, in rank then slot order."""
    out = []
    for r, i in zip(*np.nonzero(g[:, :, 1] >> 31)):
        r, rec = int(r), g[r, i].tolist()
        out.append({
            "epoch": rec[0] | ((rec[1] & 0x7FFFFFFF) << 32), "nonce": rec[2] & 0xFFFFFFFF,
            "ntime": rec[3] & 0xFFFFFFFF, "version": rec[4] & 0xFFFFFFFF,
            "extranonce2": (rec[5] & 0xFFFFFFFF) | (rec[6] << 32), "rank": rec[7] >> 16,
            "device_index": rec[7] & 0xFFFF, "found_at": rec[8] / 1e6, "device_found_at": rec[9] / 1e6,
            "orig_rank": members[r] if r < len(members) else r,
        })
    return out


def job_payload(job: dict | None) -> bytes:
    """The R1 blob: 4-byte length + the job as JSON (bytes values hex-encoded), padded to JOB_BLOB_BYTES."""
    import json

    payload = json.dumps(_encode(job)).encode() if job is not None else b""
    if len(payload) + 4 > JOB_BLOB_BYTES:
        raise ValueError(f"job blob too large for broadcast ({len(payload)} bytes)")
    return (len(payload).to_bytes(4, "little") + payload).ljust(JOB_BLOB_BYTES, b"\0")


def job_from_payload(buf: bytes) -> dict | None:
    import json

    n = int.from_bytes(buf[:4], "little")
    if n == 0:
        return None
    return _decode(json.loads(buf[4 : 4 + n].decode()))


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
