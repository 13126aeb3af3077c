"""Pool-protocol abstraction: scheme registry, jobs, share submissions, sessions.

Parity: internal/poolproto/poolproto.go
  * ProtocolID / FromURL / knownSchemes / StripScheme ..... poolproto.go:73-133
  * Job / ShareSubmission / ShareResult ................... poolproto.go:140-189
  * Connection / Session / PoolNoticeReceiver / Dialer .... poolproto.go:195-259
  * Credentials ........................................... poolproto.go:262-279
  * Register / Lookup / Available / DialURL ............... poolproto.go:290-353
  * ErrUnknownProtocol / ErrHandshakeFailed / ErrShareRejected

Differences by design: a Job carries everything needed to build
headers — the V1 coinbase parts and merkle branches (the reference drops them,
so its V1 shares hash MerkleRoot=0) — plus the share target and negotiated
BIP320 version mask; job ids are opaque strings. Sessions are asyncio objects.
"""
from __future__ import annotations

import abc
import asyncio
import time
from dataclasses import dataclass, field
from enum import Enum


class PoolProtoError(Exception):
    pass


class UnknownProtocol(PoolProtoError):
    pass


class HandshakeFailed(PoolProtoError):
    pass


class ShareRejected(PoolProtoError):
    pass


class FatalPoolError(PoolProtoError):
    """Stops the reconnect loop (e.g. SetupConnectionError; engine/run.go:1196-1198)."""


class ProtocolID(str, Enum):
    STRATUM_V1 = "stratum-v1"
    STRATUM_V1_TLS = "stratum-v1-tls"
    STRATUM_V2 = "stratum-v2"
    STRATUM_V2_TLS = "stratum-v2-tls"
    DATUM = "datum"
    UNKNOWN = ""

    def post_quantum_ready(self) -> bool:
        return False

    @property
    def uses_tls(self) -> bool:
        return self in (ProtocolID.STRATUM_V1_TLS, ProtocolID.STRATUM_V2_TLS)


KNOWN_SCHEMES = (
    ("stratum+v2tls://", ProtocolID.STRATUM_V2_TLS),
    ("stratum+v2://", ProtocolID.STRATUM_V2),
    ("stratum+tls://", ProtocolID.STRATUM_V1_TLS),
    ("stratum+tcp://", ProtocolID.STRATUM_V1),
    ("datum://", ProtocolID.DATUM),
)


def from_url(url: str) -> ProtocolID:
    for prefix, proto in KNOWN_SCHEMES:
        if url.startswith(prefix):
            return proto
    return ProtocolID.UNKNOWN


def strip_scheme(url: str) -> str:
    for prefix, _ in KNOWN_SCHEMES:
        if len(url) > len(prefix) and url.startswith(prefix):
            return url[len(prefix):]
    raise UnknownProtocol(f"poolproto: unknown protocol: {url!r}")


def split_host_port(hostport: str, default_port: int) -> tuple[str, int]:
    hostport = hostport.split("/", 1)[0]
    if hostport.startswith("["):
        host, _, rest = hostport[1:].partition("]")
        port = rest.lstrip(":")
        return host, int(port) if port else default_port
    host, sep, port = hostport.rpartition(":")
    if not sep:
        return hostport, default_port
    return host, int(port)


def extranonce2_bytes(value: int, size: int) -> bytes:
    """Wire bytes of a rolled extranonce2: little-endian, exactly `size` bytes. The native runtime rolls at most the
    low 8 bytes and zero-fills the rest of the coinbase field (csrc/runtime/miner_common.cpp
    merkle_root_from_coinbase), so a pool asking for extranonce2_size > 8 gets the same zero padding here."""
    if size <= 0:
        return b""
    return (value & 0xFFFFFFFFFFFFFFFF).to_bytes(max(8, size), "little")[:size]


@dataclass
class Job:
    job_id: str
    version: int = 0
    prev_hash: bytes = bytes(32)          # header byte order
    merkle_root: bytes | None = None      # fixed root (SV2 standard channel); None when built from coinbase
    ntime: int = 0
    nbits: int = 0
    clean_jobs: bool = False
    received_at: float = field(default_factory=time.time)
    target: bytes | None = None           # share target (LE, MSB at [31])
    version_mask: int = 0                 # negotiated BIP320 rollable bits
    channel_id: int = 0
    # Stratum V1 coinbase construction
    coinb1: bytes | None = None
    coinb2: bytes | None = None
    extranonce1: bytes = b""
    extranonce2_size: int = 0
    merkle_branches: list[bytes] = field(default_factory=list)
    algorithm: str = "sha256d"

    def header_prefix(self, merkle_root: bytes) -> bytes:
        import struct

        return (struct.pack("<I", self.version & 0xFFFFFFFF) + self.prev_hash + merkle_root
                + struct.pack("<II", self.ntime & 0xFFFFFFFF, self.nbits & 0xFFFFFFFF))

    def template(self) -> dict:
        """Native-runtime job template (see csrc/include/otedama/runtime.h)."""
        root = self.merkle_root if self.merkle_root is not None else bytes(32)
        t = {
            "header": self.header_prefix(root) + bytes(4),
            "target": self.target or b"\xff" * 32,
            "job_id": self.job_id,
            "channel_id": self.channel_id,
            "version_mask": self.version_mask,
            "algo": self.algorithm,
        }
        if self.coinb1 is not None:
            t.update(coinb1=self.coinb1, coinb2=self.coinb2 or b"", extranonce1=self.extranonce1,
                     extranonce2_size=self.extranonce2_size, merkle_branches=list(self.merkle_branches))
        return t


@dataclass
class ShareSubmission:
    job_id: str
    nonce: int
    ntime: int
    version: int = 0
    extranonce2: bytes = b""
    worker: str = ""


@dataclass
class ShareResult:
    accepted: bool
    reason: str = ""
    difficulty: float = 0.0
    latency_ms: float = 0.0


@dataclass
class Credentials:
    user: str = ""
    password: str = ""
    pool_pubkey: bytes = b""
    tls_root_cas_pem: bytes = b""
    worker: str = ""
    version_rolling: bool = True
    vendor: str = "Otedama"
    hardware: str = "v3.0.0"
    firmware: str = "main"
    device: str = "gfx950"
    nominal_hashrate: float = 0.0
    extended_channel: bool = False   # SV2: open an extended channel and roll extranonce under the pool's prefix
    noise: bool = False              # SV2: Noise NX channel encryption (implied by a pinned pool_pubkey)
    noise_suite: str = "ellswift"    # SV2 Noise suite: "ellswift" (BIP324 encodings, current spec) | "legacy"


class Session(abc.ABC):
    """A negotiated pool session. ``jobs`` yields Job, or None = pause (no valid work)."""

    jobs: asyncio.Queue
    notices: asyncio.Queue

    @abc.abstractmethod
    async def submit(self, sub: ShareSubmission, timeout: float = 30.0) -> ShareResult:
        ...

    @abc.abstractmethod
    def suggested_difficulty(self) -> float:
        ...

    @abc.abstractmethod
    async def close(self) -> None:
        ...

    @property
    @abc.abstractmethod
    def closed(self) -> bool:
        ...

    @property
    def protocol(self) -> ProtocolID:
        return ProtocolID.UNKNOWN

    @property
    def remote_addr(self) -> str:
        return ""

    async def wait_closed(self) -> None:
        while not self.closed:
            await asyncio.sleep(0.05)


class Dialer(abc.ABC):
    @property
    @abc.abstractmethod
    def protocol(self) -> ProtocolID:
        ...

    @abc.abstractmethod
    async def dial(self, url: str, creds: Credentials, timeout: float = 10.0) -> Session:
        """Connect and negotiate; returns a live session."""


_registry: dict[ProtocolID, Dialer] = {}


def register(d: Dialer) -> None:
    if d is None:
        raise PoolProtoError("poolproto: Register called with nil Dialer")
    if d.protocol == ProtocolID.UNKNOWN:
        raise PoolProtoError("poolproto: Dialer returned ProtocolUnknown")
    if d.protocol in _registry:
        raise PoolProtoError(f"poolproto: protocol {d.protocol.value!r} already registered")
    _registry[d.protocol] = d


def lookup(pid: ProtocolID) -> Dialer:
    try:
        return _registry[pid]
    except KeyError:
        raise UnknownProtocol(f"poolproto: unknown protocol: {pid.value!r}") from None


def available() -> list[ProtocolID]:
    return list(_registry)


async def dial_url(url: str, creds: Credentials, timeout: float = 10.0) -> Session:
    proto = from_url(url)
    if proto == ProtocolID.UNKNOWN:
        raise UnknownProtocol(f"poolproto: unknown protocol: cannot infer protocol from {url!r}")
    return await lookup(proto).dial(url, creds, timeout=timeout)


def put_drop_oldest(q: asyncio.Queue, item) -> None:
    """Non-blocking send that drops the oldest queued item when full (stratumv1.go:299-325)."""
    try:
        q.put_nowait(item)
    except asyncio.QueueFull:
        try:
            q.get_nowait()
        except asyncio.QueueEmpty:
            pass
        try:
            q.put_nowait(item)
        except asyncio.QueueFull:
            pass
