"""Stratum V1 (JSON-RPC over newline-delimited TCP/TLS) client.

Parity: internal/poolproto/stratumv1/{stratumv1,parse,dialer,tls}.go
  * session / readLoop with 5-minute read deadline ....... stratumv1.go:77-174
  * 64 KiB line cap (misbehaving pool -> session ends) ... stratumv1.go:73,183-194
  * dispatch: responses by id; mining.notify (clean_jobs
    purges queued jobs, drop-oldest), set_difficulty,
    set_extranonce, client.show_message, client.reconnect
    / mining.reconnect (host NOT followed) ............... stratumv1.go:209-325
  * call(): id-correlated pending map, 10 s write deadline stratumv1.go:418-458
  * Negotiate: subscribe -> authorize (must be true) ->
    extranonce.subscribe (errors tolerated) .............. dialer.go:109-174
  * parseNotify / parseDifficulty / parseSetExtranonce /
    parseShowMessage / parseReconnect / parseSubscribeResult  parse.go:33-204

Reference defects fixed: the coinbase parts and merkle branches
are kept (the reference hashes MerkleRoot=0), prev-hash words are converted to
header byte order, job ids stay opaque strings, the configured worker name and
the rolled extranonce2 are submitted, BIP310 version rolling is negotiated via
mining.configure and the rolled bits are submitted as the 6th parameter.
"""
from __future__ import annotations

import asyncio
import dataclasses
import json
import math
import time

from otedama_amd.models.header import target_from_difficulty
from otedama_amd.poolproto.base import (
    Credentials,
    Dialer,
    FatalPoolError,
    HandshakeFailed,
    Job,
    PoolProtoError,
    ProtocolID,
    Session,
    ShareResult,
    ShareSubmission,
    put_drop_oldest,
    register,
    split_host_port,
    strip_scheme,
)
from otedama_amd.stratum import tls

MAX_LINE_BYTES = 64 << 10
READ_DEADLINE = 300.0
WRITE_DEADLINE = 10.0
BIP320_MASK = 0x1FFFE000
MAX_EXTRANONCE2_SIZE = 32  # bytes; a larger (or negative) size from a pool is treated as malformed
USER_AGENT = "Otedama/3.0.0-mi355x"


def prevhash_from_stratum(hexstr: str) -> bytes:
    """mining.notify prevhash (8 byte-swapped 32-bit words) -> header byte order."""
    b = bytes.fromhex(hexstr)
    if len(b) != 32:
        raise ValueError("prevhash must be 32 bytes")
    return b"".join(b[i:i + 4][::-1] for i in range(0, 32, 4))


def prevhash_to_stratum(header_prev: bytes) -> str:
    return b"".join(header_prev[i:i + 4][::-1] for i in range(0, 32, 4)).hex()


def parse_notify(params) -> Job:
    if not isinstance(params, list) or len(params) < 9:
        raise ValueError(f"notify: expected 9 params, got {len(params) if isinstance(params, list) else 'non-list'}")
    job_id, prev, coinb1, coinb2, branches, version, nbits, ntime, clean = params[:9]
    if not isinstance(job_id, str):
        job_id = str(job_id)
    if isinstance(clean, bool):
        clean_jobs = clean
    elif isinstance(clean, (int, float)):
        clean_jobs = clean != 0
    else:
        raise ValueError("notify: clean_jobs must be bool or number")
    return Job(
        job_id=job_id,
        version=int(version, 16) & 0xFFFFFFFF,
        prev_hash=prevhash_from_stratum(prev),
        ntime=int(ntime, 16) & 0xFFFFFFFF,
        nbits=int(nbits, 16) & 0xFFFFFFFF,
        clean_jobs=clean_jobs,
        coinb1=bytes.fromhex(coinb1),
        coinb2=bytes.fromhex(coinb2),
        merkle_branches=[bytes.fromhex(b) for b in branches],
    )


def parse_difficulty(params) -> float | None:
    if isinstance(params, list) and params and isinstance(params[0], (int, float)) and not isinstance(params[0], bool):
        return float(params[0])
    return None


def parse_set_extranonce(params):
    if isinstance(params, list) and len(params) >= 2 and isinstance(params[0], str) and isinstance(params[1], int):
        return params[0], params[1]
    return None


def parse_show_message(params) -> str | None:
    if isinstance(params, list) and params and isinstance(params[0], str):
        return params[0]
    return None


def parse_reconnect(params) -> dict:
    d = {"host": "", "port": 0, "wait": 0}
    if not isinstance(params, list):
        return d
    if len(params) >= 1 and isinstance(params[0], str):
        d["host"] = params[0]
    if len(params) >= 2:
        p = params[1]
        if isinstance(p, int):
            d["port"] = p
        elif isinstance(p, str) and p.isdigit():
            d["port"] = int(p)
    if len(params) >= 3 and isinstance(params[2], int):
        d["wait"] = params[2]
    return d


def parse_subscribe_result(result) -> tuple[str, int]:
    if not isinstance(result, list) or len(result) < 3:
        raise HandshakeFailed(f"stratumv1: unexpected subscribe result ({type(result).__name__})")
    en1, size = result[1], result[2]
    if not isinstance(en1, str):
        raise HandshakeFailed(f"stratumv1: extranonce1 not a string: {type(en1).__name__}")
    if not isinstance(size, (int, float)) or isinstance(size, bool):
        raise HandshakeFailed(f"stratumv1: extranonce2_size not a number: {type(size).__name__}")
    if not 0 <= size <= MAX_EXTRANONCE2_SIZE or size != int(size):
        raise HandshakeFailed(f"stratumv1: extranonce2_size {size} out of range [0, {MAX_EXTRANONCE2_SIZE}]")
    try:
        bytes.fromhex(en1)
    except ValueError:
        raise HandshakeFailed(f"stratumv1: extranonce1 is not hex: {en1[:32]!r}") from None
    return en1, int(size)


class V1Session(Session):
    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter, creds: Credentials,
                 protocol: ProtocolID, algorithm: str = "sha256d"):
        self.reader, self.writer = reader, writer
        self.creds = creds
        self._protocol = protocol
        self.algorithm = algorithm
        self.jobs: asyncio.Queue = asyncio.Queue(maxsize=8)
        self.notices: asyncio.Queue = asyncio.Queue(maxsize=8)
        self._pending: dict[int, asyncio.Future] = {}
        self._next_id = 0
        self._difficulty = 0.0
        self.extranonce1 = b""
        self.extranonce2_size = 0
        self.version_mask = 0
        self.last_reconnect: dict | None = None
        self._closed = False
        self._write_lock = asyncio.Lock()
        self._task: asyncio.Task | None = None
        self.last_job: Job | None = None
        self._job_versions: dict[str, int] = {}  # job id -> notify version (BIP310 submit param), bounded

    @property
    def protocol(self) -> ProtocolID:
        return self._protocol

    @property
    def remote_addr(self) -> str:
        peer = self.writer.get_extra_info("peername")
        return f"{peer[0]}:{peer[1]}" if peer else ""

    @property
    def closed(self) -> bool:
        return self._closed

    def start(self) -> None:
        self._task = asyncio.ensure_future(self._read_loop())

    async def _read_line(self) -> bytes:
        try:
            line = await asyncio.wait_for(self.reader.readuntil(b"\n"), READ_DEADLINE)
        except asyncio.LimitOverrunError as exc:
            raise PoolProtoError(f"stratumv1: line exceeds {MAX_LINE_BYTES} bytes; terminating session "
                                 "(misbehaving pool)") from exc
        if len(line) > MAX_LINE_BYTES:
            raise PoolProtoError(f"stratumv1: line exceeds {MAX_LINE_BYTES} bytes; terminating session")
        return line

    async def _read_loop(self) -> None:
        try:
            while not self._closed:
                line = await self._read_line()
                self._dispatch(line)
        except (asyncio.IncompleteReadError, asyncio.TimeoutError, ConnectionError, PoolProtoError, OSError):
            pass
        finally:
            await self._teardown()

    def _dispatch(self, line: bytes) -> None:
        line = line.rstrip(b"\r\n")
        if not line:
            return
        try:
            msg = json.loads(line)
        except (ValueError, UnicodeDecodeError):
            return
        if not isinstance(msg, dict):
            return
        method = msg.get("method")
        if not method and msg.get("id") is not None:
            try:
                mid = int(msg["id"])
            except (TypeError, ValueError):
                return
            fut = self._pending.pop(mid, None)
            if fut is not None and not fut.done():
                fut.set_result((msg.get("result"), msg.get("error")))
            return
        try:
            self._dispatch_method(method, msg.get("params"))
        except (ValueError, TypeError, OverflowError):
            return  # a malformed notification is dropped; it never ends the session

    def _dispatch_method(self, method, params) -> None:
        if method == "mining.notify":
            self._emit_job(parse_notify(params))
        elif method == "mining.set_difficulty":
            d = parse_difficulty(params)
            if d is not None and d > 0 and math.isfinite(d):
                self._difficulty = d
                if self.last_job is not None:
                    # Re-issue the active job with the new share target as a COPY: the original may still be
                    # queued (notify(clean=true) + set_difficulty in one read) and must keep its clean flag
                    # and target, or the engine never drops the previous prevhash's work.
                    self._emit_job(dataclasses.replace(self.last_job, clean_jobs=False))
        elif method == "mining.set_extranonce":
            r = parse_set_extranonce(params)
            if r and 0 <= r[1] <= MAX_EXTRANONCE2_SIZE:
                en1 = bytes.fromhex(r[0])
                self.extranonce1, self.extranonce2_size = en1, r[1]
        elif method == "mining.set_version_mask":
            if isinstance(params, list) and params and isinstance(params[0], str):
                self.version_mask = int(params[0], 16) & BIP320_MASK
        elif method == "client.show_message":
            n = parse_show_message(params)
            if n:
                put_drop_oldest(self.notices, n)
        elif method in ("client.reconnect", "mining.reconnect"):
            self.last_reconnect = parse_reconnect(params)
            asyncio.ensure_future(self.close())

    def _emit_job(self, job: Job) -> None:
        job.extranonce1 = self.extranonce1
        job.extranonce2_size = self.extranonce2_size
        job.version_mask = self.version_mask
        job.algorithm = self.algorithm
        diff = self._difficulty or 1.0
        from otedama_amd.models.algorithms import get as get_algo

        job.target = target_from_difficulty(diff, get_algo(self.algorithm).diff1)
        self.last_job = job
        self._job_versions.pop(job.job_id, None)
        self._job_versions[job.job_id] = job.version
        while len(self._job_versions) > 64:
            self._job_versions.pop(next(iter(self._job_versions)))
        if job.clean_jobs:
            while not self.jobs.empty():
                self.jobs.get_nowait()
        put_drop_oldest(self.jobs, job)

    async def _call(self, method: str, params: list, timeout: float = 30.0):
        if self._closed:
            raise PoolProtoError("stratumv1: session closed")
        self._next_id += 1
        mid = self._next_id
        fut = asyncio.get_running_loop().create_future()
        self._pending[mid] = fut
        body = json.dumps({"id": mid, "method": method, "params": params}).encode() + b"\n"
        try:
            async with self._write_lock:
                self.writer.write(body)
                await asyncio.wait_for(self.writer.drain(), WRITE_DEADLINE)
        except (OSError, asyncio.TimeoutError) as exc:
            self._pending.pop(mid, None)
            raise PoolProtoError(f"stratumv1: write: {exc}") from exc
        try:
            res = await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            self._pending.pop(mid, None)
            raise
        if res is None:
            raise PoolProtoError("stratumv1: session closed before response")
        return res

    async def negotiate(self) -> None:
        if self.creds.version_rolling:
            try:
                result, err = await self._call("mining.configure", [["version-rolling"], {
                    "version-rolling.mask": f"{BIP320_MASK:08x}", "version-rolling.min-bit-count": 2}], timeout=10)
                if not err and isinstance(result, dict) and result.get("version-rolling"):
                    self.version_mask = int(result.get("version-rolling.mask", "0"), 16) & BIP320_MASK
            except (PoolProtoError, asyncio.TimeoutError, ValueError):
                self.version_mask = 0  # pool does not implement BIP310
        result, err = await self._call("mining.subscribe", [USER_AGENT])
        if err:
            raise HandshakeFailed(f"stratumv1: subscribe failed: {err}")
        en1, size = parse_subscribe_result(result)
        self.extranonce1 = bytes.fromhex(en1)
        self.extranonce2_size = size
        result, err = await self._call("mining.authorize", [self.creds.user, self.creds.password or "x"])
        if err or result is not True:
            raise FatalPoolError(f"stratumv1: authorize rejected: {err or result}")
        try:
            await self._call("mining.extranonce.subscribe", [], timeout=5)
        except (PoolProtoError, asyncio.TimeoutError):
            pass  # optional (dialer.go:165-171)

    async def submit(self, sub: ShareSubmission, timeout: float = 30.0) -> ShareResult:
        worker = sub.worker or self.creds.worker or self.creds.user
        en2 = sub.extranonce2.hex() if sub.extranonce2 else "00" * self.extranonce2_size
        params = [worker, sub.job_id, en2, f"{sub.ntime & 0xFFFFFFFF:08x}", f"{sub.nonce & 0xFFFFFFFF:08x}"]
        base = self._job_versions.get(sub.job_id)
        if self.version_mask and sub.version and sub.version != base:
            # BIP310: the pool rebuilds (job_version & ~mask) | (version_bits & mask) from the version of the
            # share's OWN job (several non-clean jobs with different versions can be live at once)
            params.append(f"{sub.version & self.version_mask:08x}")
        t0 = time.perf_counter()
        result, err = await self._call("mining.submit", params, timeout=timeout)
        lat = (time.perf_counter() - t0) * 1e3
        if err:
            return ShareResult(False, _error_text(err), latency_ms=lat)
        if result is True:
            return ShareResult(True, "", self._difficulty, latency_ms=lat)
        return ShareResult(False, "rejected", latency_ms=lat)

    def suggested_difficulty(self) -> float:
        return self._difficulty

    async def _teardown(self) -> None:
        if self._closed:
            return
        self._closed = True
        for fut in self._pending.values():
            if not fut.done():
                fut.set_result(None)
        self._pending.clear()
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass

    async def close(self) -> None:
        await self._teardown()
        if self._task is not None and not self._task.done() and self._task is not asyncio.current_task():
            self._task.cancel()


def _error_text(err) -> str:
    if isinstance(err, list) and len(err) >= 2:
        return str(err[1])
    if isinstance(err, dict):
        return str(err.get("message", err))
    return str(err)


class V1Dialer(Dialer):
    def __init__(self, use_tls: bool = False, dial_fn=None):
        self.use_tls = use_tls
        self.dial_fn = dial_fn  # test seam (stratumv1/dialer.go:30)

    @property
    def protocol(self) -> ProtocolID:
        return ProtocolID.STRATUM_V1_TLS if self.use_tls else ProtocolID.STRATUM_V1

    async def dial(self, url: str, creds: Credentials, timeout: float = 10.0, algorithm: str = "sha256d") -> Session:
        rest = strip_scheme(url)
        if not rest:
            raise PoolProtoError(f"stratumv1: empty host in {url!r}")
        host, port = split_host_port(rest, 3333)
        if not host:
            raise PoolProtoError(f"stratumv1: empty host in {url!r}")
        if self.dial_fn is not None:
            reader, writer = await self.dial_fn(host, port)
        else:
            reader, writer = await tls.open_connection(host, port, self.use_tls, creds.tls_root_cas_pem or None,
                                                       timeout)
        s = V1Session(reader, writer, creds, self.protocol, algorithm)
        s.start()
        try:
            await asyncio.wait_for(s.negotiate(), timeout + 30)
        except BaseException:
            await s.close()
            raise
        return s


register(V1Dialer(False))
register(V1Dialer(True))
