"""Stratum V2 client (binary frames over TCP or TLS), standard mining channel.

Parity:
  * handshake: SetupConnection{min=max=2, endpoint=host:port, vendor/hw/fw/device}
    -> SetupConnectionSuccess | SetupConnectionError (fatal) -> OpenMiningChannel
    {ReqID 1, user, nominal hashrate} -> Success (channel id, share target) ......
    internal/engine/run.go:1173-1230
  * job / prev-hash activation state machine:
      NewMiningJob with min_ntime and a prev-hash -> active now; without min_ntime
      -> stored as a future job; SetNewPrevHash drops every job but the named one,
      activates it at max(min_ntimes), unknown job -> pause; SetTarget re-issues
      the active job ........................................ internal/engine/run.go:831-891
  * SubmitSharesStandard{channel, seq, job, nonce, ntime, version}; Success acks
    every pending seq <= last_sequence_number, Error rejects one seq;
    pending-submit map bounded at 1024 (oldest half dropped) ... run.go:892-959
  * 16 MiB frame bound before allocation (stratum/frame.go:285-293)
The reference's poolproto/stratumv2 adapter is never linked, ignores TLS and
reports every submit as accepted; this session is the one the
engine uses for stratum+v2(tls)://, with real per-share verdicts.
"""
from __future__ import annotations

import asyncio
import time
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
from otedama_amd.stratum import messages as M
from otedama_amd.stratum import tls
from otedama_amd.stratum.frame import FrameError, FrameReader
from otedama_amd.stratum.noise import NoiseError

SUBMIT_MAP_CAP = 1024
EXTENDED_MIN_EXTRANONCE = 4   # bytes of extranonce the native runtime rolls per extended channel
BIP320_MASK = 0x1FFFE000


class V2Session(Session):
    def __init__(self, reader, writer, creds: Credentials, protocol: ProtocolID, endpoint: str,
                 dialect: str = M.REFERENCE, algorithm: str = "sha256d"):
        self.reader, self.writer = reader, writer
        self.frames = FrameReader(reader)
        self.creds = creds
        self._protocol = protocol
        self.endpoint = endpoint
        self.dialect = dialect
        self.algorithm = algorithm
        self.jobs: asyncio.Queue = asyncio.Queue(maxsize=8)
        self.notices: asyncio.Queue = asyncio.Queue(maxsize=8)
        self.channel_id = 0
        self.share_target = b"\xff" * 32
        self.version_mask = 0
        self.extranonce_prefix = b""
        self.extended = False          # extended channel: jobs carry the coinbase, submits carry our extranonce
        self.extranonce_size = 0
        self._extranonce_total = 0     # prefix + miner part: fixed for the channel (spec §5.3.9)
        self._prefix_epoch = 0         # bumped by SetExtranoncePrefix; tags the job ids handed to the miner
        self._jobs: dict[int, M.NewMiningJob] = {}
        self._active: M.NewMiningJob | None = None
        self._active_ntime = 0
        self._prev_hash = bytes(32)
        self._nbits = 0
        self._have_prev = False
        self._seq = 0
        self._pending: dict[int, tuple[asyncio.Future, float]] = {}
        self._closed = False
        self._write_lock = asyncio.Lock()
        self._task: asyncio.Task | None = None
        self.last_job_received_at = 0.0
        self.dial_timing: dict[str, float] = {}
        self.log = lambda level, msg: None

    @property
    def protocol(self) -> ProtocolID:
        return self._protocol

    @property
    def closed(self) -> bool:
        return self._closed

    @property
    def remote_addr(self) -> str:
        peer = self.writer.get_extra_info("peername")
        return f"{peer[0]}:{peer[1]}" if peer else ""

    async def send(self, msg: M.Message) -> None:
        data = M.encode_message(msg, self.dialect)
        async with self._write_lock:
            self.writer.write(data)
            await asyncio.wait_for(self.writer.drain(), 10.0)  # write deadline (run.go:1251)

    async def _recv(self, timeout: float = 30.0) -> M.Message:
        f = await asyncio.wait_for(self.frames.read_frame(), timeout)
        return M.dispatch_frame(f, self.dialect)

    async def handshake(self) -> None:
        flags = M.FLAG_REQUIRES_VERSION_ROLLING if self.creds.version_rolling else 0
        host, _, port = self.endpoint.rpartition(":")
        await self.send(M.SetupConnection(
            protocol=M.MINING_PROTOCOL, min_version=2, max_version=2, flags=flags, endpoint=self.endpoint,
            vendor=self.creds.vendor, hardware_version=self.creds.hardware, firmware=self.creds.firmware,
            device_id=self.creds.device, endpoint_port=int(port) if port.isdigit() else 0))
        resp = await self._recv()
        if isinstance(resp, M.SetupConnectionError):
            raise FatalPoolError(f"pool rejected SetupConnection: {resp.error}")
        if not isinstance(resp, M.SetupConnectionSuccess):
            raise HandshakeFailed(f"expected SetupConnectionSuccess, got {type(resp).__name__}")
        if self.creds.version_rolling and resp.flags & M.FLAG_REQUIRES_VERSION_ROLLING:
            self.version_mask = BIP320_MASK
        if self.creds.extended_channel:
            await self.send(M.OpenExtendedMiningChannel(req_id=1, user=self.creds.user,
                                                        nominal_hashrate=float(self.creds.nominal_hashrate),
                                                        min_extranonce_size=EXTENDED_MIN_EXTRANONCE))
            want = M.OpenExtendedMiningChannelSuccess
        else:
            await self.send(M.OpenMiningChannel(req_id=1, user=self.creds.user,
                                                nominal_hashrate=float(self.creds.nominal_hashrate)))
            want = M.OpenMiningChannelSuccess
        resp = await self._recv()
        if isinstance(resp, M.OpenMiningChannelError):
            raise HandshakeFailed(f"pool rejected OpenMiningChannel: {resp.error}")
        if not isinstance(resp, want):
            raise HandshakeFailed(f"expected {want.__name__}, got {type(resp).__name__}")
        self.channel_id = resp.channel_id
        self.share_target = resp.target
        if self.creds.extended_channel:
            if not 0 < resp.extranonce_size <= 8:
                raise HandshakeFailed(f"extended channel: unsupported extranonce size {resp.extranonce_size}")
            self.extended = True
            self.extranonce_prefix, self.extranonce_size = resp.extranonce_prefix, resp.extranonce_size
            self._extranonce_total = len(resp.extranonce_prefix) + resp.extranonce_size
        else:
            self.extranonce_prefix = resp.extranonce

    def start(self) -> None:
        self._task = asyncio.ensure_future(self._read_loop())

    async def _read_loop(self) -> None:
        try:
            while not self._closed:
                msg = await self._recv(timeout=300.0)
                self._handle(msg)
        except (asyncio.IncompleteReadError, asyncio.TimeoutError, ConnectionError, OSError, FrameError, EOFError,
                NoiseError):
            pass  # FrameError: oversized / malformed frame or undecodable message; NoiseError: bad Noise tag
        finally:
            await self._teardown()

    # ---------------------------------------------------------- state machine
    def _job_id(self, pool_job_id: int) -> str:
        """Job id as handed to the miner: the pool's id, tagged with the extranonce-prefix epoch once the pool has
        replaced the prefix, so a share found under the old prefix is recognised at submit time."""
        return str(pool_job_id) if self._prefix_epoch == 0 else f"{pool_job_id}~{self._prefix_epoch}"

    def _start_job(self, j, ntime: int) -> None:
        self._active, self._active_ntime = j, ntime
        if isinstance(j, M.NewExtendedMiningJob):  # coinbase + merkle path: the miner builds the root per extranonce
            job = Job(job_id=self._job_id(j.job_id), version=j.version, prev_hash=self._prev_hash, merkle_root=None,
                      ntime=ntime, nbits=self._nbits, clean_jobs=True, target=self.share_target,
                      version_mask=self.version_mask if j.version_rolling_allowed else 0, channel_id=self.channel_id,
                      coinb1=j.coinbase_prefix, coinb2=j.coinbase_suffix, extranonce1=self.extranonce_prefix,
                      extranonce2_size=self.extranonce_size, merkle_branches=list(j.merkle_path),
                      algorithm=self.algorithm)
        else:
            job = Job(job_id=str(j.job_id), version=j.version, prev_hash=self._prev_hash, merkle_root=j.merkle_root,
                      ntime=ntime, nbits=self._nbits, clean_jobs=True, target=self.share_target,
                      version_mask=self.version_mask, channel_id=self.channel_id, algorithm=self.algorithm)
        put_drop_oldest(self.jobs, job)

    def _handle(self, msg: M.Message) -> None:
        if isinstance(msg, (M.NewMiningJob, M.NewExtendedMiningJob)):
            self._jobs[msg.job_id] = msg
            self.last_job_received_at = time.time()
            if msg.has_min_ntime and self._have_prev:
                self._start_job(msg, msg.min_ntime)
                self.log("info", f"engine: job {msg.job_id} version=0x{msg.version:08X} active")
            elif not msg.has_min_ntime:
                self.log("info", f"engine: job {msg.job_id} stored (future job, awaiting prev-hash)")
            else:
                self.log("info", f"engine: job {msg.job_id} held (no prev-hash yet)")
        elif isinstance(msg, M.SetNewPrevHash):
            self._prev_hash, self._nbits, self._have_prev = msg.prev_hash, msg.nbits, True
            named = self._jobs.get(msg.job_id)
            self._jobs = {}
            if named is not None:
                self._jobs[msg.job_id] = named
                ntime = max(msg.min_ntime, named.min_ntime if named.has_min_ntime else 0)
                self._start_job(named, ntime)
                self.log("info", f"engine: new prev-hash, job {msg.job_id} nBits=0x{msg.nbits:08X}")
            else:
                self._active = None
                put_drop_oldest(self.jobs, None)
                self.log("warn", f"engine: SetNewPrevHash names unknown job {msg.job_id}; pausing until next job")
        elif isinstance(msg, M.SetTarget):
            self.share_target = msg.max_target
            if self._active is not None and self._have_prev:
                self._start_job(self._active, self._active_ntime)
            self.log("info", "engine: share target updated by pool")
        elif isinstance(msg, M.SubmitSharesSuccess):
            now = time.perf_counter()
            for seq in [s for s in self._pending if s <= msg.last_sequence_number]:
                fut, sent = self._pending.pop(seq)
                if not fut.done():
                    fut.set_result(ShareResult(True, "", latency_ms=(now - sent) * 1e3))
        elif isinstance(msg, M.SubmitSharesError):
            ent = self._pending.pop(msg.sequence_number, None)
            if ent is not None and not ent[0].done():
                ent[0].set_result(ShareResult(False, msg.error, latency_ms=(time.perf_counter() - ent[1]) * 1e3))
        elif isinstance(msg, M.SetExtranoncePrefix):
            # spec §5.3.9: a new prefix for this channel's extranonce space. The channel's total extranonce length
            # is fixed, so the miner's rollable part is what the new prefix leaves. On an extended channel the active
            # job is re-issued (clean) under a new prefix epoch: the miner rebuilds every coinbase under the new
            # prefix and shares found under the old one are dropped at submit instead of being sent to be rejected.
            # A standard channel's merkle roots come from the pool and change with its next job.
            if msg.channel_id == self.channel_id:
                prefix = bytes(msg.extranonce_prefix)
                if self.extended:
                    size = self._extranonce_total - len(prefix)
                    if not 0 < size <= 8:
                        self.log("error", f"engine: SetExtranoncePrefix leaves {size} extranonce bytes "
                                          f"(prefix {len(prefix)} of {self._extranonce_total}); closing the session")
                        asyncio.ensure_future(self.close())
                        return
                    self.extranonce_size = size
                self.extranonce_prefix = prefix
                self._prefix_epoch += 1
                self.log("info", f"engine: extranonce prefix updated by pool ({len(prefix)} bytes, "
                                 f"{self.extranonce_size} rollable)")
                if self.extended and self._active is not None and self._have_prev:
                    self._start_job(self._active, self._active_ntime)
        elif isinstance(msg, M.Reconnect):
            put_drop_oldest(self.notices, f"pool requested reconnect to {msg.new_host}:{msg.new_port} (not followed)")
            asyncio.ensure_future(self.close())
        elif isinstance(msg, M.CloseChannel):
            asyncio.ensure_future(self.close())

    async def submit(self, sub: ShareSubmission, timeout: float = 30.0) -> ShareResult:
        if self._closed:
            raise PoolProtoError("stratumv2: session closed")
        jid, _, ep = str(sub.job_id).partition("~")
        try:
            job_id, epoch = int(jid), int(ep or 0)
        except ValueError:
            return ShareResult(False, f"stale-job (unknown job id {sub.job_id!r})")
        if self.extended and epoch != self._prefix_epoch:
            return ShareResult(False, "stale-prefix (found under a replaced extranonce prefix; not submitted)")
        self._seq = (self._seq + 1) & 0xFFFFFFFF
        seq = self._seq
        fut = asyncio.get_running_loop().create_future()
        self._pending[seq] = (fut, time.perf_counter())
        if len(self._pending) > SUBMIT_MAP_CAP:
            cutoff = seq - SUBMIT_MAP_CAP // 2
            for s in [s for s in self._pending if s < cutoff]:
                f, _ = self._pending.pop(s)
                if not f.done():
                    f.set_result(ShareResult(False, "unacknowledged (submit map overflow)"))
        try:
            if self.extended:
                await self.send(M.SubmitSharesExtended(self.channel_id, seq, job_id, sub.nonce, sub.ntime,
                                                       sub.version, bytes(sub.extranonce2)))
            else:
                await self.send(M.SubmitSharesStandard(self.channel_id, seq, job_id, sub.nonce, sub.ntime,
                                                       sub.version))
        except (OSError, asyncio.TimeoutError) as exc:
            self._pending.pop(seq, None)
            raise PoolProtoError(f"stratumv2: submit: {exc}") from exc
        try:
            return await asyncio.wait_for(asyncio.shield(fut), timeout)
        except asyncio.TimeoutError:
            self._pending.pop(seq, None)
            return ShareResult(False, "timeout waiting for pool verdict")

    def suggested_difficulty(self) -> float:
        from otedama_amd.models.header import difficulty_from_target

        return difficulty_from_target(self.share_target)

    async def _teardown(self) -> None:
        if self._closed:
            return
        self._closed = True
        for fut, _ in self._pending.values():
            if not fut.done():
                fut.set_exception(PoolProtoError("stratumv2: session closed before verdict"))
                fut.exception()  # mark retrieved: the submitter may already have timed out
        self._pending.clear()
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass

    async def close(self) -> None:
        await self._teardown()
        if self._task is not None and not self._task.done() and self._task is not asyncio.current_task():
            self._task.cancel()


async def noise_connect(reader, writer, creds: Credentials, timeout: float, log=None):
    """Noise NX initiator over an open (TCP or TLS) stream; returns the encrypted reader/writer pair.

    With `creds.pool_pubkey` (the pool's 32-byte x-only authority key) the responder's static key must carry a
    certificate signed by that authority and valid now (SV2 spec §4.5 SignatureNoiseMessage); anything else is a
    FatalPoolError so the engine fails over instead of mining on an unauthenticated channel. Without a pinned key
    the channel is encrypted but the pool is not authenticated, which is logged."""
    from otedama_amd.stratum import noise

    try:
        er, ew, payload, static = await noise.client_handshake(reader, writer, timeout=timeout,
                                                               suite=creds.noise_suite or noise.DEFAULT_SUITE)
    except (noise.NoiseError, asyncio.IncompleteReadError, asyncio.TimeoutError) as exc:
        writer.close()
        raise HandshakeFailed(f"noise handshake: {exc}") from exc
    if creds.pool_pubkey:
        if not noise.verify_certificate(payload, static, creds.pool_pubkey, int(time.time())):
            writer.close()
            raise FatalPoolError("noise: pool certificate does not verify against the pinned authority key")
    elif log is not None:
        log("warn", "stratumv2: Noise channel is encrypted but the pool is not authenticated (no pool_pubkey)")
    return er, ew


class V2Dialer(Dialer):
    def __init__(self, use_tls: bool = False, dialect: str = M.REFERENCE, dial_fn=None):
        self.use_tls = use_tls
        self.dialect = dialect
        self.dial_fn = dial_fn

    @property
    def protocol(self) -> ProtocolID:
        return ProtocolID.STRATUM_V2_TLS if self.use_tls else ProtocolID.STRATUM_V2

    async def dial(self, url: str, creds: Credentials, timeout: float = 10.0, algorithm: str = "sha256d",
                   log=None) -> Session:
        rest = strip_scheme(url)
        host, port = split_host_port(rest, 3336)
        timing = {"dial": time.time()}  # wall clock of each connection step (engine start-up phases)
        if self.dial_fn is not None:
            reader, writer = await self.dial_fn(host, port)
        else:
            reader, writer = await tls.open_connection(host, port, self.use_tls, creds.tls_root_cas_pem or None,
                                                       timeout)
        timing["tcp"] = time.time()
        if creds.noise or creds.pool_pubkey:
            reader, writer = await noise_connect(reader, writer, creds, timeout, log)
            timing["noise"] = time.time()
        s = V2Session(reader, writer, creds, self.protocol, f"{host}:{port}", self.dialect, algorithm)
        s.dial_timing = timing
        if log is not None:
            s.log = log
        try:
            await asyncio.wait_for(s.handshake(), timeout + 30)
            timing["channel_open"] = time.time()
        except BaseException:
            await s.close()
            raise
        s.start()
        return s


register(V2Dialer(False))
register(V2Dialer(True))

