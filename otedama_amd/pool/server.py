"""Local Stratum pool: SV2 + V1 listeners, job lifecycle, share validation,
vardiff, duplicate / stale detection, share journal, block payouts.

[NO REFERENCE CODE] — the reference v3 is a client only ("Pool operator mode"
removed, CHANGELOG.md:6623-6624). Wire formats follow the
reference encoders (stratum/messages.go, handshake.go) so
the reference client and this framework's client can both mine against it,
and — unlike the reference's test fakes (engine/integration_test.go:23-209,
run_test.go:32-166) — every share is re-hashed and validated.

Validation of a submitted share:
  1. job known and from the current block            else "stale-job"
  2. version only differs inside the negotiated BIP320 mask   "invalid-version-bits"
  3. ntime in [job ntime, now + 2h]                           "invalid-ntime"
  4. (job, extranonce, ntime, nonce, version) not seen yet    "duplicate-share"
  5. header hash (sha256d or scrypt) <= share target
     (current difficulty, or the previous one within 10 s of a retarget)
                                                              "low-difficulty-share"
  6. hash <= network target (nBits) -> block found: PPLNS payouts, new block
The reject strings land in the engine's reject taxonomy (engine/stats.go:263-277).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import json
import os
import struct
import time
from collections import OrderedDict, deque
from dataclasses import dataclass, field

from otedama_amd.metrics import Registry
from otedama_amd.models import algorithms
from otedama_amd.models.header import TargetError, hash_to_int, target_from_difficulty, target_from_nbits
from otedama_amd.pool.journal import Journal, ShareRow
from otedama_amd.pool.template import BlockTemplate, TemplateSource, merkle_root_from_branches
from otedama_amd.pool.vardiff import Vardiff, VardiffConfig, VardiffState
from otedama_amd.poolproto.stratumv1 import prevhash_to_stratum
from otedama_amd.stratum import messages as M
from otedama_amd.stratum.frame import FrameReader

BIP320_MASK = 0x1FFFE000
EN1_SIZE = 4
EN2_SIZE = 4
MAX_NTIME_FUTURE = 7200
RETARGET_GRACE = 10.0
SETTLE_BAND = 0.25  # a retarget that moves the difficulty by more than this fraction means the worker is converging
MAX_SHARES_PER_JOB = 1 << 20  # credited headers kept per live job before the job is retired


@dataclass
class PoolOptions:
    algorithm: str = "sha256d"
    listen_sv2: str = "127.0.0.1:0"
    listen_v1: str = "127.0.0.1:0"
    payout_address: str | None = None
    initial_difficulty: float = 1.0
    # Pin every connection at initial_difficulty: no vardiff retargets, no start from the channel's nominal hashrate,
    # no saved difficulty (the latency probe and benchmarks measure at a known, enforced difficulty).
    fixed_difficulty: bool = False
    target_share_seconds: float = 10.0
    retarget_seconds: float = 30.0
    min_difficulty: float = 1e-6
    nbits: int = 0x1703A30C
    n_txs: int = 7
    job_interval: float = 30.0
    block_interval: float = 600.0
    journal_path: str = ":memory:"
    payout_scheme: str = "pplns"
    coinbase_message: str = "/otedama-mi355x/"
    dialect: str = M.REFERENCE
    allow_version_rolling: bool = True
    # SV2 Noise NX (spec §4): the SV2 listener runs the responder handshake, sending a certificate for its static key
    # signed by the authority key (0 = a fresh authority per process; its x-only public key is `noise_authority_pub`).
    noise: bool = False
    noise_authority_secret: int = 0
    noise_cert_seconds: int = 365 * 86400
    noise_suite: str = ""  # "" = accept both suites (by message 1's length); "ellswift" | "legacy" = only that one


@dataclass
class PoolJob:
    job_int: int
    block: BlockTemplate
    version: int
    ntime: int
    coinb1: bytes
    coinb2: bytes
    branches: list[bytes]
    clean: bool
    created: float = field(default_factory=time.time)

    @property
    def job_id(self) -> str:
        return f"{self.job_int:x}"


@dataclass
class Verdict:
    accepted: bool
    reason: str = ""
    difficulty: float = 0.0
    hash: bytes = b""
    block: bool = False


class _Worker:
    def __init__(self, name: str, vd: VardiffState, version_mask: int):
        self.name = name
        self.vd = vd
        self.prev_difficulty = vd.difficulty
        self.retarget_at = 0.0
        self.version_mask = version_mask
        self.accepted = 0
        self.rejected = 0
        self.opened_at = time.monotonic()
        self.retargets = 0
        self.last_retarget_at = 0.0  # monotonic time of the last difficulty change (0 = never moved)
        # monotonic time of the last retarget larger than SETTLE_BAND (0 = none): after it the worker is in steady
        # state, where vardiff only follows the Poisson noise of its window (~1/sqrt(shares per window))
        self.last_big_retarget_at = 0.0

    def retargeted(self, old: float, new: float | None = None) -> None:
        """The worker's difficulty just moved away from `old`. Shares already in flight were found against some
        difficulty of the last RETARGET_GRACE seconds: the grace honours the lowest of them, not only the one
        before this retarget (vardiff ramps through several steps in its first second at a high share rate)."""
        now = time.monotonic()
        recent = now - self.retarget_at < RETARGET_GRACE
        self.prev_difficulty = min(self.prev_difficulty, old) if recent else old
        self.retarget_at = now
        self.retargets += 1
        self.last_retarget_at = now
        if new is None or old <= 0 or abs(new / old - 1.0) > SETTLE_BAND:
            self.last_big_retarget_at = now


class PoolServer:
    def __init__(self, opts: PoolOptions | None = None, registry: Registry | None = None, log=None):
        self.opts = opts or PoolOptions()
        self.algo = algorithms.get(self.opts.algorithm)
        self.log = log or (lambda level, msg: None)
        self.templates = TemplateSource(self.opts.payout_address, nbits=self.opts.nbits, n_txs=self.opts.n_txs,
                                        coinbase_message=self.opts.coinbase_message)
        self.vardiff = Vardiff(VardiffConfig(target_share_seconds=self.opts.target_share_seconds,
                                             retarget_seconds=self.opts.retarget_seconds,
                                             min_difficulty=self.opts.min_difficulty),
                               diff1_hashes=float(2 ** 256) / self.algo.diff1)
        self.journal = Journal(self.opts.journal_path)
        # share-hash workers for slow PoW (scrypt); sized to the host, never more than 8 threads
        self._hash_pool = concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1),
                                                                thread_name_prefix="otedama-pool-hash")
        # hashlib.scrypt holds the GIL; the native C++ scrypt releases it, so the workers run in parallel. The pool
        # loads the extension once at start (native SV2 frame splitting and AEAD for every connection too) rather
        # than on its first connection.
        self._slow_hash = self.algo.hash
        from otedama_amd.ops.native import load

        n = load(build_if_missing=False)
        if n is not None and self.algo.name == "scrypt":
            self._slow_hash = n.scrypt_1024_1_1
        self.block: BlockTemplate | None = None
        self.jobs: "OrderedDict[str, PoolJob]" = OrderedDict()
        self._job_counter = 0
        # Headers already credited, per live job: bounded by the 16 retained jobs x MAX_SHARES_PER_JOB and dropped
        # with the job, instead of one set that only a new block clears.
        self._seen: dict[str, set] = {}
        self._en_counter = int.from_bytes(os.urandom(2), "little") << 16
        self._v1: set[_V1Conn] = set()
        self._v2: set[_V2Conn] = set()
        self._servers: list[asyncio.base_events.Server] = []
        self._tasks: list[asyncio.Task] = []
        self.addr_sv2 = ""
        self.addr_v1 = ""
        self.blocks_found = 0
        self.noise_authority_pub = b""
        if self.opts.noise:
            from otedama_amd.stratum import noise

            auth_priv, self.noise_authority_pub = noise.keypair(self.opts.noise_authority_secret or None)
            self._noise_static, static_pub = noise.keypair()
            now = int(time.time())
            self._noise_cert = noise.certificate_payload(static_pub, auth_priv, now - 3600,
                                                         now + self.opts.noise_cert_seconds)
        self.accepted = 0
        self.rejected = 0
        self.reject_reasons: dict[str, int] = {}
        self.started_at = time.monotonic()
        self._validate_ms: deque = deque(maxlen=8192)  # submit received -> verdict, per share
        self._validate_log: deque = deque(maxlen=8192)  # (CLOCK_MONOTONIC at the verdict, ms): windowed quantiles
        # CLOCK_MONOTONIC time each new block's clean job was handed to every connection (a node's job-switch probe
        # times each rank's device from here: parallel/node_probe.py)
        self.new_block_at: deque = deque(maxlen=256)
        self._init_metrics(registry)

    # ------------------------------------------------------------ metrics
    def _init_metrics(self, reg: Registry | None) -> None:
        self.registry = reg or Registry()
        lab = {"algo": self.algo.name}
        r = self.registry
        self.m_accepted = r.new_counter("otedama_pool_shares_total", "Shares validated by the local pool.",
                                        {**lab, "status": "accepted"})
        self.m_rejected = r.new_counter("otedama_pool_shares_total", "Shares validated by the local pool.",
                                        {**lab, "status": "rejected"})
        self.m_blocks = r.new_counter("otedama_pool_blocks_found_total", "Blocks found by the local pool.", lab)
        self.m_clients = r.new_gauge("otedama_pool_connected_clients", "Connected miners.", lab)
        self.m_hashrate = r.new_gauge("otedama_pool_hashrate_hashes_per_second",
                                      "Pool hashrate estimated from accepted share work.", lab)
        self.m_work = r.new_counter("otedama_pool_accepted_work_total",
                                    "Sum of accepted share difficulties.", lab, float_value=True)
        self._work_t0 = time.monotonic()
        self._work_sum = 0.0

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self.new_block()
        if self.opts.listen_sv2:
            h, p = _split(self.opts.listen_sv2)
            srv = await asyncio.start_server(self._serve_v2, h, p)
            self._servers.append(srv)
            a = srv.sockets[0].getsockname()
            self.addr_sv2 = f"{a[0]}:{a[1]}"
        if self.opts.listen_v1:
            h, p = _split(self.opts.listen_v1)
            srv = await asyncio.start_server(self._serve_v1, h, p, limit=64 * 1024)
            self._servers.append(srv)
            a = srv.sockets[0].getsockname()
            self.addr_v1 = f"{a[0]}:{a[1]}"
        self._tasks.append(asyncio.ensure_future(self._refresh_loop()))
        if not self.opts.fixed_difficulty and self.opts.retarget_seconds > 0:
            self._tasks.append(asyncio.ensure_future(self._vardiff_loop()))
        self.log("info", f"pool[{self.algo.name}]: listening sv2={self.addr_sv2 or '-'} v1={self.addr_v1 or '-'}")
        if self.opts.noise:
            self.log("info", f"pool[{self.algo.name}]: sv2 Noise NX on; authority pubkey "
                             f"{self.noise_authority_pub.hex()}")

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        for s in self._servers:
            s.close()
        for c in list(self._v1) + list(self._v2):
            c.close()
        for s in self._servers:
            try:
                await asyncio.wait_for(s.wait_closed(), 2)
            except asyncio.TimeoutError:
                pass
        self._hash_pool.shutdown(wait=False, cancel_futures=True)
        self.journal.close()

    async def _refresh_loop(self) -> None:
        last_block = time.monotonic()
        while True:
            await asyncio.sleep(min(self.opts.job_interval, self.opts.block_interval))
            if time.monotonic() - last_block >= self.opts.block_interval:
                last_block = time.monotonic()
                self.new_block()
            else:
                self.new_job(clean=False)
            self._update_hashrate()

    async def _vardiff_loop(self) -> None:
        """Vardiff's periodic look also runs without a share: a worker whose difficulty is far too high may send
        nothing for a whole period, and must still be eased down (pool/vardiff.py's no-share rule)."""
        period = min(max(self.opts.retarget_seconds / 2.0, 0.25), 15.0)
        while True:
            await asyncio.sleep(period)
            for c in list(self._v1):
                if c.worker is not None and self._tick_worker(c.worker) is not None:
                    c._send_difficulty()
            for c in list(self._v2):
                for ch, (w, _prefix) in list(c.channels.items()):
                    new = self._tick_worker(w)
                    if new is not None:
                        c._send(M.SetTarget(ch, self.share_target(new)))

    def _tick_worker(self, w: "_Worker") -> float | None:
        old = w.vd.difficulty
        new = self.vardiff.maybe_retarget(w.vd)
        if new is not None:
            w.retargeted(old, new)
            self.journal.save_worker(w.name, new)
        return new

    def _update_hashrate(self) -> None:
        dt = time.monotonic() - self._work_t0
        if dt > 0:
            self.m_hashrate.set(self._work_sum * self.vardiff.diff1_hashes / dt)
        self._work_t0, self._work_sum = time.monotonic(), 0.0

    # ------------------------------------------------------------ jobs
    def new_block(self) -> PoolJob:
        self.block = self.templates.next_block()
        self.jobs.clear()
        self._seen.clear()
        job = self._make_job(clean=True)
        self.new_block_at.append(time.monotonic())
        self.log("info", f"pool[{self.algo.name}]: new block height={self.block.height}")
        return job

    def new_job(self, clean: bool = False) -> PoolJob:
        return self._make_job(clean)

    def _make_job(self, clean: bool) -> PoolJob:
        assert self.block is not None
        self._job_counter += 1
        coinb1, coinb2 = self.block.coinbase_parts(EN1_SIZE + EN2_SIZE)
        job = PoolJob(self._job_counter, self.block, self.block.version, max(int(time.time()), self.block.ntime),
                      coinb1, coinb2, self.block.branches(), clean)
        self.jobs[job.job_id] = job
        self._seen[job.job_id] = set()
        while len(self.jobs) > 16:
            old, _ = self.jobs.popitem(last=False)
            self._seen.pop(old, None)
        for c in list(self._v1):
            c.send_job(job)
        for c in list(self._v2):
            c.send_job(job)
        return job

    def next_extranonce(self, size: int) -> bytes:
        self._en_counter += 1
        return (self._en_counter & ((1 << (8 * size)) - 1)).to_bytes(size, "big")

    def header_for(self, job: PoolJob, extranonce: bytes, version: int, ntime: int, nonce: int) -> bytes:
        coinbase = job.coinb1 + extranonce + job.coinb2
        from otedama_amd.models.header import sha256d

        root = merkle_root_from_branches(sha256d(coinbase), job.branches)
        return (struct.pack("<I", version & 0xFFFFFFFF) + job.block.prev_hash + root
                + struct.pack("<III", ntime & 0xFFFFFFFF, job.block.nbits, nonce & 0xFFFFFFFF))

    def merkle_root_for(self, job: PoolJob, extranonce: bytes) -> bytes:
        from otedama_amd.models.header import sha256d

        return merkle_root_from_branches(sha256d(job.coinb1 + extranonce + job.coinb2), job.branches)

    # ------------------------------------------------------------ validation
    def validate(self, worker: _Worker, job_id: str, extranonce: bytes, ntime: int, nonce: int,
                 version: int) -> Verdict:
        pre = self._precheck(worker, job_id, extranonce, ntime, nonce, version)
        if isinstance(pre, Verdict):
            return pre
        job, key, hdr = pre
        return self._finish(worker, job_id, job, key, self.algo.hash(hdr))

    async def validate_async(self, worker: _Worker, job_id: str, extranonce: bytes, ntime: int, nonce: int,
                             version: int) -> Verdict:
        """validate() with the header hash off the event loop for slow algorithms (scrypt: ~ms per share,
        GIL released), so a burst of shares from many GPUs does not stall every other connection."""
        t0 = time.perf_counter()
        pre = self._precheck(worker, job_id, extranonce, ntime, nonce, version)
        if isinstance(pre, Verdict):
            v = pre
        else:
            job, key, hdr = pre
            if self.algo.name == "sha256d":
                h = self.algo.hash(hdr)  # ~1 us: cheaper inline than a thread hop
            else:
                h = await asyncio.get_running_loop().run_in_executor(self._hash_pool, self._slow_hash, hdr)
            v = self._finish(worker, job_id, job, key, h)
        ms = (time.perf_counter() - t0) * 1e3
        self._validate_ms.append(ms)
        self._validate_log.append((time.monotonic(), ms))
        return v

    def share_target(self, difficulty: float) -> bytes:
        """Share target for a difficulty, clamped to 2^256-1 (below ~diff1/2^256 the target would overflow)."""
        try:
            return target_from_difficulty(difficulty, self.algo.diff1)
        except TargetError:
            return b"\xff" * 32

    def _precheck(self, worker: _Worker, job_id: str, extranonce: bytes, ntime: int, nonce: int, version: int):
        job = self.jobs.get(job_id)
        if job is None or job.block is not self.block:
            return self._reject(worker, job_id, "stale-job")
        if (version ^ job.version) & ~worker.version_mask & 0xFFFFFFFF:
            return self._reject(worker, job_id, "invalid-version-bits")
        if ntime < job.ntime or ntime > max(time.time(), job.ntime) + MAX_NTIME_FUTURE:
            return self._reject(worker, job_id, "invalid-ntime")
        # Duplicates are keyed on the full 80-byte header, not on the job id: every job of one block shares the
        # coinbase parts and merkle branches, so one (extranonce, ntime, nonce, version) submitted under several
        # live job ids is the same work and is credited once.
        hdr = self.header_for(job, extranonce, version, ntime, nonce)
        if self._credited(hdr):
            return self._reject(worker, job_id, "duplicate-share")
        return job, hdr, hdr

    def _finish(self, worker: _Worker, job_id: str, job: PoolJob, key: tuple, h: bytes) -> Verdict:
        # re-checked after the (possibly off-loop) hash: a new block or an identical concurrent submit
        if job.block is not self.block:
            return self._reject(worker, job_id, "stale-job")
        if self._credited(key):
            return self._reject(worker, job_id, "duplicate-share")
        seen = self._seen.get(job_id)
        if seen is None or self.jobs.get(job_id) is not job:  # job retired while the share was being hashed
            return self._reject(worker, job_id, "stale-job")
        hv = hash_to_int(h)
        diff = worker.vd.difficulty
        if hv > hash_to_int(self.share_target(diff)):
            grace = time.monotonic() - worker.retarget_at < RETARGET_GRACE
            if grace and hv <= hash_to_int(self.share_target(worker.prev_difficulty)):
                diff = worker.prev_difficulty
            else:
                return self._reject(worker, job_id, "low-difficulty-share", h)
        seen.add(key)
        if len(seen) >= MAX_SHARES_PER_JOB:  # cap reached: retire the job (later shares for it are stale)
            self.jobs.pop(job_id, None)
            self._seen.pop(job_id, None)
            self.new_job()
        is_block = hv <= hash_to_int(target_from_nbits(job.block.nbits))
        worker.accepted += 1
        self.accepted += 1
        self.m_accepted.inc()
        self.m_work.add(diff)  # real difficulty, fractional below 1
        self._work_sum += diff
        self.journal.append(ShareRow(time.time(), worker.name, self.algo.name, job_id, diff, True, "", h[::-1].hex(),
                                     is_block))
        if is_block:
            self.blocks_found += 1
            self.m_blocks.inc()
            pay = self.journal.record_block(job.block.height, h[::-1].hex(), worker.name, job.block.coinbase_value,
                                            self.opts.payout_scheme)
            self.log("info", f"pool[{self.algo.name}]: BLOCK FOUND height={job.block.height} by {worker.name} "
                             f"payouts={json.dumps(pay)}")
            asyncio.get_event_loop().call_soon(self.new_block)
        return Verdict(True, "", diff, h, is_block)

    def _credited(self, hdr: bytes) -> bool:
        """Duplicates are keyed on the full header across every live job of the block (see _precheck)."""
        return any(hdr in s for s in self._seen.values())

    def _reject(self, worker: _Worker, job_id: str, reason: str, h: bytes = b"") -> Verdict:
        worker.rejected += 1
        self.rejected += 1
        self.reject_reasons[reason] = self.reject_reasons.get(reason, 0) + 1
        self.m_rejected.inc()
        self.journal.append(ShareRow(time.time(), worker.name, self.algo.name, job_id, worker.vd.difficulty, False,
                                     reason, h[::-1].hex() if h else ""))
        return Verdict(False, reason, 0.0, h)

    def new_worker(self, name: str, version_mask: int) -> _Worker:
        d = None if self.opts.fixed_difficulty else self.journal.load_worker(name)
        return _Worker(name, self.vardiff.new_state(d or self.opts.initial_difficulty), version_mask)

    def start_difficulty(self, w: _Worker, nominal_hashrate: float) -> None:
        """SV2 OpenMiningChannel / UpdateChannel: start a worker without saved state from its nominal hashrate
        (pinned pools keep initial_difficulty)."""
        if self.opts.fixed_difficulty or nominal_hashrate <= 0:
            return
        w.vd.difficulty = self.vardiff.difficulty_for_hashrate(nominal_hashrate)
        w.prev_difficulty = w.vd.difficulty

    def after_accept(self, w: _Worker, credited: float | None = None) -> float | None:
        """Vardiff's bookkeeping of an accepted share; ``credited``: the difficulty the share was accepted at (lower
        than the one in force for a grace share after a raise)."""
        if self.opts.fixed_difficulty:
            w.vd.shares += 1
            w.vd.total_shares += 1
            return None
        old = w.vd.difficulty
        weight = credited / old if credited and old > 0 else 1.0
        new = self.vardiff.on_share(w.vd, weight)
        if new is not None:
            w.retargeted(old, new)
            self.journal.save_worker(w.name, new)
        return new

    def _live_workers(self) -> list[_Worker]:
        # called from the HTTP server thread: list() snapshots each container in one C-level call under the GIL
        live = [c.worker for c in list(self._v1) if c.worker is not None]
        for c in list(self._v2):
            live += [w for w, _prefix in list(c.channels.values())]
        return live

    def workers(self, limit: int = 100) -> list[dict]:
        """Journal totals per worker, merged with the live sessions' vardiff state (GET /api/v1/workers)."""
        rows = {r["worker"]: dict(r, algorithm=self.algo.name, connected=0, difficulty=r["saved_difficulty"])
                for r in self.journal.worker_summary(limit)}
        for w in self._live_workers():
            r = rows.setdefault(w.name, {"worker": w.name, "algorithm": self.algo.name, "accepted": 0, "rejected": 0,
                                         "accepted_work": 0.0, "last_share": 0.0, "blocks": 0,
                                         "saved_difficulty": None, "connected": 0})
            r["connected"] += 1
            r["difficulty"] = w.vd.difficulty
        return sorted(rows.values(), key=lambda r: (-r["accepted_work"], r["worker"]))[:limit]

    def blocks(self, limit: int = 20) -> list[dict]:
        return [dict(b, algorithm=self.algo.name) for b in self.journal.recent_blocks(limit)]

    def validate_log(self) -> list:
        """(CLOCK_MONOTONIC, submit -> verdict ms) of the most recent validations: a caller windows them itself
        (the exit stats line of `otedama pool`; pool/pool_probe.py)."""
        return [(round(t, 6), round(ms, 4)) for t, ms in self._validate_log]

    def validation_ms(self, q: float) -> float | None:
        """Nearest-rank quantile of submit-received -> verdict (header rebuild, PoW hash, duplicate check)."""
        xs = sorted(self._validate_ms)
        return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None

    def _vardiff_view(self, w: _Worker) -> dict:
        """Vardiff's estimator for one live worker, read without touching it (this runs on the HTTP thread): the
        shares it rests on, the difficulty ratio it points to (far from 1 = a retarget is on its way), and whether
        it has settled (pool/vardiff.py: no refinement left and none pending; the pool probe opens its window on it)."""
        if self.opts.fixed_difficulty:
            return {"window_shares": w.vd.shares, "window_ratio": None, "settled": True}
        dstar, n = self.vardiff.estimate(w.vd, mutate=False)
        return {"window_shares": n, "window_ratio": dstar / w.vd.difficulty if dstar else None,
                "settled": self.vardiff.settled(w.vd, mutate=False)}

    def stats(self) -> dict:
        now = time.monotonic()
        live = self._live_workers()
        return {
            "algorithm": self.algo.name, "height": self.block.height if self.block else 0,
            "clients_v1": len(self._v1), "clients_v2": len(self._v2), "accepted": self.accepted,
            "rejected": self.rejected, "reject_reasons": dict(self.reject_reasons), "blocks_found": self.blocks_found,
            "hashrate": self.m_hashrate.value(), "sv2": self.addr_sv2, "v1": self.addr_v1,
            "uptime_s": now - self.started_at,
            "accepted_per_s": self.accepted / max(now - self.started_at, 1e-9),
            "validate_ms": {"p50": self.validation_ms(0.5), "p95": self.validation_ms(0.95),
                            "p99": self.validation_ms(0.99), "samples": len(self._validate_ms)},
            "fixed_difficulty": self.opts.fixed_difficulty,
            "new_block_at": list(self.new_block_at)[-64:],
            # per live connection: the difficulty in force, how often vardiff moved it, and when it last moved
            # (seconds after the channel opened: the time vardiff took to reach the difficulty it holds)
            "workers": [{"name": w.name, "difficulty": w.vd.difficulty, "accepted": w.accepted,
                         "rejected": w.rejected, "retargets": w.retargets, "age_s": now - w.opened_at,
                         "settled_after_s": (w.last_retarget_at - w.opened_at) if w.retargets else 0.0,
                         # steady state: seconds from the channel's open to its last retarget of more than
                         # SETTLE_BAND, and how long ago that was
                         "converged_after_s": (w.last_big_retarget_at - w.opened_at) if w.last_big_retarget_at else 0.0,
                         "steady_for_s": now - (w.last_big_retarget_at or w.opened_at),
                         **self._vardiff_view(w)}
                        for w in live],
        }

    # ------------------------------------------------------------ listeners
    async def _serve_v1(self, reader, writer) -> None:
        c = _V1Conn(self, reader, writer)
        self._v1.add(c)
        self.m_clients.set(len(self._v1) + len(self._v2))
        try:
            await c.run()
        finally:
            self._v1.discard(c)
            self.m_clients.set(len(self._v1) + len(self._v2))

    async def _serve_v2(self, reader, writer) -> None:
        if self.opts.noise:
            from otedama_amd.stratum import noise

            try:
                reader, writer = await noise.server_handshake(reader, writer, self._noise_static, self._noise_cert,
                                                              suite=self.opts.noise_suite or None)
            except (noise.NoiseError, asyncio.IncompleteReadError, asyncio.TimeoutError, ConnectionError, OSError):
                writer.close()
                self.reject_reasons["noise-handshake"] = self.reject_reasons.get("noise-handshake", 0) + 1
                return
        c = _V2Conn(self, reader, writer)
        self._v2.add(c)
        self.m_clients.set(len(self._v1) + len(self._v2))
        try:
            await c.run()
        finally:
            self._v2.discard(c)
            self.m_clients.set(len(self._v1) + len(self._v2))


def _split(addr: str) -> tuple[str, int]:
    h, _, p = addr.rpartition(":")
    return h or "0.0.0.0", int(p or 0)


class _V1Conn:
    """One Stratum V1 miner connection (JSON-RPC lines)."""

    def __init__(self, pool: PoolServer, reader, writer):
        self.pool, self.reader, self.writer = pool, reader, writer
        self.en1 = pool.next_extranonce(EN1_SIZE)
        self.subscribed = False
        self.authorized = False
        self.version_mask = 0
        self.worker: _Worker | None = None

    def close(self) -> None:
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass

    def _write(self, obj) -> None:
        try:
            self.writer.write(json.dumps(obj).encode() + b"\n")
        except Exception:  # noqa: BLE001
            pass

    def send_job(self, job: PoolJob) -> None:
        if not (self.subscribed and self.authorized):
            return
        self._write({"id": None, "method": "mining.notify", "params": [
            job.job_id, prevhash_to_stratum(job.block.prev_hash), job.coinb1.hex(), job.coinb2.hex(),
            [b.hex() for b in job.branches], f"{job.version:08x}", f"{job.block.nbits:08x}", f"{job.ntime:08x}",
            job.clean]})

    def _send_difficulty(self) -> None:
        self._write({"id": None, "method": "mining.set_difficulty", "params": [self.worker.vd.difficulty]})

    async def run(self) -> None:
        try:
            while True:
                line = await asyncio.wait_for(self.reader.readuntil(b"\n"), 600)
                try:
                    msg = json.loads(line)
                except ValueError:
                    continue
                if isinstance(msg, dict):
                    try:
                        await self._handle(msg)
                    except (ValueError, TypeError, AttributeError, KeyError, IndexError):
                        # malformed parameters (e.g. a non-string configure mask): answer, keep the connection
                        if msg.get("id") is not None:
                            self._write({"id": msg.get("id"), "result": None,
                                         "error": [20, "invalid parameters", None]})
        except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, asyncio.TimeoutError, ConnectionError,
                OSError):
            pass
        finally:
            self.close()

    async def _handle(self, msg: dict) -> None:
        mid, method, params = msg.get("id"), msg.get("method"), msg.get("params") or []
        if method == "mining.configure":
            res = {}
            exts = params[0] if params and isinstance(params[0], list) else []
            if "version-rolling" in exts and self.pool.opts.allow_version_rolling:
                req = params[1].get("version-rolling.mask", "ffffffff") if len(params) > 1 and isinstance(
                    params[1], dict) else "ffffffff"
                self.version_mask = int(req, 16) & BIP320_MASK
                res = {"version-rolling": True, "version-rolling.mask": f"{self.version_mask:08x}"}
            self._write({"id": mid, "result": res, "error": None})
        elif method == "mining.subscribe":
            self.subscribed = True
            self._write({"id": mid, "result": [[["mining.notify", self.en1.hex()]], self.en1.hex(), EN2_SIZE],
                         "error": None})
        elif method == "mining.authorize":
            user = params[0] if params and isinstance(params[0], str) else ""
            if not user:
                self._write({"id": mid, "result": False, "error": [24, "unauthorized worker", None]})
                return
            self.authorized = True
            self.worker = self.pool.new_worker(user, self.version_mask)
            self._write({"id": mid, "result": True, "error": None})
            self._send_difficulty()
            if self.pool.jobs:
                self.send_job(next(reversed(self.pool.jobs.values())))
        elif method in ("mining.extranonce.subscribe", "extranonce.subscribe"):
            self._write({"id": mid, "result": True, "error": None})
        elif method == "mining.submit":
            if not self.authorized or self.worker is None:
                self._write({"id": mid, "result": None, "error": [24, "unauthorized worker", None]})
                return
            try:
                _w, job_id, en2_hex, ntime_hex, nonce_hex = params[:5]
                en2 = bytes.fromhex(en2_hex)
                ntime, nonce = int(ntime_hex, 16), int(nonce_hex, 16)
                job = self.pool.jobs.get(str(job_id))
                base_version = job.version if job else 0
                # BIP310: version = (job_version & ~mask) | (version_bits & mask); bits outside
                # the mask make the version differ from the job outside the mask -> rejected.
                vbits = int(params[5], 16) if len(params) > 5 and params[5] else None
                if vbits is None:
                    version = base_version
                elif vbits & ~self.version_mask & 0xFFFFFFFF:
                    version = base_version ^ (vbits & ~self.version_mask)
                else:
                    version = (base_version & ~self.version_mask) | vbits
                if len(en2) != EN2_SIZE:
                    raise ValueError("bad extranonce2 size")
            except (ValueError, TypeError, IndexError):
                self._write({"id": mid, "result": None, "error": [20, "invalid submit parameters", None]})
                return
            v = await self.pool.validate_async(self.worker, str(job_id), self.en1 + en2, ntime, nonce, version)
            if v.accepted:
                self._write({"id": mid, "result": True, "error": None})
                if self.pool.after_accept(self.worker, v.difficulty) is not None:
                    self._send_difficulty()
            else:
                code = {"stale-job": 21, "duplicate-share": 22, "low-difficulty-share": 23}.get(v.reason, 20)
                self._write({"id": mid, "result": None, "error": [code, v.reason, None]})
        elif mid is not None:
            self._write({"id": mid, "result": None, "error": [20, f"unknown method {method}", None]})


class _V2Conn:
    """One Stratum V2 miner connection: standard channels (header-only jobs, merkle root per channel) and
    extended channels (coinbase prefix/suffix + merkle path; the miner rolls EN2_SIZE extranonce bytes after the
    pool's EN1_SIZE prefix and submits them in SubmitSharesExtended)."""

    def __init__(self, pool: PoolServer, reader, writer):
        self.pool, self.reader, self.writer = pool, reader, writer
        self.frames = FrameReader(reader)
        self.dialect = pool.opts.dialect
        self.version_rolling = False
        self.channels: dict[int, tuple[_Worker, bytes]] = {}  # channel id -> (worker, extranonce prefix)
        self.extended: set[int] = set()
        self._next_channel = 1
        self.setup = False

    def close(self) -> None:
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass

    def _send(self, msg: M.Message) -> None:
        try:
            self.writer.write(M.encode_message(msg, self.dialect))
        except Exception:  # noqa: BLE001
            pass

    def _job_msgs(self, ch: int, job: PoolJob, prefix: bytes, future: bool) -> list[M.Message]:
        if ch in self.extended:
            j = M.NewExtendedMiningJob(ch, job.job_int, has_min_ntime=not future, min_ntime=0 if future else job.ntime,
                                       version=job.version, version_rolling_allowed=self.version_rolling,
                                       merkle_path=list(job.branches), coinbase_prefix=job.coinb1,
                                       coinbase_suffix=job.coinb2)
        else:
            root = self.pool.merkle_root_for(job, prefix)
            j = M.NewMiningJob(ch, job.job_int, has_min_ntime=not future, min_ntime=0 if future else job.ntime,
                               version=job.version, merkle_root=root)
        if future:
            return [j, M.SetNewPrevHash(ch, job.job_int, job.block.prev_hash, job.ntime, job.block.nbits)]
        return [j]

    def send_job(self, job: PoolJob) -> None:
        for ch, (_w, prefix) in self.channels.items():
            for m in self._job_msgs(ch, job, prefix, future=job.clean):
                self._send(m)

    async def run(self) -> None:
        try:
            while True:
                f = await asyncio.wait_for(self.frames.read_frame(), 600)
                msg = M.dispatch_frame(f, self.dialect)
                await self._handle(msg)
                await self.writer.drain()
        except (asyncio.IncompleteReadError, asyncio.TimeoutError, ConnectionError, OSError, M.MessageError,
                EOFError):
            pass
        finally:
            self.close()

    async def _handle(self, msg: M.Message) -> None:
        if isinstance(msg, M.SetupConnection):
            try:
                M.validate_setup_connection(msg)
                if not msg.min_version <= 2 <= msg.max_version:
                    raise M.MessageError("unsupported-protocol-version")
            except M.MessageError as exc:
                self._send(M.SetupConnectionError(0, str(exc)[:255]))
                return
            self.setup = True
            self.version_rolling = bool(msg.flags & M.FLAG_REQUIRES_VERSION_ROLLING) and \
                self.pool.opts.allow_version_rolling
            self._send(M.SetupConnectionSuccess(2, M.FLAG_REQUIRES_VERSION_ROLLING if self.version_rolling else 0))
        elif isinstance(msg, (M.OpenMiningChannel, M.OpenExtendedMiningChannel)):
            extended = isinstance(msg, M.OpenExtendedMiningChannel)
            if not self.setup or not msg.user:
                self._send(M.OpenMiningChannelError(msg.req_id, "unknown-user" if self.setup else "setup-required"))
                return
            if extended and msg.min_extranonce_size > EN2_SIZE:
                self._send(M.OpenMiningChannelError(msg.req_id, "min-extranonce-size-too-large"))
                return
            ch = self._next_channel
            self._next_channel += 1
            prefix = self.pool.next_extranonce(EN1_SIZE if extended else EN1_SIZE + EN2_SIZE)
            w = self.pool.new_worker(msg.user, BIP320_MASK if self.version_rolling else 0)
            if self.pool.opts.fixed_difficulty or self.pool.journal.load_worker(msg.user) is None:
                self.pool.start_difficulty(w, msg.nominal_hashrate)
            self.channels[ch] = (w, prefix)
            target = self.pool.share_target(w.vd.difficulty)
            if extended:
                self.extended.add(ch)
                self._send(M.OpenExtendedMiningChannelSuccess(msg.req_id, ch, target, EN2_SIZE, prefix))
            else:
                self._send(M.OpenMiningChannelSuccess(msg.req_id, ch, target, prefix, extranonce2_size=0))
            if self.pool.jobs:
                for m in self._job_msgs(ch, next(reversed(self.pool.jobs.values())), prefix, future=True):
                    self._send(m)
        elif isinstance(msg, (M.SubmitSharesStandard, M.SubmitSharesExtended)):
            ent = self.channels.get(msg.channel_id)
            extended = isinstance(msg, M.SubmitSharesExtended)
            if ent is None or extended != (msg.channel_id in self.extended):
                self._send(M.SubmitSharesError(msg.channel_id, msg.sequence_number, "invalid-channel-id"))
                return
            w, prefix = ent
            if extended:
                if len(msg.extranonce) != EN2_SIZE:
                    self._send(M.SubmitSharesError(msg.channel_id, msg.sequence_number, "invalid-extranonce-size"))
                    return
                prefix = prefix + msg.extranonce
            v = await self.pool.validate_async(w, f"{msg.job_id:x}", prefix, msg.ntime, msg.nonce, msg.nversion)
            if v.accepted:
                self._send(M.SubmitSharesSuccess(msg.channel_id, msg.sequence_number, 1, max(int(v.difficulty), 1)))
                new = self.pool.after_accept(w, v.difficulty)
                if new is not None:
                    self._send(M.SetTarget(msg.channel_id, self.pool.share_target(new)))
            else:
                self._send(M.SubmitSharesError(msg.channel_id, msg.sequence_number, v.reason))
        elif isinstance(msg, M.UpdateChannel):
            ent = self.channels.get(msg.channel_id)
            if ent is not None and msg.nominal_hashrate > 0 and not self.pool.opts.fixed_difficulty:
                w = ent[0]
                old = w.vd.difficulty
                w.vd.difficulty = self.pool.vardiff.difficulty_for_hashrate(msg.nominal_hashrate)
                w.retargeted(old, w.vd.difficulty)
                self._send(M.SetTarget(msg.channel_id, self.pool.share_target(w.vd.difficulty)))
        elif isinstance(msg, M.CloseChannel):
            self.channels.pop(msg.channel_id, None)
            self.extended.discard(msg.channel_id)
