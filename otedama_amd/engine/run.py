"""Top-level orchestrator: devices -> miners -> pool session -> shares -> metrics.

Parity: internal/engine/run.go + setup.go + arbitrate.go + fanin.go
  * Options (config, clock, output, logger func(level,msg), no_tui, stats
    interval, max reconnect attempts, wallet passphrases, metrics, on_ready) run.go:71-108
  * curtail_decision (never on stale/fallback price) ............... run.go:123-135
  * Run phases: metrics + uptime ticker, wallet, device detection,
    miner start, rates (fallback 95000, 5 min), curtail loop (30 s),
    providers, arbitration loop, TUI, reconnect loop ................ run.go:140-339
  * reconnect loop: pool failover immediately, payout-address
    failover only if the address never connected, backoff 1 s x2 ->
    64 s, fatal errors stop, MaxReconnectAttempts ................... run.go:343-521
  * session loop (stats tick: windowed hashrate, drops, stall
    detection, sats, productive seconds, power/J-per-TH, acceptance
    warning >= 20 judged & < 97%, latency p50/95/99) ................. run.go:610-961
  * arbitration glue (quotes -> streams, 3 min staleness prune,
    Decide every 30 s, pause devices moved to AI / idle) ............. arbitrate.go:62-299
  * pool_urls / payout_addresses / session_user / mask_addr .......... setup.go:213-270

Differences: one pool-agnostic session loop drives both
Stratum V1 and V2 (both through otedama_amd.poolproto, with real verdicts);
stream yields use NET sats/s (the reference uses gross, arbitrate.go:187-195);
the simulated AI provider is opt-in because on MI355X it would idle real GPU
mining for a simulated quote; GPU faults drop the device's stripe and
rebalance the rest.
"""
from __future__ import annotations

import asyncio
import collections
import json
import os
import sys
import time
from dataclasses import dataclass
from typing import Callable, TextIO

from otedama_amd import arbitration as arb
from otedama_amd import hal
from otedama_amd.config import DEFAULT_POOL_URL, Config
from otedama_amd.engine.metrics import EngineMetrics
from otedama_amd.engine.miners import MinerSet
from otedama_amd.engine.stats import (
    HashrateMonitor,
    HashrateWindow,
    LatencyTracker,
    SatsAccountant,
    UptimeAccountant,
    effective_yield,
    hashrate_string,
    publish_btc_rate,
    publish_difficulty,
    reject_class,
)
from otedama_amd.metrics import Registry, runtime_collector
from otedama_amd.models.algorithms import get as get_algorithm
from otedama_amd.poolproto import Credentials, FatalPoolError, Job, ShareSubmission
from otedama_amd.poolproto.base import extranonce2_bytes, from_url, lookup
from otedama_amd.provider import AkashProvider, MiningProvider
from otedama_amd.utils.bounded import BoundedSet
from otedama_amd.utils.clock import SYSTEM, Clock
from otedama_amd.utils.trace import mark as trace_mark

RECONNECT_BACKOFF_INITIAL = 1.0
RECONNECT_BACKOFF_MAX = 64.0
STREAM_STALE_TIMEOUT = 180.0
DEFAULT_HYSTERESIS = 0.05
SHARE_POLL_INTERVAL = 0.005  # share-queue poll for miner sets without wake-up fds (test fakes)
SHARE_WAKE_FALLBACK = 0.25   # with eventfds: safety re-poll interval (a missed wake-up costs at most this)
SUBMIT_KEYS_CAP = 1024  # unacked-submit map bound (internal/engine/run.go:726)
TARGET_GRACE = 10.0     # the local pool's window (pool/server.py RETARGET_GRACE): the most a pools[].target_grace may
                        # usefully be; the engine applies the grace of the pool it is connected to (default 0 = off)


@dataclass
class Options:
    config: Config
    clock: Clock = SYSTEM
    output: TextIO | None = None
    logger: Callable[[str, str], None] | None = None
    no_tui: bool = True
    stats_interval: float = 10.0
    max_reconnect_attempts: int = 0
    wallet_passphrase: str = ""
    wallet_mnemonic_passphrase: str = ""
    metrics: Registry | None = None
    on_ready: Callable[[bool], None] | None = None
    devices: list | None = None              # test seam: skip HAL detection
    rate_fetcher: object | None = None       # test seam
    enable_ai_provider: bool = False
    arbitration_interval: float = 30.0
    curtail_interval: float = 30.0
    rates_interval: float = 300.0
    fetch_rates: bool = True
    dashboard: object | None = None
    node_comm: object | None = None          # parallel.comm.NodeComm when launched under torchrun


def curtail_decision(curr: bool, rate: float, fresh: bool, threshold: float) -> tuple[bool, bool]:
    if threshold <= 0 or not fresh or rate <= 0:
        return curr, False
    if rate < threshold and not curr:
        return True, True
    if rate >= threshold and curr:
        return False, True
    return curr, False


def pool_urls(cfg: Config) -> list[str]:
    return [p.url for p in cfg.pools] if cfg.pools else [DEFAULT_POOL_URL]


def payout_addresses(cfg: Config) -> list[str]:
    seen, out = set(), []
    for a in [cfg.bitcoin_address, *cfg.bitcoin_addresses]:
        if a and a not in seen:
            seen.add(a)
            out.append(a)
    return out


def session_user(pool_user: str, addr: str, worker: str) -> str:
    if pool_user:
        return pool_user
    return f"{addr}.{worker}" if worker else addr


def mask_addr(a: str) -> str:
    return a if len(a) <= 12 else a[:6] + "…" + a[-4:]



# Start-up marks taken before the engine exists (otedama run in node mode: torch import, the process group's
# rendezvous); the engine starts its own marks from these (startup phases in /debug/stats and the node report).
EARLY_MARKS: dict[str, float] = {}


def mark_early(name: str) -> None:
    EARLY_MARKS.setdefault(name, time.time())


def _process_start_wall() -> float:
    """Wall-clock time this process started, to ~10 ms: its start in clock ticks after boot (/proc/self/stat
    field 22) against the uptime now (/proc/uptime); 0.0 where /proc is unavailable."""
    try:
        with open("/proc/self/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        with open("/proc/uptime") as f:
            uptime = float(f.read().split()[0])
        started = int(fields[19]) / os.sysconf("SC_CLK_TCK")
        return time.time() - (uptime - started)
    except (OSError, ValueError, IndexError):
        return 0.0

class Engine:
    def __init__(self, opts: Options):
        self.opts = opts
        self.cfg = opts.config
        self.log = opts.logger or (lambda level, msg: None)
        self.registry = opts.metrics or Registry()
        self.m = EngineMetrics(self.registry)
        self.registry.register_collector(runtime_collector())
        self.algorithm = get_algorithm(self.cfg.mining.algorithm)
        self.start_time = opts.clock.now()
        self._marks: dict[str, float] = dict(EARLY_MARKS)
        self.devices: list = []
        self.miners: MinerSet | None = None
        self.curtailed = False
        self.latency = LatencyTracker(256)           # submit -> accept (reference semantics)
        self.pipeline_latency = LatencyTracker(4096)  # host-verified hit -> accept
        self.device_latency = LatencyTracker(4096)    # the kernel's hit (device clock) -> accept
        # the same, split by where the share was found: this process's devices, or another rank of the node (its
        # share crossed the R2 gather; parallel/node.py)
        self.device_latency_by_origin = {"local": LatencyTracker(4096), "remote": LatencyTracker(4096)}
        # accepted shares: (monotonic, device hit -> accept ms | None, origin, device, host verify -> accept ms | None)
        # (time, hit -> accept ms, origin, device, host-verify -> accept ms) per accepted share, for the node report
        # (OTEDAMA_NODE_REPORT) only: a production engine keeps no per-share history (it was ~200 B per share, 3 MB
        # of RSS growth over a 6500-share soak, profiles/r5/k_node_soak)
        self.accept_log: collections.deque = collections.deque(
            maxlen=16384 if os.environ.get("OTEDAMA_NODE_REPORT") else 0)
        self.hash_window = HashrateWindow()
        self.current_hashrate = 0.0
        self.device_hashrates: dict[str, float] = {}
        self.pool_url = ""
        self.connected = False
        self.stalled = False
        self.est_sats = 0.0
        self.wallet_fingerprint = ""
        self.activity: dict[str, float] = {}
        self._active_job: Job | None = None
        self._valid_jobs: set[str] = set()
        self._job_targets: dict[str, int | None] = {}  # job id -> its current share target (int, LE)
        # job id -> (the easier target in force before the last raise, monotonic time of the raise): a share found
        # against it and still queued is submitted within TARGET_GRACE (pools credit such in-flight shares)
        self._prev_targets: dict[str, tuple[int, float]] = {}
        self._target_grace = 0.0  # the connected pool's pools[].target_grace
        self._submitted = BoundedSet(SUBMIT_KEYS_CAP)  # run.go:720-726: cap 1024, oldest half dropped
        self._session = None
        self._providers: list = []
        self._rate_fetcher = opts.rate_fetcher
        self._tasks: list[asyncio.Task] = []
        self._submit_tasks: set[asyncio.Task] = set()
        self._hashmon = HashrateMonitor(0, 3, self.log)
        self._uptime = UptimeAccountant()
        self._sats = SatsAccountant()
        self._last_dropped = 0
        self._busy_prev: dict[str, tuple[float, float, int]] = {}  # device -> (busy_seconds, at, launches)
        self._lost_prev: dict[tuple[str, str], int] = {}  # (device, cause) -> candidates lost so far
        self.dashboard = opts.dashboard

    # ---------------------------------------------------------------- API
    def stats(self) -> dict:
        return {
            "hashrate": self.current_hashrate, "hashrate_str": hashrate_string(self.current_hashrate),
            "devices": {k: v for k, v in self.device_hashrates.items()},
            "shares_found": self.m.shares_found.value(), "shares_submitted": self.m.shares_submitted.value(),
            "accepted": self.m.shares_accepted.value(), "rejected": self.m.shares_rejected.value(),
            "latency_p50_ms": self.latency.quantile(0.5), "latency_p95_ms": self.latency.quantile(0.95),
            "pool": self.pool_url, "connected": self.connected, "curtailed": self.curtailed,
            "stalled": self.stalled, "uptime": self.opts.clock.now() - self.start_time,
            "algorithm": self.algorithm.name, "wallet": self.wallet_fingerprint,
            "est_sats": self.est_sats, "activity": dict(self.activity),
        }

    def debug_stats(self) -> dict:
        """GET /debug/stats: raw native counters and the scheduler state behind them,
        for diagnosing a device or node without attaching a profiler."""
        import resource
        import threading as _th

        ms = self.miners
        devs = {}
        if ms is not None:
            raw = ms.device_stats()
            stalled = set(ms.stalled())
            for m in ms.miners:
                st = dict(raw.get(m.id, {}))
                up = max(self.opts.clock.now() - self.start_time, 1e-9)
                st.update({"stripe_start": m.stripe_index, "stripe_stride": m.stripe_stride, "paused": m.paused,
                           "retired": m.retired, "stalled": m.id in stalled, "hashrate": m.hashrate,
                           "idle_samples": m.idle_samples, "busy_ratio": st.get("busy_seconds", 0.0) / up})
                devs[m.id] = st
            for rid in getattr(ms, "remote_ids", []):
                devs[rid] = dict(raw.get(rid, {}), hashrate=ms.hashrate_of(rid), stalled=rid in stalled)
        link = getattr(ms, "link", None)
        return {
            "epoch": ms.epoch if ms is not None else 0,
            "devices": devs,
            "node": None if link is None else {
                "rank": link.rank, "world": link.world, "tick_s": link.tick, "counter_rows": link.rows,
                "generation": link.comm.info.generation, "members": list(link.comm.info.members),
                "lost_ranks": list(getattr(ms, "lost_ranks", [])), "device_collectives": link.comm.collectives,
                "ops": link.ops_run, "reforms": link.reforms,
                "op_p50_s": link.tick_quantile(0.5), "op_p99_s": link.tick_quantile(0.99),
                "error": str(link.error) if link.error else None},
            "submit_tasks_inflight": len(self._submit_tasks),
            "startup": self._startup(),
            "latency_ms": {"p50": self.latency.quantile(0.5), "p95": self.latency.quantile(0.95),
                           "p99": self.latency.quantile(0.99)},
            "hit_to_accept_ms": {"p50": self.device_latency.quantile(0.5), "p95": self.device_latency.quantile(0.95),
                                 "p99": self.device_latency.quantile(0.99)},
            "process": {"threads": _th.active_count(),
                        "max_rss_mib": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0},
        }

    def _startup(self) -> dict:
        """Process start -> first completed GPU batch, per device (device processes report their first hash), and
        this process's resident set (BENCHMARKS.md:105-129 reports <1 s to hashing and 25 MB)."""
        out = {}
        t0 = _process_start_wall()
        try:
            import psutil

            p = psutil.Process()
            t0 = t0 or p.create_time()  # psutil's is only as precise as the boot time (whole seconds)
            out["rss_mib"] = p.memory_info().rss / 2**20
            kids = p.children(recursive=True)
            out["children_rss_mib"] = sum(k.memory_info().rss for k in kids) / 2**20
        except Exception:  # noqa: BLE001 - psutil missing or a child gone
            pass
        ms = self.miners
        firsts, phases, native = {}, {}, {}
        for m in getattr(ms, "miners", []) or []:
            wall = float(getattr(m.native, "first_hash_wall", 0.0) or 0.0)
            if wall and t0:
                firsts[m.id] = wall - t0
                ct = getattr(m.native, "child_timing", {}) or {}
                phases[m.id] = {k: (v - t0) if v else None for k, v in ct.items()}
            try:
                nat = m.native.stats().get("native_startup_ms") or m.native.stats().get("startup_ms")
            except Exception:  # noqa: BLE001 - a miner without stats
                nat = None
            if nat:
                native[m.id] = dict(nat)
        out["first_hash_after_start_s"] = firsts
        # seconds after engine start: child main, native loaded, miner started, first job in, first batch running
        out["device_process_phases_s"] = phases
        out["native_phases_ms"] = native  # inside the device thread: hip_set_device, buffers, clock_calibration, ...
        # this process: run() entered, devices named, miners (device processes) started, pool dial / connected,
        # first job handed to the devices; seconds after process start
        out["engine_phases_s"] = {k: (v - t0) for k, v in self._marks.items()} if t0 else {}
        return out

    def enforced_share_difficulty(self) -> float | None:
        """Difficulty of the share target in force for the active job (the pool's SetTarget /
        OpenMiningChannelSuccess / set_difficulty), as diff1 / target; None without a job."""
        job = self._active_job
        tgt = self._job_targets.get(job.job_id) if job is not None else None
        return self.algorithm.diff1 / tgt if tgt else None

    def device_list(self) -> list[dict]:
        return [{"id": d.identity().id, "family": d.identity().family.value, "vendor": d.identity().vendor,
                 "model": d.identity().model, "capabilities": d.capabilities().__dict__} for d in self.devices]

    # ---------------------------------------------------------------- run
    def _mark(self, name: str) -> None:
        """Wall time of the first occurrence of a start-up event (engine_phases_s in /debug/stats)."""
        self._marks.setdefault(name, time.time())

    async def run(self) -> None:
        cfg = self.cfg
        self._mark("run")
        self.m.uptime.set(0)
        self.m.start_time.set(self.start_time)
        if cfg.power_watts > 0 and cfg.electricity_price_per_kwh > 0:
            self.m.power_cost_usd_per_hour.set(cfg.power_watts / 1000 * cfg.electricity_price_per_kwh)
        self._tasks.append(asyncio.ensure_future(self._uptime_loop()))
        try:
            self.wallet_fingerprint = self._setup_wallet()
            self.devices = self.opts.devices if self.opts.devices is not None else await asyncio.to_thread(
                self._detect_devices)
            self.log("info", f"engine: detected {len(self.devices)} device(s)")
            self._mark("devices_detected")
            for d in self.devices:
                self.log("info", f"engine: device {d.identity()} caps={d.capabilities()}")
            node = self.opts.node_comm
            world = max(node.info.world_size, 1) if node is not None else 1
            # one process per GPU; a node rank runs its GPU's miner in a device process too, so a kernel fault never
            # takes the pool session or the RCCL communicator with it
            gpus = any(d.identity().family == hal.Family.GPU for d in self.devices)
            isolation = "process" if (cfg.mining.isolation == "process" and (gpus or node is not None)) else "thread"
            self.miners = MinerSet(self.devices, self.algorithm.name, cfg.mining.batch_nonces, cfg.mining.cpu_threads,
                                   rank=0, world_size=world, log=self.log, sha_variants=cfg.mining.sha_variants,
                                   isolation=isolation)
            if node is not None and node.info.capacity > 1:
                from otedama_amd.parallel.node import NodeMinerSet

                self.miners = NodeMinerSet(self.miners, node, log=self.log)
                self.log("info", f"engine: node mode, {world} ranks over {node.info.backend}")
            if len(self.miners) == 0:
                raise RuntimeError(f"engine: no device can mine {self.algorithm.name}")
            self.miners.start()
            self._mark("miners_started")
            if self._rate_fetcher is None:
                from otedama_amd.rates import Fetcher

                self._rate_fetcher = Fetcher(95_000.0, log=lambda msg: self.log("warn", msg))
                if self.opts.fetch_rates:
                    self._rate_fetcher.start_background(self.opts.rates_interval)
            self._tasks.append(asyncio.ensure_future(self._curtail_loop()))
            self._start_providers()
            self._tasks.append(asyncio.ensure_future(self._arbitration_loop()))
            if self.dashboard is not None:
                self.dashboard.start()
            report = os.environ.get("OTEDAMA_NODE_REPORT", "")
            if report:
                self._tasks.append(asyncio.ensure_future(self._report_loop(report)))
            await self._reconnect_loop()
        finally:
            for t in self._tasks:
                t.cancel()
            for p in self._providers:
                await p.stop()
            if self.miners is not None:
                self.miners.stop()
            if self.dashboard is not None:
                self.dashboard.stop()
            if self._rate_fetcher is not None and hasattr(self._rate_fetcher, "stop"):
                self._rate_fetcher.stop()
            if self.opts.on_ready:
                self.opts.on_ready(False)

    # ---------------------------------------------------------------- node report
    def timeline_counters(self) -> dict[str, list]:
        """Per device (local) and per rank (remote): [cumulative hashes, device-timeline time they had completed]
        — one consistent pair each, so a rate over two samples is exact (bench.py's node section)."""
        out: dict[str, list] = {}
        ms = self.miners
        if ms is None:
            return out
        for dev, st in ms.device_stats().items():
            out[dev] = [int(st.get("hashes", 0)), float(st.get("hashes_done_at_s", 0.0) or 0.0)]
        for r, (h, done) in dict(getattr(ms, "_hb_pairs", {})).items():  # remote ranks: their heartbeat's pair
            out[f"rank{r}"] = [int(h), float(done)]
        return out

    def node_report(self) -> dict:
        """Snapshot of the node as rank 0 sees it (OTEDAMA_NODE_REPORT): counters, device-timeline pairs, share
        verdicts, hit -> accept latency by origin and the collective accounting."""
        ms = self.miners
        link = getattr(ms, "link", None)
        info = link.comm.info if link is not None else None

        def q(t: LatencyTracker) -> dict:
            return {"p50": t.quantile(0.5), "p95": t.quantile(0.95), "p99": t.quantile(0.99), "samples": t.count()}

        rep = {
            "mono": time.monotonic(), "wall": time.time(), "pid": os.getpid(),
            "connected": self.connected, "algorithm": self.algorithm.name,
            "hashrate": self.current_hashrate, "counters": self.timeline_counters(),
            "shares_found": self.m.shares_found.value(), "submitted": self.m.shares_submitted.value(),
            "accepted": self.m.shares_accepted.value(), "rejected": self.m.shares_rejected.value(),
            "stale_skipped": self.m.stale_skipped.value(), "below_target_skipped": self.m.below_target_skipped.value(),
            "hit_to_accept_ms": {k: q(t) for k, t in self.device_latency_by_origin.items()},
            "submit_to_accept_ms": q(self.latency),
            "share_difficulty": self.enforced_share_difficulty(),
            "world": info.world_size if info is not None else 1,
            "members": list(info.members) if info is not None else [0],
            "backend": info.backend if info is not None else "none",
            "generation": info.generation if info is not None else 0,
        }
        if link is not None:
            hbs = {}
            try:
                hbs = ms.heartbeats_snapshot()
            except Exception:  # noqa: BLE001 - store gone: shutting down
                pass
            rep.update({
                "leader_collectives": link.comm.collectives,
                "follower_collectives": {f"rank{r}": int(hb.get("coll", 0)) for r, hb in hbs.items()},
                "follower_pending": {f"rank{r}": int(hb.get("pending", 0)) for r, hb in hbs.items()},
                "ops": link.ops_run, "reforms": link.reforms, "lost_ranks": list(ms.lost_ranks),
                "leader_incarnation": ms.incarnation, "remote_stale": ms.remote_stale,
                "share_previews": ms.share_previews, "share_gathered_first": ms.share_gathered_first,
                "previews_refused": getattr(ms, "previews_refused", 0),
                "op_p50_ms": link.tick_quantile(0.5) * 1e3, "op_p99_ms": link.tick_quantile(0.99) * 1e3,
                "job_set_at": list(ms.job_set_at), "job_bcast_at": list(ms.job_bcast_at)})
        # (epoch, CLOCK_MONOTONIC) of each new work's first batch running: rank 0's devices and every follower's
        # heartbeat (the node job-switch probe, parallel/node_probe.py)
        # start-up of this rank, seconds after its process started: torch imported, process group formed, engine
        # phases (devices, miners, pool connect, first job), and the device process's first batch
        t0 = getattr(self, "_t0_wall", None)
        if t0 is None:
            t0 = self._t0_wall = _process_start_wall()
        if t0:
            ph = {k: round(v - t0, 3) for k, v in self._marks.items()}
            for m in getattr(getattr(ms, "local", ms), "miners", []) or []:
                wall = float(getattr(m.native, "first_hash_wall", 0.0) or 0.0)
                if wall:
                    ph.setdefault("first_batch_running", round(wall - t0, 3))
            rep["startup_phases_s"] = ph
            rep["process_start_wall"] = t0
        local = getattr(ms, "local", ms)
        ws = {"rank0": sorted(tuple(x) for st in (local.device_stats().values() if local is not None else [])
                              for x in (st.get("work_started") or []))[-32:]}
        if link is not None:
            for r, hb in hbs.items():
                ws[f"rank{r}"] = [tuple(x) for x in hb.get("ws", [])]
            rep["job_applied"] = {f"rank{r}": [tuple(x) for x in hb.get("ja", [])] for r, hb in hbs.items()}
        rep["work_started"] = ws
        return rep

    def node_status(self) -> dict:
        """GET /api/v1/node: the multi-GPU node as its leader sees it (membership, generation, data plane, each rank's
        rate and heartbeat, share delivery). A standalone engine reports a one-rank node."""
        ms = self.miners
        link = getattr(ms, "link", None)
        if link is None:
            return {"world": 1, "members": [0], "backend": "none", "generation": 0, "ranks": {}}
        info = link.comm.info
        try:
            hbs = ms.heartbeats_snapshot()
        except Exception:  # noqa: BLE001 - store gone: shutting down
            hbs = {}
        now = time.time()
        ranks = {"rank0": {"hashrate": sum(self.device_hashrates.get(d.id, 0.0) for d in ms.local.miners),
                           "leader": True}}
        for r, hb in hbs.items():
            ranks[f"rank{r}"] = {"hashrate": self.device_hashrates.get(f"rank{r}", 0.0),
                                 "heartbeat_age_s": round(now - float(hb.get("t", 0.0) or 0.0), 3),
                                 "generation": hb.get("gen"), "pending_shares": int(hb.get("pending", 0)),
                                 "collectives": int(hb.get("coll", 0)), "pid": hb.get("pid"),
                                 "member": r in info.members}
        return {"world": info.world_size, "capacity": ms.capacity, "members": list(info.members),
                "backend": info.backend, "generation": info.generation, "leader_incarnation": ms.incarnation,
                "lost_ranks": list(ms.lost_ranks), "reforms": link.reforms, "ops": link.ops_run,
                "leader_collectives": link.comm.collectives,
                "op_p50_ms": link.tick_quantile(0.5) * 1e3, "op_p99_ms": link.tick_quantile(0.99) * 1e3,
                "share_previews": ms.share_previews, "share_gathered_first": ms.share_gathered_first,
                "remote_stale": ms.remote_stale, "ranks": ranks}

    async def _report_loop(self, path: str, period: float = 0.5) -> None:
        """Write node_report() to ``path`` every ``period`` s (atomic rename), with the accepted shares'
        (monotonic, hit -> accept ms, origin) and a bounded series of counter samples."""
        samples: collections.deque = collections.deque(maxlen=2400)
        while True:
            await asyncio.sleep(period)
            try:
                rep = self.node_report()
                samples.append([rep["mono"], rep["counters"]])
                rep["samples"] = list(samples)
                rep["accept_log"] = list(self.accept_log)
                tmp = f"{path}.tmp"
                with open(tmp, "w") as f:
                    json.dump(rep, f)
                os.replace(tmp, path)
            except Exception as exc:  # noqa: BLE001 - reporting never stops the engine
                self.log("warn", f"engine: node report: {exc}")

    def _detect_devices(self) -> list:
        # device processes open their GPUs themselves: name them from the KFD topology without a HIP runtime here
        gpu_free = self.cfg.mining.isolation == "process"
        reg = hal.default_registry(self.cfg.mining.cpu_threads, gpu_free=gpu_free)
        devs = hal.Detector(reg, lambda drv, msg, err: self.log("warn", f"hal: {drv}: {msg}: {err}")).detect()
        sel = self.cfg.mining.gpus.strip().lower()
        if sel == "none":
            devs = [d for d in devs if d.identity().family != hal.Family.GPU]
        elif sel not in ("", "all"):
            keep = {int(x) for x in sel.split(",") if x.strip().isdigit()}
            devs = [d for d in devs if d.identity().family != hal.Family.GPU or d.index in keep]
        return devs

    def _setup_wallet(self) -> str:
        if not self.opts.wallet_passphrase or not self.cfg.data_dir:
            return ""
        try:
            from otedama_amd.lightning.wallet import WalletManager, recovery_phrase_banner
        except ImportError:
            return ""
        try:
            wm = WalletManager(self.cfg.data_dir, self.opts.wallet_passphrase,
                               mnemonic_passphrase=self.opts.wallet_mnemonic_passphrase)
        except Exception as exc:  # noqa: BLE001
            self.log("warn", f"wallet: {exc}")
            return ""
        if wm.is_new:
            self.log("info", "wallet: new wallet created — back up your recovery phrase")
            out = self.opts.output or sys.stdout
            out.write(recovery_phrase_banner(wm.mnemonic, wm.fingerprint))
            out.flush()
        self.log("info", f"wallet: fingerprint {wm.fingerprint}")
        return wm.fingerprint

    async def _uptime_loop(self) -> None:
        while True:
            await asyncio.sleep(1.0)
            self.m.uptime.set(self.opts.clock.now() - self.start_time)

    # ---------------------------------------------------------- curtail
    async def _curtail_loop(self) -> None:
        while True:
            publish_btc_rate(self.m, self._rate_fetcher)
            threshold = self.cfg.curtail_below_btc_usd
            rate, fresh = self._rate_fetcher.btc_usd_rate()
            nxt, changed = curtail_decision(self.curtailed, rate, fresh, threshold)
            if changed:
                self.curtailed = nxt
                if nxt:
                    self.miners.pause_all()
                    self.m.curtailed.set(1)
                    self.log("info", f"engine: curtailed — BTC/USD ${rate:.0f} below threshold ${threshold:.0f}; "
                                     "hashing paused")
                else:
                    self.m.curtailed.set(0)
                    self.log("info", f"engine: uncurtailed — BTC/USD ${rate:.0f} above threshold "
                                     f"${threshold:.0f}; hashing resumes")
                    if self._active_job is not None:
                        self.miners.set_job(self._active_job.template())
            await asyncio.sleep(self.opts.curtail_interval)

    # ---------------------------------------------------------- providers / arbitration
    def _start_providers(self) -> None:
        url = pool_urls(self.cfg)[0]
        mp = MiningProvider(url, self._rate_fetcher, hashrate_func=lambda dev: self.device_hashrates.get(dev, 0.0),
                            algorithm=self.algorithm.name)
        mp.start(self.devices)
        self._providers.append(mp)
        if self.opts.enable_ai_provider:
            ap = AkashProvider(self._rate_fetcher)
            ap.start(self.devices)
            self._providers.append(ap)

    async def _next_quote(self):
        gets = [asyncio.ensure_future(p.quotes.get()) for p in self._providers]
        try:
            done, pending = await asyncio.wait(gets, return_when=asyncio.FIRST_COMPLETED)
        finally:
            for g in gets:
                if not g.done():
                    g.cancel()
        return [d.result() for d in done]

    async def _arbitration_loop(self) -> None:
        dev_refs = [arb.DeviceRef(d.identity(), d.capabilities()) for d in self.devices]
        streams: dict[str, arb.Stream] = {}
        last_quote: dict[str, float] = {}
        prev: arb.Allocation | None = None
        margin = self.cfg.arbitration_hysteresis_pct or DEFAULT_HYSTERESIS
        deadline = time.monotonic() + self.opts.arbitration_interval
        while True:
            timeout = max(deadline - time.monotonic(), 0)
            try:
                quotes = await asyncio.wait_for(self._next_quote(), timeout)
            except asyncio.TimeoutError:
                quotes = None
            for q in quotes or []:
                key = update_stream(streams, q)
                last_quote[key] = q.at or time.time()
            if time.monotonic() < deadline:
                continue
            deadline = time.monotonic() + self.opts.arbitration_interval
            now = time.time()
            for key in [k for k, t in last_quote.items() if now - t > STREAM_STALE_TIMEOUT]:
                streams.pop(key, None)
                last_quote.pop(key, None)
                self.log("info", f"arbitration: stream {key!r} expired (no quote in 3m0s); no longer routing to it")
            merged = streams_slice(streams)
            self.m.active_streams.set(len(merged))
            try:
                alloc = arb.decide(arb.Input(dev_refs, merged, prev, arb.Policy.MAXIMIZE_EARNINGS, margin,
                                             self.cfg.min_yield_sats_per_sec))
            except arb.ArbitrationError as exc:
                self.log("warn", f"arbitration: {exc}")
                continue
            prev_skipped = prev.skipped_device if prev else 0
            prev = alloc
            foregone = 0.0
            for a in alloc.assignments:
                if a.switched_from_id:
                    self.m.arbitration_switches.inc()
                if a.held:
                    self.m.arbitration_holds.inc()
                foregone += a.foregone_sats_per_sec
            self.m.arbitration_foregone.set(foregone)
            self.m.arbitration_expected_yield.set(alloc.total_yield)
            self.m.devices_idle.set(alloc.skipped_device)
            self.activity = {}
            for a in alloc.assignments:
                if not a.idle():
                    self.activity[a.stream] = self.activity.get(a.stream, 0.0) + a.expected_yield
            if alloc.skipped_device != prev_skipped:
                if alloc.skipped_device:
                    self.log("info", f"arbitration: {alloc.skipped_device} device(s) now idle (no viable stream, "
                                     "or below min_yield_sats_per_sec floor)")
                else:
                    self.log("info", "arbitration: all devices now have a viable stream")
            self._apply_allocation(alloc)

    def _apply_allocation(self, alloc: arb.Allocation) -> None:
        for a in alloc.assignments:
            mining = (not a.idle()) and not a.stream.startswith("ai.")
            changed = self.miners.pause_device(a.device_id, paused=not mining)
            if a.idle():
                self.log("info", f"arbitration: {a.device_id} idle ({a.reason or 'no compatible stream'})")
            elif a.switched_from_id:
                was_ai, now_ai = a.switched_from_id.startswith("ai."), a.stream.startswith("ai.")
                if not was_ai and now_ai:
                    self.log("info", f"arbitration: {a.device_id} → AI inference ({a.expected_yield:.0f} sat/s)")
                elif was_ai and not now_ai:
                    self.log("info", f"arbitration: {a.device_id} → mining ({a.expected_yield:.0f} sat/s)")
                else:
                    self.log("info", f"arbitration: {a.device_id} switched to {a.stream} "
                                     f"({a.expected_yield:.0f} sat/s)")
            del changed

    # ---------------------------------------------------------- reconnect loop
    async def _reconnect_loop(self) -> None:
        pools = pool_urls(self.cfg)
        addrs = payout_addresses(self.cfg) or [""]
        pool_idx = addr_idx = attempt = 0
        addr_connected = False
        backoff = RECONNECT_BACKOFF_INITIAL
        while True:
            attempt += 1
            if self.opts.max_reconnect_attempts > 0 and attempt > self.opts.max_reconnect_attempts:
                raise RuntimeError(f"engine: exceeded {self.opts.max_reconnect_attempts} reconnect attempts")
            url = pools[pool_idx]
            pc = self.cfg.pools[pool_idx] if pool_idx < len(self.cfg.pools) else None
            user = session_user(pc.user if pc else "", addrs[addr_idx], self.cfg.workers.name)
            loc = f"attempt {attempt}"
            if len(pools) > 1:
                loc += f", pool {pool_idx + 1}/{len(pools)}"
            if len(addrs) > 1:
                loc += f", address {addr_idx + 1}/{len(addrs)}"
            self.log("info", f"engine: connecting to {url} ({loc})")
            self.m.pool_connect_attempts.inc()
            self.m.pool_active_index.set(pool_idx)
            self.m.payout_active_index.set(addr_idx)
            if addrs[addr_idx]:
                self.m.set_active_payout(mask_addr(addrs[addr_idx]))
            self.m.pool_connection_state.set(1)
            self.pool_url = url

            def on_connected():
                nonlocal addr_connected
                addr_connected = True
                if self.opts.on_ready:
                    self.opts.on_ready(True)

            err: BaseException | None = None
            try:
                await self._run_session(url, user, pc, on_connected)
            except asyncio.CancelledError:
                raise
            except BaseException as exc:  # noqa: BLE001
                err = exc
            if err is not None:
                self.m.pool_connect_failures.inc()
            self.m.pool_connection_state.set(0)
            self.connected = False
            if self.opts.on_ready:
                self.opts.on_ready(False)
            if isinstance(err, FatalPoolError):
                raise err
            if len(pools) > 1:
                pool_idx = (pool_idx + 1) % len(pools)
                if pool_idx != 0:
                    self.log("warn", f"engine: session ended: {err}; failing over to next pool")
                    continue
            if not addr_connected and len(addrs) > 1:
                prev_i = addr_idx
                addr_idx = (addr_idx + 1) % len(addrs)
                pool_idx = 0
                if addr_idx != 0:
                    self.log("warn", f"engine: payout address {mask_addr(addrs[prev_i])} ({prev_i + 1}/{len(addrs)}) "
                                     f"could not establish a session on any pool; failing over to "
                                     f"{mask_addr(addrs[addr_idx])} ({addr_idx + 1}/{len(addrs)})")
                    continue
                addr_connected = False
                self.log("warn", f"engine: none of the {len(addrs)} configured payout addresses could connect; "
                                 f"backing off {backoff:.0f}s and retrying from the primary")
            elif len(pools) > 1:
                self.log("warn", f"engine: all {len(pools)} pools failed; backing off {backoff:.0f}s")
            else:
                self.log("warn", f"engine: session ended: {err}; reconnecting in {backoff:.0f}s")
            await asyncio.sleep(backoff)
            if backoff < RECONNECT_BACKOFF_MAX:
                backoff *= 2

    # ---------------------------------------------------------- session
    async def _dial(self, url: str, creds: Credentials):
        proto = from_url(url)
        d = lookup(proto)
        kw = {"algorithm": self.algorithm.name}
        if proto.value.startswith("stratum-v2"):
            kw["log"] = self.log
        return await d.dial(url, creds, **kw)

    async def _run_session(self, url: str, user: str, pc, on_connected) -> None:
        ca = b""
        if pc is not None and pc.tls_ca_file:
            with open(pc.tls_ca_file, "rb") as f:
                ca = f.read()
        gpu = any(d.identity().family == hal.Family.GPU for d in self.devices)
        creds = Credentials(user=user, password=(pc.password if pc else "") or "x", tls_root_cas_pem=ca,
                            worker=user, version_rolling=self.cfg.mining.version_rolling,
                            device="gfx950" if gpu else "cpu", hardware="v3.0.0",
                            nominal_hashrate=self.current_hashrate,
                            extended_channel=bool(pc.sv2_extended_channel) if pc is not None else False,
                            noise=bool(pc.noise) if pc is not None else False,
                            pool_pubkey=bytes.fromhex(pc.pool_pubkey) if pc is not None and pc.pool_pubkey else b"",
                            noise_suite=pc.noise_suite if pc is not None else "ellswift")
        self._target_grace = min(float(pc.target_grace), TARGET_GRACE) if pc is not None else 0.0
        self._mark("pool_dial")
        session = await self._dial(url, creds)
        self._mark("pool_connected")
        for k, v in (getattr(session, "dial_timing", None) or {}).items():
            self._marks.setdefault(f"pool_{k}", v)
        self._session = session
        self.connected = True
        self.m.pool_connection_state.set(2)
        self.log("info", f"engine: connected to {url} ({session.protocol.value})")
        on_connected()
        tasks = [asyncio.ensure_future(self._job_pump(session)), asyncio.ensure_future(self._share_pump(session)),
                 asyncio.ensure_future(self._stats_loop(session)), asyncio.ensure_future(self._notice_pump(session))]
        try:
            closed = asyncio.ensure_future(session.wait_closed())
            done, _ = await asyncio.wait(tasks + [closed], return_when=asyncio.FIRST_COMPLETED)
            for t in done:
                if t is not closed and t.exception() is not None:
                    raise t.exception()
            raise ConnectionError("engine: pool closed connection")
        finally:
            for t in tasks:
                t.cancel()
            await session.close()
            self._session = None
            self.miners.pause_all()
            self._active_job = None
            self._valid_jobs.clear()
            self._job_targets.clear()
            self._prev_targets.clear()

    async def _notice_pump(self, session) -> None:
        while True:
            n = await session.notices.get()
            self.log("info", f"engine: pool notice: {n}")

    async def _job_pump(self, session) -> None:
        while True:
            job = await session.jobs.get()
            self.m.last_job_received.set(time.time())
            if job is None:
                self._active_job = None
                self._valid_jobs.clear()
                self._job_targets.clear()
                self._prev_targets.clear()
                self.miners.pause_all()
                continue
            if job.clean_jobs:
                if job.job_id not in self._valid_jobs:
                    self._submitted.clear()
                self._valid_jobs = {job.job_id}
                self._job_targets = {k: v for k, v in self._job_targets.items() if k == job.job_id}
                self._prev_targets = {k: v for k, v in self._prev_targets.items() if k == job.job_id}
            else:
                self._valid_jobs.add(job.job_id)
            # the job's current share target: a target-only update (SV2 SetTarget) re-issues the same job id
            new_t = int.from_bytes(job.target, "little") if job.target else None
            old_t = self._job_targets.get(job.job_id)
            if old_t is not None and new_t is not None and new_t < old_t:
                self._prev_targets[job.job_id] = (old_t, time.monotonic())
            self._job_targets[job.job_id] = new_t
            self._active_job = job
            publish_difficulty(self.m, session.suggested_difficulty(), self.current_hashrate,
                               float(2 ** 256) / self.algorithm.diff1)
            if self.curtailed:
                self.log("debug", f"engine: job {job.job_id} ignored (curtailed)")
                continue
            self.miners.set_job(job.template())
            self._mark("first_job_to_devices")
            self.log("info", f"engine: job {job.job_id} version=0x{job.version:08X} active")

    async def _share_pump(self, session) -> None:
        """Drain the miners' share queues. Native queues signal an eventfd on every push (loop.add_reader), so a
        share is picked up within one event-loop turn of being queued instead of a polling interval."""
        loop = asyncio.get_running_loop()
        wake = asyncio.Event()
        fds = list(self.miners.share_fds()) if hasattr(self.miners, "share_fds") else []
        for fd in fds:
            loop.add_reader(fd, _ack_eventfd, fd, wake)
        try:
            await self._share_pump_loop(session, wake, bool(fds))
        finally:
            for fd in fds:
                try:
                    loop.remove_reader(fd)
                except (ValueError, OSError):
                    pass

    async def _share_pump_loop(self, session, wake: asyncio.Event, has_fds: bool) -> None:
        while True:
            shares = self.miners.poll(256)  # native queue drain; releases the GIL, never blocks
            if not shares:
                wake.clear()
                shares = self.miners.poll(256)  # re-check after clearing: a push in between is not lost
            if not shares:
                if has_fds:
                    try:
                        await asyncio.wait_for(wake.wait(), SHARE_WAKE_FALLBACK)
                    except asyncio.TimeoutError:
                        pass
                else:
                    await asyncio.sleep(SHARE_POLL_INTERVAL)
                continue
            for s in shares:
                self.m.shares_found.inc()
                self.m.inc_shares_found_for_device(s["device_id"])
                if s["job_id"] not in self._valid_jobs:
                    self.m.stale_skipped.inc()
                    continue
                # Verified on the device's host thread against the target it had then; a share still queued when
                # the pool raised the target would only be rejected as low-difficulty (the vardiff race right after
                # connect), so it is dropped here instead.
                tgt, h = self._job_targets.get(s["job_id"]), s.get("hash")
                if tgt is not None and h and int.from_bytes(h, "little") > tgt:
                    prev = self._prev_targets.get(s["job_id"])
                    hv = int.from_bytes(h, "little")
                    if prev is None or hv > prev[0] or time.monotonic() - prev[1] > self._target_grace:
                        self.m.below_target_skipped.inc()
                        continue
                en2 = extranonce2_bytes(s["extranonce2"], s["extranonce2_size"])
                key = (s["job_id"], s["nonce"], s["ntime"], s["version"], en2)
                if key in self._submitted:  # defence in depth: never send a pool a duplicate
                    continue
                self._submitted.add(key)
                sub = ShareSubmission(s["job_id"], s["nonce"], s["ntime"], s["version"], en2)
                t = asyncio.ensure_future(self._submit(session, sub, s.get("found_at", 0.0),
                                                       s.get("device_found_at", 0.0), s.get("device_id", "")))
                self._submit_tasks.add(t)
                t.add_done_callback(self._submit_tasks.discard)

    async def _submit(self, session, sub: ShareSubmission, found_at: float = 0.0,
                      device_found_at: float = 0.0, device_id: str = "") -> None:
        self.m.shares_submitted.inc()
        trace_mark("otd.share.submit")
        try:
            res = await session.submit(sub)
        except Exception as exc:  # noqa: BLE001
            self.log("warn", f"engine: submit share: {exc}")
            return
        trace_mark("otd.share.ack")
        if res.accepted:
            self.m.shares_accepted.inc()
            self.latency.record(res.latency_ms)
            now = time.monotonic()
            origin = "remote" if device_id.startswith("rank") else "local"
            host_ms = dev_ms = None
            if found_at > 0:  # host verify -> pool accept (native queue + submit + pool validation)
                host_ms = (now - found_at) * 1e3
                self.pipeline_latency.record(host_ms)
            if device_found_at > 0:  # the kernel's hit (s_memrealtime on the host clock) -> pool accept
                dev_ms = (now - device_found_at) * 1e3
                self.device_latency.record(dev_ms)
                self.device_latency_by_origin[origin].record(dev_ms)
            self.accept_log.append((now, dev_ms, origin, device_id, host_ms))
            self.log("info", f"engine: share accepted job={sub.job_id} nonce=0x{sub.nonce:08X} "
                             f"({res.latency_ms:.1f} ms)")
        else:
            cat, diag = reject_class(res.reason)
            self.m.shares_rejected.inc()
            self.m.reject_reason(cat).inc()
            self.m.touch_last_reject(cat, time.time())
            self.log("warn", f"engine: share rejected: {res.reason} ({diag})")

    async def _stats_loop(self, session) -> None:
        while True:
            await asyncio.sleep(self.opts.stats_interval)
            self.tick_stats(session)

    def tick_stats(self, session=None) -> None:
        now = self.opts.clock.now()
        total = self.miners.total_hashes()
        rate = self.hash_window.observe(total, now)
        self.device_hashrates = self.miners.update_hashrates()
        exact = getattr(self.miners, "exact_total", None)
        exact_rate = exact() if exact is not None else None
        if exact_rate is not None:  # GPU miners: device-timeline spans, no launch quantization
            rate = exact_rate
        self.current_hashrate = rate
        for dev, r in self.device_hashrates.items():
            self.m.set_device_hashrate(dev, r)
        shares = self.m.shares_found.value()
        self.log("info", f"engine: hashrate={hashrate_string(rate)} shares={shares}")
        dropped = self.miners.total_dropped()
        if dropped > self._last_dropped:
            self.log("warn", f"engine: dropped {dropped - self._last_dropped} found share(s) — share submission is "
                             "not keeping up with discovery")
            self._last_dropped = dropped
        for dev, err in self.miners.retire_faulted():
            self.log("error", f"engine: device {dev} faulted: {err}")
        stalled_devs = self.miners.stalled()
        dstats = self.miners.device_stats()
        self._publish_device_activity(dstats, now)
        self._publish_candidate_losses(dstats)
        link = getattr(self.miners, "link", None)
        if link is not None:
            self.m.node_ranks.set(link.world)
            self.m.node_collective_seconds.set(link.tick_quantile(0.5))
            self.m.node_collective_p99.set(link.tick_quantile(0.99))
            self.m.node_collectives.set(link.comm.collectives)
            self.m.node_generation.set(max(getattr(getattr(link.comm, "info", None), "generation", 0), 0))
            self.m.node_lost_ranks.set(len(getattr(self.miners, "lost_ranks", []) or []))
            self.m.node_share_previews.set(getattr(self.miners, "share_previews", 0))
            self.m.node_remote_stale.set(getattr(self.miners, "remote_stale", 0))
        self.m.devices_faulted.set(sum(1 for s in dstats.values() if s["faulted"]))
        self.m.devices_stalled.set(len(stalled_devs))
        self.m.devices_active.set(len(self.miners.live()) - len(stalled_devs))
        if self.curtailed:
            self.m.up.set(1)
            self.stalled = False
        else:
            self._hashmon.observe(rate)
            self.stalled = self._hashmon.stalled()
            self.m.up.set(0 if self.stalled else 1)
        self.est_sats = self._sats.observe(now, self.m.arbitration_expected_yield.value(), rate > 0 and not self.stalled)
        self.m.hashrate.set(rate)
        self._uptime.observe(now, rate > 0 and not self.stalled, self.m.productive_seconds)
        self.m.effective_yield.set(effective_yield(self.m.arbitration_expected_yield.value(),
                                                   float(self.m.productive_seconds.value()), self.m.uptime.value()))
        if self.cfg.power_watts > 0:
            self.m.power_watts.set(self.cfg.power_watts)
            if rate > 0:
                self.m.joules_per_terahash.set(self.cfg.power_watts * 1e12 / rate)
        acc_rate, judged = self.m.update_share_rates()
        if judged >= 20 and acc_rate < 0.97:
            self.log("warn", f"engine: share acceptance {acc_rate * 100:.1f}% ({self.m.shares_accepted.value()}/"
                             f"{judged}) — check the reject-reason breakdown")
        if self.device_latency.quantile(0.5) > 0:
            self.m.hit_latency_p50.set(self.device_latency.quantile(0.5))
            self.m.hit_latency_p95.set(self.device_latency.quantile(0.95))
            self.m.hit_latency_p99.set(self.device_latency.quantile(0.99))
        switches = [float(st.get("last_job_switch_ms", 0.0) or 0.0) for st in dstats.values()]
        if switches:
            self.m.job_switch_ms.set(max(switches))
        p95 = self.latency.quantile(0.95)
        if p95 > 0:
            p50, p99 = self.latency.quantile(0.5), self.latency.quantile(0.99)
            self.log("info", f"engine: submit latency p50={p50:.0f}ms p95={p95:.0f}ms p99={p99:.0f}ms")
            self.m.submit_latency_p50.set(p50)
            self.m.submit_latency_p95.set(p95)
            self.m.submit_latency_p99.set(p99)
        if session is not None:
            publish_difficulty(self.m, session.suggested_difficulty(), rate, float(2 ** 256) / self.algorithm.diff1)
        if self.dashboard is not None:
            self.dashboard.update(self.stats())


    def _publish_device_activity(self, dstats: dict, now: float) -> None:
        """Per-device busy ratio and launch counts from the native miners' cumulative stats (remote node ranks
        report only hash/share counters and are skipped)."""
        for dev, st in dstats.items():
            if "busy_seconds" not in st:
                continue
            busy, launches = float(st["busy_seconds"]), int(st.get("launches", 0))
            prev = self._busy_prev.get(dev)
            self._busy_prev[dev] = (busy, now, launches)
            if prev is None:
                continue
            dt = now - prev[1]
            if dt > 0:
                threads = max(int(st.get("threads", 1) or 1), 1)
                self.m.set_device_busy(dev, min(max((busy - prev[0]) / (dt * threads), 0.0), 1.0))
            self.m.add_device_launches(dev, launches - prev[2])

    def _publish_candidate_losses(self, dstats: dict) -> None:
        """Kernel candidates that never reached the share queue (device hit-ring overflow, scrypt verifier queue
        bound): counted per device and cause, and warned about when they grow."""
        for dev, st in dstats.items():
            for key, cause in (("ring_overflow", "ring_overflow"), ("verify_dropped", "verify_queue_full")):
                n = int(st.get(key, 0) or 0)
                prev = self._lost_prev.get((dev, cause), 0)
                if n > prev:
                    self.m.add_device_candidates_lost(dev, cause, n - prev)
                    self.log("warn", f"engine: device {dev} lost {n - prev} candidate(s) ({cause}); the share "
                                     "target is too easy for the device's launch size / verifier")
                self._lost_prev[(dev, cause)] = n


def _ack_eventfd(fd: int, wake: asyncio.Event) -> None:
    """add_reader callback: reset the native queue's eventfd and wake the share pump."""
    try:
        os.read(fd, 8)
    except (BlockingIOError, InterruptedError):
        pass
    wake.set()


def update_stream(streams: dict[str, arb.Stream], q) -> str:
    """Quote -> stream keyed provider:device; NET yield (fixes arbitrate.go:187-195)."""
    key = f"{q.provider_id}:{q.device_id}"
    s = streams.get(key) or arb.Stream(id=q.provider_id)
    s.id = q.provider_id
    s.accepts_families = list(q.accepted_families)
    y = arb.Yield(q.yield_.net_sats_per_second, q.yield_.confidence)
    if q.device_id:
        s.yield_per_device[q.device_id] = y
    s.default_yield = y
    s.is_bitcoin_mining = q.provider_id == "mining.stratum"
    streams[key] = s
    return key


def streams_slice(streams: dict[str, arb.Stream]) -> list[arb.Stream]:
    merged: dict[str, arb.Stream] = {}
    for s in streams.values():
        rep = merged.get(s.id)
        if rep is not None:
            rep.yield_per_device.update(s.yield_per_device)
        else:
            merged[s.id] = arb.Stream(s.id, list(s.accepts_families), dict(s.yield_per_device), s.default_yield,
                                      s.privacy_rating, s.environmental_rating, s.is_bitcoin_mining)
    return list(merged.values())


async def run(opts: Options) -> None:
    await Engine(opts).run()


__all__ = ["Engine", "Options", "curtail_decision", "mask_addr", "payout_addresses", "pool_urls", "run",
           "session_user", "streams_slice", "update_stream"]
