"""Device miners: native GpuMiner per MI355X + CpuMiner, with disjoint stripes.

Parity: internal/engine/setup.go startMinerWorkers (:59-77) + miner.Worker
(internal/miner/worker.go) + the share fan-in (internal/engine/fanin.go:22-68).
Each device runs a native host thread (csrc/runtime) that owns its HIP stream
and launch loop; this class only hands out job templates (with the device's
variant stripe) and drains the native share queues.

Reference defect fixed: every device gets a disjoint slice of the search space
instead of the identical Work (engine/run.go:1294-1296).

Isolation (``isolation="process"``, the default for GPUs in ``otedama run``):
every device runs in a child process of its own (engine/devproc.py), so a
kernel fault that aborts a process takes one device down, not the node.

Device faults (the reference has no GPU path and a dead worker
goroutine just stops contributing): a device whose miner died (HIP error in its
host thread, or its process exited) is retired and the rank's variant class is
re-split among the survivors AT ONCE, starting past the high-water mark of every
device's cursor on the current work (the native miners report the next variant
they have not started, tagged with the job epoch), so the dead device's residue
class keeps being searched and nothing is searched twice. A dead device process
is replaced after a backoff (1 s doubling to 64 s, internal/engine/run.go:56-63);
when the fresh process reports in, the stripes are re-split again to include it.
Per-device stalls (a live device with work whose hash counter stopped moving for
``stall_samples`` ticks) are reported by ``stalled()``.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field

from otedama_amd.hal import Family, SimpleDevice
from otedama_amd.ops.native import require_native
from otedama_amd.ops.tuning import sha256d_grid
from otedama_amd.parallel.partition import stripe_for

# Template keys that do not change the search space (same as the native same_work()).
_NOT_WORK = frozenset({"target", "job_id", "epoch", "channel_id", "variant_start", "variant_stride"})
RESPAWN_BACKOFF_INITIAL = 1.0
RESPAWN_BACKOFF_MAX = 64.0
RESPAWN_HEALTHY_RESET = 60.0  # a process that ran this long resets its backoff
# Re-split margin in variant groups: a device may start one more 128-variant group between its last cursor report
# and the re-split, so the new base clears every reported cursor by two groups of the old stride.
RESPLIT_GROUPS = 2
GROUP = 128


def _work_key(t: dict | None):
    return None if t is None else repr(sorted((k, v) for k, v in t.items() if k not in _NOT_WORK))


@dataclass
class DeviceMiner:
    device: SimpleDevice
    native: object
    stripe_index: int = 0
    stripe_stride: int = 1
    paused: bool = False
    retired: bool = False  # faulted and removed from the stripe plan
    last_hashes: int = 0
    last_done_at: float = 0.0  # device-timeline completion time of last_hashes (GPU miners)
    hashrate: float = 0.0
    exact: bool = False  # hashrate came from a device-timeline span (not a wall-clock sample) at the last tick
    timeline: bool = False  # the miner reports device-timeline completions (GPU); CPU counters move continuously
    idle_samples: int = 0  # consecutive stats ticks with work but no hash progress
    extra: dict = field(default_factory=dict)
    backoff: float = RESPAWN_BACKOFF_INITIAL
    respawn_timer: threading.Timer | None = None

    @property
    def id(self) -> str:
        return self.device.identity().id


def variant_space(t: dict) -> int:
    """Number of header variants of a template: 2^popcount(version_mask) x extranonce2 values x (ntime_roll + 1),
    saturating at 2^64 - 1 (csrc/runtime/miner_common.cpp JobTemplate::variant_space)."""
    cap = (1 << 64) - 1
    e2 = 1
    if t.get("coinb1") is not None and int(t.get("extranonce2_size", 0) or 0) > 0:
        size = int(t["extranonce2_size"])
        e2 = cap if size >= 8 else 1 << (8 * size)
    v = 1 << bin(int(t.get("version_mask", 0) or 0) & 0xFFFFFFFF).count("1")
    return min(e2 * v * (int(t.get("ntime_roll", 0) or 0) + 1), cap)


class MinerSet:
    def __init__(self, devices: list, algorithm: str = "sha256d", batch_nonces: int = 1 << 32,
                 cpu_threads: int = 0, rank: int = 0, world_size: int = 1, log=None, queue_cap: int = 4096,
                 stall_samples: int = 3, sha_variants: int = 128, isolation: str = "thread"):
        if isolation not in ("thread", "process"):
            raise ValueError("isolation must be 'thread' or 'process'")
        # with every device in its own process this process never needs the extension (or the HIP runtime it links)
        N = require_native() if isolation == "thread" else None
        self.N = N
        self.algorithm = algorithm
        self.isolation = isolation
        self.log = log or (lambda level, msg: None)
        self.miners: list[DeviceMiner] = []
        self._lock = threading.RLock()
        self._stopped = False
        gpus = [d for d in devices if d.identity().family == Family.GPU and d.index >= 0
                and d.capabilities().supports(algorithm)]
        for d in gpus:
            cus = int(d.extra.get("cus", 256))
            if isolation == "process":
                from otedama_amd.engine.devproc import DeviceProcess

                m = DeviceProcess(d.index, d.identity().id, batch_nonces=batch_nonces, grid=sha256d_grid(cus),
                                  queue_cap=queue_cap, sha_variants=sha_variants, log=self.log,
                                  on_exit=self._on_process_exit, on_ready=self._on_process_ready)
            else:
                m = N.GpuMiner(d.index, d.identity().id, batch_nonces=batch_nonces, grid=sha256d_grid(cus), queue_cap=queue_cap,
                               sha_variants=sha_variants)
            self.miners.append(DeviceMiner(d, m))
        cpus = [d for d in devices if d.identity().family == Family.CPU and d.capabilities().supports(algorithm)]
        if cpus and (cpu_threads > 0 or not gpus):
            if isolation == "process":
                # one process per CPU device (production has one, cpu-0; tests model several devices this way)
                from otedama_amd.engine.devproc import DeviceProcess

                for d in cpus:
                    threads = max(int(cpu_threads or d.threads or 1), 1)
                    m = DeviceProcess(-1, d.identity().id, queue_cap=queue_cap, cpu_threads=threads, log=self.log,
                                      on_exit=self._on_process_exit, on_ready=self._on_process_ready)
                    self.miners.append(DeviceMiner(d, m, extra={"threads": threads}))
            else:
                threads = cpu_threads or cpus[0].threads
                self.miners.append(DeviceMiner(cpus[0], N.CpuMiner(threads, cpus[0].identity().id, queue_cap),
                                               extra={"threads": max(int(threads or 1), 1)}))
        self.rank, self.world_size = rank, world_size
        self.stall_samples = max(1, stall_samples)
        self._restripe_pending = False
        self._variant_base = 0   # local re-split offset on top of the template's (node-level) variant_base
        self._work_epoch0 = 0    # first epoch of the current work (cursor reports older than this are ignored)
        self.resplits = 0
        self._restripe()
        self._epoch = 0
        self._template: dict | None = None
        self._t_last = time.monotonic()

    def _restripe(self) -> None:
        live = [m for m in self.miners if not m.retired]
        for i, m in enumerate(live):
            st = stripe_for(self.rank, self.world_size, i, len(live))
            m.stripe_index, m.stripe_stride = st.start, st.stride

    @property
    def stripe_total(self) -> int:
        """Variant stride of this rank's live devices (world x live)."""
        return self.world_size * max(1, sum(1 for m in self.miners if not m.retired))

    def __len__(self) -> int:
        return len(self.miners)

    def start(self) -> None:
        for m in self.miners:
            m.native.start()

    def stop(self) -> None:
        with self._lock:
            self._stopped = True
            for m in self.miners:
                if m.respawn_timer is not None:
                    m.respawn_timer.cancel()
        for m in self.miners:
            m.native.stop()

    def set_rank(self, rank: int, world_size: int) -> None:
        """Node re-formed (parallel/node.py): this rank's residue class changed. Takes effect with the next
        set_job (the node leader re-sends the job, with a fresh variant_base, right after a re-form)."""
        with self._lock:
            self.rank, self.world_size = rank, world_size
            self._variant_base = 0
            self._restripe()

    def set_job(self, template: dict | None, epoch: int | None = None) -> int:
        """Hand a job template to every non-paused device; returns the new epoch.

        ``epoch`` is given by node workers so hits map back to rank 0's job table."""
        with self._lock:
            self._epoch = epoch if epoch is not None else self._epoch + 1
            new = dict(template) if template is not None else None
            if new is not None and _work_key(new) != _work_key(self._template):
                # new work: cursors restart, the local re-split offset is void
                self._work_epoch0 = self._epoch
                self._variant_base = 0
                if self._restripe_pending:
                    self._restripe()
                    self._restripe_pending = False
                    self.log("info", f"miners: variant stripes re-split over {len(self.live())} live device(s)")
            self._template = new
            for m in self.miners:
                self._apply(m)
            return self._epoch

    def _apply(self, m: DeviceMiner) -> None:
        if m.retired:
            return
        if self._template is None or m.paused:
            m.native.set_job(None)
            return
        t = dict(self._template)
        node_base = int(t.pop("variant_base", 0) or 0)
        t["epoch"] = self._epoch
        t["variant_start"] = node_base + self._variant_base + m.stripe_index
        t["variant_stride"] = m.stripe_stride
        m.native.set_job(t)

    def live(self) -> list[DeviceMiner]:
        return [m for m in self.miners if not m.retired]

    # ------------------------------------------------------------------ faults and re-splits
    def high_water(self) -> int:
        """Highest 'next unstarted variant' reported by any device (live or dead) for the current work."""
        hw = 0
        for m in self.miners:
            try:
                st = m.native.stats()
            except Exception:  # noqa: BLE001
                continue
            if int(st.get("variant_epoch", -1)) >= self._work_epoch0 > 0:
                hw = max(hw, int(st.get("variant_next", 0)))
        return hw

    def _resplit_now(self, why: str) -> None:
        """Re-split this rank's class over the live devices past every cursor of the current work, and re-issue
        the work at once (caller holds the lock). Falls back to a re-split at the next new work when the jump
        does not fit in the job's variant space."""
        live = self.live()
        old = [(m.stripe_index, m.stripe_stride) for m in self.miners]
        old_stride = max((st for _, st in old), default=1)
        self._restripe()
        if self._template is None or not live:
            self._restripe_pending = False
            return
        t = self._template
        node_base = int(t.get("variant_base", 0) or 0)
        hw = self.high_water()
        base = max(hw - node_base, 0) + RESPLIT_GROUPS * GROUP * old_stride
        # a device cursor sits in this rank's residue class (rank mod world): the offset itself must stay a multiple
        # of world_size, or the new stripes would land in another rank's class (duplicates there, a gap here)
        base = -(-base // self.world_size) * self.world_size
        probe = {k: v for k, v in t.items() if k != "variant_base"}
        try:
            space = int(self.N.variant_space(probe)) if self.N is not None else variant_space(probe)
        except Exception:  # noqa: BLE001 - a template the native side cannot parse: keep the deferred path
            space = 0
        if node_base + base + self.stripe_total > space:
            for m, (i, st) in zip(self.miners, old):  # keep the running stripes until the next new work
                m.stripe_index, m.stripe_stride = i, st
            self._restripe_pending = True
            self.log("warn", f"miners: {why}; variant space exhausted for an immediate re-split, the "
                             f"{len(live)} live device(s) take the new stripes with the next work")
            return
        self._variant_base = base
        self._restripe_pending = False
        self.resplits += 1
        for m in self.miners:
            self._apply(m)
        self.log("info", f"miners: {why}; {len(live)} live device(s) re-split from variant {node_base + base}")

    def _on_process_exit(self, dp) -> None:
        """A device process died (reader thread): retire its device, re-split, schedule a fresh process."""
        with self._lock:
            if self._stopped:
                return
            for m in self.miners:
                if m.native is dp and not m.retired:
                    m.retired = True
                    m.hashrate = 0.0
                    self._resplit_now(f"device {m.id} lost ({dp.error})")
                    self._schedule_respawn(m)

    def _schedule_respawn(self, m: DeviceMiner) -> None:
        if m.respawn_timer is not None:
            m.respawn_timer.cancel()
        ready_at = getattr(m.native, "ready_at", 0.0)
        if ready_at and time.monotonic() - ready_at >= RESPAWN_HEALTHY_RESET:
            m.backoff = RESPAWN_BACKOFF_INITIAL
        delay = m.backoff
        m.backoff = min(m.backoff * 2, RESPAWN_BACKOFF_MAX)
        m.respawn_timer = threading.Timer(delay, self._respawn, args=(m,))
        m.respawn_timer.daemon = True
        m.respawn_timer.start()
        self.log("info", f"miners: restarting {m.id} in {delay:.0f}s")

    def _respawn(self, m: DeviceMiner) -> None:
        with self._lock:
            if self._stopped or not m.retired:
                return
        try:
            spawned = m.native.restart(replay_job=False)  # its stripe is re-assigned past every cursor once ready
        except Exception as exc:  # noqa: BLE001
            self.log("error", f"miners: restart of {m.id} failed: {exc}")
            spawned = False
        if spawned is False:  # failed, or the killed child was not reaped yet (restart() refuses a live process)
            with self._lock:
                if not self._stopped and m.retired:
                    self._schedule_respawn(m)

    def _on_process_ready(self, dp) -> None:
        """A (re)spawned device process is mining: bring its device back into the stripe plan."""
        with self._lock:
            if self._stopped:
                return
            for m in self.miners:
                if m.native is dp and m.retired:
                    m.retired = False
                    m.idle_samples = 0
                    self._resplit_now(f"device {m.id} back (process restart {dp.restarts})")

    def retire_faulted(self) -> list[tuple[str, str]]:
        """Retire devices whose native thread died; returns the newly retired ``(id, error)``. The survivors take
        over the retired stripes at once (see module doc); a device process is also restarted."""
        out = []
        with self._lock:
            newly = []
            for m in self.miners:
                if m.retired:
                    continue
                st = m.native.stats()
                if st["faulted"]:
                    m.retired = True
                    m.hashrate = 0.0
                    if not hasattr(m.native, "restart"):
                        m.native.stop()
                    out.append((m.id, st["error"]))
                    newly.append(m)
            if out:
                live = len(self.live())
                for dev, err in out:
                    self.log("error", f"miners: device {dev} faulted ({err}); retired, {live} device(s) left")
                self._resplit_now(", ".join(f"device {d} faulted" for d, _ in out))
                for m in newly:
                    if hasattr(m.native, "restart"):
                        if getattr(m.native, "alive", False):
                            m.native.kill()  # a faulted context is unusable: replace the process
                        self._schedule_respawn(m)
        return out

    def stalled(self) -> list[str]:
        """Live devices that have work but made no hash progress for ``stall_samples`` ticks."""
        return [m.id for m in self.miners if not m.retired and m.idle_samples >= self.stall_samples]

    @property
    def epoch(self) -> int:
        return self._epoch

    def pause_device(self, device_id: str, paused: bool = True) -> bool:
        with self._lock:
            for m in self.miners:
                if m.id == device_id:
                    if m.paused != paused:
                        m.paused = paused
                        self._apply(m)
                    return True
        return False

    def pause_all(self) -> None:
        self.set_job(None)

    def poll(self, max_per_device: int = 256) -> list[dict]:
        out = []
        for m in self.miners:
            out.extend(m.native.poll(max_per_device))
        return out

    def share_fds(self) -> list[int]:
        """eventfds that turn readable when a device queues a share (native ShareQueue / device process)."""
        return [m.native.share_fd() for m in self.miners if hasattr(m.native, "share_fd")]

    def device_stats(self) -> dict[str, dict]:
        out = {}
        for m in self.miners:
            st = m.native.stats()
            if "threads" in m.extra:  # CPU: busy_seconds sums thread time
                st["threads"] = m.extra["threads"]
            out[m.id] = st
        return out

    def total_hashes(self) -> int:
        return sum(s["hashes"] for s in self.device_stats().values())

    def total_dropped(self) -> int:
        return sum(s["dropped"] for s in self.device_stats().values())

    def faulted(self) -> list[tuple[str, str]]:
        return [(k, s["error"]) for k, s in self.device_stats().items() if s["faulted"]]

    def update_hashrates(self) -> dict[str, float]:
        now = time.monotonic()
        dt = max(now - self._t_last, 1e-6)
        self._t_last = now
        rates = {}
        working = self._template is not None
        for m in self.miners:
            st = m.native.stats()
            h = st["hashes"]
            done = float(st.get("hashes_done_at_s", 0.0) or 0.0)
            # GPU counters move in whole launches (2^32 hashes, ~0.22 s): over the device-timeline span between the
            # counted completions the rate is exact; sampled against wall time it jitters by a launch per interval
            span = done - m.last_done_at
            m.exact = False
            m.timeline = done > 0
            if m.retired:
                m.hashrate = 0.0
            elif done > 0 and m.last_done_at > 0 and span > 0 and h > m.last_hashes:
                m.hashrate = (h - m.last_hashes) / span
                m.exact = True
            else:
                m.hashrate = max(h - m.last_hashes, 0) / dt
            m.last_done_at = done
            if working and not m.paused and not m.retired and h == m.last_hashes:
                m.idle_samples += 1
                if m.idle_samples == self.stall_samples:
                    self.log("warn", f"miners: device {m.id} made no hash progress for {m.idle_samples} "
                                     "samples with work assigned (hung kernel / thermal / driver?)")
            else:
                m.idle_samples = 0
            m.last_hashes = h
            rates[m.id] = m.hashrate
        return rates

    def exact_total(self) -> float | None:
        """Sum of the device rates when every live GPU miner's rate at the last tick came from a device-timeline span
        (CPU miners add their wall-clock rate), else None (the engine then keeps its wall-clock window). A wall-clock window over GPU counters that move a
        whole launch (2^32 hashes) at a time, refreshed by a device process's heartbeats, misreads a short interval
        by a launch or more (a 1 s window at 19.3 GH/s read 25.7)."""
        live = [m for m in self.miners if not m.retired]
        if not any(m.exact for m in live) or any(m.timeline and not m.exact for m in live):
            return None
        # CPU miners (no device timeline) count continuously: their wall-clock rate is already smooth
        return sum(m.hashrate for m in live)

    def hashrate_of(self, device_id: str) -> float:
        for m in self.miners:
            if m.id == device_id:
                return m.hashrate
        return 0.0
