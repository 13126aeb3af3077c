"""Device miners: native GpuMiner per MI355X + CpuMiner, with disjoint stripes.

Parity: internal/engine/setup.go startMinerWorkers (:59-77) + miner.Worker
(internal/miner/worker.go) + the share fan-in (internal/engine/fanin.go:22-68).
Each device runs a native host thread (csrc/runtime) that owns its HIP stream
and launch loop; this class only hands out job templates (with the device's
variant stripe) and drains the native share queues.

Reference defect fixed: every device gets a disjoint slice of the search space
instead of the identical Work (engine/run.go:1294-1296).

Device faults (the reference has no GPU path and a dead worker
goroutine just stops contributing): a GpuMiner whose host thread died on a HIP
error is retired by ``retire_faulted()`` and the rank's variant class is
re-split among the surviving devices (parallel/partition.py). The new stripes
take effect with the next *new* work: switching stripes mid-job would restart
the survivors' cursors over variants they already searched and re-submit
duplicate shares. Per-device stalls (a live device with work whose hash counter
stopped moving for ``stall_samples`` ticks) are reported by ``stalled()``.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field

from otedama_amd.hal import Family, SimpleDevice
from otedama_amd.ops.native import require_native
from otedama_amd.parallel.partition import stripe_for

# Template keys that do not change the search space (same as the native same_work()).
_NOT_WORK = frozenset({"target", "job_id", "epoch", "channel_id", "variant_start", "variant_stride"})


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
    hashrate: float = 0.0
    idle_samples: int = 0  # consecutive stats ticks with work but no hash progress
    extra: dict = field(default_factory=dict)

    @property
    def id(self) -> str:
        return self.device.identity().id


class MinerSet:
    def __init__(self, devices: list, algorithm: str = "sha256d", batch_nonces: int = 1 << 29,
                 cpu_threads: int = 0, rank: int = 0, world_size: int = 1, log=None, queue_cap: int = 4096,
                 stall_samples: int = 3, sha_variants: int = 128):
        N = require_native()
        self.algorithm = algorithm
        self.log = log or (lambda level, msg: None)
        self.miners: list[DeviceMiner] = []
        gpus = [d for d in devices if d.identity().family == Family.GPU and d.index >= 0
                and d.capabilities().supports(algorithm)]
        for d in gpus:
            cus = int(d.extra.get("cus", 256))
            m = N.GpuMiner(d.index, d.identity().id, batch_nonces=batch_nonces, grid=cus * 6, queue_cap=queue_cap,
                           sha_variants=sha_variants)
            self.miners.append(DeviceMiner(d, m))
        cpus = [d for d in devices if d.identity().family == Family.CPU]
        if cpus and algorithm == "sha256d" and (cpu_threads > 0 or not gpus):
            threads = cpu_threads or cpus[0].threads
            self.miners.append(DeviceMiner(cpus[0], N.CpuMiner(threads, cpus[0].identity().id, queue_cap),
                                           extra={"threads": max(int(threads or 1), 1)}))
        self.rank, self.world_size = rank, world_size
        self.stall_samples = max(1, stall_samples)
        self._restripe_pending = False
        self._restripe()
        self._lock = threading.Lock()
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
        for m in self.miners:
            m.native.stop()

    def set_job(self, template: dict | None, epoch: int | None = None) -> int:
        """Hand a job template to every non-paused device; returns the new epoch.

        ``epoch`` is given by node workers so hits map back to rank 0's job table."""
        with self._lock:
            self._epoch = epoch if epoch is not None else self._epoch + 1
            new = dict(template) if template is not None else None
            if self._restripe_pending and new is not None and _work_key(new) != _work_key(self._template):
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
        t["epoch"] = self._epoch
        t["variant_start"] = m.stripe_index
        t["variant_stride"] = m.stripe_stride
        m.native.set_job(t)

    def live(self) -> list[DeviceMiner]:
        return [m for m in self.miners if not m.retired]

    def retire_faulted(self) -> list[tuple[str, str]]:
        """Retire devices whose native thread died; returns the newly retired ``(id, error)``.

        The survivors take over the retired stripes at the next new work (see module doc)."""
        out = []
        with self._lock:
            for m in self.miners:
                if m.retired:
                    continue
                st = m.native.stats()
                if st["faulted"]:
                    m.retired = True
                    m.hashrate = 0.0
                    m.native.stop()
                    out.append((m.id, st["error"]))
            if out:
                self._restripe_pending = True
                live = len(self.live())
                for dev, err in out:
                    self.log("error", f"miners: device {dev} faulted ({err}); retired, {live} device(s) left")
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
            h = m.native.stats()["hashes"]
            m.hashrate = 0.0 if m.retired else max(h - m.last_hashes, 0) / dt
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

    def hashrate_of(self, device_id: str) -> float:
        for m in self.miners:
            if m.id == device_id:
                return m.hashrate
        return 0.0
