"""Device miners: native GpuMiner per MI355X + CpuMiner, with disjoint stripes.

Parity: internal/engine/setup.go startMinerWorkers (:59-77) + miner.Worker
(internal/miner/worker.go) + the share fan-in (internal/engine/fanin.go:22-68).
Each device runs a native host thread (csrc/runtime) that owns its HIP stream
and launch loop; this class only hands out job templates (with the device's
variant stripe) and drains the native share queues.

Reference defect fixed: every device gets a disjoint slice of the search space
instead of the identical Work (engine/run.go:1294-1296).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field

from otedama_amd.hal import Family, SimpleDevice
from otedama_amd.ops.native import require_native


@dataclass
class DeviceMiner:
    device: SimpleDevice
    native: object
    stripe_index: int = 0
    paused: bool = False
    last_hashes: int = 0
    hashrate: float = 0.0
    extra: dict = field(default_factory=dict)

    @property
    def id(self) -> str:
        return self.device.identity().id


class MinerSet:
    def __init__(self, devices: list, algorithm: str = "sha256d", batch_nonces: int = 1 << 29,
                 cpu_threads: int = 0, rank: int = 0, world_size: int = 1, log=None, queue_cap: int = 4096):
        N = require_native()
        self.algorithm = algorithm
        self.log = log or (lambda level, msg: None)
        self.miners: list[DeviceMiner] = []
        gpus = [d for d in devices if d.identity().family == Family.GPU and d.index >= 0
                and d.capabilities().supports(algorithm)]
        for d in gpus:
            cus = int(d.extra.get("cus", 256))
            m = N.GpuMiner(d.index, d.identity().id, batch_nonces=batch_nonces, grid=cus * 6, queue_cap=queue_cap)
            self.miners.append(DeviceMiner(d, m))
        cpus = [d for d in devices if d.identity().family == Family.CPU]
        if cpus and algorithm == "sha256d" and (cpu_threads > 0 or not gpus):
            threads = cpu_threads or cpus[0].threads
            self.miners.append(DeviceMiner(cpus[0], N.CpuMiner(threads, cpus[0].identity().id, queue_cap)))
        # global stripe: device g of G across the node (ranks x local devices)
        local = len(self.miners)
        self.stripe_total = max(local, 1) * world_size
        for i, m in enumerate(self.miners):
            m.stripe_index = rank * max(local, 1) + i
        self._lock = threading.Lock()
        self._epoch = 0
        self._template: dict | None = None
        self._t_last = time.monotonic()

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
            self._template = dict(template) if template is not None else None
            for m in self.miners:
                self._apply(m)
            return self._epoch

    def _apply(self, m: DeviceMiner) -> None:
        if self._template is None or m.paused:
            m.native.set_job(None)
            return
        t = dict(self._template)
        t["epoch"] = self._epoch
        t["variant_start"] = m.stripe_index
        t["variant_stride"] = self.stripe_total
        m.native.set_job(t)

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

    def device_stats(self) -> dict[str, dict]:
        return {m.id: m.native.stats() for m in self.miners}

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
        for m in self.miners:
            h = m.native.stats()["hashes"]
            m.hashrate = max(h - m.last_hashes, 0) / dt
            m.last_hashes = h
            rates[m.id] = m.hashrate
        return rates

    def hashrate_of(self, device_id: str) -> float:
        for m in self.miners:
            if m.id == device_id:
                return m.hashrate
        return 0.0
