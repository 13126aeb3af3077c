"""Multi-GPU node: one rank per MI355X, rank 0 talks to the pool, all ranks hash.

The reference's multi-device path is N goroutine workers fed the same Work
through channels and a share fan-in (internal/engine/setup.go:59-77,
internal/engine/fanin.go:22-68). Here every GPU is its own process
(torchrun, RCCL over xGMI) and the fan-out / fan-in are collectives run in
lockstep by a tick thread on every rank:

  tick:  R1a broadcast control word  [seq, stop, epoch, 0]       32 B
         R1b broadcast job blob       only when seq changed       ≤ 4 KiB
         R2  all_gather share slots   64 × 9 int64 per rank       4.6 KiB/rank
         R3  all_gather counters      [hashes, shares, dropped, faulted]

Each rank's native miners search the disjoint variant stripes
``rank + world*i (mod world*live)`` (parallel/partition.py), so nothing but
jobs, hits and counters ever crosses xGMI. The tick (default 10 ms) bounds the
extra share latency of non-primary ranks; hashing never waits on it because
kernels run on the miners' own HIP streams and the collectives on NodeComm's
comm stream.

``NodeMinerSet`` (rank 0) has the MinerSet API the engine uses; ``NodeWorker``
(ranks > 0) just follows the broadcast jobs.
"""
from __future__ import annotations

import collections
import threading
import time

from otedama_amd.engine.miners import MinerSet
from otedama_amd.parallel.comm import NodeComm
from otedama_amd.utils.trace import span

DEFAULT_TICK = 0.010


class _Link:
    """Lockstep tick shared by rank 0 and workers."""

    def __init__(self, local: MinerSet, comm: NodeComm, tick: float):
        self.local = local
        self.comm = comm
        self.tick = tick
        self.rank = comm.info.rank
        self.world = comm.info.world_size
        self.rows: list[list[int]] = [[0, 0, 0, 0] for _ in range(self.world)]
        self.last_tick_seconds = 0.0  # wall time of the last R1/R2/R3 round (otedama_node_collective_seconds)
        self._seen_seq = 0
        self.error: BaseException | None = None

    def local_counters(self) -> list[int]:
        st = self.local.device_stats().values()
        return [sum(s["hashes"] for s in st), sum(s["shares"] for s in st), sum(s["dropped"] for s in st),
                sum(1 for s in st if s["faulted"])]

    def step(self, ctl_words: list[int] | None, job: dict | None, outgoing: list[dict]) -> tuple:
        """One tick; returns (stop, job_or_None_if_unchanged, changed, gathered_shares)."""
        t0 = time.perf_counter()
        with span("otd.node.tick"):
            with span("otd.node.R1_control"):
                ctl = self.comm.broadcast_control(ctl_words or [0, 0, 0, 0])
            seq, stop = ctl[0], ctl[1]
            changed, new_job = False, None
            if seq != self._seen_seq:
                with span("otd.node.R1_job"):
                    new_job = self.comm.broadcast_job(job)
                self._seen_seq = seq
                changed = True
            with span("otd.node.R2_shares"):
                shares = self.comm.gather_shares(outgoing)
            with span("otd.node.R3_counters"):
                self.rows = self.comm.gather_counters(self.local_counters())
        self.last_tick_seconds = time.perf_counter() - t0
        return bool(stop), new_job, changed, shares


class NodeMinerSet:
    """Rank-0 facade: local MinerSet + every other rank through collectives."""

    def __init__(self, local: MinerSet, comm: NodeComm, tick: float = DEFAULT_TICK, log=None):
        self.local = local
        self.comm = comm
        self.link = _Link(local, comm, tick)
        self.log = log or (lambda level, msg: None)
        self.algorithm = local.algorithm
        self._lock = threading.Lock()
        self._seq = 0
        self._stop = False
        self._blob: dict | None = None
        self._paused: set[str] = set()
        self._jobs: dict[int, dict] = {}          # epoch -> job meta for remote shares
        self._remote = collections.deque(maxlen=65536)
        self._thread: threading.Thread | None = None
        self._last_rows = [[0, 0, 0, 0] for _ in range(comm.info.world_size)]
        self._rates: dict[str, float] = {}
        self._t_last = time.monotonic()
        self.remote_ids = [f"rank{r}" for r in range(1, comm.info.world_size)]
        self._remote_faults = [0] * comm.info.world_size   # faulted-device count already reported
        self._remote_idle = [0] * comm.info.world_size     # ticks without hash progress

    # MinerSet API ------------------------------------------------------------
    def __len__(self) -> int:
        return len(self.local) * self.comm.info.world_size

    @property
    def miners(self):
        return self.local.miners

    @property
    def epoch(self) -> int:
        return self.local.epoch

    def start(self) -> None:
        self.local.start()
        self._thread = threading.Thread(target=self._loop, name="otedama-node-r0", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        with self._lock:
            self._stop = True
            self._seq += 1
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None
        self.local.stop()

    def set_job(self, template: dict | None) -> int:
        with self._lock:
            ep = self.local.set_job(template)
            if template is not None:
                self._jobs[ep] = {"job_id": template.get("job_id", ""), "channel_id": template.get("channel_id", 0),
                                  "extranonce2_size": int(template.get("extranonce2_size", 0) or 0)}
                for old in [e for e in self._jobs if e < ep - 64]:
                    del self._jobs[old]
            self._publish(template, ep)
            return ep

    def _publish(self, template: dict | None, epoch: int) -> None:
        blob = None
        if template is not None:
            blob = {k: v for k, v in template.items() if k not in ("variant_start", "variant_stride")}
            blob["epoch"] = epoch
        self._blob = {"job": blob, "paused": sorted(self._paused)}
        self._seq += 1

    def pause_device(self, device_id: str, paused: bool = True) -> bool:
        if self.local.pause_device(device_id, paused):
            return True
        if device_id in self.remote_ids:
            with self._lock:
                if paused:
                    self._paused.add(device_id)
                else:
                    self._paused.discard(device_id)
                self._blob = dict(self._blob or {"job": None}, paused=sorted(self._paused))
                self._seq += 1
            return True
        return False

    def pause_all(self) -> None:
        self.set_job(None)

    def poll(self, max_per_device: int = 256) -> list[dict]:
        out = self.local.poll(max_per_device)
        n = max_per_device * max(len(self.remote_ids), 1)
        while self._remote and n > 0:
            out.append(self._remote.popleft())
            n -= 1
        return out

    def device_stats(self) -> dict[str, dict]:
        d = dict(self.local.device_stats())
        for r, rid in enumerate(self.remote_ids, start=1):
            row = self._last_rows[r]
            d[rid] = {"hashes": row[0], "shares": row[1], "dropped": row[2], "faulted": bool(row[3]),
                      "error": "remote device fault" if row[3] else "", "candidates": 0, "launches": 0}
        return d

    def total_hashes(self) -> int:
        return self.local.total_hashes() + sum(r[0] for r in self._last_rows[1:])

    def total_dropped(self) -> int:
        return self.local.total_dropped() + sum(r[2] for r in self._last_rows[1:])

    def faulted(self) -> list[tuple[str, str]]:
        out = self.local.faulted()
        out += [(rid, "remote device fault") for r, rid in enumerate(self.remote_ids, start=1)
                if self._last_rows[r][3]]
        return out

    def retire_faulted(self) -> list[tuple[str, str]]:
        """Local faults are retired here; a remote rank retires its own devices (NodeWorker) and
        re-splits its variant class, so rank 0 only reports the new fault count once."""
        out = self.local.retire_faulted()
        for r, rid in enumerate(self.remote_ids, start=1):
            n = self._last_rows[r][3]
            if n > self._remote_faults[r]:
                out.append((rid, f"{n - self._remote_faults[r]} device(s) faulted on {rid}"))
                self._remote_faults[r] = n
        return out

    def stalled(self) -> list[str]:
        stall = self.local.stall_samples
        return self.local.stalled() + [rid for r, rid in enumerate(self.remote_ids, start=1)
                                       if self._remote_idle[r] >= stall]

    def live(self):
        return self.local.live()

    def update_hashrates(self) -> dict[str, float]:
        rates = self.local.update_hashrates()
        now = time.monotonic()
        dt = max(now - self._t_last, 1e-6)
        self._t_last = now
        prev = getattr(self, "_prev_rows", None) or [[0, 0, 0, 0] for _ in self._last_rows]
        working = self._blob is not None and self._blob.get("job") is not None
        for r, rid in enumerate(self.remote_ids, start=1):
            rates[rid] = max(self._last_rows[r][0] - prev[r][0], 0) / dt
            idle = working and rid not in self._paused and self._last_rows[r][0] == prev[r][0]
            self._remote_idle[r] = self._remote_idle[r] + 1 if idle else 0
        self._prev_rows = [list(x) for x in self._last_rows]
        self._rates = rates
        return rates

    def hashrate_of(self, device_id: str) -> float:
        return self._rates.get(device_id, self.local.hashrate_of(device_id))

    # tick thread --------------------------------------------------------------
    def _loop(self) -> None:
        info = self.comm.info
        if info.device.type == "cuda":
            import torch

            torch.cuda.set_device(info.device)
        try:
            while True:
                with self._lock:
                    ctl = [self._seq, int(self._stop), self.local.epoch, 0]
                    blob = self._blob
                stop, _, _, shares = self.link.step(ctl, blob, [])
                self._last_rows = self.link.rows
                for s in shares:
                    if s["rank"] == 0:
                        continue
                    meta = self._jobs.get(s["epoch"])
                    if meta is None:
                        continue  # job older than the retained window: stale
                    s.update(meta)
                    s["device_id"] = f"rank{s['rank']}"
                    self._remote.append(s)
                if stop:
                    return
                time.sleep(self.link.tick)
        except BaseException as exc:  # noqa: BLE001
            self.link.error = exc
            self.log("error", f"node: collective loop failed: {exc}")


class NodeWorker:
    """Ranks > 0: follow rank 0's jobs, return hits and counters, until told to stop."""

    def __init__(self, local: MinerSet, comm: NodeComm, tick: float = DEFAULT_TICK, log=None):
        self.local = local
        self.comm = comm
        self.link = _Link(local, comm, tick)
        self.log = log or (lambda level, msg: None)
        self.rank_id = f"rank{comm.info.rank}"
        self.health_every = max(1, int(1.0 / max(tick, 1e-3)))  # fault check about once a second

    def run(self) -> None:
        self.local.start()
        try:
            pending: list[dict] = []
            n = 0
            while True:
                pending.extend(self.local.poll(256))
                out, pending = pending[:64], pending[64:]
                stop, blob, changed, _ = self.link.step(None, None, out)
                if changed and blob is not None:
                    self._apply(blob)
                if stop:
                    return
                n += 1
                if n % self.health_every == 0:
                    self.local.retire_faulted()  # survivors re-split this rank's class on the next job
                time.sleep(self.link.tick)
        finally:
            self.local.stop()

    def _apply(self, blob: dict) -> None:
        job = blob.get("job")
        paused = self.rank_id in set(blob.get("paused", []))
        if job is None or paused:
            self.local.set_job(None)
            return
        self.local.set_job(job, epoch=int(job["epoch"]))
