"""Multi-GPU node: one rank per MI355X, rank 0 talks to the pool, all ranks hash.

The reference's multi-device path is N goroutine workers fed the same Work through channels and a share fan-in
(internal/engine/setup.go:59-77, internal/engine/fanin.go:22-68). Here every GPU is its own process and the
fan-out / fan-in are RCCL collectives over xGMI, issued only when there is something to move:

  control plane (rendezvous TCPStore, no device work)     data plane (RCCL, bounded, per generation)
  ─────────────────────────────────────────────────────   ───────────────────────────────────────────
  otd/op/<k>     the leader's ordered op log              R1 broadcast job blob      on a new job / re-form
  otd/pending    shares waiting on followers (counter)    R2 all_gather share slots  when otd/pending > 0
  otd/hb/<r>     heartbeat: time, cursor, counters (2 Hz)  R3 all_gather counters     once per stats interval
  otd/dead/<r>   set by the supervisor when r exits
  otd/join/<r>   a replacement process asking to join

Every rank runs the ops of the log in order; a collective is entered only when the leader has posted it, so in
steady state a rank issues about one device collective per stats interval (10 s) plus one per share burst — not
hundreds per second. Hashing never waits on any of this: kernels run on the miners' HIP streams.

Rank loss (reference analogues: the partial-failure-tolerant detector
internal/hal/registry.go:138-201 and the failover loop internal/engine/run.go:368-521): the leader declares a
follower dead when the supervisor marks it, its heartbeat is older than HB_TIMEOUT, or a collective with it fails
or passes its deadline. It then posts a re-form: every survivor aborts the process group and forms the next
generation (store prefix otd-g<gen>) with the survivors, ranks renumbered, and the leader re-broadcasts the job
with a ``variant_base`` past every cursor the ranks reported, so the dead rank's residue class is searched by
the survivors from there on and nothing is searched twice. A replacement process (supervisor respawn) asks to
join and is added by the next re-form. Rank 0 is the pool session: its loss ends the node (the supervisor
restarts it). Over gloo (CPU hosts, tests) one limit remains: a rank blocked in a ring collective that the dead
rank's neighbours abandoned gives up after its bounded deadline, but tearing that group down waits out gloo's own
op timeout (OTEDAMA_PG_TIMEOUT), so that re-form can take that long; RCCL groups are aborted at once.

``NodeMinerSet`` (rank 0) has the MinerSet API the engine uses; ``NodeWorker`` (ranks > 0) follows the op log.
"""
from __future__ import annotations

import collections
import json
import os
import threading
import time

from otedama_amd.engine.miners import GROUP, RESPLIT_GROUPS, MinerSet
from otedama_amd.parallel.comm import SHARE_SLOTS, NodeComm
from otedama_amd.utils.trace import span

DEFAULT_TICK = 0.005       # leader control-loop period (store polls only; no device work)
HB_INTERVAL = 0.5          # heartbeat period
HB_TIMEOUT = 2.0           # a follower whose heartbeat is older is dead
LIVENESS_EVERY = 0.25      # leader liveness check period
STATS_INTERVAL = 10.0      # R3 cadence (the reference's stats tick, internal/engine/run.go:377-380)
OP_POLL_MAX = 0.004        # follower op-log poll interval ceiling
PREFIX = "otd/"


def _k(*parts) -> str:
    return PREFIX + "/".join(str(p) for p in parts)


def _store_get(store, key: str):
    try:
        if not store.check([key]):
            return None
        return store.get(key)
    except Exception:  # noqa: BLE001
        return None


class _Heartbeat:
    """Publishes this rank's liveness and cursor every HB_INTERVAL on a store connection of its own (the rank's
    op loop may sit in a bounded collective meanwhile)."""

    def __init__(self, store, orig_rank: int, local: MinerSet):
        self.store = store.clone() if hasattr(store, "clone") else store
        self.orig = orig_rank
        self.local = local
        self.stop = threading.Event()
        self.th = threading.Thread(target=self._loop, name=f"otedama-hb-{orig_rank}", daemon=True)

    def start(self):
        self.th.start()

    def payload(self) -> dict:
        st = list(self.local.device_stats().values())
        return {"t": time.time(), "hw": self.local.high_water(), "ep": self.local.epoch,
                "hashes": sum(s["hashes"] for s in st), "shares": sum(s["shares"] for s in st),
                "dropped": sum(s["dropped"] for s in st), "faulted": sum(1 for s in st if s["faulted"]),
                # device-timeline completion time of the counted hashes (one GPU per rank): exact rate windows
                "done": st[0].get("hashes_done_at_s", 0.0) if len(st) == 1 else 0.0,
                "pid": os.getpid()}

    def _loop(self):
        while not self.stop.is_set():
            try:
                self.store.set(_k("hb", self.orig), json.dumps(self.payload()))
            except Exception:  # noqa: BLE001 - store gone: the node is shutting down
                return
            self.stop.wait(HB_INTERVAL)


class _Link:
    """Op execution shared by leader and followers: one op = at most one collective, in log order."""

    def __init__(self, local: MinerSet, comm: NodeComm, log):
        self.local = local
        self.comm = comm
        self.log = log
        self.store = comm.info.store
        self.rows: list[list[int]] = [[0, 0, 0, 0] for _ in range(comm.info.world_size)]
        self.error: BaseException | None = None
        self.tick_seconds: collections.deque = collections.deque(maxlen=1024)  # per-op wall time
        self.ops_run = 0
        self.reforms = 0

    @property
    def rank(self) -> int:
        return self.comm.info.rank

    @property
    def world(self) -> int:
        return self.comm.info.world_size

    @property
    def tick(self) -> float:
        return DEFAULT_TICK

    def local_counters(self) -> list[int]:
        st = self.local.device_stats().values()
        return [sum(s["hashes"] for s in st), sum(s["shares"] for s in st), sum(s["dropped"] for s in st),
                sum(1 for s in st if s["faulted"])]

    def run_op(self, op: dict, blob, outgoing: list[dict]):
        """Execute one op; returns (job_blob | None, gathered shares | None)."""
        t0 = time.perf_counter()
        kind = op["op"]
        job, shares = None, None
        try:
            with span(f"otd.node.{kind}"):
                if kind == "job":
                    job = self.comm.broadcast_job(blob)                      # R1
                elif kind == "gather":
                    shares = self.comm.gather_shares(outgoing)               # R2
                elif kind == "stats":
                    self.rows = self.comm.gather_counters(self.local_counters())  # R3
                elif kind == "reform":
                    self.comm.reform(list(op["members"]), int(op["gen"]))
                    self.local.set_rank(self.comm.info.rank, self.comm.info.world_size)
                    self.rows = [[0, 0, 0, 0] for _ in range(self.comm.info.world_size)]
                    self.reforms += 1
        finally:
            self.tick_seconds.append(time.perf_counter() - t0)
            self.ops_run += 1
        return job, shares

    def tick_quantile(self, q: float) -> float:
        xs = sorted(self.tick_seconds)
        if not xs:
            return 0.0
        return xs[min(len(xs) - 1, int(q * len(xs)))]


class NodeMinerSet:
    """Rank-0 facade: local MinerSet + every other rank through the op log and collectives."""

    def __init__(self, local: MinerSet, comm: NodeComm, tick: float = DEFAULT_TICK, log=None,
                 stats_interval: float = STATS_INTERVAL, hb_timeout: float = HB_TIMEOUT):
        comm.bounded = True
        self.local = local
        self.comm = comm
        self.log = log or (lambda level, msg: None)
        self.link = _Link(local, comm, self.log)
        self.tick = tick
        self.stats_interval = stats_interval
        self.hb_timeout = hb_timeout
        self.algorithm = local.algorithm
        self.store = comm.info.store
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._seq = 0
        self._sent_seq = 0
        self._stop = False
        self._blob: dict | None = None
        self._template: dict | None = None
        self._epoch = 0
        self._variant_base = 0
        self._paused: set[str] = set()
        self._jobs: dict[int, dict] = {}          # epoch -> job meta for remote shares
        self._remote = collections.deque(maxlen=65536)
        self._remote_efd = os.eventfd(0, os.EFD_NONBLOCK | os.EFD_CLOEXEC)
        self._thread: threading.Thread | None = None
        self._op_k = 0
        self._gen = comm.info.generation
        self._gen_started = time.monotonic()
        self.capacity = comm.info.world_size       # orig ranks 0..capacity-1 may exist
        self._rows_by_orig: dict[int, list[int]] = {}
        self.row_times: dict[int, float] = {}  # wall time at which each remote rank's counter row was produced
        self.row_done_at: dict[int, float] = {}  # device-timeline time its counted hashes had completed
        self._prev_rows: dict[int, list[int]] = {}
        self._hb_pairs: dict[int, tuple[int, float]] = {}  # (hashes, device-timeline time they had completed) of
        # a rank's latest heartbeat: one consistent pair (R3 rows carry no completion time)
        self._prev_pairs: dict[int, tuple[int, float]] = {}
        self._exact: dict[int, bool] = {}  # the rank's last rate came from a device-timeline span
        self._rates: dict[str, float] = {}
        self._t_last = time.monotonic()
        self._remote_faults: dict[int, int] = {}
        self._remote_idle: dict[int, int] = {}
        self.lost_ranks: list[int] = []
        self._hb = _Heartbeat(self.store, comm.info.orig_rank, local) if self.store is not None else None

    # MinerSet API ------------------------------------------------------------
    @property
    def remote_ids(self) -> list[str]:
        return [f"rank{r}" for r in range(1, self.capacity)]

    def __len__(self) -> int:
        return len(self.local) * self.comm.info.world_size

    @property
    def miners(self):
        return self.local.miners

    @property
    def epoch(self) -> int:
        return self._epoch

    def start(self) -> None:
        self.local.start()
        if self._hb is not None:
            self._hb.start()
        if self.store is not None:
            self.store.set(_k("next"), "0")
        self._thread = threading.Thread(target=self._loop, name="otedama-node-r0", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        with self._lock:
            self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None
        if self._hb is not None:
            self._hb.stop.set()
        self.local.stop()

    def set_job(self, template: dict | None) -> int:
        with self._lock:
            self._template = dict(template) if template is not None else None
            if template is not None and self._variant_base:
                # new work: the re-split offset of the previous work is void
                from otedama_amd.engine.miners import _work_key

                if _work_key(template) != getattr(self, "_work_key", None):
                    self._variant_base = 0
            if template is not None:
                from otedama_amd.engine.miners import _work_key

                self._work_key = _work_key(template)
            ep = self.local.set_job(self._with_base(self._template))
            self._epoch = ep
            if template is not None:
                self._jobs[ep] = {"job_id": template.get("job_id", ""), "channel_id": template.get("channel_id", 0),
                                  "extranonce2_size": int(template.get("extranonce2_size", 0) or 0)}
                for old in [e for e in self._jobs if e < ep - 64]:
                    del self._jobs[old]
            self._publish()
        self._wake.set()
        return ep

    def _with_base(self, template: dict | None) -> dict | None:
        if template is None or not self._variant_base:
            return template
        return dict(template, variant_base=self._variant_base)

    def _publish(self) -> None:
        blob = None
        if self._template is not None:
            blob = {k: v for k, v in self._template.items() if k not in ("variant_start", "variant_stride")}
            blob["epoch"] = self._epoch
            if self._variant_base:
                blob["variant_base"] = self._variant_base
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
                self._publish()
            self._wake.set()
            return True
        return False

    def pause_all(self) -> None:
        self.set_job(None)

    def poll(self, max_per_device: int = 256) -> list[dict]:
        out = self.local.poll(max_per_device)
        n = max_per_device * max(self.capacity - 1, 1)
        while self._remote and n > 0:
            out.append(self._remote.popleft())
            n -= 1
        return out

    def share_fds(self) -> list[int]:
        return list(self.local.share_fds()) + [self._remote_efd]

    def device_stats(self) -> dict[str, dict]:
        d = dict(self.local.device_stats())
        for r in range(1, self.capacity):
            row = self._rows_by_orig.get(r, [0, 0, 0, 0])
            lost = r in self.lost_ranks
            d[f"rank{r}"] = {"hashes": row[0], "shares": row[1], "dropped": row[2], "faulted": bool(row[3]) or lost,
                             "error": "rank lost" if lost else ("remote device fault" if row[3] else ""),
                             "candidates": 0, "launches": 0, "counted_at": self.row_times.get(r, 0.0),
                             "hashes_done_at_s": self.row_done_at.get(r, 0.0)}
        return d

    def total_hashes(self) -> int:
        return self.local.total_hashes() + sum(r[0] for o, r in self._rows_by_orig.items() if o != 0)

    def total_dropped(self) -> int:
        return self.local.total_dropped() + sum(r[2] for o, r in self._rows_by_orig.items() if o != 0)

    def faulted(self) -> list[tuple[str, str]]:
        out = self.local.faulted()
        for r in range(1, self.capacity):
            if r in self.lost_ranks:
                out.append((f"rank{r}", "rank lost"))
            elif self._rows_by_orig.get(r, [0, 0, 0, 0])[3]:
                out.append((f"rank{r}", "remote device fault"))
        return out

    def retire_faulted(self) -> list[tuple[str, str]]:
        """Local faults are retired here; a remote rank retires its own devices (NodeWorker) and re-splits its
        class; lost ranks are reported once."""
        out = self.local.retire_faulted()
        for r in range(1, self.capacity):
            n = self._rows_by_orig.get(r, [0, 0, 0, 0])[3]
            if n > self._remote_faults.get(r, 0):
                out.append((f"rank{r}", f"{n - self._remote_faults.get(r, 0)} device(s) faulted on rank{r}"))
                self._remote_faults[r] = n
        return out

    def stalled(self) -> list[str]:
        stall = self.local.stall_samples
        return self.local.stalled() + [f"rank{r}" for r, n in self._remote_idle.items() if n >= stall]

    def live(self):
        return self.local.live()

    def update_hashrates(self) -> dict[str, float]:
        rates = self.local.update_hashrates()
        now = time.monotonic()
        dt = max(now - self._t_last, 1e-6)
        self._t_last = now
        working = self._blob is not None and self._blob.get("job") is not None
        members = set(self.comm.info.members)
        for r in range(1, self.capacity):
            row, prev = self._rows_by_orig.get(r, [0, 0, 0, 0]), self._prev_rows.get(r, [0, 0, 0, 0])
            rid = f"rank{r}"
            # as MinerSet.update_hashrates: between two counted completions on the rank's own device timeline the
            # rate is exact; a wall-clock sample of launch-sized counter steps jitters by a launch per interval
            (h, done), (ph, pdone) = self._hb_pairs.get(r, (0, 0.0)), self._prev_pairs.get(r, (0, 0.0))
            self._exact[r] = done > 0 and pdone > 0 and done > pdone and h > ph
            rates[rid] = (h - ph) / (done - pdone) if self._exact[r] else max(row[0] - prev[0], 0) / dt
            if r in self._hb_pairs:
                self._prev_pairs[r] = self._hb_pairs[r]
            idle = working and r in members and rid not in self._paused and row[0] == prev[0]
            self._remote_idle[r] = self._remote_idle.get(r, 0) + 1 if idle else 0
            self._prev_rows[r] = list(row)
        self._rates = rates
        return rates

    def exact_total(self) -> float | None:
        """Node total from device-timeline rates when the local miners and every member rank have one (see
        MinerSet.exact_total), else None."""
        local = self.local.exact_total()
        members = set(self.comm.info.members)
        remote = [r for r in range(1, self.capacity) if r in members]
        if local is None or not all(self._exact.get(r, False) for r in remote):
            return None
        return local + sum(self._rates.get(f"rank{r}", 0.0) for r in remote)

    def hashrate_of(self, device_id: str) -> float:
        return self._rates.get(device_id, self.local.hashrate_of(device_id))

    # leader loop --------------------------------------------------------------
    def _post(self, op: dict) -> None:
        op["gen"] = op.get("gen", self._gen)
        self.store.set(_k("op", self._op_k), json.dumps(op))
        self._op_k += 1
        self.store.set(_k("next"), str(self._op_k))

    def _heartbeats(self) -> dict[int, dict]:
        keys = [_k("hb", r) for r in range(1, self.capacity)]
        out = {}
        for r, key in zip(range(1, self.capacity), keys):
            raw = _store_get(self.store, key)
            if raw is not None:
                try:
                    out[r] = json.loads(raw)
                except ValueError:
                    pass
        return out

    def _dead_and_joiners(self) -> tuple[list[int], list[int]]:
        now = time.time()
        hbs = self._heartbeats()
        members = self.comm.info.members
        for r, hb in hbs.items():  # per-rank counters between R3 rounds (store only, no device collective)
            if r in members and now - hb["t"] <= self.hb_timeout:
                self._rows_by_orig[r] = [int(hb.get("hashes", 0)), int(hb.get("shares", 0)),
                                         int(hb.get("dropped", 0)), int(hb.get("faulted", 0))]
                self.row_times[r] = float(hb["t"])
                self.row_done_at[r] = float(hb.get("done", 0.0) or 0.0)
                self._hb_pairs[r] = (int(hb.get("hashes", 0)), self.row_done_at[r])
        dead = []
        grace = time.monotonic() - self._gen_started < self.hb_timeout  # members of a new generation get one
        for r in members[1:]:                                           # timeout to (re)start heartbeating
            hb = hbs.get(r)
            marked = _store_get(self.store, _k("dead", r)) is not None
            stale = (hb is None and not grace) or (hb is not None and now - hb["t"] > self.hb_timeout)
            if marked or stale:
                dead.append(r)
        joiners = []
        for r in range(1, self.capacity):
            if r in members:
                continue
            hb = hbs.get(r)
            if _store_get(self.store, _k("join", r)) is not None and hb is not None and now - hb["t"] <= self.hb_timeout:
                joiners.append(r)
        return dead, joiners

    def _reform(self, dead: list[int], joiners: list[int], why: str) -> None:
        info = self.comm.info
        old_world = info.world_size
        members = [r for r in info.members if r not in dead] + sorted(joiners)
        members = [0] + sorted(r for r in members if r != 0)
        # every cursor of the current work: the survivors' heartbeats and this rank's own devices
        hw = self.local.high_water()
        for r, hb in self._heartbeats().items():
            if hb.get("ep", 0) >= self.local._work_epoch0 > 0:
                hw = max(hw, int(hb.get("hw", 0)))
        local_devs = max(len(self.local.miners), 1)
        base = hw + RESPLIT_GROUPS * GROUP * old_world * local_devs
        self._gen += 1
        self._gen_started = time.monotonic()
        with span("otd.node.reform"):
            self._post({"op": "reform", "gen": self._gen, "members": members})
            self.link.run_op({"op": "reform", "members": members, "gen": self._gen}, None, [])
        for r in dead:
            if r not in self.lost_ranks:
                self.lost_ranks.append(r)
            self._rows_by_orig.pop(r, None)
            try:
                self.store.delete_key(_k("dead", r))
            except Exception:  # noqa: BLE001
                pass
        for r in joiners:
            if r in self.lost_ranks:
                self.lost_ranks.remove(r)
            try:
                self.store.delete_key(_k("join", r))
            except Exception:  # noqa: BLE001
                pass
        with self._lock:
            if self._template is not None:
                self._variant_base = base
                self._epoch = self.local.set_job(self._with_base(self._template))
                self._jobs[self._epoch] = self._jobs.get(self._epoch) or {
                    "job_id": self._template.get("job_id", ""), "channel_id": self._template.get("channel_id", 0),
                    "extranonce2_size": int(self._template.get("extranonce2_size", 0) or 0)}
            self._publish()
        self.log("warn", f"node: {why}; generation {self._gen}: ranks {members} (world {len(members)}), "
                         f"variants re-split from {base}")

    def _try_reform(self, dead: list[int], joiners: list[int], why: str) -> None:
        try:
            self._reform(dead, joiners, why)
        except Exception as exc:  # noqa: BLE001 - e.g. a member died during the re-form: the next check retries
            self.log("error", f"node: re-form failed ({type(exc).__name__}: {exc}); retrying")
            self.comm.abort()
        self._sent_seq = -1  # (re-)broadcast the job on the new generation

    def _loop(self) -> None:
        info = self.comm.info
        if info.device.type == "cuda":
            import torch

            torch.cuda.set_device(info.device)
        next_live = next_stats = time.monotonic()
        try:
            while True:
                with self._lock:
                    stop = self._stop
                    seq, blob = self._seq, self._blob
                if stop:
                    if self.store is not None and info.world_size > 1:
                        self._post({"op": "stop"})
                    return
                now = time.monotonic()
                try:
                    if now >= next_live and self.store is not None:
                        next_live = now + LIVENESS_EVERY
                        dead, joiners = self._dead_and_joiners()
                        if dead or joiners:
                            why = ", ".join([f"rank {r} lost" for r in dead] + [f"rank {r} joins" for r in joiners])
                            self._try_reform(dead, joiners, why)
                            continue
                    if info.world_size > 1 and seq != self._sent_seq:
                        self._post({"op": "job"})
                        self.link.run_op({"op": "job"}, blob, [])
                        self._sent_seq = seq
                    if info.world_size > 1 and int(self.store.add(_k("pending"), 0)) > 0:
                        self._post({"op": "gather"})
                        _, shares = self.link.run_op({"op": "gather"}, None, [])
                        self._take(shares or [])
                    if now >= next_stats:
                        next_stats = now + self.stats_interval
                        if info.world_size > 1:
                            self._post({"op": "stats"})
                        self.link.run_op({"op": "stats"}, None, [])
                        for gi, row in enumerate(self.link.rows):
                            if gi < len(info.members):
                                self._rows_by_orig[info.members[gi]] = list(row)
                except Exception as exc:  # noqa: BLE001 - a collective failed: find who is gone and re-form
                    if self.store is not None and _store_get(self.store, _k("stopping")) is not None:
                        # the supervisor is stopping every rank (SIGTERM): a follower that left first is no loss
                        self.log("info", "node: stopping (the supervisor is shutting the node down)")
                        return
                    self.log("warn", f"node: collective failed ({type(exc).__name__}: {exc}); checking ranks")
                    self.link.error = exc
                    # the peer that broke it shows up as dead within one heartbeat timeout (its process exited, or
                    # it stopped heartbeating); re-form without it, or with everyone if it was transient
                    end = time.monotonic() + self.hb_timeout + 1.0
                    dead, joiners = self._dead_and_joiners()
                    while not dead and time.monotonic() < end:
                        time.sleep(0.1)
                        dead, joiners = self._dead_and_joiners()
                    self._try_reform(dead, joiners, "collective failure" + (f", ranks {dead} lost" if dead else ""))
                    continue
                self._wake.wait(self.tick)
                self._wake.clear()
        except BaseException as exc:  # noqa: BLE001
            self.link.error = exc
            self.log("error", f"node: control loop failed: {exc}")

    def _take(self, shares: list[dict]) -> None:
        n = 0
        for s in shares:
            if s["orig_rank"] == self.comm.info.orig_rank:
                continue
            n += 1
            meta = self._jobs.get(s["epoch"])
            if meta is None:
                continue  # job older than the retained window: stale
            s.update(meta)
            s["device_id"] = f"rank{s['orig_rank']}"
            self._remote.append(s)
        if n:
            self.store.add(_k("pending"), -n)
            os.eventfd_write(self._remote_efd, 1)


class NodeWorker:
    """Ranks > 0: follow the leader's op log (jobs, share gathers, counters, re-forms) until told to stop."""

    def __init__(self, local: MinerSet, comm: NodeComm, tick: float = DEFAULT_TICK, log=None, joining: bool = False):
        comm.bounded = True
        self.local = local
        self.comm = comm
        self.link = _Link(local, comm, log or (lambda level, msg: None))
        self.log = self.link.log
        self.rank_id = f"rank{comm.info.orig_rank}"
        self.store = comm.info.store
        self.joining = joining
        self._hb = _Heartbeat(self.store, comm.info.orig_rank, local)
        self._pending: list[dict] = []
        self._plock = threading.Lock()
        self._stop = threading.Event()

    def _share_loop(self) -> None:
        """Wake on the local miners' share eventfds and announce new shares to the leader at once (otd/pending);
        they travel with the next R2 gather the leader posts."""
        import select

        store = self.store.clone() if hasattr(self.store, "clone") else self.store
        fds = list(self.local.share_fds())
        while not self._stop.is_set():
            if fds:
                ready, _, _ = select.select(fds, [], [], 0.25)
                for fd in ready:
                    try:
                        os.read(fd, 8)
                    except BlockingIOError:
                        pass
            else:
                self._stop.wait(0.01)
            new = self.local.poll(256)
            if new:
                with self._plock:
                    self._pending.extend(new)
                try:
                    store.add(_k("pending"), len(new))
                except Exception:  # noqa: BLE001 - store gone: shutting down
                    return

    def run(self) -> None:
        self.local.start()
        self._hb.start()
        share_th = threading.Thread(target=self._share_loop, name=f"otedama-node-shares-{self.rank_id}", daemon=True)
        share_th.start()
        info = self.comm.info
        k = 0
        if self.joining:
            raw = _store_get(self.store, _k("next"))
            k = int(raw) if raw is not None else 0
            self.store.set(_k("join", info.orig_rank), "1")
        broken = False  # the current group failed a collective: skip collectives until the next re-form
        try:
            idle = 0.0
            while True:
                key = _k("op", k)
                # poll, backing off from 0.5 ms to OP_POLL_MAX while the log is quiet (store.wait would log a c10d
                # warning on every timeout); an op is picked up within OP_POLL_MAX
                if not self.store.check([key]):
                    idle = min(OP_POLL_MAX, idle * 2 if idle else 0.0005)
                    time.sleep(idle)
                    continue
                idle = 0.0
                op = json.loads(self.store.get(key))
                k += 1
                kind = op["op"]
                if kind == "stop":
                    return
                if kind == "reform":
                    if info.orig_rank in op["members"]:
                        try:
                            self.link.run_op(op, None, [])
                            broken = False
                            self.log("info", f"node: {self.rank_id} is rank {info.rank}/{info.world_size} of "
                                             f"generation {info.generation}")
                        except Exception as exc:  # noqa: BLE001
                            self.log("error", f"node: re-form failed: {exc}")
                            broken = True
                    else:
                        broken = True  # excluded: wait to be re-admitted (join) by a later re-form
                        self.store.set(_k("join", info.orig_rank), "1")
                    continue
                if info.generation < 0 or broken or op.get("gen") != info.generation:
                    continue  # not (yet) a member of the generation this op belongs to
                try:
                    if kind == "job":
                        blob, _ = self.link.run_op(op, None, [])
                        if blob is not None:
                            self._apply(blob)
                    elif kind == "gather":
                        with self._plock:
                            out, self._pending = self._pending[:SHARE_SLOTS], self._pending[SHARE_SLOTS:]
                        try:
                            self.link.run_op(op, None, out)
                        except Exception:
                            with self._plock:  # not delivered: keep them for the next gather
                                self._pending[:0] = out
                            raise
                    elif kind == "stats":
                        self.link.run_op(op, None, [])
                        self.local.retire_faulted()  # survivors re-split this rank's class at once
                except Exception as exc:  # noqa: BLE001 - leave this group; the leader re-forms
                    self.log("warn", f"node: {self.rank_id}: collective failed ({type(exc).__name__}: {exc})")
                    self.comm.abort()
                    broken = True
        finally:
            self._stop.set()
            self._hb.stop.set()
            share_th.join(timeout=5)
            self.local.stop()

    def _apply(self, blob: dict) -> None:
        job = blob.get("job")
        paused = self.rank_id in set(blob.get("paused", []))
        if job is None or paused:
            self.local.set_job(None)
            return
        self.local.set_job(job, epoch=int(job["epoch"]))
