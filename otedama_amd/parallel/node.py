"""Multi-GPU node: one rank per MI355X, rank 0 talks to the pool, all ranks hash.

The reference's multi-device path is N goroutine workers fed the same Work through channels and a share fan-in
(internal/engine/setup.go:59-77, internal/engine/fanin.go:22-68). Here every GPU is its own process and the
fan-out / fan-in are RCCL collectives over xGMI, issued only when there is something to move:

  control plane (rendezvous TCPStore, no device work)     data plane (RCCL, bounded, per generation)
  ─────────────────────────────────────────────────────   ───────────────────────────────────────────
  otd/op/<k>     the leader's ordered op log              R1 broadcast job blob      on a new job / re-form
  otd/next       ops posted so far                        R2 all_gather share slots  when a follower rings
  otd/hb/<r>     heartbeat: time, cursor, counters (2 Hz)  R3 all_gather counters     once per stats interval
  otd/bell/<r>   the rank's doorbell port (loopback UDP)
  otd/gen        the current process-group generation
  otd/dead/<r>   set by the supervisor when r exits
  otd/join/<r>   a replacement process asking to join

Every rank runs the ops of the log in order; a collective is entered only when the leader has posted it, so in
steady state a rank issues about one device collective per stats interval (10 s) plus one per share burst — not
hundreds per second. Hashing never waits on any of this: kernels run in each rank's device process (engine/devproc.py),
so a GPU fault kills that child, not the rank that holds the RCCL communicator and, on rank 0, the pool session.

Nothing on the share path sleeps on a timer: a follower whose device process pushed a share rings the leader's
doorbell, the leader logs the R2 gather op in the store and rings every follower's doorbell with the op itself, and
the followers enter the gather at once (a doorbell is a loopback datagram; the op travels inline, so no store round
trip sits between a follower's wake-up and the collective; the store stays the source of truth, so a lost datagram
costs one fallback poll, <= 50 ms; a lost share ring is covered by the pending count in the follower's heartbeat). Share records carry the kernel's own hit time, so the leader records device hit ->
pool accept for remote ranks' shares the same way as for its own.

Share previews: the R2 gather is a device collective, and on a GPU that the sibling device process saturates it waits
for a wave slot (~1 ms p50 under SHA-256d, up to ~15 ms p99 under scrypt, profiles/r5/e_reserve_cus). A follower
therefore also sends each new share record to the leader's preview port (otd/spv, a loopback datagram read by a
thread of its own), and the leader submits it on arrival. R2 stays the consistent delivery: every share still
travels in a gather (a lost datagram, a restarted leader), and the leader admits each share once, whichever path
brings it first (key: rank, epoch, nonce, ntime, version, extranonce2).

Rank loss (reference analogues: the partial-failure-tolerant detector
internal/hal/registry.go:138-201 and the failover loop internal/engine/run.go:368-521): the leader declares a
follower dead when the supervisor marks it, its heartbeat is older than HB_TIMEOUT, or a collective with it fails
or passes its deadline. It then posts a re-form: every survivor aborts the process group and forms the next
generation (store prefix otd-g<gen>) with the survivors, ranks renumbered, and the leader re-broadcasts the job
with a ``variant_base`` past every cursor the ranks reported, so the dead rank's residue class is searched by
the survivors from there on and nothing is searched twice. A replacement process (supervisor respawn) asks to
join and is added by the next re-form.

Leader loss: rank 0 holds the pool session; when it dies the supervisor restarts it after a backoff. Meanwhile the
followers keep hashing their last job (their collectives with the dead leader fail at their deadline and they wait
for a re-form). The restarted leader resumes the op log after the last op its predecessor posted, forms the next
generation from every follower that is still heartbeating, reconnects to the pool and broadcasts the new work. Its
job epochs live in a namespace of their own (incarnation << 40), so a follower's share of the old leader's job can
never be mapped onto a new job: it is dropped as stale. Over gloo (CPU hosts, tests) one limit remains: a rank blocked in a ring collective that the dead
rank's neighbours abandoned gives up after its bounded deadline, but tearing that group down waits out gloo's own
op timeout (OTEDAMA_PG_TIMEOUT), so that re-form can take that long; RCCL groups are aborted at once.

``NodeMinerSet`` (rank 0) has the MinerSet API the engine uses; ``NodeWorker`` (ranks > 0) follows the op log.
"""
from __future__ import annotations

import collections
import json
import os
import random
import select
import socket
import threading
import time

from otedama_amd.engine.miners import GROUP, RESPLIT_GROUPS, MinerSet
from otedama_amd.parallel.commbase import SHARE_SLOTS, SHARE_WORDS, pack_shares, unpack_shares
from otedama_amd.utils.trace import span

DEFAULT_TICK = 0.005       # reported control-loop granularity (the loop itself waits on its doorbell)
HB_INTERVAL = 0.5          # heartbeat period
HB_TIMEOUT = 2.0           # a follower whose heartbeat is older is dead
LIVENESS_EVERY = 0.25      # leader liveness check period
STATS_INTERVAL = 10.0      # R3 cadence (the reference's stats tick, internal/engine/run.go:377-380)
BELL_FALLBACK = 0.05       # doorbell wait ceiling: a lost datagram delays an op or a gather by at most this
PREVIEW_GRACE = 0.02       # a follower rings for the R2 of previewed shares this long after the first preview
PENDING_CAP = 8192         # shares a follower holds for the leader (drop-oldest past it, counted)
OP_RETAIN = 4096           # op log entries kept in the store (~1 h at the quiet node's ~1 op/s); older ones deleted
EPOCH_SHIFT = 40           # leader incarnation i numbers its job epochs from (i - 1) << EPOCH_SHIFT
PREFIX = "otd/"
PREVIEW_MAX = 60000        # largest job-preview datagram (loopback UDP allows 65507 bytes); bigger jobs go by R1 only
SEEN_MAX = 65536           # share keys the leader remembers to admit each share once (preview and R2 both carry it)
SEEN_TTL = 120.0           # ... for this long: R2 follows a preview within ~20 ms, or after a re-form within seconds


def share_preview_msgs(shares: list[dict], orig_rank: int) -> list[bytes]:
    """Share-preview datagrams: b"p" + the sender's orig rank (2 bytes) + up to SHARE_SLOTS R2 records each."""
    out = []
    for i in range(0, len(shares), SHARE_SLOTS):
        part = shares[i:i + SHARE_SLOTS]
        rows = pack_shares(part, orig_rank)[: len(part)]
        out.append(b"p" + orig_rank.to_bytes(2, "little") + rows.tobytes())
    return out


def parse_share_preview(msg: bytes) -> list[dict]:
    """The share records of a preview datagram (orig_rank set from its header); [] for anything malformed."""
    body = msg[3:]
    if msg[:1] != b"p" or not body or len(body) % (8 * SHARE_WORDS):
        return []
    import numpy as np

    orig = int.from_bytes(msg[1:3], "little")
    rows = np.frombuffer(body, dtype=np.int64).reshape(1, -1, SHARE_WORDS)
    return unpack_shares(rows, [orig])


def share_key(s: dict) -> int:
    """A share's identity for the leader's admit-once check, as one 64-bit hash (a tuple of six ints per remembered
    share was ~320 B of the leader's heap; tracemalloc, profiles/r5/n_rss)."""
    return hash((s["orig_rank"], s["epoch"], s["nonce"], s.get("ntime", 0), s.get("version", 0),
                 s.get("extranonce2", 0)))


def op_retain() -> int:
    """Op log entries the leader keeps (OTEDAMA_NODE_OP_RETAIN, tests shrink it). The store lives in the supervisor
    for the node's lifetime, so an untrimmed log would grow by one entry per job, gather and stats op, for weeks."""
    try:
        return max(16, int(os.environ.get("OTEDAMA_NODE_OP_RETAIN", OP_RETAIN)))
    except ValueError:
        return OP_RETAIN


def _k(*parts) -> str:
    return PREFIX + "/".join(str(p) for p in parts)


def _store_get(store, key: str, timeout: float | None = None):
    """The key's value, or None when it is absent or the store failed. ``timeout`` bounds the get itself: a key
    deleted between the check and the get (the leader trimming the op log) would otherwise block the caller for the
    store's whole timeout."""
    try:
        if not store.check([key]):
            return None
        if timeout is None or not hasattr(store, "set_timeout"):
            return store.get(key)
        import datetime

        prev = getattr(store, "timeout", None)
        store.set_timeout(datetime.timedelta(seconds=timeout))
        try:
            return store.get(key)
        finally:
            if prev is not None:
                store.set_timeout(prev)
    except Exception:  # noqa: BLE001
        return None


def _clone(store):
    return store.clone() if hasattr(store, "clone") else store


class _Bell:
    """A rank's doorbell: a loopback UDP socket whose port is published at otd/bell/<orig>. ``ring(r, msg)`` sends
    one datagram to rank r (ports are looked up in the store and cached for a couple of seconds: a restarted rank has
    a new one): b"s" (a follower has shares), b"o" (look at the op log), or b"o" + an op inline (``op_msg``).
    ``wait(t)`` blocks until a datagram arrives or t passes and returns the datagrams received."""

    PORT_TTL = 2.0
    # Fault injection (tests): this fraction of datagrams is dropped, so the store-poll fallback carries
    # every op and share ring (the node must still work, only slower).
    DROP = float(os.environ.get("OTEDAMA_FAULT_BELL_DROP", "0") or 0)

    def __init__(self, store, orig_rank: int):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.setblocking(False)
        self.port = self.sock.getsockname()[1]
        self.orig = orig_rank
        self.store = _clone(store) if store is not None else None
        self._lock = threading.Lock()
        self._ports: dict = {}  # orig rank or store key -> (port, looked up at)
        self.rings = 0
        self.dropped = 0  # fault injection only
        if self.store is not None:
            self.store.set(_k("bell", orig_rank), str(self.port))

    def _port_of(self, orig: int) -> int | None:
        if orig == self.orig:
            return self.port
        now = time.monotonic()
        with self._lock:
            hit = self._ports.get(orig)
            if hit is not None and now - hit[1] < self.PORT_TTL:
                return hit[0]
            raw = _store_get(self.store, _k("bell", orig)) if self.store is not None else None
            if raw is None:
                return hit[0] if hit else None
            port = int(raw)
            self._ports[orig] = (port, now)
            return port

    def port_at(self, key: str) -> int | None:
        """A port published at ``key`` (cached for PORT_TTL, like the doorbell ports: a restarted leader has a new
        one)."""
        now = time.monotonic()
        with self._lock:
            hit = self._ports.get(key)
            if hit is not None and now - hit[1] < self.PORT_TTL:
                return hit[0]
            raw = _store_get(self.store, key) if self.store is not None else None
            if raw is None:
                return hit[0] if hit else None
            port = int(raw)
            self._ports[key] = (port, now)
            return port

    def ring(self, orig: int, kind: bytes = b"o") -> None:
        port = self._port_of(orig)
        if port is None:
            return
        if self.DROP and random.random() < self.DROP:
            self.dropped += 1
            return
        try:
            self.sock.sendto(kind, ("127.0.0.1", port))
            self.rings += 1
        except OSError:
            pass  # the store stays authoritative: the peer's fallback poll picks the work up

    def send_port(self, port: int, msg: bytes) -> bool:
        """One datagram to a loopback port (the leader's share-preview port); subject to the same fault injection."""
        if self.DROP and random.random() < self.DROP:
            self.dropped += 1
            return False
        try:
            self.sock.sendto(msg, ("127.0.0.1", port))
            return True
        except OSError:
            return False

    def wait(self, timeout: float) -> list[bytes]:
        got: list[bytes] = []
        try:
            ready, _, _ = select.select([self.sock], [], [], max(timeout, 0.0))
        except (OSError, ValueError):
            return got
        if ready:
            while True:
                try:
                    got.append(self.sock.recv(65536))
                except (BlockingIOError, OSError):
                    break
        return got

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


def op_msg(k: int, raw: str) -> bytes:
    """Doorbell datagram carrying op ``k`` of the log (its JSON exactly as stored at otd/op/<k>)."""
    return b"o" + k.to_bytes(8, "little") + raw.encode()


def parse_op_msg(msg: bytes) -> tuple[int, dict] | None:
    """(k, op) of an inline-op datagram; None for a bare wake-up or anything unparsable."""
    if len(msg) <= 9 or msg[:1] != b"o":
        return None
    try:
        return int.from_bytes(msg[1:9], "little"), json.loads(msg[9:])
    except ValueError:
        return None


class _Heartbeat:
    """Publishes this rank's liveness and cursor every HB_INTERVAL on a store connection of its own (the rank's
    op loop may sit in a bounded collective meanwhile)."""

    def __init__(self, store, orig_rank: int, local: MinerSet, comm: NodeComm | None = None):
        self._origin = store
        self.store = _clone(store)
        self.failures = 0  # store writes that failed (each retried on a fresh connection)
        self.orig = orig_rank
        self.local = local
        self.comm = comm
        self.extra: dict = {}  # owner-supplied fields (e.g. pending shares)
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
                "coll": self.comm.collectives if self.comm is not None else 0,
                # (epoch, CLOCK_MONOTONIC) of the latest new work's first batch running on this rank's device(s)
                "ws": sorted(tuple(x) for s in st for x in (s.get("work_started") or []))[-8:],
                "gen": self.comm.info.generation if self.comm is not None else 0,
                "pid": os.getpid(), **self.extra}

    def _loop(self):
        """One heartbeat per HB_INTERVAL. A failed write (the store stalled past its timeout, a reset connection) is
        retried on a fresh connection at the next beat: a heartbeat thread that gave up would leave a live rank
        looking dead to the leader for good (never re-admitted). At shutdown the store is gone and the process with
        it."""
        while not self.stop.is_set():
            try:
                self.store.set(_k("hb", self.orig), json.dumps(self.payload()))
            except Exception:  # noqa: BLE001
                self.failures += 1
                try:
                    self.store = _clone(self._origin)
                except Exception:  # noqa: BLE001 - not reachable now: try again at the next beat
                    pass
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
        self._bell = _Bell(self.store, comm.info.orig_rank) if self.store is not None else None
        self._wake = threading.Event()  # stores without doorbells (single-rank tests)
        self._gather_wanted = False
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
        # remote shares are admitted once, from a preview datagram or an R2 gather, whichever comes first:
        # share_key -> monotonic time it was first seen, oldest first, pruned past SEEN_TTL and SEEN_MAX
        self._seen: collections.OrderedDict = collections.OrderedDict()
        self._take_lock = threading.Lock()
        self.share_previews = 0        # remote shares first admitted from a preview datagram
        self.share_gathered_first = 0  # ... first from an R2 gather (a lost or late datagram)
        self.previews_refused = 0      # preview datagrams not from the sending rank's doorbell socket
        self._spv: socket.socket | None = None
        self._spv_thread: threading.Thread | None = None
        self._thread: threading.Thread | None = None
        self._op_k = 0
        self._retain = op_retain()
        self._gen = comm.info.generation
        self._gen_started = time.monotonic()
        self.capacity = max(comm.info.capacity, comm.info.world_size, 1)  # orig ranks 0..capacity-1 may exist
        # A leader that the supervisor restarted joins the store without a process group (generation -1): it takes
        # the op log over and forms the next generation with the live followers before anything else.
        self.takeover = comm.info.generation < 0
        self.incarnation = int(self.store.add(_k("leader_inc"), 1)) if self.store is not None else 1
        self._epoch = (self.incarnation - 1) << EPOCH_SHIFT
        # blob seqs live in the incarnation's namespace too: a restarted leader's first blob must order after every
        # blob of its predecessor (followers apply only newer seqs)
        self._seq = (self.incarnation - 1) << EPOCH_SHIFT
        local._epoch = max(local._epoch, self._epoch)
        self.remote_stale = 0  # remote shares of a job the leader no longer knows (e.g. a previous incarnation's)
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
        self._fail_at = 0.0  # monotonic time of the last failed collective (re-forms wait for its stragglers)
        self._hb = _Heartbeat(self.store, comm.info.orig_rank, local, comm) if self.store is not None else None
        # node-wide job switch accounting (CLOCK_MONOTONIC): when the engine handed rank 0 each new job, and when the
        # R1 broadcast carrying it completed on rank 0
        self.job_set_at: collections.deque = collections.deque(maxlen=64)
        self.job_bcast_at: collections.deque = collections.deque(maxlen=64)

    # MinerSet API ------------------------------------------------------------
    @property
    def remote_ids(self) -> list[str]:
        return [f"rank{r}" for r in range(1, self.capacity)]

    def __len__(self) -> int:
        return len(self.local) * max(self.comm.info.world_size, 1)

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
        if self.store is not None and not self.takeover:
            self.store.set(_k("next"), "0")
            self.store.set(_k("gen"), str(self._gen))
        if self.store is not None and self.capacity > 1:
            self._spv = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            self._spv.bind(("127.0.0.1", 0))
            self._spv.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
            self._spv.setblocking(False)
            self.store.set(_k("spv"), str(self._spv.getsockname()[1]))
            self._spv_thread = threading.Thread(target=self._spv_loop, name="otedama-node-spv", daemon=True)
            self._spv_thread.start()
        self._thread = threading.Thread(target=self._loop, name="otedama-node-r0", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        with self._lock:
            self._stop = True
        self._poke()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None
        if self._hb is not None:
            self._hb.stop.set()
        if self._spv_thread is not None:
            self._spv_thread.join(timeout=2)
            self._spv_thread = None
        if self._spv is not None:
            self._spv.close()
            self._spv = None
        self.local.stop()
        if self._bell is not None:
            self._bell.close()

    def _poke(self) -> None:
        """Wake the leader loop (a new job, a pause, stop)."""
        self._wake.set()
        if self._bell is not None:
            self._bell.ring(self._bell.orig, b"w")

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
            self.job_set_at.append((ep, time.monotonic()))
            if template is not None:
                self._jobs[ep] = {"job_id": template.get("job_id", ""), "channel_id": template.get("channel_id", 0),
                                  "extranonce2_size": int(template.get("extranonce2_size", 0) or 0)}
                for old in [e for e in self._jobs if e < ep - 64]:
                    del self._jobs[old]
            self._publish()
            preview = self._blob if template is not None else None
        self._poke()
        if preview is not None:
            self._preview(preview)
        return ep

    def _preview(self, blob: dict) -> None:
        """Job preview: ring every follower with the new job itself, from the engine's thread, before the leader
        loop logs the job op and runs its R1 broadcast. A follower starts the work from the datagram at once; the
        R1 that follows is the consistent delivery (it also covers a lost datagram, and a job too big for one).
        Ordering is by the blob's seq, so a preview never rolls a follower back, and a preview of an older process
        group generation is ignored."""
        if self._bell is None or self.comm.info.world_size <= 1:
            return
        from otedama_amd.parallel.commbase import _encode

        msg = b"j" + json.dumps({"gen": self._gen, "blob": _encode(blob)}).encode()
        if len(msg) > PREVIEW_MAX:
            return
        for r in list(self.comm.info.members):
            if r != self.comm.info.orig_rank:
                self._bell.ring(r, msg)

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
        self._seq += 1
        # seq orders the leader's blobs: a follower never goes back to an older one (a preview can overtake the op
        # log, parallel/node.py NodeWorker._apply)
        self._blob = {"job": blob, "paused": sorted(self._paused), "seq": self._seq}

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
            self._poke()
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

    def heartbeats_snapshot(self) -> dict[int, dict]:
        """The followers' latest heartbeats, read on a store connection of the caller's own (the engine's report
        task runs in another thread than the leader loop, which owns ``self.store``)."""
        if self.store is None:
            return {}
        if getattr(self, "_snap_store", None) is None:
            self._snap_store = _clone(self.store)
        return self._heartbeats(self._snap_store)

    # leader loop --------------------------------------------------------------
    def _post(self, op: dict) -> None:
        op["gen"] = op.get("gen", self._gen)
        raw, k = json.dumps(op), self._op_k
        # The log first: a follower may act on an op it got from the doorbell, so that op must already be the log's
        # entry k (a leader that died between ringing and logging would leave a successor free to post a different
        # op k, which such a follower would skip).
        self.store.set(_k("op", k), raw)
        self._op_k += 1
        if self._bell is not None:  # the followers' op loops wait on their doorbells: the op rides the datagram
            msg = op_msg(k, raw)
            targets = op["members"] if op.get("op") == "reform" else self.comm.info.members
            for r in targets:
                if r != self.comm.info.orig_rank:
                    self._bell.ring(r, msg)
        self.store.set(_k("next"), str(self._op_k))
        if k >= self._retain:  # trim: a follower this far behind re-joins from otd/next instead (its op loop)
            try:
                self.store.delete_key(_k("op", k - self._retain))
            except Exception:  # noqa: BLE001 - trimming is best effort; the next post retries the next entry
                pass

    def _heartbeats(self, store=None) -> dict[int, dict]:
        store = store or self.store
        keys = [_k("hb", r) for r in range(1, self.capacity)]
        out = {}
        for r, key in zip(range(1, self.capacity), keys):
            raw = _store_get(store, key)
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
                if int(hb.get("pending", 0) or 0) > 0:
                    # shares waiting on a follower: gather even if its doorbell rings were lost (the store is the
                    # truth for the share path too; this bounds a lost ring by LIVENESS_EVERY + HB_INTERVAL)
                    self._gather_wanted = True
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

    def _await_left(self, members: list[int], timeout: float) -> list[int]:
        """Wait until no member of ``members`` is still tearing down a failed group (heartbeat ``broken`` newer than
        its ``left``), at most ``timeout`` s; returns the members still busy at the end. Members whose collective
        is about to time out publish ``broken`` within the bounded deadline of the failure, so the wait starts no
        earlier than that (``_fail_at``)."""
        settle = self._fail_at + self.comm.deadline + HB_INTERVAL
        end = time.monotonic() + timeout
        busy: list[int] = []
        while True:
            now = time.monotonic()
            hbs = self._heartbeats()
            busy = [r for r in members if r != self.comm.info.orig_rank and r in hbs
                    and int(hbs[r].get("broken", -1)) > int(hbs[r].get("left", -1))]
            if (not busy and now >= settle) or now >= end:
                return busy
            time.sleep(0.05)

    def _reform(self, dead: list[int], joiners: list[int], why: str, members: list[int] | None = None) -> None:
        info = self.comm.info
        old_world = info.world_size
        if members is None:
            members = [r for r in info.members if r not in dead] + sorted(joiners)
        members = [0] + sorted(r for r in members if r != 0)
        from otedama_amd.parallel.commbase import PG_TIMEOUT_S

        busy = self._await_left(members, PG_TIMEOUT_S + 5.0)
        if busy:
            self.log("warn", f"node: ranks {busy} still leaving the failed group; re-forming anyway")
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
            self.store.set(_k("gen"), str(self._gen))
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

    def _try_reform(self, dead: list[int], joiners: list[int], why: str, members: list[int] | None = None) -> None:
        try:
            self._reform(dead, joiners, why, members)
        except Exception as exc:  # noqa: BLE001 - e.g. a member died during the re-form: the next check retries
            self.log("error", f"node: re-form failed ({type(exc).__name__}: {exc}); retrying")
            self.comm.abort()
        self._sent_seq = -1  # (re-)broadcast the job on the new generation

    def _take_over(self) -> None:
        """A restarted leader: continue the op log after the last op the previous leader posted (it may have died
        between posting an op and bumping otd/next), and form the next generation from every follower whose
        heartbeat is fresh. Followers keep hashing their last job until the new job arrives."""
        store = self.store
        k = int(_store_get(store, _k("next")) or 0)
        while store.check([_k("op", k)]):
            k += 1
        self._op_k = k
        self._gen = int(_store_get(store, _k("gen")) or 0)
        try:
            store.delete_key(_k("dead", 0))
        except Exception:  # noqa: BLE001
            pass
        # followers heartbeat every HB_INTERVAL: give one a full timeout to show up after this process's start-up
        end = time.monotonic() + self.hb_timeout
        live: list[int] = []
        while True:
            now = time.time()
            live = sorted(r for r, hb in self._heartbeats().items()
                          if now - hb["t"] <= self.hb_timeout and _store_get(store, _k("dead", r)) is None)
            if len(live) >= self.capacity - 1 or time.monotonic() >= end:
                break
            time.sleep(0.1)
        for r in live:
            try:
                store.delete_key(_k("join", r))
            except Exception:  # noqa: BLE001
                pass
        self.lost_ranks = [r for r in range(1, self.capacity) if r not in live]
        self._try_reform([], [], f"leader restarted (incarnation {self.incarnation}); followers {live}",
                         members=[0] + live)
        self.takeover = False

    def _loop(self) -> None:
        info = self.comm.info
        self.comm.bind_thread()  # the comm's device is this thread's (HIP device state is per thread)
        next_live = next_stats = time.monotonic()
        try:
            if self.takeover and self.store is not None:
                self._take_over()
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
                    # a new job goes out first (the switch latency of every follower waits on it); the liveness check
                    # (a store round trip per rank) after
                    if info.world_size > 1 and seq != self._sent_seq:
                        self._post({"op": "job"})
                        self.link.run_op({"op": "job"}, blob, [])
                        self._sent_seq = seq
                        job = (blob or {}).get("job") or {}
                        self.job_bcast_at.append((int(job.get("epoch", 0) or 0), time.monotonic()))
                    if now >= next_live and self.store is not None:
                        next_live = now + LIVENESS_EVERY
                        dead, joiners = self._dead_and_joiners()
                        if dead or joiners:
                            why = ", ".join([f"rank {r} lost" for r in dead] + [f"rank {r} joins" for r in joiners])
                            self._try_reform(dead, joiners, why)
                            continue
                    if info.world_size > 1 and self._gather_wanted:
                        self._gather_wanted = False
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
                    self._fail_at = time.monotonic()
                    self.comm.abort()  # tear down now (gloo waits out its op timeout), in parallel with the followers
                    # the peer that broke it shows up as dead within one heartbeat timeout (its process exited, or
                    # it stopped heartbeating); re-form without it, or with everyone if it was transient
                    end = time.monotonic() + self.hb_timeout + 1.0
                    dead, joiners = self._dead_and_joiners()
                    while not dead and time.monotonic() < end:
                        time.sleep(0.1)
                        dead, joiners = self._dead_and_joiners()
                    self._try_reform(dead, joiners, "collective failure" + (f", ranks {dead} lost" if dead else ""))
                    continue
                self._wait(min(next_live, next_stats) - time.monotonic())
        except BaseException as exc:  # noqa: BLE001
            self.link.error = exc
            self.log("error", f"node: control loop failed: {exc}")

    def _wait(self, timeout: float) -> None:
        """Sleep until a doorbell (a follower's shares, a local job / pause / stop) or ``timeout``."""
        timeout = min(max(timeout, 0.0), LIVENESS_EVERY)
        if self._bell is None:
            self._wake.wait(min(timeout, self.tick))
            self._wake.clear()
            return
        got = self._bell.wait(timeout)
        self._wake.clear()
        if any(m[:1] == b"s" for m in got):
            self._gather_wanted = True

    def _spv_loop(self) -> None:
        """Share previews: submit a follower's shares as their datagram arrives, whatever the leader loop is doing
        (it may sit in a collective that waits for a wave slot)."""
        sock = self._spv
        while not self._stop:
            try:
                ready, _, _ = select.select([sock], [], [], 0.25)
            except (OSError, ValueError):
                return
            while ready:
                try:
                    msg, src = sock.recvfrom(65536)
                except (BlockingIOError, OSError):
                    break
                try:
                    # a preview comes from its rank's doorbell socket (otd/bell/<rank>): anything else on this
                    # loopback port (a stale sender of an earlier node on this host) is dropped
                    if len(msg) < 3 or self._bell is None or \
                            src[1] != self._bell._port_of(int.from_bytes(msg[1:3], "little")):
                        self.previews_refused += 1
                        continue
                    shares = parse_share_preview(msg)
                    if shares:
                        self._take(shares, preview=True)
                except Exception as exc:  # noqa: BLE001 - one bad datagram must not end the previews (R2 covers it)
                    self.log("warn", f"node: share preview dropped ({type(exc).__name__}: {exc})")

    def _take(self, shares: list[dict], preview: bool = False) -> None:
        n = 0
        me = self.comm.info.orig_rank
        now = time.monotonic()
        with self._take_lock:
            seen = self._seen
            while seen and (len(seen) > SEEN_MAX or now - next(iter(seen.values())) > SEEN_TTL):
                seen.popitem(last=False)
            for s in shares:
                if s["orig_rank"] == me:
                    continue
                key = share_key(s)
                if key in seen:
                    continue  # already admitted by the other path
                seen[key] = now
                meta = self._jobs.get(s["epoch"])
                if meta is None:
                    self.remote_stale += 1  # a job older than the retained window, or a previous leader's
                    continue
                s.update(meta)
                s["device_id"] = f"rank{s['orig_rank']}"
                self._remote.append(s)
                n += 1
                if preview:
                    self.share_previews += 1
                else:
                    self.share_gathered_first += 1
        if not preview:
            per_rank = collections.Counter(s["orig_rank"] for s in shares)
            if per_rank and max(per_rank.values()) >= SHARE_SLOTS:
                self._gather_wanted = True  # a rank filled its slot array: it may hold more
        if n:
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
        self._hb = _Heartbeat(self.store, comm.info.orig_rank, local, comm)
        self._bell = _Bell(self.store, comm.info.orig_rank)
        self._pending: list[dict] = []
        self._hb.extra["pending"] = 0  # before the heartbeat thread starts: the share thread only updates it
        # (epoch, CLOCK_MONOTONIC) of the latest jobs this rank handed its devices (node job-switch breakdown)
        self._applied: collections.deque = collections.deque(maxlen=8)
        self._hb.extra["ja"] = []
        self.pending_dropped = 0  # shares dropped past PENDING_CAP (a leader that stays away)
        self.previews = 0  # jobs started from a preview datagram ahead of their R1 broadcast
        self.previews_sent = 0  # share-preview datagrams sent to the leader
        # OTEDAMA_NODE_SHARE_PREVIEWS=0: shares travel by R2 only (the A/B baseline)
        self._share_previews = os.environ.get("OTEDAMA_NODE_SHARE_PREVIEWS", "1") != "0"
        self._seq_applied = 0  # seq of the leader blob this rank runs (previews and R1 only move it forward)
        self._plock = threading.Lock()
        self._stop = threading.Event()

    def _share_loop(self) -> None:
        """Wake on the local miners' share eventfds, send the new shares to the leader's preview port and ring its
        doorbell for the R2 gather that delivers them consistently. With a preview out, the ring waits PREVIEW_GRACE,
        so the gather (and the collective's device work) stays out of the leader's way while it submits the
        previewed shares, and the shares of that window share one gather. Without one (previews off, no port yet, a
        failed send) the ring goes at once. While shares are still waiting (a lost datagram, a leader that is being
        restarted, more than one gather's worth) the bell is rung again every BELL_FALLBACK."""
        while not self._stop.is_set():
            try:
                self._share_pass()
            except Exception as exc:  # noqa: BLE001 - the share path must outlive one bad pass
                self.log("warn", f"node: {self.rank_id}: share loop error ({type(exc).__name__}: {exc})")
                self._stop.wait(BELL_FALLBACK)

    def _share_pass(self) -> None:
        """The share loop's body (see _share_loop); returns only on stop or an error."""
        fds = list(self.local.share_fds())
        last_ring = 0.0
        hold_until = None  # a preview went out: ring for its R2 at this time
        while not self._stop.is_set():
            wait = BELL_FALLBACK if hold_until is None else max(0.0, min(BELL_FALLBACK, hold_until - time.monotonic()))
            if fds:
                ready, _, _ = select.select(fds, [], [], wait)
                for fd in ready:
                    try:
                        os.read(fd, 8)
                    except BlockingIOError:
                        pass
            else:
                self._stop.wait(min(wait, 0.01))
            new = self.local.poll(256)
            with self._plock:
                if new:
                    self._pending.extend(new)
                    over = len(self._pending) - PENDING_CAP
                    if over > 0:
                        del self._pending[:over]
                        self.pending_dropped += over
                waiting = len(self._pending)
            self._hb.extra["pending"] = waiting
            now = time.monotonic()
            ring = False
            if new:
                sent = False
                if self._share_previews:
                    port = self._bell.port_at(_k("spv"))
                    if port is not None:
                        sent = True
                        for msg in share_preview_msgs(new, self.comm.info.orig_rank):
                            if self._bell.send_port(port, msg):
                                self.previews_sent += 1
                            else:
                                sent = False
                if sent:
                    hold_until = hold_until or now + PREVIEW_GRACE
                else:
                    ring = True
            if waiting and hold_until is not None and now >= hold_until:
                ring = True
            elif waiting and hold_until is None and now - last_ring >= BELL_FALLBACK:
                ring = True
            if ring:
                self._bell.ring(0, b"s")
                last_ring, hold_until = now, None
            elif not waiting:
                hold_until = None

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
        inline: dict[int, dict] = {}  # ops that arrived on the doorbell ahead of this loop reaching them
        retain, lag_checked = op_retain(), time.monotonic()
        try:
            while True:
                # the leader rings this rank's doorbell with each op as it posts it; the store log is the truth for
                # an op whose datagram was lost, and the fallback wait bounds that case
                op = inline.pop(k, None)
                if op is None:
                    key = _k("op", k)
                    raw = None
                    if self.store.check([key]):
                        raw = _store_get(self.store, key, timeout=2.0)  # None: trimmed since the check
                    else:
                        msgs = self._bell.wait(BELL_FALLBACK)
                        for msg in msgs:
                            if msg[:1] == b"j":
                                self._take_preview(msg, broken)
                                continue
                            got = parse_op_msg(msg)
                            if got is not None and got[0] >= k and len(inline) < 4096:
                                inline[got[0]] = got[1]
                    if raw is None:
                        # Behind the trimmed log? Checked on a timer whether or not datagrams arrive: on a busy node
                        # the doorbell rings often, and op k may be gone for good.
                        now = time.monotonic()
                        if now - lag_checked >= 1.0:
                            lag_checked = now
                            nxt = int(_store_get(self.store, _k("next")) or 0)
                            if nxt - k > retain:  # op k was trimmed from the log: re-join from the current end
                                self.log("warn", f"node: {self.rank_id} fell {nxt - k} ops behind the log; re-joining")
                                k, broken = nxt, True
                                inline.clear()
                                self._leave_group()
                                self.store.set(_k("join", info.orig_rank), "1")
                        continue
                    op = json.loads(raw)
                k += 1
                kind = op["op"]
                if kind == "stop":
                    return
                if kind == "reform":
                    cur = _store_get(self.store, _k("gen"), timeout=2.0)
                    if cur is not None and int(cur) > int(op["gen"]):
                        # superseded: the leader gave up on this generation (a member joined too late, e.g. one
                        # stuck tearing down a gloo group) and posted a newer one further down the log; joining it now
                        # would only wait out the rendezvous timeout while the leader waits in the next one
                        broken = True
                        continue
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
                            self._apply(blob)  # a no-op when its preview was applied already (same seq)
                    elif kind == "gather":
                        with self._plock:
                            out, self._pending = self._pending[:SHARE_SLOTS], self._pending[SHARE_SLOTS:]
                        try:
                            self.link.run_op(op, None, out)
                        except Exception:
                            with self._plock:  # not delivered: keep them for the next gather
                                self._pending[:0] = out
                            raise
                        with self._plock:
                            more = bool(self._pending)
                        if more:
                            self._bell.ring(0, b"s")
                    elif kind == "stats":
                        self.link.run_op(op, None, [])
                        self.local.retire_faulted()  # survivors re-split this rank's class at once
                except Exception as exc:  # noqa: BLE001 - leave this group; the leader re-forms
                    self.log("warn", f"node: {self.rank_id}: collective failed ({type(exc).__name__}: {exc})")
                    self._leave_group()
                    broken = True
        finally:
            self._stop.set()
            self._hb.stop.set()
            share_th.join(timeout=5)
            self.local.stop()
            self._bell.close()

    def _leave_group(self) -> None:
        """Abort the current group, telling the leader through the heartbeat: ``broken`` = the generation whose
        collective failed, ``left`` = the generation whose teardown finished. Tearing a gloo group down waits out
        its op timeout (RCCL aborts at once); the leader posts the next re-form only once every broken member has
        left (NodeMinerSet._await_left), so nobody reaches the rendezvous after the leader gave up on it."""
        gen = self.comm.info.generation
        self._hb.extra["broken"] = gen
        try:
            self.comm.abort()
        finally:
            self._hb.extra["left"] = gen

    def _take_preview(self, msg: bytes, broken: bool) -> None:
        """A job preview from the leader (NodeMinerSet._preview): start it if it belongs to this rank's current
        generation and is newer than what runs."""
        try:
            d = json.loads(msg[1:])
        except ValueError:
            return
        info = self.comm.info
        if broken or info.generation < 0 or d.get("gen") != info.generation:
            return
        from otedama_amd.parallel.commbase import _decode

        if self._apply(_decode(d.get("blob") or {})):
            self.previews += 1

    def _apply(self, blob: dict) -> bool:
        """Hand the leader's blob to the local devices; False when it is not newer than the one running (by seq)."""
        seq = int(blob.get("seq", 0) or 0)
        if seq and seq <= self._seq_applied:
            return False
        if seq:
            self._seq_applied = seq
        job = blob.get("job")
        paused = self.rank_id in set(blob.get("paused", []))
        if job is None or paused:
            self.local.set_job(None)
            return True
        self.local.set_job(job, epoch=int(job["epoch"]))
        self._applied.append((int(job["epoch"]), time.monotonic()))
        self._hb.extra["ja"] = list(self._applied)
        return True
