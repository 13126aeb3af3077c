"""One process per GPU: fault containment for the single-host miner.

A kernel memory fault or a hung device aborts the process that owns the HIP context. With every GPU's miner in
the engine process, one bad GPU would stop all eight. Here each device runs in a child process of its own
(``python -m otedama_amd.engine.devproc``), spawned before anything touches the GPU, and the engine process
stays GPU-free:

  parent (engine)                                child (one per GPU, no torch)
  DeviceProcess.set_job ── job frame ──────────▶ native GpuMiner.set_job
  share_fd (eventfd) ◀── shares frame ◀──────── ShareQueue eventfd -> poll()   (pushed the moment they are queued)
  stats() ◀───────────── stats frame (2 Hz) ─── GpuMiner.stats()              (also the heartbeat)

Frames are a 4-byte little-endian length + msgpack over a Unix socketpair. A child that dies (signal, HIP fault,
``faulted`` stats) closes its socket: the parent marks the device faulted at once (MinerSet re-splits its stripe
over the survivors) and ``restart()`` brings up a fresh process, which rejoins with the current job.

Reference analogue: a dead worker goroutine just stops contributing and the partial-failure-tolerant detector
keeps the other devices (internal/hal/registry.go:138-201); failover/backoff as in
internal/engine/run.go:368-521.
"""
from __future__ import annotations

import collections
import os
import select
import signal
import socket
import struct
import subprocess
import sys
import threading
import time

import msgpack

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STATS_PERIOD = 0.5      # child -> parent stats / heartbeat
_HDR = struct.Struct("<I")
MAX_FRAME = 64 << 20

# counters that survive a respawn (summed over the device's processes)
_CUMULATIVE = ("hashes", "candidates", "shares", "dropped", "launches", "rejected_candidates", "variant_launches",
               "busy_seconds", "job_switches", "aborted_launches", "ring_hits", "ring_overflow", "verify_dropped")


def _send(sock: socket.socket, obj, lock: threading.Lock | None = None) -> None:
    data = msgpack.packb(obj, use_bin_type=True)
    frame = _HDR.pack(len(data)) + data
    if lock is None:
        sock.sendall(frame)
    else:
        with lock:
            sock.sendall(frame)


class _Framer:
    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes) -> list:
        self.buf += data
        out = []
        while len(self.buf) >= 4:
            (n,) = _HDR.unpack_from(self.buf)
            if n > MAX_FRAME:
                raise ValueError(f"frame of {n} bytes exceeds {MAX_FRAME}")
            if len(self.buf) < 4 + n:
                break
            out.append(msgpack.unpackb(bytes(self.buf[4 : 4 + n]), raw=False))
            del self.buf[: 4 + n]
        return out


DEVICE_HW_QUEUES = ""  # default cap on a device process's normal-priority hardware queues ("" = the runtime's 4)


class DeviceProcess:
    """Parent-side handle with the native miner's interface (start/stop/set_job/poll/stats/share_fd)."""

    def __init__(self, device_index: int, device_id: str, batch_nonces: int = 1 << 32, grid: int = 1536,
                 queue_cap: int = 4096, sha_variants: int = 128, cpu_threads: int = 0, log=None,
                 on_exit=None, on_ready=None, env: dict | None = None):
        self.device_index = device_index
        self.device_id = device_id
        self.args = {"batch": batch_nonces, "grid": grid, "queue_cap": queue_cap, "sha_variants": sha_variants,
                     "cpu_threads": cpu_threads}
        self.log = log or (lambda level, msg: None)
        self.on_exit = on_exit      # callback(DeviceProcess) when a child dies unexpectedly
        self.on_ready = on_ready    # callback(DeviceProcess) when a (re)spawned child reports in
        self.env = env
        self._lock = threading.Lock()
        self._send_lock = threading.Lock()
        self._shares: collections.deque = collections.deque()
        self._efd = os.eventfd(0, os.EFD_NONBLOCK | os.EFD_CLOEXEC)
        self._job: dict | None = None
        self._proc: subprocess.Popen | None = None
        self._sock: socket.socket | None = None
        self._reader: threading.Thread | None = None
        self._child: dict = {}           # latest stats of the running child
        self._base = {k: 0 for k in _CUMULATIVE}
        self._stopping = False
        self.exit_code: int | None = None
        self.error = ""
        self.restarts = 0
        self.ready_at = 0.0
        self.spawned_at = 0.0
        self.startup_seconds = 0.0       # spawn -> child reported its miner running
        self.first_hash_wall = 0.0       # wall clock when the child's first batch was running
        self.child_timing: dict = {}     # wall clock: child main(), native module loaded, first batch done
        self.native_startup_ms: dict = {}  # the native miner thread's own phases (hip_set_device, buffers, ...)

    # ------------------------------------------------------------- lifecycle
    def start(self) -> None:
        self._spawn()

    def _spawn(self) -> None:
        parent, child = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        env = dict(os.environ if self.env is None else self.env)
        env["OTEDAMA_NO_TORCH"] = "1"
        env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        # Hardware queues of the child's HIP runtime (each one a 173 MiB host mapping, profiles/r4/c_host_abort):
        # OTEDAMA_DEVICE_HW_QUEUES caps them through GPU_MAX_HW_QUEUES unless that is set explicitly.
        hwq = env.get("OTEDAMA_DEVICE_HW_QUEUES", DEVICE_HW_QUEUES)
        if hwq and "GPU_MAX_HW_QUEUES" not in env:
            env["GPU_MAX_HW_QUEUES"] = str(hwq)
        a = self.args
        cmd = [sys.executable, "-m", "otedama_amd.engine.devproc", "--fd", str(child.fileno()),
               "--device", str(self.device_index), "--id", self.device_id, "--batch", str(a["batch"]),
               "--grid", str(a["grid"]), "--queue-cap", str(a["queue_cap"]), "--sha-variants", str(a["sha_variants"]),
               "--cpu-threads", str(a["cpu_threads"])]
        self.spawned_at = time.monotonic()
        self._proc = subprocess.Popen(cmd, pass_fds=(child.fileno(),), env=env, cwd=ROOT)
        child.close()
        self._sock = parent
        self.exit_code = None
        self.error = ""
        self._stopping = False
        self._child = {}
        self._reader = threading.Thread(target=self._read_loop, args=(parent, self._proc),
                                        name=f"otedama-devproc-{self.device_id}", daemon=True)
        self._reader.start()
        if self._job is not None:
            self._post({"op": "job", "t": self._job})

    def stop(self) -> None:
        self._stopping = True
        self._post({"op": "stop"})
        p = self._proc
        if p is not None:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if self._reader is not None:
            self._reader.join(timeout=5)
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass

    def restart(self, replay_job: bool = True) -> bool:
        """Replace a dead child with a fresh process; False (nothing spawned) while the old child has not been
        reaped yet — the caller retries later. ``replay_job``: re-send the last job at once; a MinerSet passes
        False and applies a fresh stripe when the process reports ready, because replaying the dead process's
        stripe would search its nonces a second time."""
        if self.alive:
            return False
        if not replay_job:
            self._job = None
        with self._lock:
            for k in _CUMULATIVE:
                self._base[k] += self._child.get(k, 0)
            self._child = {}
        self.restarts += 1
        self._spawn()
        return True

    def kill(self, sig: int = signal.SIGKILL) -> None:
        """Fault injection (tests / chaos): signal the child."""
        if self._proc is not None and self._proc.poll() is None:
            self._proc.send_signal(sig)

    @property
    def alive(self) -> bool:
        return self._proc is not None and self._proc.poll() is None and self.exit_code is None

    @property
    def pid(self) -> int:
        return self._proc.pid if self._proc is not None else 0

    # ------------------------------------------------------------- miner interface
    def set_job(self, template: dict | None) -> None:
        self._job = dict(template) if template is not None else None
        # "sent" (CLOCK_MONOTONIC, shared by both processes): the child reports the hop, frame -> native set_job
        self._post({"op": "job", "t": self._job, "sent": time.monotonic()})

    def poll(self, max_items: int = 256) -> list[dict]:
        out = []
        with self._lock:
            while self._shares and len(out) < max_items:
                out.append(self._shares.popleft())
        return out

    def share_fd(self) -> int:
        return self._efd

    def stats(self) -> dict:
        with self._lock:
            st = dict(self._child)
            for k in _CUMULATIVE:
                st[k] = self._base[k] + st.get(k, 0)
        st.setdefault("error", "")
        st.setdefault("faulted", False)
        if self.exit_code is not None:
            st["faulted"] = True
            st["error"] = self.error
        st["process_restarts"] = self.restarts
        st["pid"] = self.pid
        st["startup_seconds"] = self.startup_seconds
        st["first_hash_wall"] = self.first_hash_wall
        st["child_timing"] = dict(self.child_timing)
        st["native_startup_ms"] = dict(self.native_startup_ms)
        return st

    # ------------------------------------------------------------- plumbing
    def _post(self, obj) -> None:
        s = self._sock
        if s is None:
            return
        try:
            _send(s, obj, self._send_lock)
        except OSError:
            pass  # the reader notices the dead child

    def _read_loop(self, sock: socket.socket, proc: subprocess.Popen) -> None:
        fr = _Framer()
        while True:
            try:
                data = sock.recv(1 << 20)
            except OSError:
                data = b""
            if not data:
                break
            try:
                msgs = fr.feed(data)
            except ValueError as exc:
                self.log("error", f"devproc {self.device_id}: bad frame: {exc}")
                break
            for m in msgs:
                op = m.get("op")
                if op == "shares":
                    with self._lock:
                        self._shares.extend(m["s"])
                    os.eventfd_write(self._efd, 1)
                elif op == "stats":
                    with self._lock:
                        self._child = m["st"]
                elif op == "first_hash":
                    self.first_hash_wall = float(m.get("wall", 0.0))
                    self.child_timing = {"main": m.get("t_main", 0.0), "native_loaded": m.get("t_native", 0.0),
                                         "miner_started": m.get("t_started", 0.0), "first_job": m.get("t_job", 0.0),
                                         "first_hash": self.first_hash_wall}
                    self.native_startup_ms = dict(m.get("native_ms") or {})
                elif op == "ready":
                    self.ready_at = time.monotonic()
                    self.startup_seconds = self.ready_at - self.spawned_at
                    if self.on_ready is not None:
                        self.on_ready(self)
        # EOF: the child exited (or is exiting). Its socket is closed here, not left to garbage collection once a
        # restart replaces self._sock (a closed socket object makes a late _post raise OSError, which it ignores).
        try:
            sock.close()
        except OSError:
            pass
        try:
            rc = proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            proc.kill()
            rc = proc.wait()
        if proc is not self._proc:
            return  # a restart already replaced this child: its exit says nothing about the new one
        last_err = self._child.get("error", "")
        self.exit_code = rc
        self.error = (f"device process exited with code {rc}" if rc >= 0 else
                      f"device process killed by signal {-rc}") + (f": {last_err}" if last_err else "")
        if not self._stopping:
            self.log("error", f"devproc {self.device_id}: {self.error}")
            if self.on_exit is not None:
                self.on_exit(self)


# ----------------------------------------------------------------------------- child
def _child(argv: list[str]) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="otedama_amd.engine.devproc")
    ap.add_argument("--fd", type=int, required=True)
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--id", required=True)
    ap.add_argument("--batch", type=int, default=1 << 32)
    ap.add_argument("--grid", type=int, default=1536)
    ap.add_argument("--queue-cap", type=int, default=4096)
    ap.add_argument("--sha-variants", type=int, default=128)
    ap.add_argument("--cpu-threads", type=int, default=0, help="> 0: a native CpuMiner instead of a GPU (tests)")
    a = ap.parse_args(argv)
    t_main = time.time()
    os.environ["OTEDAMA_NO_TORCH"] = "1"
    sock = socket.socket(fileno=a.fd)
    from otedama_amd.ops.native import require_native

    N = require_native()
    t_native = time.time()
    if a.cpu_threads > 0:
        m = N.CpuMiner(a.cpu_threads, a.id, a.queue_cap)
    else:
        m = N.GpuMiner(a.device, a.id, batch_nonces=a.batch, grid=a.grid, queue_cap=a.queue_cap,
                       sha_variants=a.sha_variants)
    m.start()
    t_started = time.time()
    t_job = 0.0
    _send(sock, {"op": "ready", "pid": os.getpid()})
    efd = m.share_fd()
    poller = select.poll()
    poller.register(sock.fileno(), select.POLLIN)
    poller.register(efd, select.POLLIN)
    fr = _Framer()
    hops: collections.deque = collections.deque(maxlen=64)  # job frame sent (parent) -> native set_job, ms
    next_stats = 0.0
    first_hash = False  # until the first batch is running: poll fast and report it at once (start-up timing)
    rc = 0
    try:
        while True:
            timeout = max(0.0, next_stats - time.monotonic())
            if not first_hash:
                timeout = min(timeout, 0.005)
            for fd, _ev in poller.poll(timeout * 1e3):
                if fd == efd:
                    try:
                        os.read(efd, 8)
                    except BlockingIOError:
                        pass
                    shares = m.poll(4096)
                    if shares:
                        _send(sock, {"op": "shares", "s": shares})
                    continue
                data = sock.recv(1 << 20)
                if not data:  # parent gone: stop mining
                    return 0
                for msg in fr.feed(data):
                    if msg.get("op") == "job":
                        m.set_job(msg.get("t"))
                        if msg.get("sent"):
                            hops.append((time.monotonic() - float(msg["sent"])) * 1e3)
                        t_job = t_job or time.time()
                    elif msg.get("op") == "stop":
                        return 0
            if not first_hash and (m.stats()["job_switches"] > 0 or m.stats()["hashes"] > 0):
                # hashing has begun: the first batch of the first job is running on the device (CPU: counted)
                first_hash = True
                _send(sock, {"op": "first_hash", "wall": time.time(), "t_main": t_main, "t_native": t_native,
                             "t_started": t_started, "t_job": t_job,
                             "native_ms": dict(m.stats().get("startup_ms", {}))})
                next_stats = 0.0
            if time.monotonic() >= next_stats:
                st = m.stats()
                st["job_hop_ms"] = list(hops)
                _send(sock, {"op": "stats", "st": st})
                next_stats = time.monotonic() + STATS_PERIOD
                if st.get("faulted"):
                    rc = 3  # a faulted HIP context is unusable: exit so the parent starts a fresh process
                    return rc
    except (BrokenPipeError, ConnectionResetError):
        return 0
    finally:
        m.stop()
        shares = m.poll(1 << 16)
        if shares:
            try:
                _send(sock, {"op": "shares", "s": shares})
            except OSError:
                pass
        try:
            st = m.stats()
            st["job_hop_ms"] = list(hops)
            _send(sock, {"op": "stats", "st": st})
        except OSError:
            pass


if __name__ == "__main__":
    sys.exit(_child(sys.argv[1:]))
