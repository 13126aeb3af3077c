"""Deadlines for a multi-rank run that must always report (bench.py; VERDICT r4, "next round" item 1).

The driver gets one 8-GPU run of ``bench.py --gpus 8``. If the RCCL rendezvous, a collective or a kernel hangs in it,
the run must still print its JSON line: the sections that finished, the one that did not and why, and for a failed
start every rank's last phase plus the tail of its stderr and of its RCCL log. The reference's rule is the same in
miniature: no I/O of its engine waits without a deadline (internal/engine/run.go:1251, a 10 s write deadline; the
V1 read loop's 5 min deadline, internal/poolproto/stratumv1/stratumv1.go:166).

``RankGuard`` runs in every rank:

* sections: ``with guard.section("scrypt", budget_s):``. A watchdog thread fires when the section (or the whole run's
  deadline) passes. It never waits on the main thread, which may be stuck inside a HIP call or a collective.
* rank 0 fires by emitting the JSON through the ``emit`` callback (everything measured so far plus the error), asking
  every other live rank to leave (SIGUSR1), and calling ``os._exit``. The other ranks fire ``margin`` seconds later
  than rank 0 would, so rank 0 reports first. A rank that gets SIGUSR1 leaves with code 0, so a torchrun agent sees
  a clean job. A SIGTERM (torchrun tearing the job down after a peer died, the driver's timeout, the launcher's
  deadline) makes rank 0 emit at once, for the same reason.
* signals reach the watchdog through ``signal.set_wakeup_fd``: CPython's C-level handler writes the signal number to
  a pipe even while the main thread sits in C code. No signal mask is changed, so child processes (the node, the
  pool) inherit normal signal handling.
* every rank keeps a status file ``rank<r>.json`` (pid, phase, times, last error) in a run directory shared by the job
  (keyed by MASTER_PORT and the torchrun run id). With ``tee_stderr`` it copies its stderr to ``rank<r>.stderr``
  there, and RCCL's log (``NCCL_DEBUG=WARN``) goes to ``rccl.<host>.<pid>.log`` there. ``diagnose()`` reads all of
  these back for the error JSON.

Fault hooks for the CPU rehearsal tests: ``OTEDAMA_BENCH_FAULT=stuck:<rank>:<section>[,...]`` makes that rank hang
at the start of that section (an uninterruptible-looking sleep), ``exit:<rank>:<section>`` makes it exit with code 7;
``fail:<rank>:probe`` / ``hang:<rank>:probe`` make that rank's data-plane probe child fail or hang
(parallel/rccl_probe.py); ``slow:<rank>:arrive`` delays that rank's arrival at the probe by OTEDAMA_FAULT_SLOW_S
(a cold-start skew); ``fail:<rank>:native`` fails its in-process native init after the probe;
``fail:<rank>:<section>`` makes that section raise at its start.
"""
from __future__ import annotations

import contextlib
import glob
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

SIG_PEER_STOP = signal.SIGUSR1
STDERR_TAIL = 600       # bytes of each rank's stderr kept in an error JSON
RCCL_TAIL = 400         # bytes of each RCCL log kept
STALE_S = 300.0         # ranks of one job start within this of each other (the guard starts before `import torch`)


def run_dir_for(env=None) -> str:
    """The directory every rank of one job shares: same MASTER_PORT and torchrun run id, same host."""
    env = os.environ if env is None else env
    key = "".join(c if c.isalnum() else "_" for c in env.get("TORCHELASTIC_RUN_ID", "") or "local")[:40]
    port = env.get("MASTER_PORT")
    if port is None:  # a single process (no rendezvous): a directory of its own
        port, key = "solo", f"pid{os.getpid()}"
    d = os.path.join(tempfile.gettempdir(), f"otedama-run-{port}-{key}")
    os.makedirs(d, exist_ok=True)
    return d


def _tail(path: str, n: int) -> str:
    try:
        with open(path, "rb") as f:
            f.seek(0, os.SEEK_END)
            size = f.tell()
            f.seek(max(0, size - n))
            return f.read().decode("utf-8", "replace")
    except OSError:
        return ""


def _pid_is_rank(pid: int, marker: str) -> bool:
    """The pid is still a process of this job (guards against signalling a recycled pid)."""
    try:
        with open(f"/proc/{pid}/cmdline", "rb") as f:
            return marker.encode() in f.read()
    except OSError:
        return False


def fault_for(rank: int, section: str, env=None) -> str | None:
    """The injected fault for (rank, section), if any: 'stuck' or 'exit'."""
    spec = (os.environ if env is None else env).get("OTEDAMA_BENCH_FAULT", "")
    for item in filter(None, (s.strip() for s in spec.split(","))):
        parts = item.split(":")
        if len(parts) == 3 and parts[0] in ("stuck", "exit", "fail", "hang", "slow") and parts[2] == section:
            try:
                if int(parts[1]) == rank:
                    return parts[0]
            except ValueError:
                continue
    return None


class RankGuard:
    """Per-rank section deadlines and the always-report exit path (module docstring)."""

    PROGRESS_EVERY = 30.0  # rank 0: a "still in section X" line at least this often (a silent run looks hung)

    def __init__(self, rank: int, world: int, deadline_s: float, emit=None, run_dir: str | None = None,
                 margin_s: float = 30.0, marker: str = "bench.py", poll_s: float = 0.25, progress: bool = True):
        self.rank, self.world = rank, world
        self.t0 = time.monotonic()
        self.t_start_wall = time.time()
        self.margin = 0.0 if rank == 0 else margin_s
        self.deadline_s = deadline_s
        self.end = self.t0 + deadline_s + self.margin
        self.emit = emit            # rank 0: emit(errors: dict, reason: str) -> int (exit code); prints the JSON
        self.run_dir = run_dir or run_dir_for()
        self.marker = marker
        self.poll_s = poll_s
        self.current: str | None = None
        self.section_end: float | None = None
        self.section_budget = 0.0
        self.sections: dict[str, dict] = {}   # name -> {"s": seconds, "status": ok|error|timeout|skipped}
        self.errors: dict[str, str] = {}
        self._lock = threading.RLock()
        self._fired = False
        self._rfd = self._wfd = -1
        self._tee: subprocess.Popen | None = None
        self.status_path = os.path.join(self.run_dir, f"rank{rank}.json")
        self.phase = "start"
        self.progress_on = progress and rank == 0
        self._last_progress = time.monotonic()
        self.headline_done = False  # set by the run once its critical (headline) sections completed

    def progress(self, msg: str) -> None:
        """One line on stderr from rank 0: section starts / ends and a periodic heartbeat, so a watcher that kills
        silent commands (and a human reading the log) sees the run is alive and where it is."""
        if not self.progress_on:
            return
        self._last_progress = time.monotonic()
        try:
            os.write(2, f"[bench +{self.elapsed():.1f}s] {msg}\n".encode())
        except OSError:
            pass

    # ------------------------------------------------------------------ set-up
    def start(self, tee_stderr: bool = False) -> "RankGuard":
        if tee_stderr:
            self._tee_stderr()
        self._write_status()
        self._rfd, self._wfd = os.pipe()
        os.set_blocking(self._wfd, False)
        try:
            signal.set_wakeup_fd(self._wfd, warn_on_full_buffer=False)
            for sig in (signal.SIGTERM, SIG_PEER_STOP):
                signal.signal(sig, lambda *_: None)  # the watchdog acts on the wake-up byte
        except ValueError:  # not the main thread (in-process tests): deadlines still work, signals keep defaults
            pass
        threading.Thread(target=self._watch, name=f"otedama-guard-{self.rank}", daemon=True).start()
        return self

    def _tee_stderr(self) -> None:
        """Copy this process's stderr (fd 2, so C-level output too) into the run directory through a `tee` child:
        a separate process, so a main thread stuck in C code can never block it."""
        path = os.path.join(self.run_dir, f"rank{self.rank}.stderr")
        try:
            orig = os.dup(2)
            self._tee = subprocess.Popen(["tee", "-a", path], stdin=subprocess.PIPE, stdout=orig,
                                         stderr=subprocess.DEVNULL, pass_fds=(orig,), start_new_session=True)
            os.dup2(self._tee.stdin.fileno(), 2)  # sys.stderr writes to fd 2, so it follows
            os.close(orig)
        except OSError:
            self._tee = None

    def _write_status(self, **extra) -> None:
        st = {"rank": self.rank, "world": self.world, "pid": os.getpid(), "host": socket.gethostname(),
              "t_start": self.t_start_wall,
              "phase": self.phase, "section": self.current, "t_wall": time.time(),
              "elapsed_s": round(time.monotonic() - self.t0, 3), "sections": self.sections,
              "errors": self.errors, **extra}
        tmp = self.status_path + ".tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(st, f)
            os.replace(tmp, self.status_path)
        except OSError:
            pass

    def set_phase(self, phase: str) -> None:
        self.phase = phase
        self._write_status()

    # ------------------------------------------------------------------ sections
    def remaining(self) -> float:
        return self.end - self.margin - time.monotonic()

    def elapsed(self) -> float:
        return time.monotonic() - self.t0

    @contextlib.contextmanager
    def section(self, name: str, budget_s: float, critical: bool = False):
        """Run a section under its own deadline (capped by the run's). An exception is recorded in ``errors`` and
        swallowed, so the run goes on to its next section; a ``critical`` section (the pre-flight, the headline)
        re-raises it."""
        t = time.monotonic()
        with self._lock:
            self.current = name
            self.section_budget = budget_s
            self.section_end = min(t + budget_s + self.margin, self.end)
            self.phase = f"section:{name}"
        self._write_status()
        self.progress(f"section {name}: start (budget {budget_s:.0f} s)")
        fault = fault_for(self.rank, name)
        if fault == "stuck":
            while True:
                time.sleep(3600)
        if fault == "exit":
            os._exit(7)
        try:
            if fault == "fail":  # tests: the section raises at once (a start that failed, not a hang)
                raise RuntimeError(f"injected failure in section {name}")
            yield
        except Exception as exc:  # noqa: BLE001 - a failed section is recorded; the run goes on
            with self._lock:
                self.errors[name] = f"{type(exc).__name__}: {exc}"[:500]
                self.sections[name] = {"s": round(time.monotonic() - t, 2), "status": "error"}
                self.current = self.section_end = None
            self._write_status()
            self.progress(f"section {name}: FAILED {self.errors[name]}")
            if critical:
                raise
            return
        with self._lock:
            if self.sections.get(name, {}).get("status") not in ("timeout", "terminated"):  # the watchdog's verdict
                self.sections[name] = {"s": round(time.monotonic() - t, 2), "status": "ok"}  # stands
            self.current = self.section_end = None
        self._write_status()
        self.progress(f"section {name}: done in {time.monotonic() - t:.1f} s")

    def skip(self, name: str, why: str) -> None:
        with self._lock:
            self.sections[name] = {"s": 0.0, "status": "skipped", "why": why}
        self._write_status()
        self.progress(f"section {name}: skipped ({why})")

    def finish(self) -> bool:
        """The run is complete: nothing may fire after this, and the caller prints its own JSON. False when the
        watchdog fired first (it is printing and exiting: the caller must not print)."""
        with self._lock:
            if self._fired:
                return False
            self._fired = True
            self.phase = "done"
        self._write_status(exited=True)
        return True

    # ------------------------------------------------------------------ watchdog
    def _watch(self) -> None:
        import select

        while True:
            try:
                ready, _, _ = select.select([self._rfd], [], [], self.poll_s)
            except (OSError, ValueError):
                ready = []
            if ready:
                try:
                    data = os.read(self._rfd, 64)
                except OSError:
                    data = b""
                for b in data:
                    if b == SIG_PEER_STOP:
                        self._leave(0, "stopped by rank 0")
                    elif b == signal.SIGTERM:
                        self.fire(f"terminated (SIGTERM) during {self._where()}", timeout=False)
            now = time.monotonic()
            with self._lock:
                sec, send, budget = self.current, self.section_end, self.section_budget
            if self.progress_on and now - self._last_progress >= self.PROGRESS_EVERY:
                self.progress(f"still in {self._where()}")
            if sec is not None and send is not None and now > send:
                if now >= self.end:
                    self.fire(f"bench deadline ({self.deadline_s:.0f} s) passed in section {sec}", section=sec)
                else:
                    self.fire(f"timeout after {budget:.0f} s", section=sec)
            elif now >= self.end:
                self.fire(f"bench deadline ({self.deadline_s:.0f} s) passed during {self._where()}")

    def _where(self) -> str:
        return f"section {self.current}" if self.current else f"phase {self.phase}"

    def fire(self, reason: str, section: str | None = None, timeout: bool = True) -> None:
        """Report and leave. Rank 0 emits the JSON (what finished + this error), stops its peers, and exits."""
        with self._lock:
            if self._fired:
                return
            self._fired = True
            sec = section or self.current
            key = sec or self.phase
            self.errors[key] = reason
            if sec:
                self.sections[sec] = {"s": round(time.monotonic() - self.t0, 2), "status": "timeout" if timeout
                                      else "terminated"}
        self._write_status(fired=reason)
        # a follower whose watchdog fires after the headline was measured leaves cleanly: rank 0 holds the headline
        # and reports this section's failure in its line; a non-zero exit would make torchrun (or the launcher) call
        # the whole job failed
        code = 0 if self.headline_done else 3
        if self.rank == 0:
            if self.emit is not None:
                try:
                    code = int(self.emit(dict(self.errors), f"{key}: {reason}"))
                except Exception as exc:  # noqa: BLE001 - still exit; say why on stderr
                    print(f"guard: emit failed: {type(exc).__name__}: {exc}", file=sys.stderr, flush=True)
                    code = 1
            self.stop_peers()
        self.stop_children()
        self._leave(code, reason)

    def stop_children(self, grace: float = 5.0) -> None:
        """A section that overran may have left processes of its own (a node, a pool, miners): SIGTERM the direct
        children (they stop their own trees), then SIGKILL whatever is left below this process."""
        try:
            import psutil
        except ImportError:
            return
        try:
            me = psutil.Process()
            keep = {self._tee.pid} if self._tee is not None else set()
            kids = [c for c in me.children() if c.pid not in keep]
            for c in kids:
                with contextlib.suppress(psutil.Error):
                    c.terminate()
            psutil.wait_procs(kids, timeout=grace)
            for c in me.children(recursive=True):
                if c.pid not in keep:
                    with contextlib.suppress(psutil.Error):
                        c.kill()
        except psutil.Error:
            pass

    def _leave(self, code: int, why: str) -> None:
        self.phase = f"exit:{why}"[:200]
        self._write_status(exited=True)
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:  # noqa: BLE001
            pass
        os._exit(code)

    def stop_peers(self) -> list[int]:
        """SIGUSR1 to every other rank of this job that is still running; returns the pids signalled."""
        sent = []
        if self.world <= 1:
            return sent
        for r, st in self.peer_status().items():
            pid = int(st.get("pid", 0) or 0)
            if not 0 < r < self.world or st.get("world") != self.world:
                continue
            if pid and pid != os.getpid() and not st.get("exited") and _pid_is_rank(pid, self.marker):
                try:
                    os.kill(pid, SIG_PEER_STOP)
                    sent.append(pid)
                except OSError:
                    pass
        return sent

    # ------------------------------------------------------------------ diagnosis
    def peer_status(self) -> dict[int, dict]:
        """Status files of this job's ranks (a file left by an earlier job on the same port is older than
        STALE_S before this rank's start and is ignored)."""
        out = {}
        for path in glob.glob(os.path.join(self.run_dir, "rank*.json")):
            try:
                with open(path) as f:
                    st = json.load(f)
                if float(st.get("t_start", 0.0)) >= self.t_start_wall - STALE_S:
                    out[int(st["rank"])] = st
            except (OSError, ValueError, KeyError, TypeError):
                continue
        return out

    def diagnose(self) -> dict:
        return diagnose_run_dir(self.run_dir, self.world, self.t_start_wall, self.marker)


def diagnose_run_dir(run_dir: str, world: int, t_start: float, marker: str = "bench.py") -> dict:
    """Every rank's last phase, age and liveness, the tail of its stderr, and the RCCL log tails (files older than
    STALE_S before ``t_start`` belong to an earlier job and are ignored)."""
    now = time.time()
    sts = {}
    for path in glob.glob(os.path.join(run_dir, "rank*.json")):
        try:
            with open(path) as f:
                st = json.load(f)
            if float(st.get("t_start", 0.0)) >= t_start - STALE_S:
                sts[int(st["rank"])] = st
        except (OSError, ValueError, KeyError, TypeError):
            continue
    ranks = {}
    for r in range(world):
        st = sts.get(r)
        if st is None:
            ranks[str(r)] = {"checked_in": False,
                             "stderr_tail": _tail(os.path.join(run_dir, f"rank{r}.stderr"), STDERR_TAIL) or None}
            continue
        pid = int(st.get("pid", 0) or 0)
        ranks[str(r)] = {"checked_in": True, "phase": st.get("phase"), "pid": pid,
                         "alive": bool(pid) and _pid_is_rank(pid, marker) and not st.get("exited"),
                         "status_age_s": round(now - float(st.get("t_wall", now)), 1),
                         "errors": st.get("errors") or None,
                         "stderr_tail": _tail(os.path.join(run_dir, f"rank{r}.stderr"), STDERR_TAIL) or None}
    rccl = {os.path.basename(p): _tail(p, RCCL_TAIL) for p in sorted(glob.glob(os.path.join(run_dir, "rccl.*.log")))
            if os.path.getmtime(p) >= t_start - STALE_S}
    seen = sorted(int(r) for r, v in ranks.items() if v.get("checked_in"))
    phases: dict[str, list[int]] = {}
    for r, v in ranks.items():
        phases.setdefault(v.get("phase") or "not started", []).append(int(r))
    return {"world_size": world, "ranks_checked_in": seen, "phases": phases, "ranks": ranks,
            "rccl_logs": {k: v for k, v in rccl.items() if v} or None, "run_dir": run_dir}
