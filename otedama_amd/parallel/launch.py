"""One process per GPU without torchrun: spawn N rank processes of a command.

torchrun's agent tears the whole job down when one worker dies, and the driver
runs ``bench.py --gpus N`` directly; both need a launcher of our own. The
parent never touches the GPU (counting devices with ``torch.cuda.device_count``
does not initialise HIP on this image), never ``exec``s, and hands every child
the torch.distributed env contract (RANK / LOCAL_RANK / WORLD_SIZE /
LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT). Children run as fresh
interpreters (``subprocess``), so each one initialises only its own device.

Reference analogue: the per-device worker start-up of
internal/engine/setup.go:59-77 (goroutines there, processes here: a GPU fault
that aborts one process cannot take the other GPUs with it).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Sequence

MASTER_ADDR = "127.0.0.1"  # the container hostname may not resolve
FINAL_EXIT_CODES = (0, 64, 78)  # rank 0 exit codes that end a node: clean stop, usage error, configuration error
# A rank 0 that keeps dying young (an unhandled exception, a pool that always refuses the credentials) is not
# restarted forever: after this many consecutive restarts that each lived less than QUICK_EXIT_S the node stops with
# rank 0's code, so an outer service manager sees the failure.
RANK0_MAX_QUICK_RESTARTS = 5
QUICK_EXIT_S = 60.0


def free_port() -> int:
    s = socket.socket()
    s.bind((MASTER_ADDR, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus_kfd() -> int:
    """GPUs in the KFD topology that a child may use (honours HIP/ROCR/CUDA_VISIBLE_DEVICES); 0 without a KFD
    topology. Never imports torch."""
    from otedama_amd.hal import KFD_TOPOLOGY_PATH, KFDDriver

    if not os.path.isdir(KFD_TOPOLOGY_PATH):
        return 0
    try:
        return len(KFDDriver().enumerate())
    except Exception:  # noqa: BLE001 - an unreadable topology: no GPUs
        return 0


def visible_gpus() -> int:
    """HIP devices visible to a child (honours HIP/ROCR/CUDA_VISIBLE_DEVICES) without initialising HIP here: from
    the KFD topology in sysfs (no torch import, so the supervisor stays small), else torch's device count."""
    from otedama_amd.hal import KFD_TOPOLOGY_PATH, KFDDriver

    if os.path.isdir(KFD_TOPOLOGY_PATH):
        n = len(KFDDriver().enumerate())
        if n:
            return n
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001 - no torch / no driver: no GPUs
        return 0


def rank_env(rank: int, world: int, port: int, base: dict | None = None, **extra: str) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR=MASTER_ADDR, MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL peer buffers)
    env.update({k: str(v) for k, v in extra.items()})
    return env


def _stop_all(procs: list[subprocess.Popen], grace: float = 10.0) -> None:
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    deadline = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def run_ranks(cmd: Sequence[str], world: int, port: int | None = None, env: dict | None = None,
              stdout_rank0_only: bool = True, poll: float = 0.1, deadline: float | None = None,
              on_rank0_line=None, **extra: str) -> int:
    """Run ``cmd`` as ``world`` ranks and wait. The first rank to fail stops the others; returns its exit code
    (0 when every rank succeeded). Only rank 0's stdout is kept when ``stdout_rank0_only`` (one JSON line).

    ``deadline`` (seconds): past it every rank gets SIGTERM, then SIGKILL after a grace period, and the return code
    is 124 (timeout(1)'s). ``on_rank0_line(line)``: rank 0's stdout is read through this process (and still
    forwarded to ours) so the caller can tell whether rank 0 reported before it ended."""
    import threading

    port = port or free_port()
    procs: list[subprocess.Popen] = []
    prev = {}
    readers: list[threading.Thread] = []

    def forward(sig, _frame):  # the driver's timeout / Ctrl-C reaches every rank
        _stop_all(procs, grace=5.0)
        sys.exit(128 + sig)

    def pump(stream) -> None:
        for raw in iter(stream.readline, b""):
            try:
                sys.stdout.buffer.write(raw)
                sys.stdout.flush()
            except (OSError, ValueError):
                pass
            try:
                on_rank0_line(raw.decode("utf-8", "replace"))
            except Exception:  # noqa: BLE001 - observing must never break forwarding
                pass
        stream.close()

    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            prev[sig] = signal.signal(sig, forward)
        except ValueError:  # not the main thread
            pass
    end = time.monotonic() + deadline if deadline else None
    try:
        for r in range(world):
            out = None if (r == 0 or not stdout_rank0_only) else subprocess.DEVNULL
            if r == 0 and on_rank0_line is not None:
                out = subprocess.PIPE
            procs.append(subprocess.Popen(list(cmd), env=rank_env(r, world, port, env, **extra), stdout=out))
            if out is subprocess.PIPE:
                th = threading.Thread(target=pump, args=(procs[-1].stdout,), daemon=True)
                th.start()
                readers.append(th)
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"launch: rank {r} exited with code {c}; stopping the other ranks", file=sys.stderr)
                _stop_all(procs)
                return c if c > 0 else 128 - c
            if all(c == 0 for c in codes):
                return 0
            if end is not None and time.monotonic() > end:
                print(f"launch: ranks still running after the {deadline:.0f} s deadline; stopping them",
                      file=sys.stderr)
                _stop_all(procs)
                return 124
            time.sleep(poll)
    finally:
        _stop_all(procs, grace=5.0)
        for th in readers:
            th.join(timeout=5)
        for sig, h in prev.items():
            signal.signal(sig, h)


def supervise_node(cmd: Sequence[str], world: int, port: int | None = None, env: dict | None = None,
                   respawn: bool = True, backoff_initial: float = 1.0, backoff_max: float = 64.0, log=None,
                   stop_event=None) -> int:
    """Run a fault-tolerant node: ``world`` ranks of ``cmd`` around a rendezvous store hosted HERE (this
    process is GPU-free, torch-free and outlives any rank; parallel/kvstore.py serves torch's TCPStore protocol, so
    the ranks join it with plain ``dist.TCPStore`` clients).

    A follower (rank > 0) that exits is marked ``otd/dead/<r>`` in the store (the leader re-forms the process
    group without it within one liveness check, parallel/node.py) and, with ``respawn``, restarted after a backoff
    (1 s doubling to 64 s, internal/engine/run.go:56-63) as a joiner that the leader re-admits.

    Rank 0 (the leader: pool session + job fan-out) that dies is restarted the same way, as a leader that takes the
    running node over (parallel/node.py ``NodeMinerSet._take_over``); the followers keep hashing meanwhile. Only a
    clean exit (0), a usage / configuration error (64 / 78, which a restart cannot fix) or ``respawn=False`` ends
    the node with rank 0's exit code; so does a rank 0 that died RANK0_MAX_QUICK_RESTARTS times in a row, each time
    within QUICK_EXIT_S of its start."""
    from .kvstore import StoreServer

    log = log or (lambda msg: print(f"[node] {msg}", file=sys.stderr, flush=True))
    store = StoreServer(MASTER_ADDR, port or 0)  # torch's TCPStore protocol without importing torch (~25 MiB)
    port = store.port
    procs: dict[int, subprocess.Popen] = {}
    backoff = {r: backoff_initial for r in range(world)}
    respawn_at: dict[int, float] = {}
    started: dict[int, float] = {}
    quick_exits = 0  # consecutive rank-0 exits within QUICK_EXIT_S of its start

    def spawn(r: int, join: bool) -> None:
        extra = {"OTEDAMA_STORE_HOSTED": "1"}
        if join:
            extra["OTEDAMA_NODE_JOIN"] = "1"
        procs[r] = subprocess.Popen(list(cmd), env=rank_env(r, world, port, env, **extra))
        started[r] = time.monotonic()

    prev = {}
    stopping = []

    def forward(sig, _frame):  # a clean stop: every rank gets SIGTERM and shuts down like `otedama run` does
        stopping.append(sig)

    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            prev[sig] = signal.signal(sig, forward)
        except ValueError:
            pass
    try:
        for r in range(world):
            spawn(r, join=False)
        while True:
            if stopping:
                log(f"signal {stopping[0]}: stopping the node")
                store.set("otd/stopping", "1")  # the leader then takes a follower's exit for the shutdown it is
                _stop_all(list(procs.values()), grace=30.0)
                rc0 = procs[0].returncode if 0 in procs else None
                return 0 if rc0 in (0, -signal.SIGTERM, 128 + signal.SIGTERM) else (rc0 or 0)
            if stop_event is not None and stop_event.is_set():
                return 0
            rc0 = procs[0].poll() if 0 in procs else None
            if rc0 is not None and (not respawn or rc0 in FINAL_EXIT_CODES):
                log(f"rank 0 exited with code {rc0}; stopping the node")
                return rc0
            if rc0 is not None:
                lived = time.monotonic() - started.get(0, time.monotonic())
                quick_exits = quick_exits + 1 if lived < QUICK_EXIT_S else 0
                if quick_exits >= RANK0_MAX_QUICK_RESTARTS:
                    log(f"rank 0 exited with code {rc0} after {lived:.0f}s, {quick_exits} times in a row within "
                        f"{QUICK_EXIT_S:.0f}s of starting; stopping the node")
                    return rc0
            now = time.monotonic()
            for r in range(world):
                p = procs.get(r)
                if p is not None and p.poll() is not None:
                    log(f"rank {r} exited with code {p.returncode}" + (
                        "; the followers keep hashing their last job until it is back" if r == 0 else ""))
                    store.set(f"otd/dead/{r}", str(p.returncode))
                    del procs[r]
                    if now - started.get(r, now) > 60.0:
                        backoff[r] = backoff_initial  # it had been healthy: start the backoff over
                    if respawn:
                        respawn_at[r] = now + backoff[r]
                        log(f"rank {r}: restarting in {backoff[r]:.0f}s")
                        backoff[r] = min(backoff[r] * 2, backoff_max)
                if r not in procs and r in respawn_at and now >= respawn_at[r]:
                    del respawn_at[r]
                    try:
                        store.delete_key(f"otd/dead/{r}")
                    except Exception:  # noqa: BLE001
                        pass
                    spawn(r, join=True)
            time.sleep(0.05)
    finally:
        _stop_all(list(procs.values()), grace=10.0)
        store.close()
        for sig, h in prev.items():
            signal.signal(sig, h)
