"""Pre-flight of the bench's data plane: can RCCL form a group of every rank here, within a deadline?

The driver gets one 8-GPU run of ``bench.py --gpus 8``, and it is the first time RCCL runs at world size > 1 (the
one-GPU box cannot: RCCL refuses two ranks on one device). If RCCL cannot form the group or hangs in it, the run
must still measure its headline. The headline is the kernels' hash rate; the collectives only gather hits and
counters. So before the bench creates its process group, every rank starts a child process that forms a
torch.distributed RCCL group of all ranks (the same library the bench then uses) and runs one all_reduce. The
child runs under a deadline and is SIGKILLed when it passes, so a hang in RCCL costs the deadline and nothing else.
Every rank publishes its child's verdict in the rendezvous store and reads the others'. When all of them succeeded,
the bench runs over RCCL. When any failed, every rank runs over gloo together: host collectives, the kernels still
on each rank's own GPU. The JSON reports which (``preflight.data_plane``). The same node on gloo is what
``OTEDAMA_DIST_BACKEND=gloo`` rehearses on one GPU (profiles/r5/m_torchrun2).

Reference: its engine never waits on I/O without a deadline (internal/engine/run.go:1251).

Child usage (internal): python -m otedama_amd.parallel.rccl_probe   (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* and
OTEDAMA_PROBE_PREFIX in the environment; OTEDAMA_PROBE_BACKEND=gloo exercises the mechanics on CPU hosts).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

PROBE_TIMEOUT_S = 60.0
# How long a rank at the probe waits for its peers to reach it before starting its child anyway. The ranks' cold
# `import torch` on a fresh node runs at each rank's own pace (up to a minute or two); a child started before its
# peers arrive would spend its deadline on their import, and a skew past it would read as an RCCL failure.
ARRIVE_TIMEOUT_S = 120.0


def _prefix() -> str:
    run = "".join(c if c.isalnum() else "_" for c in os.environ.get("TORCHELASTIC_RUN_ID", "") or "local")[:40]
    return f"otd-probe-{run}"


def _why(stderr: str) -> str:
    """The informative line of a failed child's stderr: the last error-looking line that is not a warning (torch
    prints a destroy_process_group warning at exit after the real error), else the last line."""
    lines = [ln.strip() for ln in stderr.strip().splitlines() if ln.strip()]
    for ln in reversed(lines):
        if "Warning" in ln or "warn(" in ln:
            continue
        if any(k in ln for k in ("Error", "error", "Duplicate", "NCCL", "nccl", "Exception", "failure")):
            return ln[:300]
    return (lines[-1] if lines else "no output")[:300]


def run_probe(store, rank: int, world: int, timeout: float | None = None, fault: str | None = None,
              arrive_timeout: float = ARRIVE_TIMEOUT_S) -> dict:
    """Run this rank's probe child, publish its verdict, and return every rank's ({"ok", "ranks", "seconds",
    "arrive_s"}). The child starts once every rank has reached the probe (or after ``arrive_timeout``), so its
    deadline measures RCCL and not the ranks' start-up skew.
    ``fault="fail"`` makes this rank's child fail (tests); ``"hang"`` makes it hang past the deadline.
    ``timeout``: default OTEDAMA_PROBE_TIMEOUT, else PROBE_TIMEOUT_S."""
    if timeout is None:
        timeout = float(os.environ.get("OTEDAMA_PROBE_TIMEOUT", PROBE_TIMEOUT_S))
    prefix = _prefix()
    t_arrive = time.monotonic()
    store.set(f"{prefix}/arrive/{rank}", "1")
    arrived = [f"{prefix}/arrive/{r}" for r in range(world)]
    end = t_arrive + arrive_timeout
    while not store.check(arrived) and time.monotonic() < end:
        time.sleep(0.05)
    t0 = time.monotonic()
    env = dict(os.environ, OTEDAMA_PROBE_PREFIX=prefix)
    if fault:
        env["OTEDAMA_PROBE_FAULT"] = fault
    reason = ""
    proc = subprocess.Popen([sys.executable, "-m", "otedama_amd.parallel.rccl_probe"], env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        out, err = proc.communicate(timeout=timeout)
        ok = proc.returncode == 0 and "probe ok" in out
        if not ok:
            reason = f"exit code {proc.returncode}: " + _why(err)
    except subprocess.TimeoutExpired:
        proc.kill()
        proc.communicate()
        ok, reason = False, f"no group within {timeout:.0f} s (killed)"
    mine = {"ok": ok, "s": round(time.monotonic() - t0, 2), **({"reason": reason} if reason else {})}
    store.set(f"{prefix}/result/{rank}", json.dumps(mine))
    ranks: dict = {}
    end = time.monotonic() + timeout + 30.0
    for r in range(world):
        key = f"{prefix}/result/{r}"
        while not store.check([key]) and time.monotonic() < end:
            time.sleep(0.05)
        ranks[str(r)] = json.loads(store.get(key)) if store.check([key]) else {"ok": False, "reason": "no verdict"}
    return {"ok": all(v.get("ok") for v in ranks.values()), "ranks": ranks, "seconds": round(time.monotonic() - t0, 2),
            "arrive_s": round(t0 - t_arrive, 2)}


def _child() -> int:
    import datetime

    fault = os.environ.get("OTEDAMA_PROBE_FAULT", "")
    if fault == "fail":
        print("probe: injected failure", file=sys.stderr)
        return 3
    if fault == "hang":
        time.sleep(3600)
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = os.environ.get("OTEDAMA_PROBE_BACKEND", "nccl")
    store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                          is_master=False, timeout=datetime.timedelta(seconds=PROBE_TIMEOUT_S),
                          wait_for_workers=False)
    kw = {}
    dev = torch.device("cpu")
    if backend == "nccl":
        # one rank per GPU on a node (local < device count); ranks sharing one GPU (a rehearsal) land on the same
        # device, where RCCL refuses the group: the real failure the fallback exists for
        dev = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}")
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
    dist.init_process_group(backend, rank=rank, world_size=world,
                            store=dist.PrefixStore(os.environ["OTEDAMA_PROBE_PREFIX"] + "/pg", store),
                            timeout=datetime.timedelta(seconds=PROBE_TIMEOUT_S), **kw)
    t = torch.ones(4, device=dev)
    dist.all_reduce(t)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if int(t[0].item()) != world:
        print(f"probe: all_reduce summed {t[0].item()}, expected {world}", file=sys.stderr)
        return 4
    # every rank's collective finished before any of them leaves (a peer still finishing its part must not lose a
    # partner), then no teardown: the process exit releases the communicator and the GPU context
    prefix = os.environ["OTEDAMA_PROBE_PREFIX"]
    store.set(f"{prefix}/done/{rank}", "1")
    store.wait([f"{prefix}/done/{r}" for r in range(world)], datetime.timedelta(seconds=30))
    print("probe ok", flush=True)
    os._exit(0)


if __name__ == "__main__":
    sys.exit(_child())
