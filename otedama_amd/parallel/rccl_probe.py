"""Pre-flight of the bench's data plane: can the native RCCL module form a group of every rank here, within a deadline?

The driver gets one 8-GPU run of ``bench.py --gpus 8``, and it is the first time RCCL runs at world size > 1 (the
one-GPU box cannot: RCCL refuses two ranks on one device). If RCCL cannot form the group or hangs in it, the run
must still measure its headline. The headline is the kernels' hash rate; the collectives only gather hits and
counters. So before the bench forms its communicator, every rank starts a child process that forms a group of all
ranks with the SAME implementation the bench and the node then use, ``otedama_amd._rccl`` (``RcclComm``: the unique
id through the rendezvous store, one all_reduce), and no torch in the child. The child runs under a deadline and is
SIGKILLed when it passes, so a hang in RCCL costs the deadline and nothing else.

Every rank publishes its child's verdict in the store. Rank 0 collects them and publishes ONE decision; every rank
reads that decision, so all ranks pick the same data plane (ranks deciding from the verdicts each of them
happened to read could split between RCCL and gloo). When every child succeeded, the bench runs over the native
module ("rccl-native"); otherwise every rank runs over gloo together: host collectives, the kernels still on each
rank's own GPU. The JSON reports which (``preflight.data_plane``).

Deadlines: ``run_probe(budget=...)`` derives the arrival wait, the child deadline and the verdict wait from the time
the caller has left (bench.py passes what remains of its pre-flight section, minus a reserve for the gloo fallback),
so the probe's worst case (skewed arrival + a hung child) ends inside the section.

Reference: its engine never waits on I/O without a deadline (internal/engine/run.go:1251).

Child usage (internal): python -m otedama_amd.parallel.rccl_probe   (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* and
OTEDAMA_PROBE_PREFIX in the environment; OTEDAMA_RCCL_MODULE=loopback_rccl runs the same protocol on CPU hosts).
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
    return f"otd-probe-{run}-{os.environ.get('MASTER_PORT', '0')}"


def _why(stderr: str) -> str:
    """The informative line of a failed child's stderr: the last error-looking line that is not a warning, else the
    last line."""
    lines = [ln.strip() for ln in stderr.strip().splitlines() if ln.strip()]
    for ln in reversed(lines):
        if "Warning" in ln or "warn(" in ln:
            continue
        if any(k in ln for k in ("Error", "error", "Duplicate", "NCCL", "nccl", "Exception", "failure")):
            return ln[:300]
    return (lines[-1] if lines else "no output")[:300]


def plan(budget: float | None, timeout: float, arrive_timeout: float) -> tuple[float, float, float]:
    """(arrive wait, child deadline, verdict wait) within ``budget`` seconds: the three add up to at most the budget,
    the child keeps at least 10 s, and without a budget the defaults stand."""
    verdict = timeout + 30.0
    if budget is None:
        return arrive_timeout, timeout, verdict
    budget = max(budget, 20.0)
    timeout = max(10.0, min(timeout, 0.4 * budget))
    arrive_timeout = max(1.0, min(arrive_timeout, budget - timeout - 10.0, 0.4 * budget))
    verdict = max(5.0, budget - arrive_timeout - timeout)
    return arrive_timeout, timeout, verdict


def run_probe(store, rank: int, world: int, timeout: float | None = None, fault: str | None = None,
              arrive_timeout: float = ARRIVE_TIMEOUT_S, budget: float | None = None) -> dict:
    """Run this rank's probe child, publish its verdict, and return the decision every rank shares ({"ok", "ranks",
    "seconds", "arrive_s", "impl"}). The child starts once every rank has reached the probe (or after the arrival
    wait), so its deadline measures RCCL and not the ranks' start-up skew.
    ``fault="fail"`` makes this rank's child fail (tests); ``"hang"`` makes it hang past the deadline.
    ``timeout``: default OTEDAMA_PROBE_TIMEOUT, else PROBE_TIMEOUT_S. ``budget``: seconds the whole probe may take."""
    if timeout is None:
        timeout = float(os.environ.get("OTEDAMA_PROBE_TIMEOUT", PROBE_TIMEOUT_S))
    arrive_timeout, timeout, verdict_wait = plan(budget, timeout, arrive_timeout)
    prefix = _prefix()
    t_arrive = time.monotonic()
    store.set(f"{prefix}/arrive/{rank}", "1")
    arrived = [f"{prefix}/arrive/{r}" for r in range(world)]
    end = t_arrive + arrive_timeout
    while not store.check(arrived) and time.monotonic() < end:
        time.sleep(0.05)
    t0 = time.monotonic()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # the package's parent
    env = dict(os.environ, OTEDAMA_PROBE_PREFIX=prefix, OTEDAMA_PROBE_TIMEOUT=str(timeout),
               PYTHONPATH=os.pathsep.join(p for p in (root, os.environ.get("PYTHONPATH", "")) if p))
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
    decision_key = f"{prefix}/decision"
    if rank == 0:
        ranks: dict = {}
        end = time.monotonic() + verdict_wait
        for r in range(world):
            key = f"{prefix}/result/{r}"
            while not store.check([key]) and time.monotonic() < end:
                time.sleep(0.05)
            ranks[str(r)] = json.loads(store.get(key)) if store.check([key]) else {"ok": False, "reason": "no verdict"}
        decision = {"ok": all(v.get("ok") for v in ranks.values()), "ranks": ranks}
        store.set(decision_key, json.dumps(decision))
    else:
        # rank 0 decides within verdict_wait of its own child's end; wait past that (a rank 0 that never decides is
        # dead, and the run fails with it anyway)
        end = time.monotonic() + verdict_wait + 10.0
        while not store.check([decision_key]) and time.monotonic() < end:
            time.sleep(0.05)
        decision = json.loads(store.get(decision_key)) if store.check([decision_key]) else \
            {"ok": False, "ranks": {str(rank): mine}, "reason": "no decision from rank 0"}
    return {**decision, "impl": "rccl-native" if decision["ok"] else "gloo",
            "seconds": round(time.monotonic() - t0, 2), "arrive_s": round(t0 - t_arrive, 2),
            "deadlines_s": [round(arrive_timeout, 1), round(timeout, 1), round(verdict_wait, 1)]}


def _child() -> int:
    fault = os.environ.get("OTEDAMA_PROBE_FAULT", "")
    if fault == "fail":
        print("probe: injected failure", file=sys.stderr)
        return 3
    if fault == "hang":
        time.sleep(3600)
    import numpy as np

    from otedama_amd.parallel.kvclient import StoreClient
    from otedama_amd.parallel.launch import visible_gpus_kfd
    from otedama_amd.parallel.rcclcomm import _wait_get, rccl_module

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    timeout = float(os.environ.get("OTEDAMA_PROBE_TIMEOUT", PROBE_TIMEOUT_S))
    prefix = os.environ["OTEDAMA_PROBE_PREFIX"]
    store = StoreClient(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), timeout=timeout)
    mod = rccl_module()
    key = f"{prefix}/uid"
    if rank == 0:
        store.set(key, mod.unique_id())
    uid = _wait_get(store, key, timeout)
    # one rank per GPU on a node (local < device count); ranks sharing one GPU (a rehearsal) land on the same device,
    # where RCCL refuses the group: the real failure the fallback exists for
    device = local % max(1, visible_gpus_kfd())
    rc = mod.RcclComm(device, world, rank, uid, timeout)
    got = np.frombuffer(rc.all_reduce(np.ones(1, dtype=np.int64).tobytes(), "i64", "sum", timeout), dtype=np.int64)
    if int(got[0]) != world:
        print(f"probe: all_reduce summed {int(got[0])}, expected {world}", file=sys.stderr)
        return 4
    # every rank's collective finished before any of them leaves (a peer still finishing its part must not lose a
    # partner), then no teardown: the process exit releases the communicator and the GPU context
    store.set(f"{prefix}/done/{rank}", "1")
    for r in range(world):
        _wait_get(store, f"{prefix}/done/{r}", 30.0)
    print("probe ok", flush=True)
    os._exit(0)


if __name__ == "__main__":
    sys.exit(_child())
