"""``otedama node`` — a fault-tolerant multi-GPU node: one ``otedama run`` rank per GPU under a GPU-free supervisor.

The supervisor (otedama_amd/parallel/launch.py ``supervise_node``) hosts the rendezvous store, starts rank r on
GPU r (torch.distributed over RCCL; rank 0 holds the pool session), marks a follower that exits as dead so the
leader re-forms the group without it, and restarts it after a backoff as a joiner (parallel/node.py). Unlike
torchrun, a dead follower does not tear the node down.

Usage: otedama node --gpus N [run flags...]
"""
from __future__ import annotations

import os
import sys
from typing import TextIO

from otedama_amd.cli.main import EXIT_OK, EXIT_RUNTIME, EXIT_USAGE

HELP = """Usage: otedama node --gpus N [--no-respawn] [run flags...]
       otedama node status [--http-addr HOST:PORT] [--json]

Run N ranks of `otedama run` (one per GPU, RCCL collectives between them) under a supervisor that
survives the loss of any rank but rank 0 and restarts lost ranks. Every other flag is passed to
`otedama run` on every rank.

`otedama node status` asks a running node's leader (rank 0's --http-addr, default
$OTEDAMA_HTTP_ADDR or 127.0.0.1:8080) for its view: membership, process-group generation,
data plane, and each rank's rate, heartbeat age and pending shares.
"""


def _fmt_rate(h: float) -> str:
    for unit, div in (("TH/s", 1e12), ("GH/s", 1e9), ("MH/s", 1e6), ("kH/s", 1e3)):
        if h >= div:
            return f"{h / div:.2f} {unit}"
    return f"{h:.0f} H/s"


def render_status(st: dict) -> str:
    """The table `otedama node status` prints for GET /api/v1/node."""
    lines = [f"node: {st.get('world', 1)} ranks over {st.get('backend', 'none')}, generation {st.get('generation', 0)}"
             f", leader incarnation {st.get('leader_incarnation', 1)}",
             f"members {st.get('members', [0])}; lost {st.get('lost_ranks', []) or 'none'}; re-forms "
             f"{st.get('reforms', 0)}; node ops p50 {st.get('op_p50_ms', 0.0):.2f} ms / p99 "
             f"{st.get('op_p99_ms', 0.0):.2f} ms",
             f"remote shares: {st.get('share_previews', 0)} from previews, {st.get('share_gathered_first', 0)} first "
             f"by R2, {st.get('remote_stale', 0)} stale",
             f"{'rank':<8}{'rate':>14}{'heartbeat':>12}{'gen':>6}{'pending':>9}{'collectives':>13}"]
    total = 0.0
    for name in sorted(st.get("ranks", {}), key=lambda k: int(k[4:]) if k[4:].isdigit() else 1 << 30):
        r = st["ranks"][name]
        total += float(r.get("hashrate", 0.0) or 0.0)
        hb = "leader" if r.get("leader") else f"{r.get('heartbeat_age_s', 0.0):.1f} s"
        mark = "" if r.get("leader") or r.get("member", True) else " (out)"
        lines.append(f"{name + mark:<8}{_fmt_rate(float(r.get('hashrate', 0.0) or 0.0)):>14}{hb:>12}"
                     f"{'' if r.get('generation') is None else r['generation']:>6}{r.get('pending_shares', ''):>9}"
                     f"{r.get('collectives', ''):>13}")
    lines.append(f"{'total':<8}{_fmt_rate(total):>14}")
    return "\n".join(lines) + "\n"


def cmd_node_status(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    import json
    import urllib.error
    import urllib.request

    addr, as_json = os.environ.get("OTEDAMA_HTTP_ADDR") or "127.0.0.1:8080", False
    it = iter(args)
    for a in it:
        if a in ("-h", "--help"):
            stdout.write(HELP)
            return EXIT_OK
        if a in ("--http-addr", "-http-addr"):
            addr = next(it, addr)
        elif a.startswith("--http-addr="):
            addr = a.split("=", 1)[1]
        elif a == "--json":
            as_json = True
        else:
            stderr.write(f"otedama node status: unknown flag {a}\n" + HELP)
            return EXIT_USAGE
    try:
        with urllib.request.urlopen(f"http://{addr}/api/v1/node", timeout=5) as r:
            st = json.loads(r.read())
    except (urllib.error.URLError, OSError, ValueError) as exc:
        stderr.write(f"otedama node status: no node answering at {addr} ({exc})\n")
        return EXIT_RUNTIME
    stdout.write(json.dumps(st, indent=2) + "\n" if as_json else render_status(st))
    return EXIT_OK


def cmd_node(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    if args and args[0] == "status":
        return cmd_node_status(args[1:], stdout, stderr)
    gpus, respawn, rest = 0, True, []
    it = iter(args)
    for a in it:
        if a in ("-h", "--help", "-help"):
            stdout.write(HELP)
            return EXIT_OK
        if a in ("--gpus", "-gpus"):
            gpus = int(next(it, "0") or 0)
        elif a.startswith("--gpus=") or a.startswith("-gpus="):
            gpus = int(a.split("=", 1)[1] or 0)
        elif a == "--no-respawn":
            respawn = False
        else:
            rest.append(a)
    if gpus < 1:
        stderr.write("otedama node: --gpus N (N >= 1) is required\n" + HELP)
        return EXIT_USAGE
    from otedama_amd.parallel.launch import supervise_node, visible_gpus

    from otedama_amd.parallel.rcclcomm import cpu_standin

    if os.environ.get("OTEDAMA_DIST_BACKEND") != "gloo" and not cpu_standin():
        n = visible_gpus()
        if n < gpus:
            stderr.write(f"otedama node: --gpus {gpus} needs {gpus} visible GPUs, this host has {n}\n")
            return EXIT_USAGE
    cmd = [sys.executable, "-m", "otedama_amd", "run", *rest]
    return supervise_node(cmd, gpus, respawn=respawn, log=lambda m: stderr.write(f"[node] {m}\n"))
