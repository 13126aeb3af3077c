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

from otedama_amd.cli.main import EXIT_OK, EXIT_USAGE

HELP = """Usage: otedama node --gpus N [--no-respawn] [run flags...]

Run N ranks of `otedama run` (one per GPU, RCCL collectives between them) under a supervisor that
survives the loss of any rank but rank 0 and restarts lost ranks. Every other flag is passed to
`otedama run` on every rank.
"""


def cmd_node(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
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
