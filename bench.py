#!/usr/bin/env python3
"""Headline benchmark: whole-node SHA-256d hashes/sec (+ scrypt, X11) on N MI355X.

BASELINE.json metric: "hashes/sec (whole node) SHA-256d + scrypt at 1/2/4/8
MI355X; p50 share latency". Reference headline: ~75 MH/s SHA-256d on a whole
Ryzen 9 7950X (BENCHMARKS.md:46, CPU only).

Ranks: one process per GPU. ``python bench.py --gpus N`` with no torchrun env
spawns the N ranks itself (otedama_amd/parallel/launch.py: fresh interpreters,
the parent never touches the GPU) and exits non-zero when fewer than N GPUs
are visible; under torchrun (WORLD_SIZE set) ``--gpus`` must equal WORLD_SIZE.

Every run reports (otedama_amd/parallel/guard.py). Each rank runs its sections
under deadlines watched by a thread that never waits on the main thread:
  preflight  rendezvous + one tiny all_reduce (the first RCCL traffic) under
             --preflight-timeout; on failure rank 0 prints an error JSON with
             the ranks that checked in, each rank's phase, the tail of its
             stderr and of its RCCL log (NCCL_DEBUG=WARN), and exits non-zero;
  sha256d    the headline (below);
  single, scrypt, x11, miner   all ranks; cpu, latency, node, pool   rank 0.
A section that overruns its budget (or the run's --deadline) is recorded as
{"error": "timeout after X s"} and the JSON is printed with everything measured
so far; a SIGTERM (torchrun tearing the job down, the driver's timeout) makes
rank 0 print it too. The ``summary`` key comes LAST so a tail of the output
always carries every headline.

One timed step on each rank =
  R1  control broadcast from rank 0 when the variant group changes (the job
      blob itself went out once, before timing),
  K1  SHA-256d search over this rank's next 128 BIP320 header variants (two per
      lane of otd_sha256d_search_vn<2,0>, fixed midstate per variant, variants
      striped across ranks) x 2^28 nonces; 16 consecutive steps tile the full
      2^32 nonce space of each variant (--sha-chains 1: 64 variants x 2^29;
      --sha-kernel k: K variants x 2^32),
  R2  all_gather of every rank's on-device hit slots, on the comm stream and
      overlapped with the next step's kernel (double-buffered slots),
then R3 (all_reduce of the hash counters) once after the last step.
Data: synthetic 80-byte block headers (random prev-hash / merkle root), share
target = difficulty 1. Every hit of the timed region is de-duplicated by
(header variant, nonce), re-verified on the CPU, and compared with the Poisson
expectation (z-score). Weak scaling: per-GPU work is fixed as N grows.

Then BASELINE config 2 verbatim (one fixed midstate, full 2^32 nonces, the
single-header kernel), scrypt(1024,1,1) (HBM-resident scratchpads; hits re-
verified with hashlib.scrypt), X11 (nonce ranges partitioned across ranks; hits
re-verified with the C++ chain), scrypt and X11 through the production miner,
BASELINE config 1 (the CPU miner), the share-latency and job-switch probes, the
production node (``otedama node --gpus N``) per algorithm with its node-wide job
switch, and BASELINE config 5 (mixed pool, vardiff, steady state).

``--cpu-rehearsal`` runs the same rank/launcher/collective code with gloo and
the native CPU scanner in place of the kernels (tests/test_bench_launcher.py);
its JSON says so in ``data`` and ``rehearsal``.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import json
import math
import os
import sys
import threading
import time

BASELINE_HPS = 75e6  # BENCHMARKS.md:46 (whole 7950X, SHA-256d)
METRIC = "hashes/sec (whole node) SHA-256d + scrypt at 1/2/4/8 MI355X; p50 share latency"
DEFAULT_DEADLINE_S = 500.0  # the driver's run limit is 600 s: report well inside it


def synthetic_job(seed: int = 1) -> dict:
    from otedama_amd.models.header import DIFF1_TARGET_INT, int_to_hash

    h = hashlib.sha256(f"otedama-bench-{seed}".encode()).digest()
    prev = hashlib.sha256(h).digest()
    header = (0x20000000).to_bytes(4, "little") + prev + h + (1_700_000_000).to_bytes(4, "little") \
        + (0x1703A30C).to_bytes(4, "little") + bytes(4)
    return {
        "header": header,
        "target": int_to_hash(DIFF1_TARGET_INT),
        "epoch": 1,
        "job_id": "bench",
        "version_mask": 0x1FFFE000,  # BIP320 version rolling: 2^16 variants
        "ntime_roll": 0,
    }


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--grid", type=int, default=0, help="SHA-256d blocks (0 = CUs x resident blocks)")
    ap.add_argument("--sha-kernel", choices=("v", "k"), default="v",
                    help="v: 64 x --sha-chains version variants per wave, block-2 schedule on the scalar unit (default); "
                         "k: --sha-variants variants per lane")
    ap.add_argument("--sha-chains", type=int, choices=(1, 2), default=2,
                    help="v kernel: variants per lane (2: 128 variants per wave-group, 4 waves/SIMD; 1: 64, 8 waves)")
    ap.add_argument("--sha-variants", type=int, default=8,
                    help="k kernel: BIP320 version variants per launch sharing the block-2 schedule (1 = single midstate)")
    ap.add_argument("--single-midstate-headers", type=int, default=2,
                    help="BASELINE config 2 pass: headers x full 2^32 nonces each (0 = skip)")
    ap.add_argument("--scrypt-steps", type=int, default=-1, help="-1 = same as --steps; 0 = skip")
    ap.add_argument("--scrypt-gap", type=int, default=1)
    ap.add_argument("--scrypt-kernel", choices=("coop", "lane"), default="coop")
    ap.add_argument("--x11-steps", type=int, default=-1, help="-1 = same as --steps; 0 = skip")
    ap.add_argument("--miner-seconds", type=float, default=-1.0,
                    help="scrypt / X11 through the production GpuMiner: recorded seconds each (-1 = 8 on GPUs; 0 = skip)")
    ap.add_argument("--comm-ops", type=int, default=200,
                    help="comm section: ops of each of R1 / R2 / R3 / R2_dev per phase (0 = skip the section)")
    ap.add_argument("--comm-hz", type=float, default=100.0, help="comm section: op cadence")
    ap.add_argument("--comm-load", default="sha256d,scrypt",
                    help="comm section: algorithms every rank mines while the ops run (after the idle phase)")
    ap.add_argument("--comm-busbw-mib", type=int, default=256, help="comm section: all_gather size for the bus bandwidth")
    ap.add_argument("--seed", type=int, default=1,
                    help="synthetic header seed: the hit count of a seed is one Poisson draw, repeated on every run")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--node-seconds", type=float, default=-1.0,
                    help="production node section (otedama node --gpus N + local pool): recorded seconds per "
                         "algorithm (-1 = 8 on GPUs, 0 in the CPU rehearsal; 0 = skip)")
    ap.add_argument("--node-warmup", type=float, default=3.0)
    ap.add_argument("--node-algorithms", default="sha256d,x11,scrypt",
                    help="algorithms the node section runs, each against a pool of its own (BASELINE config 4: x11)")
    ap.add_argument("--node-switches", type=int, default=8,
                    help="forced new blocks (SetNewPrevHash) per node run for the node-wide job switch (0 = none)")
    ap.add_argument("--pool-seconds", type=float, default=-1.0,
                    help="BASELINE config 5 (mixed SHA-256d + scrypt pool, vardiff on): recorded seconds after every "
                         "worker settled (-1 = 45 on GPUs, 0 in the CPU rehearsal; 0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0,
                    help="BASELINE config 1 (native CPU miner, single thread and all cores): seconds each (0 = skip)")
    ap.add_argument("--deadline", type=float, default=DEFAULT_DEADLINE_S,
                    help="seconds from start by which rank 0 prints its JSON, whatever is still running")
    ap.add_argument("--preflight-timeout", type=float, default=240.0,
                    help="seconds from start for the rendezvous and the first collective (cold `import torch` "
                         "included)")
    ap.add_argument("--section-timeouts", default="",
                    help="override section budgets, e.g. node=60,pool=90 (seconds)")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="gloo + native CPU scanner instead of the GPU kernels (launcher / collective tests)")
    ap.add_argument("--cpu-nonces", type=int, default=1 << 12, help="rehearsal: nonces per variant per step")
    return ap.parse_args(argv)


# The benchmark is not the fault-tolerant node: a rank that is slow to start (a cold first `import torch` on a fresh
# node can take a minute) or busy re-verifying hits must not trip the node's 30 s collective bound. Set before
# otedama_amd.parallel is imported (it reads the bound at import); spawned ranks inherit it. The rank guard's section
# deadlines (parallel/guard.py) are what bounds a hang.
BENCH_PG_TIMEOUT_S = "600"


def main(argv=None) -> int:
    os.environ.setdefault("OTEDAMA_PG_TIMEOUT", BENCH_PG_TIMEOUT_S)
    args = parse_args(argv)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return launch(args, sys.argv[1:] if argv is None else list(argv))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} (torchrun "
              "--nproc-per-node must equal --gpus)", file=sys.stderr)
        return 2
    return run_rank(args)


def launch(args, argv: list[str]) -> int:
    """No torchrun env and N > 1: spawn the N ranks here (never exec; this process stays GPU-free). The launcher
    has a deadline of its own past the ranks' (SIGTERM, then SIGKILL) and prints an error JSON itself when rank 0
    never printed one (e.g. it was killed)."""
    import shutil

    from otedama_amd.parallel.guard import diagnose_run_dir, run_dir_for
    from otedama_amd.parallel.launch import free_port, run_ranks, visible_gpus

    if not args.cpu_rehearsal and os.environ.get("OTEDAMA_DIST_BACKEND") != "gloo":
        n = visible_gpus()
        if n < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this host has {n}; "
                  "refusing to report a smaller node as N GPUs", file=sys.stderr)
            return 2
    port = free_port()
    run_dir = run_dir_for({"MASTER_PORT": str(port)})
    shutil.rmtree(run_dir, ignore_errors=True)
    os.makedirs(run_dir, exist_ok=True)
    seen = []
    t0 = time.time()
    rc = run_ranks([sys.executable, os.path.abspath(__file__), *argv], args.gpus, port=port,
                   deadline=args.deadline + 60.0, on_rank0_line=lambda ln: seen.append(ln.startswith('{"metric"')))
    if not any(seen):
        out = error_output(args, args.gpus, f"rank 0 printed no result (launcher exit code {rc})",
                           {"launcher": f"exit code {rc}"}, diagnose_run_dir(run_dir, args.gpus, t0))
        print(finalize(out), flush=True)
        return rc or 1
    return rc


# --------------------------------------------------------------------------- search back-ends
class _CpuSearch:
    """Rehearsal stand-in for the version-parallel kernel: the native CPU scanner over K variants."""

    def __init__(self, native, k: int, cap: int = 1024):
        import torch

        self.N, self.k, self.cap, self.grid = native, k, cap, 0
        self.out = torch.zeros(1 + 2 * cap, dtype=torch.int32)

    def prepare(self, hdrs, target):
        return (list(hdrs), target)

    def launch(self, prep, base, count, out=None):
        hdrs, target = prep
        out = self.out if out is None else out
        pairs = []
        for vi, h in enumerate(hdrs):
            pairs += [(n, vi) for n in self.N.cpu_scan_sha256d(h, target, base & 0xFFFFFFFF, count)]
        out.zero_()
        out[0] = len(pairs)
        for i, (n, vi) in enumerate(pairs[: self.cap]):
            out[1 + 2 * i] = n - (1 << 32) if n >= 1 << 31 else n
            out[2 + 2 * i] = vi
        return out


def _sha_name(args, K: int, use_v: bool) -> str:
    if args.cpu_rehearsal:
        return "cpu_scan_sha256d (rehearsal)"
    if use_v:
        return "otd_sha256d_search_vn<2,0>" if args.sha_chains == 2 else "otd_sha256d_search_v<8>"
    return f"otd_sha256d_search_k<{K}>" if K > 1 else "otd_sha256d_search"


def _poisson(found: int, hashes: int, target_int: int) -> tuple[float, float]:
    exp = hashes * (target_int + 1) / 2.0 ** 256
    return exp, ((found - exp) / math.sqrt(exp) if exp > 0 else 0.0)


def _r(x, digits: int = 4):
    """Compact number for the summary (4 significant digits)."""
    if x is None or isinstance(x, bool) or not isinstance(x, (int, float)):
        return x
    if x == 0 or not math.isfinite(x):
        return x
    return float(f"{x:.{digits}g}")


def _base_config(args, world: int = 1) -> dict:
    return {"model": "sha256d", "global_batch": None, "seq_len": 80, "parallelism": f"dp{world}"}


def _short_errors(errors: dict | None, n: int = 160) -> dict | None:
    return {str(k)[:40]: str(v)[:n] for k, v in errors.items()} if errors else None


@contextlib.contextmanager
def _stdout_to_stderr():
    """fd 1 points at fd 2 inside: C-level prints (RCCL's init banner) stay off the stdout whose last line is the
    driver's."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        try:
            sys.stdout.flush()
        finally:
            os.dup2(saved, 1)
            os.close(saved)


def _link_counts(links) -> dict | None:
    out: dict = {}
    for ln in links or []:
        out[str(ln.get("type"))] = out.get(str(ln.get("type")), 0) + 1
    return out or None


def _data_plane_note(dp: dict) -> str | None:
    probe = dp.get("probe") or {}
    if probe and not probe.get("ok"):
        bad = [(r, v) for r, v in sorted((probe.get("ranks") or {}).items()) if not v.get("ok")]
        if bad:
            return f"probe: rank {bad[0][0]}: {bad[0][1].get('reason', '?')}"[:160]
        return f"probe: {probe.get('reason', 'failed')}"[:160]
    if dp.get("native_error"):
        return str(dp["native_error"])[:160]
    return None


def error_output(args, world: int, error: str, errors: dict, diagnosis: dict | None) -> dict:
    """The result of a run that has no headline (the pre-flight failed, or rank 0 never reported). The diagnosis
    (every rank's stderr and RCCL log tail) stays in the detail file; the line carries the phases only."""
    phases = {k[:48]: v for k, v in ((diagnosis or {}).get("phases") or {}).items()}
    return {
        "metric": METRIC, "value": None, "unit": "hashes/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic 80-byte block headers", "config": _base_config(args, world),
        "error": error, "errors": errors, "diagnosis": diagnosis,
        "summary": {"world_size": world, "error": str(error)[:300], "errors": _short_errors(errors),
                    "ranks_checked_in": (diagnosis or {}).get("ranks_checked_in"),
                    "rank_phases": phases or None},
    }


# ------------------------------------------------------------------------------ the printed line
# The driver parses the LAST line of stdout and keeps only a tail of it: BENCH_r05's 25 KB line came back unparsed
# (missing #1). The line is the driver contract (CONTRACT_KEYS, a short ``config``), the path of the
# detail file, and the compact ``summary`` last; every full section object goes to the detail file.
LINE_CAP = 6144
CONTRACT_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data")
CONFIG_KEYS = ("model", "global_batch", "seq_len", "parallelism", "kernel", "variants_per_step")
# summary keys dropped first when a line would still pass LINE_CAP (long error texts, per-rank lists)
_DROP_ORDER = ("rank_phases", "sections_s", "ranks_seen", "per_rank_hps", "job_switch_p50_ms", "node_rejected",
               "cfg5_pool_validate_p50_ms", "errors", "node_hps")


def detail_paths() -> list[str]:
    """Where the full result goes: OTEDAMA_BENCH_DETAIL if set, else ./bench_detail.json and
    ./gpurun_out/bench_detail.json (the part of a GPU box's tree that comes back)."""
    p = os.environ.get("OTEDAMA_BENCH_DETAIL")
    if p:
        return [p]
    return [os.path.abspath("bench_detail.json"), os.path.abspath(os.path.join("gpurun_out", "bench_detail.json"))]


def write_detail(full: dict) -> str | None:
    """Write the full result (every section object) to the detail file(s); the first path written, or None."""
    first = None
    blob = json.dumps(full, default=str)
    for p in detail_paths():
        try:
            os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
            tmp = f"{p}.{os.getpid()}.tmp"
            with open(tmp, "w") as f:
                f.write(blob)
            os.replace(tmp, p)
            first = first or p
        except OSError:
            continue
    return first


def compact_line(full: dict, detail: str | None) -> str:
    """The one JSON line rank 0 prints: driver contract keys, a config of <= 6 short fields, the detail path, and
    ``summary`` last, capped at LINE_CAP bytes (summary keys are dropped in _DROP_ORDER, then strings cut, if a
    pathological run would pass it)."""
    line = {k: full.get(k) for k in CONTRACT_KEYS}
    cfg = full.get("config") or {}
    line["config"] = {k: (cfg[k][:60] if isinstance(cfg[k], str) else cfg[k]) for k in CONFIG_KEYS if k in cfg}
    if full.get("error") is not None:
        line["error"] = str(full["error"])[:300]
    line["detail"] = os.path.basename(detail) if detail else None
    summary = dict(full.get("summary") or {})
    line["summary"] = summary
    s = json.dumps(line, default=str)
    for k in _DROP_ORDER:
        if len(s) <= LINE_CAP:
            break
        if k in summary:
            summary.pop(k)
            summary.setdefault("dropped", []).append(k)
            s = json.dumps(line, default=str)
    if len(s) > LINE_CAP:  # last resort: every summary value as a short string
        line["summary"] = {k: (v if isinstance(v, (int, float, bool)) or v is None else str(v)[:40])
                           for k, v in list(summary.items())[:60]}
        s = json.dumps(line, default=str)
    return s


def finalize(full: dict) -> str:
    """Write the detail file, say where on stderr, and return the line to print."""
    detail = write_detail(full)
    if detail:
        try:
            os.write(2, f"bench.py: full result -> {detail}\n".encode())
        except OSError:
            pass
    return compact_line(full, detail)


# --------------------------------------------------------------------------- the run
class Bench:
    """One rank of the benchmark. Sections fill ``R``; ``output()`` turns whatever is in it into the JSON line."""

    def __init__(self, args, rank: int, world: int):
        self.args = args
        self.rank, self.world = rank, world
        self.cpu = args.cpu_rehearsal
        self.R: dict = {}
        self.guard = None
        self.info = self.comm = self.N = self.dev = None
        self.budgets = self._budgets()
        # run_rank raised GPU_MAX_HW_QUEUES for this process; preflight restores the previous value once HIP is up
        self.hw_queues_raised, self.hw_queues_prev = False, None

    # ------------------------------------------------------------------ budgets
    def _budgets(self) -> dict[str, float]:
        a = self.args
        ssteps = a.steps if a.scrypt_steps < 0 else a.scrypt_steps
        xsteps = a.steps if a.x11_steps < 0 else a.x11_steps
        miner_s = self.miner_seconds()
        node_s, pool_s = self.node_seconds(), self.pool_seconds()
        algos = max(1, len(self.node_algorithms()))
        b = {"sha256d": 120.0 + 5.0 * (a.steps + a.warmup), "single": 90.0, "scrypt": 90.0 + 3.0 * ssteps,
             "x11": 90.0 + 2.0 * xsteps, "miner": 2 * (miner_s + 60.0), "cpu": 40.0 + 3.0 * a.cpu_seconds,
             "comm": 60.0 + len(self.comm_phases()) * (30.0 + 4 * a.comm_ops / 100.0),
             "latency": 180.0, "node": algos * (150.0 + node_s + a.node_warmup + 4.0 * a.node_switches),
             "pool": 240.0 + pool_s}
        for item in filter(None, (s.strip() for s in a.section_timeouts.split(","))):
            k, _, v = item.partition("=")
            b[k.strip()] = float(v)
        return b

    def miner_seconds(self) -> float:
        return self.args.miner_seconds if self.args.miner_seconds >= 0 else (0.0 if self.cpu else 8.0)

    def node_seconds(self) -> float:
        return self.args.node_seconds if self.args.node_seconds >= 0 else (0.0 if self.cpu else 8.0)

    def pool_seconds(self) -> float:
        return self.args.pool_seconds if self.args.pool_seconds >= 0 else (0.0 if self.cpu else 45.0)

    def comm_phases(self) -> list[str]:
        """The comm section's phases: idle, then under each mining algorithm (GPUs only: the CPU rehearsal has no
        device process to load the data plane with)."""
        algos = [] if self.cpu else [x.strip() for x in self.args.comm_load.split(",") if x.strip()]
        return ["idle", *algos]

    def node_algorithms(self) -> list[str]:
        return [x.strip() for x in self.args.node_algorithms.split(",") if x.strip()]

    # ------------------------------------------------------------------ driver
    def run(self) -> int:
        g = self.guard
        try:
            with g.section("preflight", max(10.0, self.args.preflight_timeout - g.elapsed()), critical=True):
                self.preflight()
        except Exception as exc:  # noqa: BLE001 - a start that failed outright (not a hang): report it
            return self.fail("preflight", f"{type(exc).__name__}: {exc}")
        try:
            with g.section("sha256d", self.budgets["sha256d"], critical=True):
                self.sha256d()
        except Exception as exc:  # noqa: BLE001
            return self.fail("sha256d", f"{type(exc).__name__}: {exc}")
        g.headline_done = True  # every rank holds the headline now (its last collective included rank 0)
        # sections every rank takes part in (collectives): rank 0 decides whether there is time and tells the rest
        need = {"single": 15.0, "scrypt": 30.0, "x11": 20.0, "miner": 2 * (self.miner_seconds() + 20.0),
                "comm": 30.0 + 2 * len(self.comm_phases()) * 12.0}
        # After the headline every collective is bounded (half the section's budget, at most 120 s): a rank stuck in
        # one of these sections costs that section (CollectiveTimeout on the others), not the rank-0 sections after
        # them; once the data plane failed, the remaining collective sections are skipped with the reason.
        broken = ""
        for name, fn in (("single", self.single), ("scrypt", self.scrypt), ("x11", self.x11),
                         ("miner", self.miner), ("comm", self.comm_section)):
            if not self.wanted(name):
                continue
            if broken:
                g.skip(name, f"data plane unusable after {broken}")
                continue
            go = g.remaining() >= need[name] if self.rank == 0 else True
            if self.world > 1:
                try:
                    with self.bounded_comm(60.0):
                        go = bool(self.comm.broadcast_control([int(go)])[0])
                except Exception as exc:  # noqa: BLE001 - a peer is gone or stuck
                    broken = f"{name} go/no-go: {type(exc).__name__}"
                    g.skip(name, f"data plane unusable: {type(exc).__name__}: {exc}"[:200])
                    continue
            if not go:
                g.skip(name, f"bench deadline: {g.remaining():.0f} s left")
                continue
            with g.section(name, self.budgets[name]):
                with self.bounded_comm(min(120.0, self.budgets[name] / 2.0)):
                    fn()
            err = g.errors.get(name, "")
            if self.world > 1 and ("CollectiveTimeout" in err or "rccl" in err.lower()):
                broken = name
        if self.rank != 0:
            g.finish()
            self.shutdown()
            return 0
        need0 = {"cpu": 2.5 * self.args.cpu_seconds + 5, "latency": 60.0,
                 "node": 40.0 + self.node_seconds() + self.args.node_warmup, "pool": 90.0 + self.pool_seconds()}
        for name, fn in (("cpu", self.cpu_miner), ("latency", self.latency), ("node", self.node),
                         ("pool", self.pool)):
            if not self.wanted(name):
                continue
            if g.remaining() < need0[name]:
                g.skip(name, f"bench deadline: {g.remaining():.0f} s left")
                continue
            with g.section(name, self.budgets[name]):
                fn()
        if not g.finish():
            while True:  # the watchdog fired meanwhile and is printing / exiting
                time.sleep(1)
        print(finalize(self.output(dict(g.errors))), flush=True)
        self.shutdown()
        return 0

    def wanted(self, name: str) -> bool:
        a, cpu = self.args, self.cpu
        return {
            "single": a.single_midstate_headers > 0 and not cpu,
            "scrypt": (a.steps if a.scrypt_steps < 0 else a.scrypt_steps) > 0 and not cpu,
            "x11": (a.x11_steps if a.x11_steps >= 0 else a.steps) > 0 and not cpu,
            "miner": self.miner_seconds() > 0,
            "comm": a.comm_ops > 0,
            "cpu": a.cpu_seconds > 0,
            "latency": not a.no_latency and not cpu,
            "node": self.node_seconds() > 0 and bool(self.node_algorithms()),
            "pool": self.pool_seconds() > 0,
        }[name]

    def fail(self, section: str, error: str) -> int:
        """A critical section failed with an exception: rank 0 reports, every rank leaves non-zero."""
        g = self.guard
        g.errors.setdefault(section, error)
        if self.rank == 0 and g.finish():
            print(finalize(self.output(dict(g.errors), fatal=error)), flush=True)
            g.stop_peers()
        else:
            g.finish()
        return 1

    def emit(self, errors: dict, reason: str) -> int:
        """Watchdog path (rank 0): print the JSON with what finished; exit code 0 when the headline was measured."""
        out = self.output(errors, fatal=None if "sha" in self.R else reason)
        os.write(1, (finalize(out) + "\n").encode())
        return 0 if "sha" in self.R else 1

    SHUTDOWN_S = 20.0  # bound on tearing the process group down once the JSON is out

    def shutdown(self) -> None:
        """Tear the process group down, bounded: at world > 1 the peers may already be gone (the other ranks leave
        after their last collective section while rank 0 runs the node and pool sections), and a teardown that
        waited on them must not hold this process (and the driver's torchrun) open after the JSON line is out."""
        if self.info is None or self.comm is None:
            return

        def run():
            with contextlib.suppress(Exception):
                self.comm.close()

        th = threading.Thread(target=run, name="otedama-bench-shutdown", daemon=True)
        th.start()
        th.join(self.SHUTDOWN_S)
        if th.is_alive():
            print(f"bench.py: rank {self.rank}: process-group teardown did not finish in {self.SHUTDOWN_S:.0f} s; "
                  "leaving without it", file=sys.stderr, flush=True)
            sys.stdout.flush()
            os._exit(0)

    # ------------------------------------------------------------------ sections
    PREFLIGHT_RESERVE_S = 40.0  # of the pre-flight budget kept back from the probe for a gloo fallback's init

    def native_wanted(self) -> bool:
        """The bench's data plane is the node's: the native RCCL module (parallel/rcclcomm.py) on GPUs, or its CPU
        stand-in when OTEDAMA_RCCL_MODULE names one (the rehearsal of that path). OTEDAMA_BENCH_COMM=torch keeps
        torch.distributed; OTEDAMA_DIST_BACKEND=gloo (ranks sharing one GPU) and the plain CPU rehearsal use gloo."""
        mode = os.environ.get("OTEDAMA_BENCH_COMM", "").lower()
        if mode in ("torch", "native"):
            return mode == "native"
        if os.environ.get("OTEDAMA_RCCL_MODULE"):
            return True
        return not self.cpu and os.environ.get("OTEDAMA_DIST_BACKEND") != "gloo"

    def open_native(self, store, timeout: float):
        """(NativeNodeComm, error): every rank forms the native communicator, then all ranks agree through the store;
        if any rank failed, every rank drops it (error set) and the caller falls back together."""
        import torch

        from otedama_amd.parallel.commbase import DistInfo
        from otedama_amd.parallel.rcclcomm import NativeNodeComm, _wait_get, cpu_standin

        local = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        dev = torch.device("cpu") if (self.cpu or cpu_standin()) else torch.device(f"cuda:{local}")
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        info = DistInfo(self.rank, self.world, local, "rccl", dev, store=store)
        comm, err = None, ""
        try:
            from otedama_amd.parallel.guard import fault_for

            if fault_for(self.rank, "native") == "fail":  # tests: this rank's in-process init fails after the probe
                raise RuntimeError("injected native init failure")
            comm = NativeNodeComm(info, bounded=False, force=True, device_stream=True)
            with _stdout_to_stderr():  # RCCL prints a version banner on stdout at init, whatever NCCL_DEBUG says
                comm.reform(list(range(self.world)), 1, timeout=timeout)
        except Exception as exc:  # noqa: BLE001 - decided together below
            comm, err = None, f"{type(exc).__name__}: {exc}"[:300]
        if self.world > 1:
            store.set(f"otd-bench/native/{self.rank}", "1" if comm is not None else "0" + err)
            try:
                flags = [_wait_get(store, f"otd-bench/native/{r}", timeout + 10.0) for r in range(self.world)]
            except TimeoutError as exc:
                flags, err = [], err or str(exc)
            if len(flags) != self.world or any(f != b"1" for f in flags):
                # every failed rank's reason (a rank that failed at once makes the others' inits time out)
                bad = {r: f[1:].decode(errors="replace")[:100] for r, f in enumerate(flags) if f != b"1"}
                err = f"native communicator failed on rank(s) {sorted(bad)}: {bad}" if bad else err
                if comm is not None:
                    comm.close()
                comm = None
        return comm, err

    def preflight(self) -> None:
        t0 = time.monotonic()
        self.guard.set_phase("import")
        import torch

        from otedama_amd.ops import native
        from otedama_amd.parallel import NodeComm, init_from_env

        cpu = self.cpu
        if not cpu and not torch.cuda.is_available():
            raise RuntimeError("bench.py requires a GPU (HIP); run `python -m otedama_amd.cli bench-cpu` for the CPU "
                               "config (or --cpu-rehearsal for the launcher/collective rehearsal)")
        if not cpu and self.world > 1 and os.environ.get("OTEDAMA_DIST_BACKEND") != "gloo":
            local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
            if local >= torch.cuda.device_count():
                raise RuntimeError(f"rank with LOCAL_RANK={local} has no GPU ({torch.cuda.device_count()} visible)")
        self.N = native.require_native()
        t_import = time.monotonic()
        self.guard.set_phase("rendezvous")
        backend, store, probe = ("gloo" if cpu else None), None, None
        native_on = self.native_wanted()
        left = lambda: max(20.0, self.args.preflight_timeout - self.guard.elapsed())  # noqa: E731
        if self.world > 1 and (native_on or os.environ.get("OTEDAMA_BENCH_PROBE") == "1"):
            # Can the native RCCL module form a group of every rank, within a deadline? Checked in child processes
            # first (parallel/rccl_probe.py): a hang there costs the deadline, not the run. If any rank's check fails,
            # every rank runs over gloo together (rank 0's one decision) and the headline is still measured.
            from otedama_amd.parallel.comm import connect_store_from_env
            from otedama_amd.parallel.guard import fault_for
            from otedama_amd.parallel.rccl_probe import run_probe

            self.guard.set_phase("data-plane probe")
            store = connect_store_from_env()
            if fault_for(self.rank, "arrive") == "slow":  # tests: a rank that reaches the probe late
                time.sleep(float(os.environ.get("OTEDAMA_FAULT_SLOW_S", "25")))
            probe = run_probe(store, self.rank, self.world, fault=fault_for(self.rank, "probe"),
                              budget=left() - self.PREFLIGHT_RESERVE_S)
            if not probe["ok"]:
                native_on, backend = False, "gloo"
            self.guard.set_phase("rendezvous")
        comm, native_err = None, ""
        if native_on:
            # the probe's children formed the same group in probe["seconds"]: the in-process init gets a few times
            # that (a rank whose init fails outright leaves its peers waiting in theirs until this bound)
            bound = 60.0 if probe is None else max(15.0, 4.0 * float(probe.get("seconds") or 0.0))
            comm, native_err = self.open_native(store, timeout=min(bound, max(10.0, left() - 30.0)))
            if comm is None and self.world > 1:
                backend = "gloo"
        if backend == "gloo" and self.world > 1:
            os.environ["OTEDAMA_DIST_BACKEND"] = "gloo"  # the node / pool sections' processes follow
        if comm is not None:
            self.info, impl = comm.info, "rccl-native"
        else:
            self.info = init_from_env(backend=backend, use_gpu=not cpu, store=store)
            comm = NodeComm(self.info)
            impl = {"nccl": "torch-nccl"}.get(self.info.backend, self.info.backend)
        self.comm = comm
        self.dev = self.info.device
        if self.hw_queues_raised:  # HIP and the communicator are up: children started later get the value they had
            if self.hw_queues_prev is None:
                os.environ.pop("GPU_MAX_HW_QUEUES", None)
            else:
                os.environ["GPU_MAX_HW_QUEUES"] = self.hw_queues_prev
        t_pg = time.monotonic()
        self.guard.set_phase("first-collective")
        total = self.comm.allreduce_counters(1)[0]  # the first collective on the data plane (RCCL on GPUs)
        rows = self.comm.gather_counters([self.info.rank, os.getpid(), 0, 0])
        self.comm.barrier()
        t1 = time.monotonic()
        if total != self.world:
            raise RuntimeError(f"pre-flight all_reduce summed {total}, expected {self.world}")
        self.R["preflight"] = {"ok": True, "ranks": sorted(int(r[0]) for r in rows),
                               "data_plane": {"impl": impl, "backend": self.info.backend, "probe": probe,
                                              **({"native_error": native_err} if native_err else {})},
                               "import_s": round(t_import - t0, 2), "rendezvous_s": round(t_pg - t_import, 2),
                               "first_collectives_ms": round((t1 - t_pg) * 1e3, 2),
                               "since_start_s": round(self.guard.elapsed(), 2), "backend": self.info.backend}

    def sync(self) -> None:
        if not self.cpu:
            import torch

            torch.cuda.synchronize(self.dev)

    def barrier(self) -> None:
        self.comm.barrier()

    def sha256d(self) -> None:
        import torch

        from otedama_amd.parallel import stripe_for
        from otedama_amd.utils.trace import span

        args, N, comm, info, dev, cpu = self.args, self.N, self.comm, self.info, self.dev, self.cpu
        world = info.world_size
        sync = self.sync
        job = comm.broadcast_job(synthetic_job(args.seed) if info.is_primary else None)  # R1: the job blob, once
        if cpu:
            from otedama_amd.models.header import int_to_hash

            job["target"] = int_to_hash((1 << 244) - 1)  # ~1 hit per 4096 hashes: the rehearsal exercises R2
        self.job = job
        target_int = int.from_bytes(job["target"], "little")
        stripe = stripe_for(info.rank, info.world_size)
        self.stripe = stripe
        use_v = args.sha_kernel == "v" or cpu
        s1 = None
        if cpu:
            K, V_COUNT = 4, max(1, args.cpu_nonces)
            steps_per_group = 2
            search = _CpuSearch(N, K)
        elif use_v:
            # One step = 64 x chains version variants (chains per lane of a wave) x 2^35 / that many nonces = 2^35
            # hashes, the same work as the K=8 step (8 x 2^32); 8 x chains consecutive steps tile the full 2^32 nonces
            # of one variant group. Two chains run the 4-waves/SIMD build at 128 blocks/CU (profiles/r2/sha_v2).
            from otedama_amd.ops.search import SHA256D_V2_BLOCKS_PER_CU, Sha256dSearchV, default_grid

            K = N.SHA256D_V_GROUP * args.sha_chains
            V_COUNT = (1 << 35) // K
            steps_per_group = (1 << 32) // V_COUNT
            s1 = torch.cuda.Stream(dev)
            if args.sha_chains == 2:
                search = Sha256dSearchV(dev, grid=args.grid or default_grid(dev, SHA256D_V2_BLOCKS_PER_CU), chains=2,
                                        occupancy8=False)
            else:
                search = Sha256dSearchV(dev, grid=args.grid or None)
        else:
            from otedama_amd.ops.search import Sha256dSearch, Sha256dSearchK

            V_COUNT, steps_per_group = 1 << 32, 1
            K = max(k for k in (1, *N.SHA256D_K_VALUES) if k <= max(1, args.sha_variants))
            search = Sha256dSearchK(dev, k=K, grid=args.grid or None) if K > 1 else \
                Sha256dSearch(dev, grid=args.grid or None)
        SUB_LAUNCHES = 8  # 2^32 hashes per launch
        slot_words = 1 + (2 if K > 1 else 1) * search.cap
        # double-buffered hit slots: step i writes outs[i % 2] while R2 of step i-1 reads the other one
        outs = [torch.zeros(slot_words, dtype=torch.int32, device=dev) for _ in range(2)]
        gathered = [torch.zeros(world, slot_words, dtype=torch.int32, device=dev) for _ in range(2)]
        r2_seen = torch.zeros(1, dtype=torch.int64, device=dev)  # hits of every rank that arrived through R2
        r2_done: list = [None, None]
        ctl = torch.zeros(4, dtype=torch.int64, device=dev)

        def variant_params(step: int) -> tuple[list[bytes], bytes]:
            hdrs = [N.variant_header(job, stripe.start + (step * K + j) * stripe.stride)[0] for j in range(K)]
            if K > 1:
                return hdrs, N.sha256d_prepare_k(hdrs, job["target"])
            return hdrs, N.sha256d_prepare(hdrs[0], job["target"])

        v_groups: dict[int, tuple[list[bytes], object]] = {}

        def v_group(q: int):
            # variant group q of this rank: stripe positions Kq .. Kq+K-1; the table is uploaded once, before timing
            if q not in v_groups:
                hdrs = [N.variant_header(job, stripe.start + (q * K + j) * stripe.stride)[0] for j in range(K)]
                v_groups[q] = (hdrs, search.prepare(hdrs, job["target"]))
            return v_groups[q]

        hits_log: list = []
        last_group = [-1]

        def step(i: int, record: bool) -> None:
            with span("otd.bench.sha256d_step"):
                _step(i, record)

        def _step(i: int, record: bool) -> None:
            b = i % 2
            q = i // steps_per_group
            if world > 1 and q != last_group[0]:  # R1 on change: rank 0 announces the next variant group
                if info.is_primary:
                    ctl.fill_(q)
                comm.run_async(lambda: comm.broadcast_tensor(ctl))
                last_group[0] = q
            if r2_done[b] is not None:  # the gather that read this slot two steps ago must be done before reuse
                torch.cuda.current_stream(dev).wait_event(r2_done[b])
            out = outs[b]
            if use_v:  # K1: 128 variants x 1/16 of the nonce space (W3 window)
                hdr, prep = v_group(q)
                if cpu:
                    search.launch(prep, (i % steps_per_group) * V_COUNT, V_COUNT, out)
                else:
                    # the step's window as SUB_LAUNCHES launches of 2^32 hashes alternating over two streams, as the
                    # production miner issues them (a launch's last waves overlap the next launch's first); on three
                    # boxes this measured -0.2% .. +0.35% against one 2^35-hash launch (profiles/r3/s_paths)
                    s0 = torch.cuda.current_stream(dev)
                    out[:1].zero_()
                    s1.wait_stream(s0)
                    sub = V_COUNT // SUB_LAUNCHES
                    lo = (i % steps_per_group) * V_COUNT
                    for j in range(SUB_LAUNCHES):
                        search.launch_into(prep, lo + j * sub, sub, out, s0 if j % 2 == 0 else s1)
                    # The step's consumers (the hit copy, R2) go behind its last launch on s1, which waits for s0's
                    # last launch only: s0 starts the next step at once and that launch overlaps this step's tail, as
                    # the production miner's two streams never join.
                    s1.wait_stream(s0)
            else:
                hdr, params = variant_params(i)
                search.launch(params, 0, 1 << 32, out=out)  # K1: full 2^32 nonce space
            tail = s1 if (use_v and not cpu) else None
            with torch.cuda.stream(tail) if tail is not None else contextlib.nullcontext():
                if record:  # with the nonce window the step covered (W3 = bswap(nonce) for the v kernel)
                    lo = (i % steps_per_group) * V_COUNT if use_v else 0
                    hits_log.append((hdr, out.clone(), lo, V_COUNT if use_v else 1 << 32))

                def r2(o=out, g=gathered[b]):
                    comm.gather_tensor(g, o)  # device-resident on the native data plane (a copy at world 1 on torch)
                    r2_seen.add_(g[:, 0].clamp(max=search.cap).sum())

                r2_done[b] = comm.run_async(r2)  # R2 overlaps the next step's kernel

        # Warmup steps take the stripe positions right after the timed ones (steps .. steps+W-1), so every position
        # used stays inside the 2^16 BIP320 variant space: (steps + W) * K * world <= 65536.
        positions = ((args.steps + args.warmup + steps_per_group - 1) // steps_per_group + 1) * K if use_v \
            else (args.steps + args.warmup) * K
        if positions * world > 1 << 16:
            raise SystemExit("bench.py: (steps + warmup) x variants x GPUs exceeds the 2^16 version-rolling space")
        self.positions = positions
        if use_v:  # variant tables for every step, timed and warmup, built and uploaded before the timed region
            for i in range(args.steps + args.warmup):
                v_group(i // steps_per_group)
        for i in range(args.warmup):
            step(args.steps + i, False)
        sync()
        self.barrier()
        sync()
        r2_seen.zero_()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, True)
        step_hashes = K * (V_COUNT if use_v else 1 << 32)
        total = comm.allreduce_counters(args.steps * step_hashes)[0] if world > 1 else args.steps * step_hashes  # R3
        sync()
        self.barrier()
        sync()
        t_local = time.perf_counter() - t0
        elapsed = comm.allreduce_max(t_local)
        sha_hps = total / elapsed
        # per-rank rates + which ranks actually took part in the collectives (RCCL world check)
        rows = comm.gather_counters([info.rank, args.steps * step_hashes, int(t_local * 1e6), int(r2_seen.item())])
        ranks_seen = sorted(int(r[0]) for r in rows)
        per_rank_hps = [r[1] / max(r[2] * 1e-6, 1e-9) for r in sorted(rows)]

        # Re-verify every hit of the timed region on the CPU (full 256-bit compare), de-duplicated by (variant, nonce).
        found = verified = dups = outside = 0
        seen: set = set()
        for hdrs, buf, lo, cnt in hits_log:
            host = buf.cpu().tolist()
            n = min(host[0] & 0xFFFFFFFF, search.cap)
            pairs = [(host[1 + 2 * i], host[2 + 2 * i]) for i in range(n)] if K > 1 else \
                [(x, 0) for x in host[1 : 1 + n]]
            for nonce, vi in pairs:
                nonce &= 0xFFFFFFFF
                found += 1
                w = nonce if cpu or not use_v else int.from_bytes(nonce.to_bytes(4, "little"), "big")
                outside += not lo <= w < lo + cnt  # a hit outside the window the step was asked to search
                if not 0 <= vi < K:
                    continue
                hdr = hdrs[vi]
                key = (hdr[:76], nonce)
                if key in seen:
                    dups += 1
                    continue
                seen.add(key)
                h = hashlib.sha256(hashlib.sha256(hdr[:76] + nonce.to_bytes(4, "little")).digest()).digest()
                if int.from_bytes(h, "little") <= target_int:
                    verified += 1
        found, verified, dups, outside = comm.allreduce_counters(found, verified, dups, outside)
        expected, z = _poisson(verified, total, target_int)
        self.R["sha"] = {
            "hps": sha_hps, "elapsed": elapsed, "K": K, "V_COUNT": V_COUNT, "use_v": use_v,
            "steps_per_group": steps_per_group, "step_hashes": step_hashes, "grid": search.grid,
            "ranks_seen": ranks_seen, "per_rank_hps": per_rank_hps, "found": found, "verified": verified,
            "dups": dups, "outside": outside, "expected": expected, "z": z,
            "r2_hits": rows[0][3] if rows else 0,  # rank 0's R2 view of every rank's hit counts
        }

    def single(self) -> None:
        """BASELINE config 2 verbatim: one fixed midstate, full 2^32 nonces per header."""
        import torch

        from otedama_amd.ops.search import Sha256dSearch

        N, job, stripe, comm, world = self.N, self.job, self.stripe, self.comm, self.info.world_size
        target_int = int.from_bytes(job["target"], "little")
        ss = Sha256dSearch(self.dev)
        heads = [N.variant_header(job, stripe.start + (self.positions + j) * stripe.stride)[0]
                 for j in range(self.args.single_midstate_headers)]
        params = [N.sha256d_prepare(h, job["target"]) for h in heads]
        ss.launch(params[0], 0, 1 << 24)  # warm the kernel
        self.sync()
        self.barrier()
        self.sync()
        souts = []
        t0 = time.perf_counter()
        for p in params:
            souts.append(ss.launch(p, 0, 1 << 32, out=torch.zeros_like(ss.out)).buf)
        self.sync()
        self.barrier()
        self.sync()
        s_el = comm.allreduce_max(time.perf_counter() - t0)
        s_total = len(params) * (1 << 32) * world
        s_found = s_ok = 0
        for h, buf in zip(heads, souts):
            host = buf.cpu().tolist()
            for nonce in host[1 : 1 + min(host[0] & 0xFFFFFFFF, ss.cap)]:
                nonce &= 0xFFFFFFFF
                s_found += 1
                d = hashlib.sha256(hashlib.sha256(h[:76] + nonce.to_bytes(4, "little")).digest()).digest()
                s_ok += int.from_bytes(d, "little") <= target_int
        s_found, s_ok, _, _ = comm.allreduce_counters(s_found, s_ok)
        self.R["single"] = {"hashes_per_sec": s_total / s_el, "kernel": "otd_sha256d_search",
                            "headers_per_rank": len(params), "nonces_per_header": 1 << 32, "grid": ss.grid,
                            "hits_found": s_found, "hits_verified": s_ok,
                            "hits_expected": _poisson(s_ok, s_total, target_int)[0]}
        del ss

    def scrypt(self) -> None:
        import torch

        from otedama_amd.models.algorithms import ALGORITHMS
        from otedama_amd.models.header import int_to_hash
        from otedama_amd.ops.search import ScryptSearch

        args, N, comm, info = self.args, self.N, self.comm, self.info
        world = info.world_size
        ssteps = args.steps if args.scrypt_steps < 0 else args.scrypt_steps
        sc = ScryptSearch(self.dev, gap=args.scrypt_gap, kernel=args.scrypt_kernel)
        s_int = ALGORITHMS["scrypt"].diff1
        starget = int_to_hash(s_int)
        hdr, _, _, _ = N.variant_header(self.job, self.stripe.start)
        sparams = N.scrypt_prepare(hdr, starget)
        sc.launch(sparams, 0)
        self.sync()
        self.barrier()
        self.sync()
        sbufs = []
        t0 = time.perf_counter()
        for i in range(ssteps):
            base = ((i * world + info.rank) * sc.batch) & 0xFFFFFFFF  # ranks partition the nonce range
            sbufs.append(sc.launch(sparams, base).buf.clone())
        self.sync()
        self.barrier()
        self.sync()
        selapsed = comm.allreduce_max(time.perf_counter() - t0)
        stotal = comm.allreduce_counters(ssteps * sc.batch)[0] if world > 1 else ssteps * sc.batch
        # re-verify up to 64 hits per rank with hashlib.scrypt (CPU, ~1 ms each)
        sfound = sver = schecked = 0
        for buf in sbufs:
            host = buf.cpu().tolist()
            for nonce in host[1 : 1 + min(host[0] & 0xFFFFFFFF, sc.cap)]:
                sfound += 1
                if schecked >= 64:
                    continue
                schecked += 1
                h80 = hdr[:76] + (nonce & 0xFFFFFFFF).to_bytes(4, "little")
                d = hashlib.scrypt(h80, salt=h80, n=1024, r=1, p=1, dklen=32)
                sver += int.from_bytes(d, "little") <= s_int
        sfound, sver, schecked, _ = comm.allreduce_counters(sfound, sver, schecked)
        self.R["scrypt_hps"] = self.R["scrypt_kernel_hps"] = stotal / selapsed
        self.R["scrypt"] = {"kernel": sc.kernel, "lookup_gap": 1 if sc.kernel == "coop" else sc.gap,
                            "lanes": sc.batch, "scratch_gib_per_gpu": round(sc.scratch_bytes / 2**30, 2),
                            "hits_found": sfound, "hits_checked": schecked, "hits_verified": sver,
                            "hits_expected": _poisson(sfound, stotal, s_int)[0],
                            "hit_target": "scrypt diff 1 (0xFFFF<<224)", "kernel_path_hashes_per_sec": stotal / selapsed}
        del sc
        torch.cuda.empty_cache()

    def x11(self) -> None:
        """BASELINE config 4: X11 with the nonce range partitioned across ranks (rank r takes batches r, r + N, ...).
        Target 2^-20 so every step yields hits that are re-verified on the CPU."""
        import torch

        from otedama_amd.models.header import int_to_hash
        from otedama_amd.ops.search import X11Search

        args, N, comm, info = self.args, self.N, self.comm, self.info
        world = info.world_size
        xsteps = args.steps if args.x11_steps < 0 else args.x11_steps
        xs = X11Search(self.dev, cap=4096)
        xtarget_int = (1 << 236) - 1
        hdr, _, _, _ = N.variant_header(self.job, self.stripe.start)
        xparams = N.x11_prepare(hdr, int_to_hash(xtarget_int))
        xs.launch(xparams, 0)
        self.sync()
        self.barrier()
        self.sync()
        xhits: list = []
        t0 = time.perf_counter()
        for i in range(xsteps):
            base = ((i * world + info.rank) * xs.batch) & 0xFFFFFFFF
            xhits.append(xs.launch(xparams, base).buf.clone())
        self.sync()
        self.barrier()
        self.sync()
        xelapsed = comm.allreduce_max(time.perf_counter() - t0)
        xtotal = comm.allreduce_counters(xsteps * xs.batch)[0] if world > 1 else xsteps * xs.batch
        xfound = xver = 0
        for buf in xhits:
            host = buf.cpu().tolist()
            for nonce in host[1 : 1 + min(host[0] & 0xFFFFFFFF, xs.cap)]:
                xfound += 1
                h = N.x11(hdr[:76] + (nonce & 0xFFFFFFFF).to_bytes(4, "little"))
                xver += int.from_bytes(h, "little") <= xtarget_int
        xfound, xver, _, _ = comm.allreduce_counters(xfound, xver)
        self.R["x11_hps"] = self.R["x11_kernel_hps"] = xtotal / xelapsed
        self.R["x11"] = {"batch_per_launch": xs.batch, "kernels": "11 stage kernels per batch (tools/bench_x11.py)",
                         "hits_found": xfound, "hits_verified": xver, "hit_target": "2^-20",
                         "hits_expected": _poisson(xfound, xtotal, xtarget_int)[0],
                         "kernel_path_hashes_per_sec": xtotal / xelapsed}
        del xs
        torch.cuda.empty_cache()

    def miner(self) -> None:
        """scrypt and X11 through the production miner. The kernel sections above time the ops-API launches one
        after another. The production miner runs scrypt as two half-grid batches side by side and X11 with a digest
        plane per slot, in a device process of its own; its exact rate over whole launches there, with every share
        re-verified, is the scrypt / X11 figure (the kernel-path rate stays beside it). In this torch process the same
        miner measured 16.2-16.4 MH/s against 17.2-17.5 in fresh processes (profiles/r4/h_bench_sections, i_bisect)."""
        import torch

        from otedama_amd.engine.miner_probe import measure_miner
        from otedama_amd.models.algorithms import ALGORITHMS

        comm, info = self.comm, self.info
        miner_s = self.miner_seconds()
        for algo, tgt in (("scrypt", ALGORITHMS["scrypt"].diff1), ("x11", (1 << 236) - 1)):
            if algo not in self.R:  # its kernel section was skipped or failed
                continue
            self.barrier()
            try:
                r = measure_miner(self.N, self.dev.index or 0, algo, tgt, seconds=miner_s, rank=info.rank,
                                  world=info.world_size, seed=self.args.seed, process=True)
                err = ""
            except Exception as exc:  # noqa: BLE001 - auxiliary: the kernel-path figure stays
                r, err = {"hashes_per_sec": 0.0, "shares": 0, "shares_rechecked": 0, "shares_recheck_ok": 0,
                          "faulted": True}, f"{type(exc).__name__}: {exc}"
            tot, shares_n, chk, chk_ok = comm.allreduce_counters(int(r["hashes_per_sec"]), r["shares"],
                                                                 r["shares_rechecked"], r["shares_recheck_ok"])
            faults = comm.allreduce_counters(int(bool(r.get("faulted")) or bool(err)))[0]
            miner = dict(r, node_hashes_per_sec=float(tot), node_shares=shares_n, node_shares_rechecked=chk,
                         node_shares_recheck_ok=chk_ok, ranks_faulted=faults, window_seconds=miner_s)
            if err:
                miner["error"] = err
            info_d = self.R[algo]
            info_d["miner"] = miner
            used = not faults and chk == chk_ok and tot > 0  # every re-hashed share held and no rank faulted
            if used:
                self.R[f"{algo}_hps"] = float(tot)
            info_d["rate_source"] = "production miner (see miner)" if used else "kernel path"
        if not self.cpu:
            torch.cuda.empty_cache()

    @contextlib.contextmanager
    def bounded_comm(self, deadline: float):
        """Every collective inside raises CollectiveTimeout after ``deadline`` s instead of waiting for a peer that
        never comes (parallel/comm.py and parallel/rcclcomm.py ``bounded`` mode)."""
        comm = self.comm
        saved = comm.bounded, comm.deadline
        comm.bounded, comm.deadline = True, deadline
        try:
            yield
        finally:
            comm.bounded, comm.deadline = saved

    COMM_OP_DEADLINE_S = 30.0  # the comm section's bound on one collective (ops take ~0.1-20 ms)

    def comm_section(self) -> None:
        """The run's own data plane measured across every rank (parallel/comm_probe.py measure_node_comm): the node's
        R1 / R2 / R3 and the device-resident R2 as p50 / p99 over --comm-ops each, idle and with every rank's GPU
        mining, the miner-rate change the ops cause, and one large all_gather's bus bandwidth (xGMI or not)."""
        from otedama_amd.parallel.comm_probe import measure_node_comm

        # Every op of this section is bounded: a collective that one rank never joins raises (CollectiveTimeout)
        # instead of holding the run until the section's watchdog, which would end it before the node and pool
        # sections. It is the last section every rank takes part in, so a communicator broken here harms nothing.
        with self.bounded_comm(min(self.COMM_OP_DEADLINE_S, max(5.0, self.budgets["comm"] / 4.0))):
            self.R["comm"] = measure_node_comm(self.comm, self.dev, phases=self.comm_phases(), ops=self.args.comm_ops,
                                               cadence_hz=self.args.comm_hz,
                                               busbw_bytes=(4 << 20) if self.cpu else self.args.comm_busbw_mib << 20,
                                               say=self.guard.progress)
        self.R["comm"]["impl"] = (self.R.get("preflight") or {}).get("data_plane", {}).get("impl")
        if not self.cpu:  # the links the collectives ran on (KFD topology; ranks' GPUs are ordinals 0..N-1)
            from otedama_amd import hal

            topo = hal.kfd_topology()
            mine = set(range(self.world))
            links = [ln for ln in topo["links"] if ln["from"] in mine and ln["to"] in mine]
            self.R["comm"]["topology"] = {"gpus": topo["gpus"][: self.world], "links": links}

    def cpu_miner(self) -> None:
        """BASELINE config 1: the native CPU miner, single thread and all cores of this box's CPU share."""
        from otedama_amd.cli.bench_cmd import bench_cpu, cpu_share

        self.R["cpu"] = bench_cpu(self.args.cpu_seconds, cpu_share(), single_seconds=self.args.cpu_seconds)

    def latency(self) -> None:
        """End-to-end share latency against the local pool in a separate process (2^32-nonce batches), then the
        job-switch time of the device process for SHA-256d, scrypt and X11 (set_job -> new work running)."""
        from otedama_amd.engine.latency_probe import (measure_device_startup, measure_job_switch,
                                                      measure_share_latency)

        idx = self.dev.index or 0
        try:
            self.R["latency"] = measure_share_latency(device_index=idx, seconds=6.0)
        except Exception as exc:  # noqa: BLE001 - each probe is reported on its own
            self.R["latency"] = {"error": f"{type(exc).__name__}: {exc}"}
        switch = {}
        for algo in ("sha256d", "scrypt", "x11"):
            try:
                switch[algo] = measure_job_switch(device_index=idx, algorithm=algo)
            except Exception as exc:  # noqa: BLE001
                switch[algo] = {"error": f"{type(exc).__name__}: {exc}"}
        self.R["switch"] = switch
        try:
            self.R["startup"] = measure_device_startup(device_index=idx)
        except Exception as exc:  # noqa: BLE001
            self.R["startup"] = {"error": f"{type(exc).__name__}: {exc}"}

    def node(self) -> None:
        """The production node (`otedama node --gpus N`: supervisor, N RCCL ranks, a device process per GPU, rank 0
        on the pool session), once per algorithm against a pool of that algorithm, with forced new blocks for the
        node-wide job switch. Runs after every other rank has left its kernel sections."""
        from otedama_amd.parallel.node_probe import measure_node

        algos = self.node_algorithms()
        per_algo: dict = {}
        self.R["node"] = {"algorithms": per_algo}
        each = self.budgets["node"] / max(1, len(algos))
        for algo in algos:
            if self.guard.remaining() < 40.0 + self.node_seconds():
                per_algo[algo] = {"skipped": f"bench deadline: {self.guard.remaining():.0f} s left"}
                continue
            try:
                per_algo[algo] = measure_node(self.world, seconds=self.node_seconds(), warmup=self.args.node_warmup,
                                              cpu=self.cpu, algorithm=algo, switches=self.args.node_switches,
                                              startup_timeout=min(150.0, each - 20.0))
            except Exception as exc:  # noqa: BLE001
                per_algo[algo] = {"error": f"{type(exc).__name__}: {exc}"}
        if "sha256d" in per_algo:  # the SHA-256d run is the node headline (its keys at the top of "node")
            self.R["node"] = dict(per_algo["sha256d"], algorithms=per_algo)

    def pool(self) -> None:
        from otedama_amd.pool.pool_probe import measure_pool

        self.R["pool"] = measure_pool(self.world, seconds=self.pool_seconds(), cpu=self.cpu,
                                      difficulty=0.001 if self.cpu else 1.0)

    # ------------------------------------------------------------------ output
    def output(self, errors: dict, fatal: str | None = None) -> dict:
        args, R, cpu = self.args, dict(self.R), self.cpu
        world = self.info.world_size if self.info is not None else self.world
        backend = self.info.backend if self.info is not None else None
        sha = R.get("sha")
        g = self.guard
        if sha is None:
            out = error_output(args, world, fatal or "no headline", errors,
                               g.diagnose() if g is not None and world > 1 or self.world > 1 else None)
            out["preflight"] = R.get("preflight")
            out["sections"] = g.sections if g is not None else None
            out["summary"] = dict(out.pop("summary"), backend=backend, sections_s=self._section_times())
            return out
        K, V_COUNT, use_v = sha["K"], sha["V_COUNT"], sha["use_v"]
        latency = R.get("latency") if isinstance(R.get("latency"), dict) else {}
        switch = R.get("switch") or {}
        node = R.get("node")
        single = R.get("single") or {}
        out = {
            "metric": METRIC,
            "value": sha["hps"],
            "unit": "hashes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": sha["elapsed"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": sha["hps"] / BASELINE_HPS,
            "dtype": "u32",
            "data": ("synthetic 80-byte block headers (random prev-hash/merkle root), share target = difficulty 1"
                     if not cpu else "CPU REHEARSAL (gloo + native CPU scanner, share target 2^-12): not a GPU "
                                     "measurement"),
            "config": {
                "model": "sha256d",
                "global_batch": sha["step_hashes"] * world,
                "seq_len": 80,
                "parallelism": f"dp{world}",
                "kernel": _sha_name(args, K, use_v),
                "variants_per_step": K,
                "nonce_split": ("per-rank variant stripe; "
                                + (f"{K} variants x 2^{(V_COUNT).bit_length() - 1} nonces per step, "
                                   f"{sha['steps_per_group']} steps tile 2^32 per variant" if use_v
                                   else "full 2^32 nonces per variant per step")),
                "algorithm": ("SHA-256d nonce search, fixed midstate per variant; " + (
                    f"{K} BIP320 version variants per wave ({max(K // 64, 1)} per lane) share the block-2 message "
                    "schedule, computed on the scalar unit" if use_v else
                    f"{K} BIP320 version variants per launch share the block-2 message schedule")),
                "grid": sha["grid"],
            },
            "world_size": world,
            "dist_backend": backend,
            "rccl_ranks_seen": sha["ranks_seen"],
            "per_rank_hashes_per_sec": sha["per_rank_hps"],
            "rehearsal": "cpu-gloo" if cpu else (
                "gloo-shared-gpu" if os.environ.get("OTEDAMA_DIST_BACKEND") == "gloo" and world > 1 else None),
            "preflight": R.get("preflight"),
            "sha256d_hashes_per_sec": sha["hps"],
            "sha256d_per_gpu_hashes_per_sec": sha["hps"] / world,
            "sha256d_single_midstate_hashes_per_sec": single.get("hashes_per_sec"),
            "sha256d_single_midstate": single,
            "hits_found": sha["found"],
            "hits_verified": sha["verified"],
            "hits_duplicate": sha["dups"],
            "hits_outside_window": sha["outside"],
            "hits_expected": sha["expected"],
            "hits_z": sha["z"],
            "hits_seed": args.seed,  # fixed synthetic headers: every run of this seed draws the same hits
            "hits_r2_gathered": sha["r2_hits"],
            "scrypt_hashes_per_sec": R.get("scrypt_hps"),
            "scrypt": R.get("scrypt") or {},
            "x11_hashes_per_sec": R.get("x11_hps"),
            "x11": R.get("x11") or {},
            # the run's data plane measured across every rank (comm section)
            "comm": R.get("comm"),
            "p50_share_latency_ms": latency.get("p50_ms"),
            "device_hit_to_accept_p50_ms": latency.get("device_hit_to_accept_p50_ms"),
            "device_hit_to_accept_p95_ms": latency.get("device_hit_to_accept_p95_ms"),
            "share_latency": R.get("latency"),
            "job_switch_ms": {a: v.get("p50_ms") for a, v in switch.items()} or None,
            "job_switch": switch or None,
            "device_process_startup_s": (R.get("startup") or {}).get("spawn_to_first_batch_s"),
            "device_process_startup": R.get("startup"),
            # the production node (otedama node: supervisor + N RCCL ranks + device processes + local pool)
            "node_hashes_per_sec": (node or {}).get("total_hashes_per_sec"),
            "node": node,
            # BASELINE config 1 (reference: ~2.5 MH/s single thread, ~75 MH/s whole 7950X; BENCHMARKS.md:25-28,44-49)
            "cpu_single_thread_hashes_per_sec": (R.get("cpu") or {}).get("sha256d_single_thread_hps"),
            "cpu_all_cores_hashes_per_sec": (R.get("cpu") or {}).get("sha256d_all_threads_hps"),
            "cpu": R.get("cpu"),
            # BASELINE config 5: mixed SHA-256d + scrypt pool with vardiff, windowed in steady state
            "pool": R.get("pool"),
            "sections": g.sections if g is not None else None,
            "errors": errors or None,
        }
        out["summary"] = self.summary(out, errors)  # LAST: the driver keeps only the tail of stdout
        return out

    def _section_times(self) -> dict:
        g = self.guard
        return {k: v.get("s") for k, v in (g.sections if g is not None else {}).items()}

    def summary(self, out: dict, errors: dict) -> dict:
        """The compact part of the printed line. Every figure names the BASELINE config it answers (cfg1..cfg5,
        BASELINE.json "configs"); the N>1 evidence (rank spread, node efficiency against this run's own per-GPU kernel
        rate, the share delivery split, lost ranks, the data plane and its measured collectives) sits beside it."""
        node = out.get("node") or {}
        pool = (out.get("pool") or {}).get("algorithms") or {}
        lat = out.get("share_latency") or {}
        cpu = out.get("cpu") or {}
        nalg = node.get("algorithms") or {}
        js = node.get("job_switch") or {}
        world = out["world_size"]
        per_rank = [x for x in out.get("per_rank_hashes_per_sec") or [] if x]
        workers = [w for v in pool.values() for w in v.get("workers") or []]
        ivt = [w.get("interval_vs_target") for w in workers if w.get("interval_vs_target") is not None]
        dp = ((out.get("preflight") or {}).get("data_plane") or {})
        comm = self.R.get("comm") or {}
        comm_lat = {ph: comm.get(ph) or {} for ph in ("idle", "sha256d", "scrypt") if comm.get(ph)}

        def p99(op):
            v = {ph: _r((d.get(op) or {}).get("p99_ms")) for ph, d in comm_lat.items()}
            return v or None

        node_sha = (nalg.get("sha256d") or {}).get("total_hashes_per_sec")
        return {
            "cfg2_version_rolled_hps": _r(out["value"]),
            "cfg2_single_midstate_hps": _r(out.get("sha256d_single_midstate_hashes_per_sec")),
            "cfg2_per_gpu_hps": _r(out["value"] / max(world, 1)) if out.get("value") else None,
            "cfg3_scrypt_hps": _r(out.get("scrypt_hashes_per_sec")),
            "cfg3_scrypt_kernel_hps": _r(self.R.get("scrypt_kernel_hps")),
            "cfg4_x11_hps": _r(out.get("x11_hashes_per_sec")),
            "cfg4_x11_node_hps": _r((nalg.get("x11") or {}).get("total_hashes_per_sec")),
            "cfg1_cpu_1t_hps": _r(cpu.get("sha256d_single_thread_hps")),
            "cfg1_cpu_all_hps": _r(cpu.get("sha256d_all_threads_hps")),
            "cfg5_pool_validated_per_s": {a: _r(v.get("validated_shares_per_sec")) for a, v in pool.items()} or None,
            "cfg5_pool_validations": {a: (v.get("validate_ms") or {}).get("samples") for a, v in pool.items()} or None,
            "cfg5_pool_validate_p50_ms": {a: _r((v.get("validate_ms") or {}).get("p50")) for a, v in pool.items()}
            or None,
            "cfg5_pool_interval_vs_target": [_r(min(ivt), 3), _r(max(ivt), 3)] if ivt else None,
            "cfg5_pool_retargets_in_window": sum(int(w.get("retargets_in_window") or 0) for w in workers)
            if workers else None,
            # every worker's vardiff settled before the measurement window opened
            "cfg5_pool_steady": all(w.get("settled_after_s") is not None and w.get("window_opened_after_s") is not None
                                    and w["settled_after_s"] <= w["window_opened_after_s"] for w in workers)
            if workers else None,
            "share_latency_p50_ms": _r(lat.get("p50_ms")),
            "device_hit_to_accept_p50_ms": _r(lat.get("device_hit_to_accept_p50_ms")),
            "job_switch_p50_ms": {a: _r(v) for a, v in (out.get("job_switch_ms") or {}).items()} or None,
            "hits_verified": out.get("hits_verified"),
            "hits_z": _r(out.get("hits_z"), 3),
            # the production node (otedama node --gpus N), per algorithm
            "node_hps": {a: _r(v.get("total_hashes_per_sec")) for a, v in nalg.items()} or None,
            "node_rejected": {a: v.get("pool_rejected") for a, v in nalg.items()} or None,
            "node_job_switch_worst_p50_ms": _r(js.get("worst_rank_p50_ms")),
            "node_op_p99_ms": _r(node.get("op_p99_ms")),
            "node_time_to_hashing_s": node.get("time_to_hashing_s"),
            # N > 1 evidence
            "world_size": world,
            "ranks_seen": out["rccl_ranks_seen"],
            "per_rank_hps": [_r(x, 3) for x in per_rank] if world > 1 else None,
            "rank_rate_min_max": _r(min(per_rank) / max(per_rank), 3) if per_rank else None,
            "rank_efficiency": _r(node_sha / out["value"], 3) if node_sha and out.get("value") else None,
            "remote_hit_to_accept_p50_ms": _r((node.get("hit_to_accept_remote") or {}).get("p50_ms")),
            "shares_via_preview": sum(int(v.get("share_previews") or 0) for v in nalg.values()) if nalg else None,
            "shares_via_r2": sum(int(v.get("share_gathered_first") or 0) for v in nalg.values()) if nalg else None,
            "reforms": sum(int(v.get("reforms") or 0) for v in nalg.values()) if nalg else None,
            "lost_ranks": sorted({r for v in nalg.values() for r in v.get("lost_ranks") or []}) if nalg else None,
            "node_backend": node.get("dist_backend"),
            "data_plane": dp.get("impl") or out["dist_backend"],
            # why it is not rccl-native at N > 1 (the probe's first failing rank, or the in-process init's error)
            "data_plane_note": _data_plane_note(dp),
            "comm_r1_p99_ms": p99("R1"),
            "comm_r2_p99_ms": p99("R2"),
            "comm_r3_p99_ms": p99("R3"),
            "comm_r2_dev_p99_ms": p99("R2_dev"),
            "comm_busbw_gbps": _r((comm.get("busbw") or {}).get("busbw_gbps")),
            # directed GPU pairs of this run by link type (KFD topology): what the bus bandwidth ran over
            "comm_links": _link_counts((comm.get("topology") or {}).get("links")),
            "comm_miner_rate_change_pct": comm.get("miner_rate_change_pct"),
            "sections_s": self._section_times(),
            "errors": _short_errors(errors),
        }


# HIP hardware queues for the bench process itself (read at HIP init, and by RCCL at communicator init). The native
# data plane's communicator brings streams of its own (RCCL's, the comm stream); at the runtime's default of 4
# queues per process the second search stream then shares a queue and its launches no longer overlap the first's:
# -0.25% on the headline, which 8 queues recover (profiles/r6/f_dataplane_ab/). Only this process: the value is
# dropped from the environment once HIP and the communicator are up, so the device processes, node and pool started
# later keep their own defaults.
BENCH_HW_QUEUES = "8"


def run_rank(args) -> int:
    from otedama_amd.parallel.guard import RankGuard, run_dir_for

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    run_dir = run_dir_for()
    # RCCL's messages into the run directory, where an error JSON reads them back, and never on stdout, whose last
    # line is the driver's (at N=1 an unset NCCL_DEBUG let RCCL print its version banner there)
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    os.environ.setdefault("NCCL_DEBUG_FILE", os.path.join(run_dir, "rccl.%h.%p.log"))
    bench = Bench(args, rank, world)
    prev = os.environ.get("GPU_MAX_HW_QUEUES")
    if not args.cpu_rehearsal and (prev is None or (prev.isdigit() and int(prev) < int(BENCH_HW_QUEUES))):
        os.environ["GPU_MAX_HW_QUEUES"] = BENCH_HW_QUEUES  # the box may export the runtime's default (4) explicitly
        bench.hw_queues_raised, bench.hw_queues_prev = True, prev
    bench.guard = RankGuard(rank, world, args.deadline, emit=bench.emit if rank == 0 else None, run_dir=run_dir)
    bench.guard.start(tee_stderr=world > 1)
    return bench.run()


if __name__ == "__main__":
    sys.exit(main())
