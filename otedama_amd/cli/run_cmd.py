"""``otedama run`` (cmd/otedama/run.go:122-322)."""
from __future__ import annotations

import asyncio
import os
import signal
import sys
from typing import TextIO

from otedama_amd import i18n
from otedama_amd.cli.main import (
    EXIT_CONFIG,
    EXIT_OK,
    EXIT_RUNTIME,
    flag_values,
    load_config,
    parse_subcommand,
    run_flagset,
)


def _is_terminal(f) -> bool:
    try:
        return os.isatty(f.fileno())
    except (AttributeError, OSError, ValueError):
        return False


class _Tee:
    def __init__(self, *ws):
        self.ws = ws

    def write(self, s):
        for w in self.ws:
            w.write(s)
        return len(s)

    def flush(self):
        for w in self.ws:
            w.flush()


def build_logger(no_tui: bool, log_file: str, cfg, stdout: TextIO):
    """Sink matrix: TUI on/off x --log-file (cmd/otedama/run.go:251-303)."""
    from otedama_amd.utils import logger as L

    fw = None
    if log_file:
        try:
            fd = os.open(log_file, os.O_CREAT | os.O_WRONLY | os.O_APPEND, 0o600)
            fw = os.fdopen(fd, "a")
        except OSError as exc:
            sys.stderr.write(f"warning: cannot open --log-file {log_file!r}: {exc}\n")
    if not no_tui:
        if fw is None:
            return L.discard(), (lambda: None)
        w = fw
    elif fw is not None:
        w = _Tee(stdout, fw)
    else:
        w = stdout
    lg = L.new(L.parse_level(cfg.log_level), "json" if cfg.log_format == "json" else "text", w)
    return lg, (lambda: fw.close() if fw else None)


def cmd_run(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    from otedama_amd import config as C

    fs = run_flagset("run", stderr)
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    wallet_pass = fs["wallet-passphrase"] or os.environ.get("OTEDAMA_WALLET_PASSPHRASE", "")
    mnemonic_pass = fs["wallet-mnemonic-passphrase"] or os.environ.get("OTEDAMA_WALLET_MNEMONIC_PASSPHRASE", "")
    no_tui = fs["no-tui"] or not _is_terminal(stdout)
    file_cfg = load_config(fs, stderr)
    for w in C.env_warnings():
        stderr.write(f"config: warning: {w}\n")
    cfg = C.resolve(file_cfg, None, flag_values(fs))
    if fs["algorithm"]:
        cfg.mining.algorithm = fs["algorithm"]
    if fs["gpus"]:
        cfg.mining.gpus = fs["gpus"]
    if fs["cpu-threads"] >= 0:
        cfg.mining.cpu_threads = fs["cpu-threads"]
    try:
        cfg.validate()
    except C.ConfigError as exc:
        stderr.write(f"{exc}\n")
        return EXIT_CONFIG
    bundle = i18n.new_bundle()
    lang = i18n.detect_lang(cfg.language) if cfg.language else i18n.detect_lang_from_env()

    def logln(level: str, mid: str, data=None) -> None:
        stdout.write(f"[{level}] {bundle.render_with(lang, mid, data)}\n")
        stdout.flush()

    if fs["dry-run"]:
        stdout.write("dry-run: configuration is valid; would start run\n")
        return EXIT_OK
    node = None
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 and cfg.mining.isolation == "process":
        # the GPUs belong to device processes: this process never touches them, so it loads the native host
        # code without torch (start-up and RSS; ops/native.py)
        os.environ.setdefault("OTEDAMA_NO_TORCH", "1")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # node mode (otedama node / torchrun): one rank per GPU; rank 0 is the pool-facing engine. A rank the
        # supervisor restarted after a loss joins the running node instead of forming it.
        from otedama_amd.engine.run import mark_early
        from otedama_amd.parallel.rcclcomm import native_wanted, open_node_comm

        # On GPUs the ranks run the native RCCL data plane and never import torch (parallel/rcclcomm.py); gloo
        # rehearsals and CPU hosts use torch.distributed.
        if native_wanted():
            os.environ.setdefault("OTEDAMA_NO_TORCH", "1")
        mark_early("comm_open")
        # a replacement process: followers join the running node; rank 0 restarted by the supervisor takes the
        # node over as its leader (parallel/node.py NodeMinerSet._take_over)
        joining = os.environ.get("OTEDAMA_NODE_JOIN") == "1"
        info, comm = open_node_comm(joining, host_buffers=not native_wanted(),
                                    log=lambda m: (stdout.write(f"[warn] {m}\n"), stdout.flush()))
        mark_early("process_group_ready")
        # the rank's HIP ordinal (init_from_env maps local ranks onto the visible GPUs; on an 8-GPU node it is the
        # local rank, on a 1-GPU rehearsal over gloo every rank shares GPU 0)
        cfg.mining.gpus = str(info.device.index if info.device.type == "cuda" else info.local_rank)
        # equal device count per rank keeps the stripes disjoint: the rank's GPU, or (a CPU-only rehearsal node over
        # gloo) one CPU miner per rank
        cfg.mining.cpu_threads = 0 if info.device.type == "cuda" else max(1, cfg.mining.cpu_threads)
        if info.orig_rank > 0:
            return _run_node_worker(cfg, info, comm, stdout, joining)
        node = comm
        no_tui = True
    logln("info", i18n.STARTUP_READY)
    pool_url = cfg.pools[0].url if cfg.pools else C.DEFAULT_POOL_URL
    logln("info", i18n.STARTUP_POOL_CONNECTING, {"url": pool_url})
    structlog, close_log = build_logger(no_tui, fs["log-file"], cfg, stdout)
    try:
        return asyncio.run(_run_async(cfg, fs, no_tui, wallet_pass, mnemonic_pass, structlog, stdout, stderr, logln,
                                      node))
    finally:
        close_log()
        if node is not None:
            node.close()


def _run_node_worker(cfg, info, comm, stdout, joining: bool = False) -> int:
    """Ranks > 0 of a node: mine rank 0's jobs on the local GPU until rank 0 stops."""
    from otedama_amd import hal
    from otedama_amd.engine.miners import MinerSet
    from otedama_amd.parallel.node import NodeWorker

    on_gpu = info.device.type == "cuda"
    # the GPU's miner runs in a device process of its own (engine/devproc.py): a kernel fault kills that child, not
    # this rank and its RCCL communicator; the devices are named from the KFD topology
    isolation = cfg.mining.isolation
    devs = hal.Detector(hal.default_registry(cfg.mining.cpu_threads, gpu_free=isolation == "process")).detect()
    gpu = info.device.index if on_gpu else info.local_rank
    if on_gpu:
        devs = [d for d in devs if d.identity().family == hal.Family.GPU and d.index == gpu]
    else:  # CPU-only rehearsal node: this rank's CPU miner
        devs = [d for d in devs if d.identity().family == hal.Family.CPU]
    local = MinerSet(devs, cfg.mining.algorithm, cfg.mining.batch_nonces, 0 if on_gpu else cfg.mining.cpu_threads,
                     rank=max(info.rank, 0), world_size=max(info.world_size, 1), sha_variants=cfg.mining.sha_variants,
                     isolation=isolation, log=lambda lvl, msg: stdout.write(f"[{lvl}] {msg}\n"))
    stdout.write(f"[info] node: rank {info.orig_rank} {'joining' if joining else f'of {info.world_size}'} mining on "
                 f"GPU {gpu} ({len(local)} device(s))\n")
    try:
        def wlog(lvl: str, msg: str) -> None:  # flushed: a follower's log must survive its SIGKILL
            stdout.write(f"[{lvl}] {msg}\n")
            stdout.flush()

        NodeWorker(local, comm, log=wlog, joining=joining).run()
    finally:
        comm.close()
    return EXIT_OK


async def _run_async(cfg, fs, no_tui, wallet_pass, mnemonic_pass, structlog, stdout, stderr, logln, node=None) -> int:
    from otedama_amd.engine.run import Engine, Options
    from otedama_amd.httpserver import HTTPServer
    from otedama_amd.metrics import Registry

    reg = Registry()
    srv = None
    dashboard = None
    if not no_tui:
        from otedama_amd.tui import Dashboard

        dashboard = Dashboard(stdout)
        import shutil

        dashboard.set_width(shutil.get_terminal_size((80, 24)).columns)  # not pinned to 80 (tui/dashboard.go:545)
    eng_holder: dict = {}
    if cfg.http_addr:
        srv = HTTPServer(cfg.http_addr, reg, fs["pprof"], api={
            "stats": lambda: eng_holder["e"].stats() if "e" in eng_holder else {},
            "devices": lambda: eng_holder["e"].device_list() if "e" in eng_holder else [],
            "debug_stats": lambda: eng_holder["e"].debug_stats() if "e" in eng_holder else {},
            "node": lambda: eng_holder["e"].node_status() if "e" in eng_holder else {},
        })
        try:
            srv.start()
            stdout.write(f"[info] http: listening on {srv.addr}\n")
            stdout.flush()
        except OSError as exc:
            stderr.write(f"warning: cannot start HTTP server: {exc}\n")
            srv = None
    engine = Engine(Options(config=cfg, output=stdout, logger=structlog.adapter(), no_tui=no_tui,
                            wallet_passphrase=wallet_pass, wallet_mnemonic_passphrase=mnemonic_pass, metrics=reg,
                            on_ready=(srv.set_ready if srv else None), enable_ai_provider=fs["enable-ai-provider"],
                            dashboard=dashboard, node_comm=node))
    eng_holder["e"] = engine
    loop = asyncio.get_running_loop()
    task = asyncio.ensure_future(engine.run())
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, task.cancel)
        except (NotImplementedError, RuntimeError):
            pass
    rc = EXIT_OK
    try:
        await task
    except asyncio.CancelledError:
        pass
    except Exception as exc:  # noqa: BLE001
        structlog.error("engine", error=str(exc))
        stdout.write(f"[error] {exc}\n")
        rc = EXIT_RUNTIME
    finally:
        if srv is not None:
            srv.stop()
    if rc == EXIT_OK:
        logln("info", i18n.STATUS_SHUTTING_DOWN)
    return rc
