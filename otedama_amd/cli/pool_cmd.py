"""``otedama pool`` — run the local validating Stratum pool [NO REFERENCE CODE].

One process can serve several algorithms (``--algorithms sha256d,scrypt``):
each gets its own SV2 + V1 listener pair (ports increment per algorithm), its
own vardiff / diff1 constant and share journal, and all publish into one
/metrics registry — the "mixed SHA-256d + scrypt workers" pool of BASELINE.json
config 5.

Settings come from flags, then the config file's ``pool_server`` section (plus ``http_addr``), then the flag
defaults: an explicitly given flag always wins.
"""
from __future__ import annotations

import asyncio
import json
import signal
from typing import TextIO

from otedama_amd.cli.flags import FlagSet
from otedama_amd.cli.main import EXIT_CONFIG, EXIT_OK, EXIT_RUNTIME, parse_subcommand


def _bump(addr: str, k: int) -> str:
    if not addr:
        return ""
    h, _, p = addr.rpartition(":")
    return f"{h}:{int(p) + k}" if p and int(p) else addr


def apply_config_file(fs: FlagSet, stderr: TextIO) -> None:
    """Fill every flag the user did not give from the config file's pool_server section."""
    from otedama_amd.cli.main import load_config

    cfg = load_config(fs, stderr)
    ps = cfg.pool_server
    pairs = (("algorithms", ps.algorithm), ("listen-sv2", ps.listen_sv2), ("listen-v1", ps.listen_v1),
             ("difficulty", ps.initial_difficulty), ("share-seconds", ps.target_share_seconds),
             ("retarget-seconds", ps.vardiff_retarget_seconds), ("journal", ps.journal_path),
             ("http-addr", cfg.http_addr))
    default = type(ps)()
    for flag, value in pairs:
        unset_in_file = flag != "http-addr" and value == getattr(default, _FILE_FIELD[flag])
        if flag in fs.set_flags or unset_in_file or value in ("", None):
            continue
        fs.values[flag] = value
    fs.values["coinbase-message"] = ps.coinbase_message


_FILE_FIELD = {"algorithms": "algorithm", "listen-sv2": "listen_sv2", "listen-v1": "listen_v1",
               "difficulty": "initial_difficulty", "share-seconds": "target_share_seconds",
               "retarget-seconds": "vardiff_retarget_seconds", "journal": "journal_path"}


def cmd_pool(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    fs = FlagSet("pool", stderr)
    fs.string("algorithms", "sha256d", "Comma-separated algorithms to serve (sha256d, scrypt, x11).")
    fs.string("listen-sv2", "127.0.0.1:3336", "Stratum V2 listen address (port +1 per extra algorithm).")
    fs.string("listen-v1", "127.0.0.1:3333", "Stratum V1 listen address (port +1 per extra algorithm).")
    fs.string("payout-address", "", "Operator address paid by the coinbase (empty = OP_RETURN).")
    fs.float("difficulty", 1.0, "Initial share difficulty.")
    fs.bool("fixed-difficulty", False, "Pin every connection at --difficulty (vardiff off).")
    fs.float("share-seconds", 10.0, "Vardiff target seconds between shares per connection.")
    fs.float("retarget-seconds", 30.0, "Vardiff retarget window.")
    fs.float("block-interval", 600.0, "Seconds between synthetic network blocks.")
    fs.float("job-interval", 30.0, "Seconds between job refreshes (new ntime).")
    fs.string("journal", "", "SQLite share journal path (empty = in-memory).")
    fs.string("payout-scheme", "pplns", "Block payout accounting: pplns | prop.")
    fs.string("http-addr", "", "Address for /metrics /healthz /api/v1/{pool,workers,blocks} (empty disables).")
    fs.string("dialect", "reference", "SV2 wire dialect: reference | spec.")
    fs.bool("sv2-noise", False, "Encrypt SV2 connections with Noise NX (miners pin the printed authority key).")
    fs.string("noise-suite", "", "Noise suites accepted: empty = both, ellswift (current SV2) or legacy.")
    fs.string("noise-authority-key", "", "Hex secp256k1 secret signing the Noise certificate (empty = fresh per run).")
    fs.float("duration", 0.0, "Stop after this many seconds (0 = run until signalled).")
    fs.string("config", "", "Path to the YAML config file (default: $OTEDAMA_CONFIG or ~/.config/otedama/config.yaml).")
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    apply_config_file(fs, stderr)
    algos = [a.strip() for a in fs["algorithms"].split(",") if a.strip()]
    for a in algos:
        if a not in ("sha256d", "scrypt", "x11"):
            stderr.write(f"pool: unsupported algorithm {a!r} (sha256d, scrypt, x11)\n")
            return EXIT_CONFIG
    if fs["payout-address"]:
        from otedama_amd.config import validate_bitcoin_address

        err = validate_bitcoin_address(fs["payout-address"])
        if err:
            stderr.write(f"pool: payout address invalid: {err}\n")
            return EXIT_CONFIG
    if fs["noise-suite"] not in ("", "ellswift", "legacy"):
        stderr.write("pool: --noise-suite must be ellswift or legacy (empty accepts both)\n")
        return EXIT_CONFIG
    if fs["noise-authority-key"]:
        from otedama_amd.btccrypto import N as CURVE_ORDER

        try:
            key = bytes.fromhex(fs["noise-authority-key"])
        except ValueError:
            key = b""
        if len(key) != 32 or not 0 < int.from_bytes(key, "big") < CURVE_ORDER:
            stderr.write("pool: --noise-authority-key must be 64 hex characters (a secp256k1 secret in [1, n))\n")
            return EXIT_CONFIG
    try:
        return asyncio.run(_serve(fs, algos, stdout))
    except OSError as exc:
        stderr.write(f"pool: {exc}\n")
        return EXIT_RUNTIME


async def _serve(fs, algos: list[str], stdout: TextIO) -> int:
    from otedama_amd.httpserver import HTTPServer
    from otedama_amd.metrics import Registry
    from otedama_amd.pool.server import PoolOptions, PoolServer

    reg = Registry()
    pools = []
    for k, algo in enumerate(algos):
        journal = fs["journal"]
        if journal and len(algos) > 1:
            journal = journal.replace(".db", f".{algo}.db") if journal.endswith(".db") else f"{journal}.{algo}"
        opts = PoolOptions(algorithm=algo, listen_sv2=_bump(fs["listen-sv2"], k), listen_v1=_bump(fs["listen-v1"], k),
                           payout_address=fs["payout-address"] or None, initial_difficulty=fs["difficulty"],
                           fixed_difficulty=fs["fixed-difficulty"],
                           target_share_seconds=fs["share-seconds"], retarget_seconds=fs["retarget-seconds"],
                           block_interval=fs["block-interval"], job_interval=fs["job-interval"],
                           journal_path=journal or ":memory:", payout_scheme=fs["payout-scheme"],
                           dialect=fs["dialect"], noise=fs["sv2-noise"], noise_suite=fs["noise-suite"],
                           coinbase_message=fs.values.get("coinbase-message", PoolOptions.coinbase_message),
                           noise_authority_secret=int(fs["noise-authority-key"] or "0", 16))

        def log(level, msg):
            stdout.write(f"[{level}] {msg}\n")
            stdout.flush()

        p = PoolServer(opts, reg, log)
        await p.start()
        pools.append(p)
    srv = None
    if fs["http-addr"]:
        srv = HTTPServer(fs["http-addr"], reg, api={"pool": lambda: [p.stats() for p in pools],
                                                    "stats": lambda: [p.stats() for p in pools],
                                                    "workers": lambda: [w for p in pools for w in p.workers()],
                                                    "blocks": lambda: [b for p in pools for b in p.blocks()]})
        srv.start()
        srv.set_ready(True)
        stdout.write(f"[info] http: listening on {srv.addr}\n")
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    try:  # SIGUSR1: a new network block now, on every algorithm (operators and probes test stale-work handling)
        loop.add_signal_handler(signal.SIGUSR1, lambda: [p.new_block() for p in pools])
    except (NotImplementedError, RuntimeError, AttributeError):
        pass
    if fs["duration"] > 0:
        loop.call_later(fs["duration"], stop.set)
    await stop.wait()
    for p in pools:  # the exit line carries the timed validation log too (windowed quantiles for probes)
        stdout.write(json.dumps(dict(p.stats(), validate_log=p.validate_log())) + "\n")
        await p.stop()
    if srv:
        srv.stop()
    return EXIT_OK
