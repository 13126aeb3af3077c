"""``otedama`` command-line interface.

Parity: cmd/otedama
  * dispatcher, exit codes 0/1/64/78, --help to stdout ......... main.go:49-169
  * run (15 flags, env fallbacks for wallet secrets, TUI auto-off
    when stdout is not a terminal, dry-run, SIGINT/SIGTERM,
    logger sink matrix, HTTP server) ............................ run.go:31-322
  * config show [--origin] [--json] / config validate .......... config.go:38-212
  * strict YAML config file discovery (--config, OTEDAMA_CONFIG,
    ~/.config/otedama/config.yaml) .............................. configfile.go:20-59
  * doctor / service / version / completion ...................... doctor.go, service.go,
                                                                  version.go, completion.go
MI355X additions: ``pool`` (run the local validating Stratum pool),
``bench`` (hash-rate benchmarks on CPU / GPU), ``devices`` (HAL listing).
"""
from __future__ import annotations

import json
import os
import sys
import unicodedata
from typing import TextIO

from otedama_amd.cli.flags import ErrHelp, FlagError, FlagSet, has_help_flag

EXIT_OK, EXIT_RUNTIME, EXIT_USAGE, EXIT_CONFIG = 0, 1, 64, 78

USAGE = """Otedama — MI355X mining engine, Stratum pool and compute arbitration.

Usage:
  otedama <command> [flags]

Commands:
  run        Start mining (gfx950 GPUs + CPU) against the configured pools.
  node       Run one rank per GPU under a fault-tolerant supervisor (RCCL node).
  pool       Run the local Stratum V1/V2 pool (share validation, vardiff).
  bench      Measure hash rates (sha256d / scrypt, CPU and GPU).
  devices    List detected mining devices.
  version    Print version information and exit.
  config     Inspect or validate the effective configuration.
  service    Install/uninstall as a background service.
  doctor     Run self-diagnostic checks.
  completion Generate a shell-completion script (bash|zsh|fish).
  help       Print this help and exit.

Getting started (zero-configuration):
  otedama run --bitcoin-address bc1q...

With Lightning wallet:
  otedama run --bitcoin-address bc1q... --wallet-passphrase "strong passphrase"

Exit codes:
  0   success
  1   runtime error (engine, network, I/O failure)
  64  usage error  (unknown flag or subcommand)
  78  config error (invalid address, bad log level, etc.)
  doctor uses 0=pass, 1=warn, 2=fail instead of the above.

Run 'otedama <command> --help' for per-command flags.
"""


def run_flagset(name: str, out: TextIO) -> FlagSet:
    fs = FlagSet(name, out)
    fs.string("bitcoin-address", "", "Bitcoin address for mining rewards (required).")
    fs.string("log-level", "", "Log level (debug|info|warn|error).")
    fs.string("language", "", "UI language as BCP 47 tag (e.g., ja, en, zh-CN).")
    fs.string("data-dir", "", "Directory for persistent data.")
    fs.string("config", "", "Path to config.yaml (optional).")
    fs.bool("dry-run", False, "(run only) Validate configuration and exit without starting.")
    fs.bool("no-tui", False, "(run only) Disable the terminal dashboard (plain log output).")
    fs.string("wallet-passphrase", "", "(run only) Passphrase to unlock/create the Lightning wallet. If empty, "
                                       "wallet is skipped.")
    fs.string("wallet-mnemonic-passphrase", "", "(run only) Optional BIP-39 \"25th word\" passphrase, applied only "
                                                "when a new wallet is created.")
    fs.string("log-format", "", "Log output format: text or json.")
    fs.string("log-file", "", "(run only) Append structured logs to this file (written even while the TUI is "
                              "active).")
    fs.string("http-addr", "", "Address for HTTP metrics/health endpoints (e.g. 127.0.0.1:9090). Empty disables.")
    fs.bool("pprof", False, "(run only) Mount /debug/pprof/ profiling (only on loopback/private addresses).")
    fs.bool("origin", False, "(config show only) Annotate each value with the layer that set it "
                             "(default/file/env/flag).")
    fs.bool("json", False, "(config show only) Emit the resolved configuration as a JSON object instead of text.")
    # MI355X additions
    fs.string("algorithm", "", "(run only) Proof-of-work algorithm: sha256d | scrypt | x11.")
    fs.string("gpus", "", "(run only) GPUs to mine on: all | none | comma-separated HIP ordinals.")
    fs.int("cpu-threads", -1, "(run only) CPU miner threads (0 = only when no GPU; -1 = config).")
    fs.bool("enable-ai-provider", False, "(run only) Enable the simulated AI-inference yield provider in "
                                         "arbitration.")
    return fs


def parse_subcommand(fs: FlagSet, args: list[str], stdout: TextIO, stderr: TextIO) -> int | None:
    fs.out = stdout if has_help_flag(args) else stderr
    try:
        fs.parse(args)
    except ErrHelp:
        return EXIT_OK
    except FlagError:
        return EXIT_USAGE
    return None


def load_config(fs: FlagSet, stderr: TextIO):
    from otedama_amd import config as C

    path = fs["config"] or C.default_config_path()
    cfg, warn = C.load_config_file(path)
    if warn:
        stderr.write(f"warning: {warn}\n")
    return cfg


def flag_values(fs: FlagSet):
    from otedama_amd.config import FlagValues

    return FlagValues(bitcoin_address=fs["bitcoin-address"], log_level=fs["log-level"], log_format=fs["log-format"],
                      language=fs["language"], data_dir=fs["data-dir"], http_addr=fs["http-addr"])


def safe_display(v: str) -> str:
    if not v:
        return "(default)"
    cleaned = "".join(ch for ch in v if unicodedata.category(ch) != "Cc")
    return cleaned or "(default)"


# ------------------------------------------------------------------ config
def cmd_config(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    if not args:
        stderr.write("otedama config: expected subcommand (show|validate)\n")
        return EXIT_USAGE
    sub, rest = args[0], args[1:]
    if sub == "show":
        return cmd_config_show(rest, stdout, stderr)
    if sub == "validate":
        return cmd_config_validate(rest, stdout, stderr)
    if sub in ("help", "--help", "-h"):
        stdout.write("otedama config: expected subcommand (show|validate)\n")
        return EXIT_OK
    stderr.write(f"otedama config: unknown subcommand {sub!r}\n")
    return EXIT_USAGE


def cmd_config_show(args, stdout, stderr) -> int:
    from otedama_amd import config as C

    fs = run_flagset("config show", stderr)
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    cfg, o = C.resolve_with_origins(load_config(fs, stderr), None, flag_values(fs))
    if fs["json"]:
        doc = {
            "bitcoin_address": cfg.bitcoin_address, "log_level": cfg.log_level, "log_format": cfg.log_format,
            "language": cfg.language, "data_dir": cfg.data_dir, "worker_name": cfg.workers.name,
            "arbitration_hysteresis_pct": cfg.arbitration_hysteresis_pct,
            "curtail_below_btc_usd": cfg.curtail_below_btc_usd, "min_yield_sats_per_sec": cfg.min_yield_sats_per_sec,
            "power_watts": cfg.power_watts, "electricity_price_per_kwh": cfg.electricity_price_per_kwh,
            "http_addr": cfg.http_addr, "pools": [p.url for p in cfg.pools],
            "mining": cfg.to_dict()["mining"], "pool_server": cfg.to_dict()["pool_server"],
        }
        if cfg.bitcoin_addresses:
            doc["bitcoin_addresses"] = cfg.bitcoin_addresses
        if fs["origin"]:
            doc["origins"] = {k: str(v) for k, v in o.items()}
        stdout.write(json.dumps(doc, indent=2, ensure_ascii=False) + "\n")
        return EXIT_OK

    def tag(k):
        return f" [{o[k]}]" if fs["origin"] else ""

    w = stdout.write
    w(f"bitcoin_address: {safe_display(cfg.bitcoin_address)}{tag('bitcoin_address')}\n")
    if cfg.bitcoin_addresses:
        w(f"bitcoin_addresses (failover): {len(cfg.bitcoin_addresses)}{tag('bitcoin_addresses')}\n")
        for i, a in enumerate(cfg.bitcoin_addresses):
            w(f"  [{i + 1}] {safe_display(a)}\n")
    w(f"log_level:       {cfg.log_level}{tag('log_level')}\n")
    w(f"log_format:      {cfg.log_format}{tag('log_format')}\n")
    w(f"language:        {safe_display(cfg.language)}{tag('language')}\n")
    w(f"data_dir:        {safe_display(cfg.data_dir)}{tag('data_dir')}\n")
    w(f"worker_name:     {safe_display(cfg.workers.name)}{tag('worker_name')}\n")
    from otedama_amd.metrics import format_float as g

    w(f"arbitration_hysteresis_pct: {g(cfg.arbitration_hysteresis_pct)}{tag('arbitration_hysteresis_pct')}\n")
    w(f"curtail_below_btc_usd:      {g(cfg.curtail_below_btc_usd)}{tag('curtail_below_btc_usd')}\n")
    w(f"min_yield_sats_per_sec:     {g(cfg.min_yield_sats_per_sec)}{tag('min_yield_sats_per_sec')}\n")
    w(f"power_watts:                {g(cfg.power_watts)}{tag('power_watts')}\n")
    w(f"electricity_price_per_kwh:  {g(cfg.electricity_price_per_kwh)}{tag('electricity_price_per_kwh')}\n")
    w(f"http_addr:                  {safe_display(cfg.http_addr)}{tag('http_addr')}\n")
    w(f"mining:                     algorithm={cfg.mining.algorithm} gpus={cfg.mining.gpus} "
      f"cpu_threads={cfg.mining.cpu_threads}{tag('mining')}\n")
    if not cfg.pools:
        w(f"pools:           (built-in default){tag('pools')}\n")
    else:
        w(f"pools:           {len(cfg.pools)} configured{tag('pools')}\n")
        for i, p in enumerate(cfg.pools):
            w(f"  [{i + 1}] {safe_display(p.url)}\n")
    return EXIT_OK


def cmd_config_validate(args, stdout, stderr) -> int:
    from otedama_amd import config as C

    fs = run_flagset("config validate", stderr)
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    file_cfg = load_config(fs, stderr)
    for w in C.env_warnings():
        stderr.write(f"config: warning: {w}\n")
    cfg = C.resolve(file_cfg, None, flag_values(fs))
    try:
        cfg.validate()
    except C.ConfigError as exc:
        stderr.write(f"{exc}\n")
        return EXIT_CONFIG
    stdout.write("configuration is valid\n")
    return EXIT_OK


# ------------------------------------------------------------------ version
def cmd_version(args, stdout, stderr) -> int:
    from otedama_amd import version

    fs = FlagSet("version", stderr)
    fs.bool("json", False, "Emit version information as JSON.")
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    info = version.get()
    if fs["json"]:
        stdout.write(json.dumps(info.to_dict(), indent=2) + "\n")
    else:
        stdout.write(str(info) + "\n")
    return EXIT_OK


# ------------------------------------------------------------------ dispatcher
COMMANDS = ("run", "node", "pool", "bench", "devices", "version", "config", "service", "doctor", "completion", "help")


def run(args: list[str], stdout: TextIO = sys.stdout, stderr: TextIO = sys.stderr) -> int:
    if not args:
        stderr.write(USAGE)
        return EXIT_USAGE
    cmd, rest = args[0], args[1:]
    if cmd == "run":
        from otedama_amd.cli.run_cmd import cmd_run

        return cmd_run(rest, stdout, stderr)
    if cmd == "node":
        from otedama_amd.cli.node_cmd import cmd_node

        return cmd_node(rest, stdout, stderr)
    if cmd == "pool":
        from otedama_amd.cli.pool_cmd import cmd_pool

        return cmd_pool(rest, stdout, stderr)
    if cmd == "bench":
        from otedama_amd.cli.bench_cmd import cmd_bench

        return cmd_bench(rest, stdout, stderr)
    if cmd == "devices":
        from otedama_amd.cli.bench_cmd import cmd_devices

        return cmd_devices(rest, stdout, stderr)
    if cmd in ("version", "--version", "-v"):
        return cmd_version(rest, stdout, stderr)
    if cmd == "config":
        return cmd_config(rest, stdout, stderr)
    if cmd == "service":
        from otedama_amd.cli.service_cmd import cmd_service

        return cmd_service(rest, stdout, stderr)
    if cmd == "doctor":
        from otedama_amd.cli.doctor_cmd import cmd_doctor

        return cmd_doctor(rest, stdout, stderr)
    if cmd == "completion":
        from otedama_amd.cli.completion import cmd_completion

        return cmd_completion(rest, stdout, stderr)
    if cmd in ("help", "--help", "-h"):
        stdout.write(USAGE)
        return EXIT_OK
    stderr.write(f"otedama: unknown subcommand {cmd!r}\n")
    stderr.write(USAGE)
    return EXIT_USAGE


def main() -> None:
    """Process entry point (``otedama`` / ``python -m otedama_amd``)."""
    if sys.argv[1:2] == ["pool"]:
        # the pool never touches a GPU: its native extension binds to the system HIP runtime without torch
        # (~1-2 s and ~500 MB less at start on a GPU host; ops/native.py)
        os.environ.setdefault("OTEDAMA_NO_TORCH", "1")
    sys.exit(run(sys.argv[1:]))


if __name__ == "__main__":
    main()


__all__ = ["run", "main", "EXIT_OK", "EXIT_RUNTIME", "EXIT_USAGE", "EXIT_CONFIG", "os"]
