"""``otedama service install|uninstall|status`` (cmd/otedama/service.go:15-113)."""
from __future__ import annotations

from typing import TextIO

from otedama_amd import daemon
from otedama_amd.cli.flags import FlagSet
from otedama_amd.cli.main import EXIT_OK, EXIT_RUNTIME, EXIT_USAGE, parse_subcommand

# injectable seams (cmd/otedama/service.go:15-18)
new_daemon_manager = daemon.Manager
manager_install = lambda m: m.install()  # noqa: E731
manager_uninstall = lambda m: m.uninstall()  # noqa: E731
manager_status = lambda m: m.status()  # noqa: E731

USAGE = "otedama service: expected subcommand (install|uninstall|status)\n"


def cmd_service(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    if not args:
        stderr.write(USAGE)
        return EXIT_USAGE
    sub = args[0]
    if sub == "install":
        return _install(args[1:], stdout, stderr)
    if sub == "uninstall":
        return _simple(manager_uninstall, "uninstall", stdout, stderr)
    if sub == "status":
        return _status(stdout, stderr)
    if sub in ("help", "--help", "-h"):
        stdout.write(USAGE)
        return EXIT_OK
    stderr.write(f"otedama service: unknown subcommand {sub!r}\n")
    return EXIT_USAGE


def _install(args, stdout, stderr) -> int:
    fs = FlagSet("service install", stderr)
    fs.string("config", "", "Path to config.yaml for the service.")
    fs.string("data-dir", "", "Data directory for the service.")
    fs.string("bitcoin-address", "", "Payout address to embed in the service definition (required when no "
                                     "config file is specified).")
    fs.string("log-level", "", "Log level for the service (debug|info|warn|error).")
    fs.string("log-format", "", "Log format for the service (text|json).")
    fs.string("language", "", "UI language for the service (en, ja, ...).")
    fs.int("node-gpus", 0, "Run the multi-GPU node (one rank per GPU over RCCL) on this many GPUs instead of "
                           "`otedama run`.")
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    try:
        if fs["node-gpus"] < 0:
            stderr.write("service install: --node-gpus must be >= 0\n")
            return EXIT_USAGE
        mgr = new_daemon_manager(fs["config"], fs["data-dir"], daemon.ServiceFlags(
            fs["bitcoin-address"], fs["log-level"], fs["log-format"], fs["language"], fs["node-gpus"]))
    except Exception as exc:  # noqa: BLE001
        stderr.write(f"service: {exc}\n")
        return EXIT_RUNTIME
    try:
        manager_install(mgr)
    except Exception as exc:  # noqa: BLE001
        stderr.write(f"service install failed: {exc}\n")
        return EXIT_RUNTIME
    stdout.write("Otedama service installed and started.\nIt will start automatically on login.\n")
    return EXIT_OK


def _simple(fn, what, stdout, stderr) -> int:
    try:
        mgr = new_daemon_manager("", "", daemon.ServiceFlags())
    except Exception as exc:  # noqa: BLE001
        stderr.write(f"service: {exc}\n")
        return EXIT_RUNTIME
    try:
        fn(mgr)
    except Exception as exc:  # noqa: BLE001
        stderr.write(f"service {what} failed: {exc}\n")
        return EXIT_RUNTIME
    stdout.write("Otedama service uninstalled.\n")
    return EXIT_OK


def _status(stdout, stderr) -> int:
    try:
        mgr = new_daemon_manager("", "", daemon.ServiceFlags())
        st = manager_status(mgr)
    except Exception as exc:  # noqa: BLE001
        stderr.write(f"service status: {exc}\n")
        return EXIT_RUNTIME
    if st.installed:
        stdout.write(f"Otedama service: installed, {'running' if st.running else 'stopped'}\n")
    else:
        stdout.write("Otedama service: not installed\nRun 'otedama service install' to install.\n")
    return EXIT_OK
