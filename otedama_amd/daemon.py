"""Background-service installation: systemd user unit, launchd agent, Windows sc.exe.

Parity: internal/daemon/service.go
  * ServiceFlags / Manager / NewManager ............... service.go:55-90
  * Install / Uninstall / Status per platform ......... service.go:93-132
  * systemd user unit with hardening + ReadWritePaths .. service.go:195-235
  * launchd plist (RunAtLoad, KeepAlive, log paths) .... service.go:289-323
  * sc.exe create/stop/delete/query .................... service.go:347-383
  * serviceArgv / quoting / xml escaping ................ service.go:394-455
  * injectable run_cmd and platform (test seams) ........ service.go:38,457-463
The service runs ``<python> -m otedama_amd run ...``; the systemd unit also
keeps the ROCm device nodes reachable and pins HSA_ENABLE_IPC_MODE_LEGACY=0
for multi-process RCCL.
"""
from __future__ import annotations

import os
import subprocess
import sys
from dataclasses import dataclass
from pathlib import Path

from otedama_amd.config import default_data_dir

SYSTEMD_UNIT_NAME = "otedama.service"
LAUNCHD_LABEL = "com.otedama.daemon"


class DaemonError(RuntimeError):
    pass


def _default_run_cmd(name: str, *args: str) -> None:
    res = subprocess.run([name, *args], capture_output=True, text=True)
    if res.returncode != 0:
        raise DaemonError(f"{name} {list(args)}: exit {res.returncode}: {res.stdout}{res.stderr}")


def _default_output(name: str, *args: str) -> tuple[str, bool]:
    try:
        res = subprocess.run([name, *args], capture_output=True, text=True)
    except OSError as exc:
        return str(exc), False
    return res.stdout, res.returncode == 0


run_cmd = _default_run_cmd      # test seam
cmd_output = _default_output    # test seam
platform = sys.platform         # test seam ("linux", "darwin", "win32")


@dataclass
class ServiceFlags:
    bitcoin_address: str = ""
    log_level: str = ""
    log_format: str = ""
    language: str = ""
    node_gpus: int = 0  # > 0: the service runs the multi-GPU node (`otedama node --gpus N`) instead of `otedama run`


@dataclass
class ServiceStatus:
    installed: bool = False
    running: bool = False
    pid: int = 0
    details: str = ""


_GO_ESCAPES = {"\\": "\\\\", '"': '\\"', "\a": "\\a", "\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r",
               "\t": "\\t", "\v": "\\v"}


def _go_quote(s: str) -> str:
    """Go's %q of a string: backslash escapes for quote, backslash and control characters; printable text
    (including non-ASCII) unchanged."""
    out = []
    for c in s:
        if c in _GO_ESCAPES:
            out.append(_GO_ESCAPES[c])
        elif ord(c) < 0x20 or ord(c) == 0x7F:
            out.append(f"\\x{ord(c):02x}")
        elif not c.isprintable():
            out.append(f"\\u{ord(c):04x}" if ord(c) <= 0xFFFF else f"\\U{ord(c):08x}")
        else:
            out.append(c)
    return '"' + "".join(out) + '"'


def quote_token(s: str) -> str:
    """service.go:436-441: a token with a space, tab or double quote is Go-quoted (both systemd ExecStart= and
    sc.exe binPath= accept C-style escapes); anything else is returned unchanged."""
    if any(c in s for c in ' \t"'):
        return _go_quote(s)
    return s


def xml_escape(s: str) -> str:
    return (s.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;").replace('"', "&quot;")
            .replace("'", "&apos;"))


class Manager:
    def __init__(self, config_path: str = "", data_dir: str = "", flags: ServiceFlags | None = None,
                 executable: str | None = None, home: str | None = None):
        self.executable = os.path.realpath(executable or sys.executable)
        self.config_path = config_path
        self.data_dir = data_dir
        self.flags = flags or ServiceFlags()
        self.home = home  # None: $HOME / the password database, as os.UserHomeDir

    # ------------------------------------------------------------------ argv
    def service_argv(self) -> list[str]:
        # the node's supervisor restarts lost ranks itself; the service manager restarts the supervisor
        argv = ["node", "--gpus", str(self.flags.node_gpus)] if self.flags.node_gpus > 0 else ["run"]
        if self.config_path:
            argv += ["--config", self.config_path]
        if self.data_dir:
            argv += ["--data-dir", self.data_dir]
        f = self.flags
        for flag, v in (("--bitcoin-address", f.bitcoin_address), ("--log-level", f.log_level),
                        ("--log-format", f.log_format), ("--language", f.language)):
            if v:
                argv += [flag, v]
        return argv

    def program_argv(self) -> list[str]:
        return [self.executable, "-m", "otedama_amd", *self.service_argv()]

    def service_args(self) -> str:
        return " ".join(quote_token(a) for a in self.program_argv()[1:])

    def _home(self) -> Path:
        home = self.home if self.home is not None else os.environ.get("HOME", "")
        if not home:
            raise DaemonError("daemon: home directory not set ($HOME is empty)")
        return Path(home)

    def _service_dir(self, *parts: str) -> Path:
        """~/<parts>, created (0755) if missing (service.go:139-149, 241-251)."""
        d = self._home().joinpath(*parts)
        try:
            d.mkdir(mode=0o755, parents=True, exist_ok=True)
        except OSError as exc:
            raise DaemonError(f"daemon: create {d}: {exc}") from exc
        return d

    # ------------------------------------------------------------------ systemd
    def systemd_unit_path(self) -> Path:
        return self._service_dir(".config", "systemd", "user") / SYSTEMD_UNIT_NAME

    def systemd_unit(self) -> str:
        data = self.data_dir or default_data_dir()
        rw = f"ReadWritePaths={quote_token(data)}\n" if data else ""
        return f"""[Unit]
Description=Otedama — MI355X mining engine
After=network-online.target
Wants=network-online.target

[Service]
Type=simple
ExecStart={quote_token(self.executable)} {self.service_args()}
Restart=on-failure
RestartSec=10s
StandardOutput=journal
StandardError=journal
SyslogIdentifier=otedama
Environment=HSA_ENABLE_IPC_MODE_LEGACY=0

# Security hardening (GPU device nodes /dev/kfd and /dev/dri stay reachable)
NoNewPrivileges=true
ProtectHome=read-only
PrivateTmp=true
{rw}
[Install]
WantedBy=default.target
"""

    # ------------------------------------------------------------------ launchd
    def launchd_plist_path(self) -> Path:
        return self._service_dir("Library", "LaunchAgents") / f"{LAUNCHD_LABEL}.plist"

    def launchd_log_dir(self) -> Path:
        """~/Library/Logs (per-user, not world-readable /tmp); /tmp only when the home directory is unknown or the
        Logs directory cannot be created (service.go:333-343)."""
        try:
            return self._service_dir("Library", "Logs")
        except DaemonError:
            return Path("/tmp")

    def launchd_plist(self) -> str:
        entries = "".join(f"\t\t<string>{xml_escape(a)}</string>\n" for a in self.program_argv() if a)
        logs = self.launchd_log_dir()
        return f"""<?xml version="1.0" encoding="UTF-8"?>
<!DOCTYPE plist PUBLIC "-//Apple//DTD PLIST 1.0//EN"
    "http://www.apple.com/DTDs/PropertyList-1.0.dtd">
<plist version="1.0">
<dict>
    <key>Label</key>
    <string>{LAUNCHD_LABEL}</string>
    <key>ProgramArguments</key>
    <array>
{entries}    </array>
    <key>RunAtLoad</key>
    <true/>
    <key>KeepAlive</key>
    <true/>
    <key>StandardOutPath</key>
    <string>{logs / 'otedama.log'}</string>
    <key>StandardErrorPath</key>
    <string>{logs / 'otedama.err'}</string>
</dict>
</plist>
"""

    # ------------------------------------------------------------------ ops
    def install(self) -> None:
        p = _platform()
        if p == "linux":
            try:
                path = self.systemd_unit_path()
            except DaemonError as exc:
                raise DaemonError(f"daemon: systemd unit dir: {exc}") from exc
            _write(path, self.systemd_unit(), "daemon: write systemd unit")
            _step("daemon: systemctl daemon-reload", "systemctl", "--user", "daemon-reload")
            _step("daemon: systemctl enable", "systemctl", "--user", "enable", "--now", SYSTEMD_UNIT_NAME)
        elif p == "darwin":
            path = self.launchd_plist_path()
            _write(path, self.launchd_plist(), "daemon: write plist")
            run_cmd("launchctl", "load", "-w", str(path))
        elif p == "windows":
            run_cmd("sc.exe", "create", "Otedama", "binPath=", f'"{self.executable}" {self.service_args()}',
                    "start=", "auto", "DisplayName=", "Otedama Mining Service")
        else:
            raise DaemonError(f"daemon: unsupported platform {p!r}")

    def uninstall(self) -> None:
        p = _platform()
        if p == "linux":
            try:
                run_cmd("systemctl", "--user", "disable", "--now", SYSTEMD_UNIT_NAME)
            except DaemonError:
                pass
            self.systemd_unit_path().unlink()
        elif p == "darwin":
            path = self.launchd_plist_path()
            try:
                run_cmd("launchctl", "unload", "-w", str(path))
            except DaemonError:
                pass
            path.unlink()
        elif p == "windows":
            try:
                run_cmd("sc.exe", "stop", "Otedama")
            except DaemonError:
                pass
            run_cmd("sc.exe", "delete", "Otedama")
        else:
            raise DaemonError(f"daemon: unsupported platform {p!r}")

    def status(self) -> ServiceStatus:
        p = _platform()
        if p == "linux":
            out, ok = cmd_output("systemctl", "--user", "is-active", SYSTEMD_UNIT_NAME)
            return ServiceStatus(_exists(self.systemd_unit_path), ok and out.strip() == "active", 0, out)
        if p == "darwin":
            out, ok = cmd_output("launchctl", "list", LAUNCHD_LABEL)
            return ServiceStatus(_exists(self.launchd_plist_path), ok and "Could not find" not in out, 0, out)
        if p == "windows":
            out, ok = cmd_output("sc.exe", "query", "Otedama")
            return ServiceStatus(ok, ok and "RUNNING" in out, 0, out) if ok else ServiceStatus()
        raise DaemonError(f"daemon: unsupported platform {p!r}")


def _exists(path_fn) -> bool:
    """Status never fails on an unknown home directory: the service is then simply not installed."""
    try:
        return path_fn().exists()
    except DaemonError:
        return False


def _write(path: Path, text: str, what: str) -> None:
    try:
        path.write_text(text)
        os.chmod(path, 0o644)
    except OSError as exc:
        raise DaemonError(f"{what}: {exc}") from exc


def _step(what: str, name: str, *args: str) -> None:
    try:
        run_cmd(name, *args)
    except DaemonError as exc:
        raise DaemonError(f"{what}: {exc}") from exc


def _platform() -> str:
    p = platform
    if p.startswith("win"):
        return "windows"
    if p.startswith("linux"):
        return "linux"
    return p
