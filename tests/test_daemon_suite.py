"""internal/daemon/service_test.go, case by case, for what test_daemon.py does not pin already: unit/plist paths
(home unset, directory creation, mkdir and write failures), the unit and plist contents one property at a time,
argv quoting with spaces, symlink resolution, the per-step error wrapping of install, and every platform's
install / uninstall / status through the run_cmd / cmd_output / platform seams."""
from __future__ import annotations

import os
import stat
import xml.etree.ElementTree as ET

import pytest

from otedama_amd import daemon as D

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


@pytest.fixture
def fake(monkeypatch):
    """Records every command; ``fail`` maps a command prefix to the error run_cmd raises for it; ``out`` maps a
    command to the (stdout, ok) cmd_output returns."""

    class F:
        log: list = []
        fail: dict = {}
        out: dict = {}

    F.log, F.fail, F.out = [], {}, {}

    def run_cmd(name, *args):
        F.log.append((name, *args))
        for prefix, err in F.fail.items():
            if (name, *args)[:len(prefix)] == prefix:
                raise err

    def cmd_output(name, *args):
        F.log.append((name, *args))
        return F.out.get((name, *args), ("", False))

    monkeypatch.setattr(D, "run_cmd", run_cmd)
    monkeypatch.setattr(D, "cmd_output", cmd_output)
    return F


def mgr(tmp_path, home="home", exe=None, config="", data_dir=None, **flags):
    if exe is None:
        exe = "/opt/otd/bin/python3"  # does not exist: realpath leaves it unchanged
    return D.Manager(config, str(tmp_path / "data") if data_dir is None else data_dir, D.ServiceFlags(**flags),
                     executable=exe, home=None if home is None else str(tmp_path / home))


# ------------------------------------------------------------------ paths
def test_systemd_unit_path_uses_user_config_and_creates_directory(tmp_path):
    p = mgr(tmp_path).systemd_unit_path()
    assert p == tmp_path / "home" / ".config" / "systemd" / "user" / "otedama.service"
    assert p.parent.is_dir() and stat.S_IMODE(p.parent.stat().st_mode) & 0o755 == 0o755


def test_systemd_unit_path_errors_when_home_unset(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", "")
    with pytest.raises(D.DaemonError):
        mgr(tmp_path, home=None).systemd_unit_path()


def test_launchd_plist_path_uses_library_launch_agents(tmp_path):
    p = mgr(tmp_path).launchd_plist_path()
    assert p == tmp_path / "home" / "Library" / "LaunchAgents" / "com.otedama.daemon.plist" and p.parent.is_dir()


def test_launchd_plist_path_errors_when_home_unset(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", "")
    with pytest.raises(D.DaemonError):
        mgr(tmp_path, home=None).launchd_plist_path()


def test_home_defaults_to_env(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", str(tmp_path / "envhome"))
    assert str(mgr(tmp_path, home=None).systemd_unit_path()).startswith(str(tmp_path / "envhome"))


@pytest.mark.parametrize("which", ["systemd_unit_path", "launchd_plist_path"])
def test_path_mkdir_error(tmp_path, which):
    (tmp_path / "home").write_text("a file where the home directory should be")
    with pytest.raises(D.DaemonError):
        getattr(mgr(tmp_path), which)()


# ------------------------------------------------------------------ systemd unit
def test_systemd_unit_has_security_hardening(tmp_path):
    u = mgr(tmp_path).systemd_unit()
    for line in ("NoNewPrivileges=true", "ProtectHome=read-only", "PrivateTmp=true"):
        assert line in u.splitlines()


def test_systemd_unit_read_write_paths_match_data_dir(tmp_path):
    u = mgr(tmp_path, data_dir="/srv/otedama data").systemd_unit()
    assert 'ReadWritePaths="/srv/otedama data"' in u.splitlines()
    u = mgr(tmp_path, data_dir="/srv/otd").systemd_unit()
    assert "ReadWritePaths=/srv/otd" in u.splitlines()


def test_systemd_unit_restart_network_target_and_args(tmp_path):
    u = mgr(tmp_path, bitcoin_address=ADDR).systemd_unit().splitlines()
    assert "Restart=on-failure" in u and "RestartSec=10s" in u
    assert "After=network-online.target" in u and "Wants=network-online.target" in u
    assert "WantedBy=default.target" in u  # user target, not multi-user
    exec_start = next(line for line in u if line.startswith("ExecStart="))
    assert exec_start.startswith("ExecStart=/opt/otd/bin/python3 -m otedama_amd run ") and ADDR in exec_start
    for field in ("[Unit]", "[Service]", "[Install]", "Type=simple", "SyslogIdentifier=otedama"):
        assert field in u


def test_systemd_unit_quotes_binary_path_with_spaces_only(tmp_path):
    exe = tmp_path / "John Doe" / "python3"
    exe.parent.mkdir()
    exe.write_text("")
    u = mgr(tmp_path, exe=str(exe)).systemd_unit()
    assert f'ExecStart="{exe}" -m otedama_amd run' in u
    u = mgr(tmp_path).systemd_unit()
    assert "ExecStart=/opt/otd/bin/python3 -m" in u and 'ExecStart="' not in u


# ------------------------------------------------------------------ launchd plist
def _plist(m) -> ET.Element:
    text = m.launchd_plist()
    return ET.fromstring(text[text.index("<plist"):])


def test_launchd_plist_is_valid_xml_with_label_run_at_load_and_logs(tmp_path):
    m = mgr(tmp_path)
    d = _plist(m).find("dict")
    keys = [k.text for k in d.findall("key")]
    assert keys == ["Label", "ProgramArguments", "RunAtLoad", "KeepAlive", "StandardOutPath", "StandardErrorPath"]
    vals = list(d)
    assert vals[keys.index("Label") * 2 + 1].text == "com.otedama.daemon"
    assert vals[keys.index("RunAtLoad") * 2 + 1].tag == "true"
    out = vals[keys.index("StandardOutPath") * 2 + 1].text
    err = vals[keys.index("StandardErrorPath") * 2 + 1].text
    logs = str(tmp_path / "home" / "Library" / "Logs")
    assert out == os.path.join(logs, "otedama.log") and err == os.path.join(logs, "otedama.err")


def test_launchd_logs_fall_back_to_tmp_without_home(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", "")
    assert "<string>/tmp/otedama.log</string>" in mgr(tmp_path, home=None).launchd_plist()


def test_launchd_program_arguments_keep_spaces_as_one_string(tmp_path):
    m = mgr(tmp_path, config="/Users/John Doe/config & more.yaml")
    args = [s.text for s in _plist(m).find("dict").find("array")]
    assert args[:4] == ["/opt/otd/bin/python3", "-m", "otedama_amd", "run"]
    assert "/Users/John Doe/config & more.yaml" in args  # unescaped by the parser: one element, intact


def test_launchd_plist_skips_empty_binary_path(tmp_path):
    m = mgr(tmp_path)
    m.executable = ""
    args = [s.text for s in _plist(m).find("dict").find("array")]
    assert args and all(args) and args[0] == "-m"


# ------------------------------------------------------------------ argv
def test_service_args_start_with_run_and_quote_spaces(tmp_path):
    m = mgr(tmp_path, config="/home/John Doe/otedama.yaml", data_dir="")
    assert m.service_argv()[0] == "run"
    assert m.service_args().endswith('run --config "/home/John Doe/otedama.yaml"')


def test_service_args_empty_config_and_data_dir_omitted(tmp_path):
    assert mgr(tmp_path, data_dir="").service_argv() == ["run"]


def test_service_args_include_config_data_dir_and_every_flag(tmp_path):
    m = mgr(tmp_path, config="/c.yaml", data_dir="/d", bitcoin_address=ADDR, log_level="debug", log_format="json",
            language="ja")
    assert m.service_argv() == ["run", "--config", "/c.yaml", "--data-dir", "/d", "--bitcoin-address", ADDR,
                                "--log-level", "debug", "--log-format", "json", "--language", "ja"]


def test_service_argv_preserves_values_with_spaces(tmp_path):
    m = mgr(tmp_path, config="/a b/c d.yaml")
    assert "/a b/c d.yaml" in m.service_argv()


# ------------------------------------------------------------------ manager
def test_new_manager_resolves_symlinks(tmp_path):
    real = tmp_path / "real-python"
    real.write_text("")
    link = tmp_path / "link-python"
    link.symlink_to(real)
    assert D.Manager(executable=str(link), home=str(tmp_path)).executable == str(real)


def test_new_manager_defaults_to_the_running_interpreter():
    import sys

    assert D.Manager().executable == os.path.realpath(sys.executable)


def test_service_status_zero_value_is_not_running():
    s = D.ServiceStatus()
    assert not s.installed and not s.running and s.pid == 0 and s.details == ""


def test_default_run_cmd(tmp_path):
    D._default_run_cmd("true")
    with pytest.raises(D.DaemonError):
        D._default_run_cmd("false")


# ------------------------------------------------------------------ linux
def test_install_systemd_writes_unit_and_calls_systemctl_twice(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path)
    m.install()
    assert fake.log == [("systemctl", "--user", "daemon-reload"),
                        ("systemctl", "--user", "enable", "--now", "otedama.service")]
    p = m.systemd_unit_path()
    assert p.read_text() == m.systemd_unit() and stat.S_IMODE(p.stat().st_mode) == 0o644


@pytest.mark.parametrize("step,msg", [(("systemctl", "--user", "daemon-reload"), "daemon-reload"),
                                      (("systemctl", "--user", "enable"), "systemctl enable")])
def test_install_systemd_step_errors_are_wrapped(tmp_path, fake, monkeypatch, step, msg):
    monkeypatch.setattr(D, "platform", "linux")
    fake.fail[step] = D.DaemonError("boom")
    with pytest.raises(D.DaemonError, match=msg):
        mgr(tmp_path).install()


def test_install_systemd_unit_path_error(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    (tmp_path / "home").write_text("")
    with pytest.raises(D.DaemonError, match="systemd unit dir"):
        mgr(tmp_path).install()
    assert fake.log == []


def test_install_systemd_write_file_error(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path)
    m.systemd_unit_path().mkdir()  # a directory where the unit file goes
    with pytest.raises(D.DaemonError, match="write systemd unit"):
        m.install()
    assert fake.log == []


def test_uninstall_systemd_success_and_file_not_found(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path)
    m.install()
    fake.log.clear()
    m.uninstall()
    assert fake.log == [("systemctl", "--user", "disable", "--now", "otedama.service")]
    assert not m.systemd_unit_path().exists()
    with pytest.raises(FileNotFoundError):
        m.uninstall()


def test_uninstall_systemd_unit_path_error(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    (tmp_path / "home").write_text("")
    with pytest.raises(D.DaemonError):
        mgr(tmp_path).uninstall()


def test_status_systemd(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path)
    assert m.status() == D.ServiceStatus(False, False, 0, "")
    m.install()
    fake.out[("systemctl", "--user", "is-active", "otedama.service")] = ("active\n", True)
    s = m.status()
    assert s.installed and s.running and s.details == "active\n"


def test_status_without_home_is_not_installed(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    monkeypatch.setenv("HOME", "")
    assert not mgr(tmp_path, home=None).status().installed


# ------------------------------------------------------------------ darwin
def test_install_launchd_calls_launchctl(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "darwin")
    m = mgr(tmp_path)
    m.install()
    p = m.launchd_plist_path()
    assert fake.log == [("launchctl", "load", "-w", str(p))] and p.read_text() == m.launchd_plist()


def test_install_launchd_run_cmd_error(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "darwin")
    fake.fail[("launchctl",)] = D.DaemonError("launchctl failed")
    with pytest.raises(D.DaemonError, match="launchctl failed"):
        mgr(tmp_path).install()


def test_install_launchd_plist_path_and_write_errors(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "darwin")
    m = mgr(tmp_path)
    m.launchd_plist_path().mkdir()
    with pytest.raises(D.DaemonError, match="write plist"):
        m.install()
    (tmp_path / "home2").write_text("")
    with pytest.raises(D.DaemonError):
        mgr(tmp_path, home="home2").install()
    with pytest.raises(D.DaemonError):
        mgr(tmp_path, home="home2").uninstall()
    assert fake.log == []


def test_uninstall_and_status_launchd(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "darwin")
    m = mgr(tmp_path)
    m.install()
    fake.fail[("launchctl", "unload")] = D.DaemonError("not loaded")  # ignored
    fake.out[("launchctl", "list", "com.otedama.daemon")] = ('{ "PID" = 42; }', True)
    s = m.status()
    assert s.installed and s.running
    m.uninstall()
    assert not m.launchd_plist_path().exists()
    fake.out[("launchctl", "list", "com.otedama.daemon")] = ("Could not find service", True)
    assert m.status() == D.ServiceStatus(False, False, 0, "Could not find service")


# ------------------------------------------------------------------ windows
def test_install_windows_service_calls_sc_exe(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "win32")
    m = mgr(tmp_path, bitcoin_address=ADDR)
    m.install()
    (cmd,) = fake.log
    assert cmd[:3] == ("sc.exe", "create", "Otedama") and cmd[3] == "binPath="
    assert cmd[4] == f'"/opt/otd/bin/python3" {m.service_args()}'
    assert cmd[5:] == ("start=", "auto", "DisplayName=", "Otedama Mining Service")


def test_install_windows_service_error(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "win32")
    fake.fail[("sc.exe", "create")] = D.DaemonError("access denied")
    with pytest.raises(D.DaemonError, match="access denied"):
        mgr(tmp_path).install()


def test_uninstall_windows_stop_error_ignored_delete_error_raised(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "win32")
    fake.fail[("sc.exe", "stop")] = D.DaemonError("not running")
    mgr(tmp_path).uninstall()
    assert fake.log == [("sc.exe", "stop", "Otedama"), ("sc.exe", "delete", "Otedama")]
    fake.fail[("sc.exe", "delete")] = D.DaemonError("no such service")
    with pytest.raises(D.DaemonError, match="no such service"):
        mgr(tmp_path).uninstall()


def test_status_windows_service(tmp_path, fake, monkeypatch):
    monkeypatch.setattr(D, "platform", "win32")
    fake.out[("sc.exe", "query", "Otedama")] = ("STATE : 4 RUNNING", True)
    s = mgr(tmp_path).status()
    assert s.installed and s.running
    fake.out[("sc.exe", "query", "Otedama")] = ("STATE : 1 STOPPED", True)
    s = mgr(tmp_path).status()
    assert s.installed and not s.running


def test_status_windows_sc_exe_not_found_is_not_installed(tmp_path, monkeypatch):
    monkeypatch.setattr(D, "platform", "win32")
    monkeypatch.setattr(D, "cmd_output", D._default_output)
    monkeypatch.setenv("PATH", str(tmp_path))  # no sc.exe anywhere
    assert mgr(tmp_path).status() == D.ServiceStatus()


# ------------------------------------------------------------------ dispatch
@pytest.mark.parametrize("plat", ["freebsd", "plan9", "aix"])
@pytest.mark.parametrize("op", ["install", "uninstall", "status"])
def test_unsupported_platform(tmp_path, fake, monkeypatch, plat, op):
    monkeypatch.setattr(D, "platform", plat)
    with pytest.raises(D.DaemonError, match="unsupported platform"):
        getattr(mgr(tmp_path), op)()
    assert fake.log == []


@pytest.mark.parametrize("plat,tool", [("linux", "systemctl"), ("darwin", "launchctl"), ("win32", "sc.exe")])
def test_dispatch_by_platform(tmp_path, fake, monkeypatch, plat, tool):
    monkeypatch.setattr(D, "platform", plat)
    m = mgr(tmp_path)
    m.install()
    m.status()
    m.uninstall()
    assert fake.log and {c[0] for c in fake.log} == {tool}
