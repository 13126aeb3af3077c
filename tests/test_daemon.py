"""Service manager: argv composition, quoting / XML escaping, systemd unit, launchd plist, sc.exe commands and
install / uninstall / status on each platform through the run_cmd / cmd_output / platform seams.

Mirrors internal/daemon/service_test.go (TestServiceArgv_*, TestQuoteToken_*, TestSystemdUnit_*,
TestLaunchdPlist_*, TestInstall*/TestUninstall*/TestStatus* with the runCmd and goos fakes).
"""
from __future__ import annotations

import xml.etree.ElementTree as ET

import pytest

from otedama_amd import daemon as D

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


class _Log(list):
    outputs: dict


@pytest.fixture
def calls(monkeypatch):
    log = _Log()
    outputs = {}

    def run_cmd(name, *args):
        log.append((name, *args))
        if (name, *args) in outputs and isinstance(outputs[(name, *args)], Exception):
            raise outputs[(name, *args)]

    def cmd_output(name, *args):
        log.append((name, *args))
        return outputs.get((name, *args), ("", False))

    monkeypatch.setattr(D, "run_cmd", run_cmd)
    monkeypatch.setattr(D, "cmd_output", cmd_output)
    log.outputs = outputs
    return log


def mgr(tmp_path, **kw):
    return D.Manager(kw.pop("config", ""), kw.pop("data_dir", str(tmp_path / "data")),
                     D.ServiceFlags(**kw), executable="/usr/bin/python3", home=str(tmp_path / "home"))


# ------------------------------------------------------------------ argv / quoting
def test_service_argv_includes_only_set_flags(tmp_path):
    m = mgr(tmp_path, config="/etc/otd.yaml", bitcoin_address=ADDR, log_level="debug")
    assert m.service_argv() == ["run", "--config", "/etc/otd.yaml", "--data-dir", str(tmp_path / "data"),
                                "--bitcoin-address", ADDR, "--log-level", "debug"]
    m2 = D.Manager(executable="/usr/bin/python3", home=str(tmp_path))
    assert m2.service_argv() == ["run"]
    assert m2.program_argv()[:3] == [m2.executable, "-m", "otedama_amd"]


def test_node_service_runs_the_supervisor(tmp_path):
    m = mgr(tmp_path, config="/etc/otd.yaml", bitcoin_address=ADDR, node_gpus=8)
    assert m.service_argv()[:3] == ["node", "--gpus", "8"]
    assert m.service_argv()[3:] == ["--config", "/etc/otd.yaml", "--data-dir", str(tmp_path / "data"),
                                    "--bitcoin-address", ADDR]
    assert f"ExecStart={m.executable} -m otedama_amd node --gpus 8 --config /etc/otd.yaml" in m.systemd_unit()


def test_all_flags_in_order(tmp_path):
    m = mgr(tmp_path, bitcoin_address=ADDR, log_level="warn", log_format="json", language="ja")
    argv = m.service_argv()
    assert argv[-8:] == ["--bitcoin-address", ADDR, "--log-level", "warn", "--log-format", "json", "--language", "ja"]


@pytest.mark.parametrize("s,want", [("plain", "plain"), ("with space", '"with space"'), ('q"uote', '"q\\"uote"'),
                                    ("tab\there", '"tab\\there"'), ('a b\\c', '"a b\\\\c"'), ("", "")])
def test_quote_token(s, want):
    assert D.quote_token(s) == want


@pytest.mark.parametrize("s,want", [("a&b", "a&amp;b"), ("<x>", "&lt;x&gt;"), ('"\'', "&quot;&apos;"), ("ok", "ok")])
def test_xml_escape(s, want):
    assert D.xml_escape(s) == want


# ------------------------------------------------------------------ systemd
def test_systemd_unit_contents(tmp_path):
    m = mgr(tmp_path, data_dir=str(tmp_path / "my data"), bitcoin_address=ADDR)
    u = m.systemd_unit()
    assert u.startswith("[Unit]\nDescription=Otedama")
    assert "After=network-online.target\nWants=network-online.target\n" in u
    assert (f"ExecStart={m.executable} -m otedama_amd run --data-dir \"{tmp_path / 'my data'}\" "
            f"--bitcoin-address {ADDR}\n") in u
    for line in ("Type=simple", "Restart=on-failure", "RestartSec=10s", "StandardOutput=journal",
                 "SyslogIdentifier=otedama", "NoNewPrivileges=true", "ProtectHome=read-only", "PrivateTmp=true",
                 "Environment=HSA_ENABLE_IPC_MODE_LEGACY=0", "WantedBy=default.target"):
        assert line + "\n" in u
    assert f'ReadWritePaths="{tmp_path / "my data"}"\n' in u  # the wallet dir stays writable under ProtectHome


def test_systemd_unit_defaults_the_data_dir_carve_out(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.delenv("XDG_DATA_HOME", raising=False)
    m = D.Manager(executable="/usr/bin/python3", home=str(tmp_path))
    assert f"ReadWritePaths={tmp_path}/.local/share/otedama\n" in m.systemd_unit()


def test_systemd_unit_path(tmp_path):
    assert mgr(tmp_path).systemd_unit_path() == tmp_path / "home" / ".config" / "systemd" / "user" / "otedama.service"


# ------------------------------------------------------------------ launchd
def test_launchd_plist_is_valid_xml_with_escaped_arguments(tmp_path):
    m = mgr(tmp_path, data_dir=str(tmp_path / "a&b <c>"), bitcoin_address=ADDR)
    plist = m.launchd_plist()
    root = ET.fromstring(plist.split("\n", 3)[3])  # skip the XML declaration / DOCTYPE lines
    d = root.find("dict")
    keys = [k.text for k in d.findall("key")]
    assert keys == ["Label", "ProgramArguments", "RunAtLoad", "KeepAlive", "StandardOutPath", "StandardErrorPath"]
    args = [s.text for s in d.find("array").findall("string")]
    assert args == m.program_argv() and str(tmp_path / "a&b <c>") in args
    assert d.findall("string")[0].text == D.LAUNCHD_LABEL
    assert plist.count("<true/>") == 2 and "Library/Logs/otedama.log" in plist


def test_launchd_plist_path(tmp_path):
    assert mgr(tmp_path).launchd_plist_path() == tmp_path / "home" / "Library" / "LaunchAgents" / \
        "com.otedama.daemon.plist"


# ------------------------------------------------------------------ install / uninstall / status
def test_linux_install_writes_the_unit_and_enables_it(tmp_path, calls, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path, bitcoin_address=ADDR)
    m.install()
    assert m.systemd_unit_path().read_text() == m.systemd_unit()
    assert calls == [("systemctl", "--user", "daemon-reload"), ("systemctl", "--user", "enable", "--now",
                                                                 "otedama.service")]


def test_linux_uninstall_tolerates_a_failed_disable(tmp_path, calls, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path)
    m.install()
    calls.outputs[("systemctl", "--user", "disable", "--now", "otedama.service")] = D.DaemonError("not loaded")
    m.uninstall()
    assert not m.systemd_unit_path().exists()


def test_linux_uninstall_when_not_installed_raises(tmp_path, calls, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    with pytest.raises(FileNotFoundError):
        mgr(tmp_path).uninstall()


@pytest.mark.parametrize("out,ok,running", [("active\n", True, True), ("inactive\n", False, False),
                                            ("activating\n", False, False)])
def test_linux_status(tmp_path, calls, monkeypatch, out, ok, running):
    monkeypatch.setattr(D, "platform", "linux")
    m = mgr(tmp_path)
    calls.outputs[("systemctl", "--user", "is-active", "otedama.service")] = (out, ok)
    st = m.status()
    assert not st.installed and st.running is running and st.details == out
    m.install()
    assert m.status().installed


def test_darwin_install_uninstall_status(tmp_path, calls, monkeypatch):
    monkeypatch.setattr(D, "platform", "darwin")
    m = mgr(tmp_path)
    m.install()
    path = str(m.launchd_plist_path())
    assert m.launchd_plist_path().read_text() == m.launchd_plist() and calls[-1] == ("launchctl", "load", "-w", path)
    calls.outputs[("launchctl", "list", "com.otedama.daemon")] = ('{ "PID" = 42; }', True)
    st = m.status()
    assert st.installed and st.running
    calls.outputs[("launchctl", "list", "com.otedama.daemon")] = ("Could not find service", True)
    assert not m.status().running
    m.uninstall()
    assert ("launchctl", "unload", "-w", path) in calls and not m.launchd_plist_path().exists()


def test_windows_install_uninstall_status(tmp_path, calls, monkeypatch):
    monkeypatch.setattr(D, "platform", "win32")
    m = mgr(tmp_path, bitcoin_address=ADDR)
    m.install()
    name, *args = calls[-1]
    assert name == "sc.exe" and args[:3] == ["create", "Otedama", "binPath="]
    assert args[3].startswith(f'"{m.executable}" -m otedama_amd run') and ADDR in args[3]
    assert args[4:] == ["start=", "auto", "DisplayName=", "Otedama Mining Service"]
    calls.outputs[("sc.exe", "query", "Otedama")] = ("STATE : 4 RUNNING", True)
    st = m.status()
    assert st.installed and st.running
    calls.outputs[("sc.exe", "query", "Otedama")] = ("The specified service does not exist", False)
    assert m.status() == D.ServiceStatus()
    calls.outputs[("sc.exe", "stop", "Otedama")] = D.DaemonError("not started")
    m.uninstall()
    assert calls[-1] == ("sc.exe", "delete", "Otedama")


@pytest.mark.parametrize("op", ["install", "uninstall", "status"])
def test_unsupported_platform(tmp_path, calls, monkeypatch, op):
    monkeypatch.setattr(D, "platform", "sunos5")
    with pytest.raises(D.DaemonError, match="unsupported platform"):
        getattr(mgr(tmp_path), op)()


def test_install_propagates_command_failures(tmp_path, calls, monkeypatch):
    monkeypatch.setattr(D, "platform", "linux")
    calls.outputs[("systemctl", "--user", "daemon-reload")] = D.DaemonError("no user bus")
    with pytest.raises(D.DaemonError, match="no user bus"):
        mgr(tmp_path).install()


def test_default_run_cmd_reports_exit_status():
    with pytest.raises(D.DaemonError, match="exit 3"):
        D._default_run_cmd("sh", "-c", "echo nope; exit 3")
    D._default_run_cmd("true")
    out, ok = D._default_output("sh", "-c", "echo hi")
    assert (out, ok) == ("hi\n", True)
    out, ok = D._default_output("/nonexistent/binary")
    assert not ok and out


@pytest.mark.parametrize("p,want", [("linux", "linux"), ("linux2", "linux"), ("win32", "windows"), ("cygwin", "cygwin"),
                                    ("darwin", "darwin")])
def test_platform_normalisation(monkeypatch, p, want):
    monkeypatch.setattr(D, "platform", p)
    assert D._platform() == want
