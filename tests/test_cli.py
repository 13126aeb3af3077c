"""CLI dispatcher and subcommands: exit codes, help routing, config show/validate, version, completion,
service seams, run dry-run / env fallbacks / logger sink matrix, pool config-file wiring.

Mirrors cmd/otedama/*_test.go (TestRun_*, TestConfigShow_*, TestConfigValidate_*, TestService*_*,
TestBuildLogger_*, TestApplyRunEnvFallbacks_*, TestLoadConfigFile_*, TestSafeDisplay_*, TestHasHelpFlag).
"""
from __future__ import annotations

import io
import json
import os
import stat

import pytest

from otedama_amd import daemon
from otedama_amd.cli import main as cli
from otedama_amd.cli import pool_cmd, run_cmd, service_cmd
from otedama_amd.cli.flags import FlagSet, has_help_flag

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"
ADDR2 = "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa"


@pytest.fixture(autouse=True)
def _clean_env(monkeypatch, tmp_path):
    for k in list(os.environ):
        if k.startswith("OTEDAMA_"):
            monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    monkeypatch.delenv("XDG_DATA_HOME", raising=False)


def _cli(*args):
    out, err = io.StringIO(), io.StringIO()
    rc = cli.run(list(args), out, err)
    return rc, out.getvalue(), err.getvalue()


# ------------------------------------------------------------------ dispatcher
def test_exit_code_constants():
    assert (cli.EXIT_OK, cli.EXIT_RUNTIME, cli.EXIT_USAGE, cli.EXIT_CONFIG) == (0, 1, 64, 78)


def test_no_args_prints_usage_to_stderr_with_exit_64():
    rc, out, err = _cli()
    assert rc == 64 and out == "" and "Usage:" in err


def test_usage_lists_exit_codes_and_every_command():
    for code in ("0   success", "1   runtime", "64  usage", "78  config"):
        assert code in cli.USAGE
    for c in cli.COMMANDS:
        assert f"  {c}" in cli.USAGE


@pytest.mark.parametrize("h", ["help", "--help", "-h"])
def test_help_goes_to_stdout_with_exit_0(h):
    rc, out, err = _cli(h)
    assert rc == 0 and "Usage:" in out and err == ""


@pytest.mark.parametrize("cmd", ["frobnicate", "Run", "--bogus"])
def test_unknown_subcommand_is_usage_error(cmd):
    rc, out, err = _cli(cmd)
    assert rc == 64 and "unknown subcommand" in err and out == ""


@pytest.mark.parametrize("sub", [["run"], ["config", "show"], ["config", "validate"], ["doctor"], ["version"],
                                 ["service", "install"], ["pool"]])
def test_subcommand_help_exits_zero_on_stdout(sub):
    rc, out, err = _cli(*sub, "--help")
    assert rc == 0 and "Usage of" in out and err == ""


@pytest.mark.parametrize("sub", [["run"], ["config", "show"], ["config", "validate"], ["doctor"], ["version"],
                                 ["service", "install"], ["pool"]])
def test_subcommand_unknown_flag_is_usage_error_on_stderr(sub):
    rc, out, err = _cli(*sub, "--no-such-flag")
    assert rc == 64 and "flag provided but not defined: -no-such-flag" in err and out == ""


@pytest.mark.parametrize("args,want", [
    (["--help"], True), (["-h"], True), (["-help"], True), (["x", "--help"], True),
    (["--", "--help"], False), ([], False), (["--helpful"], False),
])
def test_has_help_flag(args, want):
    assert has_help_flag(args) is want


# ------------------------------------------------------------------ flags (Go flag semantics)
def _fs():
    fs = FlagSet("t", io.StringIO())
    fs.string("s", "d", "")
    fs.int("n", 3, "")
    fs.float("f", 1.5, "")
    fs.bool("b", False, "")
    return fs


@pytest.mark.parametrize("args,want", [
    (["-s", "x"], {"s": "x"}), (["--s=y"], {"s": "y"}), (["-n", "7"], {"n": 7}), (["-f=2.5"], {"f": 2.5}),
    (["-b"], {"b": True}), (["-b=false"], {"b": False}), (["--b=T"], {"b": True}), (["-b=0"], {"b": False}),
])
def test_flag_forms(args, want):
    fs = _fs()
    fs.parse(args)
    for k, v in want.items():
        assert fs[k] == v
    assert fs.set_flags == set(want)


@pytest.mark.parametrize("args", [["-n", "x"], ["-f", "1.2.3"], ["-b=maybe"], ["-s"], ["---s", "x"], ["-zz"]])
def test_flag_errors(args):
    from otedama_amd.cli.flags import FlagError

    with pytest.raises(FlagError):
        _fs().parse(args)


def test_flag_parsing_stops_at_positional_and_double_dash():
    fs = _fs()
    assert fs.parse(["-s", "a", "pos", "-n", "2"]) == ["pos", "-n", "2"] and fs["n"] == 3
    fs = _fs()
    assert fs.parse(["--", "-s"]) == ["-s"] and fs["s"] == "d"


def test_flag_usage_shows_non_zero_defaults():
    u = _fs().usage()
    assert "-s string" in u and "(default 'd')" in u and "-b\n" in u and "(default False)" not in u


# ------------------------------------------------------------------ version
def test_version_plain_and_json():
    rc, out, _ = _cli("version")
    assert rc == 0 and out.startswith("otedama ")
    rc, out, _ = _cli("version", "--json")
    doc = json.loads(out)
    assert rc == 0 and {"version", "commit"} <= set(doc)


@pytest.mark.parametrize("alias", ["--version", "-v"])
def test_version_aliases(alias):
    assert _cli(alias)[0] == 0


# ------------------------------------------------------------------ config show / validate
def test_config_requires_a_subcommand():
    rc, _, err = _cli("config")
    assert rc == 64 and "expected subcommand" in err
    rc, _, err = _cli("config", "dump")
    assert rc == 64 and "unknown subcommand" in err
    assert _cli("config", "help")[0] == 0


def test_config_validate_missing_address_is_config_error():
    rc, out, err = _cli("config", "validate")
    assert rc == 78 and "bitcoin_address is required" in err


def test_config_validate_valid_address():
    rc, out, _ = _cli("config", "validate", "--bitcoin-address", ADDR)
    assert rc == 0 and out == "configuration is valid\n"


def test_config_validate_invalid_address():
    rc, _, err = _cli("config", "validate", "--bitcoin-address", ADDR[:-1] + "x")
    assert rc == 78 and "checksum" in err


def test_config_validate_warns_on_malformed_numeric_env(monkeypatch):
    monkeypatch.setenv("OTEDAMA_POWER_WATTS", "a-lot")
    rc, _, err = _cli("config", "validate", "--bitcoin-address", ADDR)
    assert rc == 0 and "OTEDAMA_POWER_WATTS" in err and "not a valid number" in err


def test_config_show_default_values_with_origin():
    rc, out, _ = _cli("config", "show", "--origin")
    assert rc == 0
    assert "bitcoin_address: (default) [default]" in out
    assert "log_level:       info [default]" in out
    assert "pools:           (built-in default) [default]" in out


def test_config_show_without_origin_has_no_annotations():
    rc, out, _ = _cli("config", "show", "--bitcoin-address", ADDR)
    assert rc == 0 and "[default]" not in out and "[flag]" not in out and ADDR in out


def test_config_show_flag_env_and_file_annotations(tmp_path, monkeypatch):
    p = tmp_path / "c.yaml"
    p.write_text("log_format: json\npools:\n  - url: stratum+tcp://a.example:3333\n"
                 f"bitcoin_addresses: [{ADDR2}]\n")
    monkeypatch.setenv("OTEDAMA_POWER_WATTS", "640")
    rc, out, _ = _cli("config", "show", "--config", str(p), "--origin", "--log-level", "debug")
    assert rc == 0
    assert "log_level:       debug [flag]" in out
    assert "log_format:      json [file]" in out
    assert "power_watts:                640 [env]" in out
    assert "pools:           1 configured [file]" in out and "[1] stratum+tcp://a.example:3333" in out
    assert "bitcoin_addresses (failover): 1 [file]" in out and f"[1] {ADDR2}" in out


def test_config_show_json(tmp_path, monkeypatch):
    p = tmp_path / "c.yaml"
    p.write_text("pools:\n  - url: stratum+v2://b.example:3336\nmining:\n  algorithm: scrypt\n")
    monkeypatch.setenv("OTEDAMA_MIN_YIELD_SATS_PER_SEC", "1.25")
    rc, out, _ = _cli("config", "show", "--config", str(p), "--json", "--origin", "--bitcoin-address", ADDR,
                      "--http-addr", "127.0.0.1:9100")
    doc = json.loads(out)
    assert rc == 0 and doc["bitcoin_address"] == ADDR and doc["http_addr"] == "127.0.0.1:9100"
    assert doc["pools"] == ["stratum+v2://b.example:3336"] and doc["mining"]["algorithm"] == "scrypt"
    assert doc["min_yield_sats_per_sec"] == 1.25
    assert doc["origins"]["http_addr"] == "flag" and doc["origins"]["min_yield_sats_per_sec"] == "env"
    assert doc["origins"]["pools"] == "file" and doc["origins"]["log_level"] == "default"
    assert "bitcoin_addresses" not in doc


def test_config_show_json_without_origin_has_no_origins():
    doc = json.loads(_cli("config", "show", "--json")[1])
    assert "origins" not in doc


def test_config_show_strips_control_characters():
    rc, out, _ = _cli("config", "show", "--language", "ja\x1b[31m\x07")
    assert rc == 0 and "\x1b" not in out and "\x07" not in out and "ja[31m" in out


def test_config_file_parse_error_warns_and_is_ignored(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("log_levell: debug\n")
    rc, out, err = _cli("config", "show", "--config", str(p))
    assert rc == 0 and "warning: config file" in err and "log_levell" in err and "log_level:       info" in out


def test_config_file_from_otedama_config_env(tmp_path, monkeypatch):
    p = tmp_path / "env.yaml"
    p.write_text("log_level: warn\n")
    monkeypatch.setenv("OTEDAMA_CONFIG", str(p))
    assert "log_level:       warn [file]" in _cli("config", "show", "--origin")[1]


def test_config_file_from_default_home_path(tmp_path):
    d = tmp_path / "home" / ".config" / "otedama"
    d.mkdir(parents=True)
    (d / "config.yaml").write_text("log_format: json\n")
    assert "log_format:      json [file]" in _cli("config", "show", "--origin")[1]


@pytest.mark.parametrize("v,want", [("", "(default)"), ("abc", "abc"), ("a\nb\tc", "abc"), ("\x00\x01", "(default)"),
                                    ("日本語", "日本語")])
def test_safe_display(v, want):
    assert cli.safe_display(v) == want


# ------------------------------------------------------------------ run (dry-run paths only)
def test_run_dry_run_requires_address():
    rc, _, err = _cli("run", "--dry-run")
    assert rc == 78 and "bitcoin_address is required" in err


def test_run_invalid_address_exits_config():
    assert _cli("run", "--dry-run", "--bitcoin-address", "3" * 30)[0] == 78


@pytest.mark.parametrize("extra", [[], ["--log-format", "json"], ["--http-addr", "127.0.0.1:0"], ["--no-tui"],
                                   ["--algorithm", "scrypt"], ["--gpus", "none"], ["--cpu-threads", "2"]])
def test_run_dry_run_variants(extra):
    rc, out, _ = _cli("run", "--dry-run", "--bitcoin-address", ADDR, *extra)
    assert rc == 0 and "dry-run: configuration is valid" in out


def test_run_bad_algorithm_is_config_error():
    rc, _, err = _cli("run", "--dry-run", "--bitcoin-address", ADDR, "--algorithm", "ethash")
    assert rc == 78 and "mining.algorithm" in err


def test_run_malformed_numeric_env_warns_and_succeeds(monkeypatch):
    monkeypatch.setenv("OTEDAMA_CURTAIL_BELOW_BTC_USD", "cheap")
    rc, _, err = _cli("run", "--dry-run", "--bitcoin-address", ADDR)
    assert rc == 0 and "OTEDAMA_CURTAIL_BELOW_BTC_USD" in err


def test_run_address_from_env(monkeypatch):
    monkeypatch.setenv("OTEDAMA_BITCOIN_ADDRESS", ADDR)
    assert _cli("run", "--dry-run")[0] == 0


# logger sink matrix (run.go:251-303)
class _Cfg:
    log_level = "info"
    log_format = "text"


def test_build_logger_tui_without_file_discards():
    out = io.StringIO()
    lg, close = run_cmd.build_logger(False, "", _Cfg(), out)
    lg.info("hello")
    close()
    assert out.getvalue() == ""


@pytest.mark.parametrize("fmt", ["text", "json"])
def test_build_logger_no_tui_writes_to_stdout(fmt):
    cfg = _Cfg()
    cfg.log_format = fmt
    out = io.StringIO()
    lg, close = run_cmd.build_logger(True, "", cfg, out)
    lg.info("hello", k=1)
    close()
    line = out.getvalue().strip()
    if fmt == "json":
        doc = json.loads(line)
        assert doc["msg"] == "hello" and doc["k"] == 1
    else:
        assert "hello" in line and "k=1" in line


def test_build_logger_tui_with_file_writes_file_only(tmp_path):
    out = io.StringIO()
    f = tmp_path / "o.log"
    lg, close = run_cmd.build_logger(False, str(f), _Cfg(), out)
    lg.info("to-file")
    close()
    assert out.getvalue() == "" and "to-file" in f.read_text()
    assert stat.S_IMODE(f.stat().st_mode) == 0o600


def test_build_logger_no_tui_with_file_writes_both(tmp_path):
    out = io.StringIO()
    f = tmp_path / "o.log"
    lg, close = run_cmd.build_logger(True, str(f), _Cfg(), out)
    lg.warn("both")
    close()
    assert "both" in out.getvalue() and "both" in f.read_text()


def test_build_logger_unopenable_file_does_not_raise(tmp_path, capsys):
    out = io.StringIO()
    lg, close = run_cmd.build_logger(True, str(tmp_path / "no" / "such" / "dir.log"), _Cfg(), out)
    lg.info("still logs")
    close()
    assert "still logs" in out.getvalue() and "cannot open --log-file" in capsys.readouterr().err


def test_is_terminal_false_for_files_pipes_and_closed(tmp_path):
    f = open(tmp_path / "x", "w")
    assert run_cmd._is_terminal(f) is False
    f.close()
    assert run_cmd._is_terminal(f) is False
    r, w = os.pipe()
    with os.fdopen(w, "w") as wf:
        assert run_cmd._is_terminal(wf) is False
    os.close(r)
    assert run_cmd._is_terminal(io.StringIO()) is False


# ------------------------------------------------------------------ service (injected seams)
class _FakeMgr:
    def __init__(self, *a, **k):
        self.args = a


@pytest.fixture
def fake_service(monkeypatch):
    calls = []
    monkeypatch.setattr(service_cmd, "new_daemon_manager", lambda *a: calls.append(("new", a)) or _FakeMgr(*a))
    monkeypatch.setattr(service_cmd, "manager_install", lambda m: calls.append(("install", m.args)))
    monkeypatch.setattr(service_cmd, "manager_uninstall", lambda m: calls.append(("uninstall",)))
    return calls


def test_service_requires_subcommand(fake_service):
    rc, _, err = _cli("service")
    assert rc == 64 and "expected subcommand" in err
    rc, _, err = _cli("service", "restart")
    assert rc == 64 and "unknown subcommand" in err
    rc, out, _ = _cli("service", "--help")
    assert rc == 0 and "install|uninstall|status" in out
    assert fake_service == []


def test_service_install_success_passes_flags(fake_service):
    rc, out, _ = _cli("service", "install", "--bitcoin-address", ADDR, "--log-level", "debug", "--data-dir", "/d")
    assert rc == 0 and "installed and started" in out
    (_, (cfg, data_dir, flags)), (what, _) = fake_service
    assert what == "install" and data_dir == "/d" and flags.bitcoin_address == ADDR and flags.log_level == "debug"


def test_service_install_node_mode(fake_service):
    """--node-gpus N: the service runs the multi-GPU node (its supervisor restarts ranks; the service manager restarts
    the supervisor)."""
    rc, _, _ = _cli("service", "install", "--bitcoin-address", ADDR, "--node-gpus", "8")
    assert rc == 0
    (_, (_, _, flags)), _ = fake_service
    assert flags.node_gpus == 8
    assert _cli("service", "install", "--node-gpus", "-1")[0] == 64


def test_service_install_bad_flag(fake_service):
    assert _cli("service", "install", "--frob")[0] == 64 and fake_service == []


@pytest.mark.parametrize("sub", ["install", "uninstall", "status"])
def test_service_manager_errors_are_runtime(monkeypatch, sub):
    def boom(*a):
        raise RuntimeError("no service manager")

    monkeypatch.setattr(service_cmd, "new_daemon_manager", boom)
    rc, _, err = _cli("service", sub)
    assert rc == 1 and "no service manager" in err


@pytest.mark.parametrize("sub,seam", [("install", "manager_install"), ("uninstall", "manager_uninstall"),
                                      ("status", "manager_status")])
def test_service_operation_errors_are_runtime(monkeypatch, sub, seam):
    monkeypatch.setattr(service_cmd, "new_daemon_manager", lambda *a: _FakeMgr())

    def boom(m):
        raise OSError("systemctl exited 1")

    monkeypatch.setattr(service_cmd, seam, boom)
    rc, _, err = _cli("service", sub)
    assert rc == 1 and "systemctl exited 1" in err


@pytest.mark.parametrize("installed,running,needle", [(False, False, "not installed"),
                                                      (True, False, "installed, stopped"),
                                                      (True, True, "installed, running")])
def test_service_status_states(monkeypatch, installed, running, needle):
    monkeypatch.setattr(service_cmd, "new_daemon_manager", lambda *a: _FakeMgr())
    monkeypatch.setattr(service_cmd, "manager_status",
                        lambda m: daemon.ServiceStatus(installed=installed, running=running))
    rc, out, _ = _cli("service", "status")
    assert rc == 0 and needle in out


def test_service_uninstall_success(fake_service):
    rc, out, _ = _cli("service", "uninstall")
    assert rc == 0 and "uninstalled" in out and ("uninstall",) in fake_service


# ------------------------------------------------------------------ completion
@pytest.mark.parametrize("shell,marker", [("bash", "complete -F"), ("zsh", "#compdef"), ("fish", "complete -c")])
def test_completion_scripts(shell, marker):
    rc, out, _ = _cli("completion", shell)
    assert rc == 0 and marker in out
    for c in ("run", "pool", "doctor", "service", "config"):
        assert c in out


@pytest.mark.parametrize("args", [[], ["tcsh"], ["bash", "zsh"]])
def test_completion_rejects_bad_args(args):
    assert _cli("completion", *args)[0] == 64


# ------------------------------------------------------------------ pool: config file wiring
def _capture_pool_opts(monkeypatch):
    seen = {}

    async def fake_serve(fs, algos, stdout):
        seen.update({k: fs[k] for k in ("listen-sv2", "listen-v1", "difficulty", "share-seconds", "retarget-seconds",
                                        "journal", "http-addr")})
        seen["algos"] = algos
        seen["coinbase"] = fs.values.get("coinbase-message")
        return 0

    monkeypatch.setattr(pool_cmd, "_serve", fake_serve)
    return seen


def test_pool_reads_pool_server_section(tmp_path, monkeypatch):
    seen = _capture_pool_opts(monkeypatch)
    p = tmp_path / "c.yaml"
    p.write_text("http_addr: 127.0.0.1:9555\npool_server:\n  listen_sv2: 0.0.0.0:4336\n  listen_v1: 0.0.0.0:4333\n"
                 "  algorithm: scrypt\n  initial_difficulty: 0.25\n  target_share_seconds: 4\n"
                 "  vardiff_retarget_seconds: 12\n  journal_path: /tmp/j.db\n  coinbase_message: /mine/\n")
    rc, _, err = _cli("pool", "--config", str(p))
    assert rc == 0, err
    assert seen == {"listen-sv2": "0.0.0.0:4336", "listen-v1": "0.0.0.0:4333", "difficulty": 0.25,
                    "share-seconds": 4.0, "retarget-seconds": 12.0, "journal": "/tmp/j.db",
                    "http-addr": "127.0.0.1:9555", "algos": ["scrypt"], "coinbase": "/mine/"}


def test_pool_flags_beat_the_config_file(tmp_path, monkeypatch):
    seen = _capture_pool_opts(monkeypatch)
    p = tmp_path / "c.yaml"
    p.write_text("pool_server:\n  listen_sv2: 0.0.0.0:4336\n  algorithm: scrypt\n  initial_difficulty: 0.25\n")
    rc, _, _ = _cli("pool", "--config", str(p), "--listen-sv2", "127.0.0.1:5000", "--algorithms", "sha256d,x11",
                    "--difficulty", "2")
    assert rc == 0
    assert seen["listen-sv2"] == "127.0.0.1:5000" and seen["algos"] == ["sha256d", "x11"] and seen["difficulty"] == 2
    assert seen["listen-v1"] == "127.0.0.1:3333"  # flag default: the file left it empty


def test_pool_without_config_keeps_flag_defaults(monkeypatch):
    seen = _capture_pool_opts(monkeypatch)
    assert _cli("pool")[0] == 0
    assert seen["listen-sv2"] == "127.0.0.1:3336" and seen["algos"] == ["sha256d"] and seen["difficulty"] == 1.0


@pytest.mark.parametrize("args,needle", [(["--algorithms", "ethash"], "unsupported algorithm"),
                                         (["--payout-address", "bc1qnope"], "payout address invalid"),
                                         (["--noise-authority-key", "zz"], "noise-authority-key")])
def test_pool_config_errors(monkeypatch, args, needle):
    _capture_pool_opts(monkeypatch)
    rc, _, err = _cli("pool", *args)
    assert rc == 78 and needle in err


@pytest.mark.parametrize("addr,k,want", [("127.0.0.1:3336", 0, "127.0.0.1:3336"), ("127.0.0.1:3336", 2, "127.0.0.1:3338"),
                                         ("127.0.0.1:0", 3, "127.0.0.1:0"), ("", 1, ""), ("[::1]:10", 1, "[::1]:11")])
def test_pool_port_bump(addr, k, want):
    assert pool_cmd._bump(addr, k) == want


def test_node_status_renders_the_leaders_view_and_fails_without_a_node():
    import io

    from otedama_amd.cli.node_cmd import cmd_node, render_status

    st = {"world": 2, "backend": "rccl", "generation": 3, "leader_incarnation": 2, "members": [0, 1],
          "lost_ranks": [], "reforms": 3, "op_p50_ms": 0.4, "op_p99_ms": 1.2, "share_previews": 10,
          "share_gathered_first": 1, "remote_stale": 0,
          "ranks": {"rank0": {"hashrate": 19.4e9, "leader": True},
                    "rank1": {"hashrate": 19.3e9, "heartbeat_age_s": 0.3, "generation": 3, "pending_shares": 0,
                              "collectives": 42, "member": True}}}
    out = render_status(st)
    assert "node: 2 ranks over rccl, generation 3, leader incarnation 2" in out
    assert "19.40 GH/s" in out and "19.30 GH/s" in out and "38.70 GH/s" in out and "10 from previews" in out
    err = io.StringIO()
    assert cmd_node(["status", "--http-addr", "127.0.0.1:1"], io.StringIO(), err) == 1
    assert "no node answering" in err.getvalue()
