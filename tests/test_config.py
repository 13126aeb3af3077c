"""Layered config: precedence, origins, zero-value caveat, env warnings, validation, strict YAML.

Mirrors the behaviours the reference pins in internal/config/config_test.go and configfile_test.go
(TestResolve_*, TestResolveWithOrigins_*, TestValidate_*, TestEnvWarnings_*, TestConfigFile_*,
TestArbitrationHysteresisPct_*), table-driven over every layer and field.
"""
from __future__ import annotations

import json
import re
from pathlib import Path

import pytest

from otedama_amd import config as C

ROOT = Path(__file__).resolve().parent.parent
ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"  # P2WPKH (bech32)
GOOD_ADDRS = [
    ADDR,
    "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa",  # P2PKH (genesis coinbase)
    "3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy",  # P2SH
    "bc1p5d7rjq7g6rdk2yhzks9smlaqtedr4dekq08ge8ztwac72sfr9rusxg3297",  # P2TR (bech32m)
    "bc1qrp33g0q5c5txsp9arysrx4k6zdkfs4nce4xj0gdcccefvpysxf3qccfmv3",  # P2WSH
]
O = C.ValueOrigin


def _typo(addr: str) -> str:
    """Flip one data character so the checksum breaks but the shape stays valid."""
    i = len(addr) // 2
    alphabet = "qpzry9x8gf2tvdw0s3jn54khce6mua7l" if addr.startswith("bc1") else \
        "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
    c = addr[i]
    repl = next(ch for ch in alphabet if ch != c)
    return addr[:i] + repl + addr[i + 1:]


def _file(text: str) -> C.Config:
    return C.parse_config_yaml(text)


# ------------------------------------------------------------------ defaults
def test_defaults_have_no_address_and_reference_values():
    d = C.Config()
    assert d.bitcoin_address == "" and d.bitcoin_addresses == [] and d.pools == []
    assert d.log_level == "info" and d.log_format == "text"
    assert d.arbitration_hysteresis_pct == pytest.approx(0.05)
    assert d.curtail_below_btc_usd == d.min_yield_sats_per_sec == d.power_watts == d.electricity_price_per_kwh == 0
    assert d.http_addr == ""
    assert C.DEFAULT_POOL_URL == "stratum+v2://public.stratum.slushpool.com:3336"


def test_zero_configuration_startup_only_needs_an_address():
    cfg = C.resolve(C.Config(), {}, C.FlagValues(bitcoin_address=ADDR))
    cfg.validate()
    assert cfg.log_level == "info" and cfg.log_format == "text" and cfg.data_dir


# ------------------------------------------------------------------ precedence
STRING_FIELDS = [
    # (config field, env var, flag attr, two distinct valid values)
    ("log_level", "OTEDAMA_LOG_LEVEL", "log_level", ("debug", "error")),
    ("log_format", "OTEDAMA_LOG_FORMAT", "log_format", ("json", "text")),
    ("language", "OTEDAMA_LANGUAGE", "language", ("ja", "de")),
    ("data_dir", "OTEDAMA_DATA_DIR", "data_dir", ("/tmp/otd-file", "/tmp/otd-env")),
    ("http_addr", "OTEDAMA_HTTP_ADDR", "http_addr", ("127.0.0.1:9100", "127.0.0.1:9200")),
    ("bitcoin_address", "OTEDAMA_BITCOIN_ADDRESS", "bitcoin_address", (GOOD_ADDRS[1], GOOD_ADDRS[2])),
]


@pytest.mark.parametrize("field,env_key,flag,vals", STRING_FIELDS, ids=[f[0] for f in STRING_FIELDS])
def test_string_field_precedence_flag_env_file_default(field, env_key, flag, vals):
    file_val, env_val = vals
    f = _file(f"{field}: {json.dumps(file_val)}\n")
    # file only
    cfg, o = C.resolve_with_origins(f, {}, C.FlagValues())
    assert getattr(cfg, field) == file_val and o[field] == O.FILE
    # env beats file
    cfg, o = C.resolve_with_origins(f, {env_key: env_val}, C.FlagValues())
    assert getattr(cfg, field) == env_val and o[field] == O.ENV
    # flag beats env
    flag_val = vals[0] if field != "log_format" else "json"
    cfg, o = C.resolve_with_origins(f, {env_key: env_val}, C.FlagValues(**{flag: flag_val}))
    assert getattr(cfg, field) == flag_val and o[field] == O.FLAG


@pytest.mark.parametrize("field,env_key,flag,vals", STRING_FIELDS, ids=[f[0] for f in STRING_FIELDS])
def test_empty_higher_layer_does_not_override_lower(field, env_key, flag, vals):
    f = _file(f"{field}: {json.dumps(vals[0])}\n")
    cfg, o = C.resolve_with_origins(f, {env_key: ""}, C.FlagValues(**{flag: ""}))
    assert getattr(cfg, field) == vals[0] and o[field] == O.FILE


def test_file_log_format_not_clobbered_by_flag_default():
    cfg = C.resolve(_file("log_format: json\n"), {}, C.FlagValues())
    assert cfg.log_format == "json"


def test_empty_file_does_not_clobber_defaults():
    cfg, o = C.resolve_with_origins(_file(""), {}, C.FlagValues())
    assert cfg.log_format == "text" and cfg.log_level == "info"
    assert all(v == O.DEFAULT for k, v in o.items() if k != "data_dir")


NUMERIC_FIELDS = [
    ("arbitration_hysteresis_pct", "OTEDAMA_ARBITRATION_HYSTERESIS_PCT", 0.2, 0.3),
    ("min_yield_sats_per_sec", "OTEDAMA_MIN_YIELD_SATS_PER_SEC", 0.5, 2.5),
    ("curtail_below_btc_usd", "OTEDAMA_CURTAIL_BELOW_BTC_USD", 30000.0, 42000.5),
    ("power_watts", "OTEDAMA_POWER_WATTS", 750.0, 1400.0),
    ("electricity_price_per_kwh", "OTEDAMA_ELECTRICITY_PRICE_PER_KWH", 0.12, 0.31),
]


@pytest.mark.parametrize("field,env_key,file_val,env_val", NUMERIC_FIELDS, ids=[f[0] for f in NUMERIC_FIELDS])
def test_numeric_field_file_then_env(field, env_key, file_val, env_val):
    f = _file(f"{field}: {file_val}\n")
    cfg, o = C.resolve_with_origins(f, {}, C.FlagValues())
    assert getattr(cfg, field) == pytest.approx(file_val) and o[field] == O.FILE
    cfg, o = C.resolve_with_origins(f, {env_key: str(env_val)}, C.FlagValues())
    assert getattr(cfg, field) == pytest.approx(env_val) and o[field] == O.ENV


@pytest.mark.parametrize("field,env_key,file_val,env_val", NUMERIC_FIELDS, ids=[f[0] for f in NUMERIC_FIELDS])
@pytest.mark.parametrize("bad", ["abc", "1.2.3", "", "0x", "--1"])
def test_numeric_env_invalid_is_ignored(field, env_key, file_val, env_val, bad):
    f = _file(f"{field}: {file_val}\n")
    cfg, o = C.resolve_with_origins(f, {env_key: bad}, C.FlagValues())
    assert getattr(cfg, field) == pytest.approx(file_val) and o[field] == O.FILE


@pytest.mark.parametrize("field,env_key,file_val,env_val", NUMERIC_FIELDS, ids=[f[0] for f in NUMERIC_FIELDS])
def test_numeric_zero_in_file_means_unset_but_env_can_force_zero(field, env_key, file_val, env_val):
    default = getattr(C.Config(), field)
    cfg, o = C.resolve_with_origins(_file(f"{field}: 0\n"), {}, C.FlagValues())
    assert getattr(cfg, field) == default and o[field] == O.DEFAULT
    cfg, o = C.resolve_with_origins(_file(f"{field}: {file_val}\n"), {env_key: "0"}, C.FlagValues())
    assert getattr(cfg, field) == 0 and o[field] == O.ENV


def test_hysteresis_default_is_preserved_through_resolve():
    cfg = C.resolve(C.Config(), {}, C.FlagValues())
    assert cfg.arbitration_hysteresis_pct == pytest.approx(0.05)


def test_pools_addresses_and_worker_name_come_from_file():
    f = _file(
        f"bitcoin_addresses: [{GOOD_ADDRS[1]}, {GOOD_ADDRS[2]}]\n"
        "pools:\n  - url: stratum+tcp://a.example:3333\n    payout_scheme: pplns\n"
        "  - url: stratum+v2://b.example:3336\n"
        "workers:\n  name: rig7\n")
    cfg, o = C.resolve_with_origins(f, {}, C.FlagValues())
    assert cfg.bitcoin_addresses == GOOD_ADDRS[1:3] and o["bitcoin_addresses"] == O.FILE
    assert [p.url for p in cfg.pools] == ["stratum+tcp://a.example:3333", "stratum+v2://b.example:3336"]
    assert o["pools"] == O.FILE and cfg.pools[0].payout_scheme == "pplns"
    assert cfg.workers.name == "rig7" and o["worker_name"] == O.FILE


def test_resolve_with_origins_agrees_with_resolve():
    f = _file(f"log_level: warn\npower_watts: 500\nbitcoin_address: {ADDR}\n")
    env = {"OTEDAMA_LOG_FORMAT": "json", "OTEDAMA_POWER_WATTS": "700"}
    flags = C.FlagValues(language="ja")
    a = C.resolve(f, env, flags)
    b, _ = C.resolve_with_origins(f, env, flags)
    assert a == b


def test_value_origin_strings():
    assert [str(v) for v in O] == ["default", "file", "env", "flag"]


def test_data_dir_default_origin_stays_default():
    cfg, o = C.resolve_with_origins(C.Config(), {"HOME": "/home/u"}, C.FlagValues())
    assert cfg.data_dir and o["data_dir"] == O.DEFAULT


@pytest.mark.parametrize("platform,env,want", [
    ("linux", {"HOME": "/home/u"}, "/home/u/.local/share/otedama"),
    ("linux", {"HOME": "/home/u", "XDG_DATA_HOME": "/xdg"}, "/xdg/otedama"),
    ("darwin", {"HOME": "/Users/u"}, "/Users/u/Library/Application Support/Otedama"),
    ("win32", {"APPDATA": "C:\\Users\\u\\AppData\\Roaming"}, "C:\\Users\\u\\AppData\\Roaming/Otedama"),
    ("win32", {}, ""),
])
def test_default_data_dir_per_os(platform, env, want):
    got = C.default_data_dir(env, platform)
    assert got.replace("\\", "/") == want.replace("\\", "/")


# ------------------------------------------------------------------ env warnings
def test_env_warnings_flag_every_malformed_numeric_var():
    env = {k: "nope" for k, _ in C.NUMERIC_ENV_VARS}
    w = C.env_warnings(env)
    assert len(w) == len(C.NUMERIC_ENV_VARS)
    for (k, _), line in zip(C.NUMERIC_ENV_VARS, w):
        assert line.startswith(k) and "not a valid number" in line


def test_env_warnings_none_when_valid_or_unset():
    assert C.env_warnings({}) == []
    assert C.env_warnings({k: "1.5" for k, _ in C.NUMERIC_ENV_VARS}) == []


def test_env_warnings_ignore_non_numeric_vars():
    assert C.env_warnings({"OTEDAMA_LOG_LEVEL": "bogus", "OTEDAMA_BITCOIN_ADDRESS": "x"}) == []


def test_env_warnings_default_to_process_env(monkeypatch):
    monkeypatch.setenv("OTEDAMA_POWER_WATTS", "lots")
    assert any("OTEDAMA_POWER_WATTS" in w for w in C.env_warnings())


# ------------------------------------------------------------------ validation
def _issues(cfg: C.Config) -> list[str]:
    try:
        cfg.validate()
    except C.ConfigError as exc:
        return [ln.strip()[2:] for ln in str(exc).splitlines()[1:]]
    return []


def test_validate_requires_an_address():
    assert any("bitcoin_address is required" in i for i in _issues(C.Config()))


@pytest.mark.parametrize("addr", GOOD_ADDRS)
def test_validate_accepts_valid_addresses(addr):
    assert _issues(C.Config(bitcoin_address=addr)) == []
    assert _issues(C.Config(bitcoin_addresses=[addr])) == []


@pytest.mark.parametrize("addr,needle", [
    ("bc1short", "too short"),
    ("bc1" + "q" * 100, "too long"),
    ("tb1qw508d6qejxtdg4y5r3zarvary0c5xw7kxpjzsx", "does not start"),
    ("2N2JD6wb56AfK4tfmM6PwdVmoYk2dCKf4Br", "does not start"),
    ("bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdx", "checksum"),
])
def test_validate_rejects_invalid_addresses(addr, needle):
    issues = _issues(C.Config(bitcoin_address=addr))
    assert len(issues) == 1 and needle in issues[0]


@pytest.mark.parametrize("addr", GOOD_ADDRS)
def test_validate_rejects_checksum_typo(addr):
    bad = _typo(addr)
    assert any("checksum" in i for i in _issues(C.Config(bitcoin_address=bad)))
    issues = _issues(C.Config(bitcoin_address=ADDR, bitcoin_addresses=[GOOD_ADDRS[1], bad]))
    assert len(issues) == 1 and issues[0].startswith("bitcoin_addresses[1]")


def test_validate_empty_entry_in_failover_list():
    issues = _issues(C.Config(bitcoin_addresses=[ADDR, ""]))
    assert issues == ["bitcoin_addresses[1] is empty"]


@pytest.mark.parametrize("level", ["debug", "info", "warn", "error"])
def test_validate_accepts_log_levels(level):
    assert _issues(C.Config(bitcoin_address=ADDR, log_level=level)) == []


@pytest.mark.parametrize("level", ["trace", "WARNING", "fatal", "Info"])
def test_validate_rejects_unknown_log_level(level):
    assert any("log_level" in i for i in _issues(C.Config(bitcoin_address=ADDR, log_level=level)))


@pytest.mark.parametrize("fmt,ok", [("text", True), ("json", True), ("yaml", False), ("JSON", False)])
def test_validate_log_format(fmt, ok):
    assert (_issues(C.Config(bitcoin_address=ADDR, log_format=fmt)) == []) is ok


@pytest.mark.parametrize("url,ok", [
    ("stratum+tcp://pool.example:3333", True),
    ("stratum+tls://pool.example:443", True),
    ("stratum+v2://pool.example:3336", True),
    ("stratum+v2tls://pool.example:3336", True),
    ("stratum+tcp://", False),
    ("http://pool.example", False),
    ("pool.example:3333", False),
    ("datum://pool.example:23334", False),
    ("stratum+ssl://pool.example", False),
])
def test_validate_pool_urls(url, ok):
    issues = _issues(C.Config(bitcoin_address=ADDR, pools=[C.PoolConfig(url=url)]))
    assert (issues == []) is ok


def test_validate_empty_pool_url():
    assert _issues(C.Config(bitcoin_address=ADDR, pools=[C.PoolConfig()])) == ["pools[0].url is empty"]


@pytest.mark.parametrize("scheme,ok", [("", True), ("fpps", True), ("pplns", True), ("tides", True),
                                       ("solo", True), ("pps", False), ("PPLNS", False)])
def test_validate_payout_scheme(scheme, ok):
    cfg = C.Config(bitcoin_address=ADDR, pools=[C.PoolConfig(url="stratum+tcp://p:1", payout_scheme=scheme)])
    assert (_issues(cfg) == []) is ok


@pytest.mark.parametrize("v,ok", [(0.0, True), (0.05, True), (0.999, True), (1.0, False), (-0.01, False), (5, False)])
def test_validate_hysteresis_range(v, ok):
    assert (_issues(C.Config(bitcoin_address=ADDR, arbitration_hysteresis_pct=v)) == []) is ok


@pytest.mark.parametrize("field", ["curtail_below_btc_usd", "min_yield_sats_per_sec", "power_watts",
                                   "electricity_price_per_kwh"])
@pytest.mark.parametrize("v,ok", [(0.0, True), (12.5, True), (-0.0001, False), (-100, False)])
def test_validate_non_negative_fields(field, v, ok):
    issues = _issues(C.Config(bitcoin_address=ADDR, **{field: v}))
    assert (issues == []) is ok
    if not ok:
        assert issues[0].startswith(field) and "must be >= 0" in issues[0]


def test_validate_aggregates_every_issue():
    cfg = C.Config(bitcoin_address="nope", log_level="loud", log_format="xml",
                   pools=[C.PoolConfig(url="http://x", payout_scheme="pps")], arbitration_hysteresis_pct=2,
                   power_watts=-1)
    issues = _issues(cfg)
    assert [re.match(r"[a-z_\[\]0-9.]+", i).group(0) for i in issues] == [
        "bitcoin_address", "log_level", "log_format", "pools[0].url", "pools[0].payout_scheme",
        "arbitration_hysteresis_pct", "power_watts"]


@pytest.mark.parametrize("mining,ok", [
    ({"algorithm": "sha256d"}, True), ({"algorithm": "scrypt"}, True), ({"algorithm": "x11"}, True),
    ({"algorithm": "ethash"}, False), ({"cpu_threads": -1}, False),
    ({"batch_nonces": 1 << 16}, True), ({"batch_nonces": 1 << 32}, True),
    ({"batch_nonces": 1000}, False), ({"batch_nonces": (1 << 32) + 1}, False),
    ({"sha_variants": 128}, True), ({"sha_variants": 64}, True), ({"sha_variants": 8}, True),
    ({"sha_variants": 1}, True), ({"sha_variants": 0}, False), ({"sha_variants": 32}, False),
    ({"sha_variants": 256}, False),
])
def test_validate_mining_section(mining, ok):
    cfg = C.Config(bitcoin_address=ADDR, mining=C.MiningConfig(**mining))
    assert (_issues(cfg) == []) is ok


@pytest.mark.parametrize("ps,ok", [({"initial_difficulty": 0.001}, True), ({"initial_difficulty": 0}, False),
                                   ({"target_share_seconds": 0}, False), ({"target_share_seconds": 2.5}, True)])
def test_validate_pool_server_section(ps, ok):
    cfg = C.Config(bitcoin_address=ADDR, pool_server=C.PoolServerConfig(**ps))
    assert (_issues(cfg) == []) is ok


# ------------------------------------------------------------------ YAML file
def test_config_file_round_trip(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text(f"bitcoin_address: {ADDR}\nlog_level: debug\nlog_format: json\npower_watts: 900\n"
                 "pools:\n  - url: stratum+v2://p.example:3336\n    user: me.rig\n    password: pw\n"
                 "mining:\n  algorithm: x11\n  batch_nonces: 1048576\n  sha_variants: 64\n")
    f, warn = C.load_config_file(str(p))
    assert warn is None
    assert (f.bitcoin_address, f.log_level, f.log_format, f.power_watts) == (ADDR, "debug", "json", 900.0)
    assert f.pools[0].user == "me.rig" and f.pools[0].password == "pw"
    assert f.mining.algorithm == "x11" and f.mining.batch_nonces == 1 << 20 and f.mining.sha_variants == 64


def test_missing_config_file_is_ok(tmp_path):
    f, warn = C.load_config_file(str(tmp_path / "nope.yaml"))
    assert warn is None and f == C.Config()
    assert C.load_config_file("") == (C.Config(), None)


@pytest.mark.parametrize("text", ["", "\n", "# only a comment\n", "---\n"])
def test_empty_config_file_is_valid(tmp_path, text):
    p = tmp_path / "c.yaml"
    p.write_text(text)
    f, warn = C.load_config_file(str(p))
    assert warn is None and f == C.Config()


@pytest.mark.parametrize("text,needle", [
    ("bitcoin_addres: x\n", "bitcoin_addres"),
    ("pools:\n  - url: stratum+tcp://a:1\n    passwd: x\n", "passwd"),
    ("workers:\n  nmae: x\n", "nmae"),
    ("mining:\n  algo: scrypt\n", "algo"),
    ("log_level: [a, b]\n", "log_level"),
    ("power_watts: lots\n", "power_watts"),
    ("pools: stratum+tcp://a:1\n", "pools"),
    ("bitcoin_addresses: x\n", "bitcoin_addresses"),
    ("mining:\n  batch_nonces: 1.5\n", "batch_nonces"),
    ("mining:\n  version_rolling: yes-please\n", "version_rolling"),
    ("key: [unclosed\n", ""),
    ("- just\n- a list\n", "mapping"),
])
def test_strict_yaml_rejects_whole_file(tmp_path, text, needle):
    p = tmp_path / "c.yaml"
    p.write_text(f"bitcoin_address: {ADDR}\n" + text if not text.startswith("-") else text)
    f, warn = C.load_config_file(str(p))
    assert warn and "ignored" in warn and needle in warn
    assert f == C.Config()  # the whole file is dropped, not just the bad key


def test_unreadable_config_path_warns(tmp_path):
    f, warn = C.load_config_file(str(tmp_path))  # a directory
    assert warn and f == C.Config()


def test_yaml_scalar_coercions():
    f = _file("http_addr: 9100\nlanguage: null\npower_watts: 5\n")
    assert f.http_addr == "9100" and f.language == "" and f.power_watts == 5.0


def test_file_flag_override_and_precedence_over_defaults(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("log_level: debug\n")
    f, _ = C.load_config_file(str(p))
    assert C.resolve(f, {}, C.FlagValues()).log_level == "debug"
    assert C.resolve(f, {}, C.FlagValues(log_level="error")).log_level == "error"


@pytest.mark.parametrize("env,want", [
    ({"OTEDAMA_CONFIG": "/etc/otd.yaml", "HOME": "/home/u"}, "/etc/otd.yaml"),
    ({"HOME": "/home/u"}, "/home/u/.config/otedama/config.yaml"),
])
def test_default_config_path(env, want):
    assert C.default_config_path(env) == want


def test_example_file_is_valid_and_documents_every_field():
    text = (ROOT / "config.yaml.example").read_text()
    cfg, warn = C.load_config_file(str(ROOT / "config.yaml.example"))
    assert warn is None
    cfg.validate()
    import dataclasses

    for f in dataclasses.fields(C.Config):
        assert re.search(rf"^#?\s*{f.name}:", text, re.M), f"config.yaml.example does not document {f.name}"
    for sub in (C.PoolConfig, C.MiningConfig, C.PoolServerConfig, C.WorkerConfig):
        for f in dataclasses.fields(sub):
            assert re.search(rf"^\s*#?\s*-?\s*{f.name}:", text, re.M), \
                f"config.yaml.example does not document {sub.__name__}.{f.name}"
