"""Layered configuration: defaults < file < env < flags, with per-field origins.

Parity: internal/config/config.go
  * Config / PoolConfig / WorkerConfig schema ........ config.go:59-229
  * Defaults (hysteresis 0.05, info, text) ........... config.go:236-250
  * FlagValues / Origins / ValueOrigin ............... config.go:261-312
  * numericEnvVars + EnvWarnings ..................... config.go:333-385
  * ResolveWithOrigins (zero value = unset in file) .. config.go:390-541
  * DefaultDataDir (XDG / macOS / Windows) ........... config.go:556-579
  * Validate (aggregated issues) ..................... config.go:586-664
  * address and pool-URL rules ....................... config.go:670-709
  * strict YAML loader (unknown key -> whole file
    rejected with a warning; empty file is valid) .... cmd/otedama/configfile.go:20-59

MI355X additions (all optional, same precedence rules): ``mining`` (algorithm,
gpus, cpu_threads, batch_nonces, version rolling) and ``pool_server`` (the local
Stratum pool: listen addresses, vardiff, journal).
"""
from __future__ import annotations

import dataclasses
import os
import sys
from dataclasses import dataclass, field
from enum import IntEnum
from pathlib import Path

import yaml

from otedama_amd import btccrypto

DEFAULT_POOL_URL = "stratum+v2://public.stratum.slushpool.com:3336"
VALID_POOL_SCHEMES = ("stratum+tcp://", "stratum+tls://", "stratum+v2://", "stratum+v2tls://")
PAYOUT_SCHEMES = ("", "fpps", "pplns", "tides", "solo")


class ConfigError(ValueError):
    pass


def _is_xonly_hex(s: str) -> bool:
    try:
        return len(s) == 64 and len(bytes.fromhex(s)) == 32
    except ValueError:
        return False


@dataclass
class PoolConfig:
    url: str = ""
    user: str = ""
    password: str = ""
    payout_scheme: str = ""
    tls_ca_file: str = ""
    sv2_extended_channel: bool = False  # SV2 only: extended channel (miner-side extranonce rolling)
    noise: bool = False                 # SV2 only: Noise NX encryption (spec §4); implied by pool_pubkey
    pool_pubkey: str = ""               # SV2 only: pinned authority key (64 hex chars, x-only secp256k1)
    noise_suite: str = "ellswift"       # SV2 Noise: "ellswift" (Noise_NX_Secp256k1+EllSwift_ChaChaPoly_SHA256, the
                                        # current spec) or "legacy" (32-byte x-only keys, rounds 1-2 wire format)
    target_grace: float = 0.0           # seconds after a difficulty raise during which shares found under the
                                        # previous, easier target are still submitted. Only for pools known to credit
                                        # them (otedama pool: RETARGET_GRACE 10 s); 0 = off, every share below the
                                        # target in force is dropped locally instead of being rejected by the pool


@dataclass
class WorkerConfig:
    name: str = ""


@dataclass
class MiningConfig:
    algorithm: str = "sha256d"          # sha256d | scrypt | x11
    gpus: str = "all"                   # "all", "none", or comma list of device indices
    cpu_threads: int = 0                # 0 = CPU miner only when no GPU is present
    batch_nonces: int = 1 << 32         # hashes per launch (SHA-256d): hits leave the GPU as they are found and new
                                        # work aborts a running launch, so only the launch tail / per-wave set-up cost
                                        # depends on it (2^32: ~0.22 s launches)
    version_rolling: bool = True        # BIP320 (negotiated with the pool)
    ntime_roll: int = 0
    sha_variants: int = 128             # SHA-256d header variants per GPU launch: 128 / 64 (version-parallel, two or
                                        # one per lane), 1..16 (K variants per lane; 1 = single midstate)
    isolation: str = "process"          # GPUs: "process" = one device process per GPU (a GPU fault stops one device,
                                        # the engine stays GPU-free); "thread" = every GPU's miner in this process


@dataclass
class PoolServerConfig:
    listen_sv2: str = ""                # e.g. 0.0.0.0:3336
    listen_v1: str = ""                 # e.g. 0.0.0.0:3333
    algorithm: str = "sha256d"
    initial_difficulty: float = 1.0
    target_share_seconds: float = 10.0
    vardiff_retarget_seconds: float = 30.0
    journal_path: str = ""
    coinbase_message: str = "/otedama-mi355x/"


@dataclass
class Config:
    bitcoin_address: str = ""
    bitcoin_addresses: list[str] = field(default_factory=list)
    pools: list[PoolConfig] = field(default_factory=list)
    workers: WorkerConfig = field(default_factory=WorkerConfig)
    language: str = ""
    log_level: str = "info"
    log_format: str = "text"
    data_dir: str = ""
    arbitration_hysteresis_pct: float = 0.05
    curtail_below_btc_usd: float = 0.0
    min_yield_sats_per_sec: float = 0.0
    power_watts: float = 0.0
    electricity_price_per_kwh: float = 0.0
    http_addr: str = ""
    mining: MiningConfig = field(default_factory=MiningConfig)
    pool_server: PoolServerConfig = field(default_factory=PoolServerConfig)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def validate(self) -> None:
        issues: list[str] = []
        if not self.bitcoin_address and not self.bitcoin_addresses:
            issues.append("bitcoin_address is required (set via --bitcoin-address, OTEDAMA_BITCOIN_ADDRESS, "
                          "or config file)")
        elif self.bitcoin_address:
            err = validate_bitcoin_address(self.bitcoin_address)
            if err:
                issues.append(f"bitcoin_address invalid: {err}")
        for i, a in enumerate(self.bitcoin_addresses):
            if not a:
                issues.append(f"bitcoin_addresses[{i}] is empty")
            else:
                err = validate_bitcoin_address(a)
                if err:
                    issues.append(f"bitcoin_addresses[{i}] invalid: {err}")
        if self.log_level not in ("debug", "info", "warn", "error", ""):
            issues.append(f"log_level {self.log_level!r} is not one of debug, info, warn, error")
        if self.log_format not in ("text", "json", ""):
            issues.append(f"log_format {self.log_format!r} is not one of text, json")
        for i, p in enumerate(self.pools):
            if not p.url:
                issues.append(f"pools[{i}].url is empty")
            else:
                err = validate_pool_url(p.url)
                if err:
                    issues.append(f"pools[{i}].url invalid: {err}")
            if (p.noise or p.pool_pubkey) and p.url and not p.url.startswith(("stratum+v2://", "stratum+v2tls://")):
                issues.append(f"pools[{i}]: noise / pool_pubkey apply to stratum+v2 URLs only")
            if not 0.0 <= float(p.target_grace) <= 60.0:
                issues.append(f"pools[{i}].target_grace {p.target_grace!r} must be within 0..60 seconds")
            if p.noise_suite not in ("ellswift", "legacy"):
                issues.append(f"pools[{i}].noise_suite {p.noise_suite!r} is not one of ellswift, legacy")
            if p.pool_pubkey and not _is_xonly_hex(p.pool_pubkey):
                issues.append(f"pools[{i}].pool_pubkey must be 64 hex characters (x-only secp256k1 key)")
            if p.payout_scheme not in PAYOUT_SCHEMES:
                issues.append(f"pools[{i}].payout_scheme {p.payout_scheme!r} is not one of fpps, pplns, tides, solo")
        if not 0 <= self.arbitration_hysteresis_pct < 1.0:
            issues.append(f"arbitration_hysteresis_pct {self.arbitration_hysteresis_pct:.4f} is out of range [0.0, 1.0)")
        for name, fmt_ in (("curtail_below_btc_usd", ".2f"), ("min_yield_sats_per_sec", ".4f"),
                           ("power_watts", ".2f"), ("electricity_price_per_kwh", ".4f")):
            v = getattr(self, name)
            if v < 0:
                issues.append(f"{name} {v:{fmt_}} must be >= 0 (0 = disabled)")
        if self.mining.algorithm not in ("sha256d", "scrypt", "x11"):
            issues.append(f"mining.algorithm {self.mining.algorithm!r} is not one of sha256d, scrypt, x11")
        if self.mining.cpu_threads < 0:
            issues.append("mining.cpu_threads must be >= 0")
        if not 1 << 16 <= self.mining.batch_nonces <= 1 << 32:
            issues.append("mining.batch_nonces must be in [65536, 2^32]")
        if self.mining.sha_variants not in (64, 128) and not 1 <= self.mining.sha_variants <= 16:
            issues.append(f"mining.sha_variants {self.mining.sha_variants} must be 128, 64 or 1..16")
        if self.mining.isolation not in ("process", "thread"):
            issues.append(f"mining.isolation {self.mining.isolation!r} must be process or thread")
        if self.pool_server.initial_difficulty <= 0:
            issues.append("pool_server.initial_difficulty must be > 0")
        if self.pool_server.target_share_seconds <= 0:
            issues.append("pool_server.target_share_seconds must be > 0")
        if issues:
            raise ConfigError("config validation failed:\n  - " + "\n  - ".join(issues))


class ValueOrigin(IntEnum):
    DEFAULT = 0
    FILE = 1
    ENV = 2
    FLAG = 3

    def __str__(self) -> str:
        return self.name.lower()


@dataclass
class FlagValues:
    bitcoin_address: str = ""
    log_level: str = ""
    log_format: str = ""
    language: str = ""
    data_dir: str = ""
    http_addr: str = ""


ORIGIN_FIELDS = (
    "bitcoin_address", "bitcoin_addresses", "pools", "worker_name", "language", "log_level", "log_format",
    "data_dir", "arbitration_hysteresis_pct", "curtail_below_btc_usd", "min_yield_sats_per_sec", "power_watts",
    "electricity_price_per_kwh", "http_addr", "mining", "pool_server",
)

NUMERIC_ENV_VARS = (
    ("OTEDAMA_ARBITRATION_HYSTERESIS_PCT", "arbitration_hysteresis_pct"),
    ("OTEDAMA_MIN_YIELD_SATS_PER_SEC", "min_yield_sats_per_sec"),
    ("OTEDAMA_CURTAIL_BELOW_BTC_USD", "curtail_below_btc_usd"),
    ("OTEDAMA_POWER_WATTS", "power_watts"),
    ("OTEDAMA_ELECTRICITY_PRICE_PER_KWH", "electricity_price_per_kwh"),
)
STRING_ENV_VARS = (
    ("OTEDAMA_BITCOIN_ADDRESS", "bitcoin_address"),
    ("OTEDAMA_LOG_LEVEL", "log_level"),
    ("OTEDAMA_LOG_FORMAT", "log_format"),
    ("OTEDAMA_LANGUAGE", "language"),
    ("OTEDAMA_DATA_DIR", "data_dir"),
    ("OTEDAMA_HTTP_ADDR", "http_addr"),
)


def _parse_go_float(v: str) -> float | None:
    try:
        return float(v.strip()) if v.strip() == v else float(v)
    except ValueError:
        return None


def env_warnings(env: dict[str, str] | None = None) -> list[str]:
    get = (env or os.environ).get
    out = []
    for key, _ in NUMERIC_ENV_VARS:
        v = get(key, "")
        if v and _parse_go_float(v) is None:
            out.append(f"{key}={v!r} is not a valid number; ignoring it and using the default".replace("'", '"'))
    return out


def resolve_with_origins(from_file: Config, env: dict[str, str] | None, flags: FlagValues):
    cfg = Config()
    o = {k: ValueOrigin.DEFAULT for k in ORIGIN_FIELDS}
    f = from_file
    if f.bitcoin_address:
        cfg.bitcoin_address, o["bitcoin_address"] = f.bitcoin_address, ValueOrigin.FILE
    if f.bitcoin_addresses:
        cfg.bitcoin_addresses, o["bitcoin_addresses"] = list(f.bitcoin_addresses), ValueOrigin.FILE
    if f.pools:
        cfg.pools, o["pools"] = list(f.pools), ValueOrigin.FILE
    if f.workers.name:
        cfg.workers.name, o["worker_name"] = f.workers.name, ValueOrigin.FILE
    file_keys = getattr(f, "_file_keys", None)
    for name in ("language", "log_level", "log_format", "data_dir", "http_addr"):
        set_in_file = name in file_keys if file_keys is not None else getattr(f, name) != getattr(cfg, name)
        if getattr(f, name) and set_in_file:
            setattr(cfg, name, getattr(f, name))
            o[name] = ValueOrigin.FILE
    # zero-value caveat: a numeric 0 in the file means "unset" (config.go:427-457)
    # (a field the file never set keeps its origin DEFAULT even when the dataclass default is non-zero)
    for name in ("arbitration_hysteresis_pct", "min_yield_sats_per_sec", "curtail_below_btc_usd", "power_watts",
                 "electricity_price_per_kwh"):
        set_in_file = name in file_keys if file_keys is not None else getattr(f, name) != getattr(cfg, name)
        if getattr(f, name) != 0 and set_in_file:
            setattr(cfg, name, getattr(f, name))
            o[name] = ValueOrigin.FILE
    if f.mining != MiningConfig():
        cfg.mining, o["mining"] = dataclasses.replace(f.mining), ValueOrigin.FILE
    if f.pool_server != PoolServerConfig():
        cfg.pool_server, o["pool_server"] = dataclasses.replace(f.pool_server), ValueOrigin.FILE

    get = (lambda k: (env or {}).get(k, "")) if env is not None else (lambda k: os.environ.get(k, ""))
    for key, name in STRING_ENV_VARS:
        v = get(key)
        if v:
            setattr(cfg, name, v)
            o[name] = ValueOrigin.ENV
    for key, name in NUMERIC_ENV_VARS:
        v = get(key)
        if v:
            fv = _parse_go_float(v)
            if fv is not None:
                setattr(cfg, name, fv)
                o[name] = ValueOrigin.ENV
    for name in ("bitcoin_address", "log_level", "log_format", "language", "data_dir", "http_addr"):
        v = getattr(flags, name)
        if v:
            setattr(cfg, name, v)
            o[name] = ValueOrigin.FLAG
    if not cfg.data_dir:
        cfg.data_dir = default_data_dir(env)
    return cfg, o


def resolve(from_file: Config, env: dict[str, str] | None, flags: FlagValues) -> Config:
    return resolve_with_origins(from_file, env, flags)[0]


def default_data_dir(env: dict[str, str] | None = None, platform: str | None = None) -> str:
    get = (env if env is not None else os.environ).get
    plat = platform or sys.platform
    if plat.startswith("win"):
        appdata = get("APPDATA", "")
        return os.path.join(appdata, "Otedama") if appdata else ""
    home = get("HOME", "") or os.path.expanduser("~")
    if plat == "darwin":
        return os.path.join(home, "Library", "Application Support", "Otedama") if home else ""
    xdg = get("XDG_DATA_HOME", "")
    if xdg:
        return os.path.join(xdg, "otedama")
    return os.path.join(home, ".local", "share", "otedama") if home else ""


def validate_bitcoin_address(addr: str) -> str | None:
    if len(addr) < 26:
        return f"address is too short ({len(addr)} characters)"
    if len(addr) > 90:
        return f"address is too long ({len(addr)} characters)"
    if not addr.startswith(("1", "3", "bc1")):
        return ("address does not start with '1', '3', or 'bc1'; testnet addresses are not supported in this "
                "configuration")
    try:
        btccrypto.validate_address(addr)
    except btccrypto.BtcCryptoError as exc:
        return f"checksum verification failed (likely a typo in the address): {exc}"
    return None


def validate_pool_url(raw: str) -> str | None:
    for s in VALID_POOL_SCHEMES:
        if raw.startswith(s):
            return None if raw[len(s):] else "URL has no host after scheme"
    return "URL must start with one of: " + ", ".join(VALID_POOL_SCHEMES)


# ------------------------------------------------------------------ YAML file

def _decode_strict(cls, data, path: str):
    if data is None:
        return cls()
    if not isinstance(data, dict):
        raise ConfigError(f"{path or 'config'}: expected a mapping")
    known = {f.name: f for f in dataclasses.fields(cls)}
    kwargs = {}
    for k, v in data.items():
        if k not in known:
            raise ConfigError(f"field {k} not found in type {cls.__name__}" + (f" (at {path})" if path else ""))
        ftype = known[k].type
        sub = f"{path}.{k}" if path else k
        if ftype in ("WorkerConfig", WorkerConfig):
            kwargs[k] = _decode_strict(WorkerConfig, v, sub)
        elif ftype in ("MiningConfig", MiningConfig):
            kwargs[k] = _decode_strict(MiningConfig, v, sub)
        elif ftype in ("PoolServerConfig", PoolServerConfig):
            kwargs[k] = _decode_strict(PoolServerConfig, v, sub)
        elif k == "pools":
            if not isinstance(v, list):
                raise ConfigError(f"{sub}: expected a list")
            kwargs[k] = [_decode_strict(PoolConfig, p, f"{sub}[{i}]") for i, p in enumerate(v)]
        elif k == "bitcoin_addresses":
            if not isinstance(v, list) or not all(isinstance(a, str) for a in v):
                raise ConfigError(f"{sub}: expected a list of strings")
            kwargs[k] = list(v)
        else:
            default = known[k].default
            if isinstance(default, bool):
                if not isinstance(v, bool):
                    raise ConfigError(f"{sub}: expected a boolean")
            elif isinstance(default, float):
                if isinstance(v, bool) or not isinstance(v, (int, float)):
                    raise ConfigError(f"{sub}: expected a number")
                v = float(v)
            elif isinstance(default, int):
                if isinstance(v, bool) or not isinstance(v, int):
                    raise ConfigError(f"{sub}: expected an integer")
            elif isinstance(default, str):
                if v is None:
                    v = ""
                elif isinstance(v, (int, float)) and not isinstance(v, bool):
                    v = str(v)
                elif not isinstance(v, str):
                    raise ConfigError(f"{sub}: expected a string")
            kwargs[k] = v
    return cls(**kwargs)


def parse_config_yaml(text: str) -> Config:
    data = yaml.safe_load(text) if text.strip() else None
    cfg = _decode_strict(Config, data, "")
    # keys the file actually set (Go decodes into zero values, so only these count as FILE origin)
    cfg._file_keys = set(data) if isinstance(data, dict) else set()
    return cfg


def load_config_file(path: str | os.PathLike | None) -> tuple[Config, str | None]:
    """Returns (config, warning). Missing file -> empty config, no warning; a
    parse error or unknown key -> empty config plus a warning (whole file ignored)."""
    if not path:
        return Config(), None
    p = Path(path)
    try:
        text = p.read_text()
    except FileNotFoundError:
        return Config(), None
    except OSError as exc:
        return Config(), f"config file {p}: {exc}"
    try:
        return parse_config_yaml(text), None
    except (yaml.YAMLError, ConfigError, TypeError) as exc:
        return Config(), f"config file {p} ignored: {exc}"


def default_config_path(env: dict[str, str] | None = None) -> str:
    get = (env if env is not None else os.environ).get
    if get("OTEDAMA_CONFIG"):
        return get("OTEDAMA_CONFIG")
    home = get("HOME", "") or os.path.expanduser("~")
    return os.path.join(home, ".config", "otedama", "config.yaml") if home else ""
