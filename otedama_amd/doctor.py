"""Self-diagnosis: parallel checks with fix hints, text / JSON report, exit 0/1/2.

Parity: internal/doctor/{doctor,checks}.go
  * Status pass|warn|fail|skip with symbols ✓ ! ✗ - ............... doctor.go:43-84
  * Result / Check / Report, ExitCode 0 pass / 1 warn / 2 fail ....... doctor.go:87-129
  * Print ("[✓] Name: detail", "    → fix: ...", summary line) ...... doctor.go:132-160
  * WriteJSON (summary, duration_ms, exit_code, checks) ............. doctor.go:166-217
  * Runner.Run: every check in parallel under one deadline .......... doctor.go:226-244
  * DefaultChecks: the 17 reference checks (names kept) ............ checks.go:32-52
MI355X additions: "Native extension" (the gfx950 kernels are built and load),
"GPU runtime" (HIP devices and their ISA), "Collectives" (torch.distributed
backends for one-rank-per-GPU RCCL).
Network seams (pool dial, network endpoint, clock probe URL, resolver, DRM
path) are module attributes so tests can point them at loopback servers.
"""
from __future__ import annotations

import email.utils
import json
import os
import socket
import stat
import threading
import time
import urllib.request
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Callable, TextIO

from otedama_amd import config as C
from otedama_amd.poolproto.base import from_url, split_host_port, strip_scheme


class Status(IntEnum):
    PASS = 0
    WARN = 1
    FAIL = 2
    SKIP = 3

    def __str__(self) -> str:
        return self.name.lower()

    @property
    def symbol(self) -> str:
        return {Status.PASS: "✓", Status.WARN: "!", Status.FAIL: "✗"}.get(self, "-")


@dataclass
class Result:
    name: str = ""
    status: Status = Status.PASS
    detail: str = ""
    fix: str = ""
    elapsed: float = 0.0


@dataclass
class Check:
    name: str
    run: Callable[[], Result]


@dataclass
class Report:
    results: list[Result] = field(default_factory=list)
    duration: float = 0.0

    def exit_code(self) -> int:
        if any(r.status == Status.FAIL for r in self.results):
            return 2
        if any(r.status == Status.WARN for r in self.results):
            return 1
        return 0

    def _counts(self):
        c = {s: 0 for s in Status}
        for r in self.results:
            c[r.status] += 1
        return c

    def print(self, w: TextIO) -> None:
        for r in self.results:
            w.write(f"[{r.status.symbol}] {r.name}: {r.detail}\n")
            if r.fix:
                w.write(f"    → fix: {r.fix}\n")
        c = self._counts()
        w.write("\n")
        s = f"Summary: {c[Status.PASS]} passed, {c[Status.FAIL]} failed, {c[Status.WARN]} warning"
        if c[Status.WARN] != 1:
            s += "s"
        if c[Status.SKIP]:
            s += f", {c[Status.SKIP]} skipped"
        w.write(s + f" (completed in {self.duration * 1000:.0f}ms)\n")

    def write_json(self, w: TextIO) -> None:
        c = self._counts()
        doc = {
            "summary": {"passed": c[Status.PASS], "failed": c[Status.FAIL], "warnings": c[Status.WARN],
                        "skipped": c[Status.SKIP]},
            "duration_ms": int(self.duration * 1000), "exit_code": self.exit_code(),
            "checks": [{"name": r.name, "status": str(r.status), "detail": r.detail,
                        **({"fix": r.fix} if r.fix else {}), "elapsed_ms": int(r.elapsed * 1000)}
                       for r in self.results],
        }
        w.write(json.dumps(doc, indent=2, ensure_ascii=False) + "\n")


class Runner:
    def __init__(self, checks: list[Check], timeout: float = 30.0):
        self.checks = checks
        self.timeout = timeout

    def run(self) -> Report:
        """One daemon thread per check (doctor.go:226-244). A check still running at ``timeout`` is reported as
        FAIL "check timed out" and abandoned; the report never waits for it."""
        t0 = time.monotonic()
        results: list[Result | None] = [None] * len(self.checks)
        done = threading.Semaphore(0)

        def run_one(i: int, c: Check) -> None:
            results[i] = self._one(c)
            done.release()

        for i, c in enumerate(self.checks):
            threading.Thread(target=run_one, args=(i, c), name=f"otedama-doctor-{i}", daemon=True).start()
        deadline = t0 + self.timeout
        for _ in self.checks:
            if not done.acquire(timeout=max(0.0, deadline - time.monotonic())):
                break
        out = []
        for i, c in enumerate(self.checks):
            r = results[i]
            out.append(r if r is not None else Result(c.name, Status.FAIL, "check timed out", "", self.timeout))
        return Report(out, time.monotonic() - t0)

    @staticmethod
    def _one(c: Check) -> Result:
        t0 = time.monotonic()
        try:
            r = c.run()
        except Exception as exc:  # noqa: BLE001
            r = Result(status=Status.FAIL, detail=f"check crashed: {exc}")
        r.name = c.name
        r.elapsed = time.monotonic() - t0
        return r


# ----------------------------------------------------------------------- seams
network_check_endpoint = ("1.1.1.1", 53)
clock_skew_probe_url = "https://api.coinbase.com/v2/time"
gpu_drm_path = "/sys/class/drm"
dial_timeout = 5.0


def pool_dial(host: str, port: int, timeout: float) -> None:
    with socket.create_connection((host, port), timeout=timeout):
        pass


def resolve_host(host: str) -> list[str]:
    return sorted({ai[4][0] for ai in socket.getaddrinfo(host, None)})


# ----------------------------------------------------------------------- checks
def check_configuration(cfg: C.Config, path: str) -> Check:
    """checks.go:54-85: no config file -> warn, a named file that does not exist -> warn, a file whose resolved
    configuration fails validation -> fail, else pass. Without a file the validation errors (if any) are
    appended to the warning instead of being dropped."""
    def run():
        def invalid() -> str:
            try:
                cfg.validate()
            except C.ConfigError as exc:
                return str(exc).replace("\n", " ")
            return ""

        if not path:
            err = invalid()
            return Result(status=Status.WARN,
                          detail="no config file found; using defaults and env vars" + (f" ({err})" if err else ""),
                          fix="create ~/.config/otedama/config.yaml (see config.yaml.example)")
        if not os.path.exists(path):
            return Result(status=Status.WARN, detail=f"config file {path!r} not found",
                          fix="pass --config /path/to/config.yaml or create the default file")
        err = invalid()
        if err:
            return Result(status=Status.FAIL, detail=f"config invalid: {err}",
                          fix="edit the config file or pass missing flags on the command line")
        return Result(detail=f"loaded from {path}")
    return Check("Configuration", run)


BECH32_CHARS = "qpzry9x8gf2tvdw0s3jn54khce6mua7l"
BASE58_CHARS = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def is_bech32_char(c: str) -> bool:
    return len(c) == 1 and c in BECH32_CHARS


def is_base58_char(c: str) -> bool:
    return len(c) == 1 and c in BASE58_CHARS


def is_likely_bitcoin_address(s: str) -> bool:
    """Cheap shape check before the checksum (checks.go:862-887): 26..90 characters, ``bc1`` + lowercase bech32
    characters, or ``1``/``3`` + base58 characters."""
    s = s.strip()
    if not 26 <= len(s) <= 90:
        return False
    if s.startswith("bc1"):
        return all(is_bech32_char(c) for c in s[3:])
    if s[0] in "13":
        return all(is_base58_char(c) for c in s[1:])
    return False


def mask_address(s: str) -> str:
    """First 6 and last 4 characters around three middle dots; 10 characters or fewer unchanged (checks.go:899)."""
    return s if len(s) <= 10 else s[:6] + "\u00b7" * 3 + s[-4:]


def address_kind(addr: str) -> str:
    """Human label of the address type, so the report shows the address was understood (checks.go:128-143)."""
    from otedama_amd.btccrypto import AddressType, classify_address

    return {AddressType.P2PKH: "P2PKH legacy", AddressType.P2SH: "P2SH", AddressType.P2WPKH: "P2WPKH SegWit v0",
            AddressType.P2WSH: "P2WSH SegWit v0", AddressType.P2TR: "P2TR Taproot"}.get(
        classify_address(addr.strip()), "unrecognised type")


def append_unique(xs: list[str], x: str) -> list[str]:
    if x not in xs:
        xs.append(x)
    return xs


def check_bitcoin_address(cfg: C.Config) -> Check:
    """checks.go:87-123: shape check, then the bech32/bech32m/Base58Check checksum; the pass detail names the
    masked address and its type. Beyond the reference: no primary address but a failover list is a warning."""
    def run():
        addr = cfg.bitcoin_address
        if not addr:
            if cfg.bitcoin_addresses:
                return Result(status=Status.WARN, detail="no primary bitcoin_address; using failover list only",
                              fix="set bitcoin_address to the address you want paid first")
            return Result(status=Status.FAIL, detail="no address configured",
                          fix="pass --bitcoin-address bc1q... or set OTEDAMA_BITCOIN_ADDRESS")
        if not is_likely_bitcoin_address(addr):
            return Result(status=Status.FAIL, detail=f"{addr!r} does not look like a valid address",
                          fix="verify the address — typos here would send your earnings to strangers")
        err = C.validate_bitcoin_address(addr.strip())
        if err:
            return Result(status=Status.FAIL, detail=f"{mask_address(addr)}: {err} (checksum)",
                          fix="re-check the address character by character; the checksum does not match "
                              "(likely a typo)")
        return Result(detail=f"{mask_address(addr)} ({address_kind(addr)}, likely valid)")
    return Check("Bitcoin address", run)


def check_failover_addresses(cfg: C.Config) -> Check:
    """checks.go:149-181: every failover address gets the shape and checksum checks; the first bad entry fails
    with its index. Beyond the reference: a repeated address (or the primary listed again) is a warning."""
    def run():
        addrs = cfg.bitcoin_addresses
        if not addrs:
            return Result(status=Status.SKIP, detail="none configured")
        for i, a in enumerate(addrs):
            if not a or not is_likely_bitcoin_address(a):
                return Result(status=Status.FAIL, detail=f"bitcoin_addresses[{i}] {a!r} does not look valid",
                              fix="verify every failover address — a typo would send earnings to strangers")
            err = C.validate_bitcoin_address(a.strip())
            if err:
                return Result(status=Status.FAIL, detail=f"bitcoin_addresses[{i}] {mask_address(a)}: {err}",
                              fix="re-check the failover address; its checksum does not match (likely a typo)")
        if len(addrs) != len(set(addrs)) or cfg.bitcoin_address in addrs:
            return Result(status=Status.WARN, detail="failover list repeats an address",
                          fix="list each payout address once")
        return Result(detail=f"{len(addrs)} failover address(es), all likely valid")
    return Check("Failover payout addresses", run)


def _resolve_data_dir(cfg: C.Config) -> str:
    """The configured data dir, else the OS default the engine would use (checks.go:187-195)."""
    return cfg.data_dir or C.default_data_dir()


def check_data_dir(cfg: C.Config) -> Check:
    """checks.go:183-235: missing -> warn (created on first run), stat error / not a directory -> fail, group or
    world permission bits -> warn. Beyond the reference: an existing directory must be writable, and a missing
    one whose nearest existing parent is not writable fails (the first run could not create it)."""
    def run():
        d = _resolve_data_dir(cfg)
        if not d:
            return Result(status=Status.SKIP, detail="no home directory")
        try:
            st = os.stat(d)
        except FileNotFoundError:
            parent = os.path.dirname(os.path.abspath(d).rstrip("/")) or "/"
            while not os.path.exists(parent) and parent != "/":
                parent = os.path.dirname(parent)
            if not os.access(parent, os.W_OK):
                return Result(status=Status.FAIL, detail=f"{d} does not exist and {parent} is not writable",
                              fix=f"create {d} or choose a writable --data-dir")
            return Result(status=Status.WARN, detail=f"{d} does not exist (will be created on first run)")
        except OSError as exc:
            return Result(status=Status.FAIL, detail=f"cannot stat {d}: {exc}", fix="check filesystem permissions")
        if not stat.S_ISDIR(st.st_mode):
            return Result(status=Status.FAIL, detail=f"{d} is not a directory",
                          fix="remove the file and restart Otedama")
        if not os.access(d, os.W_OK):
            return Result(status=Status.FAIL, detail=f"{d} is not writable", fix=f"chmod u+w {d}")
        mode = st.st_mode & 0o777
        if mode & 0o077:
            return Result(status=Status.WARN, detail=f"{d} has permissions {mode:04o} (world/group readable)",
                          fix=f"run: chmod 0700 {d}")
        return Result(detail=f"{d} (exists, writable)")
    return Check("Data directory", run)


def check_wallet(cfg: C.Config) -> Check:
    """checks.go:249-292: no wallet.dat -> warn with the passphrase hint, stat error -> fail, otherwise pass with
    the public fingerprint (trimmed) or a note that the fingerprint file is missing. Beyond the reference:
    wallet.dat must parse as the seedstore format (no KDF run) and be private (mode 0600)."""
    def run():
        d = _resolve_data_dir(cfg)
        if not d:
            return Result(status=Status.SKIP, detail="no home directory; cannot locate wallet")
        path = os.path.join(d, "wallet.dat")
        try:
            st = os.stat(path)
        except FileNotFoundError:
            return Result(status=Status.WARN, detail=f"no wallet found in {d}",
                          fix="set --wallet-passphrase or OTEDAMA_WALLET_PASSPHRASE to create a wallet on next run")
        except OSError as exc:
            return Result(status=Status.FAIL, detail=f"cannot stat {path}: {exc}", fix="check filesystem permissions")
        try:
            from otedama_amd.lightning.seedstore import unmarshal

            with open(path, "rb") as f:
                unmarshal(f.read())
        except Exception as exc:  # noqa: BLE001
            return Result(status=Status.FAIL, detail=f"wallet.dat unreadable: {exc}",
                          fix="restore wallet.dat from backup or recreate it from your recovery phrase")
        mode = st.st_mode & 0o777
        if mode & 0o077:
            return Result(status=Status.WARN, detail=f"wallet.dat mode {mode:o} is too permissive",
                          fix=f"chmod 600 {path}")
        try:
            with open(os.path.join(d, "wallet.fingerprint"), encoding="utf-8", errors="replace") as f:
                fp = f.read().strip()
        except OSError:
            return Result(detail="initialized (fingerprint file missing; re-run to regenerate)")
        return Result(detail=f"initialized, fingerprint: {fp}")
    return Check("Lightning wallet", run)


def _pool_targets(cfg: C.Config, unparsed: list[str] | None = None) -> list[tuple[str, str, int]]:
    """(url, host, port) of every configured pool, or of the built-in default. URLs that do not parse are left
    out, and appended to ``unparsed`` when given."""
    urls = [p.url for p in cfg.pools] or [C.DEFAULT_POOL_URL]
    out = []
    for u in urls:
        try:
            rest = strip_scheme(u)
            proto = from_url(u)
            host, port = split_host_port(rest, 3336 if proto.value.startswith("stratum-v2") else 3333)
        except Exception:  # noqa: BLE001
            if unparsed is not None:
                unparsed.append(u)
            continue
        out.append((u, host, port))
    return out


def check_pool_reachability(cfg: C.Config) -> Check:
    """checks.go:294-330 dials the first pool only; this dials every configured pool (or the default). An
    unparseable URL counts as unreachable ("cannot parse pool URL"), so a config of only bad URLs fails."""
    def run():
        ok, bad, unparsed = [], [], []
        for u, host, port in _pool_targets(cfg, unparsed):
            t0 = time.monotonic()
            try:
                pool_dial(host, port, dial_timeout)
                ok.append(f"{host}:{port} ({(time.monotonic() - t0) * 1000:.0f}ms)")
            except OSError as exc:
                bad.append(f"{u} ({exc})")
        bad += [f"cannot parse pool URL {u!r}" for u in unparsed]
        if not bad:
            return Result(detail=f"{len(ok)} pool(s) reachable: {', '.join(ok)}")
        if ok:
            return Result(status=Status.WARN, detail=f"unreachable: {'; '.join(bad)}",
                          fix="check the pool URL/port or remove dead pools")
        return Result(status=Status.FAIL, detail=f"no pool reachable: {'; '.join(bad)}",
                      fix="check network/firewall and the pool URLs")
    return Check("Pool reachability", run)


def check_pool_diversity(cfg: C.Config) -> Check:
    def run():
        n = len(cfg.pools)
        if n == 0:
            return Result(status=Status.WARN, detail="using built-in default pool (no failover configured)",
                          fix="add at least two pools under 'pools:' in config.yaml for automatic failover")
        if n == 1:
            return Result(status=Status.WARN,
                          detail=f"only one pool configured ({cfg.pools[0].url}) — no automatic failover",
                          fix="add a second pool under 'pools:' in config.yaml; mining stops if this pool goes down")
        return Result(detail=f"{n} pools configured; failover available")
    return Check("Pool diversity", run)


def check_pool_endpoint_diversity(cfg: C.Config) -> Check:
    def run():
        if len(cfg.pools) < 2:
            return Result(status=Status.SKIP, detail="fewer than two pools configured")
        ip_to: dict[str, list[str]] = {}
        resolved = 0
        for u, host, _ in _pool_targets(cfg):
            try:
                ips = resolve_host(host)
            except OSError:
                continue
            resolved += 1
            for ip in ips:
                ip_to.setdefault(ip, [])
                if u not in ip_to[ip]:
                    ip_to[ip].append(u)
        if resolved < 2:
            return Result(status=Status.SKIP, detail="could not resolve enough pool endpoints to compare")
        for ip, urls in ip_to.items():
            if len(urls) >= 2:
                return Result(status=Status.WARN,
                              detail=f"pools {', '.join(urls)} resolve to the same endpoint {ip} — failover is "
                                     "illusory",
                              fix="configure pools run by different operators so one outage cannot take down both")
        return Result(detail=f"{resolved} pools resolve to distinct endpoints")
    return Check("Pool endpoint diversity", run)


def check_pool_encryption(cfg: C.Config) -> Check:
    def run():
        if not cfg.pools:
            return Result(status=Status.SKIP, detail="using built-in default pool")
        plain = [p.url for p in cfg.pools if not from_url(p.url).uses_tls]
        if plain:
            return Result(status=Status.WARN, detail=f"plaintext pool connection(s): {', '.join(plain)}",
                          fix="use stratum+tls:// or stratum+v2tls:// so shares and payout address are not "
                              "exposed on the wire")
        return Result(detail="all pool connections use TLS")
    return Check("Pool connection encryption", run)


def check_pool_tls_ca(cfg: C.Config) -> Check:
    def run():
        files = [(p.url, p.tls_ca_file) for p in cfg.pools if p.tls_ca_file]
        if not files:
            return Result(status=Status.SKIP, detail="no custom TLS CA files configured")
        import ssl

        for url, f in files:
            if not os.path.exists(f):
                return Result(status=Status.FAIL, detail=f"{url}: CA file {f} does not exist",
                              fix="fix tls_ca_file or remove it to use the system roots")
            try:
                ssl.create_default_context().load_verify_locations(cafile=f)
            except (ssl.SSLError, OSError) as exc:
                return Result(status=Status.FAIL, detail=f"{url}: CA file {f} is not valid PEM: {exc}",
                              fix="provide a PEM-encoded CA bundle")
        return Result(detail=f"{len(files)} CA file(s) load")
    return Check("Pool TLS CA files", run)


def check_power_cost(cfg: C.Config) -> Check:
    def run():
        w, p = cfg.power_watts, cfg.electricity_price_per_kwh
        if w <= 0 and p <= 0:
            return Result(status=Status.SKIP, detail="power_watts / electricity_price_per_kwh not set")
        if (w > 0) != (p > 0):
            return Result(status=Status.WARN, detail="only one of power_watts / electricity_price_per_kwh is set",
                          fix="set both to get otedama_power_cost_usd_per_hour")
        return Result(detail=f"{w:g} W at ${p:g}/kWh = ${w / 1000 * p:.4f}/h")
    return Check("Power & cost config", run)


def check_env_vars() -> Check:
    def run():
        warns = C.env_warnings()
        if warns:
            return Result(status=Status.WARN, detail="; ".join(warns), fix="fix or unset the listed variables")
        n = sum(1 for k in os.environ if k.startswith("OTEDAMA_"))
        return Result(detail=f"{n} OTEDAMA_* variable(s) set; all parse")
    return Check("Environment variables", run)


def check_profitability_floor(cfg: C.Config) -> Check:
    def run():
        if cfg.min_yield_sats_per_sec <= 0:
            return Result(status=Status.SKIP, detail="min_yield_sats_per_sec not set (devices never idled for yield)")
        return Result(detail=f"devices idle below {cfg.min_yield_sats_per_sec:g} sats/s")
    return Check("Profitability floor", run)


def check_payout_scheme(cfg: C.Config) -> Check:
    desc = {"fpps": "FPPS — smooth payouts, pool absorbs variance (typically higher fee)",
            "pplns": "PPLNS — lower fee, miner absorbs variance; expect payout variability",
            "tides": "TIDES — non-custodial coinbase payouts",
            "solo": "Solo — full block reward or nothing; only viable for large miners"}

    def run():
        if not cfg.pools:
            return Result(status=Status.SKIP, detail="no pools configured; using built-in default")
        lines, unknown = [], False
        for p in cfg.pools:
            try:
                host = strip_scheme(p.url)
            except Exception:  # noqa: BLE001 - unknown scheme or empty host: show the raw URL
                host = p.url
            if p.payout_scheme in desc:
                lines.append(f"{host}: {desc[p.payout_scheme]}")
            else:
                lines.append(f"{host}: scheme not set")
                unknown = True
        return Result(detail="; ".join(lines),
                      fix="set payout_scheme: fpps/pplns/tides/solo in config.yaml for variance/custody context"
                      if unknown else "")
    return Check("Pool payout schemes", run)


def check_hardware() -> Check:
    def run():
        detail = f"{os.cpu_count() or 1}-core CPU"
        try:
            from otedama_amd.ops.native import load

            n = load(build_if_missing=False)
            gpus = n.gpu_device_count() if n else 0
        except Exception:  # noqa: BLE001
            gpus = 0
        if gpus:
            return Result(detail=detail + f", {gpus} HIP GPU(s)")
        drm = 0
        try:
            drm = sum(1 for e in os.listdir(gpu_drm_path) if e.startswith("renderD"))
        except OSError:
            pass
        if drm:
            # checks.go:696-705 reports DRM render nodes as "GPU(s) detected" (pass). Here the gfx950 kernels need
            # the HIP runtime too, so render nodes without a HIP device are a warning.
            return Result(status=Status.WARN, detail=detail + f", {drm} GPU(s) detected (render nodes) but no HIP "
                                                              "device",
                          fix="install the ROCm runtime / amdgpu driver so the gfx950 kernels can run")
        return Result(detail=detail + ", no GPU detected (CPU SHA-NI miner only)")
    return Check("Hardware", run)


def check_network() -> Check:
    """checks.go:728-746: a TCP dial of 1.1.1.1:53 (3 s); unreachable is a failure."""
    def run():
        host, port = network_check_endpoint
        try:
            pool_dial(host, port, min(dial_timeout, 3.0))
        except OSError as exc:
            return Result(status=Status.FAIL, detail=f"cannot reach {host}:{port}: {exc}",
                          fix="check your firewall, proxy, or VPN")
        return Result(detail="IPv4 OK")
    return Check("Network", run)


CLOCK_SKEW_WARN_SECS = 120.0  # checks.go:761 (= the rate fetcher's skew warning)
CLOCK_SKEW_FAIL_SECS = 300.0  # checks.go:766: most TLS stacks start rejecting certificates


def check_clock() -> Check:
    """checks.go:768-852: GET the probe URL and compare its Date header. An unreachable probe, a missing or an
    unparseable Date header warn; skew > 120 s warns, > 300 s fails. The body is drained (bounded, 8 KiB)
    before the connection closes."""
    def run():
        try:
            req = urllib.request.Request(clock_skew_probe_url, method="GET",
                                         headers={"User-Agent": f"Otedama/{_version()} (doctor)"})
        except ValueError as exc:
            return Result(status=Status.WARN, detail=f"could not build request: {exc}",
                          fix="this is an internal error; report it")
        try:
            with urllib.request.urlopen(req, timeout=dial_timeout) as resp:  # noqa: S310
                date = resp.headers.get("Date")
                resp.read(8 << 10)
        except Exception as exc:  # noqa: BLE001
            return Result(status=Status.WARN, detail=f"cannot reach clock probe endpoint: {exc}",
                          fix="check internet connectivity; re-run when online to verify clock accuracy")
        if not date:
            return Result(status=Status.WARN, detail="server returned no Date header; cannot measure clock skew",
                          fix="try again; if persistent, the probe endpoint may have changed")
        try:
            skew = abs(time.time() - email.utils.parsedate_to_datetime(date).timestamp())
        except (TypeError, ValueError) as exc:
            return Result(status=Status.WARN, detail=f"cannot parse server Date header {date[:40]!r}: {exc}",
                          fix="try again; if persistent, the probe endpoint date format may have changed")
        if skew > CLOCK_SKEW_FAIL_SECS:
            return Result(status=Status.FAIL,
                          detail=f"local clock is {skew:.0f} s off server time (threshold {CLOCK_SKEW_FAIL_SECS:.0f} s)",
                          fix="synchronise your system clock (e.g. `timedatectl set-ntp true`); skew >300 s breaks "
                              "TLS certificate validation and mining nTime checks")
        if skew > CLOCK_SKEW_WARN_SECS:
            return Result(status=Status.WARN,
                          detail=f"local clock is {skew:.0f} s off server time (warn threshold "
                                 f"{CLOCK_SKEW_WARN_SECS:.0f} s)",
                          fix="synchronise your system clock; skew above 120 s may cause TLS errors or stale rate "
                              "judgements")
        return Result(detail=f"clock skew {skew:.1f} s (within {CLOCK_SKEW_WARN_SECS:.0f} s threshold)")
    return Check("System clock accuracy", run)


def _version() -> str:
    try:
        from otedama_amd import version

        return version.get().version
    except Exception:  # noqa: BLE001
        return "dev"


def check_native() -> Check:
    def run():
        from otedama_amd.ops.native import load

        n = load(build_if_missing=False)
        if n is None:
            return Result(status=Status.FAIL, detail="otedama_amd._native not built",
                          fix="python -m otedama_amd._build (needs ROCm hipcc for gfx950)")
        scan = n.cpu_scan_method() if hasattr(n, "cpu_scan_method") else "?"
        return Result(detail=f"native extension loaded (SHA-NI={'yes' if n.cpu_has_sha_ni() else 'no'}, "
                             f"CPU scan: {scan})")
    return Check("Native extension", run)


def check_gpu_runtime() -> Check:
    def run():
        from otedama_amd.ops.native import load

        n = load(build_if_missing=False)
        if n is None or n.gpu_device_count() == 0:
            return Result(status=Status.SKIP, detail="no HIP device visible")
        archs = [n.gpu_arch_name(i).split(":")[0] for i in range(n.gpu_device_count())]
        other = [a for a in archs if a != "gfx950"]
        if other:
            return Result(status=Status.WARN, detail=f"devices {archs}: kernels are built for gfx950 only",
                          fix="MI355X (gfx950) is the supported GPU")
        return Result(detail=f"{len(archs)} x gfx950 ({n.gpu_cu_count(0)} CUs each)")
    return Check("GPU runtime", run)


def check_collectives() -> Check:
    """The multi-GPU data plane: the native RCCL module the node and bench.py use (``otedama_amd._rccl``), the
    torch.distributed fallback backends, dmabuf IPC, and the xGMI links between the visible GPUs (KFD topology)."""
    def run():
        status, fix, parts = Status.PASS, "", []
        try:
            from otedama_amd.parallel.rcclcomm import rccl_module

            parts.append(f"native RCCL module {rccl_module().version()}")
        except Exception as exc:  # noqa: BLE001
            status, fix = Status.WARN, "python -m otedama_amd._build (builds otedama_amd._rccl against librccl)"
            parts.append(f"native RCCL module unavailable ({type(exc).__name__})")
        try:
            import torch.distributed as dist

            nccl = dist.is_nccl_available()
            parts.append(f"fallback backends: nccl(RCCL)={'yes' if nccl else 'no'}, "
                         f"gloo={'yes' if dist.is_gloo_available() else 'no'}")
        except Exception as exc:  # noqa: BLE001
            nccl = False
            parts.append(f"torch.distributed unavailable ({type(exc).__name__})")
        if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "") != "0" and nccl:
            status, fix = Status.WARN, "export HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC) for multi-process RCCL"
            parts.append("HSA_ENABLE_IPC_MODE_LEGACY is not 0")
        from otedama_amd import hal

        topo = hal.kfd_topology()
        n = len(topo["gpus"])
        if n > 1:
            pairs = n * (n - 1)
            x = sum(1 for ln in topo["links"] if ln.get("type") == "xgmi")
            hives = {g.get("hive_id") for g in topo["gpus"]}
            parts.append(f"{n} GPUs: {x}/{pairs} directed pairs on xGMI, {len(hives)} hive(s)")
            if x < pairs and status == Status.PASS:
                status = Status.WARN
                fix = "GPU pairs without xGMI move R1/R2/R3 over PCIe; check the node's topology (rocm-smi --showtopo)"
        return Result(status=status, detail="; ".join(parts), fix=fix)
    return Check("Collectives", run)


def check_pow_self_test(cfg: C.Config) -> Check:
    """CPU oracle of the configured algorithm vs its known answer; on a gfx950 box also one tiny GPU search
    that must find the known nonce (SHA-256d / X11 genesis blocks) or match the oracle (scrypt)."""
    def run():
        from otedama_amd.models import algorithms

        algo = cfg.mining.algorithm
        try:
            detail = algorithms.self_test(algo)
        except Exception as exc:  # noqa: BLE001 - any failure is the finding
            return Result(status=Status.FAIL, detail=str(exc), fix="rebuild the native extension (make build)")
        from otedama_amd.ops.native import load

        n = load(build_if_missing=False)
        if n is None or n.gpu_device_count() == 0 or not n.gpu_arch_name(0).startswith("gfx950"):
            return Result(detail=detail + "; no gfx950 device for the GPU kernel check")
        try:
            detail += "; " + _gpu_kernel_self_test(algo)
        except Exception as exc:  # noqa: BLE001
            return Result(status=Status.FAIL, detail=f"{detail}; GPU kernel: {exc}",
                          fix="run `python -m pytest tests -m gpu` to locate the failing kernel")
        return Result(detail=detail)
    return Check("PoW self-test", run)


def _gpu_kernel_self_test(algo: str) -> str:
    import torch

    from otedama_amd.models import algorithms
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import ScryptSearch, Sha256dSearch, X11Search

    if algo == "scrypt":
        hdr = bytes(range(76)) + bytes(4)
        s = ScryptSearch("cuda:0", grid=64)
        got = s.search(hdr, int_to_hash((1 << 256) - 1), 0, 4)
        if sorted(got) != [0, 1, 2, 3]:
            raise AssertionError(f"scrypt kernel hits {got}")
        torch.cuda.synchronize()
        return "gfx950 scrypt kernel ran"
    hdr_hex, nonce, _ = algorithms.KNOWN_ANSWERS[algo]
    hdr = bytes.fromhex(hdr_hex)
    bits = int.from_bytes(hdr[72:76], "little")
    target = int_to_hash((bits & 0xFFFFFF) << (8 * ((bits >> 24) - 3)))
    s = Sha256dSearch("cuda:0") if algo == "sha256d" else X11Search("cuda:0", batch=1 << 16)
    got = s.search(hdr, target, nonce - 1000, 1 << 16)
    if nonce not in got:
        raise AssertionError(f"{algo} kernel missed the genesis nonce ({got})")
    return f"gfx950 {algo} kernel finds the genesis nonce"


def default_checks(cfg: C.Config, config_path: str = "") -> list[Check]:
    return [
        check_configuration(cfg, config_path), check_bitcoin_address(cfg), check_failover_addresses(cfg),
        check_data_dir(cfg), check_wallet(cfg), check_pool_reachability(cfg), check_pool_diversity(cfg),
        check_pool_endpoint_diversity(cfg), check_pool_encryption(cfg), check_pool_tls_ca(cfg),
        check_power_cost(cfg), check_env_vars(), check_profitability_floor(cfg), check_payout_scheme(cfg),
        check_hardware(), check_network(), check_clock(), check_native(), check_gpu_runtime(), check_collectives(),
        check_pow_self_test(cfg),
    ]
