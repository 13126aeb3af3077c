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
    def run():
        try:
            cfg.validate()
        except C.ConfigError as exc:
            return Result(status=Status.FAIL, detail=str(exc).replace("\n", " "),
                          fix="fix the listed fields via flags, OTEDAMA_* env vars or the config file")
        src = path or C.default_config_path()
        exists = bool(src) and os.path.exists(src)
        return Result(detail=f"configuration valid ({'file ' + src if exists else 'no config file; flags/env only'})")
    return Check("Configuration", run)


def check_bitcoin_address(cfg: C.Config) -> Check:
    def run():
        if not cfg.bitcoin_address:
            if cfg.bitcoin_addresses:
                return Result(status=Status.WARN, detail="no primary bitcoin_address; using failover list only",
                              fix="set bitcoin_address to the address you want paid first")
            return Result(status=Status.FAIL, detail="bitcoin_address is not set",
                          fix="pass --bitcoin-address or set OTEDAMA_BITCOIN_ADDRESS")
        err = C.validate_bitcoin_address(cfg.bitcoin_address)
        if err:
            return Result(status=Status.FAIL, detail=err, fix="re-copy the address from your wallet")
        from otedama_amd.btccrypto import classify_address

        return Result(detail=f"{cfg.bitcoin_address[:6]}…{cfg.bitcoin_address[-4:]} "
                             f"({classify_address(cfg.bitcoin_address)}) checksum OK")
    return Check("Bitcoin address", run)


def check_failover_addresses(cfg: C.Config) -> Check:
    def run():
        if not cfg.bitcoin_addresses:
            return Result(status=Status.SKIP, detail="no failover payout addresses configured")
        bad = [a for a in cfg.bitcoin_addresses if C.validate_bitcoin_address(a)]
        if bad:
            return Result(status=Status.FAIL, detail=f"{len(bad)} invalid failover address(es)",
                          fix="fix or remove the invalid entries under bitcoin_addresses")
        dup = len(cfg.bitcoin_addresses) != len(set(cfg.bitcoin_addresses))
        if dup or cfg.bitcoin_address in cfg.bitcoin_addresses:
            return Result(status=Status.WARN, detail="failover list repeats an address",
                          fix="list each payout address once")
        return Result(detail=f"{len(cfg.bitcoin_addresses)} failover address(es) valid")
    return Check("Failover payout addresses", run)


def check_data_dir(cfg: C.Config) -> Check:
    def run():
        d = cfg.data_dir
        if not d:
            return Result(status=Status.WARN, detail="data directory could not be determined",
                          fix="pass --data-dir or set OTEDAMA_DATA_DIR")
        if not os.path.exists(d):
            parent = os.path.dirname(os.path.abspath(d).rstrip("/")) or "/"
            while not os.path.exists(parent) and parent != "/":
                parent = os.path.dirname(parent)
            if os.access(parent, os.W_OK):
                return Result(detail=f"{d} does not exist yet; it will be created (parent writable)")
            return Result(status=Status.FAIL, detail=f"{d} does not exist and {parent} is not writable",
                          fix=f"create {d} or choose a writable --data-dir")
        if not os.path.isdir(d):
            return Result(status=Status.FAIL, detail=f"{d} is not a directory", fix="point --data-dir at a directory")
        if not os.access(d, os.W_OK):
            return Result(status=Status.FAIL, detail=f"{d} is not writable", fix=f"chmod u+w {d}")
        mode = os.stat(d).st_mode & 0o777
        if mode & 0o077:
            return Result(status=Status.WARN, detail=f"{d} is accessible by other users (mode {mode:o})",
                          fix=f"chmod 700 {d} (the wallet lives here)")
        return Result(detail=f"{d} writable (mode {mode:o})")
    return Check("Data directory", run)


def check_wallet(cfg: C.Config) -> Check:
    def run():
        path = os.path.join(cfg.data_dir or "", "wallet.dat")
        if not cfg.data_dir or not os.path.exists(path):
            return Result(status=Status.SKIP, detail="no wallet.dat (created on first run with --wallet-passphrase)")
        mode = os.stat(path).st_mode & 0o777
        try:
            from otedama_amd.lightning.seedstore import unmarshal

            with open(path, "rb") as f:
                unmarshal(f.read())
        except Exception as exc:  # noqa: BLE001
            return Result(status=Status.FAIL, detail=f"wallet.dat unreadable: {exc}",
                          fix="restore wallet.dat from backup or recreate it from your recovery phrase")
        if mode & 0o077:
            return Result(status=Status.WARN, detail=f"wallet.dat mode {mode:o} is too permissive",
                          fix=f"chmod 600 {path}")
        return Result(detail=f"wallet.dat present, format OK (mode {mode:o})")
    return Check("Lightning wallet", run)


def _pool_targets(cfg: C.Config) -> list[tuple[str, str, int]]:
    urls = [p.url for p in cfg.pools] or [C.DEFAULT_POOL_URL]
    out = []
    for u in urls:
        try:
            rest = strip_scheme(u)
        except Exception:  # noqa: BLE001
            continue
        proto = from_url(u)
        host, port = split_host_port(rest, 3336 if proto.value.startswith("stratum-v2") else 3333)
        out.append((u, host, port))
    return out


def check_pool_reachability(cfg: C.Config) -> Check:
    def run():
        ok, bad = [], []
        for u, host, port in _pool_targets(cfg):
            try:
                pool_dial(host, port, dial_timeout)
                ok.append(u)
            except OSError as exc:
                bad.append(f"{u} ({exc})")
        if not bad:
            return Result(detail=f"{len(ok)} pool(s) reachable")
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
            return Result(status=Status.WARN, detail=detail + f", {drm} render node(s) but no HIP device",
                          fix="install the ROCm runtime / amdgpu driver so the gfx950 kernels can run")
        return Result(detail=detail + ", no GPU detected (CPU SHA-NI miner only)")
    return Check("Hardware", run)


def check_network() -> Check:
    def run():
        try:
            pool_dial(network_check_endpoint[0], network_check_endpoint[1], dial_timeout)
        except OSError as exc:
            return Result(status=Status.WARN, detail=f"cannot reach {network_check_endpoint[0]}:"
                                                     f"{network_check_endpoint[1]}: {exc}",
                          fix="check internet connectivity (pools and price sources need it)")
        return Result(detail="internet reachable")
    return Check("Network", run)


def check_clock() -> Check:
    def run():
        try:
            req = urllib.request.Request(clock_skew_probe_url, method="HEAD")
            with urllib.request.urlopen(req, timeout=dial_timeout) as resp:  # noqa: S310
                date = resp.headers.get("Date")
        except Exception as exc:  # noqa: BLE001
            return Result(status=Status.SKIP, detail=f"clock probe unavailable: {exc}")
        if not date:
            return Result(status=Status.SKIP, detail="probe returned no Date header")
        try:
            skew = abs(time.time() - email.utils.parsedate_to_datetime(date).timestamp())
        except (TypeError, ValueError):
            return Result(status=Status.SKIP, detail=f"probe returned an unparseable Date header {date[:40]!r}")
        if skew > 120:
            return Result(status=Status.WARN, detail=f"local clock is {skew:.0f}s off server time",
                          fix="enable NTP (timedatectl set-ntp true); share nTime and TLS depend on it")
        return Result(detail=f"clock within {skew:.1f}s of server time")
    return Check("System clock accuracy", run)


def check_native() -> Check:
    def run():
        from otedama_amd.ops.native import load

        n = load(build_if_missing=False)
        if n is None:
            return Result(status=Status.FAIL, detail="otedama_amd._native not built",
                          fix="python -m otedama_amd._build (needs ROCm hipcc for gfx950)")
        return Result(detail=f"native extension loaded (SHA-NI={'yes' if n.cpu_has_sha_ni() else 'no'})")
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
    def run():
        try:
            import torch.distributed as dist
        except Exception as exc:  # noqa: BLE001
            return Result(status=Status.WARN, detail=f"torch.distributed unavailable: {exc}",
                          fix="multi-GPU mining needs PyTorch with RCCL")
        nccl = dist.is_nccl_available()
        if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "") != "0" and nccl:
            return Result(status=Status.WARN, detail="RCCL available but HSA_ENABLE_IPC_MODE_LEGACY is not 0",
                          fix="export HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC) for multi-process RCCL")
        return Result(detail=f"torch.distributed backends: nccl(RCCL)={'yes' if nccl else 'no'}, "
                             f"gloo={'yes' if dist.is_gloo_available() else 'no'}")
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
