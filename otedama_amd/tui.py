"""Live terminal dashboard: cursor-home repaint once a second, fixed column budget.

Parity: internal/tui/dashboard.go
  * Stats / ProviderStats snapshot ............................ dashboard.go:47-103
  * start / stop (hide/show cursor, loop joined before Stop writes) .. :132-160
  * update (latest snapshot wins; rendered on the 1 s tick) ........ :163-220
  * sections MINING / EARNINGS / ARBITRATION / WALLET + footer ..... :222-257
  * mining line: normal, ⚠ stalled, ⏸ paused (curtailed), idle count :269-298
  * pool line keeps the connection status visible on narrow widths . :300-327
  * ANSI-aware visible_len / truncate_visible / pad_right ........... :460-528
  * format_hash_rate / format_duration / sats_to_display / set_width  :420-566
Each line is cleared, truncated to the width and padded so a frame always
overwrites the previous one in place (no wrap, no scroll).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import TextIO

RESET, BOLD, DIM = "\x1b[0m", "\x1b[1m", "\x1b[2m"
CYAN, GREEN, YELLOW, RED, WHITE = "\x1b[36m", "\x1b[32m", "\x1b[33m", "\x1b[31m", "\x1b[37m"
HOME, CLEAR_LINE = "\x1b[H", "\x1b[2K"


@dataclass
class ProviderStats:
    name: str = ""
    sats_per_second: float = 0.0
    active: bool = False


@dataclass
class Stats:
    hash_rate: float = 0.0
    shares_found: int = 0
    shares_sent: int = 0
    pool_url: str = ""
    pool_latency_ms: float = 0.0
    connected: bool = False
    providers: list[ProviderStats] = field(default_factory=list)
    wallet_fingerprint: str = ""
    est_sats_earned: int = 0
    uptime: float = 0.0
    devices: int = 0
    language: str = ""
    stalled: bool = False
    curtailed: bool = False
    devices_idle: int = 0
    algorithm: str = "sha256d"

    @classmethod
    def from_engine(cls, d: dict) -> "Stats":
        """Adapter from Engine.stats()."""
        return cls(hash_rate=float(d.get("hashrate", 0.0)), shares_found=int(d.get("shares_found", 0)),
                   shares_sent=int(d.get("shares_submitted", 0)), pool_url=d.get("pool", ""),
                   pool_latency_ms=float(d.get("latency_p50_ms", 0.0) or 0.0), connected=bool(d.get("connected")),
                   providers=[ProviderStats(**p) for p in d.get("providers", [])],
                   wallet_fingerprint=d.get("wallet", ""), est_sats_earned=int(d.get("est_sats", 0)),
                   uptime=float(d.get("uptime", 0.0)), devices=len(d.get("devices", {})),
                   stalled=bool(d.get("stalled")), curtailed=bool(d.get("curtailed")),
                   devices_idle=int(d.get("devices_idle", 0)), algorithm=d.get("algorithm", "sha256d"))


# ------------------------------------------------------------------ formatting
def format_hash_rate(hps: float) -> str:
    for scale, unit in ((1e15, "PH/s"), (1e12, "TH/s"), (1e9, "GH/s"), (1e6, "MH/s"), (1e3, "kH/s")):
        if hps >= scale:
            return f"{hps / scale:.2f} {unit}"
    return f"{hps:.0f} H/s"


def format_duration(seconds: float) -> str:
    s = int(seconds)
    h, m, sec = s // 3600, (s // 60) % 60, s % 60
    if h:
        return f"{h}h {m}m {sec}s"
    if m:
        return f"{m}m {sec}s"
    return f"{sec}s"


def sats_to_display(sats: int) -> str:
    if sats >= 100_000_000:
        return f"{sats / 1e8:.4f} BTC"
    if sats >= 1000:
        return f"{sats} sats ({sats / 1e8:.5f} BTC)"
    return f"{sats} sats"


def default_sats_per_hash() -> float:
    """Display-only estimate (network 1e21 H/s, 3.125 BTC reward, 600 s blocks)."""
    return 3.125e8 / (1e21 * 600.0)


def _csi_end(ch: str) -> bool:
    return "@" <= ch <= "~" and ch != "["


def visible_len(s: str) -> int:
    n, in_esc = 0, False
    for ch in s:
        if in_esc:
            in_esc = not _csi_end(ch)
        elif ch == "\x1b":
            in_esc = True
        else:
            n += 1
    return n


def truncate_visible(s: str, max_visible: int) -> str:
    if max_visible <= 0:
        return ""
    out, n, in_esc = [], 0, False
    for ch in s:
        if in_esc:
            out.append(ch)
            in_esc = not _csi_end(ch)
            continue
        if ch == "\x1b":
            in_esc = True
            out.append(ch)
            continue
        if n >= max_visible:
            break
        out.append(ch)
        n += 1
    return "".join(out) + RESET


def pad_right(s: str, width: int) -> str:
    return s + " " * max(0, width - visible_len(s))


def truncate_to_budget(s: str, budget: int) -> str:
    if budget <= 0:
        return ""
    if len(s) <= budget:
        return s
    return s[:budget] if budget < 4 else s[:budget - 3] + "..."


def shorten_url(url: str, max_len: int) -> str:
    if len(url) <= max_len or max_len < 4:
        return url
    return url[:max_len - 3] + "..."


# ------------------------------------------------------------------ dashboard
class Dashboard:
    def __init__(self, w: TextIO, interval: float = 1.0):
        self.w = w
        self.interval = interval
        self.cols = 80
        self._lock = threading.Lock()
        self._last = Stats()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def set_width(self, cols: int) -> None:
        if cols >= 40:
            self.cols = cols

    def start(self) -> None:
        if self._thread is not None:
            return
        self.w.write("\x1b[?25l\x1b[2J" + HOME)
        self._thread = threading.Thread(target=self._loop, name="otedama-tui", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        if self._thread is None:
            return
        self._stop.set()
        self._thread.join()
        self._thread = None
        self.w.write("\x1b[?25h\n")
        self.w.flush()

    def update(self, s: Stats | dict) -> None:
        if isinstance(s, dict):
            s = Stats.from_engine(s)
        with self._lock:
            self._last = s

    def _loop(self) -> None:
        while not self._stop.wait(self.interval):
            with self._lock:
                s = self._last
            try:
                self.w.write(self.render(s))
                self.w.flush()
            except (OSError, ValueError):
                return

    # -------------------------------------------------------------- frame
    def render(self, s: Stats) -> str:
        cols = self.cols
        lines = [pad_right(f"{BOLD}{CYAN}  Otedama{RESET}{DIM} — MI355X mining & compute arbitration{RESET}", cols), "",
                 f"{BOLD}{WHITE}MINING{RESET}", self.mining_line(s), self.pool_line(s), "",
                 f"{BOLD}{WHITE}EARNINGS{RESET}", self.earnings_line(s)]
        if s.providers:
            lines += ["", f"{BOLD}{WHITE}ARBITRATION{RESET}"] + [self.provider_line(p) for p in s.providers]
        lines += ["", f"{BOLD}{WHITE}WALLET{RESET}", self.wallet_line(s), "", self.footer(s)]
        out = [HOME]
        for ln in lines:
            if visible_len(ln) > cols:
                ln = truncate_visible(ln, cols)
            out.append(CLEAR_LINE + ln + " " * max(0, cols - visible_len(ln)) + "\r\n")
        return "".join(out)

    def mining_line(self, s: Stats) -> str:
        rate = format_hash_rate(s.hash_rate)
        devs = f"{s.devices} device(s)" + (f", {s.devices_idle} idle" if s.devices_idle else "")
        shares = f"shares: {s.shares_sent} sent / {s.shares_found} found"
        if s.curtailed:
            prefix = f"  {CYAN}{rate:<14} ⏸ paused (price below threshold){RESET}  "
        elif s.stalled:
            prefix = f"  {YELLOW}{rate:<14} ⚠ stalled{RESET}  {DIM + devs + RESET:<20}  "
        else:
            prefix = f"  {GREEN}{rate:<14}{RESET}  {DIM + devs + RESET:<20}  "
        return prefix + DIM + truncate_to_budget(shares, self.cols - visible_len(prefix)) + RESET

    def pool_line(self, s: Stats) -> str:
        plain, status = "✗ disconnected", RED + "✗ disconnected" + RESET
        if s.connected:
            lat = f" ({s.pool_latency_ms:.0f}ms)" if s.pool_latency_ms > 0 else ""
            plain = "✓ connected" + lat
            status = GREEN + "✓ connected" + RESET + DIM + lat + RESET
        prefix = "  Pool: "
        budget = max(8, self.cols - len(prefix) - len(plain) - 2)
        url = shorten_url(s.pool_url, budget)
        return f"{prefix}{DIM}{url}{RESET}{' ' * (budget - len(url))}  {status}"

    def earnings_line(self, s: Stats) -> str:
        per_day = s.hash_rate * default_sats_per_hash() * 86400
        per_day += sum(p.sats_per_second * 86400 for p in s.providers if p.active)
        total = f"{BOLD}{YELLOW}{per_day:.0f} sats/day{RESET}"
        return f"  {total:<30}  {DIM}est. earned: ~{s.est_sats_earned} sats{RESET}"

    @staticmethod
    def provider_line(p: ProviderStats) -> str:
        active = GREEN + "● active" + RESET if p.active else DIM + "○ idle" + RESET
        return f"  {p.name:<30}  {f'{p.sats_per_second:.1f} sats/s':<12}  {active}"

    @staticmethod
    def wallet_line(s: Stats) -> str:
        return f"  Fingerprint: {CYAN}{s.wallet_fingerprint or 'not initialized'}{RESET}"

    def footer(self, s: Stats) -> str:
        left = f"  uptime: {format_duration(s.uptime)}   algo: {s.algorithm}"
        right = DIM + "Ctrl+C to exit" + RESET
        return left + " " * max(1, self.cols - visible_len(left) - visible_len(right) - 2) + right
