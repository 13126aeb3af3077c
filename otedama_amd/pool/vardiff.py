"""Per-connection variable difficulty. [NO REFERENCE CODE]

The only related reference code is the share-interval estimate
``interval = D * 2^32 / H`` (internal/engine/stats.go:502-513, publishDifficulty);
vardiff inverts it: every retarget window the observed share interval moves the
difficulty toward ``target_share_seconds``, bounded per step (x4 / /4) and
globally (min/max), with a 10% dead band so it does not flap.

A window's interval estimate from n shares is itself noisy (Poisson: relative spread ~1/sqrt(n)), so a retarget also
needs the deviation to be significant, |ln ratio| >= noise_z / sqrt(n), judged once per retarget period (a test at
every share finds a noise excursion sooner or later). A window that is not significant keeps accumulating shares, up
to max_window_factor retarget periods, instead of being thrown away: a miner on target is left alone, and a real 2x
mismatch is corrected at the first look. At a 0.1 s share target the pool bench saw >25% retargets on noise alone
after vardiff had settled (profiles/r5/g_bench), and the window must open on steady workers only.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field


@dataclass
class VardiffConfig:
    target_share_seconds: float = 10.0
    retarget_seconds: float = 30.0
    min_difficulty: float = 1e-6
    max_difficulty: float = 1e15
    max_step: float = 4.0
    dead_band: float = 0.10
    min_shares: int = 16            # retarget early once this many shares arrived early_factor x faster than target
    # A burst of shares at the right rate is common (Poisson), so an early retarget needs strong evidence: at 2x, a
    # worker already at its target retargeted on noise several times a minute at a 0.1 s share interval (each a
    # difficulty doubling and a correction back). At 4x after 16 shares a worker on target never fires early, one at
    # 2x in ~1-2% of windows; a new worker at 1000x its difficulty still reaches its level in a few dozen shares.
    early_factor: float = 4.0
    noise_z: float = 3.0            # significance of a window's deviation, in standard errors of its estimate
    max_window_factor: float = 8.0  # an insignificant window accumulates up to this many retarget periods


@dataclass
class VardiffState:
    difficulty: float
    window_start: float = field(default_factory=time.monotonic)
    shares: float = 0.0         # shares in the window, a grace share counting its credited fraction
    accepted_work: float = 0.0      # sum of share difficulties in the window
    total_shares: int = 0
    looks: int = 0                  # retarget periods of this window already judged insignificant


class Vardiff:
    def __init__(self, cfg: VardiffConfig | None = None, diff1_hashes: float = 2.0 ** 32, clock=time.monotonic):
        self.cfg = cfg or VardiffConfig()
        self.diff1_hashes = diff1_hashes  # expected hashes per difficulty-1 share
        self.clock = clock

    def new_state(self, difficulty: float) -> VardiffState:
        return VardiffState(self.clamp(difficulty), self.clock())

    def clamp(self, d: float) -> float:
        return min(max(d, self.cfg.min_difficulty), self.cfg.max_difficulty)

    def on_share(self, st: VardiffState, weight: float = 1.0) -> float | None:
        """Record an accepted share; returns a new difficulty when a retarget fires. ``weight``: the share's credited
        difficulty over the one in force. A share the pool took at the previous, lower difficulty in the grace after
        a raise is worth that fraction of a share. Counted whole, the old-rate shares of the grace read as a miner
        still too fast, and vardiff raised again and then walked back (late >25% retargets in the pool probe)."""
        w = min(max(weight, 0.0), 1.0)
        st.shares += w
        st.total_shares += 1
        st.accepted_work += st.difficulty * w
        return self.maybe_retarget(st)

    def maybe_retarget(self, st: VardiffState) -> float | None:
        now = self.clock()
        elapsed = now - st.window_start
        c = self.cfg
        early = st.shares >= c.min_shares and elapsed < c.target_share_seconds * st.shares / c.early_factor
        # the window is looked at once per retarget period (a test at every share would find a noise excursion)
        due = elapsed >= c.retarget_seconds * (st.looks + 1)
        if not due and not early:
            return None
        if st.shares == 0:
            ratio = 1.0 / c.max_step if elapsed >= 2 * c.retarget_seconds else 0.5
        else:
            observed = elapsed / st.shares
            ratio = c.target_share_seconds / max(observed, 1e-9)
            young = elapsed < c.max_window_factor * c.retarget_seconds
            if not early and young and abs(math.log(max(ratio, 1e-300))) < c.noise_z / math.sqrt(st.shares):
                st.looks = int(elapsed // c.retarget_seconds)  # within the estimate's own noise: let it sharpen
                return None
        ratio = min(max(ratio, 1.0 / c.max_step), c.max_step)
        st.window_start, st.shares, st.accepted_work, st.looks = now, 0, 0.0, 0
        new = self.clamp(st.difficulty * ratio)
        if abs(new - st.difficulty) <= c.dead_band * st.difficulty:
            return None
        st.difficulty = new
        return new

    def estimated_hashrate(self, st: VardiffState) -> float:
        """H/s implied by the window's accepted work (D * diff1_hashes / interval)."""
        elapsed = max(self.clock() - st.window_start, 1e-9)
        return st.accepted_work * self.diff1_hashes / elapsed

    def difficulty_for_hashrate(self, hashrate: float) -> float:
        """Inverse of interval = D * diff1_hashes / H for the target interval."""
        if hashrate <= 0:
            return self.clamp(1.0)
        return self.clamp(hashrate * self.cfg.target_share_seconds / self.diff1_hashes)
