"""Per-connection variable difficulty. [NO REFERENCE CODE]

The only related reference code is the share-interval relation ``interval = D * 2^32 / H``
(internal/engine/stats.go:502-513, publishDifficulty); vardiff inverts it: the difficulty that gives the target share
interval is ``D* = H * T / diff1_hashes``.

Estimator (the round-5 windowed z-test left a 24% error in place for tens of seconds):
the maximum-likelihood rate of a Poisson process whose difficulty changed along the way. Shares arrive at
H / (diff1_hashes * D(t)), so over a window the worker's rate is ``shares / integral(dt / D(t))`` (shares per unit
of "exposure"), whatever difficulties were in force: the window is NOT reset on a retarget, every share since the
worker connected (up to ``max_window_shares`` and ``max_window_factor`` retarget periods back) keeps sharpening one
estimate, and its relative error falls as 1/sqrt(n). (A stretch at a far too high difficulty, with one late share,
adds almost no exposure, so it cannot bias the estimate as a sum of credited work over time would.)

Decisions, once per retarget period (and early for a worker far too fast):
  * significant: |ln(D*/D)| > z / sqrt(n). ``z`` is ``noise_z`` scaled down when a period holds few shares (at the
    default 10 s target / 30 s period a 2x mismatch is corrected at the first look and a 3x one by the second,
    ADVICE r5), full strength at high share rates (a worker on target is left alone);
  * refinement: the estimate now rests on >= 4x the shares it had when D was last set (or on ~a full window), and D
    is off by more than the dead band. Each refinement needs 4x the data of the one before, so there are a few
    (16 -> 64 -> 256 -> ~1000 shares) and then none: D ends within ~1/sqrt(max_window_shares) of D*, not within the
    noise of the first look. A look that finds D within the dead band on that much data confirms it instead.
``settled()`` says when neither rule can fire any more (the pool probe opens its measurement window on it). A step is
bounded (x4 / /4) and clamped (min / max), and moves below the dead band are not sent.
"""
from __future__ import annotations

import math
import time
from collections import deque
from dataclasses import dataclass, field


@dataclass
class VardiffConfig:
    target_share_seconds: float = 10.0
    retarget_seconds: float = 30.0
    min_difficulty: float = 1e-6
    max_difficulty: float = 1e15
    max_step: float = 4.0
    dead_band: float = 0.02
    min_shares: int = 16            # retarget early once this many shares arrived early_factor x faster than target
    # A burst of shares at the right rate is common (Poisson), so an early retarget needs strong evidence: at 4x after
    # 16 shares a worker on target never fires early; a new worker at 1000x its difficulty still reaches its level in
    # a few dozen shares.
    early_factor: float = 4.0
    noise_z: float = 3.0            # significance of a deviation, in standard errors of the estimate
    steady_z: float = 5.0           # ... once the difficulty rests on most of a full window (settled)
    initial_z: float = 1.0          # ... while the difficulty in force rests on no shares at all (initial / nominal)
    z_full_at: float = 16.0         # expected shares per period at which noise_z applies in full (fewer: scaled down)
    max_window_shares: int = 1024   # the estimator keeps at most this many shares ...
    max_window_factor: float = 16.0  # ... and none older than this many retarget periods
    refine_factor: float = 4.0      # a refinement needs this many times the shares D was last set from


@dataclass
class VardiffState:
    difficulty: float
    window_start: float = field(default_factory=time.monotonic)  # last retarget (or open): the early path's window
    shares: float = 0.0             # credited shares since window_start (a grace share counts its fraction)
    accepted_work: float = 0.0      # sum of credited share difficulties since window_start
    total_shares: int = 0
    looks: int = 0                  # periodic looks since window_start
    # the rate estimator, kept across retargets: exposure = integral of dt / D(t) up to exp_t, and the recent shares as
    # (exposure at the share, credited share)
    exp: float = 0.0
    exp_t: float | None = None
    hist: deque = field(default_factory=deque)
    hist_start_exp: float = 0.0     # exposure where the estimator's window opens
    hist_shares: float = 0.0
    ws_exp: float = 0.0             # exposure at window_start (the segment since the last retarget)
    n_at_set: float = 0.0           # estimator shares behind the difficulty in force (0: initial / nominal)
    retargets: int = 0


CHANGE_P = 1e-4  # significance of the rate-change test (run at every look: false alarms must be rare)


def _binom_two_sided(k: int, m: int, p: float) -> float:
    """P(K <= k) or P(K >= k) for K ~ Binomial(m, p), whichever tail k is in, doubled (capped at 1). Exact for
    m <= 200; above that the normal approximation with continuity correction (a look per worker per period must
    stay cheap on a pool with many workers: the exact tail is up to m lgamma terms)."""
    if m <= 0 or not 0.0 < p < 1.0:
        return 1.0
    if m > 200:
        mu, sd = m * p, math.sqrt(m * p * (1.0 - p))
        z = max(0.0, abs(k - mu) - 0.5) / max(sd, 1e-12)
        return min(1.0, math.erfc(z / math.sqrt(2.0)))
    lp, lq = math.log(p), math.log1p(-p)

    def pmf(i: int) -> float:
        return math.exp(math.lgamma(m + 1) - math.lgamma(i + 1) - math.lgamma(m - i + 1) + i * lp + (m - i) * lq)

    tail = sum(pmf(i) for i in range(0, k + 1)) if k <= m * p else sum(pmf(i) for i in range(k, m + 1))
    return min(1.0, 2.0 * tail)


class Vardiff:
    def __init__(self, cfg: VardiffConfig | None = None, diff1_hashes: float = 2.0 ** 32, clock=time.monotonic):
        self.cfg = cfg or VardiffConfig()
        self.diff1_hashes = diff1_hashes  # expected hashes per difficulty-1 share
        self.clock = clock

    def new_state(self, difficulty: float) -> VardiffState:
        now = self.clock()
        return VardiffState(self.clamp(difficulty), now, exp_t=now)

    def clamp(self, d: float) -> float:
        return min(max(d, self.cfg.min_difficulty), self.cfg.max_difficulty)

    # ------------------------------------------------------------------ estimator
    def _advance(self, st: VardiffState, now: float) -> None:
        """Accumulate exposure up to ``now`` at the difficulty in force (call before the difficulty changes)."""
        if st.exp_t is None:
            st.exp_t = st.window_start
        if now > st.exp_t:
            st.exp += (now - st.exp_t) / st.difficulty
            st.exp_t = now

    def _trim(self, st: VardiffState, now: float) -> None:
        c = self.cfg
        # exposure is kept per share, so the time cap is applied through the share times recorded beside it
        oldest = now - self._window_s()
        while st.hist and (len(st.hist) > c.max_window_shares or st.hist[0][0] < oldest):
            _t, e, w = st.hist.popleft()
            st.hist_shares -= w
            st.hist_start_exp = e  # the window now opens at the last dropped arrival
        if not st.hist:
            st.hist_shares = 0.0

    def estimate(self, st: VardiffState, mutate: bool = True) -> tuple[float | None, float]:
        """(D*, n): the difficulty the estimator points to and the shares it rests on (None without shares).
        ``mutate=False`` reads without touching the state (another thread: the pool's HTTP API)."""
        now = self.clock()
        if mutate:
            self._advance(st, now)
            self._trim(st, now)
            exposure, n = st.exp - st.hist_start_exp, st.hist_shares
        else:
            c = self.cfg
            hist, t_exp, exp, d, start = list(st.hist), st.exp_t, st.exp, st.difficulty, st.hist_start_exp
            exp += max(0.0, now - (t_exp if t_exp is not None else st.window_start)) / d
            oldest = now - self._window_s()
            drop = 0
            while drop < len(hist) and (len(hist) - drop > c.max_window_shares or hist[drop][0] < oldest):
                start = hist[drop][1]
                drop += 1
            exposure, n = exp - start, sum(w for _t, _e, w in hist[drop:])
        if n <= 0 or exposure <= 0:
            return None, 0.0
        return self.clamp(n / exposure * self.cfg.target_share_seconds), n

    def _z(self, st: VardiffState) -> float:
        c = self.cfg
        per_period = c.retarget_seconds / max(c.target_share_seconds, 1e-12)
        # once D rests on most of a full window the test only watches for a real change of the worker's rate, over
        # many overlapping looks: a stricter z keeps its false alarms rare
        if st.n_at_set <= 0:
            # the difficulty in force came from no data (the initial or nominal one): any clear deviation moves it
            return c.initial_z
        z = c.steady_z if st.n_at_set >= 0.75 * self._full() else c.noise_z
        return z * min(1.0, math.sqrt(per_period / c.z_full_at))

    def _window_s(self) -> float:
        """The estimator's time cap: max_window_factor retarget periods, at least 64 target intervals."""
        c = self.cfg
        return max(c.max_window_factor * c.retarget_seconds, 64.0 * c.target_share_seconds)

    def _full(self) -> float:
        """Shares the estimator's window holds at the target rate."""
        c = self.cfg
        return min(c.max_window_shares, self._window_s() / max(c.target_share_seconds, 1e-12))

    def _refine_at(self, st: VardiffState) -> float:
        """Estimator shares at which the difficulty in force is next refined (or confirmed): refine_factor x the
        shares it was set on, at most a full window, and never again once it rests on most of one."""
        full = self._full()
        if st.n_at_set >= 0.75 * full:
            return math.inf
        return min(self.cfg.refine_factor * max(st.n_at_set, 4.0), 0.9 * full)

    def _verdict(self, st: VardiffState, dstar: float, n: float) -> str | None:
        """'significant', 'refine' or None for the estimate (dstar, n) against the difficulty in force."""
        c = self.cfg
        dev = abs(math.log(dstar / st.difficulty))
        if dev > self._z(st) / math.sqrt(max(n, 1e-9)):
            return "significant"
        if dev > math.log1p(c.dead_band) and n >= self._refine_at(st):
            return "refine"
        return None

    def settled(self, st: VardiffState, mutate: bool = True) -> bool:
        """Neither rule can move the difficulty any more at the worker's present rate: the difficulty in force was
        set (or confirmed) on most of a full window, so no refinement is left, and no retarget is pending."""
        dstar, n = self.estimate(st, mutate)
        if dstar is None or self._refine_at(st) != math.inf:
            return False
        return self._verdict(st, dstar, n) is None

    # ------------------------------------------------------------------ shares and retargets
    def on_share(self, st: VardiffState, weight: float = 1.0) -> float | None:
        """Record an accepted share; returns a new difficulty when a retarget fires. ``weight``: the share's credited
        difficulty over the one in force. A share the pool took at the previous, lower difficulty in the grace after
        a raise is worth that fraction of a share (and its credited work is what the estimator adds)."""
        w = min(max(weight, 0.0), 1.0)
        now = self.clock()
        self._advance(st, now)
        st.shares += w
        st.total_shares += 1
        st.accepted_work += st.difficulty * w
        st.hist.append((now, st.exp, w))
        st.hist_shares += w
        return self.maybe_retarget(st)

    def maybe_retarget(self, st: VardiffState) -> float | None:
        now = self.clock()
        elapsed = now - st.window_start
        c = self.cfg
        early = st.shares >= c.min_shares and elapsed < c.target_share_seconds * st.shares / c.early_factor
        # looked at once per retarget period (a test at every share would find a noise excursion sooner or later)
        due = elapsed >= c.retarget_seconds * (st.looks + 1)
        if not due and not early:
            return None
        if due:
            self._detect_change(st, now)
        dstar, n = self.estimate(st)
        if dstar is None:
            if elapsed < c.retarget_seconds:
                return None
            # no share for a whole period: too hard (one step down, a bigger one after two periods)
            ratio = 1.0 / c.max_step if elapsed >= 2 * c.retarget_seconds else 0.5
            return self._set(st, st.difficulty * ratio, now, 0.0)
        if early:
            return self._set(st, dstar, now, n)
        st.looks = int(elapsed // max(c.retarget_seconds, 1e-9)) if c.retarget_seconds > 0 else 0
        if self._verdict(st, dstar, n) is None:
            if n >= self._refine_at(st):
                st.n_at_set = n  # confirmed within the dead band by 4x the data: the next refinement needs 4x more
            return None
        return self._set(st, dstar, now, n)

    def _detect_change(self, st: VardiffState, now: float) -> None:
        """The worker's rate itself changed (a miner stopped, or a second miner took half the GPU): the segment since
        the last retarget disagrees with the older history by more than 20% and at CHANGE_P (the test runs at every
        look, so its false alarms must be rare), so the history is dropped and the estimate restarts from the second
        half of that stretch."""
        self._advance(st, now)
        self._trim(st, now)
        k = st.shares
        e_recent = st.exp - max(st.ws_exp, st.hist_start_exp)
        old_n, old_e = st.hist_shares - k, max(st.ws_exp, st.hist_start_exp) - st.hist_start_exp
        if old_n < 8 or old_e <= 0 or e_recent <= 0:
            return
        expect = old_n / old_e * e_recent
        # Given the m shares of both stretches, under "same rate" the recent stretch's count is Binomial(m, p) with p
        # its share of the exposure: an exact test that carries both stretches' noise (and is right for k = 0)
        m, p = int(round(old_n + k)), e_recent / (e_recent + old_e)
        if abs(k - expect) > 0.2 * expect and _binom_two_sided(int(round(k)), m, p) < CHANGE_P:
            # the change happened somewhere in the recent stretch: keep its second half only (the first may still
            # carry the old rate: a second miner joining the GPU a second or two after this worker's last retarget)
            cut = max(st.ws_exp, st.hist_start_exp) + 0.5 * e_recent
            while st.hist and st.hist[0][1] <= cut:
                _t, _e, w = st.hist.popleft()
                st.hist_shares -= w
            st.hist_start_exp = cut
            st.n_at_set = 0.0

    def _set(self, st: VardiffState, target: float, now: float, n: float) -> float | None:
        c = self.cfg
        raw = target / st.difficulty
        ratio = min(max(raw, 1.0 / c.max_step), c.max_step)
        new = self.clamp(st.difficulty * ratio)
        self._advance(st, now)
        st.window_start, st.shares, st.accepted_work, st.looks, st.ws_exp = now, 0.0, 0.0, 0, st.exp
        if abs(new - st.difficulty) <= c.dead_band * st.difficulty:
            return None
        st.difficulty = new
        # a bounded step did not reach the estimate: D does not rest on the estimator's n shares yet
        st.n_at_set = n if ratio == raw else 0.0
        st.retargets += 1
        return new

    def estimated_hashrate(self, st: VardiffState) -> float:
        """H/s implied by the estimator (D* * diff1_hashes / target interval)."""
        dstar, _ = self.estimate(st)
        return 0.0 if dstar is None else dstar * self.diff1_hashes / self.cfg.target_share_seconds

    def difficulty_for_hashrate(self, hashrate: float) -> float:
        """Inverse of interval = D * diff1_hashes / H for the target interval."""
        if hashrate <= 0:
            return self.clamp(1.0)
        return self.clamp(hashrate * self.cfg.target_share_seconds / self.diff1_hashes)
