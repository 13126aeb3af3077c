"""Pure, deterministic device -> revenue-stream allocation.

Parity: internal/arbitration/engine.go
  * Yield.Effective (sats/s x confidence, 0 when either <= 0) ...... :92-97
  * Stream (families, per-device yields, ratings, IsBitcoinMining) . :105-128
  * Policy x4 (maximize_earnings, stack_btc, maximize_privacy,
    environment_friendly) ........................................ :132-179
  * Assignment (Held, ForegoneSatsPerSec) / Allocation / Input ..... :185-267
  * Decide: devices sorted by ID, duplicate-ID and parameter guards  :291-342
  * chooseForDevice: min-yield floor, policy-score ordering with ID
    tie-break, hysteresis in policy-score space, held/foregone ..... :346-465
  * policyScore bonuses (BTC stack x1.05, +1%/rating point) ........ :470-503
Invariants (engine.go:30-50, tested as properties in tests/test_arbitration.py):
never assigns an incompatible family; non-idle assignments clear the floor;
foregone >= 0; output independent of input order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import IntEnum

from otedama_amd.hal import Capabilities, Family, Identity


class ArbitrationError(ValueError):
    pass


@dataclass(frozen=True)
class Yield:
    sats_per_second: float = 0.0
    confidence: float = 0.0

    def effective(self) -> float:
        if self.sats_per_second <= 0 or self.confidence <= 0:
            return 0.0
        return self.sats_per_second * self.confidence


@dataclass
class Stream:
    id: str
    accepts_families: list[Family] = field(default_factory=list)
    yield_per_device: dict[str, Yield] = field(default_factory=dict)
    default_yield: Yield = field(default_factory=Yield)
    privacy_rating: int = 0
    environmental_rating: int = 0
    is_bitcoin_mining: bool = False

    def accepts(self, f: Family) -> bool:
        return f in self.accepts_families

    def yield_for(self, device_id: str) -> Yield:
        return self.yield_per_device.get(device_id, self.default_yield)


class Policy(IntEnum):
    MAXIMIZE_EARNINGS = 0
    STACK_BTC = 1
    MAXIMIZE_PRIVACY = 2
    ENVIRONMENT_FRIENDLY = 3

    def __str__(self) -> str:
        return self.name.lower()

    @classmethod
    def parse(cls, s: str) -> "Policy":
        try:
            return cls[s.upper()]
        except KeyError:
            raise ArbitrationError(f"arbitration: unknown policy {s!r}") from None


@dataclass
class Assignment:
    device_id: str
    stream: str = ""
    expected_yield: float = 0.0
    switched_from_id: str = ""
    reason: str = ""
    held: bool = False
    foregone_sats_per_sec: float = 0.0

    def idle(self) -> bool:
        return self.stream == ""


@dataclass
class Allocation:
    assignments: list[Assignment] = field(default_factory=list)
    total_yield: float = 0.0
    policy: Policy = Policy.MAXIMIZE_EARNINGS
    skipped_device: int = 0


@dataclass(frozen=True)
class DeviceRef:
    identity: Identity
    capabilities: Capabilities = field(default_factory=Capabilities)


@dataclass
class Input:
    devices: list[DeviceRef]
    streams: list[Stream]
    previous: Allocation | None = None
    policy: Policy = Policy.MAXIMIZE_EARNINGS
    hysteresis_margin: float = 0.0
    min_yield_sats_per_sec: float = 0.0


BTC_STACK_BONUS = 1.05
RATING_BONUS_PER_POINT = 0.01


def policy_score(s: Stream, y: float, p: Policy) -> float:
    if p is Policy.STACK_BTC:
        return y * BTC_STACK_BONUS if s.is_bitcoin_mining else y
    if p is Policy.MAXIMIZE_PRIVACY:
        return y * (1.0 + s.privacy_rating * RATING_BONUS_PER_POINT)
    if p is Policy.ENVIRONMENT_FRIENDLY:
        return y * (1.0 + s.environmental_rating * RATING_BONUS_PER_POINT)
    return y


def decide(inp: Input) -> Allocation:
    if not isinstance(inp.policy, Policy):
        raise ArbitrationError(f"arbitration: invalid Policy {inp.policy!r}")
    if inp.hysteresis_margin < 0:
        raise ArbitrationError("arbitration: HysteresisMargin must be non-negative")
    if inp.min_yield_sats_per_sec < 0:
        raise ArbitrationError("arbitration: MinYieldSatsPerSec must be non-negative")
    seen = set()
    for d in inp.devices:
        if d.identity.id in seen:
            raise ArbitrationError(f"arbitration: duplicate device ID {d.identity.id!r}")
        seen.add(d.identity.id)
    devices = sorted(inp.devices, key=lambda d: d.identity.id)
    prev = {a.device_id: a for a in inp.previous.assignments} if inp.previous else {}
    alloc = Allocation(policy=inp.policy)
    for dev in devices:
        a = _choose(dev, inp.streams, prev.get(dev.identity.id, Assignment(dev.identity.id)), inp.policy,
                    inp.hysteresis_margin, inp.min_yield_sats_per_sec)
        if a.idle():
            alloc.skipped_device += 1
        alloc.total_yield += a.expected_yield
        alloc.assignments.append(a)
    return alloc


def _fmt_g(v: float) -> str:
    return f"{v:.4g}"


def _choose(dev: DeviceRef, streams: list[Stream], previous: Assignment, policy: Policy, hysteresis: float,
            min_yield: float) -> Assignment:
    cands: list[tuple[Stream, float]] = []
    below = False
    for s in streams:
        if not s.accepts(dev.identity.family):
            continue
        y = s.yield_for(dev.identity.id).effective()
        if y <= 0:
            continue
        if y < min_yield:
            below = True
            continue
        cands.append((s, y))
    if not cands:
        reason = "no compatible stream accepting non-zero work"
        if below:
            reason = f"all compatible streams below minimum yield floor {_fmt_g(min_yield)} sats/s"
        return Assignment(dev.identity.id, reason=reason)
    max_raw = max(y for _, y in cands)
    cands.sort(key=lambda c: c[0].id)                     # tie-break by stream id (stable)
    cands.sort(key=lambda c: -policy_score(c[0], c[1], policy))
    best, best_y = cands[0]
    best_score = policy_score(best, best_y, policy)
    if previous.stream:
        for s, y in cands:
            if s.id == previous.stream:
                inc = policy_score(s, y, policy)
                if best_score <= inc * (1.0 + hysteresis):
                    held = best.id != s.id
                    if held:
                        reason = (f"held (best gain {(best_score - inc) / max(inc, 1e-9) * 100:.2f}% below "
                                  f"hysteresis {hysteresis * 100:.2f}%)")
                    else:
                        reason = "incumbent is best; stayed"
                    return Assignment(dev.identity.id, s.id, y, reason=reason, held=held,
                                      foregone_sats_per_sec=max_raw - y)
                break
    a = Assignment(dev.identity.id, best.id, best_y, reason=f"best yield under policy {policy}",
                   foregone_sats_per_sec=max_raw - best_y)
    if previous.stream and previous.stream != best.id:
        a.switched_from_id = previous.stream
    return a


__all__ = ["Allocation", "ArbitrationError", "Assignment", "DeviceRef", "Input", "Policy", "Stream", "Yield",
           "decide", "policy_score", "math"]
