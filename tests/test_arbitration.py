"""Arbitration Decide: policies, hysteresis in policy-score space, held/foregone accounting, min-yield floor,
determinism, and the engine.go:30-50 invariants as hypothesis properties.

Mirrors internal/arbitration/engine_test.go (TestDecide_*, TestPolicy_*, TestYield_Effective and the
TestDecide_Property_* family).
"""
from __future__ import annotations

import random

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from otedama_amd import arbitration as A
from otedama_amd.hal import Capabilities, Family, Identity


def dev(i, fam=Family.GPU):
    return A.DeviceRef(Identity(f"{fam.value}-{i}", fam, "amd", "mi355x"), Capabilities(sha256d=True))


def stream(sid, y, conf=1.0, fams=(Family.GPU,), **kw):
    return A.Stream(sid, list(fams), default_yield=A.Yield(y, conf), **kw)


def one(inp: A.Input) -> A.Assignment:
    (a,) = A.decide(inp).assignments
    return a


# ------------------------------------------------------------------ types
@pytest.mark.parametrize("s,p", [("maximize_earnings", A.Policy.MAXIMIZE_EARNINGS), ("STACK_BTC", A.Policy.STACK_BTC),
                                 ("maximize_privacy", A.Policy.MAXIMIZE_PRIVACY),
                                 ("environment_friendly", A.Policy.ENVIRONMENT_FRIENDLY)])
def test_policy_parse_and_string_are_stable(s, p):
    assert A.Policy.parse(s) is p and str(p) == s.lower()


def test_policy_parse_unknown():
    with pytest.raises(A.ArbitrationError):
        A.Policy.parse("yolo")


@pytest.mark.parametrize("sats,conf,want", [(10, 0.5, 5.0), (10, 1, 10.0), (0, 1, 0.0), (10, 0, 0.0), (-1, 1, 0.0),
                                            (1, -1, 0.0)])
def test_yield_effective(sats, conf, want):
    assert A.Yield(sats, conf).effective() == want


# ------------------------------------------------------------------ guards
def test_rejects_invalid_policy():
    with pytest.raises(A.ArbitrationError, match="Policy"):
        A.decide(A.Input([dev(0)], [stream("s", 1)], policy=7))


@pytest.mark.parametrize("kw", [{"hysteresis_margin": -0.01}, {"min_yield_sats_per_sec": -1}])
def test_rejects_negative_parameters(kw):
    with pytest.raises(A.ArbitrationError, match="non-negative"):
        A.decide(A.Input([dev(0)], [stream("s", 1)], **kw))


def test_rejects_duplicate_device_ids():
    with pytest.raises(A.ArbitrationError, match="duplicate"):
        A.decide(A.Input([dev(0), dev(0)], [stream("s", 1)]))


def test_empty_input_gives_empty_allocation():
    a = A.decide(A.Input([], []))
    assert a.assignments == [] and a.total_yield == 0 and a.skipped_device == 0


# ------------------------------------------------------------------ choice
def test_each_device_gets_the_best_stream():
    a = A.decide(A.Input([dev(1), dev(0)], [stream("low", 1), stream("high", 3), stream("mid", 2)]))
    assert [(x.device_id, x.stream) for x in a.assignments] == [("gpu-0", "high"), ("gpu-1", "high")]
    assert a.total_yield == 6 and a.skipped_device == 0


def test_idle_when_no_compatible_stream():
    a = one(A.Input([dev(0, Family.CPU)], [stream("gpu-only", 5)]))
    assert a.idle() and a.reason == "no compatible stream accepting non-zero work" and a.foregone_sats_per_sec == 0


@pytest.mark.parametrize("y,conf", [(0, 1), (5, 0)])
def test_zero_yield_streams_are_ignored(y, conf):
    assert one(A.Input([dev(0)], [stream("z", y, conf)])).idle()


def test_per_device_yield_overrides_the_default():
    s = stream("s", 1)
    s.yield_per_device["gpu-1"] = A.Yield(9, 1)
    a = A.decide(A.Input([dev(0), dev(1)], [s, stream("t", 2)]))
    assert [(x.device_id, x.stream) for x in a.assignments] == [("gpu-0", "t"), ("gpu-1", "s")]


def test_equal_scores_tie_break_by_stream_id():
    assert one(A.Input([dev(0)], [stream("b", 2), stream("a", 2), stream("c", 2)])).stream == "a"


def test_stack_btc_prefers_bitcoin_mining_within_five_percent():
    ss = [stream("ai", 1.04), stream("btc", 1.0, is_bitcoin_mining=True)]
    assert one(A.Input([dev(0)], ss, policy=A.Policy.STACK_BTC)).stream == "btc"
    assert one(A.Input([dev(0)], ss)).stream == "ai"
    ss[0] = stream("ai", 1.06)
    assert one(A.Input([dev(0)], ss, policy=A.Policy.STACK_BTC)).stream == "ai"


@pytest.mark.parametrize("policy,attr", [(A.Policy.MAXIMIZE_PRIVACY, "privacy_rating"),
                                         (A.Policy.ENVIRONMENT_FRIENDLY, "environmental_rating")])
def test_rating_policies_prefer_higher_rating(policy, attr):
    ss = [stream("plain", 1.05), stream("rated", 1.0, **{attr: 10})]   # +10% score
    assert one(A.Input([dev(0)], ss, policy=policy)).stream == "rated"
    assert one(A.Input([dev(0)], ss)).stream == "plain"


@pytest.mark.parametrize("policy", list(A.Policy))
def test_policy_score_is_raw_yield_without_bonus(policy):
    assert A.policy_score(stream("s", 3), 3.0, policy) == 3.0


# ------------------------------------------------------------------ hysteresis / held / foregone
def _prev(stream_id, device="gpu-0"):
    return A.Allocation([A.Assignment(device, stream_id, 1.0)])


def test_hysteresis_keeps_the_incumbent_under_the_margin():
    a = one(A.Input([dev(0)], [stream("inc", 1.0), stream("new", 1.04)], previous=_prev("inc"),
                    hysteresis_margin=0.05))
    assert a.stream == "inc" and a.held and "held" in a.reason
    assert a.foregone_sats_per_sec == pytest.approx(0.04) and a.switched_from_id == ""


def test_hysteresis_allows_a_switch_above_the_margin():
    a = one(A.Input([dev(0)], [stream("inc", 1.0), stream("new", 1.06)], previous=_prev("inc"),
                    hysteresis_margin=0.05))
    assert a.stream == "new" and not a.held and a.switched_from_id == "inc" and a.foregone_sats_per_sec == 0


def test_incumbent_best_is_not_held():
    a = one(A.Input([dev(0)], [stream("inc", 2.0), stream("other", 1.0)], previous=_prev("inc"),
                    hysteresis_margin=0.05))
    assert a.stream == "inc" and not a.held and a.reason == "incumbent is best; stayed" and "held" not in a.reason


def test_zero_hysteresis_exact_tie_stays_on_the_incumbent():
    a = one(A.Input([dev(0)], [stream("a", 1.0), stream("b", 1.0)], previous=_prev("b")))
    assert a.stream == "b"


def test_incumbent_that_disappeared_is_replaced():
    a = one(A.Input([dev(0)], [stream("new", 1.0)], previous=_prev("gone"), hysteresis_margin=0.5))
    assert a.stream == "new" and a.switched_from_id == "gone"


def test_hysteresis_uses_policy_score_not_raw_yield():
    # raw: ai 1.04 vs btc 1.00 (4%); under stack_btc btc scores 1.05 > 1.04 -> incumbent ai is NOT best and the
    # 0.96% score gap is inside a 5% margin, so ai is held.
    ss = [stream("ai", 1.04), stream("btc", 1.0, is_bitcoin_mining=True)]
    a = one(A.Input([dev(0)], ss, previous=_prev("ai"), policy=A.Policy.STACK_BTC, hysteresis_margin=0.05))
    assert a.stream == "ai" and a.held
    # margin smaller than the score gain -> switch
    a = one(A.Input([dev(0)], ss, previous=_prev("ai"), policy=A.Policy.STACK_BTC, hysteresis_margin=0.001))
    assert a.stream == "btc" and a.switched_from_id == "ai"


def test_foregone_quantifies_policy_deviation():
    ss = [stream("ai", 1.04), stream("btc", 1.0, is_bitcoin_mining=True)]
    a = one(A.Input([dev(0)], ss, policy=A.Policy.STACK_BTC))
    assert a.stream == "btc" and a.foregone_sats_per_sec == pytest.approx(0.04)


def test_foregone_zero_when_best_and_when_idle():
    assert one(A.Input([dev(0)], [stream("a", 2), stream("b", 1)])).foregone_sats_per_sec == 0
    assert one(A.Input([dev(0)], [])).foregone_sats_per_sec == 0


# ------------------------------------------------------------------ floor
def test_floor_idles_a_device_below_it():
    a = one(A.Input([dev(0)], [stream("s", 0.5)], min_yield_sats_per_sec=1.0))
    assert a.idle() and "below minimum yield floor 1 sats/s" in a.reason


def test_floor_keeps_a_device_at_or_above_it():
    assert one(A.Input([dev(0)], [stream("s", 1.0)], min_yield_sats_per_sec=1.0)).stream == "s"


def test_floor_excludes_only_the_streams_below_it():
    ss = [stream("rated", 0.9, privacy_rating=50), stream("plain", 1.1)]
    a = one(A.Input([dev(0)], ss, policy=A.Policy.MAXIMIZE_PRIVACY, min_yield_sats_per_sec=1.0))
    assert a.stream == "plain"


def test_zero_floor_disables_it():
    assert one(A.Input([dev(0)], [stream("s", 1e-12)])).stream == "s"


# ------------------------------------------------------------------ determinism
def test_deterministic_for_identical_and_shuffled_input():
    rng = random.Random(5)
    devs = [dev(i, fam) for i in range(4) for fam in (Family.GPU, Family.CPU)]
    ss = [stream(f"s{i}", rng.uniform(0.1, 5), rng.uniform(0.1, 1), fams=rng.sample(list(Family), 2))
          for i in range(6)]
    ref = A.decide(A.Input(devs, ss))
    for _ in range(10):
        d2, s2 = devs[:], ss[:]
        rng.shuffle(d2)
        rng.shuffle(s2)
        got = A.decide(A.Input(d2, s2))
        assert [(a.device_id, a.stream, a.expected_yield) for a in got.assignments] == \
            [(a.device_id, a.stream, a.expected_yield) for a in ref.assignments]


# ------------------------------------------------------------------ properties
fams = st.sampled_from(list(Family))
streams_st = st.lists(
    st.tuples(st.floats(0, 50), st.floats(0, 1), st.lists(fams, min_size=1, max_size=3, unique=True),
              st.booleans(), st.integers(0, 20), st.integers(0, 20)),
    min_size=0, max_size=6)


def _build(raw):
    return [A.Stream(f"s{i}", f, default_yield=A.Yield(y, c), is_bitcoin_mining=b, privacy_rating=p,
                     environmental_rating=e) for i, (y, c, f, b, p, e) in enumerate(raw)]


@settings(max_examples=200, deadline=None)
@given(streams_st, st.lists(fams, min_size=1, max_size=6), st.sampled_from(list(A.Policy)), st.floats(0, 0.5),
       st.floats(0, 10))
def test_properties(raw, dev_fams, policy, hyst, floor):
    ss = _build(raw)
    devs = [dev(i, f) for i, f in enumerate(dev_fams)]
    alloc = A.decide(A.Input(devs, ss, policy=policy, hysteresis_margin=hyst, min_yield_sats_per_sec=floor))
    by_id = {s.id: s for s in ss}
    assert alloc.total_yield == pytest.approx(sum(a.expected_yield for a in alloc.assignments))
    assert alloc.skipped_device == sum(a.idle() for a in alloc.assignments)
    for d, a in zip(sorted(devs, key=lambda d: d.identity.id), alloc.assignments):
        fam = d.identity.family
        eligible = [s for s in ss if s.accepts(fam) and s.default_yield.effective() > 0
                    and s.default_yield.effective() >= floor]
        assert a.foregone_sats_per_sec >= 0
        if a.idle():
            assert not eligible  # never idle while an above-floor compatible stream exists
            continue
        s = by_id[a.stream]
        assert s.accepts(fam)  # never an incompatible family
        assert a.expected_yield >= floor  # non-idle assignments clear the floor
        # no previous allocation: the choice is the policy-score maximum (greedy is optimal per device)
        best = max(A.policy_score(x, x.default_yield.effective(), policy) for x in eligible)
        assert A.policy_score(s, a.expected_yield, policy) == pytest.approx(best)


@settings(max_examples=150, deadline=None)
@given(streams_st, st.sampled_from(list(A.Policy)), st.floats(0, 0.5), st.integers(0, 5))
def test_hold_never_costs_more_than_the_margin_in_score(raw, policy, hyst, pick):
    ss = [s for s in _build(raw) if s.accepts(Family.GPU) and s.default_yield.effective() > 0]
    if not ss:
        return
    inc = ss[pick % len(ss)]
    a = one(A.Input([dev(0)], ss, previous=_prev(inc.id), policy=policy, hysteresis_margin=hyst))
    best = max(A.policy_score(x, x.default_yield.effective(), policy) for x in ss)
    by = {x.id: x for x in ss}
    got = A.policy_score(by[a.stream], by[a.stream].default_yield.effective(), policy)
    assert best <= got * (1 + hyst) + 1e-9
    if a.held:
        assert a.stream == inc.id and a.foregone_sats_per_sec >= 0
