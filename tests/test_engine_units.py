"""Engine helper and metrics-registry units (reference internal/engine/*_test.go, internal/metrics/*_test.go):
hashrate window counter-reset saturation, uptime/sats accounting, reject taxonomy, nearest-rank latency
quantiles, stall monitor, provider yield formulas, registry validation and text exposition."""
import io
import math

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from otedama_amd import metrics as M
from otedama_amd import provider as P
from otedama_amd.engine import stats as S


@pytest.mark.parametrize("hps,s", [(0, "0 H/s"), (500, "500 H/s"), (999, "999 H/s"), (1e3, "1.00 kH/s"), (2.5e6, "2.50 MH/s"),
                                   (18.3e9, "18.30 GH/s"), (1.5e12, "1.50 TH/s"), (2e15, "2.00 PH/s"),
                                   (3e18, "3.00 EH/s")])
def test_hashrate_string(hps, s):
    assert S.hashrate_string(hps) == s


def test_hashrate_window_never_negative_or_nan():
    w = S.HashrateWindow()
    assert w.observe(100, 10.0) == 0.0          # first sample primes
    assert w.observe(1100, 11.0) == 1000.0
    assert w.observe(50, 12.0) == 0.0           # counter reset (reconnect) saturates to 0
    assert w.observe(150, 12.0) == 0.0          # zero interval
    assert w.observe(350, 14.0) == 100.0


def test_uptime_and_sats_accounting():
    reg = M.Registry()
    c = reg.new_counter("otedama_uptime_seconds_total", "x")
    u = S.UptimeAccountant()
    u.observe(0.0, True, c)
    for t in (0.4, 0.8, 1.2, 1.6, 2.0):
        u.observe(t, True, c)
    u.observe(10.0, False, c)                    # unproductive time is not counted
    assert c.value() == 2
    s = S.SatsAccountant()
    assert s.observe(0.0, 5.0, True) == 0.0
    assert s.observe(2.0, 5.0, True) == 10.0
    assert s.observe(3.0, 5.0, False) == 10.0
    assert s.observe(4.0, -1.0, True) == 10.0


@pytest.mark.parametrize("reason,cls", [
    ("stale-job", "stale"), ("Job not found", "stale"), ("duplicate-share", "duplicate"),
    ("low-difficulty-share", "difficulty"), ("above target", "difficulty"), ("high-hash", "difficulty"),
    ("invalid-version-bits", "hardware"), ("bad nonce", "hardware"), ("pool is tired", "other"),
])
def test_reject_taxonomy(reason, cls):
    assert S.reject_class(reason)[0] == cls
    assert cls in S.REJECT_CATEGORIES


def test_acceptance_and_effective_yield():
    assert S.acceptance_rate(0, 0) == 1.0
    assert S.acceptance_rate(3, 1) == 0.75
    assert S.effective_yield(10.0, 30.0, 60.0) == 5.0
    assert S.effective_yield(10.0, 90.0, 60.0) == 10.0   # clamped to 1
    assert S.effective_yield(10.0, 5.0, 0.0) == 0.0


@settings(max_examples=60, deadline=None)
@given(xs=st.lists(st.floats(0, 1e4), min_size=1, max_size=600), q=st.sampled_from([0.5, 0.95, 0.99]))
def test_latency_quantile_is_nearest_rank_over_the_ring(xs, q):
    t = S.LatencyTracker(256)
    for x in xs:
        t.record(x)
    t.record(-1.0)  # ignored
    window = xs[-256:]
    n = len(window)
    assert t.count() == n
    srt = sorted(window)
    assert t.quantile(q) == srt[min(max(int(q * n + 0.5) - 1, 0), n - 1)]


def test_stall_monitor():
    logs = []
    m = S.HashrateMonitor(floor=0.0, max_stall=3, log=lambda lvl, msg: logs.append(lvl))
    for _ in range(2):
        m.observe(0.0)
    assert not m.stalled()
    m.observe(0.0)
    assert m.stalled() and logs == ["warn"]
    m.observe(0.0)
    assert logs == ["warn"]          # warned once per stall
    m.observe(5e9)
    assert not m.stalled() and logs == ["warn", "info"]


def test_provider_yields():
    assert P.sats_per_second(3.6, 1e8 / 1e3) == pytest.approx(1.0)  # $3.6/h at 100k $/BTC -> 1 sat/s
    assert P.sats_per_second(1.0, 0) == 0.0
    assert P.Yield(10, 9, 0.5).effective() == 4.5
    assert P.Yield(10, -1, 0.5).effective() == 0.0 and P.Yield(10, 9, 0.0).effective() == 0.0


# ------------------------------------------------------------------ metrics registry
def test_registry_rejects_bad_names_and_type_clashes():
    r = M.Registry()
    for bad in ("", "1abc", "a-b", "with space"):
        with pytest.raises(M.MetricsError):
            r.new_counter(bad, "h")
    with pytest.raises(M.MetricsError):
        r.new_gauge("ok_name", "h", {"bad-label": "x"})
    r.new_counter("otedama_x_total", "h")
    with pytest.raises(M.MetricsError):
        r.new_gauge("otedama_x_total", "h")
    g = r.new_gauge("otedama_g", "h", {"device": "gpu-0"})
    assert r.new_gauge("otedama_g", "h", {"device": "gpu-0"}) is g   # idempotent per label set
    assert r.new_gauge("otedama_g", "h", {"device": "gpu-1"}) is not g
    c = r.new_counter("otedama_c_total", "h")
    with pytest.raises(M.MetricsError):
        c.add(-1)
    c.add(1 << 64)   # wraps like a uint64
    assert c.value() == 0


def test_registry_text_exposition_escaping_and_order():
    r = M.Registry()
    r.new_gauge("otedama_b", 'help with \\ and\nnewline').set(1.5)
    r.new_counter("otedama_a_total", "a", {"pool": 'x"y\\z\n'}).inc()
    r.new_gauge("otedama_nan", "n").set(float("nan"))
    r.new_gauge("otedama_inf", "n").set(math.inf)
    buf = io.StringIO()
    r.write_text(buf)
    out = buf.getvalue()
    assert out.index("otedama_a_total") < out.index("otedama_b") < out.index("otedama_inf")
    assert '# HELP otedama_b help with \\\\ and\\nnewline' in out
    assert 'otedama_a_total{pool="x\\"y\\\\z\\n"} 1' in out
    assert "# TYPE otedama_a_total counter" in out and "# TYPE otedama_b gauge" in out
    assert "otedama_nan NaN" in out and "otedama_inf +Inf" in out


@settings(max_examples=400, deadline=None)
@given(v=st.floats(1e-4, 1e6, exclude_max=True), neg=st.booleans())
def test_format_float_fast_path_matches_the_decimal_path(v, neg):
    v = -v if neg else v
    assert M.format_float(v) == M._format_float_exp(v)


def test_gauge_text_cache_follows_value_changes():
    g = M.Registry().new_gauge("otedama_t", "t")
    assert g.text() == "0"
    g.set(-0.0)
    assert g.text() == "-0"
    g.set(1.5e7)
    assert g.text() == "1.5e+07"
    g.set(float("nan"))
    assert g.text() == "NaN"
    g.set(2.0)
    assert g.text() == "2"
