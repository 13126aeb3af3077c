"""Engine orchestration, case by case: mirrors internal/engine/{run,helpers,coverage,fanin}_test.go.

The reference tests its engine through package-private helpers plus fake pools; here the same behaviours are driven
through `Engine`'s pumps, stats tick, arbitration glue and reconnect loop with in-process fakes (no sockets, no native
miners), so every branch is deterministic. Reference behaviour (file:line in /root/reference/internal/engine):
  * helpers: poolURLs / payoutAddresses / sessionUser / maskAddr ... setup.go:213-270
  * curtailDecision ................................................ run.go:123-135 (table: run_test.go:1112-1152)
  * hashrateWindow / HashrateMonitor / LatencyTracker / accountants . stats.go:151-457
  * publishBTCRate / publishDifficulty ............................. stats.go:476-513
  * setupWallet / printRecoveryPhrase .............................. setup.go:117-197
  * session: job activation, stale skip, submit verdicts, stats tick run.go:610-961
  * arbitration glue: updateStream / streamsSlice / applyAllocation  arbitrate.go:62-299
  * reconnect loop: pool-fast, address-slow, backoff 1..64 s, fatal  run.go:343-521
"""
import asyncio
from types import SimpleNamespace
import io
import re

import pytest

from otedama_amd import arbitration as arb
from otedama_amd import hal
from otedama_amd.config import DEFAULT_POOL_URL, Config, PoolConfig
from otedama_amd.engine import run as R
from otedama_amd.engine import stats as S
from otedama_amd.engine.metrics import EngineMetrics
from otedama_amd.engine.run import Engine, Options
from otedama_amd.lightning import seedstore as SS
from otedama_amd.metrics import Registry
from otedama_amd.poolproto import FatalPoolError, Job, ShareSubmission
from otedama_amd.poolproto.base import ShareResult
from otedama_amd.provider import Quote, Yield

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"
ADDR2 = "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa"


# ---------------------------------------------------------------------------------------------- fakes

class FakeMiners:
    """The MinerSet surface Engine drives (engine/miners.py)."""

    def __init__(self, ids=("cpu-0",)):
        self.ids = list(ids)
        self.jobs: list = []
        self.paused: dict[str, bool] = {i: False for i in ids}
        self.pause_all_calls = 0
        self.queue: list[dict] = []
        self.hashes = 0
        self.dropped = 0
        self.rates = {i: 0.0 for i in ids}
        self.faults: list = []
        self.stalled_ids: list = []
        self.miners = []
        self.epoch = 0

    def __len__(self):
        return len(self.ids)

    def start(self):
        pass

    def stop(self):
        pass

    def set_job(self, t):
        self.jobs.append(t)
        self.epoch += 1
        return self.epoch

    def pause_all(self):
        self.pause_all_calls += 1

    def pause_device(self, dev, paused=True):
        changed = self.paused.get(dev) != paused
        self.paused[dev] = paused
        return changed

    def poll(self, max_per_device=256):
        out, self.queue = self.queue, []
        return out

    def total_hashes(self):
        return self.hashes

    def total_dropped(self):
        return self.dropped

    def update_hashrates(self):
        return dict(self.rates)

    def retire_faulted(self):
        f, self.faults = self.faults, []
        return f

    def stalled(self):
        return list(self.stalled_ids)

    def device_stats(self):
        return {i: {"faulted": False} for i in self.ids}

    def live(self):
        return list(self.ids)


class FakeSession:
    def __init__(self, verdict=None, difficulty=1.0):
        self.jobs: asyncio.Queue = asyncio.Queue()
        self.notices: asyncio.Queue = asyncio.Queue()
        self.submitted: list[ShareSubmission] = []
        self.verdict = verdict or (lambda sub: ShareResult(True, latency_ms=5.0))
        self.difficulty = difficulty

    async def submit(self, sub):
        self.submitted.append(sub)
        v = self.verdict(sub)
        if isinstance(v, Exception):
            raise v
        return v

    def suggested_difficulty(self):
        return self.difficulty


class FakeFetcher:
    def __init__(self, rate=95000.0, fresh=True, skew=0.0, age=(0.0, False), health=(0, 0, False)):
        self.rate, self.fresh, self.skew, self.age, self.health = rate, fresh, skew, age, health

    def btc_usd_rate(self):
        return self.rate, self.fresh

    def clock_skew_seconds(self):
        return self.skew

    def rate_age(self):
        return self.age

    def source_health(self):
        return self.health


class Clock:
    def __init__(self, t=1000.0):
        self.t = t

    def now(self):
        return self.t


def cpu_device(i=0):
    return hal.SimpleDevice(hal.Identity(f"cpu-{i}", hal.Family.CPU, "test", "cpu"),
                            hal.Capabilities(sha256d=True, general_compute=True))


def gpu_device(i=0):
    return hal.SimpleDevice(hal.Identity(f"gpu-{i}", hal.Family.GPU, "AMD", "MI355X"),
                            hal.Capabilities(sha256d=True, general_compute=True, scrypt=True, x11=True), index=i)


def make_engine(cfg=None, **kw):
    logs: list[tuple[str, str]] = []
    opts = Options(config=cfg or Config(bitcoin_address=ADDR), logger=lambda lvl, msg: logs.append((lvl, msg)),
                   metrics=Registry(), clock=kw.pop("clock", Clock()), rate_fetcher=FakeFetcher(), **kw)
    eng = Engine(opts)
    eng.miners = FakeMiners()
    return eng, logs


def share(job_id="j1", nonce=1, ntime=0x60000000, version=0x20000004, dev="cpu-0", en2=0, en2_size=0, digest=None):
    s = {"job_id": job_id, "nonce": nonce, "ntime": ntime, "version": version, "device_id": dev,
         "extranonce2": en2, "extranonce2_size": en2_size, "found_at": 0.0}
    if digest is not None:
        s["hash"] = digest
    return s


async def run_pump_until(coro, cond, timeout=2.0):
    task = asyncio.ensure_future(coro)
    try:
        end = asyncio.get_event_loop().time() + timeout
        while not cond():
            if asyncio.get_event_loop().time() > end:
                raise AssertionError("condition not reached")
            await asyncio.sleep(0.005)
        await asyncio.sleep(0.01)
    finally:
        task.cancel()
        try:
            await task
        except asyncio.CancelledError:
            pass


def logged(logs, level, pattern):
    return [m for lvl, m in logs if lvl == level and re.search(pattern, m)]


# ---------------------------------------------------------------------------------------------- helpers

def test_pool_urls_empty_returns_default():
    assert R.pool_urls(Config()) == [DEFAULT_POOL_URL]


def test_pool_urls_preserves_order():
    cfg = Config(pools=[PoolConfig(url=u) for u in ("stratum+v2://a:1", "stratum+tcp://b:2", "stratum+tls://c:3")])
    assert R.pool_urls(cfg) == ["stratum+v2://a:1", "stratum+tcp://b:2", "stratum+tls://c:3"]


def test_pool_urls_single_pool():
    assert R.pool_urls(Config(pools=[PoolConfig(url="stratum+v2://x:9")])) == ["stratum+v2://x:9"]


def test_payout_addresses_primary_first_then_list():
    cfg = Config(bitcoin_address=ADDR, bitcoin_addresses=[ADDR2, "3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy"])
    assert R.payout_addresses(cfg) == [ADDR, ADDR2, "3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy"]


def test_payout_addresses_dedup_and_skip_empty():
    cfg = Config(bitcoin_address=ADDR, bitcoin_addresses=["", ADDR, ADDR2, ADDR2, ""])
    assert R.payout_addresses(cfg) == [ADDR, ADDR2]


def test_payout_addresses_list_only_no_primary():
    assert R.payout_addresses(Config(bitcoin_addresses=[ADDR2, ADDR])) == [ADDR2, ADDR]
    assert R.payout_addresses(Config()) == []


@pytest.mark.parametrize("pool_user,addr,worker,want", [
    ("acct.rig", ADDR, "w1", "acct.rig"),       # explicit pool user wins
    ("", ADDR, "w1", ADDR + ".w1"),
    ("", ADDR, "", ADDR),
    ("", "", "", ""),
])
def test_session_user_precedence(pool_user, addr, worker, want):
    assert R.session_user(pool_user, addr, worker) == want


def test_mask_addr_hides_middle():
    assert R.mask_addr(ADDR) == "bc1qar…5mdq"
    assert ADDR[6:-4] not in R.mask_addr(ADDR)


@pytest.mark.parametrize("a", ["", "bc1q", "123456789012"])
def test_mask_addr_short_or_twelve_chars_returned_as_is(a):
    assert R.mask_addr(a) == a


def test_mask_addr_thirteen_chars_masked():
    assert R.mask_addr("1234567890123") == "123456…0123"


@pytest.mark.parametrize("curr,rate,fresh,thr,want", [
    (False, 95000, False, 100000, (False, False)),   # not fresh below threshold does not curtail
    (True, 95000, False, 90000, (True, False)),      # not fresh above threshold does not uncurtail
    (False, 89000, True, 90000, (True, True)),       # fresh below threshold curtails
    (True, 95000, True, 90000, (False, True)),       # fresh above threshold uncurtails
    (True, 80000, True, 90000, (True, False)),       # already curtailed
    (False, 95000, True, 90000, (False, False)),     # already running
    (True, 90000, True, 90000, (False, True)),       # exactly at threshold is not below
    (False, 90000, True, 90000, (False, False)),
    (False, 1, True, 0, (False, False)),             # threshold 0 disables
    (True, 1, True, 0, (True, False)),
    (False, 50000, True, -1, (False, False)),        # negative threshold disabled
    (True, 0, True, 90000, (True, False)),           # zero rate never changes state
    (False, -5, True, 90000, (False, False)),        # negative rate never changes state
])
def test_curtail_decision(curr, rate, fresh, thr, want):
    assert R.curtail_decision(curr, rate, fresh, thr) == want


# ---------------------------------------------------------------------------------------------- stats helpers

def test_hashrate_window_first_sample_is_zero():
    assert S.HashrateWindow().observe(10**9, 5.0) == 0.0


def test_hashrate_window_computes_rate_over_interval():
    w = S.HashrateWindow()
    w.observe(1000, 10.0)
    assert w.observe(21000, 12.0) == 10000.0
    assert w.observe(21000 + 5 * 10**6, 17.0) == 10**6


def test_hashrate_window_stall_shows_zero_rate():
    w = S.HashrateWindow()
    w.observe(500, 1.0)
    assert w.observe(500, 2.0) == 0.0


def test_hashrate_window_saturates_on_counter_reset():
    w = S.HashrateWindow()
    w.observe(10**6, 1.0)
    assert w.observe(10, 2.0) == 0.0           # reset (reconnect): never negative
    assert w.observe(1010, 3.0) == 1000.0      # re-primed from the reset value


@pytest.mark.parametrize("dt", [0.0, -1.0])
def test_hashrate_window_zero_or_negative_delta_time_yields_zero(dt):
    w = S.HashrateWindow()
    w.observe(0, 5.0)
    assert w.observe(1000, 5.0 + dt) == 0.0


def test_hashrate_window_feeds_stall_monitor():
    w, mon = S.HashrateWindow(), S.HashrateMonitor(0, 3)
    w.observe(0, 0.0)
    for t in range(1, 4):
        mon.observe(w.observe(0, float(t)))
    assert mon.stalled()


def test_hashrate_monitor_warns_after_sustained_stall():
    logs = []
    mon = S.HashrateMonitor(0, 3, lambda lvl, msg: logs.append((lvl, msg)))
    mon.observe(0)
    mon.observe(0)
    assert not mon.stalled() and not logs
    mon.observe(0)
    assert mon.stalled()
    assert len(logged(logs, "warn", "hashrate stalled at 0 H/s for 3 consecutive samples")) == 1
    mon.observe(0)
    assert len(logs) == 1  # warned once per stall episode


def test_hashrate_monitor_resets_on_recovery():
    logs = []
    mon = S.HashrateMonitor(0, 2, lambda lvl, msg: logs.append((lvl, msg)))
    mon.observe(0)
    mon.observe(0)
    assert mon.stalled()
    mon.observe(5e9)
    assert not mon.stalled() and mon.stall_count == 0
    assert logged(logs, "info", "hashrate recovered")
    mon.observe(0)
    assert not mon.stalled()


def test_hashrate_monitor_floor_above_zero():
    mon = S.HashrateMonitor(1e6, 2)
    mon.observe(5e5)
    mon.observe(1e6)   # <= floor counts as stalled
    assert mon.stalled()
    mon.observe(1e6 + 1)
    assert not mon.stalled()


@pytest.mark.parametrize("n", [0, -4])
def test_new_hashrate_monitor_default_max_stall(n):
    assert S.HashrateMonitor(0, n).max_stall == 3


def test_latency_tracker_empty_returns_zero():
    lt = S.LatencyTracker()
    assert lt.count() == 0 and lt.quantile(0.5) == 0.0 and lt.quantile(0.99) == 0.0


def test_latency_tracker_quantiles():
    lt = S.LatencyTracker(256)
    for v in range(1, 101):
        lt.record(float(v))
    assert (lt.quantile(0.5), lt.quantile(0.95), lt.quantile(0.99)) == (50.0, 95.0, 99.0)


@pytest.mark.parametrize("q,want", [(0.0, 3.0), (-1.0, 3.0), (1.0, 40.0), (7.0, 40.0)])
def test_latency_tracker_quantile_endpoints_clamp(q, want):
    lt = S.LatencyTracker(8)
    for v in (10.0, 3.0, 40.0, 7.0):
        lt.record(v)
    assert lt.quantile(q) == want


def test_latency_tracker_ring_buffer_overwrites():
    lt = S.LatencyTracker(4)
    for v in (1000.0, 1000.0, 1000.0, 1000.0, 1.0, 2.0, 3.0, 4.0):
        lt.record(v)
    assert lt.count() == 4 and lt.quantile(1.0) == 4.0


def test_latency_tracker_ignores_negative():
    lt = S.LatencyTracker(4)
    lt.record(-1.0)
    lt.record(0.0)
    assert lt.count() == 1 and lt.quantile(0.5) == 0.0


@pytest.mark.parametrize("size", [0, -3])
def test_new_latency_tracker_default_size(size):
    lt = S.LatencyTracker(size)
    for v in range(300):
        lt.record(float(v))
    assert lt.count() == 256


@pytest.mark.parametrize("acc,rej,want", [(0, 0, 1.0), (10, 0, 1.0), (0, 5, 0.0), (3, 1, 0.75), (97, 3, 0.97)])
def test_acceptance_rate(acc, rej, want):
    assert S.acceptance_rate(acc, rej) == pytest.approx(want)


@pytest.mark.parametrize("reason,cat", [
    ("stale-prevhash", "stale"), ("Job not found", "stale"), ("unknown job", "stale"), ("duplicate share", "duplicate"),
    ("above target", "difficulty"), ("low difficulty share", "difficulty"), ("high-hash", "difficulty"),
    ("invalid-nonce", "hardware"), ("bad-version", "hardware"), ("", "other"), ("pool on fire", "other"),
])
def test_reject_class(reason, cat):
    got, diag = S.reject_class(reason)
    assert got == cat and diag.startswith(("likely cause", "cause unclassified"))


class Counter:
    def __init__(self):
        self.total = 0

    def add(self, n):
        self.total += n


def test_uptime_accountant_primes_on_first_observe():
    u, c = S.UptimeAccountant(), Counter()
    u.observe(100.0, True, c)
    assert c.total == 0 and u.last_tick == 100.0


def test_uptime_accountant_accumulates_productive_seconds():
    u, c = S.UptimeAccountant(), Counter()
    for t in (0.0, 10.0, 20.0, 30.0):
        u.observe(t, True, c)
    assert c.total == 30


def test_uptime_accountant_skips_non_productive_time():
    u, c = S.UptimeAccountant(), Counter()
    u.observe(0.0, True, c)
    u.observe(10.0, False, c)
    u.observe(15.0, True, c)
    assert c.total == 5


def test_uptime_accountant_carries_fractional_remainder():
    u, c = S.UptimeAccountant(), Counter()
    u.observe(0.0, True, c)
    for i in range(1, 5):
        u.observe(i * 0.6, True, c)  # 2.4 s of 0.6 s ticks
    assert c.total == 2 and u.accum == pytest.approx(0.4)


def test_uptime_accountant_ignores_non_positive_and_nil_counter():
    u, c = S.UptimeAccountant(), Counter()
    u.observe(10.0, True, c)
    u.observe(5.0, True, c)       # backwards clock
    u.observe(5.0, True, c)       # zero elapsed
    u.observe(20.0, True, None)   # no counter
    assert c.total == 0


def test_sats_accountant_primes_on_first_observe():
    s = S.SatsAccountant()
    assert s.observe(50.0, 100.0, True) == 0.0


def test_sats_accountant_integrates_rate_over_productive_time():
    s = S.SatsAccountant()
    s.observe(0.0, 2.0, True)
    s.observe(10.0, 2.0, True)
    assert s.observe(15.0, 4.0, True) == pytest.approx(40.0)


def test_sats_accountant_skips_non_productive_interval():
    s = S.SatsAccountant()
    s.observe(0.0, 2.0, True)
    assert s.observe(10.0, 2.0, False) == 0.0


def test_sats_accountant_skips_non_positive_rate_and_backwards_clock():
    s = S.SatsAccountant()
    s.observe(10.0, 1.0, True)
    assert s.observe(20.0, 0.0, True) == 0.0
    assert s.observe(30.0, -3.0, True) == 0.0
    assert s.observe(25.0, 1.0, True) == 0.0


def test_sats_accountant_retains_fractional_precision():
    s = S.SatsAccountant()
    s.observe(0.0, 1e-3, True)
    for i in range(1, 1001):
        s.observe(i * 0.001, 1e-3, True)
    assert s.total == pytest.approx(1e-3)


@pytest.mark.parametrize("expected,prod,up,want", [
    (10.0, 100.0, 100.0, 10.0),    # full uptime
    (10.0, 50.0, 100.0, 5.0),      # half
    (10.0, 0.0, 0.0, 0.0),         # zero uptime: 0, not NaN
    (10.0, 5.0, -1.0, 0.0),        # negative uptime
    (10.0, 200.0, 100.0, 10.0),    # fraction clamped to 1
    (0.0, 100.0, 100.0, 0.0),      # zero expected
])
def test_effective_yield(expected, prod, up, want):
    assert S.effective_yield(expected, prod, up) == pytest.approx(want)


# ---------------------------------------------------------------------------------------------- publishers

def metrics():
    reg = Registry()
    return reg, EngineMetrics(reg)


def test_publish_btc_rate_sets_gauge():
    _, m = metrics()
    S.publish_btc_rate(m, FakeFetcher(rate=101234.0))
    assert m.btc_usd_rate.value() == 101234.0


def test_publish_btc_rate_publishes_all_post_fetch_branches():
    _, m = metrics()
    S.publish_btc_rate(m, FakeFetcher(rate=90000.0, skew=2.5, age=(42.0, True), health=(2, 3, True)))
    assert (m.clock_skew_seconds.value(), m.btc_rate_age_seconds.value()) == (2.5, 42.0)
    assert (m.rate_sources_ok.value(), m.rate_sources_total.value()) == (2, 3)


def test_publish_btc_rate_skips_branches_before_fetch():
    _, m = metrics()
    m.rate_sources_total.set(7)
    S.publish_btc_rate(m, FakeFetcher(rate=0.0, skew=0.0, age=(0.0, False), health=(0, 3, False)))
    assert m.btc_usd_rate.value() == 0.0 and m.clock_skew_seconds.value() == 0.0
    assert m.btc_rate_age_seconds.value() == 0.0            # age gauge zero before any fetch
    assert m.rate_sources_total.value() == 7                # source health untouched before fetch


def test_publish_difficulty_sets_gauges_at_known_hashrate():
    _, m = metrics()
    S.publish_difficulty(m, 8.0, 2 ** 32)
    assert m.pool_difficulty.value() == 8.0
    assert m.estimated_share_interval_seconds.value() == pytest.approx(8.0)


def test_publish_difficulty_zero_hashrate_yields_zero_interval():
    _, m = metrics()
    m.estimated_share_interval_seconds.set(99)
    S.publish_difficulty(m, 8.0, 0.0)
    assert m.pool_difficulty.value() == 8.0 and m.estimated_share_interval_seconds.value() == 0.0


@pytest.mark.parametrize("d", [0.0, -1.0])
def test_publish_difficulty_zero_difficulty_is_noop(d):
    _, m = metrics()
    m.pool_difficulty.set(3.0)
    S.publish_difficulty(m, d, 1e9)
    assert m.pool_difficulty.value() == 3.0


def test_publish_difficulty_scrypt_diff1():
    _, m = metrics()
    S.publish_difficulty(m, 1.0, 65536.0, hashes_per_diff1=65536.0)
    assert m.estimated_share_interval_seconds.value() == pytest.approx(1.0)


# ---------------------------------------------------------------------------------------------- metric bundle

def test_inc_shares_found_for_device_creates_counter_and_accumulates():
    reg, m = metrics()
    assert "otedama_device_shares_found_total" not in reg.render()
    m.inc_shares_found_for_device("gpu-0")
    m.inc_shares_found_for_device("gpu-0")
    m.inc_shares_found_for_device("gpu-1")
    text = reg.render()
    assert 'otedama_device_shares_found_total{device="gpu-0"} 2' in text
    assert 'otedama_device_shares_found_total{device="gpu-1"} 1' in text


def test_inc_shares_found_for_device_empty_id_is_noop():
    reg, m = metrics()
    m.inc_shares_found_for_device("")
    assert "otedama_device_shares_found_total" not in reg.render()


def test_inc_shares_found_for_device_label_set_is_bounded():
    reg, m = metrics()
    for i in range(80):
        m.inc_shares_found_for_device(f"gpu-{i}")
    assert reg.render().count("otedama_device_shares_found_total{") == 64


@pytest.mark.parametrize("name", ["otedama_curtailed", "otedama_joules_per_terahash", "otedama_active_streams",
                                  "otedama_power_cost_usd_per_hour", "otedama_arbitration_holds_total",
                                  "otedama_effective_yield_sats_per_second", "otedama_power_watts", "otedama_up"])
def test_engine_metrics_registered_and_zero(name):
    reg, _ = metrics()
    assert re.search(rf"^{name} 0$", reg.render(), re.M)


def test_set_active_payout_exposes_active_address():
    reg, m = metrics()
    m.set_active_payout("bc1qar…5mdq")
    assert 'otedama_payout_info{address="bc1qar…5mdq"} 1' in reg.render()


def test_set_active_payout_failover_zeroes_previous():
    reg, m = metrics()
    m.set_active_payout("a…1")
    m.set_active_payout("b…2")
    text = reg.render()
    assert 'otedama_payout_info{address="a…1"} 0' in text and 'otedama_payout_info{address="b…2"} 1' in text
    m.set_active_payout("a…1")
    text = reg.render()
    assert 'otedama_payout_info{address="a…1"} 1' in text and 'otedama_payout_info{address="b…2"} 0' in text


def test_set_active_payout_unchanged_is_noop():
    reg, m = metrics()
    m.set_active_payout("a…1")
    before = reg.render()
    m.set_active_payout("a…1")
    assert reg.render() == before


def test_set_active_payout_empty_ignored():
    reg, m = metrics()
    m.set_active_payout("")
    assert "otedama_payout_info" not in reg.render()


def test_reject_reason_unknown_category_maps_to_other():
    reg, m = metrics()
    m.reject_reason("martian").inc()
    m.touch_last_reject("martian", 123.0)
    text = reg.render()
    assert 'otedama_shares_rejected_by_reason_total{reason="other"} 1' in text
    assert 'otedama_last_reject_seconds{reason="other"} 123' in text


def test_update_share_rates():
    _, m = metrics()
    m.shares_found.add(10)
    m.shares_accepted.add(6)
    m.shares_rejected.add(2)
    m.reject_reason("stale").add(1)
    rate, judged = m.update_share_rates()
    assert (rate, judged) == (0.75, 8)
    assert m.reject_rate.value() == 0.25 and m.stale_rate.value() == 0.125 and m.shares_unaccounted.value() == 2


# ---------------------------------------------------------------------------------------------- wallet setup

@pytest.fixture
def fast_kdf(monkeypatch):
    monkeypatch.setattr(SS, "SCRYPT_N", 1 << 10)


def test_setup_wallet_empty_passphrase_returns_empty(tmp_path):
    eng, logs = make_engine(Config(data_dir=str(tmp_path)))
    assert eng._setup_wallet() == "" and not list(tmp_path.iterdir())


def test_setup_wallet_empty_data_dir_returns_empty():
    eng, _ = make_engine(Config(data_dir=""), wallet_passphrase="pw")
    assert eng._setup_wallet() == ""


def test_setup_wallet_bad_data_dir_logs_warning_and_returns_empty(tmp_path, fast_kdf):
    (tmp_path / "f").write_text("x")
    eng, logs = make_engine(Config(data_dir=str(tmp_path / "f" / "d")), wallet_passphrase="pw")
    assert eng._setup_wallet() == ""
    assert logged(logs, "warn", "^wallet: .*create data dir")


def test_setup_wallet_new_wallet_returns_fingerprint_and_prints_phrase(tmp_path, fast_kdf):
    out = io.StringIO()
    eng, logs = make_engine(Config(data_dir=str(tmp_path)), wallet_passphrase="pw", output=out)
    fp = eng._setup_wallet()
    assert re.fullmatch(r"[0-9a-f]{8}", fp)
    text = out.getvalue()
    assert "WALLET RECOVERY PHRASE" in text and f"Fingerprint: {fp}" in text
    words = re.search(r"\n  ([a-z ]+)\n\n  Fingerprint", text).group(1).split()
    assert len(words) == 24
    assert logged(logs, "info", "new wallet created") and logged(logs, "info", f"fingerprint {fp}")


def test_setup_wallet_existing_wallet_does_not_reprint_phrase(tmp_path, fast_kdf):
    first, _ = make_engine(Config(data_dir=str(tmp_path)), wallet_passphrase="pw", output=io.StringIO())
    fp = first._setup_wallet()
    out = io.StringIO()
    again, logs = make_engine(Config(data_dir=str(tmp_path)), wallet_passphrase="pw", output=out)
    assert again._setup_wallet() == fp and out.getvalue() == ""
    assert not logged(logs, "info", "new wallet created")


def test_setup_wallet_wrong_passphrase_logs_and_returns_empty(tmp_path, fast_kdf):
    make_engine(Config(data_dir=str(tmp_path)), wallet_passphrase="pw", output=io.StringIO())[0]._setup_wallet()
    eng, logs = make_engine(Config(data_dir=str(tmp_path)), wallet_passphrase="nope")
    assert eng._setup_wallet() == "" and logged(logs, "warn", "unlock failed")


def test_setup_wallet_mnemonic_never_reaches_logger(tmp_path, fast_kdf):
    out = io.StringIO()
    eng, logs = make_engine(Config(data_dir=str(tmp_path)), wallet_passphrase="pw", output=out)
    eng._setup_wallet()
    words = re.search(r"\n  ([a-z ]+)\n\n  Fingerprint", out.getvalue()).group(1).split()
    joined = " ".join(m for _, m in logs)
    assert " ".join(words) not in joined
    assert sum(w in joined.split() for w in words) <= 2  # no phrase leaks word by word either


def test_setup_wallet_mnemonic_passphrase_changes_seed(tmp_path, fast_kdf):
    a, _ = make_engine(Config(data_dir=str(tmp_path / "a")), wallet_passphrase="pw", output=io.StringIO())
    b, _ = make_engine(Config(data_dir=str(tmp_path / "b")), wallet_passphrase="pw", output=io.StringIO(),
                       wallet_mnemonic_passphrase="x")
    assert a._setup_wallet() and b._setup_wallet()


# ---------------------------------------------------------------------------------------------- session pumps

def test_job_pump_clean_job_activates_and_resets_valid_set():
    async def go():
        eng, logs = make_engine()
        sess = FakeSession()
        eng._valid_jobs = {"old"}
        eng._submitted = {("old", 1, 2, 3, b"")}
        await sess.jobs.put(Job("j1", version=0x20000004, clean_jobs=True))
        await run_pump_until(eng._job_pump(sess), lambda: eng.miners.jobs)
        assert eng._valid_jobs == {"j1"} and not eng._submitted
        assert eng._active_job.job_id == "j1" and eng.miners.jobs[-1]["job_id"] == "j1"
        assert logged(logs, "info", "job j1 version=0x20000004 active")
        assert eng.m.last_job_received.value() > 0
    asyncio.run(go())


def test_job_pump_non_clean_job_extends_valid_set():
    async def go():
        eng, _ = make_engine()
        sess = FakeSession()
        await sess.jobs.put(Job("a", clean_jobs=True))
        await sess.jobs.put(Job("b", clean_jobs=False))
        await run_pump_until(eng._job_pump(sess), lambda: len(eng.miners.jobs) == 2)
        assert eng._valid_jobs == {"a", "b"} and eng._active_job.job_id == "b"
    asyncio.run(go())


def test_job_pump_clean_reissue_of_same_job_keeps_duplicate_guard():
    async def go():
        eng, _ = make_engine()
        sess = FakeSession()
        eng._valid_jobs = {"a"}
        eng._submitted = {("a", 1, 2, 3, b"")}
        await sess.jobs.put(Job("a", clean_jobs=True))   # SetTarget re-issue of the active job
        await run_pump_until(eng._job_pump(sess), lambda: eng.miners.jobs)
        assert eng._submitted == {("a", 1, 2, 3, b"")}
    asyncio.run(go())


def test_job_pump_none_pauses_and_invalidates():
    async def go():
        eng, _ = make_engine()
        sess = FakeSession()
        await sess.jobs.put(Job("a", clean_jobs=True))
        await sess.jobs.put(None)
        await run_pump_until(eng._job_pump(sess), lambda: eng.miners.pause_all_calls == 1)
        assert eng._active_job is None and not eng._valid_jobs
    asyncio.run(go())


def test_curtailment_blocks_work_application():
    async def go():
        eng, logs = make_engine()
        eng.curtailed = True
        sess = FakeSession()
        await sess.jobs.put(Job("j9", clean_jobs=True))
        await run_pump_until(eng._job_pump(sess), lambda: eng._active_job is not None)
        assert not eng.miners.jobs                       # silenced while curtailed
        assert eng._active_job.job_id == "j9"            # remembered for the uncurtail resume
        assert logged(logs, "debug", "job j9 ignored \\(curtailed\\)")
    asyncio.run(go())


def test_job_pump_publishes_pool_difficulty():
    async def go():
        eng, _ = make_engine()
        eng.current_hashrate = float(2 ** 32)
        sess = FakeSession(difficulty=16.0)
        await sess.jobs.put(Job("a", clean_jobs=True))
        await run_pump_until(eng._job_pump(sess), lambda: eng.miners.jobs)
        assert eng.m.pool_difficulty.value() == 16.0
        assert eng.m.estimated_share_interval_seconds.value() == pytest.approx(16.0, rel=1e-4)  # 2^256/diff1
    asyncio.run(go())


def test_share_pump_submits_and_echoes_job_fields():
    async def go():
        eng, _ = make_engine()
        eng._valid_jobs = {"j1"}
        sess = FakeSession()
        eng.miners.queue = [share(nonce=0xDEADBEEF, ntime=0x60000000, version=0x20000004)]
        await run_pump_until(eng._share_pump(sess), lambda: sess.submitted)
        sub = sess.submitted[0]
        assert (sub.job_id, sub.nonce, sub.ntime, sub.version) == ("j1", 0xDEADBEEF, 0x60000000, 0x20000004)
        assert eng.m.shares_found.value() == 1 and eng.m.shares_submitted.value() == 1
    asyncio.run(go())


def test_share_pump_skips_stale_job_shares():
    async def go():
        eng, _ = make_engine()
        eng._valid_jobs = {"new"}
        sess = FakeSession()
        eng.miners.queue = [share(job_id="old"), share(job_id="new", nonce=7)]
        await run_pump_until(eng._share_pump(sess), lambda: sess.submitted)
        assert [s.job_id for s in sess.submitted] == ["new"]
        assert eng.m.stale_skipped.value() == 1 and eng.m.shares_found.value() == 2
    asyncio.run(go())


def test_share_pump_drops_shares_below_a_raised_target():
    """SV2 SetTarget re-issues the job with a higher difficulty. With the pool's target_grace on (a pool that credits
    in-flight shares at the previous difficulty, as otedama pool does for RETARGET_GRACE), a queued share
    the device verified against the previous target is still submitted for that long after the raise; after the
    grace, or below even the previous target, it would be rejected as low-difficulty, so it is dropped (counted)
    instead."""
    from otedama_amd.engine import run as run_mod

    async def go():
        eng, _ = make_engine()
        eng._target_grace = run_mod.TARGET_GRACE  # pools[].target_grace: 10
        sess = FakeSession()
        easy, hard = (1 << 250).to_bytes(32, "little"), (1 << 240).to_bytes(32, "little")
        await sess.jobs.put(Job("j1", clean_jobs=True, target=easy))
        await sess.jobs.put(Job("j1", clean_jobs=True, target=hard))   # the re-issue after SetTarget
        await run_pump_until(eng._job_pump(sess), lambda: len(eng.miners.jobs) == 2)
        weak, strong = (1 << 245).to_bytes(32, "little"), (1 << 230).to_bytes(32, "little")
        too_weak = (1 << 252).to_bytes(32, "little")  # above even the previous target
        eng.miners.queue = [share(nonce=1, digest=weak), share(nonce=2, digest=strong), share(nonce=3),
                            share(nonce=4, digest=too_weak)]
        await run_pump_until(eng._share_pump(sess), lambda: len(sess.submitted) == 3)
        assert sorted(s.nonce for s in sess.submitted) == [1, 2, 3]   # in grace; no hash (CPU-style): not filtered
        assert eng.m.below_target_skipped.value() == 1
        old, at = eng._prev_targets["j1"]
        eng._prev_targets["j1"] = (old, at - run_mod.TARGET_GRACE - 1)  # the grace has passed
        eng.miners.queue = [share(nonce=5, digest=weak), share(nonce=6, digest=strong)]
        await run_pump_until(eng._share_pump(sess), lambda: len(sess.submitted) == 4)
        assert sorted(s.nonce for s in sess.submitted) == [1, 2, 3, 6]
        assert eng.m.below_target_skipped.value() == 2
    asyncio.run(go())


def test_share_pump_grace_is_off_by_default():
    """an external pool that applies SetTarget at once would reject shares found under the previous
    target as low-difficulty (counted against the miner, and rate-limited by some pools): without pools[].target_grace
    they are dropped locally right after the raise."""
    async def go():
        eng, _ = make_engine()
        assert eng._target_grace == 0.0
        sess = FakeSession()
        easy, hard = (1 << 250).to_bytes(32, "little"), (1 << 240).to_bytes(32, "little")
        await sess.jobs.put(Job("j1", clean_jobs=True, target=easy))
        await sess.jobs.put(Job("j1", clean_jobs=True, target=hard))
        await run_pump_until(eng._job_pump(sess), lambda: len(eng.miners.jobs) == 2)
        weak, strong = (1 << 245).to_bytes(32, "little"), (1 << 230).to_bytes(32, "little")
        eng.miners.queue = [share(nonce=1, digest=weak), share(nonce=2, digest=strong)]
        await run_pump_until(eng._share_pump(sess), lambda: len(sess.submitted) == 1)
        assert [s.nonce for s in sess.submitted] == [2] and eng.m.below_target_skipped.value() == 1
    asyncio.run(go())


def test_pool_target_grace_config_is_validated():
    from otedama_amd.config import Config, ConfigError, PoolConfig

    Config(bitcoin_address="bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq",
           pools=[PoolConfig(url="stratum+v2://127.0.0.1:3336", target_grace=10)]).validate()
    bad = Config(bitcoin_address="bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq",
                 pools=[PoolConfig(url="stratum+v2://127.0.0.1:3336", target_grace=-1)])
    with pytest.raises(ConfigError, match="target_grace"):
        bad.validate()


def test_share_pump_never_submits_a_duplicate():
    async def go():
        eng, _ = make_engine()
        eng._valid_jobs = {"j1"}
        sess = FakeSession()
        eng.miners.queue = [share(nonce=5), share(nonce=5), share(nonce=6)]
        await run_pump_until(eng._share_pump(sess), lambda: len(sess.submitted) == 2)
        eng.miners.queue = [share(nonce=5)]
        await run_pump_until(eng._share_pump(sess), lambda: not eng.miners.queue)
        assert sorted(s.nonce for s in sess.submitted) == [5, 6]
    asyncio.run(go())


def test_share_pump_counts_per_device_and_serialises_extranonce2():
    async def go():
        eng, _ = make_engine()
        eng._valid_jobs = {"j1"}
        sess = FakeSession()
        eng.miners.queue = [share(dev="gpu-3", en2=0x0102, en2_size=4), share(dev="gpu-3", nonce=2, en2_size=0)]
        await run_pump_until(eng._share_pump(sess), lambda: len(sess.submitted) == 2)
        ens = sorted(s.extranonce2 for s in sess.submitted)
        assert ens == [b"", b"\x02\x01\x00\x00"]
        assert 'otedama_device_shares_found_total{device="gpu-3"} 2' in eng.registry.render()
    asyncio.run(go())


def test_submit_accepted_records_latency():
    async def go():
        eng, logs = make_engine()
        sess = FakeSession(lambda sub: ShareResult(True, latency_ms=12.5))
        await eng._submit(sess, ShareSubmission("j", 0xAB, 1, 2))
        assert eng.m.shares_accepted.value() == 1 and eng.latency.quantile(0.5) == 12.5
        assert logged(logs, "info", "share accepted job=j nonce=0x000000AB \\(12.5 ms\\)")
    asyncio.run(go())


@pytest.mark.parametrize("reason,cat", [("stale-prevhash", "stale"), ("duplicate", "duplicate"),
                                        ("above target", "difficulty"), ("weird", "other")])
def test_submit_rejected_classifies_reason(reason, cat):
    async def go():
        eng, logs = make_engine()
        sess = FakeSession(lambda sub: ShareResult(False, reason=reason))
        await eng._submit(sess, ShareSubmission("j", 1, 1, 1))
        assert eng.m.shares_rejected.value() == 1 and eng.m.shares_accepted.value() == 0
        text = eng.registry.render()
        assert f'otedama_shares_rejected_by_reason_total{{reason="{cat}"}} 1' in text
        assert f'otedama_last_reject_seconds{{reason="{cat}"}}' in text
        assert logged(logs, "warn", f"share rejected: {re.escape(reason)}")
    asyncio.run(go())


def test_submit_transport_error_is_logged_not_counted():
    async def go():
        eng, logs = make_engine()
        sess = FakeSession(lambda sub: ConnectionResetError("gone"))
        await eng._submit(sess, ShareSubmission("j", 1, 1, 1))
        assert eng.m.shares_submitted.value() == 1
        assert eng.m.shares_accepted.value() == 0 and eng.m.shares_rejected.value() == 0
        assert logged(logs, "warn", "submit share: gone")
    asyncio.run(go())


# ---------------------------------------------------------------------------------------------- stats tick

def tick(eng, clock, dt, hashes):
    clock.t += dt
    eng.miners.hashes += hashes
    eng.tick_stats()


def test_tick_stats_logs_hashrate():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    tick(eng, clock, 0, 0)
    tick(eng, clock, 10, 25 * 10**9)
    assert eng.current_hashrate == 2.5e9 and eng.m.hashrate.value() == 2.5e9
    assert logged(logs, "info", r"hashrate=2\.50 GH/s shares=0")


def test_tick_stats_zero_hashrate():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    tick(eng, clock, 0, 0)
    tick(eng, clock, 10, 0)
    assert logged(logs, "info", "hashrate=0 H/s")


def test_update_liveness_curtailed_reports_healthy_and_does_not_stall():
    clock = Clock()
    eng, _ = make_engine(clock=clock)
    eng.curtailed = True
    for _ in range(6):
        tick(eng, clock, 10, 0)
    assert eng.m.up.value() == 1 and not eng.stalled


def test_update_liveness_not_curtailed_zero_hashrate_stalls():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    for _ in range(4):
        tick(eng, clock, 10, 0)
    assert eng.stalled and eng.m.up.value() == 0
    assert logged(logs, "warn", "hashrate stalled")


def test_update_liveness_healthy_hashrate_reports_up():
    clock = Clock()
    eng, _ = make_engine(clock=clock)
    for _ in range(4):
        tick(eng, clock, 10, 10**10)
    assert not eng.stalled and eng.m.up.value() == 1


def test_tick_stats_publishes_device_hashrates_and_health():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    eng.miners = FakeMiners(["gpu-0", "gpu-1"])
    eng.miners.rates = {"gpu-0": 18.7e9, "gpu-1": 0.0}
    eng.miners.stalled_ids = ["gpu-1"]
    eng.miners.faults = [("gpu-1", "hipErrorLaunchFailure")]
    tick(eng, clock, 1, 0)
    text = eng.registry.render()
    assert 'otedama_device_hashrate_hashes_per_second{device="gpu-0"} 1.87e+10' in text
    assert eng.m.devices_stalled.value() == 1 and eng.m.devices_active.value() == 1
    assert logged(logs, "error", "device gpu-1 faulted: hipErrorLaunchFailure")


def test_tick_stats_warns_on_dropped_shares_once_per_increase():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    eng.miners.dropped = 3
    tick(eng, clock, 1, 1)
    tick(eng, clock, 1, 1)
    eng.miners.dropped = 5
    tick(eng, clock, 1, 1)
    drops = logged(logs, "warn", "dropped \\d+ found share")
    assert [re.search(r"dropped (\d+)", m).group(1) for m in drops] == ["3", "2"]


def test_tick_stats_acceptance_warning_threshold():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    eng.m.shares_accepted.add(18)
    eng.m.shares_rejected.add(1)
    tick(eng, clock, 1, 1)
    assert not logged(logs, "warn", "share acceptance")        # 19 judged: too few to judge
    eng.m.shares_rejected.add(1)
    tick(eng, clock, 1, 1)
    assert logged(logs, "warn", r"share acceptance 90\.0% \(18/20\)")


def test_tick_stats_publishes_latency_quantiles():
    clock = Clock()
    eng, logs = make_engine(clock=clock)
    for v in range(1, 101):
        eng.latency.record(float(v))
    tick(eng, clock, 1, 1)
    assert (eng.m.submit_latency_p50.value(), eng.m.submit_latency_p95.value(),
            eng.m.submit_latency_p99.value()) == (50.0, 95.0, 99.0)
    assert logged(logs, "info", "submit latency p50=50ms p95=95ms p99=99ms")


def test_tick_stats_joules_per_terahash():
    clock = Clock()
    eng, _ = make_engine(Config(bitcoin_address=ADDR, power_watts=1400.0), clock=clock)
    tick(eng, clock, 0, 0)
    tick(eng, clock, 1, 10**12)
    assert eng.m.power_watts.value() == 1400.0
    assert eng.m.joules_per_terahash.value() == pytest.approx(1400.0)


def test_tick_stats_productive_seconds_and_effective_yield():
    clock = Clock()
    eng, _ = make_engine(clock=clock)
    eng.m.arbitration_expected_yield.set(2.0)
    eng.m.uptime.set(20.0)
    tick(eng, clock, 0, 0)
    tick(eng, clock, 10, 10**9)
    tick(eng, clock, 10, 10**9)
    assert eng.m.productive_seconds.value() == 20
    assert eng.est_sats == pytest.approx(40.0)
    assert eng.m.effective_yield.value() == pytest.approx(2.0)


def test_build_stats_includes_hashrate_latency_and_wallet():
    clock = Clock()
    eng, _ = make_engine(clock=clock)
    eng.wallet_fingerprint = "abcd1234"
    eng.latency.record(7.0)
    tick(eng, clock, 0, 0)
    tick(eng, clock, 1, 5 * 10**6)
    st = eng.stats()
    assert st["hashrate"] == 5e6 and st["hashrate_str"] == "5.00 MH/s"
    assert st["wallet"] == "abcd1234" and st["latency_p50_ms"] == 7.0 and st["stalled"] is False
    assert st["algorithm"] == "sha256d"


def test_dashboard_receives_stats_each_tick():
    class Dash:
        def __init__(self):
            self.updates = []

        def update(self, s):
            self.updates.append(s)
    clock = Clock()
    eng, _ = make_engine(clock=clock, dashboard=Dash())
    tick(eng, clock, 1, 1)
    tick(eng, clock, 1, 1)
    assert len(eng.dashboard.updates) == 2 and "hashrate" in eng.dashboard.updates[0]


# ---------------------------------------------------------------------------------------------- arbitration glue

def quote(provider="mining.stratum", dev="gpu-0", net=5.0, fams=(hal.Family.GPU,), at=None):
    q = Quote(provider, dev, Yield(net * 1.1, net, 0.9), list(fams))
    if at is not None:
        q.at = at
    return q


def test_update_stream_inserts_new_stream_with_net_yield():
    streams = {}
    key = R.update_stream(streams, quote(net=7.0))
    assert key == "mining.stratum:gpu-0"
    s = streams[key]
    assert s.id == "mining.stratum" and s.is_bitcoin_mining
    assert s.yield_per_device["gpu-0"].sats_per_second == 7.0  # net, not gross (arbitrate.go:187-195 fix)


def test_update_stream_ai_akash_is_not_bitcoin_mining():
    streams = {}
    R.update_stream(streams, quote(provider="ai.akash", net=100.0))
    assert not streams["ai.akash:gpu-0"].is_bitcoin_mining


def test_update_stream_updates_existing_device():
    streams = {}
    R.update_stream(streams, quote(net=1.0))
    R.update_stream(streams, quote(net=3.0))
    assert len(streams) == 1 and streams["mining.stratum:gpu-0"].yield_per_device["gpu-0"].sats_per_second == 3.0


def test_update_stream_deviceless_quote_sets_default_yield():
    streams = {}
    R.update_stream(streams, quote(dev="", net=4.0))
    s = streams["mining.stratum:"]
    assert not s.yield_per_device and s.default_yield.sats_per_second == 4.0


def test_streams_slice_empty_input():
    assert R.streams_slice({}) == []


def test_streams_slice_deduplicates_and_merges_yield_per_device():
    streams = {}
    R.update_stream(streams, quote(dev="gpu-0", net=1.0))
    R.update_stream(streams, quote(dev="gpu-1", net=2.0))
    R.update_stream(streams, quote(provider="ai.akash", dev="gpu-0", net=3.0))
    out = {s.id: s for s in R.streams_slice(streams)}
    assert set(out) == {"mining.stratum", "ai.akash"}
    assert {d: y.sats_per_second for d, y in out["mining.stratum"].yield_per_device.items()} == \
        {"gpu-0": 1.0, "gpu-1": 2.0}


def test_streams_slice_multi_device_merge_does_not_mutate_input():
    streams = {}
    R.update_stream(streams, quote(dev="gpu-0"))
    R.update_stream(streams, quote(dev="gpu-1"))
    R.streams_slice(streams)
    assert list(streams["mining.stratum:gpu-0"].yield_per_device) == ["gpu-0"]
    assert list(streams["mining.stratum:gpu-1"].yield_per_device) == ["gpu-1"]


def alloc(*assignments, skipped=0):
    return arb.Allocation(list(assignments), sum(a.expected_yield for a in assignments), skipped_device=skipped)


def test_apply_allocation_empty_assignments():
    eng, logs = make_engine()
    eng._apply_allocation(alloc())
    assert not logs and not any(eng.miners.paused.values())


def test_apply_allocation_idle_device_pauses_with_floor_reason():
    eng, logs = make_engine()
    eng._apply_allocation(alloc(arb.Assignment("cpu-0", reason="below min_yield floor")))
    assert eng.miners.paused["cpu-0"] is True
    assert logged(logs, "info", r"cpu-0 idle \(below min_yield floor\)")


def test_apply_allocation_idle_device_default_reason():
    eng, logs = make_engine()
    eng._apply_allocation(alloc(arb.Assignment("cpu-0")))
    assert logged(logs, "info", r"cpu-0 idle \(no compatible stream\)")


def test_apply_allocation_only_pauses_target_device():
    eng, _ = make_engine()
    eng.miners = FakeMiners(["gpu-0", "gpu-1"])
    eng._apply_allocation(alloc(arb.Assignment("gpu-1", "ai.akash", 50.0),
                                arb.Assignment("gpu-0", "mining.stratum", 5.0)))
    assert eng.miners.paused == {"gpu-0": False, "gpu-1": True}


def test_apply_allocation_mining_to_ai():
    eng, logs = make_engine()
    eng._apply_allocation(alloc(arb.Assignment("cpu-0", "ai.akash", 42.0, switched_from_id="mining.stratum")))
    assert eng.miners.paused["cpu-0"] is True
    assert logged(logs, "info", r"cpu-0 → AI inference \(42 sat/s\)")


def test_apply_allocation_ai_to_mining():
    eng, logs = make_engine()
    eng.miners.paused["cpu-0"] = True
    eng._apply_allocation(alloc(arb.Assignment("cpu-0", "mining.stratum", 3.0, switched_from_id="ai.akash")))
    assert eng.miners.paused["cpu-0"] is False
    assert logged(logs, "info", r"cpu-0 → mining \(3 sat/s\)")


def test_apply_allocation_generic_stream_switch_logs():
    eng, logs = make_engine()
    eng._apply_allocation(alloc(arb.Assignment("cpu-0", "mining.other", 9.0, switched_from_id="mining.stratum")))
    assert logged(logs, "info", r"cpu-0 switched to mining.other \(9 sat/s\)")


def test_apply_allocation_no_change_produces_no_log():
    eng, logs = make_engine()
    eng._apply_allocation(alloc(arb.Assignment("cpu-0", "mining.stratum", 3.0)))
    assert not logs and eng.miners.paused["cpu-0"] is False


class FakeProvider:
    def __init__(self):
        self.quotes: asyncio.Queue = asyncio.Queue()

    async def stop(self):
        pass


def arbitration_engine(devices, interval=0.05):
    eng, logs = make_engine(arbitration_interval=interval)
    eng.devices = devices
    eng.miners = FakeMiners([d.identity().id for d in devices])
    prov = FakeProvider()
    eng._providers = [prov]
    return eng, logs, prov


def test_arbitration_loop_quote_updates_streams_and_publishes_gauges():
    async def go():
        eng, logs, prov = arbitration_engine([gpu_device(0)])
        await prov.quotes.put(quote(dev="gpu-0", net=5.0))
        await run_pump_until(eng._arbitration_loop(), lambda: eng.m.active_streams.value() == 1)
        assert eng.m.arbitration_expected_yield.value() == pytest.approx(4.5)  # 5 sat/s x confidence 0.9
        assert eng.activity == {"mining.stratum": pytest.approx(4.5)}
        assert eng.m.devices_idle.value() == 0 and eng.m.arbitration_foregone.value() == 0
    asyncio.run(go())


def test_arbitration_loop_publishes_devices_idle_and_logs_transition():
    async def go():
        eng, logs, prov = arbitration_engine([gpu_device(0), cpu_device(0)])
        await prov.quotes.put(quote(dev="gpu-0", net=5.0, fams=(hal.Family.GPU,)))
        await run_pump_until(eng._arbitration_loop(), lambda: eng.m.devices_idle.value() == 1)
        assert eng.miners.paused["cpu-0"] is True and eng.miners.paused["gpu-0"] is False
        assert logged(logs, "info", r"1 device\(s\) now idle")
    asyncio.run(go())


def test_arbitration_loop_prunes_stale_streams():
    async def go():
        eng, logs, prov = arbitration_engine([gpu_device(0)])
        import time
        await prov.quotes.put(quote(dev="gpu-0", net=5.0, at=time.time() - R.STREAM_STALE_TIMEOUT - 5))
        await run_pump_until(eng._arbitration_loop(),
                             lambda: logged(logs, "info", "stream 'mining.stratum:gpu-0' expired"))
        assert eng.m.active_streams.value() == 0
    asyncio.run(go())


def test_arbitration_loop_never_assigns_incompatible_family():
    async def go():
        eng, logs, prov = arbitration_engine([cpu_device(0)])
        await prov.quotes.put(quote(provider="ai.akash", dev="", net=500.0, fams=(hal.Family.GPU,)))
        await run_pump_until(eng._arbitration_loop(), lambda: eng.m.active_streams.value() == 1)
        await asyncio.sleep(0.1)
        assert eng.miners.paused["cpu-0"] is True and eng.m.devices_idle.value() == 1
    asyncio.run(go())


def test_next_quote_merges_multiple_providers():
    async def go():
        eng, _ = make_engine()
        a, b = FakeProvider(), FakeProvider()
        eng._providers = [a, b]
        await b.quotes.put(quote(provider="ai.akash"))
        got = await asyncio.wait_for(eng._next_quote(), 1)
        assert [q.provider_id for q in got] == ["ai.akash"]
        await a.quotes.put(quote())
        got = await asyncio.wait_for(eng._next_quote(), 1)
        assert [q.provider_id for q in got] == ["mining.stratum"]
    asyncio.run(go())


# ---------------------------------------------------------------------------------------------- reconnect loop

class SessionScript:
    """Replaces Engine._run_session: per attempt, 'fail' raises, 'ok' connects then ends, 'fatal' raises fatal."""

    def __init__(self, script):
        self.script = list(script)
        self.calls: list[tuple[str, str]] = []

    async def __call__(self, url, user, pc, on_connected):
        self.calls.append((url, user))
        step = self.script.pop(0) if self.script else "fail"
        if step == "fatal":
            raise FatalPoolError("engine: SetupConnectionError: unsupported-protocol")
        if step == "ok":
            on_connected()
            raise ConnectionError("engine: pool closed connection")
        raise ConnectionRefusedError(f"dial {url}: refused")


def reconnect_engine(monkeypatch, cfg, script, attempts):
    sleeps = []

    async def fake_sleep(s):
        sleeps.append(s)
    monkeypatch.setattr(R.asyncio, "sleep", fake_sleep)
    ready = []
    eng, logs = make_engine(cfg, max_reconnect_attempts=attempts, on_ready=ready.append)
    sc = SessionScript(script)
    eng._run_session = sc
    return eng, logs, sc, sleeps, ready


def run_reconnect(eng):
    async def go():
        with pytest.raises((RuntimeError, FatalPoolError)) as ei:
            await eng._reconnect_loop()
        return ei.value
    return asyncio.run(go())


def test_reconnect_pool_failover_is_immediate_then_backoff(monkeypatch):
    cfg = Config(bitcoin_address=ADDR, pools=[PoolConfig(url=f"stratum+v2://p{i}:1") for i in range(3)])
    eng, logs, sc, sleeps, _ = reconnect_engine(monkeypatch, cfg, [], 7)
    err = run_reconnect(eng)
    assert "exceeded 7 reconnect attempts" in str(err)
    assert [u for u, _ in sc.calls] == [f"stratum+v2://p{i}:1" for i in (0, 1, 2, 0, 1, 2, 0)]
    assert sleeps == [1.0, 2.0]                           # one backoff per full cycle
    assert logged(logs, "warn", "failing over to next pool")
    assert logged(logs, "warn", "all 3 pools failed; backing off 1s")


def test_reconnect_backoff_doubles_and_caps_at_64s(monkeypatch):
    eng, logs, sc, sleeps, _ = reconnect_engine(monkeypatch, Config(bitcoin_address=ADDR), [], 10)
    run_reconnect(eng)
    assert sleeps == [1.0, 2.0, 4.0, 8.0, 16.0, 32.0, 64.0, 64.0, 64.0, 64.0]  # one per failed attempt
    assert logged(logs, "warn", "reconnecting in 64s")


def test_reconnect_address_failover_only_when_address_never_connected(monkeypatch):
    cfg = Config(bitcoin_address=ADDR, bitcoin_addresses=[ADDR2])
    eng, logs, sc, sleeps, _ = reconnect_engine(monkeypatch, cfg, ["fail", "fail", "fail"], 3)
    run_reconnect(eng)
    assert [u.split(".")[0] for _, u in sc.calls] == [ADDR, ADDR2, ADDR]
    assert sleeps == [1.0]                                # backoff only after every address failed
    assert logged(logs, "warn", r"payout address bc1qar…5mdq \(1/2\) could not establish a session")
    assert logged(logs, "warn", "none of the 2 configured payout addresses could connect")


def test_reconnect_no_address_failover_after_a_successful_session(monkeypatch):
    cfg = Config(bitcoin_address=ADDR, bitcoin_addresses=[ADDR2])
    eng, logs, sc, sleeps, ready = reconnect_engine(monkeypatch, cfg, ["ok", "fail", "fail"], 3)
    run_reconnect(eng)
    assert [u.split(".")[0] for _, u in sc.calls] == [ADDR, ADDR, ADDR]   # an outage never redirects earnings
    assert ready[:2] == [True, False]


def test_reconnect_fatal_error_stops_retries(monkeypatch):
    cfg = Config(bitcoin_address=ADDR, pools=[PoolConfig(url="stratum+v2://a:1"), PoolConfig(url="stratum+v2://b:1")])
    eng, logs, sc, sleeps, _ = reconnect_engine(monkeypatch, cfg, ["fatal"], 10)
    err = run_reconnect(eng)
    assert isinstance(err, FatalPoolError) and len(sc.calls) == 1 and not sleeps
    assert eng.m.pool_connect_failures.value() == 1


def test_reconnect_metrics_and_session_user(monkeypatch):
    cfg = Config(bitcoin_address=ADDR, pools=[PoolConfig(url="stratum+v2://a:1", user="acct.rig"),
                                               PoolConfig(url="stratum+v2://b:1")])
    cfg.workers.name = "w7"
    eng, logs, sc, sleeps, _ = reconnect_engine(monkeypatch, cfg, ["fail", "ok"], 2)
    run_reconnect(eng)
    assert sc.calls == [("stratum+v2://a:1", "acct.rig"), ("stratum+v2://b:1", ADDR + ".w7")]
    assert eng.m.pool_connect_attempts.value() == 2 and eng.m.pool_connect_failures.value() == 2
    assert eng.m.pool_active_index.value() == 1 and eng.m.pool_connection_state.value() == 0
    assert 'otedama_payout_info{address="bc1qar…5mdq"} 1' in eng.registry.render()
    assert logged(logs, "info", r"connecting to stratum\+v2://b:1 \(attempt 2, pool 2/2\)")


def test_reconnect_on_ready_tracks_session(monkeypatch):
    eng, logs, sc, sleeps, ready = reconnect_engine(monkeypatch, Config(bitcoin_address=ADDR), ["ok", "ok"], 2)
    run_reconnect(eng)
    assert ready == [True, False, True, False]


# ---------------------------------------------------------------------------------------------- run()

def test_run_without_capable_devices_fails_fast():
    async def go():
        eng = Engine(Options(config=Config(bitcoin_address=ADDR), devices=[], rate_fetcher=FakeFetcher(),
                             fetch_rates=False))
        with pytest.raises(RuntimeError, match="no device can mine sha256d"):
            await eng.run()
    asyncio.run(go())


def test_run_publishes_start_time_and_power_cost():
    async def go():
        cfg = Config(bitcoin_address=ADDR, power_watts=2000.0, electricity_price_per_kwh=0.10)
        eng = Engine(Options(config=cfg, devices=[], rate_fetcher=FakeFetcher(), fetch_rates=False))
        with pytest.raises(RuntimeError):
            await eng.run()
        assert eng.m.power_cost_usd_per_hour.value() == pytest.approx(0.2)
        assert eng.m.start_time.value() == pytest.approx(eng.start_time)
    asyncio.run(go())


def test_run_reports_not_ready_on_exit():
    ready = []

    async def go():
        eng = Engine(Options(config=Config(bitcoin_address=ADDR), devices=[], rate_fetcher=FakeFetcher(),
                             fetch_rates=False, on_ready=ready.append))
        with pytest.raises(RuntimeError):
            await eng.run()
    asyncio.run(go())
    assert ready == [False]


def test_detect_devices_honours_gpu_selection(monkeypatch):
    devs = [cpu_device(0), gpu_device(0), gpu_device(1)]

    class Det:
        def __init__(self, *a, **k):
            pass

        def detect(self):
            return list(devs)
    monkeypatch.setattr(R.hal, "Detector", Det)
    for sel, want in [("", ["cpu-0", "gpu-0", "gpu-1"]), ("all", ["cpu-0", "gpu-0", "gpu-1"]),
                      ("none", ["cpu-0"]), ("1", ["cpu-0", "gpu-1"]), ("0, 1", ["cpu-0", "gpu-0", "gpu-1"])]:
        cfg = Config(bitcoin_address=ADDR)
        cfg.mining.gpus = sel
        eng, _ = make_engine(cfg)
        assert [d.identity().id for d in eng._detect_devices()] == want, sel


def test_tick_stats_publishes_device_busy_ratio_and_launches():
    class Miners(FakeMiners):
        def __init__(self):
            super().__init__(["gpu-0", "cpu-0", "rank1"])
            self.busy = {"gpu-0": 0.0, "cpu-0": 0.0}
            self.launches = 0

        def device_stats(self):
            return {"gpu-0": {"faulted": False, "busy_seconds": self.busy["gpu-0"], "launches": self.launches},
                    "cpu-0": {"faulted": False, "busy_seconds": self.busy["cpu-0"], "launches": 0, "threads": 4},
                    "rank1": {"faulted": False, "hashes": 5}}
    clock = Clock()
    eng, _ = make_engine(clock=clock)
    eng.miners = Miners()
    tick(eng, clock, 1, 1)
    eng.miners.busy = {"gpu-0": 9.5, "cpu-0": 20.0}
    eng.miners.launches = 340
    tick(eng, clock, 10, 1)
    text = eng.registry.render()
    assert 'otedama_device_busy_ratio{device="gpu-0"} 0.95' in text
    assert 'otedama_device_busy_ratio{device="cpu-0"} 0.5' in text       # 20 thread-seconds / (10 s x 4 threads)
    assert 'otedama_device_kernel_launches_total{device="gpu-0"} 340' in text
    assert 'device="rank1"' not in text.split("otedama_device_busy_ratio")[-1].split("\n")[0]


def test_tick_stats_publishes_node_collective_tick():
    class Link:
        world = 8
        comm = SimpleNamespace(collectives=12)

        def tick_quantile(self, q):
            return 0.0004 if q == 0.5 else 0.002

    clock = Clock()
    eng, _ = make_engine(clock=clock)
    assert eng.m.node_ranks.value() == 1
    eng.miners.link = Link()
    tick(eng, clock, 1, 1)
    assert eng.m.node_ranks.value() == 8 and eng.m.node_collective_seconds.value() == pytest.approx(0.0004)
    assert eng.m.node_collective_p99.value() == pytest.approx(0.002) and eng.m.node_collectives.value() == 12
