"""Long-lived dedupe state stays bounded.

* Engine submitted-share keys: the reference caps its unacked-submit map at 1024 and drops the oldest half
  (internal/engine/run.go:720-726,944-957).
* Pool credited headers: kept per live job (16 retained), a job is retired at MAX_SHARES_PER_JOB.
* otedama_pool_accepted_work_total sums the real (fractional) share difficulty.
"""
import asyncio

import pytest

from otedama_amd.metrics import Registry
from otedama_amd.pool import server as S
from otedama_amd.utils.bounded import BoundedSet

from test_engine_suite import FakeSession, make_engine, share
from test_pool_units import ADDR


def test_bounded_set_halves_at_the_cap():
    b = BoundedSet(1024)
    peak = 0
    for i in range(100_000):
        b.add(i)
        peak = max(peak, len(b))
        assert i in b  # the newest key is always retained
    assert peak <= 1024
    assert 99_999 in b and 0 not in b and b.evicted == 100_000 - len(b)
    b.add(99_999)  # re-adding is a no-op
    assert len(b) <= 1024
    assert BoundedSet(4, [1, 2]) == {1, 2}


def test_engine_submit_keys_stay_under_the_cap_for_1e5_shares():
    eng, _ = make_engine()
    sess = FakeSession()
    eng._valid_jobs = {"j1"}
    n = 100_000

    async def go():
        pump = asyncio.ensure_future(eng._share_pump(sess))
        peak = 0
        for base in range(0, n, 4096):
            eng.miners.queue.extend(share(nonce=i) for i in range(base, min(base + 4096, n)))
            while eng.miners.queue:
                await asyncio.sleep(0)
            peak = max(peak, len(eng._submitted))
        while eng._submit_tasks:
            await asyncio.sleep(0)
        pump.cancel()
        return peak

    peak = asyncio.run(go())
    assert peak <= 1024 and len(eng._submitted) <= 1024
    assert len(sess.submitted) == n  # every distinct share still went out exactly once
    assert len({s.nonce for s in sess.submitted}) == n


def test_pool_seen_headers_stay_bounded(monkeypatch):
    monkeypatch.setattr(S, "MAX_SHARES_PER_JOB", 1000)
    p = S.PoolServer(S.PoolOptions(algorithm="sha256d", payout_address=ADDR, initial_difficulty=1e-12,
                                   min_difficulty=1e-12, listen_v1="", retarget_seconds=1e9))
    p.new_block()
    w = p.new_worker("rig", S.BIP320_MASK)
    en = bytes(S.EN1_SIZE + S.EN2_SIZE)
    peak = acc = 0
    n = 100_000
    for nonce in range(n):
        job = next(reversed(p.jobs.values()))
        acc += p.validate(w, job.job_id, en, job.ntime, nonce, job.version).accepted
        if nonce % 997 == 0:
            peak = max(peak, sum(len(s) for s in p._seen.values()))
    assert acc == n, p.reject_reasons  # diff 1e-12: the target clamps to 2^256-1
    assert peak <= 16 * 1000 and sum(len(s) for s in p._seen.values()) <= 16 * 1000
    assert len(p.jobs) <= 16 and set(p._seen) == set(p.jobs)
    # a header credited under a live job is still a duplicate
    job = next(reversed(p.jobs.values()))
    nonce = n + 1
    assert p.validate(w, job.job_id, en, job.ntime, nonce, job.version).accepted
    assert p.validate(w, job.job_id, en, job.ntime, nonce, job.version).reason == "duplicate-share"


@pytest.mark.parametrize("diff", [2.0 ** -20, 3 * 2.0 ** -22, 0.1 * 2.0 ** -16])
def test_accepted_work_counts_fractional_difficulty(diff):
    reg = Registry()
    p = S.PoolServer(S.PoolOptions(algorithm="sha256d", payout_address=ADDR, initial_difficulty=diff,
                                   min_difficulty=1e-12, listen_v1="", retarget_seconds=1e9), registry=reg)
    p.new_block()
    w = p.new_worker("rig", S.BIP320_MASK)
    w.vd.difficulty = diff
    en = bytes(S.EN1_SIZE + S.EN2_SIZE)
    job = next(iter(p.jobs.values()))
    got, nonce = 0, 0
    while got < 4 and nonce < 1 << 18:  # p(share) ~ 2^-32 / diff >= 2^-13
        got += p.validate(w, job.job_id, en, job.ntime, nonce, job.version).accepted
        nonce += 1
    assert got == 4
    assert p.m_work.value() == pytest.approx(4 * diff, rel=1e-12)
    import io

    buf = io.StringIO()
    reg.write_text(buf)
    line = [ln for ln in buf.getvalue().splitlines() if ln.startswith("otedama_pool_accepted_work_total{")][0]
    assert float(line.rsplit(" ", 1)[1]) == pytest.approx(4 * diff, rel=1e-6)
