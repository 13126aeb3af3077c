"""Yield providers: mining-yield formula, simulated Akash quotes, polling loop, drop-oldest queue, lifecycle.

Mirrors internal/provider/provider_test.go (TestMiningProvider_*, TestAkashProvider_*, TestPollingLoop_*,
TestSatsPerSecond_*, TestYield_Effective, TestStaticRateSource).
"""
from __future__ import annotations

import asyncio

import pytest

from otedama_amd import provider as P
from otedama_amd.hal import Capabilities, Family, Identity


class Dev:
    def __init__(self, did, fam, caps):
        self._id, self._caps = Identity(did, fam, "amd", "x"), caps

    def identity(self):
        return self._id

    def capabilities(self):
        return self._caps


GPU = Dev("gpu-0", Family.GPU, Capabilities(sha256d=True, general_compute=True, scrypt=True, x11=True))
GPU_NOCOMPUTE = Dev("gpu-9", Family.GPU, Capabilities(sha256d=True))
CPU = Dev("cpu-0", Family.CPU, Capabilities(sha256d=True, general_compute=True))
ASIC = Dev("asic-0", Family.ASIC, Capabilities(sha256d=True))
NOSHA = Dev("gpu-1", Family.GPU, Capabilities(general_compute=True))


class Rates:
    def __init__(self, rate=95_000.0, fresh=True):
        self.rate, self.fresh = rate, fresh

    def btc_usd_rate(self):
        return self.rate, self.fresh


def drain(q):
    out = []
    while not q.empty():
        out.append(q.get_nowait())
    return out


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 10))


# ------------------------------------------------------------------ helpers
@pytest.mark.parametrize("gross,net,conf,want", [(10, 9, 0.5, 4.5), (10, 0, 1, 0.0), (10, 9, 0, 0.0), (0, 5, 1, 5.0)])
def test_yield_effective_uses_net(gross, net, conf, want):
    assert P.Yield(gross, net, conf).effective() == want


@pytest.mark.parametrize("usd,btc,want", [(0.45, 90_000, 0.45 / 90_000 * 1e8 / 3600), (1, 0, 0.0), (-1, 90_000, 0.0),
                                          (0, 90_000, 0.0)])
def test_sats_per_second(usd, btc, want):
    assert P.sats_per_second(usd, btc) == pytest.approx(want)


def test_static_rate_source():
    assert P.StaticRateSource(12345.0).btc_usd_rate() == (12345.0, True)


def test_constants_match_the_reference():
    assert P.MIN_QUOTE_INTERVAL == 30 and P.NETWORK_HASHRATE == 1e21
    assert (P.BLOCK_REWARD_BTC, P.BLOCK_TIME_SEC, P.FALLBACK_BTC_USD) == (3.125, 600.0, 95_000.0)
    assert P.DEFAULT_HASHRATES == {Family.ASIC: 100e12, Family.GPU: 1.5e9, Family.CPU: 10e6}


# ------------------------------------------------------------------ mining provider
def _mining_sats(h):
    return h / 1e21 * 3.125 / 600 * 1e8


def test_mining_provider_id_and_name():
    m = P.MiningProvider("stratum+v2://pool:3336", Rates())
    assert m.id == "mining.stratum" and "pool:3336" in m.name()


def test_mining_quote_per_capable_device_with_static_fallback():
    m = P.MiningProvider("u", Rates())
    m.prepare([GPU, CPU, ASIC, NOSHA])
    m.publish()
    qs = {q.device_id: q for q in drain(m.quotes)}
    assert set(qs) == {"gpu-0", "cpu-0", "asic-0"}
    assert qs["asic-0"].yield_.sats_per_second == pytest.approx(_mining_sats(100e12))
    assert qs["gpu-0"].yield_.sats_per_second == pytest.approx(_mining_sats(1.5e9))
    for q in qs.values():
        assert q.provider_id == "mining.stratum"
        assert q.yield_.net_sats_per_second == pytest.approx(q.yield_.sats_per_second * 0.99)  # 1% pool fee
        assert q.accepted_families == [Family.ASIC, Family.GPU, Family.CPU] and q.yield_.confidence == 0.95


def test_mining_uses_the_live_hashrate_and_falls_back_on_zero_or_unknown():
    live = {"gpu-0": 18.8e9, "cpu-0": 0.0}
    m = P.MiningProvider("u", Rates(), hashrate_func=lambda d: live.get(d, 0.0))
    m.prepare([GPU, CPU, ASIC])
    m.publish()
    qs = {q.device_id: q.yield_.sats_per_second for q in drain(m.quotes)}
    assert qs["gpu-0"] == pytest.approx(_mining_sats(18.8e9))
    assert qs["cpu-0"] == pytest.approx(_mining_sats(10e6))
    assert qs["asic-0"] == pytest.approx(_mining_sats(100e12))


@pytest.mark.parametrize("algo,ids", [("sha256d", {"gpu-0", "cpu-0"}), ("scrypt", {"gpu-0"}), ("x11", {"gpu-0"})])
def test_mining_respects_the_configured_algorithm(algo, ids):
    m = P.MiningProvider("u", Rates(), algorithm=algo)
    m.prepare([GPU, CPU])
    m.publish()
    assert {q.device_id for q in drain(m.quotes)} == ids


@pytest.mark.parametrize("rate,fresh,conf", [(95_000, True, 0.95), (95_000, False, 0.7), (0, False, 0.7)])
def test_mining_confidence_tracks_rate_freshness(rate, fresh, conf):
    m = P.MiningProvider("u", Rates(rate, fresh))
    m.prepare([GPU])
    m.publish()
    (q,) = drain(m.quotes)
    assert q.yield_.confidence == conf and q.yield_.sats_per_second > 0


def test_mining_queue_drops_the_oldest_when_full():
    m = P.MiningProvider("u", Rates(), hashrate_func=lambda d: 1e9)
    m.prepare([GPU])
    for i in range(m.queue_size + 4):
        m.hashrate_func = lambda d, i=i: 1e9 * (i + 1)
        m.publish()
    qs = drain(m.quotes)
    assert len(qs) == 16
    assert qs[-1].yield_.sats_per_second == pytest.approx(_mining_sats(1e9 * (m.queue_size + 4)))
    assert qs[0].yield_.sats_per_second == pytest.approx(_mining_sats(1e9 * 5))


# ------------------------------------------------------------------ akash provider
def test_akash_identity_discloses_simulation():
    a = P.AkashProvider(Rates())
    assert a.id == "ai.akash" and "Akash" in a.name() and "simulated" in a.name()


def test_akash_only_gpus_with_general_compute():
    a = P.AkashProvider(Rates())
    a.prepare([GPU, GPU_NOCOMPUTE, CPU, ASIC])
    assert [d.identity().id for d in a.devices] == ["gpu-0"]
    a.publish()
    (q,) = drain(a.quotes)
    assert q.accepted_families == [Family.GPU]


def test_akash_without_gpus_emits_a_zero_yield_quote():
    a = P.AkashProvider(Rates())
    a.prepare([CPU])
    a.publish()
    (q,) = drain(a.quotes)
    assert q.device_id == "" and q.yield_.effective() == 0


def test_akash_price_is_the_midpoint_minus_20_percent():
    a = P.AkashProvider(Rates(100_000))
    a.prepare([GPU])
    a.publish()
    (q,) = drain(a.quotes)
    assert q.yield_.sats_per_second == pytest.approx(P.sats_per_second(0.45, 100_000))
    assert q.yield_.net_sats_per_second == pytest.approx(P.sats_per_second(0.36, 100_000))
    lo, hi = P.sats_per_second(0.30, 100_000), P.sats_per_second(0.60, 100_000)
    assert lo <= q.yield_.sats_per_second <= hi


@pytest.mark.parametrize("fresh,conf", [(True, 0.85), (False, 0.6)])
def test_akash_confidence(fresh, conf):
    a = P.AkashProvider(Rates(95_000, fresh))
    a.prepare([GPU])
    a.publish()
    assert drain(a.quotes)[0].yield_.confidence == conf


def test_akash_zero_rate_uses_the_fallback():
    a = P.AkashProvider(Rates(0, False))
    a.prepare([GPU])
    a.publish()
    assert drain(a.quotes)[0].yield_.sats_per_second == pytest.approx(P.sats_per_second(0.45, 95_000))


def test_akash_beats_cpu_mining():
    a, m = P.AkashProvider(Rates()), P.MiningProvider("u", Rates())
    a.prepare([GPU])
    m.prepare([CPU])
    a.publish()
    m.publish()
    assert drain(a.quotes)[0].yield_.effective() > drain(m.quotes)[0].yield_.effective()


def test_akash_queue_holds_32():
    a = P.AkashProvider(Rates())
    a.prepare([GPU])
    for _ in range(40):
        a.publish()
    assert a.quotes.qsize() == 32


# ------------------------------------------------------------------ lifecycle / polling
@pytest.mark.parametrize("cls,args", [(P.MiningProvider, ("u", Rates())), (P.AkashProvider, (Rates(),))])
def test_lifecycle(cls, args):
    async def go():
        p = cls(*args, interval=0.02)
        await p.stop()  # stop without start is safe
        p.start([GPU])
        with pytest.raises(RuntimeError, match="already started"):
            p.start([GPU])
        await asyncio.sleep(0.09)
        assert p.quotes.qsize() >= 3  # publish immediately, then every interval
        await p.stop()
        assert p._task is None and p.quotes.qsize() == 0  # state cleared for a restart
        p.start([GPU])
        await asyncio.sleep(0.01)
        assert p.quotes.qsize() >= 1
        await p.stop()
    run(go())


def test_cancelling_the_parent_task_ends_the_loop():
    async def go():
        p = P.MiningProvider("u", Rates(), interval=0.01)
        p.start([GPU])
        await asyncio.sleep(0.03)
        p._task.cancel()
        await asyncio.sleep(0.01)
        assert p._task.done()
    run(go())


def test_base_publish_is_abstract():
    with pytest.raises(NotImplementedError):
        P.PollingProvider(1).publish()
