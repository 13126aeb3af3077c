"""End-to-end slice on the CPU device: engine -> local validating pool (SV2 and
V1) -> accepted shares -> /metrics. Mirrors engine/integration_test.go
(HandshakeSucceeds, ReconnectsOnPoolFailure) with real share validation."""
import asyncio
import socket

import pytest

from otedama_amd import hal
from otedama_amd.config import Config, MiningConfig, PoolConfig
from otedama_amd.engine.run import Engine, Options, curtail_decision, mask_addr, session_user
from otedama_amd.metrics import Registry
from otedama_amd.pool.server import PoolOptions, PoolServer
from otedama_amd.provider import StaticRateSource

ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


def _cpu_devices(threads=2):
    return [hal.SimpleDevice(hal.Identity("cpu-0", hal.Family.CPU, "test", "cpu"),
                             hal.Capabilities(sha256d=True, general_compute=True), threads=threads)]


async def _run_engine_against_pool(scheme: str, seconds: float = 4.0):
    pool = PoolServer(PoolOptions(initial_difficulty=1e-3, payout_address=ADDR, retarget_seconds=5))
    await pool.start()
    addr = pool.addr_sv2 if scheme == "v2" else pool.addr_v1
    url = f"stratum+{'v2' if scheme == 'v2' else 'tcp'}://{addr}"
    cfg = Config(bitcoin_address=ADDR, pools=[PoolConfig(url=url)], mining=MiningConfig(cpu_threads=2))
    reg = Registry()
    ready = []
    eng = Engine(Options(config=cfg, metrics=reg, devices=_cpu_devices(), rate_fetcher=StaticRateSource(95000),
                         stats_interval=0.5, on_ready=ready.append, logger=lambda lvl, msg: None))
    task = asyncio.ensure_future(eng.run())
    await asyncio.sleep(seconds)
    task.cancel()
    try:
        await task
    except asyncio.CancelledError:
        pass
    await pool.stop()
    return eng, pool, reg, ready


@pytest.mark.parametrize("scheme", ["v2", "v1"])
def test_engine_mines_accepted_shares(scheme):
    eng, pool, reg, ready = asyncio.run(_run_engine_against_pool(scheme))
    assert True in ready and ready[-1] is False
    assert pool.accepted >= 1, (pool.stats(), eng.stats())
    assert eng.m.shares_accepted.value() >= 1
    assert eng.m.shares_rejected.value() <= 1
    text = reg.render()
    assert 'otedama_shares_total{status="accepted"}' in text
    assert "otedama_hashrate_hashes_per_second" in text
    assert eng.current_hashrate > 0
    assert eng.latency.quantile(0.5) > 0
    dbg = eng.debug_stats()                      # GET /debug/stats payload
    cpu = dbg["devices"]["cpu-0"]
    assert cpu["hashes"] > 0 and cpu["shares"] >= 1 and not cpu["faulted"] and not cpu["retired"]
    assert (cpu["stripe_start"], cpu["stripe_stride"]) == (0, 1) and 0 < cpu["busy_ratio"] <= 2.5
    assert dbg["epoch"] >= 1 and dbg["node"] is None and dbg["process"]["threads"] >= 1
    assert 'otedama_devices_active' in text


def test_engine_reconnects_on_pool_failure():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cfg = Config(bitcoin_address=ADDR, pools=[PoolConfig(url=f"stratum+v2://127.0.0.1:{port}")])

    async def go():
        eng = Engine(Options(config=cfg, devices=_cpu_devices(1), rate_fetcher=StaticRateSource(95000),
                             max_reconnect_attempts=2))
        with pytest.raises(RuntimeError, match="exceeded 2 reconnect attempts"):
            await asyncio.wait_for(eng.run(), 20)
        return eng

    eng = asyncio.run(go())
    assert eng.m.pool_connect_attempts.value() == 2
    assert eng.m.pool_connect_failures.value() == 2


def test_curtail_decision_table():
    assert curtail_decision(False, 50000, True, 60000) == (True, True)
    assert curtail_decision(True, 70000, True, 60000) == (False, True)
    assert curtail_decision(False, 50000, False, 60000) == (False, False)  # stale price never curtails
    assert curtail_decision(True, 0, True, 60000) == (True, False)
    assert curtail_decision(False, 50000, True, 0) == (False, False)


def test_helpers():
    assert session_user("", "bc1qxyz", "rig") == "bc1qxyz.rig"
    assert session_user("acct", "bc1qxyz", "rig") == "acct"
    assert mask_addr(ADDR) == "bc1qar…5mdq"
    assert mask_addr("short") == "short"
