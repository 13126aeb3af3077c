"""Pool under load (BASELINE config 5 shape, tools/bench_pool.py): SHA-256d, scrypt and X11 pools each take a
flood of SV2 submits from several miners. scrypt shares are hashed on the pool's native thread pool,
off the event loop. Every share is valid at the clamped minimum difficulty, so any rejection is a bug."""
import asyncio
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_pool", ROOT / "tools" / "bench_pool.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_mixed_pool_load():
    mod = _bench()

    async def both():
        return await asyncio.wait_for(asyncio.gather(mod._run_pool("sha256d", 2, 1.0, 2),
                                                     mod._run_pool("scrypt", 2, 1.0, 2),
                                                     mod._run_pool("x11", 2, 1.0, 2)), 60)

    res = asyncio.run(both())
    for r in res:
        assert r["accepted"] > 20 and r["rejected"] == 0, r
        assert r["client_verdicts"] == {"ok": r["accepted"]}, r
        assert r["ack_latency_ms"]["p50"] > 0


def test_share_target_clamps_low_difficulty():
    from otedama_amd.models.header import hash_to_int
    from otedama_amd.pool.server import PoolOptions, PoolServer

    p = PoolServer(PoolOptions(algorithm="scrypt"))
    assert p.share_target(1e-12) == b"\xff" * 32          # would overflow 256 bits
    assert hash_to_int(p.share_target(1.0)) == 0xFFFF << 224
