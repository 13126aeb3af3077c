"""Loopback pool server <-> V1 / V2 client sessions, with real share validation
(mirrors engine/integration_test.go's mock pool, but the pool re-hashes every
share — the reference fakes never do)."""
import asyncio
import struct

import pytest

from otedama_amd.models.header import hash_to_int, sha256d
from otedama_amd.ops.native import require_native
from otedama_amd.pool.server import PoolOptions, PoolServer
from otedama_amd.poolproto import Credentials, ShareSubmission
from otedama_amd.poolproto.stratumv1 import V1Dialer
from otedama_amd.poolproto.stratumv2 import V2Dialer

N = require_native()
ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


def _find_share(job, max_variants=64):
    """Mine a share for a poolproto Job on the CPU through the native runtime."""
    t = job.template()
    for v in range(max_variants):
        hdr, ver, nt, en2 = N.variant_header(t, v)
        hits = N.cpu_scan_sha256d(hdr, t["target"], 0, 1 << 20)
        if hits:
            return hits[0], ver, nt, en2, hdr
    raise AssertionError("no share found")


async def _with_pool(fn, **kw):
    opts = PoolOptions(initial_difficulty=kw.pop("diff", 2e-5), payout_address=ADDR, **kw)
    pool = PoolServer(opts)
    await pool.start()
    try:
        return await fn(pool)
    finally:
        await pool.stop()


@pytest.mark.parametrize("rolling", [True, False])
def test_sv2_share_accept_duplicate_lowdiff(rolling):
    async def body(pool):
        s = await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", Credentials(user=ADDR, version_rolling=rolling))
        job = await asyncio.wait_for(s.jobs.get(), 5)
        assert job is not None and job.merkle_root is not None
        assert (job.version_mask != 0) == rolling
        nonce, ver, nt, _en2, hdr = _find_share(job)
        h = sha256d(hdr[:76] + struct.pack("<I", nonce))
        assert hash_to_int(h) <= hash_to_int(job.target)
        r = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver))
        assert r.accepted, r
        r2 = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver))
        assert not r2.accepted and "duplicate" in r2.reason
        # a nonce that fails the target
        bad = next(n for n in range(1000) if hash_to_int(sha256d(hdr[:76] + struct.pack("<I", n)))
                   > hash_to_int(job.target))
        r3 = await s.submit(ShareSubmission(job.job_id, bad, nt, ver))
        assert not r3.accepted and "difficulty" in r3.reason
        r4 = await s.submit(ShareSubmission("65535", nonce, nt, ver))
        assert not r4.accepted and "stale" in r4.reason
        assert pool.accepted == 1 and pool.rejected == 3
        await s.close()

    asyncio.run(_with_pool(body))


def test_v1_coinbase_extranonce2_share():
    async def body(pool):
        s = await V1Dialer().dial(f"stratum+tcp://{pool.addr_v1}", Credentials(user=ADDR + ".rig1"))
        job = await asyncio.wait_for(s.jobs.get(), 5)
        assert job.coinb1 and job.coinb2 and len(job.merkle_branches) == 3  # 7 fake txs + coinbase
        assert job.extranonce2_size == 4 and len(job.extranonce1) == 4
        nonce, ver, nt, en2, hdr = _find_share(job)
        # the pool rebuilds the same header from coinb1 | en1 | en2 | coinb2
        cb = job.coinb1 + job.extranonce1 + en2.to_bytes(4, "little") + job.coinb2
        root = sha256d(cb)
        for b in job.merkle_branches:
            root = sha256d(root + b)
        assert hdr[36:68] == root
        r = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver, en2.to_bytes(4, "little")))
        assert r.accepted, r
        r2 = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver, en2.to_bytes(4, "little")))
        assert not r2.accepted and "duplicate" in r2.reason
        await s.close()

    asyncio.run(_with_pool(body))


def test_v1_version_rolling_share():
    async def body(pool):
        s = await V1Dialer().dial(f"stratum+tcp://{pool.addr_v1}", Credentials(user=ADDR))
        job = await asyncio.wait_for(s.jobs.get(), 5)
        assert job.version_mask == 0x1FFFE000
        t = dict(job.template())
        # force version rolling (no extranonce2 rolling): fixed en2 = 0 via a 1-variant coinbase space
        for v in range(1, 200):
            hdr, ver, nt, en2 = N.variant_header({**t, "extranonce2_size": 0}, v)
            if ver == job.version:
                continue
            # pool builds coinbase with en2 = 4 zero bytes; make the header match
            cb = job.coinb1 + job.extranonce1 + bytes(4) + job.coinb2
            root = sha256d(cb)
            for b in job.merkle_branches:
                root = sha256d(root + b)
            hdr = hdr[:36] + root + hdr[68:]
            hits = N.cpu_scan_sha256d(hdr, t["target"], 0, 1 << 20)
            if hits:
                r = await s.submit(ShareSubmission(job.job_id, hits[0], nt, ver, bytes(4)))
                assert r.accepted, r
                break
        else:
            raise AssertionError("no rolled share found")
        await s.close()

    asyncio.run(_with_pool(body))


def test_vardiff_retarget_sends_set_target():
    async def body(pool):
        s = await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", Credentials(user=ADDR))
        job = await asyncio.wait_for(s.jobs.get(), 5)
        t0 = s.share_target
        accepted = 0
        for v in range(40):
            hdr, ver, nt, _ = N.variant_header(job.template(), v)
            for n in N.cpu_scan_sha256d(hdr, job.target, 0, 1 << 20)[:2]:
                r = await s.submit(ShareSubmission(job.job_id, n, nt, ver))
                accepted += r.accepted
            if s.share_target != t0:
                break
        assert accepted >= 4
        # shares arrive far faster than the 10 s target -> difficulty goes up, target down
        assert hash_to_int(s.share_target) < hash_to_int(t0)
        await s.close()

    asyncio.run(_with_pool(body, retarget_seconds=0.5))


def test_setup_connection_error_is_fatal():
    from otedama_amd.poolproto import FatalPoolError
    from otedama_amd.stratum import messages as M

    async def body(pool):
        async def serve(reader, writer):
            await reader.read(100)
            writer.write(M.encode_message(M.SetupConnectionError(0, "unsupported-feature-flags")))
            await writer.drain()

        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        with pytest.raises(FatalPoolError):
            await V2Dialer().dial(f"stratum+v2://127.0.0.1:{port}", Credentials(user=ADDR))
        srv.close()

    asyncio.run(_with_pool(body))


def test_sv2_extended_channel_rolls_extranonce():
    """SV2 extended channel (spec §5.3.5-5.3.7/5.3.11/5.3.14): the job carries the coinbase and merkle path, the
    miner rolls its own extranonce after the pool's prefix, SubmitSharesExtended carries it, and the pool rebuilds
    the coinbase from prefix + extranonce before re-hashing."""
    async def body(pool):
        creds = Credentials(user=ADDR, version_rolling=True, extended_channel=True)
        s = await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", creds)
        assert s.extended and s.extranonce_size == 4 and len(s.extranonce_prefix) == 4
        job = await asyncio.wait_for(s.jobs.get(), 5)
        assert job.merkle_root is None and job.coinb1 and job.extranonce1 == s.extranonce_prefix
        assert job.extranonce2_size == 4 and job.version_mask != 0
        nonce, ver, nt, en2, hdr = None, None, None, None, None
        per_en2 = 1 << bin(job.version_mask).count("1")  # version bits are the lowest variant digit
        for v in range(per_en2, 64 * per_en2, per_en2 // 2):  # variants with a non-zero extranonce2
            hdr, ver, nt, en2 = N.variant_header(job.template(), v)
            if en2:
                hits = N.cpu_scan_sha256d(hdr, job.template()["target"], 0, 1 << 20)
                if hits:
                    nonce = hits[0]
                    break
        assert nonce is not None
        en2b = en2.to_bytes(8, "little")[:4]
        r = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver, en2b))
        assert r.accepted, r
        r2 = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver, en2b))
        assert not r2.accepted and "duplicate" in r2.reason
        r3 = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver, en2b[:3]))
        assert not r3.accepted and r3.reason == "invalid-extranonce-size"
        other = bytes(b ^ 0xFF for b in en2b)  # same nonce under another extranonce: a different header
        r4 = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver, other))
        assert not r4.accepted and "difficulty" in r4.reason
        await s.close()

    asyncio.run(_with_pool(body))


def test_sv2_over_noise_with_pinned_authority():
    """Noise NX wired end to end: the pool's SV2 listener runs the responder with a certificate signed by its
    authority key; the client pins that key, the whole SV2 session (setup, channel, job, share, verdict) runs over
    the encrypted channel, and a wrong pinned key is a FatalPoolError before any SV2 message is sent."""
    from otedama_amd.poolproto import FatalPoolError
    from otedama_amd.stratum import noise

    async def body(pool):
        assert len(pool.noise_authority_pub) == 32
        creds = Credentials(user=ADDR, pool_pubkey=pool.noise_authority_pub)
        s = await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", creds)
        assert isinstance(s.reader, noise.EncryptedReader)
        job = await asyncio.wait_for(s.jobs.get(), 5)
        nonce, ver, nt, _en2, _hdr = _find_share(job)
        r = await s.submit(ShareSubmission(job.job_id, nonce, nt, ver))
        assert r.accepted, r
        await s.close()
        _, wrong = noise.keypair()
        with pytest.raises(FatalPoolError):
            await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", Credentials(user=ADDR, pool_pubkey=wrong))
        # encrypted but unauthenticated (no pinned key) still works, with a warning
        logs = []
        s2 = await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", Credentials(user=ADDR, noise=True),
                                   log=lambda lvl, m: logs.append((lvl, m)))
        assert any("not authenticated" in m for _, m in logs)
        await asyncio.wait_for(s2.jobs.get(), 5)
        await s2.close()
        # the legacy 32-byte-key suite still authenticates against the same listener (it accepts both)
        s3 = await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}",
                                   Credentials(user=ADDR, pool_pubkey=pool.noise_authority_pub, noise_suite="legacy"))
        assert isinstance(s3.reader, noise.EncryptedReader)
        await asyncio.wait_for(s3.jobs.get(), 5)
        await s3.close()
        # a plaintext client against a Noise listener fails the handshake instead of hanging
        with pytest.raises(Exception):
            await V2Dialer().dial(f"stratum+v2://{pool.addr_sv2}", Credentials(user=ADDR), timeout=2.0)
        assert pool.accepted == 1

    asyncio.run(_with_pool(body, noise=True))
