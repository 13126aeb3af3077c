"""engine/miner_probe.py: the production miner's rate for scrypt / X11 in bench.py (GPU), and the header it
re-hashes each share on (CPU: against the native variant arithmetic)."""
import hashlib

import pytest

from otedama_amd.engine.miner_probe import _header, measure_miner
from otedama_amd.models.header import int_to_hash


def _native():
    from otedama_amd.ops.native import require_native

    return require_native()


def test_share_header_matches_the_native_variant_header():
    N = _native()
    base = hashlib.sha256(b"probe").digest()
    hdr = (0x20000000).to_bytes(4, "little") + base + hashlib.sha256(base).digest() + \
        (1_700_000_000).to_bytes(4, "little") + (0x1D00FFFF).to_bytes(4, "little") + bytes(4)
    job = {"header": hdr, "target": int_to_hash((1 << 240) - 1), "job_id": "p", "epoch": 1, "algo": "scrypt",
           "version_mask": 0x1FFFE000, "variant_start": 3, "variant_stride": 8}
    for v in (0, 1, 3, 11, 4099, 65535):
        h80, version, ntime, _ = N.variant_header(job, v)
        share = {"version": version, "ntime": ntime, "nonce": 0xDEADBEEF}
        assert _header(hdr, share) == h80[:76] + (0xDEADBEEF).to_bytes(4, "little")


@pytest.mark.gpu
@pytest.mark.parametrize("algo,target,floor,process", [("scrypt", 0xFFFF << 224, 12e6, False),
                                                       ("x11", (1 << 236) - 1, 300e6, False),
                                                       ("scrypt", 0xFFFF << 224, 12e6, True)])
def test_production_miner_rate_and_shares(algo, target, floor, process):
    """In this process and through a device process (bench.py's path): exact rate, shares re-hashed, nothing lost."""
    N = _native()
    r = measure_miner(N, 0, algo, target, seconds=2.0, warmup=1.5, recheck=16, process=process)
    assert not r["faulted"] and r["hashes_per_sec"] > floor, r
    assert r["shares"] > 0 and r["shares_rechecked"] > 0 and r["shares_recheck_ok"] == r["shares_rechecked"], r
    assert r["dropped"] == 0 and r["ring_overflow"] == 0 and r["verify_dropped"] == 0, r
