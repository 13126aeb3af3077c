"""gfx950 kernels vs the CPU oracle (run on a real MI355X via gpurun).

Numerics for an integer hash kernel are exact: the set of nonces a kernel
reports for a target must equal the set the CPU (hashlib / C++ reference)
computes for the same header window.
"""
import hashlib
import os
import struct
import time

import pytest

pytestmark = pytest.mark.gpu


def _native():
    from otedama_amd.ops.native import require_native

    return require_native()


def _ref_hits_sha256d(hdr, base, count, target_int):
    out = []
    for n in range(base, base + count):
        h = hashlib.sha256(hashlib.sha256(hdr[:76] + struct.pack("<I", n & 0xFFFFFFFF)).digest()).digest()
        if int.from_bytes(h, "little") <= target_int:
            out.append(n & 0xFFFFFFFF)
    return out


def test_native_gpu_visible():
    N = _native()
    assert N.gpu_device_count() >= 1
    assert N.gpu_arch_name(0).startswith("gfx950")


def test_sha256d_genesis_nonce():
    from otedama_amd.models.header import GENESIS_HEADER_HEX, int_to_hash
    from otedama_amd.ops.search import Sha256dSearch

    hdr = bytes.fromhex(GENESIS_HEADER_HEX)
    s = Sha256dSearch("cuda:0")
    nonce = 2083236893
    assert s.search(hdr, int_to_hash(0xFFFF << 208), nonce - 1000, 5000) == [nonce]


@pytest.mark.parametrize("seed", range(4))
def test_sha256d_matches_cpu_easy_target(seed):
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import Sha256dSearch

    rng = __import__("random").Random(seed)
    hdr = bytes(rng.getrandbits(8) for _ in range(76)) + bytes(4)
    target_int = (1 << 248) - 1  # ~1/256 hit rate -> ~256 hits in 65536
    s = Sha256dSearch("cuda:0", cap=4096)
    base = rng.getrandbits(32) & ~0xFFFF
    got = sorted(s.search(hdr, int_to_hash(target_int), base, 1 << 16))
    N = _native()
    ref = sorted(N.cpu_scan_sha256d(hdr, int_to_hash(target_int), base, 1 << 16))
    assert got == ref and len(ref) > 100
    # spot-check against hashlib too
    assert ref[:20] == _ref_hits_sha256d(hdr, base, ref[19] - base + 1, target_int)[:20]


def test_sha256d_target_hi_tie_filtered_by_host():
    """Kernel compares only the top word; a target whose top word ties must still
    produce only hits that the full compare accepts (host re-verification)."""
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import Sha256dSearch

    hdr = os.urandom(76) + bytes(4)
    target_int = (0x00FFFFFF << 224) | 0x1  # top word 0x00ffffff, low bits tiny
    s = Sha256dSearch("cuda:0", cap=4096)
    cands = s.search(hdr, int_to_hash(target_int), 0, 1 << 16)
    N = _native()
    strict = N.cpu_scan_sha256d(hdr, int_to_hash(target_int), 0, 1 << 16)
    assert set(strict) <= set(cands)


def test_sha256d_wraps_nonce_space():
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import Sha256dSearch

    hdr = os.urandom(76) + bytes(4)
    t = int_to_hash((1 << 250) - 1)
    s = Sha256dSearch("cuda:0", cap=4096)
    got = sorted(s.search(hdr, t, 0xFFFFF000, 0x2000))
    N = _native()
    ref = sorted(N.cpu_scan_sha256d(hdr, t, 0xFFFFF000, 0x1000) + N.cpu_scan_sha256d(hdr, t, 0, 0x1000))
    assert got == ref


# kernel "coop" = lane-cooperative full-line ROMix (gap 1); "lane" = one lane per hash at gap 1/2/4, and
# native code 9 = per-lane gap 1 pinned to 8 waves/SIMD. n = 200 is not a multiple of 64 (the cooperative
# kernel rounds its wave count up).
@pytest.mark.parametrize("gap,n,kernel", [(1, 192, "lane"), (2, 192, "lane"), (4, 192, "lane"), (1, 192, "coop"),
                                          (1, 200, "coop"), (9, 200, "lane"), (1, 192, "coop2"), (1, 200, "coop2"),
                                          (1, 192, "split"), (1, 200, "split")])
def test_scrypt_matches_hashlib(gap, n, kernel):
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import ScryptSearch

    hdr = os.urandom(76) + bytes(4)
    sc = ScryptSearch("cuda:0", grid=8, gap=gap, cap=1024, kernel=kernel)
    assert sc.kernel == kernel
    # target: ~1/4 of hashes pass -> checks filtering as well as hashing
    target_int = (1 << 254) - 1
    got = sorted(sc.search(hdr, int_to_hash(target_int), 5000, n))
    ref = []
    for nonce in range(5000, 5000 + n):
        h80 = hdr[:76] + struct.pack("<I", nonce)
        d = hashlib.scrypt(h80, salt=h80, n=1024, r=1, p=1, dklen=32)
        if int.from_bytes(d, "little") <= target_int:
            ref.append(nonce)
    assert got == ref and 0 < len(ref) < n


@pytest.mark.parametrize("kernel", ["lane", "coop", "coop2"])
def test_scrypt_more_lanes_than_slots(kernel):
    """count > grid*256 exercises the grid-stride reuse of a scratchpad slot (hashes checked, not just counted)."""
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import ScryptSearch

    hdr = os.urandom(76) + bytes(4)
    sc = ScryptSearch("cuda:0", grid=1, lanes_per_slot=2, cap=1024, kernel=kernel)
    target_int = (1 << 255) - 1
    got = sorted(sc.search(hdr, int_to_hash(target_int), 0, 512))
    ref = [n for n in range(512) if int.from_bytes(hashlib.scrypt(
        hdr[:76] + struct.pack("<I", n), salt=hdr[:76] + struct.pack("<I", n), n=1024, r=1, p=1, dklen=32),
        "little") <= target_int]
    assert got == ref and 100 < len(ref) < 412


@pytest.mark.parametrize("segments,n,lanes_per_slot,seg_grid", [(1, 128, 1, ""), (3, 200, 1, ""), (8, 192, 1, ""),
                                                                  (16, 256, 1, ""), (4, 512, 2, ""), (6, 960, 1, "1"),
                                                                  (32, 256, 1, "resident")])
def test_scrypt_segmented_romix_matches_hashlib(monkeypatch, segments, n, lanes_per_slot, seg_grid):
    """OTEDAMA_SCRYPT_SEGMENTS: the cooperative ROMix as S launches with X carried in xbuf (segment bounds that do
    and do not fall on the write/read boundary); with more lanes than slots the launcher keeps the one-launch
    kernel (a pad cannot be shared between two hashes across launches). OTEDAMA_SCRYPT_SEG_GRID=1: one launched
    block walks the hashes of four allocated blocks (grid-stride, each hash on its own pad)."""
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import ScryptSearch

    monkeypatch.setenv("OTEDAMA_SCRYPT_SEGMENTS", str(segments))
    monkeypatch.setenv("OTEDAMA_SCRYPT_SEG_GRID", seg_grid)
    hdr = os.urandom(76) + bytes(4)
    sc = ScryptSearch("cuda:0", grid=4 if seg_grid == "1" else 1, lanes_per_slot=lanes_per_slot, cap=1024, kernel="coop")
    target_int = (1 << 254) - 1
    got = sorted(sc.search(hdr, int_to_hash(target_int), 7000, n))
    ref = [x for x in range(7000, 7000 + n) if int.from_bytes(hashlib.scrypt(
        hdr[:76] + struct.pack("<I", x), salt=hdr[:76] + struct.pack("<I", x), n=1024, r=1, p=1, dklen=32),
        "little") <= target_int]
    assert got == ref and 0 < len(ref) < n


def test_scrypt_split_refuses_more_lanes_than_slots():
    """The split kernel keeps one hash per lane slot across its two launches: a batch larger than the grid's slots
    is refused rather than silently reusing a pad between the launches."""
    from otedama_amd.ops.search import ScryptSearch

    with pytest.raises(ValueError):
        ScryptSearch("cuda:0", grid=1, lanes_per_slot=2, kernel="split")
    sc = ScryptSearch("cuda:0", grid=1, kernel="split")
    assert sc.batch == 256


def test_gpu_miner_runtime_shares():
    from otedama_amd.models.header import int_to_hash

    N = _native()
    hdr = os.urandom(76) + bytes(4)
    tgt = int_to_hash((1 << 232) - 1)  # ~1 per 2^24
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28)
    m.set_job({"header": hdr, "target": tgt, "epoch": 3, "job_id": "j1", "version_mask": 0x1FFFE000})
    m.start()
    deadline = time.time() + 20
    shares = []
    while time.time() < deadline and len(shares) < 20:
        shares += m.poll(256)
        time.sleep(0.02)
    m.stop()
    st = m.stats()
    assert not st["faulted"], st
    assert st["hashes"] >= 1 << 28
    assert len(shares) >= 5, st
    for s in shares:
        h80 = bytearray(hdr)
        struct.pack_into("<I", h80, 0, s["version"])
        struct.pack_into("<I", h80, 76, s["nonce"])
        d = hashlib.sha256(hashlib.sha256(bytes(h80)).digest()).digest()
        assert d == s["hash"] and int.from_bytes(d, "little") <= int.from_bytes(tgt, "little")
        assert s["epoch"] == 3 and s["job_id"] == "j1"


def test_gpu_miner_runtime_scrypt_shares():
    """Production scrypt path: native GpuMiner thread + lane-cooperative ROMix, hits re-verified by hashlib."""
    from otedama_amd.models.header import int_to_hash

    N = _native()
    hdr = os.urandom(76) + bytes(4)
    tgt = int_to_hash((1 << 248) - 1)  # ~1 per 256 hashes
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 20)
    m.set_job({"header": hdr, "target": tgt, "epoch": 5, "job_id": "s1", "algo": "scrypt"})
    m.start()
    deadline = time.time() + 30
    shares = []
    while time.time() < deadline and len(shares) < 50:
        shares += m.poll(256)
        time.sleep(0.02)
    m.stop()
    st = m.stats()
    assert not st["faulted"], st
    assert len(shares) >= 20, st
    for s in shares[:50]:
        h80 = bytearray(hdr)
        struct.pack_into("<I", h80, 0, s["version"])
        struct.pack_into("<I", h80, 76, s["nonce"])
        d = hashlib.scrypt(bytes(h80), salt=bytes(h80), n=1024, r=1, p=1, dklen=32)
        assert d == s["hash"] and int.from_bytes(d, "little") <= int.from_bytes(tgt, "little")
        assert s["epoch"] == 5 and s["job_id"] == "s1"


def test_gpu_fault_retires_device_and_survivor_takes_the_stripe():
    """SURVEY §5.3 on real hardware: a GpuMiner on a HIP ordinal that does not exist faults in its
    device thread; MinerSet retires it, and at the next new work the surviving MI355X takes the whole
    variant class (stride 1) and keeps producing verified shares."""
    import dataclasses

    from otedama_amd.engine.miners import MinerSet
    from otedama_amd.hal import HIPDriver, Identity
    from otedama_amd.models.header import int_to_hash

    N = _native()
    gpu0 = HIPDriver().enumerate()[0]
    dead = dataclasses.replace(gpu0, ident=dataclasses.replace(gpu0.ident, id="gpu-dead"),
                               index=N.gpu_device_count() + 7)
    logs = []
    ms = MinerSet([gpu0, dead], batch_nonces=1 << 28, log=lambda lvl, msg: logs.append(msg))
    tgt = int_to_hash((1 << 232) - 1)
    hdr1 = os.urandom(76) + bytes(4)
    ms.start()
    try:
        ms.set_job({"header": hdr1, "target": tgt, "job_id": "a", "version_mask": 0x1FFFE000})
        deadline = time.time() + 10
        retired = []
        while time.time() < deadline and not retired:
            retired = ms.retire_faulted()
            time.sleep(0.05)
        assert [d for d, _ in retired] == ["gpu-dead"], (retired, ms.device_stats())
        assert "HIP error" in retired[0][1]
        hdr2 = os.urandom(76) + bytes(4)
        ep = ms.set_job({"header": hdr2, "target": tgt, "job_id": "b", "version_mask": 0x1FFFE000})
        assert (ms.miners[0].stripe_index, ms.miners[0].stripe_stride) == (0, 1)
        shares, deadline = [], time.time() + 20
        while time.time() < deadline and len(shares) < 10:
            shares += [s for s in ms.poll(256) if s["epoch"] == ep]
            time.sleep(0.02)
    finally:
        ms.stop()
    assert len(shares) >= 5 and all(s["device_id"] == "gpu-0" for s in shares)
    for s in shares:
        h80 = bytearray(hdr2)
        struct.pack_into("<I", h80, 0, s["version"])
        struct.pack_into("<I", h80, 76, s["nonce"])
        d = hashlib.sha256(hashlib.sha256(bytes(h80)).digest()).digest()
        assert d == s["hash"] and int.from_bytes(d, "little") <= int.from_bytes(tgt, "little")
    assert not ms.device_stats()["gpu-0"]["faulted"]
    assert any("re-split" in m for m in logs)


@pytest.mark.parametrize("k", [2, 3, 4, 6, 8, 12, 16])
def test_sha256d_k_variants_match_cpu(k):
    """K BIP320 version variants sharing block 2: every variant's hits equal the CPU scan of its own header."""
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.search import Sha256dSearchK

    rng = __import__("random").Random(100 + k)
    tail = bytes(rng.getrandbits(8) for _ in range(76))
    headers = [struct.pack("<I", 0x20000000 | (v << 13)) + tail[4:] + bytes(4) for v in range(k)]
    target_int = (1 << 248) - 1
    s = Sha256dSearchK("cuda:0", k=k, cap=4096)
    base = rng.getrandbits(32) & ~0xFFFF
    got = s.search(headers, int_to_hash(target_int), base, 1 << 16)
    N = _native()
    for v in range(k):
        ref = sorted(N.cpu_scan_sha256d(headers[v], int_to_hash(target_int), base, 1 << 16))
        assert sorted(n for n, vv in got if vv == v) == ref and len(ref) > 100
    with pytest.raises(ValueError):
        s.prepare([headers[0]] * (k - 1), bytes(32))


@pytest.mark.parametrize("algo", ["sha256d", "scrypt", "x11"])
def test_doctor_pow_self_test_runs_the_gpu_kernel(algo):
    from otedama_amd import config as C
    from otedama_amd import doctor as D

    cfg = C.Config()
    cfg.mining.algorithm = algo
    r = D.check_pow_self_test(cfg).run()
    assert r.status == D.Status.PASS, r.detail
    assert "gfx950" in r.detail and "no gfx950" not in r.detail


def test_gpu_miner_groups_v1_coinbase_variants():
    """A Stratum V1 job with a coinbase (extranonce2_size 4) and a BIP320 mask takes the version-parallel kernel:
    the variant digits put version bits lowest, so 64 neighbouring stripe positions share the merkle root and
    block 2.
    Every share re-hashes to its reported hash from the rebuilt coinbase / merkle root."""
    from otedama_amd.models.header import int_to_hash, sha256d

    N = _native()
    coinb1, coinb2, en1 = os.urandom(40), os.urandom(50), os.urandom(4)
    branches = [os.urandom(32), os.urandom(32)]
    hdr = os.urandom(76) + bytes(4)
    tgt = int_to_hash((1 << 232) - 1)
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28)
    m.set_job({"header": hdr, "target": tgt, "epoch": 4, "job_id": "v1", "version_mask": 0x1FFFE000,
               "coinb1": coinb1, "coinb2": coinb2, "extranonce1": en1, "extranonce2_size": 4,
               "merkle_branches": branches})
    m.start()
    deadline = time.time() + 20
    shares = []
    while time.time() < deadline and len(shares) < 10:
        shares += m.poll(256)
        time.sleep(0.02)
    m.stop()
    st = m.stats()
    assert not st["faulted"], st
    assert st["launches"] >= 2 and st["variant_launches"] == st["launches"], st
    assert len(shares) >= 3, st
    for s in shares:
        root = sha256d(coinb1 + en1 + s["extranonce2"].to_bytes(4, "little") + coinb2)
        for b in branches:
            root = sha256d(root + b)
        h80 = struct.pack("<I", s["version"]) + hdr[4:36] + root + hdr[68:76] + struct.pack("<I", s["nonce"])
        assert sha256d(h80) == s["hash"] and int.from_bytes(s["hash"], "little") <= int.from_bytes(tgt, "little")


def _v_headers(n, seed=b"v"):
    tail = hashlib.sha256(seed).digest() * 3
    return [struct.pack("<I", 0x20000000 | ((v & 0xFFFF) << 13)) + tail[:72] + bytes(4) for v in range(n)]


@pytest.mark.parametrize("groups,base,chains,occ", [(1, 0x12345600, 1, True), (2, 0xFFFFFC00, 1, True),
                                                  (2, 0x12345600, 2, False), (4, 0xFFFFFC00, 2, True),
                                                  (3, 0x12345600, 3, False), (4, 0xFFFFFC00, 4, False)])
def test_sha256d_v_kernel_matches_cpu(groups, base, chains, occ):
    """Version-parallel kernels (one or two variants per lane): for every variant and every W3 of the window
    (incl. the 2^32 wrap), the reported (nonce = bswap(W3), variant) pairs are exactly the CPU's shares."""
    from otedama_amd.ops.search import Sha256dSearchV

    s = Sha256dSearchV("cuda:0", cap=4096, grid=512, chains=chains, occupancy8=occ)  # ~4 hits per variant
    hs = _v_headers(64 * groups)
    target_int = (1 << 248) - 1
    count = 1024
    got = sorted(s.search(hs, target_int.to_bytes(32, "little"), base, count))
    want = []
    for vi, h in enumerate(hs):
        for i in range(count):
            w3 = (base + i) & 0xFFFFFFFF
            nonce = int.from_bytes(w3.to_bytes(4, "big"), "little")
            d = hashlib.sha256(hashlib.sha256(h[:76] + nonce.to_bytes(4, "little")).digest()).digest()
            if int.from_bytes(d, "little") <= target_int:
                want.append((nonce, vi))
    assert got == sorted(want) and len(want) > 100


def test_sha256d_v_kernel_both_builds_and_grid_contract():
    from otedama_amd.ops.search import Sha256dSearchV

    hs = _v_headers(128, b"w")
    tgt = ((1 << 248) - 1).to_bytes(32, "little")
    a = sorted(Sha256dSearchV("cuda:0", grid=256, occupancy8=False).search(hs, tgt, 7, 512))
    b = sorted(Sha256dSearchV("cuda:0", grid=256, occupancy8=True).search(hs, tgt, 7, 512))
    c = sorted(Sha256dSearchV("cuda:0", grid=1024, block=64).search(hs, tgt, 7, 512))  # one wave per block
    assert a == b == c and a
    with pytest.raises(ValueError):
        Sha256dSearchV("cuda:0", grid=1).prepare(_v_headers(64 * 8), tgt)  # 4 waves cannot split 8 groups
    with pytest.raises(ValueError):
        Sha256dSearchV("cuda:0", grid=3, block=64).prepare(hs, tgt)  # 3 waves cannot split 2 groups
    with pytest.raises(ValueError):
        Sha256dSearchV("cuda:0", block=128)
    d = sorted(Sha256dSearchV("cuda:0", grid=256, chains=2).search(hs, tgt, 7, 512))  # 128 variants, 2 per lane
    assert d == a
    with pytest.raises(ValueError):
        Sha256dSearchV("cuda:0", grid=256, chains=2).prepare(hs[:64], tgt)  # two chains need 128 variants
    with pytest.raises(ValueError):
        Sha256dSearchV("cuda:0", chains=5)
    with pytest.raises(ValueError):
        Sha256dSearchV("cuda:0", grid=256).prepare(hs[:63], tgt)


def test_sha256d_v_launch_on_a_side_stream():
    """A launch on a caller's stream waits for the variant-table upload (done on the current stream) and resets
    the hit count on the launch stream itself, so its hits equal the default-stream launch."""
    import torch

    from otedama_amd.ops.search import Sha256dSearchV

    hs = _v_headers(64, b"s")
    tgt = ((1 << 248) - 1).to_bytes(32, "little")
    s = Sha256dSearchV("cuda:0", grid=256)
    want = sorted(s.search(hs, tgt, 1000, 512))
    side = torch.cuda.Stream(device="cuda:0")
    out = torch.full((1 + 2 * s.cap,), 7, dtype=torch.int32, device="cuda:0")  # stale count must be cleared
    r = s.launch(s.prepare(hs, tgt), 1000, 512, out=out, stream=side)
    side.synchronize()
    assert sorted(r.hits()) == want and want


def test_gpu_miner_kernel_selection():
    """Default GpuMiner: version-rolling jobs take the two-chain version-parallel kernel (128 variants per launch),
    or the 64-variant one when the mask supplies fewer; with sha_variants=8 they take the K-variant kernel; a job
    without a version mask runs single-midstate."""
    from otedama_amd.models.header import int_to_hash

    N = _native()
    hdr = os.urandom(76) + bytes(4)
    tgt = int_to_hash((1 << 236) - 1)

    def run(miner, job, want):
        miner.set_job(job)
        miner.start()
        deadline = time.time() + 15
        shares = []
        while time.time() < deadline and len(shares) < want:
            shares += miner.poll(256)
            time.sleep(0.02)
        miner.stop()
        st = miner.stats()
        assert not st["faulted"], st
        for s in shares:
            h80 = bytearray(hdr)
            struct.pack_into("<I", h80, 0, s["version"])
            struct.pack_into("<I", h80, 76, s["nonce"])
            d = hashlib.sha256(hashlib.sha256(bytes(h80)).digest()).digest()
            assert d == s["hash"] and int.from_bytes(d, "little") <= int.from_bytes(tgt, "little")
        return st, shares

    job = {"header": hdr, "target": tgt, "epoch": 1, "job_id": "a", "version_mask": 0x1FFFE000}
    st, shares = run(N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28), job, 8)  # default: two variants per lane
    assert st["variant_launches"] == st["launches"] >= 2 and len(shares) >= 4
    # completed launches count whole batches; batches stopped early by stop()'s abort count the estimated part done
    full = (1 << 28) // 128 * 128
    assert (st["launches"] - st["aborted_launches"]) * full <= st["hashes"] <= st["launches"] * full
    assert len({s["version"] for s in shares}) >= 2
    st, shares = run(N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28, sha_variants=64), job, 4)  # one per lane
    assert st["variant_launches"] == st["launches"] >= 2 and len(shares) >= 2
    # only 64 versions in the mask: the default miner falls back from 128 to the 64-variant layout
    st, shares = run(N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28), dict(job, version_mask=0x7E000), 4)
    assert st["variant_launches"] == st["launches"] >= 2 and len(shares) >= 2
    st, shares = run(N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28, sha_variants=8), job, 4)
    assert st["variant_launches"] == st["launches"] >= 2 and len(shares) >= 2
    st, shares = run(N.GpuMiner(0, "gpu-0", batch_nonces=1 << 28), dict(job, version_mask=0), 2)
    assert st["variant_launches"] == 0 and st["launches"] >= 2
    assert all(s["version"] == struct.unpack_from("<I", hdr, 0)[0] for s in shares)
