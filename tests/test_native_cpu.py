"""Native host code (C++ SHA-NI SHA-256, scrypt reference, job variants, CPU miner)
against Python hashlib oracles. Runs without a GPU."""
import hashlib
import os
import struct
import time

import pytest

from otedama_amd.models.header import GENESIS_HEADER_HEX, int_to_hash, sha256d
from otedama_amd.ops.native import require_native

N = require_native()
GEN = bytes.fromhex(GENESIS_HEADER_HEX)


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 80, 119, 120, 128, 1000])
def test_sha256_lengths(n):
    data = os.urandom(n)
    assert N.sha256(data) == hashlib.sha256(data).digest()
    assert N.sha256d(data) == sha256d(data)


def test_hmac_matches_stdlib():
    import hmac

    for klen in (0, 5, 64, 80, 100):
        k = os.urandom(klen)
        m = os.urandom(77)
        assert N.hmac_sha256(k, m) == hmac.new(k, m, hashlib.sha256).digest()


def test_scrypt_reference_matches_hashlib():
    for _ in range(3):
        h = os.urandom(80)
        assert N.scrypt_1024_1_1(h) == hashlib.scrypt(h, salt=h, n=1024, r=1, p=1, dklen=32)


_BATCH_CHECK = r"""
import hashlib, os, sys
sys.path.insert(0, sys.argv[1])
from otedama_amd.ops.native import require_native
N = require_native()
for n in (1, 2, 3, 8, 9, 16, 17, 33):
    hs = [os.urandom(80) for _ in range(n)]
    assert N.scrypt_1024_1_1_batch(hs) == [hashlib.scrypt(h, salt=h, n=1024, r=1, p=1, dklen=32) for h in hs], n
print("ok")
"""


@pytest.mark.parametrize("no_avx512", ["", "1"])
def test_scrypt_batch_matches_hashlib_for_every_lane_count(no_avx512):
    """The batched host scrypt (GPU miner's verifier, CPU miner) against hashlib for 1..33 headers: 16-lane AVX-512
    passes from 9 headers on, 8-lane AVX2 passes from 3, the scalar chain below; OTEDAMA_NO_AVX512 forces the AVX2
    widths (a host without AVX2 takes the scalar chain under the same binding)."""
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("OTEDAMA_NO_AVX512", None)
    if no_avx512:
        env["OTEDAMA_NO_AVX512"] = no_avx512
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _BATCH_CHECK, root], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr[-2000:]


def test_cpu_scan_finds_genesis_nonce():
    nonce = 2083236893
    tgt = int_to_hash(0xFFFF << 208)
    assert N.cpu_scan_sha256d(GEN, tgt, nonce - 500, 1000) == [nonce]


def test_cpu_scan_matches_python_on_easy_target():
    hdr = os.urandom(76) + bytes(4)
    tgt = int_to_hash((1 << 248) - 1)  # ~1/256 of nonces
    hits = N.cpu_scan_sha256d(hdr, tgt, 1000, 4096)
    ref = [n for n in range(1000, 1000 + 4096)
           if int.from_bytes(sha256d(hdr[:76] + struct.pack("<I", n)), "little") <= int.from_bytes(tgt, "little")]
    assert hits == ref


def test_cpu_single_thread_beats_reference():
    # reference single-thread claim: ~2.5 MH/s (BENCHMARKS.md:25); SHA-NI + midstate
    if not N.cpu_has_sha_ni():
        pytest.skip("no SHA-NI on this CPU")
    t0 = time.perf_counter()
    N.cpu_scan_sha256d(GEN, bytes(32), 0, 500_000)
    rate = 500_000 / (time.perf_counter() - t0)
    assert rate > 1.0e6


def _job(**kw):
    j = {"header": GEN, "target": int_to_hash(0xFFFF << 208), "epoch": 1, "job_id": "1"}
    j.update(kw)
    return j


def test_variant_version_rolling_bits():
    mask = 0x1FFFE000
    j = _job(version_mask=mask)
    assert N.variant_space(j) == 1 << 16
    seen = set()
    for v in range(64):
        hdr, ver, nt, en2 = N.variant_header(j, v)
        assert ver & ~mask == 1 & ~mask
        assert struct.unpack_from("<I", hdr, 0)[0] == ver
        seen.add(ver)
    assert len(seen) == 64


def test_variant_ntime_rolling():
    j = _job(ntime_roll=10)
    assert N.variant_space(j) == 11
    base = struct.unpack_from("<I", GEN, 68)[0]
    for v in range(11):
        hdr, ver, nt, en2 = N.variant_header(j, v)
        assert nt == base + v
        assert struct.unpack_from("<I", hdr, 68)[0] == nt


def test_merkle_root_from_coinbase_matches_python():
    coinb1, coinb2, en1 = os.urandom(40), os.urandom(50), bytes.fromhex("f8002c90")
    branches = [os.urandom(32) for _ in range(3)]
    j = _job(coinb1=coinb1, coinb2=coinb2, extranonce1=en1, extranonce2_size=4, merkle_branches=branches)
    for en2 in (0, 1, 0xDEADBEEF):
        cb = coinb1 + en1 + en2.to_bytes(4, "little") + coinb2
        root = sha256d(cb)
        for b in branches:
            root = sha256d(root + b)
        assert N.merkle_root(j, en2) == root
        hdr, _, _, got_en2 = N.variant_header(j, en2)
        assert hdr[36:68] == root and got_en2 == en2
    assert N.variant_space(j) == 1 << 32


def test_prepare_sizes():
    assert len(N.sha256d_prepare(GEN, bytes(32))) == N.SHA256D_PARAMS_SIZE
    assert len(N.scrypt_prepare(GEN, bytes(32))) == N.SCRYPT_PARAMS_SIZE


def test_sha256d_prepare_k_accepts_only_instantiated_k():
    """The K-variant kernel exists for K in SHA256D_K_VALUES; prepare refuses other K and headers whose block 2
    (bytes 64..75) differs, since the variants share that block's message schedule."""
    assert N.SHA256D_K_VALUES == (2, 3, 4, 6, 8, 12, 16) and N.SHA256D_MAX_K == 16
    hdrs = [struct.pack("<I", 0x20000000 | (v << 13)) + GEN[4:] for v in range(16)]
    for k in range(1, 18):
        if k in N.SHA256D_K_VALUES:
            blob = N.sha256d_prepare_k(hdrs[:k], bytes(32))
            # w0..w17 + target_hi + k, then SHA256D_MAX_K variants of 18 words
            assert len(blob) == 4 * (7 + 18 * N.SHA256D_MAX_K)
            assert struct.unpack_from("<i", blob, 24)[0] == k
        else:
            with pytest.raises(ValueError):
                N.sha256d_prepare_k((hdrs * 2)[:k], bytes(32))
    bad = hdrs[:3] + [hdrs[3][:70] + b"\xff" + hdrs[3][71:]]
    with pytest.raises(ValueError):
        N.sha256d_prepare_k(bad, bytes(32))


def test_sha256d_prepare_v_table_matches_single_prepare():
    """Version-parallel layout: the kernarg block carries the shared block-2 words and the group count; the table
    holds, per variant, exactly the mid / st3 / pre3 / t2_3 words the single-midstate prepare computes."""
    assert N.SHA256D_V_GROUP == 64
    hdrs = [struct.pack("<I", 0x20000000 | (v << 13)) + GEN[4:] for v in range(128)]
    tgt = int_to_hash((1 << 240) - 1)
    params, table = N.sha256d_prepare_v(hdrs, tgt)
    w0, w1, w2, w16, w17, target_hi, groups, occ8 = struct.unpack("<8I", params)
    assert groups == 2 and occ8 == 0 and len(table) == 128 * 18 * 4
    for v in (0, 1, 63, 64, 127):
        single = N.sha256d_prepare(hdrs[v], tgt)
        mid_st3 = single[:64]
        sw0, sw1, sw2, sw16, sw17, pre3, t2_3, sth = struct.unpack_from("<8I", single, 64)
        assert (w0, w1, w2, w16, w17, target_hi) == (sw0, sw1, sw2, sw16, sw17, sth)
        row = table[72 * v: 72 * (v + 1)]
        assert row[:64] == mid_st3 and struct.unpack_from("<2I", row, 64) == (pre3, t2_3)
    for n in (0, 1, 63, 65, 100):
        with pytest.raises(ValueError):
            N.sha256d_prepare_v((hdrs * 2)[:n], tgt)
    bad = hdrs[:63] + [hdrs[63][:66] + b"\xee" + hdrs[63][67:]]
    with pytest.raises(ValueError):
        N.sha256d_prepare_v(bad, tgt)


def test_cpu_miner_runtime_emits_verified_shares():
    m = N.CpuMiner(2, "cpu-0")
    tgt = int_to_hash((1 << 244) - 1)
    m.set_job(_job(target=tgt, version_mask=0x1FFFE000, epoch=7, job_id="abc"))
    m.start()
    deadline = time.time() + 5
    shares = []
    while time.time() < deadline and len(shares) < 5:
        shares += m.poll(64)
        time.sleep(0.05)
    m.stop()
    st = m.stats()
    assert st["hashes"] > 0
    assert shares, st
    for s in shares:
        hdr = bytearray(GEN)
        struct.pack_into("<I", hdr, 0, s["version"])
        struct.pack_into("<I", hdr, 76, s["nonce"])
        h = sha256d(bytes(hdr))
        assert h == s["hash"]
        assert int.from_bytes(h, "little") <= int.from_bytes(tgt, "little")
        assert s["epoch"] == 7 and s["job_id"] == "abc" and s["device_id"] == "cpu-0"


@pytest.mark.parametrize("algo", ["scrypt", "x11"])
def test_cpu_miner_scrypt_and_x11_emit_verified_shares(algo):
    """CPU-only hosts mine scrypt / X11 through the host reference chains (256-nonce chunks): every share is
    re-hashed here (hashlib.scrypt / the native X11 oracle) and meets the target; stripes stay disjoint."""
    m = N.CpuMiner(2, "cpu-0")
    tgt_int = (1 << 251) - 1  # ~1 share per 32 hashes
    m.set_job(_job(target=int_to_hash(tgt_int), version_mask=0x1FFFE000, epoch=3, job_id="s", algo=algo))
    m.start()
    deadline = time.time() + 20
    shares = []
    while time.time() < deadline and len(shares) < 6:
        shares += m.poll(64)
        time.sleep(0.05)
    m.stop()
    shares += m.poll(4096)
    st = m.stats()
    assert st["hashes"] > 0 and shares, st
    seen = set()
    for s in shares[:40]:
        hdr = bytearray(GEN)
        struct.pack_into("<I", hdr, 0, s["version"])
        struct.pack_into("<I", hdr, 76, s["nonce"])
        if algo == "scrypt":
            h = hashlib.scrypt(bytes(hdr), salt=bytes(hdr), n=1024, r=1, p=1, dklen=32)
        else:
            h = N.x11(bytes(hdr))
        assert h == s["hash"] and int.from_bytes(h, "little") <= tgt_int
        key = (s["version"], s["nonce"])
        assert key not in seen
        seen.add(key)


def test_cpu_miner_pause_with_none_job():
    m = N.CpuMiner(1, "cpu-0")
    m.start()
    m.set_job(None)
    time.sleep(0.05)
    h0 = m.stats()["hashes"]
    time.sleep(0.1)
    assert m.stats()["hashes"] == h0
    m.stop()


@pytest.mark.parametrize("start,count", [(0, 1), (7, 2), (11, 999), (0xFFFFFF00, 513)])
def test_cpu_scan_pairs_and_tail_match_python(start, count):
    """The scan hashes nonces in interleaved pairs plus a scalar tail; any count/start (incl. the 2^32 wrap)
    gives exactly the hashlib hits, in nonce order."""
    import random

    rng = random.Random(start ^ count)
    hdr = bytes(rng.getrandbits(8) for _ in range(76)) + bytes(4)
    t_int = (1 << 250) - 1
    tgt = t_int.to_bytes(32, "little")
    got = N.cpu_scan_sha256d(hdr, tgt, start, count)
    ref = []
    for k in range(count):
        n = (start + k) & 0xFFFFFFFF
        d = hashlib.sha256(hashlib.sha256(hdr[:76] + n.to_bytes(4, "little")).digest()).digest()
        if int.from_bytes(d, "little") <= t_int:
            ref.append(n)
    assert got == ref


def test_v1_coinbase_variants_group_by_version_first():
    """Stratum V1 job with a coinbase (extranonce2_size 4) and a BIP320 mask: neighbouring variant indexes differ
    only in the version word, so they share header bytes 36..79 (merkle root, ntime, nbits) and the K-variant
    SHA-256d kernel can group them; extranonce2 rolls once per 2^popcount(mask) versions, ntime last."""
    mask = 0x1FFFE000
    coinb1, coinb2, en1 = os.urandom(40), os.urandom(50), bytes.fromhex("f8002c90")
    j = _job(coinb1=coinb1, coinb2=coinb2, extranonce1=en1, extranonce2_size=4, merkle_branches=[os.urandom(32)],
             version_mask=mask, ntime_roll=3)
    assert N.variant_space(j) == (1 << 32) * (1 << 16) * 4
    h0, v0, nt0, e0 = N.variant_header(j, 0)
    for v in range(1, 4):
        h, ver, nt, en2 = N.variant_header(j, v)
        assert h[36:] == h0[36:] and en2 == e0 == 0 and nt == nt0 and ver != v0
    h, ver, nt, en2 = N.variant_header(j, 1 << 16)
    assert en2 == 1 and ver == v0 and nt == nt0 and h[36:68] != h0[36:68]
    h, ver, nt, en2 = N.variant_header(j, (1 << 16) * (1 << 32))
    assert en2 == 0 and ver == v0 and nt == nt0 + 1
    # a device stripe (stride = world size) still groups within the version digit
    stride = 8
    hs = [N.variant_header(j, 3 + k * stride)[0] for k in range(4)]
    assert all(x[36:] == hs[0][36:] for x in hs)


def test_scrypt_verifier_queue_is_bounded_under_a_flood():
    """the GPU miner's scrypt candidates wait for host verification (~0.2-1 ms each) in a
    BoundedWorkQueue. A producer that never waits (a share target far below the device's rate) fills it to its cap
    and every further candidate is refused and counted; nothing is lost uncounted and memory stays bounded."""
    for cap, n in ((64, 5000), (8192, 20000)):
        r = N._work_queue_flood(cap, n, True)
        assert r["peak"] <= cap and r["refused"] > 0, r
        assert r["accepted"] + r["refused"] == n and r["processed"] == r["accepted"], r
    r = N._work_queue_flood(64, 50, False)  # below the cap nothing is refused
    assert r == {"accepted": 50, "refused": 0, "peak": r["peak"], "processed": 50} and r["peak"] <= 50
    # the verifier's batched consumer (pop_many of up to 16, one scrypt pass per batch): bounded the same way,
    # every accepted item hashed exactly once
    r = N._work_queue_flood(64, 3000, True, 16)
    assert r["peak"] <= 64 and r["refused"] > 0 and r["accepted"] + r["refused"] == 3000, r
    assert r["processed"] == r["accepted"], r
    r = N._work_queue_flood(4096, 300, True, 16)
    assert r["processed"] == r["accepted"] == 300 and r["refused"] == 0, r


def test_clock_bounds_track_the_window_minimum():
    """The GPU miner's device-clock estimate (otedama/clock_bounds.h): the lowest offset bound seen in the last
    `window` seconds, following drift once older, lower bounds age out."""
    from otedama_amd.ops.native import require_native

    N = require_native()
    # true offset 10.000 at t<3, drifting to 10.003 later; every sighting is late by 0..50 us (an upper bound)
    seq = [(0.0, 10.00004), (0.2, 10.00001), (0.4, 10.00003), (1.0, 10.00002), (2.1, 10.00005),
           (3.0, 10.00302), (3.5, 10.00301), (4.0, 10.00304), (4.2, 10.00303)]
    got = N._clock_bounds(2.0, seq)
    assert got[:5] == [10.00004, 10.00001, 10.00001, 10.00001, 10.00001]  # the 0.2 s bound is 1.9 s old at 2.1
    assert got[5] == pytest.approx(10.00002)   # t=3.0: 0.2 and 0.4 aged out, 1.0 is exactly 2 s old
    assert got[6] == pytest.approx(10.00005)   # t=3.5: 2.1's bound is the lowest left
    assert got[7] == pytest.approx(10.00005)
    assert got[8] == pytest.approx(10.00301)   # t=4.2: only the drifted bounds remain
    assert N._clock_bounds(2.0, [(0.0, 5.0)]) == [5.0]


@pytest.mark.parametrize("lanes", [1, 2, 3, 4, 16])
def test_cpu_scan_lanes_agree(lanes):
    """Every interleave width of the CPU scan finds the same hits (genesis nonce at its target; an easy target over
    a window that is not a multiple of the width, so the one-at-a-time tail runs too). 16 is the AVX-512 scan (the
    SHA-NI scan with 4 chains on a host without AVX-512)."""
    from otedama_amd.models.header import GENESIS_HEADER_HEX, int_to_hash
    from otedama_amd.ops.native import require_native

    N = require_native()
    hdr = bytes.fromhex(GENESIS_HEADER_HEX)
    nonce = int.from_bytes(hdr[76:80], "little")
    assert nonce in N._cpu_scan_lanes(lanes, hdr, int_to_hash(0xFFFF << 208), nonce - 1001, 4003)
    easy = int_to_hash((1 << 248) - 1)
    assert N._cpu_scan_lanes(lanes, hdr, easy, 7, 3001) == N._cpu_scan_lanes(1, hdr, easy, 7, 3001)


def test_avx512_scan_matches_python_over_random_headers():
    """The 16-lane AVX-512 SHA-256d scan against hashlib over random headers and a nonce window that wraps 2^32:
    every nonce whose double hash meets a 1-in-256 target, and no other."""
    from otedama_amd.models.header import int_to_hash

    tgt = (1 << 248) - 1
    for start in (0xFFFFF000, 0x12345670):
        h = os.urandom(80)
        want = [(start + i) & 0xFFFFFFFF for i in range(5000)
                if int.from_bytes(sha256d(h[:76] + ((start + i) & 0xFFFFFFFF).to_bytes(4, "little")), "little") <= tgt]
        assert N._cpu_scan_lanes(16, h, int_to_hash(tgt), start, 5000) == want


_GROUPS_CHECK = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
from otedama_amd.models.header import int_to_hash, sha256d
from otedama_amd.ops.native import require_native
N = require_native()
tgt = (1 << 248) - 1
h = os.urandom(80)
start = 0xFFFFFF00
want = [(start + i) & 0xFFFFFFFF for i in range(3001)
        if int.from_bytes(sha256d(h[:76] + ((start + i) & 0xFFFFFFFF).to_bytes(4, "little")), "little") <= tgt]
assert N._cpu_scan_lanes(16, h, int_to_hash(tgt), start, 3001) == want
print(N.cpu_scan_method())
"""


@pytest.mark.parametrize("groups", ["1", "2", "3", "4"])
def test_avx512_scan_groups_agree(groups):
    """1-4 sixteen-lane groups in flight (OTEDAMA_CPU_SCAN_GROUPS; default 2 on AMD, 1 elsewhere): the same hits
    as hashlib over a window that wraps 2^32 and is not a multiple of 64 (the smaller widths and the scalar tail
    finish it)."""
    import subprocess
    import sys

    if not N.cpu_scan_method().startswith("avx512"):
        pytest.skip("no AVX-512 on this host")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _GROUPS_CHECK, root], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, OTEDAMA_CPU_SCAN_GROUPS=groups))
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip() == f"avx512 16 lanes x {groups} groups"


def test_maps_check_requires_read_write_permissions():
    """the CPU-stored abort word is used only when its range is mapped rw in /proc/self/maps; a
    PROT_NONE reservation of the GPU address range (libhsakmt, small BAR) must not pass."""
    from otedama_amd.ops.native import require_native

    N = require_native()
    maps = ("7f0000000000-7f0000100000 ---p 00000000 00:00 0 \n"
            "7f0000100000-7f0000200000 rw-s 00000000 00:05 12 /dev/dri/renderD128\n"
            "7f0000200000-7f0000300000 r--p 00000000 00:00 0\n"
            "garbage line\n")
    assert not N.maps_range_writable(maps, 0x7F0000000100, 0x7F0000000200)  # PROT_NONE reservation
    assert N.maps_range_writable(maps, 0x7F0000100100, 0x7F0000100200)       # rw mapping of the BAR
    assert not N.maps_range_writable(maps, 0x7F0000200100, 0x7F0000200200)  # read-only
    assert not N.maps_range_writable(maps, 0x7F00000FFFF0, 0x7F0000100010)  # straddles two lines
    assert not N.maps_range_writable("", 0x1000, 0x1100)
