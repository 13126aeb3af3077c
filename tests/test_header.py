"""Header / hash / target math KATs (mirrors internal/miner/sha256d_test.go)."""
import math

import pytest

from otedama_amd.models import header as H


def test_genesis_hash_kat():
    hdr = bytes.fromhex(H.GENESIS_HEADER_HEX)
    assert H.hash_header(hdr).hex() == H.GENESIS_HASH_HEX
    parsed = H.Header.parse(hdr)
    assert parsed.version == 1
    assert parsed.nonce == 2083236893
    assert parsed.bits == 0x1D00FFFF
    assert parsed.time == 1231006505
    assert parsed.to_bytes() == hdr
    assert H.hash_header(parsed).hex() == H.GENESIS_HASH_HEX


def test_sha256d_empty():
    assert H.sha256d(b"").hex() == "5df6e0e2761359d30a8275058e299fcc0381534545f55cf43e41983f5d4c9456"


def test_nonce_offset_76():
    h = H.Header(nonce=0xDEADBEEF)
    b = h.to_bytes()
    assert b[76:80] == bytes.fromhex("efbeadde")


@pytest.mark.parametrize("nbits,hexle", [
    (0x1D00FFFF, "0000000000000000000000000000000000000000000000000000ffff00000000"),
    (0x1B0404CB, "00" * 24 + "cb0404" + "00" * 5),
    (0x03123456, "5634120000000000000000000000000000000000000000000000000000000000"),
])
def test_target_from_nbits(nbits, hexle):
    assert H.target_from_nbits(nbits).hex() == hexle


@pytest.mark.parametrize("bad", [0x1D80FFFF, 0x02123456, 0x1D000000, 0x22FFFFFF])
def test_target_from_nbits_rejects(bad):
    with pytest.raises(H.TargetError):
        H.target_from_nbits(bad)


@pytest.mark.parametrize("nbits", [0x1D00FFFF, 0x1B0404CB, 0x1703A30C, 0x207FFFFF, 0x04123456])
def test_nbits_roundtrip(nbits):
    assert H.nbits_from_target(H.target_from_nbits(nbits)) == nbits


def test_nbits_sign_padding():
    # 0x80 high byte needs a zero pad and a bumped exponent
    t = H.int_to_hash(0x80 << 200)
    nb = H.nbits_from_target(t)
    assert nb & 0x00800000 == 0
    assert H.target_from_nbits(nb) == t
    assert H.nbits_from_target(bytes(32)) == 0


def test_difficulty_one_equals_nbits_1d00ffff():
    assert H.target_from_difficulty(1) == H.target_from_nbits(0x1D00FFFF)


def test_fractional_difficulty():
    t = H.target_from_difficulty(0.001)
    # float64(0.001) is not exactly 1/1000 (same as the reference big.Float path)
    assert abs(H.hash_to_int(t) - (0xFFFF << 208) * 1000) < (0xFFFF << 208) * 1000 * 1e-15
    assert H.hash_to_int(H.target_from_difficulty(0.5)) == (0xFFFF << 208) * 2
    assert math.isclose(H.difficulty_from_target(t), 0.001)


@pytest.mark.parametrize("bad", [0, -1, float("inf"), float("nan")])
def test_difficulty_rejects(bad):
    with pytest.raises(H.TargetError):
        H.target_from_difficulty(bad)


def test_less_or_equal_and_meets_target():
    a = H.int_to_hash(5)
    b = H.int_to_hash(6)
    assert H.less_or_equal(a, b)
    assert H.less_or_equal(a, a)
    assert not H.less_or_equal(b, a)
    g = H.hash_header(bytes.fromhex(H.GENESIS_HEADER_HEX))
    assert H.meets_target(g, 0x1D00FFFF)
    assert not H.meets_target(g, 0x1800FFFF)
