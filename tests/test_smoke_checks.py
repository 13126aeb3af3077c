"""smoke()'s oracle comparisons: they pass on correct kernel output and FAIL on corrupted output.

The scrypt check rebuilds digests from the kernel's post-ROMix state; here that state comes from a pure-Python
ROMix (RFC 7914 §5), so the test also pins the formula digest = PBKDF2-HMAC-SHA256(header, B', 1, 32).
"""
import hashlib
import struct

import pytest

from otedama_amd.ops.smoke_checks import check_scrypt_window, check_sha256d_window, scrypt_digest_from_state

HDR76 = bytes(range(76))
QUARTER = (1 << 254) - 1


def _salsa20_8(b: list[int]) -> list[int]:
    x = list(b)

    def r(a, n):
        return ((a << n) | (a >> (32 - n))) & 0xFFFFFFFF

    for _ in range(4):
        for (o, i1, i2, s) in ((4, 0, 12, 7), (8, 4, 0, 9), (12, 8, 4, 13), (0, 12, 8, 18),
                               (9, 5, 1, 7), (13, 9, 5, 9), (1, 13, 9, 13), (5, 1, 13, 18),
                               (14, 10, 6, 7), (2, 14, 10, 9), (6, 2, 14, 13), (10, 6, 2, 18),
                               (3, 15, 11, 7), (7, 3, 15, 9), (11, 7, 3, 13), (15, 11, 7, 18),
                               (1, 0, 3, 7), (2, 1, 0, 9), (3, 2, 1, 13), (0, 3, 2, 18),
                               (6, 5, 4, 7), (7, 6, 5, 9), (4, 7, 6, 13), (5, 4, 7, 18),
                               (11, 10, 9, 7), (8, 11, 10, 9), (9, 8, 11, 13), (10, 9, 8, 18),
                               (12, 15, 14, 7), (13, 12, 15, 9), (14, 13, 12, 13), (15, 14, 13, 18)):
            x[o] ^= r((x[i1] + x[i2]) & 0xFFFFFFFF, s)
    return [(x[i] + b[i]) & 0xFFFFFFFF for i in range(16)]


def _romix_state(header80: bytes) -> bytes:
    """B' = ROMix(PBKDF2(header, header, 1, 128)) for N=1024, r=1 (little-endian words)."""
    B = hashlib.pbkdf2_hmac("sha256", header80, header80, 1, 128)
    X = list(struct.unpack("<32I", B))

    def blockmix(X):
        a = _salsa20_8([X[16 + k] ^ X[k] for k in range(16)])
        b = _salsa20_8([X[16 + k] ^ a[k] for k in range(16)])
        return a + b

    V = []
    for _ in range(1024):
        V.append(X)
        X = blockmix(X)
    for _ in range(1024):
        j = X[16] & 1023
        X = blockmix([X[k] ^ V[j][k] for k in range(32)])
    return struct.pack("<32I", *X)


def _oracle_hits(base, count, target):
    out = []
    for i in range(count):
        h = HDR76 + (base + i).to_bytes(4, "little")
        if int.from_bytes(hashlib.scrypt(h, salt=h, n=1024, r=1, p=1, dklen=32), "little") <= target:
            out.append(base + i)
    return out


def test_digest_from_romix_state_matches_hashlib():
    h = HDR76 + (7).to_bytes(4, "little")
    x = _romix_state(h)
    assert scrypt_digest_from_state(h, x) == hashlib.scrypt(h, salt=h, n=1024, r=1, p=1, dklen=32)


def test_scrypt_check_passes_on_correct_output():
    hits = _oracle_hits(100, 16, QUARTER)
    xbuf = b"".join(_romix_state(HDR76 + (100 + i).to_bytes(4, "little")) for i in range(2))
    r = check_scrypt_window(HDR76, 100, 16, QUARTER, hits, xbuf, digest_lanes=2)
    assert r["hits"] == len(hits) and r["digests_checked"] == 2


def test_scrypt_check_fails_on_a_missing_or_extra_hit():
    hits = _oracle_hits(100, 16, QUARTER)
    assert hits, "seed window has no hit"
    with pytest.raises(AssertionError, match="missing"):
        check_scrypt_window(HDR76, 100, 16, QUARTER, hits[1:])
    extra = next(n for n in range(100, 116) if n not in hits)
    with pytest.raises(AssertionError, match="extra"):
        check_scrypt_window(HDR76, 100, 16, QUARTER, hits + [extra])


def test_scrypt_check_fails_on_a_corrupted_state():
    hits = _oracle_hits(100, 16, QUARTER)
    x = bytearray(_romix_state(HDR76 + (100).to_bytes(4, "little")))
    x[5] ^= 0x01  # one flipped bit in the kernel's ROMix output
    with pytest.raises(AssertionError, match="digest of nonce 100"):
        check_scrypt_window(HDR76, 100, 16, QUARTER, hits, bytes(x), digest_lanes=1)


def test_sha256d_check():
    want = []
    for n in range(0, 512):
        d = hashlib.sha256(hashlib.sha256(HDR76 + n.to_bytes(4, "little")).digest()).digest()
        if int.from_bytes(d, "little") <= QUARTER:
            want.append(n)
    assert check_sha256d_window(HDR76, 0, 512, QUARTER, want) == len(want)
    with pytest.raises(AssertionError):
        check_sha256d_window(HDR76, 0, 512, QUARTER, want[:-1])
