"""Oracle comparisons the driver's smoke() runs on the GPU's output.

Each check takes what the kernel produced (hit nonces, and for scrypt the post-ROMix state the kernel leaves in its
exchange buffer) and compares it with the CPU oracle over the same window: ``hashlib.scrypt`` for scrypt, hashlib
SHA-256d for SHA-256d. A mismatch raises AssertionError with the differing nonces, so a corrupted kernel fails smoke
instead of passing on "some nonces came back". The known-answer style follows the reference's genesis-header KAT
(internal/miner/sha256d_test.go:24-59).
"""
from __future__ import annotations

import hashlib


def scrypt_digest(header80: bytes) -> bytes:
    return hashlib.scrypt(header80, salt=header80, n=1024, r=1, p=1, dklen=32)


def scrypt_digest_from_state(header80: bytes, x128: bytes) -> bytes:
    """scrypt's last step from the post-ROMix block B (128 bytes, little-endian words, as the kernel stores it):
    PBKDF2-HMAC-SHA256(password = header, salt = B, 1 iteration, 32 bytes)."""
    return hashlib.pbkdf2_hmac("sha256", header80, x128, 1, 32)


def check_scrypt_window(header76: bytes, base: int, count: int, target_int: int, gpu_hits: list[int],
                        xbuf: bytes | None = None, digest_lanes: int = 4) -> dict:
    """The GPU's scrypt hits over nonces [base, base + count) must equal the oracle's, and (with ``xbuf``, the
    kernel's exchange buffer: 128 bytes per lane, lane i = nonce base + i) the digests of the first
    ``digest_lanes`` lanes rebuilt from the kernel's ROMix state must equal hashlib.scrypt's."""
    want, digests = [], {}
    for i in range(count):
        n = (base + i) & 0xFFFFFFFF
        h = header76 + n.to_bytes(4, "little")
        d = scrypt_digest(h)
        digests[n] = d
        if int.from_bytes(d, "little") <= target_int:
            want.append(n)
    got = sorted(x & 0xFFFFFFFF for x in gpu_hits)
    if got != sorted(want):
        raise AssertionError(f"scrypt hits differ from hashlib.scrypt over [{base}, {base + count}): "
                             f"missing {sorted(set(want) - set(got))[:8]}, extra {sorted(set(got) - set(want))[:8]}")
    checked = 0
    if xbuf is not None:
        for i in range(min(digest_lanes, count)):
            n = (base + i) & 0xFFFFFFFF
            got_d = scrypt_digest_from_state(header76 + n.to_bytes(4, "little"), bytes(xbuf[128 * i : 128 * (i + 1)]))
            if got_d != digests[n]:
                raise AssertionError(f"scrypt digest of nonce {n}: kernel state gives {got_d.hex()}, "
                                     f"hashlib.scrypt {digests[n].hex()}")
            checked += 1
    return {"hits": len(want), "window": count, "digests_checked": checked,
            "first_digest": digests[base & 0xFFFFFFFF].hex()}


def check_sha256d_window(header76: bytes, base: int, count: int, target_int: int, gpu_hits: list[int]) -> int:
    """SHA-256d hits over [base, base + count) must equal hashlib's (small windows only: ~1 us per nonce)."""
    want = []
    for i in range(count):
        n = (base + i) & 0xFFFFFFFF
        d = hashlib.sha256(hashlib.sha256(header76 + n.to_bytes(4, "little")).digest()).digest()
        if int.from_bytes(d, "little") <= target_int:
            want.append(n)
    got = sorted(x & 0xFFFFFFFF for x in gpu_hits)
    if got != sorted(want):
        raise AssertionError(f"sha256d hits differ from hashlib over [{base}, {base + count}): "
                             f"missing {sorted(set(want) - set(got))[:8]}, extra {sorted(set(got) - set(want))[:8]}")
    return len(want)
