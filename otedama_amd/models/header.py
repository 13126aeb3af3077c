"""Block header, hash and target math (the PoW "model" data types).

Parity: internal/miner/sha256d.go
  * Header / Bytes / ParseHeader ........ sha256d.go:49-80
  * Hash.LessOrEqual .................... sha256d.go:93-103
  * SHA256d / HashHeader ................ sha256d.go:107-117
  * TargetFromNBits / NBitsFromTarget ... sha256d.go:134-205
  * diff1Target / TargetFromDifficulty .. sha256d.go:211-247
  * MeetsTarget ......................... sha256d.go:251-257

Byte-order convention (same as the reference): hashes and targets are 32-byte
little-endian integers, most-significant byte at index 31.
"""
from __future__ import annotations

import hashlib
import math
import struct
from dataclasses import dataclass, field, replace
from fractions import Fraction

HEADER_SIZE = 80
DIFF1_TARGET_INT = 0xFFFF << 208  # nBits 0x1d00ffff
MAX_TARGET = b"\xff" * 32


class TargetError(ValueError):
    """Malformed nBits / difficulty."""


def sha256d(data: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(data).digest()).digest()


def hash_to_int(h: bytes) -> int:
    return int.from_bytes(h, "little")


def int_to_hash(v: int) -> bytes:
    if v < 0 or v >= 1 << 256:
        raise TargetError("value does not fit in 256 bits")
    return v.to_bytes(32, "little")


def less_or_equal(h: bytes, other: bytes) -> bool:
    """Hash.LessOrEqual: 256-bit LE compare walking from byte 31 down."""
    return hash_to_int(h) <= hash_to_int(other)


def hash_hex(h: bytes) -> str:
    """Hash.String: lowercase hex of the raw (LE) bytes."""
    return h.hex()


@dataclass(frozen=True)
class Header:
    version: int = 0
    prev_hash: bytes = field(default=bytes(32))
    merkle_root: bytes = field(default=bytes(32))
    time: int = 0
    bits: int = 0
    nonce: int = 0

    def to_bytes(self) -> bytes:
        if len(self.prev_hash) != 32 or len(self.merkle_root) != 32:
            raise ValueError("prev_hash and merkle_root must be 32 bytes")
        return (struct.pack("<I", self.version & 0xFFFFFFFF) + bytes(self.prev_hash) + bytes(self.merkle_root)
                + struct.pack("<III", self.time & 0xFFFFFFFF, self.bits & 0xFFFFFFFF, self.nonce & 0xFFFFFFFF))

    @classmethod
    def parse(cls, b: bytes) -> "Header":
        if len(b) != HEADER_SIZE:
            raise ValueError(f"header must be {HEADER_SIZE} bytes, got {len(b)}")
        version, = struct.unpack_from("<I", b, 0)
        t, bits, nonce = struct.unpack_from("<III", b, 68)
        return cls(version, bytes(b[4:36]), bytes(b[36:68]), t, bits, nonce)

    def with_nonce(self, nonce: int) -> "Header":
        return replace(self, nonce=nonce & 0xFFFFFFFF)


def hash_header(h: Header | bytes) -> bytes:
    return sha256d(h.to_bytes() if isinstance(h, Header) else bytes(h))


def target_from_nbits(nbits: int) -> bytes:
    exp = (nbits >> 24) & 0xFF
    mant = nbits & 0x007FFFFF
    if nbits & 0x00800000:
        raise TargetError(f"nBits 0x{nbits:08X} has negative mantissa bit set")
    if exp < 3:
        raise TargetError(f"nBits 0x{nbits:08X} exponent {exp} is below minimum 3")
    if mant == 0:
        raise TargetError(f"nBits 0x{nbits:08X} has zero mantissa (target would be zero; no hash can meet it)")
    v = mant << (8 * (exp - 3))
    if v >= 1 << 256:
        raise TargetError(f"nBits 0x{nbits:08X} target overflows 256 bits")
    return int_to_hash(v)


def nbits_from_target(target: bytes) -> int:
    v = hash_to_int(target)
    if v == 0:
        return 0
    b = v.to_bytes((v.bit_length() + 7) // 8, "big")
    if b[0] & 0x80:
        b = b"\x00" + b
    exp = len(b)
    if len(b) == 1:
        mant = b[0]
    elif len(b) == 2:
        mant = (b[0] << 8) | b[1]
    else:
        mant = (b[0] << 16) | (b[1] << 8) | b[2]
    return (exp << 24) | mant


def target_from_difficulty(difficulty: float, diff1: int = DIFF1_TARGET_INT) -> bytes:
    """target = floor(diff1 / difficulty), exact rational arithmetic."""
    if not isinstance(difficulty, (int, float)) or not (difficulty > 0) or math.isinf(difficulty):
        raise TargetError(f"invalid difficulty {difficulty!r}")
    t = math.floor(Fraction(diff1) / Fraction(difficulty))
    if t <= 0:
        raise TargetError(f"difficulty {difficulty} produces a non-positive target")
    if t >= 1 << 256:
        raise TargetError(f"difficulty {difficulty} target overflows 256 bits")
    return int_to_hash(t)


def difficulty_from_target(target: bytes, diff1: int = DIFF1_TARGET_INT) -> float:
    v = hash_to_int(target)
    if v == 0:
        return math.inf
    return diff1 / v


def meets_target(h: bytes, nbits: int) -> bool:
    return less_or_equal(h, target_from_nbits(nbits))


def hash_difficulty(h: bytes, diff1: int = DIFF1_TARGET_INT) -> float:
    """Share difficulty actually achieved by a hash (diff1 / hash)."""
    v = hash_to_int(h)
    return math.inf if v == 0 else diff1 / v


GENESIS_HEADER_HEX = (
    "01000000" + "00" * 32
    + "3ba3edfd7a7b12b27ac72c3e67768f617fc81bc3888a51323a9fb8aa4b1e5e4a"
    + "29ab5f49" + "ffff001d" + "1dac2b7c"
)
GENESIS_HASH_HEX = "6fe28c0ab6f1b372c1a6a246ae63f74f931e8365e15a089c68d6190000000000"
