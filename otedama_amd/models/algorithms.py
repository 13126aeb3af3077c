"""Proof-of-work algorithm families ("models") supported by the framework.

Each family defines the header hash (a CPU oracle used for pool-side share
validation and for testing the GPU kernels), its share-difficulty-1 target and
the gfx950 search op that mines it.

  sha256d  Bitcoin double SHA-256      reference: internal/miner/sha256d.go:107-117
  scrypt   Litecoin scrypt(1024,1,1)   [NO REFERENCE CODE] (removed in v3, CHANGELOG.md:6623)
  x11      Dash 11-hash chain          [NO REFERENCE CODE] (never implemented upstream); CPU oracle
                                       csrc/cpu/x11_cpu.cpp, pinned by the Dash genesis block
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from typing import Callable

from otedama_amd.models.header import DIFF1_TARGET_INT, sha256d


def x11_hash(header80: bytes) -> bytes:
    """X11 = first 32 bytes of ECHO(SIMD(...BLAKE-512(header))) via the native CPU chain."""
    from otedama_amd.ops.native import require_native

    return require_native().x11(bytes(header80))


def scrypt_hash(header80: bytes) -> bytes:
    """scrypt(N=1024, r=1, p=1, dkLen=32) with password = salt = header."""
    return hashlib.scrypt(header80, salt=header80, n=1024, r=1, p=1, dklen=32)


@dataclass(frozen=True)
class PowAlgorithm:
    name: str
    diff1: int                       # share difficulty-1 target as an integer
    hash: Callable[[bytes], bytes]   # CPU oracle: 80-byte header -> 32-byte LE hash
    gpu: bool                        # has a gfx950 search kernel
    description: str


ALGORITHMS: dict[str, PowAlgorithm] = {
    "sha256d": PowAlgorithm("sha256d", DIFF1_TARGET_INT, sha256d, True, "Bitcoin SHA-256d"),
    # Litecoin-family pools define share difficulty 1 as 2^16 easier than Bitcoin's.
    "scrypt": PowAlgorithm("scrypt", 0xFFFF << 224, scrypt_hash, True, "Litecoin scrypt N=1024 r=1 p=1"),
    # Dash (X11) pools use the Bitcoin difficulty-1 target. The CPU chain reproduces the Dash genesis
    # block hash (tests/test_x11_kat.py); the gfx950 kernels are checked stage by stage against it.
    "x11": PowAlgorithm("x11", DIFF1_TARGET_INT, x11_hash, True, "Dash X11 (11 chained 512-bit hashes)"),
}


def get(name: str) -> PowAlgorithm:
    try:
        return ALGORITHMS[name.lower()]
    except KeyError:
        raise ValueError(f"unknown algorithm {name!r}; known: {', '.join(ALGORITHMS)}") from None
