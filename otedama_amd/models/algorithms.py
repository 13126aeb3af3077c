"""Proof-of-work algorithm families ("models") supported by the framework.

Each family defines the header hash (a CPU oracle used for pool-side share
validation and for testing the GPU kernels), its share-difficulty-1 target and
the gfx950 search op that mines it.

  sha256d  Bitcoin double SHA-256      reference: internal/miner/sha256d.go:107-117
  scrypt   Litecoin scrypt(1024,1,1)   [NO REFERENCE CODE] (removed in v3, CHANGELOG.md:6623)
  x11      Dash 11-hash chain          not offered (no validatable known-answer source; see ALGORITHMS)
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from typing import Callable

from otedama_amd.models.header import DIFF1_TARGET_INT, sha256d


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
    # X11 (Dash) is not offered: its eleven 512-bit hashes have no offline known-answer source here, so a
    # kernel could not be validated. Asking for it fails in get() with a clear error.
}


def get(name: str) -> PowAlgorithm:
    try:
        return ALGORITHMS[name.lower()]
    except KeyError:
        raise ValueError(f"unknown algorithm {name!r}; known: {', '.join(ALGORITHMS)}") from None
