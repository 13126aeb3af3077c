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


# Published known answers: (80-byte header hex, nonce, hash in display order). Bitcoin and Dash main-net
# genesis blocks; the scrypt oracle is cross-checked against hashlib.scrypt instead (no published PoW hash).
KNOWN_ANSWERS: dict[str, tuple[str, int, str]] = {
    "sha256d": ("0100000000000000000000000000000000000000000000000000000000000000000000003ba3edfd7a7b12b27ac72c3e"
                "67768f617fc81bc3888a51323a9fb8aa4b1e5e4a29ab5f49ffff001d1dac2b7c", 2083236893,
                "000000000019d6689c085ae165831e934ff763ae46a2a6c172b3f1b60a8ce26f"),
    "x11": ("010000000000000000000000000000000000000000000000000000000000000000000000c762a6567f3cc092f0684bb6"
            "2b7e00a84890b990f07cc71a6bb58d64b98e02e0022ddb52f0ff0f1ec23fb901", 28917698,
            "00000ffd590b1485b3caadc19b22e6379c733355108f107a430458cdf3407ab6"),
}


def self_test(name: str) -> str:
    """Run the CPU oracle of `name` against its known answer; returns a short description, raises on mismatch."""
    algo = get(name)
    if algo.name in KNOWN_ANSWERS:
        hdr_hex, _nonce, want = KNOWN_ANSWERS[algo.name]
        got = algo.hash(bytes.fromhex(hdr_hex))[::-1].hex()
        if got != want:
            raise AssertionError(f"{algo.name}: genesis hash {got} != published {want}")
        return f"{algo.name} CPU oracle reproduces the published genesis hash"
    hdr = bytes(range(80))
    ref = hashlib.scrypt(hdr, salt=hdr, n=1024, r=1, p=1, dklen=32)
    from otedama_amd.ops.native import load

    n = load(build_if_missing=False)
    if n is not None and n.scrypt_1024_1_1(hdr) != ref:
        raise AssertionError("scrypt: native C++ scrypt != hashlib.scrypt")
    return "scrypt native C++ oracle == hashlib.scrypt"


def get(name: str) -> PowAlgorithm:
    try:
        return ALGORITHMS[name.lower()]
    except KeyError:
        raise ValueError(f"unknown algorithm {name!r}; known: {', '.join(ALGORITHMS)}") from None
