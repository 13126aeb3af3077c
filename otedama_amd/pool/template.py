"""Block templates, coinbase construction and merkle branches for the local pool.

[NO REFERENCE CODE] — v3 of the reference removed pool operator mode
(CHANGELOG.md:6623-6624) and its V1 client never builds a coinbase
(poolproto/stratumv1/parse.go:52-54,91). This module is the pool half of the
coinbase / merkle work: a BIP34 coinbase paying the operator's
address, split around the extranonce for Stratum V1 (coinb1 | en1 | en2 | coinb2),
and fixed merkle roots for Stratum V2 standard channels (one extranonce prefix
per channel).

No bitcoind is available offline, so templates are synthetic: a random or
chained prev-hash, a configurable nBits, and optional fake transaction ids
(to exercise merkle branches of realistic depth).
"""
from __future__ import annotations

import hashlib
import os
import struct
import time
from dataclasses import dataclass, field

from otedama_amd import btccrypto
from otedama_amd.models.header import sha256d


def varint(n: int) -> bytes:
    if n < 0xFD:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    if n <= 0xFFFFFFFF:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def script_num(n: int) -> bytes:
    """Minimal CScriptNum push (BIP34 height)."""
    if n == 0:
        return b"\x00"
    out = bytearray()
    v = abs(n)
    while v:
        out.append(v & 0xFF)
        v >>= 8
    if out[-1] & 0x80:
        out.append(0x80 if n < 0 else 0)
    elif n < 0:
        out[-1] |= 0x80
    return bytes([len(out)]) + bytes(out)


def merkle_branches(txids: list[bytes]) -> list[bytes]:
    """Branches for the coinbase (index 0) given the other txids (internal byte order)."""
    branches = []
    level = [None] + list(txids)  # None = coinbase placeholder (always index 0)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        branches.append(level[1])
        level = [None] + [sha256d(level[i] + level[i + 1]) for i in range(2, len(level), 2)]
    return branches


def merkle_root_from_branches(coinbase_txid: bytes, branches: list[bytes]) -> bytes:
    root = coinbase_txid
    for b in branches:
        root = sha256d(root + b)
    return root


def merkle_root_full(txids: list[bytes]) -> bytes:
    level = list(txids)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        level = [sha256d(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
    return level[0]


@dataclass
class BlockTemplate:
    height: int
    prev_hash: bytes            # header byte order
    version: int
    nbits: int
    ntime: int
    coinbase_value: int         # satoshis
    payout_script: bytes
    txids: list[bytes] = field(default_factory=list)
    coinbase_message: bytes = b"/otedama-mi355x/"

    def coinbase_parts(self, extranonce_size: int) -> tuple[bytes, bytes]:
        """(coinb1, coinb2) around an `extranonce_size`-byte extranonce (en1 + en2)."""
        script_prefix = script_num(self.height) + bytes([len(self.coinbase_message)]) + self.coinbase_message
        script_len = len(script_prefix) + extranonce_size
        if script_len > 100:
            raise ValueError("coinbase scriptSig too long")
        coinb1 = (struct.pack("<I", 1)            # tx version
                  + b"\x01"                        # 1 input
                  + bytes(32) + b"\xff\xff\xff\xff"  # null prevout
                  + varint(script_len) + script_prefix)
        coinb2 = (b"\xff\xff\xff\xff"              # sequence
                  + b"\x01"                        # 1 output
                  + struct.pack("<Q", self.coinbase_value)
                  + varint(len(self.payout_script)) + self.payout_script
                  + b"\x00\x00\x00\x00")           # locktime
        return coinb1, coinb2

    def branches(self) -> list[bytes]:
        return merkle_branches(self.txids)

    def merkle_root(self, coinbase: bytes) -> bytes:
        return merkle_root_from_branches(sha256d(coinbase), self.branches())


class TemplateSource:
    """Synthetic chain: each new block gets a fresh prev-hash and height."""

    def __init__(self, payout_address: str | None, nbits: int = 0x1703A30C, n_txs: int = 0,
                 coinbase_message: str = "/otedama-mi355x/", seed: bytes | None = None):
        if payout_address:
            self.payout_script = btccrypto.address_script_pubkey(payout_address)
        else:
            self.payout_script = b"\x6a"  # OP_RETURN (burn) when no operator address is configured
        self.nbits = nbits
        self.n_txs = n_txs
        self.msg = coinbase_message.encode()[:40]
        self.height = 900_000
        self._prev = hashlib.sha256(seed or os.urandom(32)).digest()

    def next_block(self) -> BlockTemplate:
        self.height += 1
        self._prev = sha256d(self._prev + struct.pack("<I", self.height))
        txids = [sha256d(self._prev + struct.pack("<I", i)) for i in range(self.n_txs)]
        subsidy = 312_500_000  # 3.125 BTC (provider/mining.go:84)
        return BlockTemplate(height=self.height, prev_hash=self._prev, version=0x20000000, nbits=self.nbits,
                             ntime=int(time.time()), coinbase_value=subsidy, payout_script=self.payout_script,
                             txids=txids, coinbase_message=self.msg)
