"""BIP-39 entropy / mnemonic / seed derivation and the public seed fingerprint.

Parity: internal/lightning/seed.go
  * entropy sizes 128..256 step 32, default 256 ........... seed.go:67-117
  * WordList (exactly 2048 unique words, index lookup) ..... seed.go:121-166
  * EntropyToMnemonic / MnemonicToEntropy (checksum) ....... seed.go:187-278
  * MnemonicToSeed: PBKDF2-HMAC-SHA512 x2048, salt
    "mnemonic"+passphrase ................................. seed.go:295-303
  * Fingerprint = hex(HMAC-SHA256("otedama-fingerprint-v1", seed)[:4]) .. seed.go:313-317
The English list ships as data (bip39_english.txt, the canonical bitcoin/bips
file) and is pinned by its well-known SHA-256 at load time.
"""
from __future__ import annotations

import hashlib
import hmac
import os
import unicodedata
from functools import lru_cache
from pathlib import Path
from typing import BinaryIO, Callable

DEFAULT_ENTROPY_BITS = 256
VALID_ENTROPY_BITS = (128, 160, 192, 224, 256)
ENGLISH_SHA256 = "2f5eed53a4727b4bf8880d8f3f199efc90e58503646d9ff8eff3a2ed3b24dbda"
FINGERPRINT_KEY = b"otedama-fingerprint-v1"
SEED_BYTES = 64


class SeedError(ValueError):
    pass


Reader = Callable[[int], bytes]


def _read_exact(reader: Reader | BinaryIO | None, n: int) -> bytes:
    if reader is None:
        return os.urandom(n)
    fn = reader.read if hasattr(reader, "read") else reader
    out = b""
    while len(out) < n:
        chunk = fn(n - len(out))
        if not chunk:
            raise SeedError(f"lightning: entropy source exhausted after {len(out)} of {n} bytes")
        out += chunk
    return out


def generate_entropy(bits: int = DEFAULT_ENTROPY_BITS, reader: Reader | BinaryIO | None = None) -> bytes:
    if bits not in VALID_ENTROPY_BITS:
        raise SeedError(f"lightning: invalid entropy size {bits} bits (want one of {VALID_ENTROPY_BITS})")
    return _read_exact(reader, bits // 8)


def validate_entropy(e: bytes) -> None:
    if len(e) * 8 not in VALID_ENTROPY_BITS:
        raise SeedError(f"lightning: invalid entropy length {len(e)} bytes")


class WordList:
    def __init__(self, words: list[str]):
        if len(words) != 2048:
            raise SeedError(f"lightning: wordlist has {len(words)} words, need 2048")
        index: dict[str, int] = {}
        for i, w in enumerate(words):
            if not isinstance(w, str) or not w:
                raise SeedError(f"lightning: wordlist entry {i} is empty")
            try:
                w.encode("utf-8")
            except UnicodeEncodeError:  # lone surrogates, e.g. bytes decoded with surrogateescape
                raise SeedError(f"lightning: wordlist entry at index {i} is not valid UTF-8") from None
            if w in index:
                raise SeedError(f"lightning: wordlist contains duplicate word {w!r}")
            index[w] = i
        self._words = list(words)
        self._index = index

    def word(self, i: int) -> str:
        if not 0 <= i < 2048:
            raise SeedError(f"lightning: word index {i} out of range")
        return self._words[i]

    def index(self, word: str) -> int:
        try:
            return self._index[word]
        except KeyError:
            raise SeedError(f"lightning: word {word!r} not in wordlist") from None

    def __len__(self) -> int:
        return 2048


@lru_cache(maxsize=1)
def english_wordlist() -> WordList:
    raw = (Path(__file__).with_name("bip39_english.txt")).read_bytes()
    got = hashlib.sha256(raw).hexdigest()
    if got != ENGLISH_SHA256:
        raise SeedError(f"lightning: BIP-39 wordlist integrity check failed: {got}")
    return WordList(raw.decode().rstrip("\n").split("\n"))


def entropy_to_mnemonic(e: bytes, wl: WordList | None = None) -> list[str]:
    """BIP-39 words for `e`; `wl` defaults to the pinned English list (the reference requires a non-nil list)."""
    validate_entropy(e)
    wl = wl or english_wordlist()
    ent = len(e) * 8
    cs = ent // 32
    v = (int.from_bytes(e, "big") << cs) | (hashlib.sha256(e).digest()[0] >> (8 - cs))
    n = (ent + cs) // 11
    return [wl.word((v >> (11 * (n - 1 - i))) & 0x7FF) for i in range(n)]


def mnemonic_to_entropy(words: list[str] | str, wl: WordList | None = None) -> bytes:
    if isinstance(words, str):
        words = words.split()
    wl = wl or english_wordlist()
    n = len(words)
    if n == 0:
        raise SeedError("lightning: mnemonic is empty")
    if n not in (12, 15, 18, 21, 24):
        raise SeedError(f"lightning: mnemonic has {n} words (want 12, 15, 18, 21 or 24)")
    v = 0
    for i, w in enumerate(words):
        try:
            v = (v << 11) | wl.index(w)
        except SeedError as exc:
            raise SeedError(f"lightning: word {i}: {exc}") from None
    total = n * 11
    cs = total // 33
    ent = total - cs
    e = (v >> cs).to_bytes(ent // 8, "big")
    if (v & ((1 << cs) - 1)) != hashlib.sha256(e).digest()[0] >> (8 - cs):
        raise SeedError("lightning: mnemonic checksum mismatch; check for transcription errors")
    return e


def mnemonic_to_seed(words: list[str] | str, passphrase: str = "") -> bytes:
    phrase = words if isinstance(words, str) else " ".join(words)
    pw = unicodedata.normalize("NFKD", phrase).encode()
    salt = unicodedata.normalize("NFKD", "mnemonic" + passphrase).encode()
    return hashlib.pbkdf2_hmac("sha512", pw, salt, 2048, SEED_BYTES)


def fingerprint(seed: bytes) -> str:
    return hmac.new(FINGERPRINT_KEY, seed, hashlib.sha256).digest()[:4].hex()
