"""Seed encryption at rest: scrypt(N=2^17, r=8, p=1) → AES-256-GCM.

Parity: internal/lightning/seedstore.go
  * format: version(1)=0x01 ‖ salt(16) ‖ nonce(12) ‖ ciphertext‖tag ..... seedstore.go:12-17,51-56
  * scrypt parameters N=2^17 r=8 p=1, 32-byte key ..................... seedstore.go:68-72
  * EncryptSeed (non-empty passphrase, random salt then nonce) ......... seedstore.go:80-118
  * DecryptSeed (opaque ErrWrongPassphrase on auth failure, 64-byte
    plaintext check) ................................................... seedstore.go:125-164
  * Marshal / Unmarshal (min length 29, version check) ................ seedstore.go:180-208
Files written here decrypt with the reference and vice versa (same KDF, same
GCM nonce/tag layout). The AES-GCM itself runs in the native extension.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

from otedama_amd.lightning.seed import SEED_BYTES, Reader, SeedError, _read_exact
from otedama_amd.utils import aead

VERSION = 0x01
SCRYPT_N = 1 << 17
SCRYPT_R = 8
SCRYPT_P = 1
_MIN_LEN = 1 + 16 + 12


class WrongPassphrase(SeedError):
    def __init__(self):
        super().__init__("lightning: decryption failed (wrong passphrase or corrupted file)")


@dataclass
class EncryptedSeed:
    version: int
    salt: bytes
    nonce: bytes
    ciphertext: bytes

    def marshal(self) -> bytes:
        if self.version != VERSION:
            raise SeedError(f"lightning: Marshal: unsupported version {self.version}")
        return bytes([self.version]) + self.salt + self.nonce + self.ciphertext


def unmarshal(b: bytes) -> EncryptedSeed:
    if len(b) < _MIN_LEN:
        raise SeedError(f"lightning: EncryptedSeed too short: {len(b)} bytes, need at least {_MIN_LEN}")
    if b[0] != VERSION:
        raise SeedError(f"lightning: unsupported EncryptedSeed version {b[0]}")
    return EncryptedSeed(b[0], bytes(b[1:17]), bytes(b[17:29]), bytes(b[29:]))


def derive_key(passphrase: str, salt: bytes) -> bytes:
    return hashlib.scrypt(passphrase.encode(), salt=salt, n=SCRYPT_N, r=SCRYPT_R, p=SCRYPT_P,
                          maxmem=256 * 1024 * 1024, dklen=32)


def encrypt_seed(seed: bytes, passphrase: str, reader: Reader | None = None) -> EncryptedSeed:
    if not passphrase:
        raise SeedError("lightning: passphrase must not be empty")
    try:
        salt = _read_exact(reader, 16)
    except SeedError as exc:
        raise SeedError(f"lightning: salt generation failed: {exc}") from exc
    try:
        nonce = _read_exact(reader, 12)
    except SeedError as exc:
        raise SeedError(f"lightning: nonce generation failed: {exc}") from exc
    key = derive_key(passphrase, salt)
    return EncryptedSeed(VERSION, salt, nonce, aead.seal(aead.AES256GCM, key, nonce, seed))


def decrypt_seed(es: EncryptedSeed, passphrase: str) -> bytes:
    if es.version != VERSION:
        raise SeedError(f"lightning: unsupported EncryptedSeed version {es.version}")
    if not es.ciphertext:
        raise SeedError("lightning: EncryptedSeed has empty ciphertext")
    key = derive_key(passphrase, es.salt)
    plain = aead.open_(aead.AES256GCM, key, es.nonce, es.ciphertext)
    if plain is None:
        raise WrongPassphrase()
    if len(plain) != SEED_BYTES:
        raise SeedError(f"lightning: decrypted seed is {len(plain)} bytes, want {SEED_BYTES}")
    return plain
