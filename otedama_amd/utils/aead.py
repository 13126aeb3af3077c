"""AES-256-GCM / ChaCha20-Poly1305 through the native extension (OpenSSL EVP).

Used by the wallet seed store (internal/lightning/seedstore.go:80-164) and the
Noise transport (stratum/noise.go:211-249). Output is ciphertext || 16-byte tag.
"""
from __future__ import annotations

AES256GCM = 0
CHACHA20POLY1305 = 1
TAG_BYTES = 16


def _native():
    from otedama_amd.ops.native import require_native

    return require_native()


def seal(kind: int, key: bytes, nonce: bytes, plain: bytes, aad: bytes = b"") -> bytes:
    return _native().aead_seal(kind, bytes(key), bytes(nonce), bytes(plain), bytes(aad))


def open_(kind: int, key: bytes, nonce: bytes, sealed: bytes, aad: bytes = b"") -> bytes | None:
    """Returns the plaintext, or None when authentication fails."""
    return _native().aead_open(kind, bytes(key), bytes(nonce), bytes(sealed), bytes(aad))
