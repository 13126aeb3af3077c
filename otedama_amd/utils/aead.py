"""AES-256-GCM / ChaCha20-Poly1305 through OpenSSL's EVP interface.

Used by the wallet seed store (internal/lightning/seedstore.go:80-164) and the
Noise transport (stratum/noise.go:211-249). Output is ciphertext || 16-byte tag.

Two bindings of the same library: the native extension's (``cpu/aead.cpp``) when the extension is already in the
process (the pool, a CPU miner), else libcrypto through ctypes. A GPU-free engine (its GPUs run in device
processes) must not load the extension just to encrypt a few Noise frames a second: the extension links the HIP
runtime, ~1.4 s to page in on a cold GPU host (profiles/r3/k_startup).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import threading

AES256GCM = 0
CHACHA20POLY1305 = 1
TAG_BYTES = 16

_CTRL_SET_IVLEN = 0x9
_CTRL_GET_TAG = 0x10
_CTRL_SET_TAG = 0x11


class _LibCrypto:
    def __init__(self, lib):
        self.lib = lib
        vp, ip, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
        lib.EVP_CIPHER_CTX_new.restype = vp
        lib.EVP_CIPHER_CTX_new.argtypes = []
        lib.EVP_CIPHER_CTX_free.argtypes = [vp]
        lib.EVP_aes_256_gcm.restype = vp
        lib.EVP_chacha20_poly1305.restype = vp
        for fn in (lib.EVP_EncryptInit_ex, lib.EVP_DecryptInit_ex):
            fn.argtypes = [vp, vp, vp, cp, cp]
            fn.restype = ip
        for fn in (lib.EVP_EncryptUpdate, lib.EVP_DecryptUpdate):
            fn.argtypes = [vp, cp, ctypes.POINTER(ip), cp, ip]
            fn.restype = ip
        for fn in (lib.EVP_EncryptFinal_ex, lib.EVP_DecryptFinal_ex):
            fn.argtypes = [vp, cp, ctypes.POINTER(ip)]
            fn.restype = ip
        lib.EVP_CIPHER_CTX_ctrl.argtypes = [vp, ip, ip, vp]
        lib.EVP_CIPHER_CTX_ctrl.restype = ip
        self.ciphers = {AES256GCM: lib.EVP_aes_256_gcm(), CHACHA20POLY1305: lib.EVP_chacha20_poly1305()}

    def _ctx(self, kind: int, key: bytes, nonce: bytes, encrypt: bool):
        lib = self.lib
        if kind not in self.ciphers or len(key) != 32:
            raise ValueError(f"aead: bad cipher {kind} or key length {len(key)}")
        init = lib.EVP_EncryptInit_ex if encrypt else lib.EVP_DecryptInit_ex
        ctx = lib.EVP_CIPHER_CTX_new()
        if not ctx:
            raise MemoryError("aead: EVP_CIPHER_CTX_new")
        ok = (init(ctx, self.ciphers[kind], None, None, None) == 1
              and lib.EVP_CIPHER_CTX_ctrl(ctx, _CTRL_SET_IVLEN, len(nonce), None) == 1
              and init(ctx, None, None, key, nonce) == 1)
        if not ok:
            lib.EVP_CIPHER_CTX_free(ctx)
            raise ValueError("aead: cipher initialisation failed")
        return ctx

    def seal(self, kind: int, key: bytes, nonce: bytes, plain: bytes, aad: bytes) -> bytes:
        lib = self.lib
        ctx = self._ctx(kind, key, nonce, True)
        try:
            n = ctypes.c_int(0)
            if aad and lib.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) != 1:
                raise ValueError("aead: aad")
            out = ctypes.create_string_buffer(len(plain) + 16)
            if lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), plain, len(plain)) != 1:
                raise ValueError("aead: encrypt")
            total = n.value
            tail = ctypes.create_string_buffer(16)
            if lib.EVP_EncryptFinal_ex(ctx, tail, ctypes.byref(n)) != 1:
                raise ValueError("aead: final")
            tag = ctypes.create_string_buffer(TAG_BYTES)
            if lib.EVP_CIPHER_CTX_ctrl(ctx, _CTRL_GET_TAG, TAG_BYTES, tag) != 1:
                raise ValueError("aead: tag")
            return out.raw[:total] + tail.raw[:n.value] + tag.raw
        finally:
            lib.EVP_CIPHER_CTX_free(ctx)

    def open_(self, kind: int, key: bytes, nonce: bytes, sealed: bytes, aad: bytes) -> bytes | None:
        if len(sealed) < TAG_BYTES:
            return None
        lib = self.lib
        ct, tag = sealed[:-TAG_BYTES], sealed[-TAG_BYTES:]
        ctx = self._ctx(kind, key, nonce, False)
        try:
            n = ctypes.c_int(0)
            if aad and lib.EVP_DecryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) != 1:
                return None
            out = ctypes.create_string_buffer(len(ct) + 16)
            if lib.EVP_DecryptUpdate(ctx, out, ctypes.byref(n), ct, len(ct)) != 1:
                return None
            total = n.value
            tag_buf = ctypes.create_string_buffer(tag, TAG_BYTES)
            if lib.EVP_CIPHER_CTX_ctrl(ctx, _CTRL_SET_TAG, TAG_BYTES, tag_buf) != 1:
                return None
            tail = ctypes.create_string_buffer(16)
            if lib.EVP_DecryptFinal_ex(ctx, tail, ctypes.byref(n)) != 1:
                return None  # authentication failed
            return out.raw[:total] + tail.raw[:n.value]
        finally:
            lib.EVP_CIPHER_CTX_free(ctx)


_lock = threading.Lock()
_libcrypto: _LibCrypto | None = None
_libcrypto_tried = False


def libcrypto() -> _LibCrypto | None:
    global _libcrypto, _libcrypto_tried
    with _lock:
        if not _libcrypto_tried:
            _libcrypto_tried = True
            for name in (ctypes.util.find_library("crypto"), "libcrypto.so.3", "libcrypto.so"):
                if not name:
                    continue
                try:
                    _libcrypto = _LibCrypto(ctypes.CDLL(name))
                    break
                except (OSError, AttributeError):
                    continue
        return _libcrypto


def _backend():
    from otedama_amd.ops.native import loaded, require_native

    mod = loaded()
    if mod is not None:
        return mod.aead_seal, mod.aead_open
    lc = libcrypto()
    if lc is not None:
        return lc.seal, lc.open_
    mod = require_native()
    return mod.aead_seal, mod.aead_open


def seal(kind: int, key: bytes, nonce: bytes, plain: bytes, aad: bytes = b"") -> bytes:
    return _backend()[0](kind, bytes(key), bytes(nonce), bytes(plain), bytes(aad))


def open_(kind: int, key: bytes, nonce: bytes, sealed: bytes, aad: bytes = b"") -> bytes | None:
    """Returns the plaintext, or None when authentication fails."""
    return _backend()[1](kind, bytes(key), bytes(nonce), bytes(sealed), bytes(aad))
