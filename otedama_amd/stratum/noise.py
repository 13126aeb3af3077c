"""Noise NX for Stratum V2 (both roles) + encrypted streams, in two suites.

  * ``ellswift`` (default): ``Noise_NX_Secp256k1+EllSwift_ChaChaPoly_SHA256``, the current SV2 suite. Every public
    key on the wire is a 64-byte BIP324 ElligatorSwift encoding (stratum/ellswift.py) and each DH is BIP324's
    x-only ``v2_ecdh`` (tagged hash of initiator encoding ‖ responder encoding ‖ shared x). Message 1 is 64 bytes,
    message 2 is 64 + (64+16) + (payload+16) = 234 bytes with the 74-byte SignatureNoiseMessage.
    Parity UNPINNED: no SV2/BIP324 test vectors are reachable offline; tests pin round trips and both-sides
    agreement (tests/test_ellswift.py).
  * ``legacy``: ``Noise_NX_secp256k1_ChaChaPoly_SHA256`` with 32-byte even-y x-only keys and raw x-coordinate DH
    (round 1-2 wire format, kept for peers that speak it).
The responder tells the suites apart by message 1's length (32 vs 64 bytes); the initiator picks one.

Parity: internal/stratum/noise.go (and noise_pool.go)
  * HandshakeState / CipherState (ChaChaPoly, nonce = 0^4 ‖ LE64(n)) .. noise.go:50-90
  * initialize(protocolName): h = name padded or SHA-256(name), ck = h  noise.go:108-118
  * WriteMessage1 (-> e) / ReadMessage2 ............................... noise.go:121-170
  * mixHash / mixKey / split via HKDF-SHA256 ........................... noise.go:186-249
  * EncryptedConn: u16-LE length-prefixed AEAD frames ≤ 65535, partial
    reads buffered ...................................................... noise.go:255-329
Deliberate differences: the reference is an unwired alpha stub on P-256 that
skips ee/es and never authenticates the pool. This is the full NX pattern
(-> e ; <- e, ee, s, es, payload) on secp256k1 with 32-byte x-only keys
(even-y, BIP-340 style), the responder's static key encrypted under the
handshake hash, and an authenticated payload (e.g. a signed certificate).
DH(k, P) = x-coordinate of k·P (32 bytes). ChaCha20-Poly1305 runs in the
native extension (OpenSSL EVP); the EC arithmetic is host Python (one
handshake per connection).
"""
from __future__ import annotations

import asyncio
import hashlib
import hmac
import os
import struct

from otedama_amd import btccrypto as ec
from otedama_amd.stratum import ellswift
from otedama_amd.utils import aead

PROTOCOL_NAME = b"Noise_NX_secp256k1_ChaChaPoly_SHA256"          # legacy suite
PROTOCOL_NAME_ELLSWIFT = b"Noise_NX_Secp256k1+EllSwift_ChaChaPoly_SHA256"
SUITES = ("ellswift", "legacy")
DEFAULT_SUITE = "ellswift"
MAX_FRAME = 65535
KEY_LEN = 32
TAG = aead.TAG_BYTES


class NoiseError(Exception):
    pass


# ------------------------------------------------------------------ primitives
def hkdf(ck: bytes, ikm: bytes, n: int) -> list[bytes]:
    tk = hmac.new(ck, ikm, hashlib.sha256).digest()
    out, prev = [], b""
    for i in range(1, n + 1):
        prev = hmac.new(tk, prev + bytes([i]), hashlib.sha256).digest()
        out.append(prev)
    return out


def keypair(priv: int | None = None) -> tuple[int, bytes]:
    """Returns (secret, x-only public key); the secret is negated if needed so Y is even."""
    while priv is None or not 0 < priv < ec.N:
        priv = int.from_bytes(os.urandom(32), "big")
    x, y = ec.point_mul(ec.G, priv)
    if y & 1:
        priv = ec.N - priv
    return priv, x.to_bytes(32, "big")


def dh(priv: int, pub_xonly: bytes) -> bytes:
    pt = ec.lift_x(int.from_bytes(pub_xonly, "big"))
    if pt is None:
        raise NoiseError("noise: invalid secp256k1 public key")
    r = ec.point_mul(pt, priv)
    if r is None:
        raise NoiseError("noise: DH produced the point at infinity")
    return r[0].to_bytes(32, "big")


class CipherState:
    def __init__(self, key: bytes | None = None):
        self.k = key
        self.n = 0

    def _nonce(self) -> bytes:
        if self.n >= 2 ** 64 - 1:
            raise NoiseError("noise: nonce exhausted")
        return b"\x00" * 4 + struct.pack("<Q", self.n)

    def encrypt(self, ad: bytes, plain: bytes) -> bytes:
        if self.k is None:
            return plain
        ct = aead.seal(aead.CHACHA20POLY1305, self.k, self._nonce(), plain, ad)
        self.n += 1
        return ct

    def decrypt(self, ad: bytes, ct: bytes) -> bytes:
        if self.k is None:
            return ct
        pt = aead.open_(aead.CHACHA20POLY1305, self.k, self._nonce(), ct, ad)
        if pt is None:
            raise NoiseError("noise: decrypt failed (bad tag)")
        self.n += 1
        return pt


class SymmetricState:
    def __init__(self, name: bytes = PROTOCOL_NAME):
        self.h = name.ljust(32, b"\x00") if len(name) <= 32 else hashlib.sha256(name).digest()
        self.ck = self.h
        self.cs = CipherState()

    def mix_hash(self, data: bytes) -> None:
        self.h = hashlib.sha256(self.h + data).digest()

    def mix_key(self, ikm: bytes) -> None:
        self.ck, k = hkdf(self.ck, ikm, 2)
        self.cs = CipherState(k)

    def encrypt_and_hash(self, plain: bytes) -> bytes:
        ct = self.cs.encrypt(self.h, plain)
        self.mix_hash(ct)
        return ct

    def decrypt_and_hash(self, ct: bytes) -> bytes:
        pt = self.cs.decrypt(self.h, ct)
        self.mix_hash(ct)
        return pt

    def split(self) -> tuple[CipherState, CipherState]:
        k1, k2 = hkdf(self.ck, b"", 2)
        return CipherState(k1), CipherState(k2)


# ------------------------------------------------------------------ handshake
def _suite(suite: str) -> str:
    if suite not in SUITES:
        raise NoiseError(f"noise: unknown suite {suite!r} (want one of {', '.join(SUITES)})")
    return suite


def _ell_keypair(priv: int | None = None) -> tuple[int, bytes]:
    while priv is None or not 0 < priv < ec.N:
        priv = int.from_bytes(os.urandom(32), "big")
    return priv, ellswift.create(priv)


def _ell_xonly(enc: bytes) -> bytes:
    return ellswift.decode(enc).to_bytes(32, "big")


class Initiator:
    """Client side: -> e ; <- e, ee, s, es, payload.

    ``remote_static`` is the responder's 32-byte x-only static key in both suites (what certificates sign and what
    ``expected_static`` pins); ``remote_static_wire`` is the key as it was sent (64-byte ElligatorSwift or 32)."""

    def __init__(self, expected_static: bytes | None = None, prologue: bytes = b"", suite: str = DEFAULT_SUITE):
        self.suite = _suite(suite)
        self.klen = 64 if suite == "ellswift" else 32
        self.ss = SymmetricState(PROTOCOL_NAME_ELLSWIFT if suite == "ellswift" else PROTOCOL_NAME)
        self.ss.mix_hash(prologue)
        self.e, self.e_pub = _ell_keypair() if suite == "ellswift" else keypair()
        self.expected_static = expected_static
        self.remote_static = b""
        self.remote_static_wire = b""
        self.payload = b""
        self.send: CipherState | None = None
        self.recv: CipherState | None = None

    def _dh(self, priv: int, theirs: bytes, ours: bytes) -> bytes:
        if self.suite == "ellswift":
            return ellswift.xdh(priv, theirs, ours, initiating=True)
        return dh(priv, theirs)

    def write_message1(self) -> bytes:
        self.ss.mix_hash(self.e_pub)
        self.ss.mix_hash(b"")  # empty payload, unencrypted (no key yet)
        return self.e_pub

    def read_message2(self, msg: bytes) -> bytes:
        k = self.klen
        if len(msg) < k + k + TAG + TAG:
            raise NoiseError(f"noise: message2 too short ({len(msg)} bytes)")
        re = msg[:k]
        self.ss.mix_hash(re)
        self.ss.mix_key(self._dh(self.e, re, self.e_pub))     # ee
        rs = self.ss.decrypt_and_hash(msg[k:k + k + TAG])     # s
        rs_x = _ell_xonly(rs) if self.suite == "ellswift" else rs
        if self.expected_static is not None and not hmac.compare_digest(rs_x, self.expected_static):
            raise NoiseError("noise: responder static key does not match the pinned key")
        self.ss.mix_key(self._dh(self.e, rs, self.e_pub))     # es
        self.payload = self.ss.decrypt_and_hash(msg[k + k + TAG:])
        self.remote_static, self.remote_static_wire = rs_x, rs
        self.send, self.recv = self.ss.split()
        return self.payload

    @property
    def handshake_hash(self) -> bytes:
        return self.ss.h


class Responder:
    """Pool side, holding the long-term static key. ``suite=None`` accepts either suite, chosen by the length of
    message 1 (64 bytes: ElligatorSwift, 32: legacy); a fixed suite refuses the other."""

    def __init__(self, static_priv: int, prologue: bytes = b"", suite: str | None = None):
        self.suite = _suite(suite) if suite is not None else None
        self.prologue = prologue
        self.static_priv = static_priv
        self.s_xonly = keypair(static_priv)[1]  # what pins and certificates name, in both suites
        self.send: CipherState | None = None
        self.recv: CipherState | None = None
        self.ss: SymmetricState | None = None

    def _dh(self, priv: int, theirs: bytes, ours: bytes) -> bytes:
        if self.suite == "ellswift":
            return ellswift.xdh(priv, theirs, ours, initiating=False)
        return dh(priv, theirs)

    def read_message1(self, msg: bytes) -> None:
        by_len = {64: "ellswift", 32: "legacy"}.get(len(msg))
        if by_len is None or (self.suite is not None and by_len != self.suite):
            want = {"ellswift": "64", "legacy": "32"}.get(self.suite or "", "32 or 64")
            raise NoiseError(f"noise: message1 must be {want} bytes, got {len(msg)}")
        self.suite = by_len
        self.ss = SymmetricState(PROTOCOL_NAME_ELLSWIFT if by_len == "ellswift" else PROTOCOL_NAME)
        self.ss.mix_hash(self.prologue)
        if by_len == "ellswift":
            self.s, self.s_pub = _ell_keypair(self.static_priv)
        else:
            self.s, self.s_pub = keypair(self.static_priv)
        self.re = msg
        self.ss.mix_hash(msg)
        self.ss.mix_hash(b"")

    def write_message2(self, payload: bytes = b"") -> bytes:
        e, e_pub = _ell_keypair() if self.suite == "ellswift" else keypair()
        self.ss.mix_hash(e_pub)
        self.ss.mix_key(self._dh(e, self.re, e_pub))           # ee
        enc_s = self.ss.encrypt_and_hash(self.s_pub)
        self.ss.mix_key(self._dh(self.s, self.re, self.s_pub))  # es
        enc_p = self.ss.encrypt_and_hash(payload)
        r, i = self.ss.split()
        self.send, self.recv = i, r               # responder sends with k2, receives with k1
        return e_pub + enc_s + enc_p

    @property
    def handshake_hash(self) -> bytes:
        return self.ss.h


# ------------------------------------------------------------------ framing
def encode_frame(cs: CipherState, plain: bytes) -> bytes:
    # size check first: a refused frame must not consume a nonce (the peer would never see it)
    if len(plain) + (TAG if cs.k is not None else 0) > MAX_FRAME:
        raise NoiseError(f"noise: message too large: {len(plain) + TAG}-byte ciphertext exceeds {MAX_FRAME} "
                         f"(plaintext {len(plain)})")
    ct = cs.encrypt(b"", plain)
    return struct.pack("<H", len(ct)) + ct


class EncryptedReader:
    """StreamReader-compatible view (readexactly/read) over Noise frames."""

    def __init__(self, reader: asyncio.StreamReader, cs: CipherState):
        self._r, self._cs, self._buf = reader, cs, bytearray()

    async def _fill(self) -> None:
        n = struct.unpack("<H", await self._r.readexactly(2))[0]
        self._buf += self._cs.decrypt(b"", await self._r.readexactly(n))

    async def readexactly(self, n: int) -> bytes:
        while len(self._buf) < n:
            await self._fill()
        out = bytes(self._buf[:n])
        del self._buf[:n]
        return out

    async def read(self, n: int = -1) -> bytes:
        if not self._buf:
            try:
                await self._fill()
            except asyncio.IncompleteReadError:
                return b""
        k = len(self._buf) if n < 0 else min(n, len(self._buf))
        out = bytes(self._buf[:k])
        del self._buf[:k]
        return out


class EncryptedWriter:
    """StreamWriter-compatible write/drain/close; each write() is one or more frames."""

    def __init__(self, writer: asyncio.StreamWriter, cs: CipherState):
        self._w, self._cs = writer, cs

    def write(self, data: bytes) -> None:
        step = MAX_FRAME - TAG
        for off in range(0, max(len(data), 1), step):
            self._w.write(encode_frame(self._cs, data[off:off + step]))

    async def drain(self) -> None:
        await self._w.drain()

    def close(self) -> None:
        self._w.close()

    async def wait_closed(self) -> None:
        await self._w.wait_closed()

    def get_extra_info(self, name, default=None):
        return self._w.get_extra_info(name, default)

    def is_closing(self) -> bool:
        return self._w.is_closing()


async def _read_hs(reader: asyncio.StreamReader) -> bytes:
    n = struct.unpack("<H", await reader.readexactly(2))[0]
    return await reader.readexactly(n)


async def client_handshake(reader, writer, expected_static: bytes | None = None, timeout: float = 10.0,
                           suite: str = DEFAULT_SUITE):
    """Runs NX as initiator; returns (EncryptedReader, EncryptedWriter, server_payload, server_static x-only)."""
    hs = Initiator(expected_static, suite=suite)
    m1 = hs.write_message1()
    writer.write(struct.pack("<H", len(m1)) + m1)
    await writer.drain()
    payload = hs.read_message2(await asyncio.wait_for(_read_hs(reader), timeout))
    return EncryptedReader(reader, hs.recv), EncryptedWriter(writer, hs.send), payload, hs.remote_static


async def server_handshake(reader, writer, static_priv: int, payload: bytes = b"", timeout: float = 10.0,
                           suite: str | None = None):
    """Runs NX as responder (either suite unless ``suite`` fixes one); returns (EncryptedReader, EncryptedWriter)."""
    hs = Responder(static_priv, suite=suite)
    hs.read_message1(await asyncio.wait_for(_read_hs(reader), timeout))
    m2 = hs.write_message2(payload)
    writer.write(struct.pack("<H", len(m2)) + m2)
    await writer.drain()
    return EncryptedReader(reader, hs.recv), EncryptedWriter(writer, hs.send)


def certificate_payload(static_pub: bytes, authority_priv: int, valid_from: int, not_valid_after: int,
                        version: int = 0) -> bytes:
    """SV2-style SignatureNoiseMessage: version u16, valid_from u32, not_valid_after u32, BIP-340 sig over
    SHA-256(version ‖ valid_from ‖ not_valid_after ‖ static_pub)."""
    body = struct.pack("<HII", version, valid_from, not_valid_after)
    sig = ec.SchnorrSecp256k1().sign(authority_priv, hashlib.sha256(body + static_pub).digest())
    return body + sig


def verify_certificate(payload: bytes, static_pub: bytes, authority_pub: bytes, now: int) -> bool:
    if len(payload) != 10 + 64:
        return False
    _, vf, nva = struct.unpack("<HII", payload[:10])
    if not vf <= now <= nva:
        return False
    try:
        ec.SchnorrSecp256k1().verify(authority_pub, hashlib.sha256(payload[:10] + static_pub).digest(), payload[10:])
    except ec.BtcCryptoError:
        return False
    return True
