"""ElligatorSwift public-key encoding for secp256k1 (BIP324) and x-only ECDH over it.

Stratum V2's current Noise suite (``Noise_NX_Secp256k1+EllSwift_ChaChaPoly_SHA256``) sends every public key as
64 bytes ``u ‖ t`` (two field elements, big-endian) that decode to an x coordinate through the SwiftEC map; a
uniformly random private key gives an encoding indistinguishable from 64 random bytes. The reference names this
suite (internal/stratum/noise.go:10-32, docs/adr/ADR-011-secp256k1-for-stratum-v2-noise.md:14,124-159) but never
implemented it; this module is the full encoder, decoder and BIP324 ``v2_ecdh``.

  * ``xswiftec(u, t)``            field pair -> x coordinate on the curve (every input decodes);
  * ``xswiftec_inv(x, u, case)``  the up-to-8 preimages t for a given u (``None`` when a case has none);
  * ``encode(x)`` / ``create(priv)``  random u, random case, retry -> 64 bytes;
  * ``decode(b64)``               -> x;
  * ``xdh(priv, ell_a, ell_b, initiating)``  BIP324's x-only ECDH: TaggedHash("bip324_ellswift_xonly_ecdh",
    ell_a ‖ ell_b ‖ x(priv · decode(theirs))) with ``ell_a`` the initiator's encoding.

No published test vectors are reachable offline (bitcoin-core's ``ellswift`` vectors, BIP324's CSV): parity is
UNPINNED against them. What the tests pin instead: every case's preimage decodes back to x, the 8 cases give
distinct preimages, decode is total (every 64-byte string decodes, including u = 0, t = 0 and u³ + t² + 7 = 0),
both ECDH sides agree, and the encoding of a key decodes to that key's x.

Host Python integers: a handshake needs a handful of scalar multiplications (milliseconds), nothing per share.
"""
from __future__ import annotations

import hashlib
import os

from otedama_amd import btccrypto as ec

P = ec.P


def _sqrt(a: int) -> int | None:
    a %= P
    r = pow(a, (P + 1) // 4, P)  # P = 3 mod 4
    return r if r * r % P == a else None


def _inv(a: int) -> int:
    return pow(a, -1, P)


C = _sqrt(-3)  # sqrt(-3) mod P (the root pow() yields; BIP324's choice)
_HALF = _inv(2)


def is_x(x: int) -> bool:
    """x is the x coordinate of a curve point (x³ + 7 is a square)."""
    return _sqrt(pow(x, 3, P) + 7) is not None


def xswiftec(u: int, t: int) -> int:
    u %= P
    t %= P
    if u == 0:
        u = 1
    if t == 0:
        t = 1
    if (pow(u, 3, P) + t * t + 7) % P == 0:
        t = 2 * t % P
    X = (pow(u, 3, P) + 7 - t * t) * _inv(2 * t) % P
    Y = (X + t) * _inv(C * u) % P
    x1 = (u + 4 * Y * Y) % P
    if is_x(x1):
        return x1
    xy = X * _inv(Y) % P
    x2 = (-xy - u) * _HALF % P
    if is_x(x2):
        return x2
    return (xy - u) * _HALF % P  # g(x1)·g(x2)·g(x3) is a square: one of the three is on the curve


def xswiftec_inv(x: int, u: int, case: int) -> int | None:
    """A t with xswiftec(u, t) == x, one per ``case`` in 0..7, or None when that case has no solution.

    Bit 1 picks x as x1 (u + 4Y²) or as x2/x3; bits 0 and 2 pick the sign of sqrt(s) and of sqrt(-3)."""
    x %= P
    u %= P
    if case & 2 == 0:
        if is_x(-x - u):  # x2 and x3 both valid -> x1 valid too and decoding would return x1
            return None
        v = x
        den = (u * u + u * v + v * v) % P
        if den == 0:
            return None
        s = -(pow(u, 3, P) + 7) * _inv(den) % P
    else:
        s = (x - u) % P
        if s == 0:
            return None
        r = _sqrt(-s * (4 * (pow(u, 3, P) + 7) + 3 * s * u * u))
        if r is None:
            return None
        if case & 1 and r == 0:
            return None
        v = (r * _inv(s) - u) * _HALF % P
    w = _sqrt(s)
    if w is None or w == 0:
        return None
    k = case & 5
    if k == 0:
        return -w * (u * (1 - C) * _HALF + v) % P
    if k == 1:
        return w * (u * (1 + C) * _HALF + v) % P
    if k == 4:
        return w * (u * (1 - C) * _HALF + v) % P
    return -w * (u * (1 + C) * _HALF + v) % P


def encode(x: int, rand=os.urandom) -> bytes:
    """64-byte ElligatorSwift encoding of a curve x coordinate (random u and case; ~4 tries on average)."""
    if not is_x(x):
        raise ValueError("ellswift: x is not on secp256k1")
    while True:
        r = rand(33)
        u = int.from_bytes(r[:32], "big") % P
        if u == 0:
            continue
        t = xswiftec_inv(x, u, r[32] & 7)
        if t is not None and t != 0:
            return u.to_bytes(32, "big") + t.to_bytes(32, "big")


def decode(b64: bytes) -> int:
    if len(b64) != 64:
        raise ValueError(f"ellswift: encoding must be 64 bytes, got {len(b64)}")
    return xswiftec(int.from_bytes(b64[:32], "big"), int.from_bytes(b64[32:], "big"))


def create(priv: int, rand=os.urandom) -> bytes:
    """Encoding of priv·G (x only: priv and N - priv encode alike, so no parity fix-up is needed)."""
    pt = ec.point_mul(ec.G, priv)
    return encode(pt[0], rand)


def _tagged(tag: str, data: bytes) -> bytes:
    th = hashlib.sha256(tag.encode()).digest()
    return hashlib.sha256(th + th + data).digest()


def ecdh_x(priv: int, ell_theirs: bytes) -> bytes:
    """x coordinate of priv · decode(theirs), 32 bytes big-endian."""
    pt = ec.lift_x(decode(ell_theirs))
    r = ec.point_mul(pt, priv)
    if r is None:
        raise ValueError("ellswift: ECDH produced the point at infinity")
    return r[0].to_bytes(32, "big")


def xdh(priv: int, ell_theirs: bytes, ell_ours: bytes, initiating: bool) -> bytes:
    """BIP324 ``v2_ecdh``: both parties hash (initiator's encoding ‖ responder's encoding ‖ shared x)."""
    x = ecdh_x(priv, ell_theirs)
    a, b = (ell_ours, ell_theirs) if initiating else (ell_theirs, ell_ours)
    return _tagged("bip324_ellswift_xonly_ecdh", a + b + x)
