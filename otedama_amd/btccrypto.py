"""Bitcoin address validation and secp256k1 signature schemes.

Parity: internal/btccrypto
  * base58check decode + ValidateBase58Address ........ base58.go:33-107
  * bech32 / bech32m (BIP-173/350) ValidateBech32Address bech32.go:43-189
  * ValidateAddress (bech32 first, then base58) ........ base58.go:99
  * AddressType / ClassifyAddress / SchemeForAddressType btccrypto.go:225-345
  * Hash256 / TaggedHash (BIP-340) ..................... btccrypto.go:352-373
  * Scheme registry Register/Lookup/Schemes ............ btccrypto.go:182-215
The reference registers only stubs for ECDSA/Schnorr (secp256k1.go:23-50); here
both are real (pure-Python secp256k1: ECDSA with RFC 6979 nonces, BIP-340
Schnorr), used by tests and by the Noise handshake option (ADR-011).
"""
from __future__ import annotations

import hashlib
import hmac
import threading
from enum import IntEnum


class BtcCryptoError(ValueError):
    pass


class UnknownScheme(BtcCryptoError):
    pass


class SchemeNotImplemented(BtcCryptoError):
    pass


class NotBech32(BtcCryptoError):
    pass


class NotBase58(BtcCryptoError):
    pass


class UnrecognisedAddress(BtcCryptoError):
    pass


class InvalidSignature(BtcCryptoError):
    pass


class AddressType(IntEnum):
    UNKNOWN = 0
    P2PKH = 1
    P2SH = 2
    P2WPKH = 3
    P2WSH = 4
    P2TR = 5
    P2MR = 6

    def __str__(self) -> str:
        return "unknown" if self is AddressType.UNKNOWN else self.name


def hash256(b: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


def tagged_hash(tag: str, msg: bytes) -> bytes:
    th = hashlib.sha256(tag.encode()).digest()
    return hashlib.sha256(th + th + msg).digest()


# ----------------------------------------------------------------- base58
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def base58_decode(s: str) -> bytes:
    n = 0
    for ch in s:
        i = B58.find(ch)
        if i < 0:
            raise BtcCryptoError(f"invalid base58 character {ch!r}")
        n = n * 58 + i
    body = n.to_bytes((n.bit_length() + 7) // 8, "big") if n else b""
    lead = len(s) - len(s.lstrip("1"))
    return b"\x00" * lead + body


def base58_encode(b: bytes) -> str:
    n = int.from_bytes(b, "big")
    out = ""
    while n:
        n, r = divmod(n, 58)
        out = B58[r] + out
    return "1" * (len(b) - len(b.lstrip(b"\x00"))) + out


def base58check_encode(payload: bytes) -> str:
    return base58_encode(payload + hash256(payload)[:4])


def validate_base58_address(addr: str) -> AddressType:
    if not addr or addr.startswith(("bc1", "BC1")) or not addr.startswith(("1", "3")):
        raise NotBase58("btccrypto: not a base58 address")
    try:
        raw = base58_decode(addr)
    except BtcCryptoError as exc:
        raise BtcCryptoError(f"btccrypto: {exc}") from None
    if len(raw) != 25:
        raise BtcCryptoError(f"btccrypto: base58 address decodes to {len(raw)} bytes, want 25")
    payload, checksum = raw[:21], raw[21:]
    if hash256(payload)[:4] != checksum:
        raise BtcCryptoError("btccrypto: base58 checksum failed (likely a typo in the address)")
    if payload[0] == 0x00:
        return AddressType.P2PKH
    if payload[0] == 0x05:
        return AddressType.P2SH
    raise BtcCryptoError(f"btccrypto: unsupported base58 version byte 0x{payload[0]:02x} (mainnet P2PKH/P2SH only)")


# ----------------------------------------------------------------- bech32
BECH32_CHARSET = "qpzry9x8gf2tvdw0s3jn54khce6mua7l"
BECH32_CONST = 1
BECH32M_CONST = 0x2BC830A3


def bech32_polymod(values) -> int:
    gen = (0x3B6A57B2, 0x26508E6D, 0x1EA119FA, 0x3D4233DD, 0x2A1462B3)
    chk = 1
    for v in values:
        top = chk >> 25
        chk = ((chk & 0x1FFFFFF) << 5) ^ v
        for i in range(5):
            if (top >> i) & 1:
                chk ^= gen[i]
    return chk


def bech32_hrp_expand(hrp: str) -> list[int]:
    return [ord(c) >> 5 for c in hrp] + [0] + [ord(c) & 31 for c in hrp]


def convert_bits(data, frm: int, to: int, pad: bool) -> list[int]:
    acc = bits = 0
    maxv = (1 << to) - 1
    out = []
    for v in data:
        if v < 0 or v >> frm:
            raise BtcCryptoError(f"btccrypto: convertBits: value {v} out of range")
        acc = (acc << frm) | v
        bits += frm
        while bits >= to:
            bits -= to
            out.append((acc >> bits) & maxv)
    if pad:
        if bits:
            out.append((acc << (to - bits)) & maxv)
    elif bits >= frm or ((acc << (to - bits)) & maxv):
        raise BtcCryptoError("btccrypto: convertBits: invalid padding")
    return out


def bech32_encode_segwit(hrp: str, version: int, program: bytes) -> str:
    data = [version] + convert_bits(program, 8, 5, True)
    const = BECH32_CONST if version == 0 else BECH32M_CONST
    pm = bech32_polymod(bech32_hrp_expand(hrp) + data + [0] * 6) ^ const
    checksum = [(pm >> 5 * (5 - i)) & 31 for i in range(6)]
    return hrp + "1" + "".join(BECH32_CHARSET[d] for d in data + checksum)


def validate_bech32_address(addr: str) -> AddressType:
    if not addr.startswith(("bc1", "BC1")):
        raise NotBech32("btccrypto: not a bech32 address")
    if addr != addr.lower() and addr != addr.upper():
        raise BtcCryptoError("btccrypto: bech32 address has mixed case")
    s = addr.lower()
    if len(s) > 90:
        raise BtcCryptoError(f"btccrypto: bech32 address too long ({len(s)} > 90)")
    pos = s.rfind("1")
    if pos < 1:
        raise BtcCryptoError("btccrypto: bech32 address has no separator")
    hrp = s[:pos]
    if hrp != "bc":
        raise BtcCryptoError(f"btccrypto: unsupported human-readable part {hrp!r} (mainnet 'bc' only)")
    dp = s[pos + 1:]
    if len(dp) < 8:
        raise BtcCryptoError("btccrypto: bech32 data part too short")
    data = []
    for c in dp:
        i = BECH32_CHARSET.find(c)
        if i < 0:
            raise BtcCryptoError(f"btccrypto: invalid bech32 character {c!r}")
        data.append(i)
    version = data[0]
    if version > 16:
        raise BtcCryptoError(f"btccrypto: invalid witness version {version}")
    want = BECH32_CONST if version == 0 else BECH32M_CONST
    if bech32_polymod(bech32_hrp_expand(hrp) + data) != want:
        raise BtcCryptoError("btccrypto: bech32 checksum failed (likely a typo in the address)")
    program = convert_bits(data[1:-6], 5, 8, False)
    if not 2 <= len(program) <= 40:
        raise BtcCryptoError(f"btccrypto: witness program length {len(program)} out of range")
    if version == 0:
        if len(program) == 20:
            return AddressType.P2WPKH
        if len(program) == 32:
            return AddressType.P2WSH
        raise BtcCryptoError(f"btccrypto: v0 witness program must be 20 or 32 bytes, got {len(program)}")
    if version == 1:
        if len(program) != 32:
            raise BtcCryptoError(f"btccrypto: v1 (Taproot) program must be 32 bytes, got {len(program)}")
        return AddressType.P2TR
    raise BtcCryptoError(f"btccrypto: unsupported witness version {version}")


def validate_address(addr: str) -> AddressType:
    try:
        return validate_bech32_address(addr)
    except NotBech32:
        pass
    try:
        return validate_base58_address(addr)
    except NotBase58:
        pass
    raise UnrecognisedAddress("btccrypto: unrecognised address format (not bech32 or base58 mainnet)")


def classify_address(addr: str) -> AddressType:
    if addr.startswith("bc1p"):
        return AddressType.P2TR
    if addr.startswith("bc1q"):
        return AddressType.P2WSH if len(addr) >= 60 else AddressType.P2WPKH
    if addr.startswith("1"):
        return AddressType.P2PKH
    if addr.startswith("3"):
        return AddressType.P2SH
    return AddressType.UNKNOWN


def address_script_pubkey(addr: str) -> bytes:
    """Output script for a validated mainnet address (pool coinbase payouts)."""
    t = validate_address(addr)
    if t in (AddressType.P2PKH, AddressType.P2SH):
        h160 = base58_decode(addr)[1:21]
        if t is AddressType.P2PKH:
            return b"\x76\xa9\x14" + h160 + b"\x88\xac"
        return b"\xa9\x14" + h160 + b"\x87"
    s = addr.lower()
    data = [BECH32_CHARSET.find(c) for c in s[s.rfind("1") + 1:]]
    prog = bytes(convert_bits(data[1:-6], 5, 8, False))
    ver = data[0]
    return bytes([0x50 + ver if ver else 0, len(prog)]) + prog


# ----------------------------------------------------------------- secp256k1
P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
     0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)


def _add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2 and (y1 + y2) % P == 0:
        return None
    if p1 == p2:
        lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def _jdouble(p1):
    x, y, z = p1
    if y == 0:
        return 0, 1, 0
    ysq = y * y % P
    s = 4 * x * ysq % P
    m = 3 * x * x % P  # a = 0
    nx = (m * m - 2 * s) % P
    return nx, (m * (s - nx) - 8 * ysq * ysq) % P, 2 * y * z % P


def _jadd_affine(p1, x2, y2):
    """Jacobian + affine (mixed addition); the infinity point is z = 0."""
    x1, y1, z1 = p1
    if z1 == 0:
        return x2, y2, 1
    z1z1 = z1 * z1 % P
    u2 = x2 * z1z1 % P
    s2 = y2 * z1 * z1z1 % P
    h = (u2 - x1) % P
    r = (s2 - y1) % P
    if h == 0:
        return _jdouble(p1) if r == 0 else (0, 1, 0)
    hh = h * h % P
    hhh = h * hh % P
    v = x1 * hh % P
    nx = (r * r - hhh - 2 * v) % P
    return nx, (r * (v - nx) - y1 * hhh) % P, z1 * h % P


def point_mul(pt, k: int):
    """k·pt in Jacobian coordinates (one field inversion at the end instead of one per step)."""
    if pt is None or k % N == 0:
        return None
    x2, y2 = pt
    acc = (0, 1, 0)
    for bit in bin(k)[2:]:
        acc = _jdouble(acc)
        if bit == "1":
            acc = _jadd_affine(acc, x2, y2)
    x, y, z = acc
    if z == 0:
        return None
    zi = pow(z, -1, P)
    zi2 = zi * zi % P
    return x * zi2 % P, y * zi2 * zi % P


def lift_x(x: int):
    if x >= P:
        return None
    c = (pow(x, 3, P) + 7) % P
    y = pow(c, (P + 1) // 4, P)
    if y * y % P != c:
        return None
    return x, y if y % 2 == 0 else P - y


def pubkey_compressed(priv: int) -> bytes:
    x, y = point_mul(G, priv)
    return bytes([2 + (y & 1)]) + x.to_bytes(32, "big")


def decode_pubkey(b: bytes):
    if len(b) == 33 and b[0] in (2, 3):
        pt = lift_x(int.from_bytes(b[1:], "big"))
        if pt is None:
            raise BtcCryptoError("btccrypto: invalid public key")
        x, y = pt
        if (y & 1) != (b[0] & 1):
            y = P - y
        return x, y
    if len(b) == 65 and b[0] == 4:
        x, y = int.from_bytes(b[1:33], "big"), int.from_bytes(b[33:], "big")
        if (y * y - x * x * x - 7) % P:
            raise BtcCryptoError("btccrypto: invalid public key")
        return x, y
    if len(b) == 32:  # x-only (BIP-340)
        pt = lift_x(int.from_bytes(b, "big"))
        if pt is None:
            raise BtcCryptoError("btccrypto: invalid public key")
        return pt
    raise BtcCryptoError("btccrypto: invalid public key")


def _rfc6979(priv: int, h: bytes) -> int:
    x = priv.to_bytes(32, "big")
    v, k = b"\x01" * 32, b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + x + h, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + x + h, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    while True:
        v = hmac.new(k, v, hashlib.sha256).digest()
        t = int.from_bytes(v, "big")
        if 1 <= t < N:
            return t
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()


class EcdsaSecp256k1:
    name = "ecdsa-secp256k1"

    def sign(self, priv: int, msg32: bytes) -> bytes:
        z = int.from_bytes(msg32, "big")
        k = _rfc6979(priv, msg32)
        r = point_mul(G, k)[0] % N
        s = pow(k, N - 2, N) * (z + r * priv) % N
        if s > N // 2:
            s = N - s  # low-S
        return r.to_bytes(32, "big") + s.to_bytes(32, "big")

    def verify(self, pub: bytes, msg32: bytes, sig: bytes) -> None:
        if len(sig) != 64:
            raise InvalidSignature("btccrypto: invalid signature")
        r, s = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:], "big")
        if not (1 <= r < N and 1 <= s < N):
            raise InvalidSignature("btccrypto: invalid signature")
        q = decode_pubkey(pub)
        w = pow(s, N - 2, N)
        z = int.from_bytes(msg32, "big")
        pt = _add(point_mul(G, z * w % N), point_mul(q, r * w % N))
        if pt is None or pt[0] % N != r:
            raise InvalidSignature("btccrypto: invalid signature")


class SchnorrSecp256k1:
    """BIP-340."""

    name = "schnorr-secp256k1"

    def sign(self, priv: int, msg: bytes, aux: bytes = bytes(32)) -> bytes:
        x, y = point_mul(G, priv)
        d = priv if y % 2 == 0 else N - priv
        t = (d ^ int.from_bytes(tagged_hash("BIP0340/aux", aux), "big")).to_bytes(32, "big")
        k0 = int.from_bytes(tagged_hash("BIP0340/nonce", t + x.to_bytes(32, "big") + msg), "big") % N
        if k0 == 0:
            raise BtcCryptoError("btccrypto: bad nonce")
        rx, ry = point_mul(G, k0)
        k = k0 if ry % 2 == 0 else N - k0
        e = int.from_bytes(tagged_hash("BIP0340/challenge", rx.to_bytes(32, "big") + x.to_bytes(32, "big") + msg),
                           "big") % N
        return rx.to_bytes(32, "big") + ((k + e * d) % N).to_bytes(32, "big")

    def verify(self, pub: bytes, msg: bytes, sig: bytes) -> None:
        if len(pub) != 32 or len(sig) != 64:
            raise InvalidSignature("btccrypto: invalid signature")
        pt = lift_x(int.from_bytes(pub, "big"))
        r, s = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:], "big")
        if pt is None or r >= P or s >= N:
            raise InvalidSignature("btccrypto: invalid signature")
        e = int.from_bytes(tagged_hash("BIP0340/challenge", sig[:32] + pub + msg), "big") % N
        R = _add(point_mul(G, s), point_mul(pt, N - e))
        if R is None or R[1] % 2 or R[0] != r:
            raise InvalidSignature("btccrypto: invalid signature")


_registry_lock = threading.Lock()
_registry: dict[str, object] = {}


def register(scheme) -> None:
    with _registry_lock:
        if scheme.name in _registry:
            raise BtcCryptoError(f"btccrypto: scheme {scheme.name!r} registered twice")
        _registry[scheme.name] = scheme


def lookup(name: str):
    with _registry_lock:
        if name not in _registry:
            raise UnknownScheme(f"btccrypto: unknown signature scheme: {name!r}")
        return _registry[name]


def schemes() -> list[str]:
    with _registry_lock:
        return sorted(_registry)


def scheme_for_address_type(t: AddressType):
    if t in (AddressType.P2PKH, AddressType.P2SH, AddressType.P2WPKH, AddressType.P2WSH):
        return lookup("ecdsa-secp256k1")
    if t is AddressType.P2TR:
        return lookup("schnorr-secp256k1")
    if t is AddressType.P2MR:
        raise SchemeNotImplemented("btccrypto: scheme registered but implementation pending: P2MR (BIP-360)")
    raise UnknownScheme(f"btccrypto: unknown signature scheme: unknown address type {t}")


register(EcdsaSecp256k1())
register(SchnorrSecp256k1())
