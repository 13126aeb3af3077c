"""Bitcoin crypto helpers (C40; reference internal/btccrypto/*_test.go): published BIP-173 / BIP-350 /
BIP-340 vectors, base58check, output scripts, and sign/verify properties."""
import hashlib

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from otedama_amd import btccrypto as B


@pytest.mark.parametrize("addr,kind,script", [
    # BIP-173 examples
    ("BC1QW508D6QEJXTDG4Y5R3ZARVARY0C5XW7KV8F3T4", B.AddressType.P2WPKH,
     "0014751e76e8199196d454941c45d1b3a323f1433bd6"),
    ("bc1qrp33g0q5c5txsp9arysrx4k6zdkfs4nce4xj0gdcccefvpysxf3qccfmv3", B.AddressType.P2WSH,
     "00201863143c14c5166804bd19203356da136c985678cd4d27a1b8c6329604903262"),
    # BIP-350 (bech32m, witness v1)
    ("bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7vqzk5jj0", B.AddressType.P2TR,
     "512079be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798"),
    # base58check: the genesis coinbase address and a P2SH address
    ("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa", B.AddressType.P2PKH, "76a91462e907b15cbf27d5425399ebf6f0fb50ebb88f1888ac"),
    ("3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy", B.AddressType.P2SH, "a914b472a266d0bd89c13706a4132ccfb16f7c3b9fcb87"),
])
def test_address_vectors(addr, kind, script):
    assert B.validate_address(addr) is kind
    assert B.address_script_pubkey(addr).hex() == script
    assert B.classify_address(addr.lower() if addr.startswith("BC1") else addr) is kind


@pytest.mark.parametrize("addr", [
    "bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t5",          # checksum typo
    "bc1qW508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4",          # mixed case
    "tb1qw508d6qejxtdg4y5r3zarvary0c5xw7kxpjzsx",          # testnet hrp
    "bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7vqh2y7hd",  # v1 with a bech32 (not bech32m) checksum
    "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNb",                  # base58 checksum typo
    "2NBFNJTktNa7GZusGbDbGKRZTxdK9VVez3n",                  # testnet P2SH
    "",
    "hello",
])
def test_invalid_addresses_rejected(addr):
    with pytest.raises(B.BtcCryptoError):
        B.validate_address(addr)


@settings(max_examples=50, deadline=None)
@given(payload=st.binary(min_size=0, max_size=40))
def test_base58_roundtrip(payload):
    assert B.base58_decode(B.base58_encode(payload)) == payload
    enc = B.base58check_encode(payload)
    raw = B.base58_decode(enc)
    assert raw[:-4] == payload and raw[-4:] == B.hash256(payload)[:4]


@settings(max_examples=20, deadline=None)
@given(prog=st.binary(min_size=20, max_size=20))
def test_bech32_encode_validates(prog):
    a = B.bech32_encode_segwit("bc", 0, prog)
    assert B.validate_address(a) is B.AddressType.P2WPKH
    assert B.address_script_pubkey(a) == b"\x00\x14" + prog


def test_bip340_vector_0():
    """BIP-340 test vector 0: secret key 3, aux 0, message 0."""
    s = B.lookup("schnorr-secp256k1")
    sig = s.sign(3, bytes(32), bytes(32))
    assert sig.hex().upper() == ("E907831F80848D1069A5371B402410364BDF1C5F8307B0084C55F1CE2DCA8215"
                                 "25F66A4A85EA8B71E482A74F382D2CE5EBEEE8FDB2172F477DF4900D310536C0")
    pub = B.point_mul(B.G, 3)[0].to_bytes(32, "big")
    assert pub.hex().upper() == "F9308A019258C31049344F85F89D5229B531C845836F99B08601F113BCE036F9"
    s.verify(pub, bytes(32), sig)
    with pytest.raises(B.InvalidSignature):
        s.verify(pub, b"\x01" + bytes(31), sig)


@settings(max_examples=12, deadline=None)
@given(priv=st.integers(1, B.N - 1), msg=st.binary(min_size=1, max_size=64))
def test_ecdsa_rfc6979_roundtrip_low_s_deterministic(priv, msg):
    e = B.lookup("ecdsa-secp256k1")
    h = hashlib.sha256(msg).digest()
    sig = e.sign(priv, h)
    assert sig == e.sign(priv, h)                      # RFC 6979: deterministic
    assert int.from_bytes(sig[32:], "big") <= B.N // 2  # low-S
    pub = B.pubkey_compressed(priv)
    e.verify(pub, h, sig)
    bad = bytearray(sig)
    bad[5] ^= 1
    with pytest.raises(B.InvalidSignature):
        e.verify(pub, h, bytes(bad))
    with pytest.raises(B.InvalidSignature):
        e.verify(pub, hashlib.sha256(h).digest(), sig)


def test_scheme_registry():
    assert {"ecdsa-secp256k1", "schnorr-secp256k1"} <= set(B.schemes())
    with pytest.raises(B.UnknownScheme):
        B.lookup("rsa")
    assert B.scheme_for_address_type(B.AddressType.P2WPKH).name == "ecdsa-secp256k1"
    assert B.scheme_for_address_type(B.AddressType.P2TR).name == "schnorr-secp256k1"
