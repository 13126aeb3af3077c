"""Bitcoin crypto helpers, case by case: mirrors internal/btccrypto/{base58,bech32,btccrypto,btccrypto_extras}_test.go.

Vectors are the published BIP-173 / BIP-350 address lists (valid and invalid), well-known base58check mainnet
addresses and the Bitcoin genesis header; every address below that is expected to fail past the checksum stage passes
the checksum first, which pins the polymod. Reference behaviour (file:line in /root/reference/internal/btccrypto):
  * ValidateBase58Address ............ base58.go:56-107
  * ValidateBech32Address ............ bech32.go:110-189 (mainnet "bc" only; v0 20/32 B, v1 32 B, v2-16 refused)
  * ValidateAddress dispatch ......... base58.go:99 (bech32 first, then base58, else ErrUnrecognisedAddress)
  * AddressType / ClassifyAddress .... btccrypto.go:225-345
  * Hash256 / TaggedHash ............. btccrypto.go:352-373
  * scheme registry .................. btccrypto.go:182-215, secp256k1.go
"""
import hashlib
import re
import threading

import pytest

from otedama_amd import btccrypto as B

T = B.AddressType


@pytest.fixture
def registry_snapshot():
    saved = dict(B._registry)
    yield
    with B._registry_lock:
        B._registry.clear()
        B._registry.update(saved)


# ---------------------------------------------------------------------------------------------- base58

@pytest.mark.parametrize("addr,kind", [
    ("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa", T.P2PKH),   # genesis coinbase
    ("1BvBMSEYstWetqTFn5Au4m4GFg7xJaNVN2", T.P2PKH),
    ("1111111111111111111114oLvT2", T.P2PKH),          # hash160 = 20 zero bytes
    ("3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy", T.P2SH),
])
def test_validate_base58_address_valid_vectors(addr, kind):
    assert B.validate_base58_address(addr) is kind
    assert B.validate_address(addr) is kind


def test_validate_base58_address_typo_fails_checksum():
    good = "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa"
    for i in (5, 15, len(good) - 1):
        c = "2" if good[i] != "2" else "3"
        with pytest.raises(B.BtcCryptoError, match="checksum failed"):
            B.validate_base58_address(good[:i] + c + good[i + 1:])


@pytest.mark.parametrize("addr,ch", [("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfN0", "0"),
                                     ("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNI", "I"),
                                     ("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNl", "l"),
                                     ("3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLO", "O"),
                                     ("1A1zP1eP5QGefi2DMPTfTL5SLmv7Divf+a", "+")])
def test_validate_base58_address_invalid_char_rejected(addr, ch):
    with pytest.raises(B.BtcCryptoError, match=re.escape(f"btccrypto: invalid base58 character '{ch}'")):
        B.validate_base58_address(addr)


@pytest.mark.parametrize("addr", ["1", "11", "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNaX", "1A1zP1eP5QGefi2DMPT",
                                  "3" + "z" * 40])
def test_validate_base58_address_wrong_length_rejected(addr):
    with pytest.raises(B.BtcCryptoError, match="decodes to \\d+ bytes, want 25"):
        B.validate_base58_address(addr)


@pytest.mark.parametrize("addr", ["", "bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4", "BC1QW508",
                                  "2NBFNJTktNa7GZusGbDbGKRZTxdK9VVez3n", "mipcBbFg9gMiCh81Kj8tqqdgoZub1ZJRfn",
                                  "xpub661MyMwAqRbcF", "hello"])
def test_validate_base58_address_not_base58_returns_sentinel(addr):
    with pytest.raises(B.NotBase58):
        B.validate_base58_address(addr)


@pytest.mark.parametrize("version", [0x06, 0x07])  # the only other version bytes whose encoding starts with 1/3
def test_validate_base58_address_unsupported_version_byte(version):
    addr = B.base58check_encode(bytes([version]) + bytes(range(20)))
    assert addr[0] == "3"
    with pytest.raises(B.BtcCryptoError, match=f"unsupported base58 version byte 0x{version:02x}"):
        B.validate_base58_address(addr)


def test_base58_version_prefixes():
    assert B.base58check_encode(b"\x00" + bytes(20))[0] == "1"
    assert B.base58check_encode(b"\x05" + bytes(20))[0] == "3"
    assert B.base58check_encode(b"\x6f" + bytes(20))[0] in "mn"  # testnet: not accepted


def test_base58_leading_zero_bytes_map_to_ones():
    assert B.base58_encode(b"\x00\x00\x01") == "112"
    assert B.base58_decode("112") == b"\x00\x00\x01"
    assert B.base58_encode(b"") == "" and B.base58_decode("") == b""
    assert B.base58_decode("1111") == bytes(4)


def test_base58_encode_known_strings():
    assert B.base58_encode(b"hello world") == "StV1DL6CwTryKyV"
    assert B.base58_decode("StV1DL6CwTryKyV") == b"hello world"


# ---------------------------------------------------------------------------------------------- bech32

@pytest.mark.parametrize("addr,kind", [
    ("BC1QW508D6QEJXTDG4Y5R3ZARVARY0C5XW7KV8F3T4", T.P2WPKH),
    ("bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4", T.P2WPKH),
    ("bc1qrp33g0q5c5txsp9arysrx4k6zdkfs4nce4xj0gdcccefvpysxf3qccfmv3", T.P2WSH),
    ("bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7vqzk5jj0", T.P2TR),
])
def test_validate_bech32_address_valid_vectors(addr, kind):
    assert B.validate_bech32_address(addr) is kind
    assert B.validate_address(addr) is kind


def test_validate_bech32_address_typo_fails_checksum():
    good = "bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4"
    for i in range(4, len(good)):
        c = "q" if good[i] != "q" else "p"
        with pytest.raises(B.BtcCryptoError):
            B.validate_bech32_address(good[:i] + c + good[i + 1:])


@pytest.mark.parametrize("addr", ["bc1qW508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4",
                                  "bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7vq47Zagq",
                                  "Bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4"])
def test_validate_bech32_address_mixed_case_rejected(addr):
    if not addr.startswith(("bc1", "BC1")):
        with pytest.raises(B.NotBech32):
            B.validate_bech32_address(addr)
        return
    with pytest.raises(B.BtcCryptoError, match="mixed case"):
        B.validate_bech32_address(addr)


@pytest.mark.parametrize("addr,ch", [("bc1p38j9r5y49hruaue7wxjce0updqjuyyx0kh56v8s25huc6995vvpql3jow4", "o"),
                                     ("bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3tb", "b"),
                                     ("bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3ti", "i")])
def test_validate_bech32_address_invalid_char_rejected(addr, ch):
    with pytest.raises(B.BtcCryptoError, match=f"invalid bech32 character '{ch}'"):
        B.validate_bech32_address(addr)


def test_validate_bech32_address_too_long_rejected():
    with pytest.raises(B.BtcCryptoError, match="too long \\(91 > 90\\)"):
        B.validate_bech32_address("bc1" + "q" * 88)


@pytest.mark.parametrize("addr", ["1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa", "3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy", "",
                                  "tb1qw508d6qejxtdg4y5r3zarvary0c5xw7kxpjzsx", "bc", "b1qq"])
def test_validate_bech32_address_legacy_returns_not_bech32(addr):
    with pytest.raises(B.NotBech32):
        B.validate_bech32_address(addr)


@pytest.mark.parametrize("addr,match", [("bc1gmk9yu", "data part too short"), ("bc1", "data part too short"),
                                        ("bc1qqqqqq", "data part too short")])
def test_validate_bech32_address_no_separator_or_short_rejected(addr, match):
    with pytest.raises(B.BtcCryptoError, match=match):
        B.validate_bech32_address(addr)


def test_validate_bech32_address_invalid_witness_version_rejected():
    with pytest.raises(B.BtcCryptoError, match="invalid witness version 17"):
        B.validate_bech32_address("BC130XLXVLHEMJA6C4DQV22UAPCTQUPFHLXM9H8Z3K2E72Q4K9HCZ7VQ7ZWS8R")


def test_validate_bech32_address_wrong_hrp_rejected():
    a = B.bech32_encode_segwit("bcrt", 0, bytes(20))  # regtest hrp begins with "bc" but is not "bc"
    assert a.startswith("bcrt1")
    with pytest.raises(B.NotBech32):
        B.validate_bech32_address(a)
    b = B.bech32_encode_segwit("bc1x", 0, bytes(20))  # starts with "bc1" but the separator is later
    with pytest.raises(B.BtcCryptoError, match="unsupported human-readable part 'bc1x'"):
        B.validate_bech32_address(b)


@pytest.mark.parametrize("addr", ["BC1S0XLXVLHEMJA6C4DQV22UAPCTQUPFHLXM9H8Z3K2E72Q4K9HCZ7VQ54WELL",   # bech32 for v16
                                  "bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kemeawh",                         # bech32m for v0
                                  "bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7vqh2y7hd"])  # bech32 for v1
def test_validate_bech32_address_wrong_checksum_constant(addr):
    with pytest.raises(B.BtcCryptoError, match="checksum failed"):
        B.validate_bech32_address(addr)


def test_validate_bech32_address_v0_with_21_byte_program():
    with pytest.raises(B.BtcCryptoError, match="v0 witness program must be 20 or 32 bytes, got 21"):
        B.validate_bech32_address(B.bech32_encode_segwit("bc", 0, bytes(21)))
    with pytest.raises(B.BtcCryptoError, match="got 16"):
        B.validate_bech32_address("BC1QR508D6QEJXTDG4Y5R3ZARVARYV98GJ9P")


def test_validate_bech32_address_v1_with_31_byte_program():
    with pytest.raises(B.BtcCryptoError, match="v1 \\(Taproot\\) program must be 32 bytes, got 31"):
        B.validate_bech32_address(B.bech32_encode_segwit("bc", 1, bytes(31)))
    with pytest.raises(B.BtcCryptoError, match="got 40"):
        B.validate_bech32_address("bc1pw508d6qejxtdg4y5r3zarvary0c5xw7kw508d6qejxtdg4y5r3zarvary0c5xw7kt5nd6y")


@pytest.mark.parametrize("addr,version", [("BC1SW50QGDZ25J", 16), ("bc1zw508d6qejxtdg4y5r3zarvaryvaxxpcs", 2)])
def test_validate_bech32_address_future_witness_version(addr, version):
    with pytest.raises(B.BtcCryptoError, match=f"unsupported witness version {version}"):
        B.validate_bech32_address(addr)  # checksum valid (BIP-350 list), version not spendable here


def test_validate_bech32_address_non_canonical_padding_rejected():
    with pytest.raises(B.BtcCryptoError, match="invalid padding"):
        B.validate_bech32_address("bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7v07qwwzcrf")


@pytest.mark.parametrize("addr,n", [("bc1pw5dgrnzv", 1),
                                    ("bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7v8n0nx0muaewav253zgeav", 41)])
def test_validate_bech32_address_witness_program_length_out_of_range(addr, n):
    with pytest.raises(B.BtcCryptoError, match=f"witness program length {n} out of range"):
        B.validate_bech32_address(addr)


def test_bech32_encode_roundtrip_all_supported_kinds():
    for version, n, kind in [(0, 20, T.P2WPKH), (0, 32, T.P2WSH), (1, 32, T.P2TR)]:
        prog = hashlib.sha256(bytes([version, n])).digest()[:n] if n <= 32 else bytes(n)
        a = B.bech32_encode_segwit("bc", version, prog)
        assert B.validate_address(a) is kind and B.validate_address(a.upper()) is kind
        assert B.address_script_pubkey(a)[2:] == prog


# ---------------------------------------------------------------------------------------------- convertBits

def test_convert_bits_rejects_out_of_range_value():
    with pytest.raises(B.BtcCryptoError, match="value 32 out of range"):
        B.convert_bits([1, 2, 32], 5, 8, False)
    with pytest.raises(B.BtcCryptoError, match="out of range"):
        B.convert_bits([-1], 5, 8, True)
    with pytest.raises(B.BtcCryptoError):
        B.convert_bits([256], 8, 5, True)


def test_convert_bits_rejects_invalid_padding():
    with pytest.raises(B.BtcCryptoError, match="invalid padding"):
        B.convert_bits([31], 5, 8, False)       # 5 non-zero leftover bits
    with pytest.raises(B.BtcCryptoError, match="invalid padding"):
        B.convert_bits([0] * 9, 5, 8, False)    # 45 bits: 5 left over (>= from-width)


def test_convert_bits_pad_round_trip():
    for n in range(0, 41):
        data = list(hashlib.sha512(bytes([n])).digest()[:n]) if n <= 64 else []
        five = B.convert_bits(data, 8, 5, True)
        assert all(0 <= v < 32 for v in five) and len(five) == (8 * n + 4) // 5
        assert B.convert_bits(five, 5, 8, False) == data


# ---------------------------------------------------------------------------------------------- dispatch

def test_validate_address_dispatches_by_format():
    assert B.validate_address("bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4") is T.P2WPKH
    assert B.validate_address("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa") is T.P2PKH
    assert B.validate_address("3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy") is T.P2SH


@pytest.mark.parametrize("addr", ["", "hello", "tb1qw508d6qejxtdg4y5r3zarvary0c5xw7kxpjzsx",
                                  "2NBFNJTktNa7GZusGbDbGKRZTxdK9VVez3n", "0x52908400098527886E0F7030069857D2E4169EE7",
                                  "ltc1qw508d6qejxtdg4y5r3zarvary0c5xw7kgmn4n9"])
def test_validate_address_unrecognised_format_is_sentinel(addr):
    with pytest.raises(B.UnrecognisedAddress, match="unrecognised address format"):
        B.validate_address(addr)


@pytest.mark.parametrize("addr", ["bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t5", "1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNb"])
def test_validate_address_checksum_failure_is_not_unrecognised(addr):
    with pytest.raises(B.BtcCryptoError, match="checksum failed") as ei:
        B.validate_address(addr)
    assert not isinstance(ei.value, B.UnrecognisedAddress)


@pytest.mark.parametrize("addr,script", [
    ("1A1zP1eP5QGefi2DMPTfTL5SLmv7DivfNa", "76a91462e907b15cbf27d5425399ebf6f0fb50ebb88f1888ac"),
    ("3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy", "a914b472a266d0bd89c13706a4132ccfb16f7c3b9fcb87"),
    ("BC1QW508D6QEJXTDG4Y5R3ZARVARY0C5XW7KV8F3T4", "0014751e76e8199196d454941c45d1b3a323f1433bd6"),
    ("bc1p0xlxvlhemja6c4dqv22uapctqupfhlxm9h8z3k2e72q4k9hcz7vqzk5jj0",
     "512079be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798"),
])
def test_address_script_pubkey(addr, script):
    assert B.address_script_pubkey(addr).hex() == script


def test_address_script_pubkey_rejects_invalid():
    with pytest.raises(B.BtcCryptoError):
        B.address_script_pubkey("bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t5")


# ---------------------------------------------------------------------------------------------- AddressType

def test_address_type_all_strings_distinct():
    labels = [str(t) for t in T]
    assert all(labels) and len(set(labels)) == len(labels)


def test_address_type_unknown_string_is_not_empty():
    assert str(T.UNKNOWN) == "unknown"


def test_address_type_string_for_known_types():
    assert [str(t) for t in (T.P2PKH, T.P2SH, T.P2WPKH, T.P2WSH, T.P2TR, T.P2MR)] == \
        ["P2PKH", "P2SH", "P2WPKH", "P2WSH", "P2TR", "P2MR"]
    assert int(T.UNKNOWN) == 0  # iota order (btccrypto.go:225-248)


@pytest.mark.parametrize("addr,kind", [("bc1p0xlx", T.P2TR), ("bc1qw508d6qejxtdg4y5r3zarvary0c5xw7kv8f3t4", T.P2WPKH),
                                       ("bc1qrp33g0q5c5txsp9arysrx4k6zdkfs4nce4xj0gdcccefvpysxf3qccfmv3", T.P2WSH),
                                       ("1anything", T.P2PKH), ("3anything", T.P2SH)])
def test_classify_address_known_prefixes(addr, kind):
    assert B.classify_address(addr) is kind


def test_classify_address_taproot_distinct_from_v0():
    assert B.classify_address("bc1p" + "q" * 58) is T.P2TR
    assert B.classify_address("bc1q" + "q" * 58) is T.P2WSH


@pytest.mark.parametrize("addr", ["", "2NBFNJTktNa7GZusGbDbGKRZTxdK9VVez3n", "tb1q", "BC1QW508", "x"])
def test_classify_address_unknown_returns_unknown(addr):
    assert B.classify_address(addr) is T.UNKNOWN  # prefix-only, case-sensitive, never raises


# ---------------------------------------------------------------------------------------------- hashing

GENESIS_HEADER = bytes.fromhex(
    "01000000" + "00" * 32 + "3ba3edfd7a7b12b27ac72c3e67768f617fc81bc3888a51323a9fb8aa4b1e5e4a"
    + "29ab5f49" + "ffff001d" + "1dac2b7c")


def test_hash256_bitcoin_genesis_block_header():
    assert B.hash256(GENESIS_HEADER)[::-1].hex() == \
        "000000000019d6689c085ae165831e934ff763ae46a2a6c172b3f1b60a8ce26f"


def test_hash256_empty_input():
    assert B.hash256(b"").hex() == "5df6e0e2761359d30a8275058e299fcc0381534545f55cf43e41983f5d4c9456"


def test_hash256_known_string():
    assert B.hash256(b"hello").hex() == "9595c9df90075148eb06860365df33584b75bff782a510c6cd4883a419833d50"


def test_hash256_same_input_deterministic():
    assert B.hash256(b"otedama") == B.hash256(bytearray(b"otedama"))


def test_hash256_different_inputs_different_outputs():
    assert len({B.hash256(bytes([i])) for i in range(256)}) == 256


def test_tagged_hash_bip340_construction():
    th = hashlib.sha256(b"BIP0340/challenge").digest()
    msg = bytes(range(96))
    assert B.tagged_hash("BIP0340/challenge", msg) == hashlib.sha256(th + th + msg).digest()


def test_tagged_hash_bip340_test_vector():
    """BIP-340 vector 0's challenge: e = H_challenge(R.x || P.x || m) reproduces s = k + e*d."""
    sig = bytes.fromhex("E907831F80848D1069A5371B402410364BDF1C5F8307B0084C55F1CE2DCA8215"
                        "25F66A4A85EA8B71E482A74F382D2CE5EBEEE8FDB2172F477DF4900D310536C0")
    px = bytes.fromhex("F9308A019258C31049344F85F89D5229B531C845836F99B08601F113BCE036F9")
    e = int.from_bytes(B.tagged_hash("BIP0340/challenge", sig[:32] + px + bytes(32)), "big") % B.N
    R = B.lift_x(int.from_bytes(sig[:32], "big"))
    s = int.from_bytes(sig[32:], "big")
    P = B.lift_x(int.from_bytes(px, "big"))
    assert B.point_mul(B.G, s) == B._add(R, B.point_mul(P, e))


def test_tagged_hash_structure():
    assert len(B.tagged_hash("x", b"")) == 32
    assert B.tagged_hash("TapLeaf", b"a") != B.hash256(b"a")


def test_tagged_hash_different_tags_different_outputs():
    assert B.tagged_hash("BIP0340/aux", b"m") != B.tagged_hash("BIP0340/nonce", b"m")


def test_tagged_hash_empty_tag():
    e = hashlib.sha256(b"").digest()
    assert B.tagged_hash("", b"msg") == hashlib.sha256(e + e + b"msg").digest()


# ---------------------------------------------------------------------------------------------- scheme registry

def test_schemes_contains_builtins():
    assert {"ecdsa-secp256k1", "schnorr-secp256k1"} <= set(B.schemes())


def test_schemes_no_duplicates_and_deterministic_ordering():
    a, b = B.schemes(), B.schemes()
    assert a == b == sorted(a) and len(set(a)) == len(a)


@pytest.mark.parametrize("name", ["", "rsa", "ecdsa-secp256k1 ", "ECDSA-SECP256K1"])
def test_lookup_unknown_returns_typed_error(name):
    with pytest.raises(B.UnknownScheme, match="unknown signature scheme"):
        B.lookup(name)


def test_lookup_trailing_space_treated_as_different():
    assert B.lookup("ecdsa-secp256k1").name == "ecdsa-secp256k1"
    with pytest.raises(B.UnknownScheme):
        B.lookup("ecdsa-secp256k1 ")


def test_register_duplicate_name_refused(registry_snapshot):
    class Dup:
        name = "ecdsa-secp256k1"
    with pytest.raises(B.BtcCryptoError, match="registered twice"):
        B.register(Dup())
    assert isinstance(B.lookup("ecdsa-secp256k1"), B.EcdsaSecp256k1)


def test_registry_concurrent_register_different_names(registry_snapshot):
    class Stub:
        def __init__(self, n):
            self.name = f"stub-{n}"
    threads = [threading.Thread(target=B.register, args=(Stub(i),)) for i in range(32)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert {f"stub-{i}" for i in range(32)} <= set(B.schemes())


def test_registry_concurrent_lookup_safe():
    errors = []

    def worker():
        for _ in range(500):
            if B.lookup("schnorr-secp256k1").name != "schnorr-secp256k1":
                errors.append(1)
    ts = [threading.Thread(target=worker) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors


@pytest.mark.parametrize("kind", [T.P2PKH, T.P2SH, T.P2WPKH, T.P2WSH])
def test_scheme_for_address_type_legacy_and_v0_use_ecdsa(kind):
    assert B.scheme_for_address_type(kind) is B.lookup("ecdsa-secp256k1")


def test_scheme_for_address_type_taproot_uses_schnorr():
    assert B.scheme_for_address_type(T.P2TR) is B.lookup("schnorr-secp256k1")


def test_scheme_for_address_type_p2mr_returns_not_implemented():
    with pytest.raises(B.SchemeNotImplemented, match="P2MR"):
        B.scheme_for_address_type(T.P2MR)


def test_scheme_for_address_type_unknown_returns_error():
    with pytest.raises(B.UnknownScheme, match="unknown address type"):
        B.scheme_for_address_type(T.UNKNOWN)


# ---------------------------------------------------------------------------------------------- signatures

def test_ecdsa_rejects_malformed_signatures():
    e = B.lookup("ecdsa-secp256k1")
    pub, h = B.pubkey_compressed(7), hashlib.sha256(b"m").digest()
    for bad in (b"", bytes(63), bytes(64), B.N.to_bytes(32, "big") + (1).to_bytes(32, "big")):
        with pytest.raises(B.InvalidSignature):
            e.verify(pub, h, bad)


def test_ecdsa_accepts_uncompressed_public_key():
    e = B.lookup("ecdsa-secp256k1")
    x, y = B.point_mul(B.G, 11)
    h = hashlib.sha256(b"uncompressed").digest()
    e.verify(b"\x04" + x.to_bytes(32, "big") + y.to_bytes(32, "big"), h, e.sign(11, h))


def test_decode_pubkey_rejects_invalid_encodings():
    for bad in (b"", b"\x05" + bytes(32), b"\x02" + (B.P + 1).to_bytes(32, "big"), b"\x04" + bytes(64), bytes(31)):
        with pytest.raises(B.BtcCryptoError, match="invalid public key"):
            B.decode_pubkey(bad)


def test_schnorr_rejects_wrong_key_and_malformed_input():
    s = B.lookup("schnorr-secp256k1")
    sig = s.sign(3, bytes(32), bytes(32))
    other = B.point_mul(B.G, 4)[0].to_bytes(32, "big")
    with pytest.raises(B.InvalidSignature):
        s.verify(other, bytes(32), sig)
    pub = B.point_mul(B.G, 3)[0].to_bytes(32, "big")
    for p, sg in ((pub[:31], sig), (pub, sig[:63]), (pub, B.P.to_bytes(32, "big") + sig[32:]),
                  (pub, sig[:32] + B.N.to_bytes(32, "big"))):
        with pytest.raises(B.InvalidSignature):
            s.verify(p, bytes(32), sg)


def test_schnorr_bip340_vector_1():
    """BIP-340 test vector 1 (secret key B7E1…, aux 0…01, message 243F…)."""
    s = B.lookup("schnorr-secp256k1")
    d = int("B7E151628AED2A6ABF7158809CF4F3C762E7160F38B4DA56A784D9045190CFEF", 16)
    aux = bytes.fromhex("0000000000000000000000000000000000000000000000000000000000000001")
    msg = bytes.fromhex("243F6A8885A308D313198A2E03707344A4093822299F31D0082EFA98EC4E6C89")
    sig = s.sign(d, msg, aux)
    assert sig.hex().upper() == ("6896BD60EEAE296DB48A229FF71DFE071BDE413E6D43F917DC8DCF8C78DE3341"
                                 "8906D11AC976ABCCB20B091292BFF4EA897EFCB639EA871CFA95F6DE339E4B0A")
    pub = B.point_mul(B.G, d)[0].to_bytes(32, "big")
    assert pub.hex().upper() == "DFF1D77F2A671C5F36183726DB2341BE58FEAE1DA2DECED843240F7B502BA659"
    s.verify(pub, msg, sig)
