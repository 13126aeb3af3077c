"""Wallet seed custody: BIP-39 vectors, wallet.dat format, WalletManager lifecycle.

Mirrors internal/lightning/{seed,wallet,coverage}_test.go. The BIP-39 vectors
are the published Trezor vectors (passphrase "TREZOR"); the first also appears
in the reference's seed_test.go:249.
"""
import io
import os
import stat

import pytest

from otedama_amd.lightning import seed as S
from otedama_amd.lightning import seedstore as SS
from otedama_amd.lightning.wallet import FINGERPRINT_FILE, WALLET_FILE, WalletError, WalletManager, \
    recovery_phrase_banner

VECTORS = [
    ("00000000000000000000000000000000",
     "abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon about",
     "c55257c360c07c72029aebc1b53c05ed0362ada38ead3e3e9efa3708e53495531f09a6987599d18264c1e1c92f2cf141630c7a3c4ab7"
     "c81b2f001698e7463b04"),
    ("7f7f7f7f7f7f7f7f7f7f7f7f7f7f7f7f",
     "legal winner thank year wave sausage worth useful legal winner thank yellow",
     "2e8905819b8723fe2c1d161860e5ee1830318dbf49a83bd451cfb8440c28bd6fa457fe1296106559a3c80937a1c1069be3a3a5bd381e"
     "e6260e8d9739fce1f607"),
    ("ffffffffffffffffffffffffffffffff",
     "zoo zoo zoo zoo zoo zoo zoo zoo zoo zoo zoo wrong",
     "ac27495480225222079d7be181583751e86f571027b0497b5b5d11218e0a8a13332572917f0f8e5a589620c6f15b11c61dee327651a1"
     "4c34e18231052e48c069"),
    ("0000000000000000000000000000000000000000000000000000000000000000",
     " ".join(["abandon"] * 23 + ["art"]),
     "bda85446c68413707090a52022edd26a1c9462295029f2e60cd7c4f2bbd3097170af7a4d73245cafa9c3cca8d561a7c3de6f5d4a10be"
     "8ed2a5e608d68f92fcc8"),
]


def test_wordlist_integrity():
    wl = S.english_wordlist()
    assert len(wl) == 2048 and wl.word(0) == "abandon" and wl.word(2047) == "zoo"
    assert wl.index("zoo") == 2047
    with pytest.raises(S.SeedError):
        wl.index("notaword")


@pytest.mark.parametrize("ent,phrase,seed", VECTORS)
def test_bip39_vectors(ent, phrase, seed):
    e = bytes.fromhex(ent)
    words = S.entropy_to_mnemonic(e)
    assert " ".join(words) == phrase
    assert S.mnemonic_to_entropy(words) == e
    assert S.mnemonic_to_seed(words, "TREZOR").hex() == seed


def test_entropy_sizes_and_checksum():
    for bits in S.VALID_ENTROPY_BITS:
        e = S.generate_entropy(bits)
        words = S.entropy_to_mnemonic(e)
        assert len(words) == (bits + bits // 32) // 11
        assert S.mnemonic_to_entropy(words) == e
    with pytest.raises(S.SeedError):
        S.generate_entropy(100)
    words = S.entropy_to_mnemonic(bytes(16))
    words[-1] = "abandon"  # breaks the checksum
    with pytest.raises(S.SeedError, match="checksum"):
        S.mnemonic_to_entropy(words)
    with pytest.raises(S.SeedError):
        S.mnemonic_to_entropy(["abandon"] * 11)


def test_entropy_reader_exhaustion():
    with pytest.raises(S.SeedError, match="exhausted"):
        S.generate_entropy(256, io.BytesIO(b"\x00" * 10))


def test_wordlist_validation():
    with pytest.raises(S.SeedError):
        S.WordList(["a"] * 2048)
    with pytest.raises(S.SeedError):
        S.WordList(["a"])


def test_fingerprint():
    s1, s2 = bytes(64), bytes([1]) + bytes(63)
    f = S.fingerprint(s1)
    assert f == S.fingerprint(s1) and len(f) == 8 and int(f, 16) >= 0
    assert f != S.fingerprint(s2)


def test_seedstore_roundtrip_and_tamper():
    seed = bytes(range(64))
    es = SS.encrypt_seed(seed, "pw", io.BytesIO(bytes(range(28))))
    raw = es.marshal()
    assert raw[0] == 1 and raw[1:17] == bytes(range(16)) and raw[17:29] == bytes(range(16, 28))
    assert len(raw) == 29 + 64 + 16
    assert SS.decrypt_seed(SS.unmarshal(raw), "pw") == seed
    with pytest.raises(SS.WrongPassphrase):
        SS.decrypt_seed(SS.unmarshal(raw), "nope")
    bad = bytearray(raw)
    bad[40] ^= 1
    with pytest.raises(SS.WrongPassphrase):
        SS.decrypt_seed(SS.unmarshal(bytes(bad)), "pw")
    with pytest.raises(S.SeedError, match="too short"):
        SS.unmarshal(raw[:20])
    with pytest.raises(S.SeedError, match="version"):
        SS.unmarshal(b"\x02" + raw[1:])
    with pytest.raises(S.SeedError):
        SS.encrypt_seed(seed, "")


def test_wallet_lifecycle(tmp_path):
    d = tmp_path / "data"
    wm = WalletManager(str(d), "pass1")
    assert wm.is_new and len(wm.mnemonic) == 24 and len(wm.seed) == 64
    assert stat.S_IMODE(os.stat(d).st_mode) == 0o700
    assert stat.S_IMODE(os.stat(d / WALLET_FILE).st_mode) == 0o600
    assert (d / FINGERPRINT_FILE).read_text() == wm.fingerprint
    assert S.mnemonic_to_seed(wm.mnemonic) == wm.seed
    banner = recovery_phrase_banner(wm.mnemonic, wm.fingerprint)
    assert " ".join(wm.mnemonic) in banner and wm.fingerprint in banner
    assert recovery_phrase_banner(None, "x") == ""

    wm2 = WalletManager(str(d), "pass1")
    assert not wm2.is_new and wm2.mnemonic is None and wm2.seed == wm.seed
    with pytest.raises(WalletError, match="unlock failed"):
        WalletManager(str(d), "wrong")
    wm2.change_passphrase("pass1", "pass2")
    assert WalletManager(str(d), "pass2").seed == wm.seed
    with pytest.raises(WalletError, match="incorrect old"):
        wm2.change_passphrase("pass1", "pass3")
    with pytest.raises(WalletError):
        wm2.change_passphrase("pass2", "")
    assert not [p for p in os.listdir(d) if p.endswith(".tmp")]


def test_wallet_args(tmp_path):
    with pytest.raises(WalletError):
        WalletManager("", "p")
    with pytest.raises(WalletError):
        WalletManager(str(tmp_path), "")


def test_wallet_mnemonic_passphrase_changes_seed(tmp_path):
    r = bytes(32) + bytes(range(28))
    a = WalletManager(str(tmp_path / "a"), "p", io.BytesIO(r))
    b = WalletManager(str(tmp_path / "b"), "p", io.BytesIO(r), mnemonic_passphrase="25th")
    assert a.mnemonic == b.mnemonic and a.seed != b.seed
