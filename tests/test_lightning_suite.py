"""Wallet seed custody, case by case: mirrors internal/lightning/{seed,coverage,wallet,wallet_extras}_test.go.

Reference behaviours pinned here (file:line in /root/reference/internal/lightning):
  * entropy sizes / reader errors ............................ seed.go:67-117
  * WordList construction (length, empty, UTF-8, duplicates) .. seed.go:121-166
  * mnemonic <-> entropy (empty, count, unknown word, checksum)  seed.go:187-278
  * MnemonicToSeed / Fingerprint .............................. seed.go:295-317
  * EncryptSeed / DecryptSeed / Marshal / Unmarshal ........... seedstore.go:80-208
  * WalletManager lifecycle, atomic save, ChangePassphrase .... wallet.go:108-303
The scrypt work factor is lowered to N=2^10 for every test except the ones that pin the on-disk parameters
(`test_kdf_full_parameters_*`); the KDF is looked up at call time, so the format code under test is the same.
"""
import hashlib
import hmac
import io
import os
import stat
import threading
import unicodedata

import pytest

from otedama_amd.lightning import seed as S
from otedama_amd.lightning import seedstore as SS
from otedama_amd.lightning import wallet as W
from otedama_amd.lightning.wallet import FINGERPRINT_FILE, WALLET_FILE, WalletError, WalletManager, \
    recovery_phrase_banner


@pytest.fixture(autouse=True)
def fast_kdf(monkeypatch):
    monkeypatch.setattr(SS, "SCRYPT_N", 1 << 10)


class FailAfterN:
    """io.Reader that yields a counting pattern, then fails once `n` bytes were read (coverage_test.go:16-33)."""

    def __init__(self, n: int):
        self.remaining = n

    def read(self, k: int) -> bytes:
        if self.remaining == 0:
            return b""
        k = min(k, self.remaining)
        self.remaining -= k
        return bytes(i % 256 for i in range(k))


def synthetic_words(n: int = 2048) -> list[str]:
    return [f"w{i:04d}" for i in range(n)]


def fixed_reader(entropy: bytes = bytes(range(32)), tail: int = 4096) -> io.BytesIO:
    return io.BytesIO(entropy + bytes((7 * i) % 256 for i in range(tail)))


# ---------------------------------------------------------------------------------------------- entropy

@pytest.mark.parametrize("bits", S.VALID_ENTROPY_BITS)
def test_generate_entropy_valid_bit_counts(bits):
    e = S.generate_entropy(bits)
    assert len(e) == bits // 8
    S.validate_entropy(e)


@pytest.mark.parametrize("bits", [0, 8, 64, 96, 100, 127, 129, 288, 512, -128])
def test_generate_entropy_rejects_invalid_bit_counts(bits):
    with pytest.raises(S.SeedError, match="invalid entropy size"):
        S.generate_entropy(bits)


def test_generate_entropy_default_is_256_bits():
    assert len(S.generate_entropy()) == 32 and S.DEFAULT_ENTROPY_BITS == 256


def test_generate_entropy_uses_provided_reader():
    want = bytes(range(100, 132))
    assert S.generate_entropy(256, io.BytesIO(want + b"extra")) == want
    assert S.generate_entropy(128, lambda k: b"\xab" * k) == b"\xab" * 16


def test_generate_entropy_reads_short_chunks_until_full():
    chunks = iter([b"\x01", b"\x02\x03", b"\x04" * 13])
    assert S.generate_entropy(128, lambda k: next(chunks)) == b"\x01\x02\x03" + b"\x04" * 13


def test_generate_entropy_propagates_reader_error():
    with pytest.raises(S.SeedError, match="exhausted after 10 of 32"):
        S.generate_entropy(256, FailAfterN(10))

    def boom(_k):
        raise OSError("device gone")
    with pytest.raises(OSError, match="device gone"):
        S.generate_entropy(256, boom)


def test_generate_entropy_is_not_constant():
    assert len({S.generate_entropy(128) for _ in range(8)}) == 8


@pytest.mark.parametrize("n", [0, 3, 15, 17, 33, 64])
def test_validate_rejects_invalid_entropy_length(n):
    with pytest.raises(S.SeedError, match="invalid entropy length"):
        S.validate_entropy(bytes(n))


# ---------------------------------------------------------------------------------------------- word lists

@pytest.mark.parametrize("n", [0, 1, 2047, 2049])
def test_wordlist_rejects_wrong_length(n):
    with pytest.raises(S.SeedError, match=f"has {n} words"):
        S.WordList(synthetic_words(n))


def test_wordlist_rejects_duplicates():
    words = synthetic_words()
    words[1500] = words[3]
    with pytest.raises(S.SeedError, match="duplicate word 'w0003'"):
        S.WordList(words)


def test_wordlist_rejects_empty_word():
    words = synthetic_words()
    words[77] = ""
    with pytest.raises(S.SeedError, match="entry 77 is empty"):
        S.WordList(words)


def test_wordlist_rejects_invalid_utf8_word():
    words = synthetic_words()
    words[500] = b"\xff\xfe".decode("utf-8", "surrogateescape")
    with pytest.raises(S.SeedError, match="index 500 is not valid UTF-8"):
        S.WordList(words)


def test_wordlist_rejects_non_string_word():
    words = synthetic_words()
    words[9] = None
    with pytest.raises(S.SeedError):
        S.WordList(words)


def test_wordlist_accepts_non_ascii_words():
    words = [f"単語{i}" for i in range(2048)]
    wl = S.WordList(words)
    e = bytes(range(16))
    assert S.mnemonic_to_entropy(S.entropy_to_mnemonic(e, wl), wl) == e


def test_wordlist_is_a_defensive_copy():
    words = synthetic_words()
    wl = S.WordList(words)
    words[0] = "mutated"
    assert wl.word(0) == "w0000" and wl.index("w0000") == 0
    with pytest.raises(S.SeedError):
        wl.index("mutated")


@pytest.mark.parametrize("i", [-1, 2048, 10**6])
def test_word_rejects_out_of_bounds_index(i):
    with pytest.raises(S.SeedError, match="out of range"):
        S.WordList(synthetic_words()).word(i)


def test_index_rejects_unknown_word():
    with pytest.raises(S.SeedError, match="not in wordlist"):
        S.english_wordlist().index("bitcoinx")


def test_english_wordlist_has_exactly_2048_words():
    wl = S.english_wordlist()
    assert len(wl) == 2048
    assert len({wl.word(i) for i in range(2048)}) == 2048


def test_english_wordlist_boundary_words():
    wl = S.english_wordlist()
    assert (wl.word(0), wl.word(1), wl.word(2046), wl.word(2047)) == ("abandon", "ability", "zone", "zoo")
    assert wl.index("abandon") == 0 and wl.index("zoo") == 2047


def test_english_wordlist_is_pinned_by_sha256():
    raw = (S.Path(S.__file__).with_name("bip39_english.txt")).read_bytes()
    assert hashlib.sha256(raw).hexdigest() == S.ENGLISH_SHA256


def test_english_wordlist_words_are_sorted_lowercase_ascii():
    words = [S.english_wordlist().word(i) for i in range(2048)]
    assert words == sorted(words)
    assert all(w.isascii() and w.islower() and 3 <= len(w) <= 8 for w in words)
    assert len({w[:4] for w in words}) == 2048  # BIP-39: the first four letters identify a word


# ---------------------------------------------------------------------------------------------- mnemonics

@pytest.mark.parametrize("bits,count", [(128, 12), (160, 15), (192, 18), (224, 21), (256, 24)])
def test_entropy_to_mnemonic_word_count_matches_entropy(bits, count):
    assert len(S.entropy_to_mnemonic(bytes(bits // 8))) == count


@pytest.mark.parametrize("n", [1, 15, 31, 33])
def test_entropy_to_mnemonic_invalid_entropy(n):
    with pytest.raises(S.SeedError):
        S.entropy_to_mnemonic(bytes(n))


def test_entropy_to_mnemonic_defaults_to_english():
    e = bytes(range(16))
    assert S.entropy_to_mnemonic(e) == S.entropy_to_mnemonic(e, S.english_wordlist())


def test_entropy_mnemonic_roundtrip_deterministic():
    for bits in S.VALID_ENTROPY_BITS:
        e = hashlib.sha256(bits.to_bytes(2, "big")).digest()[: bits // 8]
        m1, m2 = S.entropy_to_mnemonic(e), S.entropy_to_mnemonic(e)
        assert m1 == m2
        assert S.mnemonic_to_entropy(m1) == e
        assert S.mnemonic_to_entropy(" ".join(m1)) == e


def test_entropy_mnemonic_roundtrip_custom_wordlist():
    wl = S.WordList(synthetic_words())
    e = bytes(range(32))
    m = S.entropy_to_mnemonic(e, wl)
    assert all(w.startswith("w") for w in m)
    assert S.mnemonic_to_entropy(m, wl) == e
    with pytest.raises(S.SeedError, match="not in wordlist"):
        S.mnemonic_to_entropy(m)  # English list: synthetic words are unknown


def test_entropy_to_mnemonic_official_all_zero_vector():
    assert " ".join(S.entropy_to_mnemonic(bytes(16))) == " ".join(["abandon"] * 11 + ["about"])
    assert " ".join(S.entropy_to_mnemonic(bytes(32))) == " ".join(["abandon"] * 23 + ["art"])


def test_entropy_to_mnemonic_official_all_ff_vector():
    assert " ".join(S.entropy_to_mnemonic(b"\xff" * 16)) == " ".join(["zoo"] * 11 + ["wrong"])
    assert " ".join(S.entropy_to_mnemonic(b"\xff" * 32)) == " ".join(["zoo"] * 23 + ["vote"])


def test_entropy_to_mnemonic_official_0x80_vector():
    assert " ".join(S.entropy_to_mnemonic(b"\x80" * 16)) == \
        "letter advice cage absurd amount doctor acoustic avoid letter advice cage above"


def test_mnemonic_entropy_all_words_reachable():
    wl = S.english_wordlist()
    for i in range(2048):
        e = (i << 117).to_bytes(16, "big")  # the first 11 bits select word 0
        m = S.entropy_to_mnemonic(e)
        assert m[0] == wl.word(i)
        assert S.mnemonic_to_entropy(m) == e


def test_mnemonic_to_entropy_detects_checksum_mismatch():
    m = S.entropy_to_mnemonic(bytes(range(16)))
    wl = S.english_wordlist()
    m[-1] = wl.word((wl.index(m[-1]) + 1) % 2048)  # low 4 bits are the checksum
    with pytest.raises(S.SeedError, match="checksum mismatch"):
        S.mnemonic_to_entropy(m)


def test_mnemonic_to_entropy_detects_swapped_words():
    m = S.entropy_to_mnemonic(bytes(range(1, 33)))
    m[0], m[1] = m[1], m[0]
    with pytest.raises(S.SeedError, match="checksum"):
        S.mnemonic_to_entropy(m)


def test_mnemonic_to_entropy_rejects_unknown_word():
    m = S.entropy_to_mnemonic(bytes(16))
    m[5] = "qwertyx"
    with pytest.raises(S.SeedError, match=r"word 5: .*'qwertyx' not in wordlist"):
        S.mnemonic_to_entropy(m)


@pytest.mark.parametrize("n", [1, 3, 11, 13, 23, 25, 48])
def test_mnemonic_to_entropy_rejects_wrong_word_count(n):
    with pytest.raises(S.SeedError, match=f"has {n} words"):
        S.mnemonic_to_entropy(["abandon"] * n)


@pytest.mark.parametrize("m", [[], "", "   "])
def test_mnemonic_to_entropy_empty_mnemonic(m):
    with pytest.raises(S.SeedError, match="mnemonic is empty"):
        S.mnemonic_to_entropy(m)


def test_mnemonic_string_is_space_separated():
    m = S.entropy_to_mnemonic(bytes(16))
    assert " ".join(m).split(" ") == m
    assert S.mnemonic_to_entropy("  ".join(m)) == bytes(16)  # str input splits on any whitespace


# ---------------------------------------------------------------------------------------------- seeds

def test_mnemonic_to_seed_deterministic():
    m = S.entropy_to_mnemonic(bytes(range(32)))
    s = S.mnemonic_to_seed(m)
    assert s == S.mnemonic_to_seed(m) == S.mnemonic_to_seed(" ".join(m))
    assert len(s) == S.SEED_BYTES == 64


def test_mnemonic_to_seed_different_passphrase_different_seed():
    m = S.entropy_to_mnemonic(bytes(16))
    seeds = {S.mnemonic_to_seed(m, p) for p in ("", "a", "A", "TREZOR", "a ")}
    assert len(seeds) == 5


def test_mnemonic_to_seed_bip39_official_vector():
    m = "abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon about"
    assert S.mnemonic_to_seed(m, "TREZOR").hex() == (
        "c55257c360c07c72029aebc1b53c05ed0362ada38ead3e3e9efa3708e53495531f09a6987599d18264c1e1c92f2cf141630c7a3c4"
        "ab7c81b2f001698e7463b04")


def test_mnemonic_to_seed_is_pbkdf2_sha512_2048():
    m = "legal winner thank year wave sausage worth useful legal winner thank yellow"
    want = hashlib.pbkdf2_hmac("sha512", m.encode(), b"mnemonicpw", 2048, 64)
    assert S.mnemonic_to_seed(m, "pw") == want


def test_mnemonic_to_seed_nfkd_normalizes_passphrase():
    m = S.entropy_to_mnemonic(bytes(16))
    composed, decomposed = "café", "café"
    assert unicodedata.normalize("NFKD", composed) == decomposed
    assert S.mnemonic_to_seed(m, composed) == S.mnemonic_to_seed(m, decomposed)


# ---------------------------------------------------------------------------------------------- fingerprint

def test_fingerprint_deterministic():
    seed = bytes(range(64))
    assert S.fingerprint(seed) == S.fingerprint(bytes(seed))


def test_fingerprint_different_seeds_different_fingerprints():
    fps = {S.fingerprint(hashlib.sha512(bytes([i])).digest()) for i in range(64)}
    assert len(fps) == 64


def test_fingerprint_is_short_hex():
    fp = S.fingerprint(bytes(64))
    assert len(fp) == 8 and fp == fp.lower() and int(fp, 16) >= 0


def test_fingerprint_is_hmac_sha256_prefix():
    seed = bytes(range(64))
    assert S.fingerprint(seed) == hmac.new(b"otedama-fingerprint-v1", seed, hashlib.sha256).hexdigest()[:8]


# ---------------------------------------------------------------------------------------------- seedstore

SEED = bytes(range(64))


def test_encrypt_decrypt_seed_roundtrip():
    es = SS.encrypt_seed(SEED, "correct horse")
    assert es.version == SS.VERSION == 1 and len(es.salt) == 16 and len(es.nonce) == 12
    assert len(es.ciphertext) == 64 + 16
    assert SS.decrypt_seed(es, "correct horse") == SEED


def test_encrypt_seed_rejects_empty_passphrase():
    with pytest.raises(S.SeedError, match="passphrase must not be empty"):
        SS.encrypt_seed(SEED, "")


def test_decrypt_seed_rejects_wrong_passphrase():
    es = SS.encrypt_seed(SEED, "right")
    for bad in ("wrong", "Right", "right ", ""):
        with pytest.raises(SS.WrongPassphrase, match="wrong passphrase or corrupted file"):
            SS.decrypt_seed(es, bad)


@pytest.mark.parametrize("offset", [1, 16, 17, 28, 29, 60, 29 + 64, 29 + 64 + 15])
def test_decrypt_seed_detects_tampering(offset):
    raw = bytearray(SS.encrypt_seed(SEED, "pw").marshal())
    raw[offset] ^= 0x01  # salt, nonce, ciphertext and tag are all authenticated (salt via the key)
    with pytest.raises(SS.WrongPassphrase):
        SS.decrypt_seed(SS.unmarshal(bytes(raw)), "pw")


def test_decrypt_seed_detects_truncation():
    raw = SS.encrypt_seed(SEED, "pw").marshal()
    with pytest.raises(SS.WrongPassphrase):
        SS.decrypt_seed(SS.unmarshal(raw[:-1]), "pw")


def test_encrypt_seed_produces_different_output_for_same_input():
    a, b = SS.encrypt_seed(SEED, "pw"), SS.encrypt_seed(SEED, "pw")
    assert a.salt != b.salt and a.nonce != b.nonce and a.ciphertext != b.ciphertext


def test_encrypt_seed_uses_reader_for_salt_then_nonce():
    es = SS.encrypt_seed(SEED, "pw", io.BytesIO(bytes(range(28))))
    assert es.salt == bytes(range(16)) and es.nonce == bytes(range(16, 28))
    again = SS.encrypt_seed(SEED, "pw", io.BytesIO(bytes(range(28))))
    assert again.ciphertext == es.ciphertext  # same key + nonce: deterministic


def test_encrypt_seed_salt_read_error():
    with pytest.raises(S.SeedError, match="salt generation failed"):
        SS.encrypt_seed(SEED, "pw", FailAfterN(5))


def test_encrypt_seed_nonce_read_error():
    with pytest.raises(S.SeedError, match="nonce generation failed"):
        SS.encrypt_seed(SEED, "pw", FailAfterN(16 + 3))


def test_encrypted_seed_contains_no_plaintext_seed():
    seed = b"SEEDSEED" * 8
    raw = SS.encrypt_seed(seed, "pw").marshal()
    assert b"SEEDSEED" not in raw and seed[:4] not in raw[29:]


def test_marshal_unmarshal_roundtrip():
    es = SS.encrypt_seed(SEED, "pw")
    raw = es.marshal()
    assert raw[0] == 1 and raw[1:17] == es.salt and raw[17:29] == es.nonce and raw[29:] == es.ciphertext
    assert SS.unmarshal(raw) == es
    assert SS.decrypt_seed(SS.unmarshal(raw), "pw") == SEED


@pytest.mark.parametrize("n", [0, 1, 16, 28])
def test_unmarshal_rejects_short_input(n):
    with pytest.raises(S.SeedError, match=f"too short: {n} bytes, need at least 29"):
        SS.unmarshal(b"\x01" * n)


@pytest.mark.parametrize("version", [0, 2, 0xFF])
def test_unmarshal_rejects_unknown_version(version):
    raw = SS.encrypt_seed(SEED, "pw").marshal()
    with pytest.raises(S.SeedError, match=f"unsupported EncryptedSeed version {version}"):
        SS.unmarshal(bytes([version]) + raw[1:])


def test_unmarshal_minimal_input_has_empty_ciphertext():
    es = SS.unmarshal(b"\x01" + bytes(28))
    assert es.ciphertext == b""
    with pytest.raises(S.SeedError, match="empty ciphertext"):
        SS.decrypt_seed(es, "pw")


def test_marshal_rejects_wrong_version():
    es = SS.encrypt_seed(SEED, "pw")
    es.version = 2
    with pytest.raises(S.SeedError, match="Marshal: unsupported version 2"):
        es.marshal()


def test_decrypt_seed_rejects_wrong_version():
    es = SS.encrypt_seed(SEED, "pw")
    es.version = 9
    with pytest.raises(S.SeedError, match="unsupported EncryptedSeed version 9"):
        SS.decrypt_seed(es, "pw")


def test_decrypt_seed_rejects_empty_ciphertext():
    es = SS.encrypt_seed(SEED, "pw")
    es.ciphertext = b""
    with pytest.raises(S.SeedError, match="empty ciphertext"):
        SS.decrypt_seed(es, "pw")


def test_decrypt_seed_rejects_wrong_plaintext_length():
    es = SS.encrypt_seed(SEED[:32], "pw")  # authentic, but not a 64-byte BIP-39 seed
    with pytest.raises(S.SeedError, match="decrypted seed is 32 bytes, want 64"):
        SS.decrypt_seed(es, "pw")


def test_derive_key_is_scrypt_32_bytes():
    salt = bytes(range(16))
    want = hashlib.scrypt(b"pw", salt=salt, n=SS.SCRYPT_N, r=8, p=1, dklen=32)
    assert SS.derive_key("pw", salt) == want and len(want) == 32


def test_kdf_full_parameters_match_reference(monkeypatch):
    monkeypatch.setattr(SS, "SCRYPT_N", 1 << 17)
    assert (SS.SCRYPT_N, SS.SCRYPT_R, SS.SCRYPT_P) == (131072, 8, 1)  # seedstore.go:68-72
    salt = b"otedama-salt-016"
    want = hashlib.scrypt(b"passphrase", salt=salt, n=1 << 17, r=8, p=1, maxmem=256 << 20, dklen=32)
    assert SS.derive_key("passphrase", salt) == want


def test_kdf_full_parameters_wallet_file_roundtrip(monkeypatch, tmp_path):
    monkeypatch.setattr(SS, "SCRYPT_N", 1 << 17)
    wm = WalletManager(str(tmp_path), "pw", fixed_reader())
    raw = (tmp_path / WALLET_FILE).read_bytes()
    key = hashlib.scrypt(b"pw", salt=raw[1:17], n=1 << 17, r=8, p=1, maxmem=256 << 20, dklen=32)
    from otedama_amd.utils import aead
    assert aead.open_(aead.AES256GCM, key, raw[17:29], raw[29:]) == wm.seed


# ---------------------------------------------------------------------------------------------- WalletManager

def test_wallet_manager_first_run_creates_file(tmp_path):
    d = tmp_path / "otedama"
    assert not d.exists()
    wm = WalletManager(str(d), "pw")
    assert (d / WALLET_FILE).is_file() and wm.is_new
    assert len((d / WALLET_FILE).read_bytes()) == 29 + 64 + 16


def test_wallet_manager_new_run_exposes_mnemonic(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    assert len(wm.mnemonic) == 24
    assert S.mnemonic_to_seed(wm.mnemonic) == wm.seed
    S.mnemonic_to_entropy(wm.mnemonic)  # checksum-valid


def test_wallet_manager_loaded_run_does_not_expose_mnemonic(tmp_path):
    WalletManager(str(tmp_path), "pw")
    wm = WalletManager(str(tmp_path), "pw")
    assert wm.mnemonic is None and not wm.is_new


def test_wallet_manager_mnemonic_is_never_written_to_disk(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    blob = b"".join(p.read_bytes() for p in tmp_path.iterdir())
    assert " ".join(wm.mnemonic).encode() not in blob
    assert not any(w.encode() in blob for w in wm.mnemonic if len(w) > 5)


def test_wallet_manager_seed_is_not_32_zero_bytes(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    assert len(wm.seed) == 64 and wm.seed != bytes(64) and wm.seed[:32] != bytes(32)


def test_wallet_manager_fingerprint_is_stable_across_load(tmp_path):
    fp = WalletManager(str(tmp_path), "pw").fingerprint
    assert WalletManager(str(tmp_path), "pw").fingerprint == fp
    assert (tmp_path / FINGERPRINT_FILE).read_text() == fp


def test_wallet_manager_first_run_fingerprint_consistent(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    assert wm.fingerprint == S.fingerprint(wm.seed) == S.fingerprint(S.mnemonic_to_seed(wm.mnemonic))


def test_wallet_manager_reload_returns_same_seed(tmp_path):
    seed = WalletManager(str(tmp_path), "pw").seed
    for _ in range(2):
        assert WalletManager(str(tmp_path), "pw").seed == seed


def test_wallet_manager_wallet_file_permissions(tmp_path):
    d = tmp_path / "nested" / "dir"
    WalletManager(str(d), "pw")
    assert stat.S_IMODE(os.stat(d).st_mode) == 0o700
    assert stat.S_IMODE(os.stat(d / WALLET_FILE).st_mode) == 0o600
    assert stat.S_IMODE(os.stat(d / FINGERPRINT_FILE).st_mode) == 0o600


def test_wallet_manager_wallet_file_not_world_readable_after_change(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    wm.change_passphrase("pw", "pw2")
    assert stat.S_IMODE(os.stat(tmp_path / WALLET_FILE).st_mode) & 0o077 == 0


def test_wallet_manager_wrong_passphrase(tmp_path):
    WalletManager(str(tmp_path), "pw")
    with pytest.raises(WalletError, match="wallet unlock failed — check your passphrase"):
        WalletManager(str(tmp_path), "pW")


def test_wallet_manager_fixed_reader_produces_deterministic_fingerprint(tmp_path):
    a = WalletManager(str(tmp_path / "a"), "pw", fixed_reader())
    b = WalletManager(str(tmp_path / "b"), "other", fixed_reader())
    assert a.fingerprint == b.fingerprint and a.mnemonic == b.mnemonic
    assert a.mnemonic == S.entropy_to_mnemonic(bytes(range(32)))


def test_wallet_manager_different_passphrases_same_entropy_same_seed(tmp_path):
    a = WalletManager(str(tmp_path / "a"), "pass-one", fixed_reader())
    b = WalletManager(str(tmp_path / "b"), "pass-two", fixed_reader())
    assert a.seed == b.seed  # the file passphrase encrypts; it does not derive
    assert (tmp_path / "a" / WALLET_FILE).read_bytes() != (tmp_path / "b" / WALLET_FILE).read_bytes()


def test_wallet_manager_with_mnemonic_passphrase_changes_derived_seed(tmp_path):
    a = WalletManager(str(tmp_path / "a"), "pw", fixed_reader())
    b = WalletManager(str(tmp_path / "b"), "pw", fixed_reader(), mnemonic_passphrase="25th word")
    assert a.mnemonic == b.mnemonic and a.seed != b.seed


def test_wallet_manager_with_mnemonic_passphrase_matches_direct_derivation(tmp_path):
    wm = WalletManager(str(tmp_path), "pw", mnemonic_passphrase="extra")
    assert wm.seed == S.mnemonic_to_seed(wm.mnemonic, "extra")


def test_wallet_manager_no_mnemonic_passphrase_matches_empty_derivation(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    assert wm.seed == S.mnemonic_to_seed(wm.mnemonic, "")


def test_wallet_manager_mnemonic_passphrase_not_needed_on_reload(tmp_path):
    seed = WalletManager(str(tmp_path), "pw", mnemonic_passphrase="extra").seed
    assert WalletManager(str(tmp_path), "pw").seed == seed  # the derived seed is what is stored
    assert WalletManager(str(tmp_path), "pw", mnemonic_passphrase="ignored").seed == seed


def test_wallet_manager_corrupted_wallet_file_fails_clean(tmp_path):
    WalletManager(str(tmp_path), "pw")
    raw = bytearray((tmp_path / WALLET_FILE).read_bytes())
    raw[50] ^= 0xFF
    (tmp_path / WALLET_FILE).write_bytes(bytes(raw))
    with pytest.raises(WalletError, match="unlock failed"):
        WalletManager(str(tmp_path), "pw")


def test_wallet_manager_garbage_version_fails_clean(tmp_path):
    (tmp_path / WALLET_FILE).write_bytes(b"\x07" + os.urandom(100))
    with pytest.raises(WalletError, match="unmarshal wallet: .*version 7"):
        WalletManager(str(tmp_path), "pw")


def test_wallet_manager_empty_wallet_file_fails_clean(tmp_path):
    (tmp_path / WALLET_FILE).write_bytes(b"")
    with pytest.raises(WalletError, match="unmarshal wallet: .*too short"):
        WalletManager(str(tmp_path), "pw")
    assert (tmp_path / WALLET_FILE).read_bytes() == b""  # never overwritten by a failed load


def test_load_existing_read_file_error(tmp_path):
    (tmp_path / WALLET_FILE).mkdir()
    with pytest.raises(WalletError, match="read wallet file"):
        WalletManager(str(tmp_path), "pw")


@pytest.mark.parametrize("data_dir,passphrase,match", [("", "pw", "dataDir must not be empty"),
                                                        ("x", "", "passphrase must not be empty")])
def test_new_wallet_manager_rejects_empty_arguments(tmp_path, data_dir, passphrase, match):
    with pytest.raises(WalletError, match=match):
        WalletManager(data_dir and str(tmp_path / data_dir), passphrase)
    assert not (tmp_path / "x").exists()


def test_new_wallet_manager_mkdir_error(tmp_path):
    (tmp_path / "file").write_text("not a directory")
    with pytest.raises(WalletError, match="create data dir"):
        WalletManager(str(tmp_path / "file" / "sub"), "pw")


def test_new_wallet_manager_entropy_error(tmp_path):
    with pytest.raises(WalletError, match="generate entropy: .*exhausted"):
        WalletManager(str(tmp_path), "pw", FailAfterN(8))
    assert not (tmp_path / WALLET_FILE).exists()


def test_create_new_encrypt_seed_error(tmp_path):
    with pytest.raises(WalletError, match="encrypt seed: .*salt generation failed"):
        WalletManager(str(tmp_path), "pw", FailAfterN(32 + 4))
    assert not (tmp_path / WALLET_FILE).exists()
    assert not list(tmp_path.iterdir())  # no temp file, no fingerprint


def test_create_new_entropy_to_mnemonic_error(tmp_path, monkeypatch):
    def broken(_e, _wl=None):
        raise S.SeedError("lightning: boom")
    monkeypatch.setattr(S, "entropy_to_mnemonic", broken)
    with pytest.raises(WalletError, match="entropy to mnemonic: lightning: boom"):
        WalletManager(str(tmp_path), "pw")


def test_save_create_temp_error(tmp_path, monkeypatch):
    def no_temp(*_a, **_k):
        raise OSError(28, "No space left on device")
    monkeypatch.setattr(W.tempfile, "mkstemp", no_temp)
    with pytest.raises(WalletError, match="create temp wallet file"):
        WalletManager(str(tmp_path), "pw")
    assert not (tmp_path / WALLET_FILE).exists()


def test_save_rename_error_target_is_directory(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    (tmp_path / WALLET_FILE).unlink()
    (tmp_path / WALLET_FILE).mkdir()
    (tmp_path / WALLET_FILE / "keep").write_text("x")
    with pytest.raises(WalletError, match="write wallet file"):
        wm._save(wm.seed, "pw", None)
    assert not [p for p in tmp_path.iterdir() if p.name.endswith(".tmp")]


def test_save_fsync_error_removes_temp(tmp_path, monkeypatch):
    wm = WalletManager(str(tmp_path), "pw")
    before = (tmp_path / WALLET_FILE).read_bytes()

    def bad_fsync(_fd):
        raise OSError(5, "I/O error")
    monkeypatch.setattr(W.os, "fsync", bad_fsync)
    with pytest.raises(WalletError, match="I/O error"):
        wm.change_passphrase("pw", "new")
    assert (tmp_path / WALLET_FILE).read_bytes() == before  # the old file survives intact
    assert not [p for p in tmp_path.iterdir() if p.name.endswith(".tmp")]


def test_fingerprint_file_write_failure_is_not_fatal(tmp_path):
    (tmp_path / FINGERPRINT_FILE).mkdir()
    wm = WalletManager(str(tmp_path), "pw")
    assert wm.is_new and (tmp_path / WALLET_FILE).is_file()


def test_change_passphrase(tmp_path):
    wm = WalletManager(str(tmp_path), "old")
    wm.change_passphrase("old", "new")
    assert WalletManager(str(tmp_path), "new").seed == wm.seed
    with pytest.raises(WalletError):
        WalletManager(str(tmp_path), "old")


def test_change_passphrase_wrong_old(tmp_path):
    wm = WalletManager(str(tmp_path), "old")
    before = (tmp_path / WALLET_FILE).read_bytes()
    with pytest.raises(WalletError, match="incorrect old passphrase"):
        wm.change_passphrase("nope", "new")
    assert (tmp_path / WALLET_FILE).read_bytes() == before


def test_change_passphrase_empty_new(tmp_path):
    wm = WalletManager(str(tmp_path), "old")
    with pytest.raises(WalletError, match="new passphrase must not be empty"):
        wm.change_passphrase("old", "")


def test_change_passphrase_twice_in_a_row(tmp_path):
    wm = WalletManager(str(tmp_path), "a")
    wm.change_passphrase("a", "b")
    wm.change_passphrase("b", "c")
    assert WalletManager(str(tmp_path), "c").seed == wm.seed
    for stale in ("a", "b"):
        with pytest.raises(WalletError):
            WalletManager(str(tmp_path), stale)


def test_change_passphrase_same_old_and_new(tmp_path):
    wm = WalletManager(str(tmp_path), "same")
    before = (tmp_path / WALLET_FILE).read_bytes()
    wm.change_passphrase("same", "same")
    after = (tmp_path / WALLET_FILE).read_bytes()
    assert after != before  # fresh salt and nonce
    assert WalletManager(str(tmp_path), "same").seed == wm.seed


def test_change_passphrase_does_not_create_temp_file(tmp_path):
    wm = WalletManager(str(tmp_path), "a")
    wm.change_passphrase("a", "b")
    assert sorted(p.name for p in tmp_path.iterdir()) == sorted([FINGERPRINT_FILE, WALLET_FILE])


def test_change_passphrase_wallet_file_missing(tmp_path):
    wm = WalletManager(str(tmp_path), "a")
    (tmp_path / WALLET_FILE).unlink()
    with pytest.raises(WalletError, match="read wallet file"):
        wm.change_passphrase("a", "b")


def test_change_passphrase_unmarshal_error(tmp_path):
    wm = WalletManager(str(tmp_path), "a")
    (tmp_path / WALLET_FILE).write_bytes(b"\x01short")
    with pytest.raises(WalletError, match="unmarshal wallet"):
        wm.change_passphrase("a", "b")


def test_change_passphrase_uses_reader(tmp_path):
    wm = WalletManager(str(tmp_path), "a")
    wm.change_passphrase("a", "b", io.BytesIO(bytes(range(100, 128))))
    raw = (tmp_path / WALLET_FILE).read_bytes()
    assert raw[1:17] == bytes(range(100, 116)) and raw[17:29] == bytes(range(116, 128))


def test_wallet_manager_concurrent_getters_are_safe(tmp_path):
    wm = WalletManager(str(tmp_path), "pw")
    want = (wm.seed, wm.fingerprint, wm.is_new)
    errors = []

    def reader():
        for _ in range(200):
            if (wm.seed, wm.fingerprint, wm.is_new) != want:
                errors.append("mismatch")
    threads = [threading.Thread(target=reader) for _ in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors


def test_recovery_phrase_banner_shows_words_in_order_once(tmp_path):
    wm = WalletManager(str(tmp_path), "pw", fixed_reader())
    banner = recovery_phrase_banner(wm.mnemonic, wm.fingerprint)
    assert " ".join(wm.mnemonic) in banner and f"Fingerprint: {wm.fingerprint}" in banner
    assert "Write these 24 words" in banner and "SHOWN ONCE" in banner
    reloaded = WalletManager(str(tmp_path), "pw")
    assert recovery_phrase_banner(reloaded.mnemonic, reloaded.fingerprint) == ""
    assert recovery_phrase_banner([], "abcd") == ""
