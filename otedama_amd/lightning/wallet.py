"""WalletManager: create-or-unlock the encrypted seed under the data directory.

Parity: internal/lightning/wallet.go
  * NewWalletManager: dataDir/passphrase required, dir 0700, create on first
    run else decrypt ........................................... wallet.go:108-150
  * Seed / Fingerprint / Mnemonic (first run only) / IsNew ....... wallet.go:153-170
  * createNew: 256-bit entropy → mnemonic → seed, wallet.fingerprint
    written best-effort ......................................... wallet.go:175-203
  * loadExisting: opaque unlock error ............................ wallet.go:206-225
  * save: temp file → fsync → chmod 0600 → rename ................ wallet.go:228-277
  * ChangePassphrase ............................................. wallet.go:282-303
Also the one-time recovery-phrase banner the engine prints
(internal/engine/setup.go:175-197): written to the console stream, never a log.
"""
from __future__ import annotations

import os
import tempfile
from pathlib import Path

from otedama_amd.lightning import seed as S
from otedama_amd.lightning import seedstore as SS

WALLET_FILE = "wallet.dat"
FINGERPRINT_FILE = "wallet.fingerprint"


class WalletError(S.SeedError):
    pass


class WalletManager:
    def __init__(self, data_dir: str, passphrase: str, reader: S.Reader | None = None,
                 wordlist: S.WordList | None = None, mnemonic_passphrase: str = ""):
        if not data_dir:
            raise WalletError("lightning: dataDir must not be empty")
        if not passphrase:
            raise WalletError("lightning: passphrase must not be empty")
        self.data_dir = Path(data_dir)
        self.wordlist = wordlist or S.english_wordlist()
        self._seed = b""
        self._mnemonic: list[str] | None = None
        try:
            self.data_dir.mkdir(mode=0o700, parents=True, exist_ok=True)
        except OSError as exc:
            raise WalletError(f"lightning: create data dir {data_dir!r}: {exc}") from exc
        try:
            (self.data_dir / WALLET_FILE).stat()
        except FileNotFoundError:
            self._create(passphrase, mnemonic_passphrase, reader)
        except OSError as exc:
            raise WalletError(f"lightning: stat wallet file: {exc}") from exc
        else:
            self._load(passphrase)

    @property
    def seed(self) -> bytes:
        return self._seed

    @property
    def fingerprint(self) -> str:
        return S.fingerprint(self._seed)

    @property
    def mnemonic(self) -> list[str] | None:
        return self._mnemonic

    @property
    def is_new(self) -> bool:
        return self._mnemonic is not None

    def _create(self, passphrase: str, mnemonic_passphrase: str, reader) -> None:
        try:
            entropy = S.generate_entropy(S.DEFAULT_ENTROPY_BITS, reader)
        except S.SeedError as exc:
            raise WalletError(f"lightning: generate entropy: {exc}") from exc
        try:
            words = S.entropy_to_mnemonic(entropy, self.wordlist)
        except S.SeedError as exc:
            raise WalletError(f"lightning: entropy to mnemonic: {exc}") from exc
        seed = S.mnemonic_to_seed(words, mnemonic_passphrase)
        self._save(seed, passphrase, reader)
        self._seed, self._mnemonic = seed, words
        try:
            fp = self.data_dir / FINGERPRINT_FILE
            fp.write_text(S.fingerprint(seed))
            os.chmod(fp, 0o600)
        except OSError:
            pass  # UI convenience only; recomputable from the seed

    def _read(self) -> SS.EncryptedSeed:
        try:
            raw = (self.data_dir / WALLET_FILE).read_bytes()
        except OSError as exc:
            raise WalletError(f"lightning: read wallet file: {exc}") from exc
        try:
            return SS.unmarshal(raw)
        except S.SeedError as exc:
            raise WalletError(f"lightning: unmarshal wallet: {exc}") from exc

    def _load(self, passphrase: str) -> None:
        es = self._read()  # read / unmarshal errors are reported as such (wallet.go:207-215)
        try:
            self._seed = SS.decrypt_seed(es, passphrase)
        except S.SeedError:
            raise WalletError("lightning: wallet unlock failed — check your passphrase") from None

    def _save(self, seed: bytes, passphrase: str, reader) -> None:
        try:
            raw = SS.encrypt_seed(seed, passphrase, reader).marshal()
        except S.SeedError as exc:
            raise WalletError(f"lightning: encrypt seed: {exc}") from exc
        try:
            fd, tmp = tempfile.mkstemp(prefix=".wallet-", suffix=".tmp", dir=self.data_dir)
        except OSError as exc:
            raise WalletError(f"lightning: create temp wallet file: {exc}") from exc
        try:
            with os.fdopen(fd, "wb") as f:
                f.write(raw)
                f.flush()
                os.fsync(f.fileno())
            os.chmod(tmp, 0o600)
            os.replace(tmp, self.data_dir / WALLET_FILE)
        except BaseException as exc:
            try:
                os.unlink(tmp)
            except OSError:
                pass
            if isinstance(exc, OSError):
                raise WalletError(f"lightning: write wallet file: {exc}") from exc
            raise

    def change_passphrase(self, old: str, new: str, reader: S.Reader | None = None) -> None:
        if not new:
            raise WalletError("lightning: new passphrase must not be empty")
        es = self._read()
        try:
            seed = SS.decrypt_seed(es, old)
        except S.SeedError:
            raise WalletError("lightning: incorrect old passphrase") from None
        self._save(seed, new, reader)


def recovery_phrase_banner(mnemonic: list[str] | None, fingerprint: str) -> str:
    """The one-time recovery-phrase block (engine/setup.go:175-197); "" when there is nothing to show."""
    if not mnemonic:
        return ""
    bar = "=" * 72
    return (f"\n{bar}\n  WALLET RECOVERY PHRASE — SHOWN ONCE, NEVER AGAIN\n{bar}\n\n"
            f"  {' '.join(mnemonic)}\n\n  Fingerprint: {fingerprint}\n\n"
            f"  Write these {len(mnemonic)} words on paper, in order, and store them somewhere\n"
            "  safe and offline. They are the ONLY way to recover your funds if\n"
            "  wallet.dat is lost or the disk fails.\n\n"
            "  This phrase is not saved to disk and is not written to any log.\n"
            "  Otedama cannot show it to you again.\n"
            f"{bar}\n\n")
