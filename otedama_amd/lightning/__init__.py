"""Receive-only wallet seed custody (BIP-39 + scrypt/AES-256-GCM wallet.dat). See internal/lightning/."""
from otedama_amd.lightning.seed import (  # noqa: F401
    SeedError, WordList, english_wordlist, entropy_to_mnemonic, fingerprint, generate_entropy,
    mnemonic_to_entropy, mnemonic_to_seed,
)
from otedama_amd.lightning.seedstore import (  # noqa: F401
    EncryptedSeed, WrongPassphrase, decrypt_seed, encrypt_seed, unmarshal,
)
from otedama_amd.lightning.wallet import WalletError, WalletManager, recovery_phrase_banner  # noqa: F401
