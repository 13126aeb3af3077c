// AEAD (AES-256-GCM, ChaCha20-Poly1305) for wallet storage and the Noise transport.
#pragma once

#include <cstddef>
#include <string>

namespace otedama {

enum class AeadKind { kAes256Gcm = 0, kChaCha20Poly1305 = 1 };
constexpr int kAeadTagBytes = 16;

// Returns ciphertext || 16-byte tag. key: 32 bytes, nonce: 12 bytes.
std::string aead_seal(AeadKind kind, const std::string& key, const std::string& nonce, const std::string& plain,
                      const std::string& aad);
// Returns false on authentication failure (wrong key or tampered data).
bool aead_open(AeadKind kind, const std::string& key, const std::string& nonce, const std::string& sealed,
               const std::string& aad, std::string* plain);

}  // namespace otedama
