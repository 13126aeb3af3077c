// Host AEAD primitives for the control plane, on OpenSSL EVP (libcrypto 3).
//
//  * AES-256-GCM: wallet.dat seed encryption (internal/lightning/seedstore.go:80-164 uses
//    Go's crypto/cipher GCM with a 12-byte nonce and 16-byte tag appended to the ciphertext;
//    we emit the same ciphertext||tag layout so files are interchangeable).
//  * ChaCha20-Poly1305 (IETF, 96-bit nonce): the Noise NX transport cipher
//    (stratum/noise.go:211-249).
// Neither is on the mining hot path, so plain EVP calls are enough.
#include "otedama/aead.h"

#include <openssl/evp.h>

#include <memory>
#include <stdexcept>

namespace otedama {
namespace {

struct CtxFree {
  void operator()(EVP_CIPHER_CTX* c) const { EVP_CIPHER_CTX_free(c); }
};
using Ctx = std::unique_ptr<EVP_CIPHER_CTX, CtxFree>;

const EVP_CIPHER* cipher_for(AeadKind k) {
  return k == AeadKind::kAes256Gcm ? EVP_aes_256_gcm() : EVP_chacha20_poly1305();
}

void check(int ok, const char* what) {
  if (ok != 1) throw std::runtime_error(std::string("aead: ") + what + " failed");
}

}  // namespace

std::string aead_seal(AeadKind kind, const std::string& key, const std::string& nonce, const std::string& plain,
                      const std::string& aad) {
  if (key.size() != 32) throw std::invalid_argument("aead: key must be 32 bytes");
  if (nonce.size() != 12) throw std::invalid_argument("aead: nonce must be 12 bytes");
  Ctx ctx(EVP_CIPHER_CTX_new());
  if (!ctx) throw std::bad_alloc();
  const auto* k = reinterpret_cast<const unsigned char*>(key.data());
  const auto* n = reinterpret_cast<const unsigned char*>(nonce.data());
  check(EVP_EncryptInit_ex(ctx.get(), cipher_for(kind), nullptr, nullptr, nullptr), "init");
  check(EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_AEAD_SET_IVLEN, 12, nullptr), "ivlen");
  check(EVP_EncryptInit_ex(ctx.get(), nullptr, nullptr, k, n), "key");
  int len = 0;
  if (!aad.empty())
    check(EVP_EncryptUpdate(ctx.get(), nullptr, &len, reinterpret_cast<const unsigned char*>(aad.data()),
                            static_cast<int>(aad.size())),
          "aad");
  std::string out(plain.size() + kAeadTagBytes, '\0');
  auto* o = reinterpret_cast<unsigned char*>(&out[0]);
  int total = 0;
  if (!plain.empty()) {
    check(EVP_EncryptUpdate(ctx.get(), o, &len, reinterpret_cast<const unsigned char*>(plain.data()),
                            static_cast<int>(plain.size())),
          "update");
    total = len;
  }
  check(EVP_EncryptFinal_ex(ctx.get(), o + total, &len), "final");
  total += len;
  check(EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_AEAD_GET_TAG, kAeadTagBytes, o + total), "tag");
  out.resize(total + kAeadTagBytes);
  return out;
}

bool aead_open(AeadKind kind, const std::string& key, const std::string& nonce, const std::string& sealed,
               const std::string& aad, std::string* plain) {
  if (key.size() != 32) throw std::invalid_argument("aead: key must be 32 bytes");
  if (nonce.size() != 12) throw std::invalid_argument("aead: nonce must be 12 bytes");
  if (sealed.size() < kAeadTagBytes) return false;
  Ctx ctx(EVP_CIPHER_CTX_new());
  if (!ctx) throw std::bad_alloc();
  const size_t clen = sealed.size() - kAeadTagBytes;
  check(EVP_DecryptInit_ex(ctx.get(), cipher_for(kind), nullptr, nullptr, nullptr), "init");
  check(EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_AEAD_SET_IVLEN, 12, nullptr), "ivlen");
  check(EVP_DecryptInit_ex(ctx.get(), nullptr, nullptr, reinterpret_cast<const unsigned char*>(key.data()),
                           reinterpret_cast<const unsigned char*>(nonce.data())),
        "key");
  int len = 0;
  if (!aad.empty())
    check(EVP_DecryptUpdate(ctx.get(), nullptr, &len, reinterpret_cast<const unsigned char*>(aad.data()),
                            static_cast<int>(aad.size())),
          "aad");
  std::string out(clen, '\0');
  auto* o = reinterpret_cast<unsigned char*>(&out[0]);
  int total = 0;
  if (clen) {
    check(EVP_DecryptUpdate(ctx.get(), o, &len, reinterpret_cast<const unsigned char*>(sealed.data()),
                            static_cast<int>(clen)),
          "update");
    total = len;
  }
  std::string tag = sealed.substr(clen);
  check(EVP_CIPHER_CTX_ctrl(ctx.get(), EVP_CTRL_AEAD_SET_TAG, kAeadTagBytes, &tag[0]), "settag");
  if (EVP_DecryptFinal_ex(ctx.get(), o + total, &len) != 1) {
    // authentication failure: wipe whatever was decrypted
    for (auto& c : out) c = 0;
    return false;
  }
  out.resize(total + len);
  *plain = std::move(out);
  return true;
}

}  // namespace otedama
