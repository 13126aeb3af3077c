// Host side of the mining runtime: job variants, share verification, the share
// queue, the CPU miner and the CPU scrypt reference.
#include <cpuid.h>
#include <immintrin.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <vector>

#include "otedama/job.h"
#include "otedama/runtime.h"
#include "otedama/sha256.h"
#include "otedama/x11.h"

namespace otedama {

// ---------------------------------------------------------------- job variants

static uint32_t popcount32(uint32_t x) { return uint32_t(__builtin_popcount(x)); }

// Scatter the low bits of `v` into the set bits of `mask` (software pdep).
static uint32_t deposit_bits(uint32_t v, uint32_t mask) {
  uint32_t out = 0;
  for (uint32_t bit = 1; mask; bit <<= 1) {
    uint32_t low = mask & (~mask + 1);
    if (v & bit) out |= low;
    mask &= mask - 1;
  }
  return out;
}

static uint64_t en2_space(const JobTemplate& j) {
  if (!j.has_coinbase || j.extranonce2_size == 0) return 1;
  if (j.extranonce2_size >= 8) return ~0ull;
  return 1ull << (8 * j.extranonce2_size);
}

uint64_t JobTemplate::variant_space() const {
  const uint64_t e = en2_space(*this);
  const uint32_t vb = popcount32(version_mask);
  const uint64_t v = vb >= 32 ? (1ull << 32) : (1ull << vb);
  const uint64_t t = uint64_t(ntime_roll) + 1;
  // saturating product
  uint64_t s = e;
  if (s > (~0ull) / v) return ~0ull;
  s *= v;
  if (s > (~0ull) / t) return ~0ull;
  return s * t;
}

void merkle_root_from_coinbase(const JobTemplate& j, uint64_t en2, uint8_t root[32]) {
  std::vector<uint8_t> cb;
  cb.reserve(j.coinb1.size() + j.extranonce1.size() + j.extranonce2_size + j.coinb2.size());
  cb.insert(cb.end(), j.coinb1.begin(), j.coinb1.end());
  cb.insert(cb.end(), j.extranonce1.begin(), j.extranonce1.end());
  for (uint32_t i = 0; i < j.extranonce2_size; ++i) cb.push_back(i < 8 ? uint8_t(en2 >> (8 * i)) : 0);
  cb.insert(cb.end(), j.coinb2.begin(), j.coinb2.end());
  sha256d(cb.data(), cb.size(), root);
  uint8_t buf[64];
  for (const auto& br : j.merkle_branches) {
    std::memcpy(buf, root, 32);
    std::memcpy(buf + 32, br.data(), br.size() < 32 ? br.size() : 32);
    sha256d(buf, 64, root);
  }
}

// Digit order of the variant index, lowest first: BIP320 version bits, then extranonce2, then ntime. Neighbouring
// stripe positions therefore differ only in the version word (block 1 of the header) and share bytes 64..79, so
// the K-variant SHA-256d kernel can group them and reuse one block-2 message schedule, also on Stratum V1 jobs
// with a coinbase (extranonce2 rolls only after the 2^popcount(mask) version variants of one merkle root are
// used). ntime rolls last: it moves the header clock forward, which pools bound.
void JobTemplate::variant_header(uint64_t v, uint8_t out[80], uint32_t* version, uint32_t* ntime,
                                 uint64_t* extranonce2) const {
  std::memcpy(out, header, 80);
  const uint32_t vb = popcount32(version_mask);
  uint32_t ver = load_le32(header);
  if (vb) {
    const uint64_t vs = vb >= 32 ? (1ull << 32) : (1ull << vb);
    const uint32_t bits = uint32_t(v % vs);
    v /= vs;
    ver = (ver & ~version_mask) | deposit_bits(bits, version_mask);
    store_le32(out, ver);
  }
  const uint64_t es = en2_space(*this);
  uint64_t en2 = 0;
  if (es > 1) {
    if (es == ~0ull) { en2 = v; v = 0; }
    else { en2 = v % es; v /= es; }
  }
  uint32_t nt = load_le32(header + 68);
  if (ntime_roll) {
    nt += uint32_t(v % (uint64_t(ntime_roll) + 1));
    store_le32(out + 68, nt);
  }
  if (has_coinbase) {
    uint8_t root[32];
    merkle_root_from_coinbase(*this, en2, root);
    std::memcpy(out + 36, root, 32);
  }
  if (version) *version = ver;
  if (ntime) *ntime = nt;
  if (extranonce2) *extranonce2 = en2;
}

// ------------------------------------------------------------------- scrypt

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void salsa20_8(uint32_t B[16]) {
  uint32_t x[16];
  std::memcpy(x, B, 64);
  for (int i = 0; i < 8; i += 2) {
    x[4] ^= rotl32(x[0] + x[12], 7);   x[8] ^= rotl32(x[4] + x[0], 9);
    x[12] ^= rotl32(x[8] + x[4], 13);  x[0] ^= rotl32(x[12] + x[8], 18);
    x[9] ^= rotl32(x[5] + x[1], 7);    x[13] ^= rotl32(x[9] + x[5], 9);
    x[1] ^= rotl32(x[13] + x[9], 13);  x[5] ^= rotl32(x[1] + x[13], 18);
    x[14] ^= rotl32(x[10] + x[6], 7);  x[2] ^= rotl32(x[14] + x[10], 9);
    x[6] ^= rotl32(x[2] + x[14], 13);  x[10] ^= rotl32(x[6] + x[2], 18);
    x[3] ^= rotl32(x[15] + x[11], 7);  x[7] ^= rotl32(x[3] + x[15], 9);
    x[11] ^= rotl32(x[7] + x[3], 13);  x[15] ^= rotl32(x[11] + x[7], 18);
    x[1] ^= rotl32(x[0] + x[3], 7);    x[2] ^= rotl32(x[1] + x[0], 9);
    x[3] ^= rotl32(x[2] + x[1], 13);   x[0] ^= rotl32(x[3] + x[2], 18);
    x[6] ^= rotl32(x[5] + x[4], 7);    x[7] ^= rotl32(x[6] + x[5], 9);
    x[4] ^= rotl32(x[7] + x[6], 13);   x[5] ^= rotl32(x[4] + x[7], 18);
    x[11] ^= rotl32(x[10] + x[9], 7);  x[8] ^= rotl32(x[11] + x[10], 9);
    x[9] ^= rotl32(x[8] + x[11], 13);  x[10] ^= rotl32(x[9] + x[8], 18);
    x[12] ^= rotl32(x[15] + x[14], 7); x[13] ^= rotl32(x[12] + x[15], 9);
    x[14] ^= rotl32(x[13] + x[12], 13); x[15] ^= rotl32(x[14] + x[13], 18);
  }
  for (int i = 0; i < 16; ++i) B[i] += x[i];
}

// scrypt(N=1024, r=1, p=1) of an 80-byte header, password = salt = header.
void scrypt_1024_1_1(const uint8_t header80[80], uint8_t out[32]) {
  uint8_t b[128];
  pbkdf2_sha256(header80, 80, header80, 80, 1, b, 128);
  uint32_t X[32];
  for (int i = 0; i < 32; ++i) X[i] = load_le32(b + 4 * i);
  // Per-thread pad: a fresh 128 KiB vector sits at glibc's mmap threshold, and the mmap/munmap pair per
  // hash serialised concurrent verifiers on the kernel mm lock (4 threads ran at 0.93x of one).
  thread_local std::vector<uint32_t> V(32 * 1024);
  for (int i = 0; i < 1024; ++i) {
    std::memcpy(&V[32 * i], X, 128);
    for (int k = 0; k < 16; ++k) X[k] ^= X[16 + k];
    salsa20_8(X);
    for (int k = 0; k < 16; ++k) X[16 + k] ^= X[k];
    salsa20_8(X + 16);
  }
  for (int i = 0; i < 1024; ++i) {
    const uint32_t j = X[16] & 1023;
    for (int k = 0; k < 32; ++k) X[k] ^= V[32 * j + k];
    for (int k = 0; k < 16; ++k) X[k] ^= X[16 + k];
    salsa20_8(X);
    for (int k = 0; k < 16; ++k) X[16 + k] ^= X[k];
    salsa20_8(X + 16);
  }
  for (int i = 0; i < 32; ++i) store_le32(b + 4 * i, X[i]);
  pbkdf2_sha256(header80, 80, b, 128, 1, out, 32);
}

// Eight scrypt(1024, 1, 1) hashes at once with AVX2: word k of lane l's 1 KiB-wide state lives in lane l of X[k], the
// 1 MiB pad holds the eight lanes' entries interleaved the same way, and each lookup gathers its lanes' own rows.
// The host verifier of the GPU miner and the CPU miner hash scrypt candidates in batches of up to eight this way.
__attribute__((target("avx2"))) static inline __m256i rotl_x8(__m256i x, int n) {
  return _mm256_or_si256(_mm256_slli_epi32(x, n), _mm256_srli_epi32(x, 32 - n));
}

__attribute__((target("avx2"))) static void salsa20_8_x8(__m256i B[16]) {
  __m256i x[16];
  for (int i = 0; i < 16; ++i) x[i] = B[i];
#define QS(a, b, c, n) x[a] = _mm256_xor_si256(x[a], rotl_x8(_mm256_add_epi32(x[b], x[c]), n))
  for (int i = 0; i < 8; i += 2) {
    QS(4, 0, 12, 7);   QS(8, 4, 0, 9);    QS(12, 8, 4, 13);   QS(0, 12, 8, 18);
    QS(9, 5, 1, 7);    QS(13, 9, 5, 9);   QS(1, 13, 9, 13);   QS(5, 1, 13, 18);
    QS(14, 10, 6, 7);  QS(2, 14, 10, 9);  QS(6, 2, 14, 13);   QS(10, 6, 2, 18);
    QS(3, 15, 11, 7);  QS(7, 3, 15, 9);   QS(11, 7, 3, 13);   QS(15, 11, 7, 18);
    QS(1, 0, 3, 7);    QS(2, 1, 0, 9);    QS(3, 2, 1, 13);    QS(0, 3, 2, 18);
    QS(6, 5, 4, 7);    QS(7, 6, 5, 9);    QS(4, 7, 6, 13);    QS(5, 4, 7, 18);
    QS(11, 10, 9, 7);  QS(8, 11, 10, 9);  QS(9, 8, 11, 13);   QS(10, 9, 8, 18);
    QS(12, 15, 14, 7); QS(13, 12, 15, 9); QS(14, 13, 12, 13); QS(15, 14, 13, 18);
  }
#undef QS
  for (int i = 0; i < 16; ++i) B[i] = _mm256_add_epi32(B[i], x[i]);
}

__attribute__((target("avx2"))) static void scrypt_romix_x8(uint32_t Xs[8][32]) {
  alignas(32) __m256i X[32];
  for (int k = 0; k < 32; ++k)
    X[k] = _mm256_setr_epi32(int(Xs[0][k]), int(Xs[1][k]), int(Xs[2][k]), int(Xs[3][k]), int(Xs[4][k]),
                             int(Xs[5][k]), int(Xs[6][k]), int(Xs[7][k]));
  // per thread, reused: 1024 entries x 32 words x 8 lanes (1 MiB). A std::vector<__m256i> would drop the type's
  // 32-byte alignment (GCC ignores attributes on template arguments) and the aligned stores would fault.
  struct Pad {
    __m256i* p = static_cast<__m256i*>(std::aligned_alloc(64, 1024 * 32 * sizeof(__m256i)));
    ~Pad() { std::free(p); }
  };
  thread_local Pad pad;
  __m256i* V = pad.p;
  if (V == nullptr) throw std::bad_alloc();
  for (int i = 0; i < 1024; ++i) {
    std::memcpy(&V[32 * size_t(i)], X, sizeof X);
    for (int k = 0; k < 16; ++k) X[k] = _mm256_xor_si256(X[k], X[16 + k]);
    salsa20_8_x8(X);
    for (int k = 0; k < 16; ++k) X[16 + k] = _mm256_xor_si256(X[16 + k], X[k]);
    salsa20_8_x8(X + 16);
  }
  const int* base = reinterpret_cast<const int*>(V);
  const __m256i lane = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
  const __m256i mask = _mm256_set1_epi32(1023);
  for (int i = 0; i < 1024; ++i) {
    // lane l's row j_l: 32-bit element (j_l * 32 + k) * 8 + l of the pad
    const __m256i row = _mm256_add_epi32(_mm256_slli_epi32(_mm256_and_si256(X[16], mask), 8), lane);
    for (int k = 0; k < 32; ++k)
      X[k] = _mm256_xor_si256(X[k], _mm256_i32gather_epi32(base, _mm256_add_epi32(row, _mm256_set1_epi32(8 * k)), 4));
    for (int k = 0; k < 16; ++k) X[k] = _mm256_xor_si256(X[k], X[16 + k]);
    salsa20_8_x8(X);
    for (int k = 0; k < 16; ++k) X[16 + k] = _mm256_xor_si256(X[16 + k], X[k]);
    salsa20_8_x8(X + 16);
  }
  alignas(32) uint32_t w[8];
  for (int k = 0; k < 32; ++k) {
    _mm256_store_si256(reinterpret_cast<__m256i*>(w), X[k]);
    for (int l = 0; l < 8; ++l) Xs[l][k] = w[l];
  }
}

static bool cpu_has_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2");
  return ok;
}

// Sixteen at once with AVX-512 (the MI355X hosts' Zen 5 cores have a full-width 512-bit datapath): same layout as
// the eight-lane pass with 16 lanes per word, and Salsa's rotates as single vprold instructions (three operations
// per step instead of the five AVX2 needs for add, shift, shift, or, xor).
__attribute__((target("avx512f"))) static void salsa20_8_x16(__m512i B[16]) {
  __m512i x[16];
  for (int i = 0; i < 16; ++i) x[i] = B[i];
#define QS(a, b, c, n) x[a] = _mm512_xor_si512(x[a], _mm512_rol_epi32(_mm512_add_epi32(x[b], x[c]), n))
  for (int i = 0; i < 8; i += 2) {
    QS(4, 0, 12, 7);   QS(8, 4, 0, 9);    QS(12, 8, 4, 13);   QS(0, 12, 8, 18);
    QS(9, 5, 1, 7);    QS(13, 9, 5, 9);   QS(1, 13, 9, 13);   QS(5, 1, 13, 18);
    QS(14, 10, 6, 7);  QS(2, 14, 10, 9);  QS(6, 2, 14, 13);   QS(10, 6, 2, 18);
    QS(3, 15, 11, 7);  QS(7, 3, 15, 9);   QS(11, 7, 3, 13);   QS(15, 11, 7, 18);
    QS(1, 0, 3, 7);    QS(2, 1, 0, 9);    QS(3, 2, 1, 13);    QS(0, 3, 2, 18);
    QS(6, 5, 4, 7);    QS(7, 6, 5, 9);    QS(4, 7, 6, 13);    QS(5, 4, 7, 18);
    QS(11, 10, 9, 7);  QS(8, 11, 10, 9);  QS(9, 8, 11, 13);   QS(10, 9, 8, 18);
    QS(12, 15, 14, 7); QS(13, 12, 15, 9); QS(14, 13, 12, 13); QS(15, 14, 13, 18);
  }
#undef QS
  for (int i = 0; i < 16; ++i) B[i] = _mm512_add_epi32(B[i], x[i]);
}

__attribute__((target("avx512f"))) static void scrypt_romix_x16(uint32_t Xs[16][32]) {
  alignas(64) __m512i X[32];
  alignas(64) uint32_t w[16];
  for (int k = 0; k < 32; ++k) {
    for (int l = 0; l < 16; ++l) w[l] = Xs[l][k];
    X[k] = _mm512_load_si512(w);
  }
  struct Pad {  // per thread, reused: 1024 entries x 32 words x 16 lanes (2 MiB)
    __m512i* p = static_cast<__m512i*>(std::aligned_alloc(64, 1024 * 32 * sizeof(__m512i)));
    ~Pad() { std::free(p); }
  };
  thread_local Pad pad;
  __m512i* V = pad.p;
  if (V == nullptr) throw std::bad_alloc();
  for (int i = 0; i < 1024; ++i) {
    for (int k = 0; k < 32; ++k) _mm512_store_si512(&V[32 * size_t(i) + k], X[k]);
    for (int k = 0; k < 16; ++k) X[k] = _mm512_xor_si512(X[k], X[16 + k]);
    salsa20_8_x16(X);
    for (int k = 0; k < 16; ++k) X[16 + k] = _mm512_xor_si512(X[16 + k], X[k]);
    salsa20_8_x16(X + 16);
  }
  const int* base = reinterpret_cast<const int*>(V);
  const __m512i lane = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  const __m512i mask = _mm512_set1_epi32(1023);
  for (int i = 0; i < 1024; ++i) {
    // lane l's row j_l: 32-bit element (j_l * 32 + k) * 16 + l of the pad
    const __m512i row = _mm512_add_epi32(_mm512_slli_epi32(_mm512_and_si512(X[16], mask), 9), lane);
    for (int k = 0; k < 32; ++k)
      X[k] = _mm512_xor_si512(X[k], _mm512_i32gather_epi32(_mm512_add_epi32(row, _mm512_set1_epi32(16 * k)), base, 4));
    for (int k = 0; k < 16; ++k) X[k] = _mm512_xor_si512(X[k], X[16 + k]);
    salsa20_8_x16(X);
    for (int k = 0; k < 16; ++k) X[16 + k] = _mm512_xor_si512(X[16 + k], X[k]);
    salsa20_8_x16(X + 16);
  }
  for (int k = 0; k < 32; ++k) {
    _mm512_store_si512(w, X[k]);
    for (int l = 0; l < 16; ++l) Xs[l][k] = w[l];
  }
}

constexpr int kScryptMin16 = 9;  // below this many headers one 16-lane pass costs more than an 8-lane one

static bool cpu_has_avx512() {
  static const bool ok = [] {
    const char* off = std::getenv("OTEDAMA_NO_AVX512");  // set (not "" / "0"): the AVX2 widths only
    return __builtin_cpu_supports("avx512f") && !(off && *off && std::strcmp(off, "0") != 0);
  }();
  return ok;
}

// One pass of up to L lanes (8: AVX2, 16: AVX-512); lanes past m repeat the last header.
template <int L>
static void scrypt_pass(int m, const uint8_t* const header80[], uint8_t* const out[]) {
  uint32_t Xs[L][32];
  uint8_t b[128];
  for (int l = 0; l < L; ++l) {
    const uint8_t* h = header80[std::min(l, m - 1)];
    pbkdf2_sha256(h, 80, h, 80, 1, b, 128);
    for (int k = 0; k < 32; ++k) Xs[l][k] = load_le32(b + 4 * k);
  }
  if constexpr (L == 16) scrypt_romix_x16(Xs);
  else scrypt_romix_x8(Xs);
  for (int l = 0; l < m; ++l) {
    for (int k = 0; k < 32; ++k) store_le32(b + 4 * k, Xs[l][k]);
    pbkdf2_sha256(header80[l], 80, b, 128, 1, out[l], 32);
  }
}

void scrypt_1024_1_1_batch(int n, const uint8_t* const header80[], uint8_t* const out[]) {
  const bool w16 = cpu_has_avx512(), w8 = cpu_has_avx2();
  for (int at = 0; at < n;) {
    const int m = n - at;
    if (w16 && m >= kScryptMin16) {
      const int t = std::min(16, m);
      scrypt_pass<16>(t, header80 + at, out + at);
      at += t;
    } else if (w8 && m >= 3) {  // eight lanes cost ~3 scalar hashes: one or two headers go the scalar way
      const int t = std::min(8, m);
      scrypt_pass<8>(t, header80 + at, out + at);
      at += t;
    } else {
      scrypt_1024_1_1(header80[at], out[at]);
      ++at;
    }
  }
}

bool verify_share(Algo algo, const uint8_t header80[80], const uint8_t target[32], uint8_t hash_out[32]) {
  if (algo == Algo::kScrypt) scrypt_1024_1_1(header80, hash_out);
  else if (algo == Algo::kX11) x11::x11(header80, 80, hash_out, nullptr);
  else sha256d(header80, 80, hash_out);
  return le256_leq(hash_out, target);
}

// -------------------------------------------------------------- share queue

ShareQueue::ShareQueue(size_t cap) : cap_(cap) {
  efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (efd_ < 0) throw std::runtime_error(std::string("eventfd: ") + std::strerror(errno));
}

ShareQueue::~ShareQueue() {
  if (efd_ >= 0) close(efd_);
}

bool ShareQueue::push(ShareRecord&& s) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() >= cap_) {
      dropped_.fetch_add(1);
      return false;
    }
    q_.push_back(std::move(s));
  }
  // Wake the consumer. The counter saturates harmlessly (EAGAIN at 2^64-2): readers drain the whole queue.
  const uint64_t one = 1;
  ssize_t rc;
  do rc = write(efd_, &one, sizeof one); while (rc < 0 && errno == EINTR);
  return true;
}

std::vector<ShareRecord> ShareQueue::drain(size_t max) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<ShareRecord> out;
  while (!q_.empty() && out.size() < max) {
    out.push_back(std::move(q_.front()));
    q_.pop_front();
  }
  return out;
}

size_t ShareQueue::size() {
  std::lock_guard<std::mutex> g(mu_);
  return q_.size();
}

// --------------------------------------------------------------- miner base

// Two templates describe the same search space when everything that feeds a
// header is equal (target / epoch / job id may differ). Re-issuing the same work
// (SV2 SetTarget, V1 set_difficulty, curtail/arbitration pause -> resume) must
// NOT restart the nonce cursor, or the device re-finds shares it already
// submitted and the pool rejects them as duplicates.
static bool same_work(const JobTemplate& a, const JobTemplate& b) {
  return a.algo == b.algo && std::memcmp(a.header, b.header, 76) == 0 && a.version_mask == b.version_mask &&
         a.ntime_roll == b.ntime_roll && a.has_coinbase == b.has_coinbase && a.coinb1 == b.coinb1 &&
         a.coinb2 == b.coinb2 && a.extranonce1 == b.extranonce1 && a.extranonce2_size == b.extranonce2_size &&
         a.merkle_branches == b.merkle_branches && a.variant_start == b.variant_start &&
         a.variant_stride == b.variant_stride;
}

void MinerBase::set_job(std::shared_ptr<const JobTemplate> job) {
  {
    std::lock_guard<std::mutex> g(job_mu_);
    if (job && (!job_ || !(last_work_ && same_work(*last_work_, *job)))) job_set_at_ = monotonic_seconds();
    if (job && !(last_work_ && same_work(*last_work_, *job))) ++job_gen_;
    if (job) last_work_ = job;
    job_ = std::move(job);
  }
  job_cv_.notify_all();
}

std::shared_ptr<const JobTemplate> MinerBase::current_job(uint64_t* gen) {
  std::unique_lock<std::mutex> g(job_mu_);
  if (!job_ && running_.load()) {
    job_cv_.wait_for(g, std::chrono::milliseconds(10));
  }
  if (gen) *gen = job_gen_;
  return job_;
}

std::shared_ptr<const JobTemplate> MinerBase::peek_job(uint64_t* gen, double* set_at) {
  std::lock_guard<std::mutex> g(job_mu_);
  if (gen) *gen = job_gen_;
  if (set_at) *set_at = job_set_at_;
  return job_;
}

MinerStats MinerBase::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  MinerStats s = stats_;
  s.dropped = queue_.dropped();
  return s;
}

// ---------------------------------------------------------- CPU SHA-256d scan

constexpr int kScanWide = 16;  // "lanes" value selecting the 16-lane AVX-512 scan

// The AVX-512 scan where the CPU has it: single thread 51-55 MH/s on the MI355X host's EPYC 9575F against 36.5 for
// SHA-NI, 28 against 11-13 on the build container's Xeon (tools/cpu_scan_ab.py, profiles/r4/r_cpu_avx512).
// Without AVX-512, nonces in flight per step of the fused SHA-NI scan, single thread (tools/cpu_lanes_ab.py,
// profiles/r4/m_cpu_lanes): AMD EPYC 9575F 21.2 / 31.3 / 35.0 / 36.4 MH/s for 1-4 lanes; the build container's Intel
// Xeon 9.8 / 11.6 / 10.3 / 10.1. So 4 on AMD cores, 2 elsewhere.
static int cpu_scan_lanes_for_this_cpu() {
  if (cpu_has_avx512_sha_scan()) return kScanWide;
  unsigned a = 0, b = 0, c = 0, d = 0;
  if (!__get_cpuid(0, &a, &b, &c, &d)) return 2;
  char vendor[13];
  std::memcpy(vendor, &b, 4);
  std::memcpy(vendor + 4, &d, 4);
  std::memcpy(vendor + 8, &c, 4);
  vendor[12] = 0;
  return std::strcmp(vendor, "AuthenticAMD") == 0 ? 4 : 2;
}

// Per-nonce work with a midstate: block 2 (16 B of header + padding) and the
// 32-byte digest block. 2 compressions per nonce instead of the reference's 3.
static inline void sha256d_from_mid(const uint32_t mid[8], uint8_t blk2[64], uint8_t dblk[64],
                                    uint8_t out[32]) {
  uint32_t st[8];
  std::memcpy(st, mid, 32);
  sha256_compress(st, blk2);
  for (int i = 0; i < 8; ++i) store_be32(dblk + 4 * i, st[i]);
  std::memcpy(st, kSha256IV, 32);
  sha256_compress(st, dblk);
  for (int i = 0; i < 8; ++i) store_be32(out + 4 * i, st[i]);
}

// L nonces per step through the interleaved compressor (SHA-NI is latency-bound in one chain: independent chains
// fill its pipeline). H7 first: the early reject.
template <int L>
static void cpu_scan_lanes(const uint32_t mid[8], const uint8_t blk2_tmpl[64], const uint8_t target[32], uint32_t start,
                           uint64_t count, std::vector<uint32_t>* hits, uint64_t* done) {
  uint8_t blk[L][64], dblk[L][64];
  uint32_t st[L][8];
  uint32_t* sp[L];
  const uint8_t* bp[L];
  const uint8_t* dp[L];
  for (int l = 0; l < L; ++l) {
    std::memcpy(blk[l], blk2_tmpl, 64);
    std::memset(dblk[l], 0, 64);
    dblk[l][32] = 0x80;
    dblk[l][62] = 0x01;  // 256 bits
    sp[l] = st[l];
    bp[l] = blk[l];
    dp[l] = dblk[l];
  }
  const uint32_t thi = load_le32(target + 28);
  uint8_t h[32];
  uint64_t i = 0;
  for (; i + L <= count; i += L) {
    for (int l = 0; l < L; ++l) {
      store_le32(blk[l] + 12, start + uint32_t(i) + uint32_t(l));
      std::memcpy(st[l], mid, 32);
    }
    sha256_compress_xn(L, sp, bp);
    for (int l = 0; l < L; ++l) {
      for (int w = 0; w < 8; ++w) store_be32(dblk[l] + 4 * w, st[l][w]);
      std::memcpy(st[l], kSha256IV, 32);
    }
    sha256_compress_xn(L, sp, dp);
    for (int l = 0; l < L; ++l) {
      if (__builtin_bswap32(st[l][7]) > thi) continue;
      for (int w = 0; w < 8; ++w) store_be32(h + 4 * w, st[l][w]);
      if (le256_leq(h, target)) hits->push_back(start + uint32_t(i) + uint32_t(l));
    }
  }
  *done = i;
}

// Lanes per step of the CPU scan (OTEDAMA_CPU_LANES overrides: 1..4 SHA-NI chains, 16 the AVX-512 scan).
static int cpu_scan_lanes_default() {
  static const int lanes = [] {
    const char* v = std::getenv("OTEDAMA_CPU_LANES");
    const int n = v ? std::atoi(v) : 0;
    return (n >= 1 && n <= 4) || n == kScanWide ? n : cpu_scan_lanes_for_this_cpu();
  }();
  return lanes;
}

std::vector<uint32_t> cpu_scan_sha256d_lanes(int lanes, const uint8_t header80[80], const uint8_t target[32],
                                             uint32_t start, uint64_t count) {
  uint32_t mid[8];
  std::memcpy(mid, kSha256IV, 32);
  sha256_compress(mid, header80);
  uint8_t blk2[64] = {0};
  std::memcpy(blk2, header80 + 64, 16);
  blk2[16] = 0x80;
  blk2[62] = 0x02;  // 640 bits
  blk2[63] = 0x80;
  std::vector<uint32_t> hits;
  uint64_t i = 0;
  uint8_t dblk[64] = {0};
  dblk[32] = 0x80;
  dblk[62] = 0x01;
  uint8_t h[32];
  const uint32_t thi = load_le32(target + 28);
  std::vector<uint32_t> cands;
  if ((lanes == kScanWide && sha256d_scan_h7_wide(mid, header80 + 64, start, count, thi, &cands, &i)) ||
      sha256d_scan_h7(lanes == kScanWide ? 4 : lanes, mid, header80 + 64, start, count, thi, &cands, &i)) {
    // SHA-NI: the fused H7 scan; its candidates get the full hash and 256-bit compare here
    for (uint32_t n : cands) {
      store_le32(blk2 + 12, n);
      sha256d_from_mid(mid, blk2, dblk, h);
      if (le256_leq(h, target)) hits.push_back(n);
    }
  } else {
    switch (lanes) {
      case 1: cpu_scan_lanes<1>(mid, blk2, target, start, count, &hits, &i); break;
      case 3: cpu_scan_lanes<3>(mid, blk2, target, start, count, &hits, &i); break;
      case 4: cpu_scan_lanes<4>(mid, blk2, target, start, count, &hits, &i); break;
      default: cpu_scan_lanes<2>(mid, blk2, target, start, count, &hits, &i); break;
    }
  }
  for (; i < count; ++i) {  // the tail, one nonce at a time
    const uint32_t nonce = start + uint32_t(i);
    store_le32(blk2 + 12, nonce);
    sha256d_from_mid(mid, blk2, dblk, h);
    if (load_le32(h + 28) <= thi && le256_leq(h, target)) hits.push_back(nonce);
  }
  return hits;
}

std::string cpu_scan_method() {
  const int lanes = cpu_scan_lanes_default();
  if (lanes == kScanWide && cpu_has_avx512_sha_scan())
    return "avx512 16 lanes x " + std::to_string(sha256d_scan_wide_groups()) + " groups";
  if (cpu_has_sha_ni()) return "sha-ni x" + std::to_string(lanes == kScanWide ? 4 : lanes);
  return "portable x" + std::to_string(lanes == kScanWide ? 2 : lanes);
}

std::vector<uint32_t> cpu_scan_sha256d(const uint8_t header80[80], const uint8_t target[32], uint32_t start,
                                       uint64_t count) {
  return cpu_scan_sha256d_lanes(cpu_scan_lanes_default(), header80, target, start, count);
}

// ------------------------------------------------------------------ CPU miner

CpuMiner::CpuMiner(int threads, std::string device_id, size_t queue_cap)
    : MinerBase(std::move(device_id), queue_cap), threads_(threads > 0 ? threads : 1) {}

CpuMiner::~CpuMiner() { stop(); }

void CpuMiner::start() {
  if (running_.exchange(true)) return;
  for (int t = 0; t < threads_; ++t) ths_.emplace_back([this, t] { loop(t); });
}

void CpuMiner::stop() {
  if (!running_.exchange(false)) return;
  job_cv_.notify_all();
  for (auto& t : ths_) if (t.joinable()) t.join();
  ths_.clear();
}

void CpuMiner::loop(int /*tid*/) {
  while (running_.load()) {
    uint64_t gen = 0;
    auto job = current_job(&gen);
    if (!job) continue;
    // SHA-256d: 64Ki-nonce chunks through the SHA-NI scanner. scrypt / X11 (CPU hosts, rehearsals): 256-nonce chunks
    // hashed one by one with the host reference functions (verify_share), ~1000x slower per nonce. A work
    // generation has one algorithm, so one chunk size per cursor generation.
    const bool sha = job->algo == Algo::kSha256d;
    const uint64_t kChunk = sha ? (1ull << 16) : 256;
    uint64_t claim;
    double fresh_at = 0;  // this thread opened a new work generation: when its first chunk was claimed
#ifdef OTEDAMA_STRESS_HOOKS
    // tools/sanitize: widen the snapshot -> claim window so job switches land inside it.
    std::this_thread::sleep_for(std::chrono::microseconds(std::hash<std::thread::id>{}(
        std::this_thread::get_id()) % 400));
#endif
    {
      std::lock_guard<std::mutex> g(cursor_mu_);
      // Generations only move forward. A thread still holding a superseded snapshot must drop
      // it, not rewind the shared cursor to its own generation: that would rescan chunks of the
      // old work already searched and emit duplicate shares.
      const uint64_t cg = cursor_gen_.load();
      if (gen < cg) continue;
      if (gen > cg) { cursor_gen_.store(gen); cursor_.store(0); fresh_at = monotonic_seconds(); }
      claim = cursor_.fetch_add(kChunk);
    }
    // claim indexes (variant-stripe slot k, nonce chunk)
    const uint64_t chunks_per_variant = (1ull << 32) / kChunk;
    const uint64_t k = claim / kChunk / chunks_per_variant;
    const uint32_t nonce0 = uint32_t((claim / kChunk % chunks_per_variant) * kChunk);
    const uint64_t v = job->variant_start + k * job->variant_stride;
    if (v >= job->variant_space()) {  // stripe exhausted: wait for new work
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      continue;
    }
    uint8_t hdr[80];
    uint32_t ver, nt;
    uint64_t en2;
    job->variant_header(v, hdr, &ver, &nt, &en2);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint32_t> hits;
    if (sha) {
      hits = cpu_scan_sha256d(hdr, job->target, nonce0, kChunk);
    } else if (job->algo == Algo::kScrypt) {
      // sixteen nonces per scrypt batch (AVX-512 lanes; two AVX2 passes without it)
      uint8_t hb[16][80], ho[16][32];
      const uint8_t* ip[16];
      uint8_t* op[16];
      for (int l = 0; l < 16; ++l) {
        std::memcpy(hb[l], hdr, 80);
        ip[l] = hb[l];
        op[l] = ho[l];
      }
      for (uint64_t i = 0; i < kChunk && running_.load(); i += 16) {
        const int n = int(std::min<uint64_t>(16, kChunk - i));
        for (int l = 0; l < n; ++l) store_le32(hb[l] + 76, nonce0 + uint32_t(i) + uint32_t(l));
        scrypt_1024_1_1_batch(n, ip, op);
        for (int l = 0; l < n; ++l)
          if (le256_leq(ho[l], job->target)) hits.push_back(nonce0 + uint32_t(i) + uint32_t(l));
      }
    } else {
      uint8_t h[32];
      for (uint64_t i = 0; i < kChunk && running_.load(); ++i) {
        store_le32(hdr + 76, nonce0 + uint32_t(i));
        if (verify_share(job->algo, hdr, job->target, h)) hits.push_back(nonce0 + uint32_t(i));
      }
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t n : hits) {
      ShareRecord s{};
      s.epoch = job->epoch; s.job_id = job->job_id; s.channel_id = job->channel_id;
      s.nonce = n; s.ntime = nt; s.version = ver; s.extranonce2 = en2;
      s.extranonce2_size = job->extranonce2_size; s.device_id = device_id_;
      s.found_at = monotonic_seconds();
      store_le32(hdr + 76, n);
      if (sha) sha256d(hdr, 80, s.hash);
      else verify_share(job->algo, hdr, job->target, s.hash);
      queue_.push(std::move(s));
    }
    std::lock_guard<std::mutex> g(stats_mu_);
    if (fresh_at > 0) {
      stats_.work_started.emplace_back(job->epoch, fresh_at);
      if (stats_.work_started.size() > 64) stats_.work_started.erase(stats_.work_started.begin());
    }
    if (stats_.variant_epoch != job->epoch) { stats_.variant_epoch = job->epoch; stats_.variant_next = 0; }
    if (v + job->variant_stride > stats_.variant_next) stats_.variant_next = v + job->variant_stride;
    stats_.hashes += kChunk;
    stats_.candidates += hits.size();
    stats_.shares += hits.size();
    stats_.busy_seconds += dt;
  }
}

}  // namespace otedama

namespace otedama {
bool maps_range_writable(const std::string& maps, uintptr_t lo, uintptr_t hi) {
  size_t pos = 0;
  while (pos < maps.size()) {
    size_t eol = maps.find('\n', pos);
    if (eol == std::string::npos) eol = maps.size();
    const std::string line = maps.substr(pos, eol - pos);
    pos = eol + 1;
    unsigned long a = 0, b = 0;
    char perms[8] = {0};
    if (std::sscanf(line.c_str(), "%lx-%lx %7s", &a, &b, perms) != 3) continue;
    if (a <= lo && hi <= b) return perms[0] == 'r' && perms[1] == 'w';
  }
  return false;
}

double monotonic_seconds() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return double(ts.tv_sec) + double(ts.tv_nsec) * 1e-9;
}
}  // namespace otedama
