// X11 (K6) CPU reference: the eleven chained 512-bit hashes
//   BLAKE-512 -> BMW-512 -> Groestl-512 -> Skein-512 -> JH-512 -> Keccak-512
//   -> Luffa-512 -> CubeHash-512 -> SHAvite-3-512 -> SIMD-512 -> ECHO-512,
// X11(header) = first 32 bytes of the ECHO-512 digest.
//
// [NO REFERENCE CODE] in shizukutanaka/Otedama: the
// reference v3 has no X11 at all. This file is written from the SHA-3 round-2/3
// algorithm definitions as plain, readable, portable C++. It is the oracle the
// gfx950 kernels are checked against and the pool's share validator for "x11".
// Speed is not a goal here.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "otedama/x11.h"

namespace otedama {
namespace x11 {

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

static inline u64 rotl64(u64 x, int n) { n &= 63; return n ? (x << n) | (x >> (64 - n)) : x; }
static inline u64 rotr64(u64 x, int n) { n &= 63; return n ? (x >> n) | (x << (64 - n)) : x; }
static inline u32 rotl32(u32 x, int n) { n &= 31; return n ? (x << n) | (x >> (32 - n)) : x; }
static inline u64 ld64be(const u8* p) { u64 v = 0; for (int i = 0; i < 8; ++i) v = (v << 8) | p[i]; return v; }
static inline u64 ld64le(const u8* p) { u64 v = 0; for (int i = 7; i >= 0; --i) v = (v << 8) | p[i]; return v; }
static inline u32 ld32le(const u8* p) { return (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24); }
static inline u32 ld32be(const u8* p) { return ((u32)p[0] << 24) | ((u32)p[1] << 16) | ((u32)p[2] << 8) | (u32)p[3]; }
static inline void st64be(u8* p, u64 v) { for (int i = 7; i >= 0; --i) { p[i] = (u8)v; v >>= 8; } }
static inline void st64le(u8* p, u64 v) { for (int i = 0; i < 8; ++i) { p[i] = (u8)v; v >>= 8; } }
static inline void st32le(u8* p, u32 v) { for (int i = 0; i < 4; ++i) { p[i] = (u8)v; v >>= 8; } }
static inline void st32be(u8* p, u32 v) { for (int i = 3; i >= 0; --i) { p[i] = (u8)v; v >>= 8; } }

// ---------------------------------------------------------------------------
// AES pieces shared by Groestl, SHAvite-3 and ECHO (S-box built from GF(2^8)).
// ---------------------------------------------------------------------------
static u8 SBOX[256];
static bool sbox_ready = false;
static inline u8 rotl8(u8 x, int n) { return (u8)((x << n) | (x >> (8 - n))); }
static void init_gmul();
static void init_sbox_impl() {
    if (sbox_ready) return;
    u8 p = 1, q = 1;
    do {
        p = (u8)(p ^ (p << 1) ^ ((p & 0x80) ? 0x1B : 0));      // p *= 3
        q ^= (u8)(q << 1); q ^= (u8)(q << 2); q ^= (u8)(q << 4);  // q /= 3
        if (q & 0x80) q ^= 0x09;
        SBOX[p] = (u8)(q ^ rotl8(q, 1) ^ rotl8(q, 2) ^ rotl8(q, 3) ^ rotl8(q, 4) ^ 0x63);
    } while (p != 1);
    SBOX[0] = 0x63;
    init_gmul();
    sbox_ready = true;
}
// Thread-safe one-time init (miner threads verify shares concurrently).
static void init_sbox() { static const bool once = (init_sbox_impl(), true); (void)once; }
const u8* aes_sbox() { init_sbox(); return SBOX; }
static inline u8 xt(u8 x) { return (u8)((x << 1) ^ ((x & 0x80) ? 0x1B : 0)); }
static inline u8 gmul(u8 a, u8 b) {
    u8 r = 0;
    while (b) { if (b & 1) r ^= a; a = xt(a); b >>= 1; }
    return r;
}
static u8 GMUL[8][256];  // GMUL[c][x] = c * x in GF(2^8), c < 8 (filled with the S-box)
static void init_gmul() {
    for (int c = 0; c < 8; ++c)
        for (int x = 0; x < 256; ++x) GMUL[c][x] = gmul((u8)x, (u8)c);
}
// One AES round on a 16-byte column-major state, round key k (null = 0).
static void aes_round(u8 s[16], const u8* k) {
    u8 t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) t[4 * c + r] = SBOX[s[4 * ((c + r) & 3) + r]];
    for (int c = 0; c < 4; ++c) {
        u8 a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c + 0] = (u8)(xt(a0) ^ xt(a1) ^ a1 ^ a2 ^ a3);
        s[4 * c + 1] = (u8)(a0 ^ xt(a1) ^ xt(a2) ^ a2 ^ a3);
        s[4 * c + 2] = (u8)(a0 ^ a1 ^ xt(a2) ^ xt(a3) ^ a3);
        s[4 * c + 3] = (u8)(xt(a0) ^ a0 ^ a1 ^ a2 ^ xt(a3));
    }
    if (k) for (int i = 0; i < 16; ++i) s[i] ^= k[i];
}
// Keyless AES round on four little-endian 32-bit column words.
static void aes_round_words(u32 w[4]) {
    u8 s[16];
    for (int i = 0; i < 4; ++i) st32le(s + 4 * i, w[i]);
    aes_round(s, nullptr);
    for (int i = 0; i < 4; ++i) w[i] = ld32le(s + 4 * i);
}

// ---------------------------------------------------------------------------
// 1. BLAKE-512: 16 rounds, big-endian words.
// ---------------------------------------------------------------------------
static const u64 BLAKE_C[16] = {
    0x243F6A8885A308D3ULL, 0x13198A2E03707344ULL, 0xA4093822299F31D0ULL, 0x082EFA98EC4E6C89ULL,
    0x452821E638D01377ULL, 0xBE5466CF34E90C6CULL, 0xC0AC29B7C97C50DDULL, 0x3F84D5B5B5470917ULL,
    0x9216D5D98979FB1BULL, 0xD1310BA698DFB5ACULL, 0x2FFD72DBD01ADFB7ULL, 0xB8E1AFED6A267E96ULL,
    0xBA7C9045F12C7F99ULL, 0x24A19947B3916CF7ULL, 0x0801F2E2858EFC16ULL, 0x636920D871574E69ULL};
static const u8 SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
static const u64 SHA512_IV[8] = {0x6A09E667F3BCC908ULL, 0xBB67AE8584CAA73BULL, 0x3C6EF372FE94F82BULL, 0xA54FF53A5F1D36F1ULL,
                                 0x510E527FADE682D1ULL, 0x9B05688C2B3E6C1FULL, 0x1F83D9ABFB41BD6BULL, 0x5BE0CD19137E2179ULL};

static void blake512_compress(u64 h[8], const u8 block[128], u64 t) {
    u64 m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = ld64be(block + 8 * i);
    for (int i = 0; i < 8; ++i) v[i] = h[i];
    for (int i = 0; i < 4; ++i) v[8 + i] = BLAKE_C[i];  // salt = 0
    v[12] = t ^ BLAKE_C[4];
    v[13] = t ^ BLAKE_C[5];
    v[14] = BLAKE_C[6];  // counter high word (messages < 2^64 bits)
    v[15] = BLAKE_C[7];
    static const int G[8][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15},
                                {0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};
    for (int r = 0; r < 16; ++r) {
        const u8* s = SIGMA[r % 10];
        for (int i = 0; i < 8; ++i) {
            u64 &a = v[G[i][0]], &b = v[G[i][1]], &c = v[G[i][2]], &d = v[G[i][3]];
            int x = s[2 * i], y = s[2 * i + 1];
            a = a + b + (m[x] ^ BLAKE_C[y]);
            d = rotr64(d ^ a, 32);
            c = c + d;
            b = rotr64(b ^ c, 25);
            a = a + b + (m[y] ^ BLAKE_C[x]);
            d = rotr64(d ^ a, 16);
            c = c + d;
            b = rotr64(b ^ c, 11);
        }
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

void blake512(const u8* msg, size_t len, u8 out[64]) {
    u64 h[8];
    memcpy(h, SHA512_IV, sizeof h);
    size_t off = 0;
    u64 bits = 0;
    while (len - off > 128) {
        bits += 1024;
        blake512_compress(h, msg + off, bits);
        off += 128;
    }
    size_t rem = len - off;
    u64 total = (u64)len * 8;
    u8 buf[256];
    memset(buf, 0, sizeof buf);
    if (rem) memcpy(buf, msg + off, rem);  // msg may be null when len == 0
    if (rem == 128) {  // full last block: padding goes in a block of its own
        blake512_compress(h, buf, total);
        memset(buf, 0, 128);
        buf[0] = 0x80;
        buf[111] |= 0x01;
        st64be(buf + 120, total);
        blake512_compress(h, buf, 0);
    } else if (rem <= 111) {
        buf[rem] = 0x80;
        buf[111] |= 0x01;
        st64be(buf + 120, total);
        blake512_compress(h, buf, rem ? total : 0);
    } else {
        buf[rem] = 0x80;
        blake512_compress(h, buf, total);
        memset(buf, 0, 128);
        buf[111] = 0x01;
        st64be(buf + 120, total);
        blake512_compress(h, buf, 0);
    }
    for (int i = 0; i < 8; ++i) st64be(out + 8 * i, h[i]);
}

// ---------------------------------------------------------------------------
// 2. BMW-512 (Blue Midnight Wish), little-endian words.
// ---------------------------------------------------------------------------
static inline u64 bmw_s0(u64 x) { return (x >> 1) ^ (x << 3) ^ rotl64(x, 4) ^ rotl64(x, 37); }
static inline u64 bmw_s1(u64 x) { return (x >> 1) ^ (x << 2) ^ rotl64(x, 13) ^ rotl64(x, 43); }
static inline u64 bmw_s2(u64 x) { return (x >> 2) ^ (x << 1) ^ rotl64(x, 19) ^ rotl64(x, 53); }
static inline u64 bmw_s3(u64 x) { return (x >> 2) ^ (x << 2) ^ rotl64(x, 28) ^ rotl64(x, 59); }
static inline u64 bmw_s4(u64 x) { return (x >> 1) ^ x; }
static inline u64 bmw_s5(u64 x) { return (x >> 2) ^ x; }
static inline u64 bmw_s(int i, u64 x) {
    switch (i) {
        case 0: return bmw_s0(x);
        case 1: return bmw_s1(x);
        case 2: return bmw_s2(x);
        case 3: return bmw_s3(x);
        default: return bmw_s4(x);
    }
}

// W_j = signed sums of five (M ^ H) words.
static const int BMW_WI[16][5] = {
    {5, 7, 10, 13, 14}, {6, 8, 11, 14, 15}, {0, 7, 9, 12, 15}, {0, 1, 8, 10, 13},
    {1, 2, 9, 11, 14}, {3, 2, 10, 12, 15}, {4, 0, 3, 11, 13}, {1, 4, 5, 12, 14},
    {2, 5, 6, 13, 15}, {0, 3, 6, 7, 14}, {8, 1, 4, 7, 15}, {8, 0, 2, 5, 9},
    {1, 3, 6, 9, 10}, {2, 4, 7, 10, 11}, {3, 5, 8, 11, 12}, {12, 4, 6, 9, 13}};
static const int BMW_WS[16][5] = {
    {1, -1, 1, 1, 1}, {1, -1, 1, 1, -1}, {1, 1, 1, -1, 1}, {1, -1, 1, -1, 1},
    {1, 1, 1, -1, -1}, {1, -1, 1, -1, 1}, {1, -1, -1, -1, 1}, {1, -1, -1, -1, -1},
    {1, -1, -1, 1, -1}, {1, -1, 1, -1, 1}, {1, -1, -1, -1, 1}, {1, -1, -1, -1, 1},
    {1, 1, -1, -1, 1}, {1, 1, 1, 1, 1}, {1, -1, 1, -1, -1}, {1, -1, -1, -1, 1}};

static void bmw512_compress(u64 H[16], const u64 M[16]) {
    u64 X[16], W[16], Q[32];
    for (int i = 0; i < 16; ++i) X[i] = M[i] ^ H[i];
    for (int j = 0; j < 16; ++j) {
        u64 w = 0;
        for (int k = 0; k < 5; ++k) w = BMW_WS[j][k] > 0 ? w + X[BMW_WI[j][k]] : w - X[BMW_WI[j][k]];
        W[j] = w;
    }
    for (int j = 0; j < 16; ++j) Q[j] = bmw_s(j % 5, W[j]) + H[(j + 1) & 15];
    // f1: 2 rounds of expand1, 14 of expand2
    for (int j = 16; j < 32; ++j) {
        int jj = j - 16;
        u64 add = rotl64(M[jj & 15], (jj & 15) + 1) + rotl64(M[(jj + 3) & 15], ((jj + 3) & 15) + 1) -
                  rotl64(M[(jj + 10) & 15], ((jj + 10) & 15) + 1) + (u64)j * 0x0555555555555555ULL;
        add ^= H[(jj + 7) & 15];
        u64 q;
        if (j < 18) {
            q = 0;
            for (int k = 0; k < 16; ++k) {
                u64 x = Q[j - 16 + k];
                switch (k & 3) {
                    case 0: q += bmw_s1(x); break;
                    case 1: q += bmw_s2(x); break;
                    case 2: q += bmw_s3(x); break;
                    default: q += bmw_s0(x); break;
                }
            }
        } else {
            q = Q[j - 16] + rotl64(Q[j - 15], 5) + Q[j - 14] + rotl64(Q[j - 13], 11) + Q[j - 12] + rotl64(Q[j - 11], 27) +
                Q[j - 10] + rotl64(Q[j - 9], 32) + Q[j - 8] + rotl64(Q[j - 7], 37) + Q[j - 6] + rotl64(Q[j - 5], 43) +
                Q[j - 4] + rotl64(Q[j - 3], 53) + bmw_s4(Q[j - 2]) + bmw_s5(Q[j - 1]);
        }
        Q[j] = q + add;
    }
    u64 XL = 0, XH = 0;
    for (int i = 16; i < 24; ++i) XL ^= Q[i];
    XH = XL;
    for (int i = 24; i < 32; ++i) XH ^= Q[i];
    u64 N[16];
    N[0] = ((XH << 5) ^ (Q[16] >> 5) ^ M[0]) + (XL ^ Q[24] ^ Q[0]);
    N[1] = ((XH >> 7) ^ (Q[17] << 8) ^ M[1]) + (XL ^ Q[25] ^ Q[1]);
    N[2] = ((XH >> 5) ^ (Q[18] << 5) ^ M[2]) + (XL ^ Q[26] ^ Q[2]);
    N[3] = ((XH >> 1) ^ (Q[19] << 5) ^ M[3]) + (XL ^ Q[27] ^ Q[3]);
    N[4] = ((XH >> 3) ^ Q[20] ^ M[4]) + (XL ^ Q[28] ^ Q[4]);
    N[5] = ((XH << 6) ^ (Q[21] >> 6) ^ M[5]) + (XL ^ Q[29] ^ Q[5]);
    N[6] = ((XH >> 4) ^ (Q[22] << 6) ^ M[6]) + (XL ^ Q[30] ^ Q[6]);
    N[7] = ((XH >> 11) ^ (Q[23] << 2) ^ M[7]) + (XL ^ Q[31] ^ Q[7]);
    N[8] = rotl64(N[4], 9) + (XH ^ Q[24] ^ M[8]) + ((XL << 8) ^ Q[23] ^ Q[8]);
    N[9] = rotl64(N[5], 10) + (XH ^ Q[25] ^ M[9]) + ((XL >> 6) ^ Q[16] ^ Q[9]);
    N[10] = rotl64(N[6], 11) + (XH ^ Q[26] ^ M[10]) + ((XL << 6) ^ Q[17] ^ Q[10]);
    N[11] = rotl64(N[7], 12) + (XH ^ Q[27] ^ M[11]) + ((XL << 4) ^ Q[18] ^ Q[11]);
    N[12] = rotl64(N[0], 13) + (XH ^ Q[28] ^ M[12]) + ((XL >> 3) ^ Q[19] ^ Q[12]);
    N[13] = rotl64(N[1], 14) + (XH ^ Q[29] ^ M[13]) + ((XL >> 4) ^ Q[20] ^ Q[13]);
    N[14] = rotl64(N[2], 15) + (XH ^ Q[30] ^ M[14]) + ((XL >> 7) ^ Q[21] ^ Q[14]);
    N[15] = rotl64(N[3], 16) + (XH ^ Q[31] ^ M[15]) + ((XL >> 2) ^ Q[22] ^ Q[15]);
    memcpy(H, N, sizeof N);
}

void bmw512(const u8* msg, size_t len, u8 out[64]) {
    u64 H[16], M[16];
    for (int i = 0; i < 16; ++i) {
        u64 v = 0;
        for (int b = 0; b < 8; ++b) v = (v << 8) | (u64)(0x80 + 8 * i + b);
        H[i] = v;
    }
    size_t off = 0;
    while (len - off >= 128) {
        for (int i = 0; i < 16; ++i) M[i] = ld64le(msg + off + 8 * i);
        bmw512_compress(H, M);
        off += 128;
    }
    u8 buf[256];
    memset(buf, 0, sizeof buf);
    size_t rem = len - off;
    if (rem) memcpy(buf, msg + off, rem);  // msg may be null when len == 0
    buf[rem] = 0x80;
    if (rem + 1 > 120) {
        for (int i = 0; i < 16; ++i) M[i] = ld64le(buf + 8 * i);
        bmw512_compress(H, M);
        memset(buf, 0, 128);
    }
    st64le(buf + 120, (u64)len * 8);
    for (int i = 0; i < 16; ++i) M[i] = ld64le(buf + 8 * i);
    bmw512_compress(H, M);
    u64 F[16];
    for (int i = 0; i < 16; ++i) F[i] = 0xAAAAAAAAAAAAAAA0ULL + (u64)i;
    bmw512_compress(F, H);
    for (int i = 0; i < 8; ++i) st64le(out + 8 * i, F[8 + i]);
}

// ---------------------------------------------------------------------------
// 3. Groestl-512: 8x16 byte state, P1024/Q1024, 14 rounds.
// ---------------------------------------------------------------------------
static void groestl_perm(u8 a[128], bool q) {
    // a[col*8 + row]
    static const int SP[8] = {0, 1, 2, 3, 4, 5, 6, 11};
    static const int SQ[8] = {1, 3, 5, 11, 0, 2, 4, 6};
    static const u8 MB[8] = {2, 2, 3, 4, 5, 3, 5, 7};
    u8 t[128];
    for (int r = 0; r < 14; ++r) {
        if (!q) {
            for (int j = 0; j < 16; ++j) a[j * 8 + 0] ^= (u8)((j << 4) ^ r);
        } else {
            for (int j = 0; j < 16; ++j) {
                for (int i = 0; i < 7; ++i) a[j * 8 + i] ^= 0xFF;
                a[j * 8 + 7] ^= (u8)(0xFF ^ (j << 4) ^ r);
            }
        }
        for (int k = 0; k < 128; ++k) a[k] = SBOX[a[k]];
        const int* sh = q ? SQ : SP;
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 16; ++j) t[j * 8 + i] = a[((j + sh[i]) & 15) * 8 + i];
        for (int j = 0; j < 16; ++j)
            for (int i = 0; i < 8; ++i) {
                u8 s = 0;
                for (int k = 0; k < 8; ++k) s ^= GMUL[MB[(k - i + 8) & 7]][t[j * 8 + k]];
                a[j * 8 + i] = s;
            }
    }
}

static void groestl512_compress(u8 h[128], const u8 m[128]) {
    u8 p[128], q[128];
    for (int i = 0; i < 128; ++i) { p[i] = h[i] ^ m[i]; q[i] = m[i]; }
    groestl_perm(p, false);
    groestl_perm(q, true);
    for (int i = 0; i < 128; ++i) h[i] ^= p[i] ^ q[i];
}

void groestl512(const u8* msg, size_t len, u8 out[64]) {
    init_sbox();
    u8 h[128];
    memset(h, 0, sizeof h);
    h[126] = 0x02;  // output length 512, 64-bit big-endian in the last bytes
    size_t off = 0;
    u64 blocks = 0;
    while (len - off >= 128) { groestl512_compress(h, msg + off); off += 128; ++blocks; }
    size_t rem = len - off;
    u8 buf[256];
    memset(buf, 0, sizeof buf);
    if (rem) memcpy(buf, msg + off, rem);  // msg may be null when len == 0
    buf[rem] = 0x80;
    size_t nb = (rem + 1 + 8 <= 128) ? 1 : 2;
    blocks += nb;
    st64be(buf + 128 * nb - 8, blocks);
    for (size_t b = 0; b < nb; ++b) groestl512_compress(h, buf + 128 * b);
    u8 p[128];
    memcpy(p, h, 128);
    groestl_perm(p, false);
    for (int i = 0; i < 64; ++i) out[i] = p[64 + i] ^ h[64 + i];
}

// ---------------------------------------------------------------------------
// 4. Skein-512-512 (Threefish-512, UBI chaining), v1.3 constants.
// ---------------------------------------------------------------------------
static const int SKEIN_R[8][4] = {{46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
                                  {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22}};
static void threefish512(const u64 key[8], const u64 tw[2], const u64 in[8], u64 out[8]) {
    u64 k[9], t[3], v[8];
    k[8] = 0x1BD11BDAA9FC1A22ULL;
    for (int i = 0; i < 8; ++i) { k[i] = key[i]; k[8] ^= key[i]; }
    t[0] = tw[0]; t[1] = tw[1]; t[2] = tw[0] ^ tw[1];
    for (int i = 0; i < 8; ++i) v[i] = in[i];
    for (int d = 0; d < 72; ++d) {
        if ((d & 3) == 0) {
            int s = d / 4;
            for (int i = 0; i < 8; ++i) v[i] += k[(s + i) % 9];
            v[5] += t[s % 3];
            v[6] += t[(s + 1) % 3];
            v[7] += (u64)s;
        }
        for (int j = 0; j < 4; ++j) {
            v[2 * j] += v[2 * j + 1];
            v[2 * j + 1] = rotl64(v[2 * j + 1], SKEIN_R[d & 7][j]) ^ v[2 * j];
        }
        u64 p[8] = {v[2], v[1], v[4], v[7], v[6], v[5], v[0], v[3]};
        memcpy(v, p, sizeof p);
    }
    for (int i = 0; i < 8; ++i) v[i] += k[(18 + i) % 9];
    v[5] += t[18 % 3];
    v[6] += t[19 % 3];
    v[7] += 18;
    for (int i = 0; i < 8; ++i) out[i] = v[i];
}

// UBI over an arbitrary byte string, type code `type`.
static void skein_ubi(u64 h[8], const u8* msg, size_t len, u64 type) {
    size_t off = 0;
    bool first = true;
    do {
        size_t n = len - off > 64 ? 64 : len - off;
        bool final = off + n == len;
        u8 blk[64];
        memset(blk, 0, 64);
        if (n) memcpy(blk, msg + off, n);
        u64 m[8], o[8];
        for (int i = 0; i < 8; ++i) m[i] = ld64le(blk + 8 * i);
        u64 tw[2] = {(u64)(off + n), (type << 56) | (first ? (1ULL << 62) : 0) | (final ? (1ULL << 63) : 0)};
        threefish512(h, tw, m, o);
        for (int i = 0; i < 8; ++i) h[i] = o[i] ^ m[i];
        off += n;
        first = false;
    } while (off < len);
}

void skein512_iv(u64 iv[8]) {
    u8 cfg[32];
    memset(cfg, 0, sizeof cfg);
    st32le(cfg, 0x33414853);  // "SHA3"
    cfg[4] = 1;               // version 1
    st64le(cfg + 8, 512);     // output bits
    for (int i = 0; i < 8; ++i) iv[i] = 0;
    skein_ubi(iv, cfg, 32, 4);
}

void skein512(const u8* msg, size_t len, u8 out[64]) {
    u64 h[8];
    skein512_iv(h);
    skein_ubi(h, msg, len, 48);
    u8 ctr[8] = {0};
    skein_ubi(h, ctr, 8, 63);
    for (int i = 0; i < 8; ++i) st64le(out + 8 * i, h[i]);
}

// ---------------------------------------------------------------------------
// 5. JH-512: E8 in the specification's grouped form (4-bit elements).
// ---------------------------------------------------------------------------
static const u8 JH_S[2][16] = {{9, 0, 4, 11, 13, 12, 3, 15, 1, 10, 2, 6, 7, 5, 8, 14},
                               {3, 12, 6, 13, 5, 7, 1, 9, 15, 2, 0, 4, 11, 10, 14, 8}};
static inline u8 jh_m2(u8 x) { return (u8)(((x << 1) & 0xF) ^ ((x & 8) ? 0x3 : 0)); }
static inline void jh_L(u8& a, u8& b) {
    // D = 2A ^ B, C = 2D ^ A over GF(2^4)/(x^4+x+1), MSB-first elements
    u8 d = (u8)(jh_m2(a) ^ b);
    u8 c = (u8)(jh_m2(d) ^ a);
    a = c;
    b = d;
}
// Destination index of element k under the permutation P_d (pi, then P', then phi).
int jh_perm_dest(int k, int dim) {
    int n = 1 << dim;
    if (k & 2) k ^= 1;                       // pi
    k = (k >> 1) + (k & 1) * (n / 2);        // P'
    if (k >= n / 2) k ^= 1;                  // phi
    return k;
}
// Round R_d on 2^d elements with constant bits cb[2^d].
static u8 JH_P8[256];  // jh_perm_dest(i, 8), tabulated with the round constants
static void jh_round(u8* e, int dim, const u8* cb) {
    int n = 1 << dim;
    for (int i = 0; i < n; ++i) e[i] = JH_S[cb[i]][e[i]];
    for (int i = 0; i < n; i += 2) jh_L(e[i], e[i + 1]);
    u8 t[256];
    if (dim == 8)
        for (int i = 0; i < n; ++i) t[JH_P8[i]] = e[i];
    else
        for (int i = 0; i < n; ++i) t[jh_perm_dest(i, dim)] = e[i];
    memcpy(e, t, n);
}
static u8 JH_C[42][256];  // round-constant bits, one per element
static bool jh_ready = false;
static void jh_init_constants_impl() {
    if (jh_ready) return;
    for (int i = 0; i < 256; ++i) JH_P8[i] = (u8)jh_perm_dest(i, 8);
    // C0 = first 256 bits of the fractional part of sqrt(2)
    static const u8 C0[32] = {0x6a, 0x09, 0xe6, 0x67, 0xf3, 0xbc, 0xc9, 0x08, 0xb2, 0xfb, 0x13, 0x66, 0xea, 0x95, 0x7d, 0x3e,
                              0x3a, 0xde, 0xc1, 0x75, 0x12, 0x77, 0x50, 0x99, 0xda, 0x2f, 0x59, 0x0b, 0x06, 0x67, 0x32, 0x2a};
    u8 c[64];
    for (int i = 0; i < 32; ++i) { c[2 * i] = C0[i] >> 4; c[2 * i + 1] = C0[i] & 0xF; }
    u8 zero[64] = {0};
    for (int r = 0; r < 42; ++r) {
        for (int i = 0; i < 64; ++i)
            for (int b = 0; b < 4; ++b) JH_C[r][4 * i + b] = (c[i] >> (3 - b)) & 1;
        jh_round(c, 6, zero);
    }
    jh_ready = true;
}
static void jh_init_constants() { static const bool once = (jh_init_constants_impl(), true); (void)once; }
const u8* jh_round_constant_bits(int r) { jh_init_constants(); return JH_C[r]; }
static void jh_E8(u8 H[128]) {
    auto bit = [&](int i) -> u8 { return (H[i >> 3] >> (7 - (i & 7))) & 1; };
    u8 e[256];
    for (int i = 0; i < 128; ++i) {
        e[2 * i] = (u8)((bit(i) << 3) | (bit(i + 256) << 2) | (bit(i + 512) << 1) | bit(i + 768));
        e[2 * i + 1] = (u8)((bit(i + 128) << 3) | (bit(i + 384) << 2) | (bit(i + 640) << 1) | bit(i + 896));
    }
    for (int r = 0; r < 42; ++r) jh_round(e, 8, JH_C[r]);
    memset(H, 0, 128);
    auto setb = [&](int i, int v) { if (v) H[i >> 3] |= (u8)(0x80 >> (i & 7)); };
    for (int i = 0; i < 128; ++i) {
        setb(i, (e[2 * i] >> 3) & 1); setb(i + 256, (e[2 * i] >> 2) & 1);
        setb(i + 512, (e[2 * i] >> 1) & 1); setb(i + 768, e[2 * i] & 1);
        setb(i + 128, (e[2 * i + 1] >> 3) & 1); setb(i + 384, (e[2 * i + 1] >> 2) & 1);
        setb(i + 640, (e[2 * i + 1] >> 1) & 1); setb(i + 896, e[2 * i + 1] & 1);
    }
}
static void jh_F8(u8 H[128], const u8 M[64]) {
    for (int i = 0; i < 64; ++i) H[i] ^= M[i];
    jh_E8(H);
    for (int i = 0; i < 64; ++i) H[64 + i] ^= M[i];
}
void jh512_iv(u8 H[128]) {
    jh_init_constants();
    memset(H, 0, 128);
    H[0] = 0x02;  // digest size 512, 16-bit big-endian
    u8 z[64] = {0};
    jh_F8(H, z);
}
void jh512(const u8* msg, size_t len, u8 out[64]) {
    u8 H[128];
    jh512_iv(H);
    size_t off = 0;
    while (len - off >= 64) { jh_F8(H, msg + off); off += 64; }
    size_t rem = len - off;
    u8 buf[128];
    memset(buf, 0, sizeof buf);
    if (rem) memcpy(buf, msg + off, rem);  // msg may be null when len == 0
    buf[rem] = 0x80;
    size_t nb = rem == 0 ? 1 : 2;
    st64be(buf + 64 * nb - 8, (u64)len * 8);  // 128-bit length, high 64 bits zero
    for (size_t b = 0; b < nb; ++b) jh_F8(H, buf + 64 * b);
    memcpy(out, H + 64, 64);
}

// ---------------------------------------------------------------------------
// 6. Keccak-512 (pre-SHA-3 padding 0x01 .. 0x80), rate 72 bytes.
// ---------------------------------------------------------------------------
void keccak_f1600(u64 A[25]) {
    static const u64 RC[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
        0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
        0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    static const int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int r = 0; r < 24; ++r) {
        u64 C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[x + 5 * y], ROT[x + 5 * y]);
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= RC[r];
    }
}
void keccak512_pad(const u8* msg, size_t len, u8 out[64], u8 padbyte) {
    u64 A[25] = {0};
    const size_t R = 72;
    size_t off = 0;
    while (len - off >= R) {
        for (size_t i = 0; i < R / 8; ++i) A[i] ^= ld64le(msg + off + 8 * i);
        keccak_f1600(A);
        off += R;
    }
    u8 buf[72];
    memset(buf, 0, sizeof buf);
    memcpy(buf, msg + off, len - off);
    buf[len - off] ^= padbyte;
    buf[R - 1] ^= 0x80;
    for (size_t i = 0; i < R / 8; ++i) A[i] ^= ld64le(buf + 8 * i);
    keccak_f1600(A);
    for (int i = 0; i < 8; ++i) st64le(out + 8 * i, A[i]);
}
void keccak512(const u8* msg, size_t len, u8 out[64]) { keccak512_pad(msg, len, out, 0x01); }

// ---------------------------------------------------------------------------
// 7. Luffa-512: w = 5 sub-permutations of 256 bits, 32-byte blocks.
// ---------------------------------------------------------------------------
static const u32 LUFFA_IV[5][8] = {
    {0x6d251e69, 0x44b051e0, 0x4eaa6fb4, 0xdbf78465, 0x6e292011, 0x90152df4, 0xee058139, 0xdef610bb},
    {0xc3b44b95, 0xd9d2f256, 0x70eee9a0, 0xde099fa3, 0x5d9b0557, 0x8fc944b3, 0xcf1ccf0e, 0x746cd581},
    {0xf7efc89d, 0x5dba5781, 0x04016ce5, 0xad659c05, 0x0306194f, 0x666d1836, 0x24aa230a, 0x8b264ae7},
    {0x858075d5, 0x36d79cce, 0xe571f7d7, 0x204b1f67, 0x35870c6a, 0x57e9e923, 0x14bcb808, 0x7cde72ce},
    {0x6c68e9be, 0x5ec41e22, 0xc825b7c7, 0xaffb4363, 0xf5df3999, 0x0fc688f1, 0xb07224cc, 0x03e86cea}};
static const u32 LUFFA_RC0[5][8] = {
    {0x303994a6, 0xc0e65299, 0x6cc33a12, 0xdc56983e, 0x1e00108f, 0x7800423d, 0x8f5b7882, 0x96e1db12},
    {0xb6de10ed, 0x70f47aae, 0x0707a3d4, 0x1c1e8f51, 0x707a3d45, 0xaeb28562, 0xbaca1589, 0x40a46f3e},
    {0xfc20d9d2, 0x34552e25, 0x7ad8818f, 0x8438764a, 0xbb6de032, 0xedb780c8, 0xd9847356, 0xa2c78434},
    {0xb213afa5, 0xc84ebe95, 0x4e608a22, 0x56d858fe, 0x343b138f, 0xd0ec4e3d, 0x2ceb4882, 0xb3ad2208},
    {0xf0d2e9e3, 0xac11d7fa, 0x1bcb66f2, 0x6f2d9bc9, 0x78602649, 0x8edae952, 0x3b6ba548, 0xedae9520}};
static const u32 LUFFA_RC4[5][8] = {
    {0xe0337818, 0x441ba90d, 0x7f34d442, 0x9389217f, 0xe5a8bce6, 0x5274baf4, 0x26889ba7, 0x9a226e9d},
    {0x01685f3d, 0x05a17cf4, 0xbd09caca, 0xf4272b28, 0x144ae5cc, 0xfaa7ae2b, 0x2e48f1c1, 0xb923c704},
    {0xe25e72c1, 0xe623bb72, 0x5c58a4a4, 0x1e38e2e7, 0x78e38b9d, 0x27586719, 0x36eda57f, 0x703aace7},
    {0xe028c9bf, 0x44756f91, 0x7e8fce32, 0x956548be, 0xfe191be2, 0x3cb226e5, 0x5944a28e, 0xa1c4c355},
    {0x5090d577, 0x2d1925ab, 0xb46496ac, 0xd1925ab0, 0x29131ab6, 0x0fc053c3, 0x3f014f0c, 0xfc053c31}};

static inline void luffa_m2(u32 a[8]) {
    u32 t = a[7];
    a[7] = a[6]; a[6] = a[5]; a[5] = a[4];
    a[4] = a[3] ^ t; a[3] = a[2] ^ t; a[2] = a[1];
    a[1] = a[0] ^ t; a[0] = t;
}
static const u8 LUFFA_SBOX[16] = {13, 14, 0, 1, 5, 10, 7, 6, 11, 3, 9, 12, 15, 8, 2, 4};
// SubCrumb on four words (x0 = least significant bit of each crumb).
// Table form (the definition) and the Luffa authors' bitsliced form; luffa_sbox_selfcheck() ties them.
static void luffa_subcrumb_table(u32& x0, u32& x1, u32& x2, u32& x3) {
    u32 y0 = 0, y1 = 0, y2 = 0, y3 = 0;
    for (int l = 0; l < 32; ++l) {
        int v = (int)(((x3 >> l) & 1) << 3 | ((x2 >> l) & 1) << 2 | ((x1 >> l) & 1) << 1 | ((x0 >> l) & 1));
        int s = LUFFA_SBOX[v];
        y0 |= (u32)(s & 1) << l; y1 |= (u32)((s >> 1) & 1) << l;
        y2 |= (u32)((s >> 2) & 1) << l; y3 |= (u32)((s >> 3) & 1) << l;
    }
    x0 = y0; x1 = y1; x2 = y2; x3 = y3;
}
static inline void luffa_subcrumb(u32& a0, u32& a1, u32& a2, u32& a3) {
    u32 t = a0;
    a0 |= a1; a2 ^= a3; a1 = ~a1; a0 ^= a3; a3 &= t; a1 ^= a3; a3 ^= a2; a2 &= a0;
    a0 = ~a0; a2 ^= a1; a1 |= a3; t ^= a1; a3 ^= a2; a2 &= a1; a1 ^= a0; a0 = t;
}
bool luffa_sbox_selfcheck() {
    u32 seed = 0x12345678u;
    for (int t = 0; t < 80; ++t) {  // t < 16: input t in every bit lane; then pseudo-random words
        u32 a[4], b[4];
        for (int k = 0; k < 4; ++k) {
            seed = seed * 1664525u + 1013904223u;
            a[k] = b[k] = t < 16 ? (((t >> k) & 1) ? 0xFFFFFFFFu : 0u) : seed;
        }
        luffa_subcrumb_table(a[0], a[1], a[2], a[3]);
        luffa_subcrumb(b[0], b[1], b[2], b[3]);
        for (int k = 0; k < 4; ++k) if (a[k] != b[k]) return false;
    }
    return true;
}
static inline void luffa_mixword(u32& u, u32& v) {
    v ^= u;
    u = rotl32(u, 2) ^ v;
    v = rotl32(v, 14) ^ u;
    u = rotl32(u, 10) ^ v;
    v = rotl32(v, 1);
}
static void luffa_Q(u32 a[8], int j) {
    for (int k = 4; k < 8; ++k) a[k] = rotl32(a[k], j);
    for (int r = 0; r < 8; ++r) {
        luffa_subcrumb(a[0], a[1], a[2], a[3]);
        luffa_subcrumb(a[5], a[6], a[7], a[4]);
        for (int k = 0; k < 4; ++k) luffa_mixword(a[k], a[k + 4]);
        a[0] ^= LUFFA_RC0[j][r];
        a[4] ^= LUFFA_RC4[j][r];
    }
}
static void luffa_round(u32 V[5][8], const u32 Min[8]) {
    u32 t[8], M[8];
    memcpy(M, Min, sizeof M);
    for (int k = 0; k < 8; ++k) t[k] = V[0][k] ^ V[1][k] ^ V[2][k] ^ V[3][k] ^ V[4][k];
    luffa_m2(t);
    for (int j = 0; j < 5; ++j)
        for (int k = 0; k < 8; ++k) V[j][k] ^= t[k];
    memcpy(t, V[0], sizeof t);
    for (int j = 0; j < 5; ++j) {
        luffa_m2(V[j]);
        const u32* nx = j < 4 ? V[j + 1] : t;
        for (int k = 0; k < 8; ++k) V[j][k] ^= nx[k];
    }
    memcpy(t, V[4], sizeof t);
    for (int j = 4; j >= 0; --j) {
        luffa_m2(V[j]);
        const u32* nx = j > 0 ? V[j - 1] : t;
        for (int k = 0; k < 8; ++k) V[j][k] ^= nx[k];
    }
    for (int j = 0; j < 5; ++j) {
        for (int k = 0; k < 8; ++k) V[j][k] ^= M[k];
        if (j < 4) luffa_m2(M);
    }
    for (int j = 0; j < 5; ++j) luffa_Q(V[j], j);
}
void luffa512(const u8* msg, size_t len, u8 out[64]) {
    u32 V[5][8], M[8];
    memcpy(V, LUFFA_IV, sizeof V);
    size_t off = 0;
    while (len - off >= 32) {
        for (int k = 0; k < 8; ++k) M[k] = ld32be(msg + off + 4 * k);
        luffa_round(V, M);
        off += 32;
    }
    u8 buf[32];
    memset(buf, 0, sizeof buf);
    memcpy(buf, msg + off, len - off);
    buf[len - off] = 0x80;
    for (int k = 0; k < 8; ++k) M[k] = ld32be(buf + 4 * k);
    luffa_round(V, M);
    u32 Z[8] = {0};
    for (int half = 0; half < 2; ++half) {
        luffa_round(V, Z);
        for (int k = 0; k < 8; ++k) st32be(out + 32 * half + 4 * k, V[0][k] ^ V[1][k] ^ V[2][k] ^ V[3][k] ^ V[4][k]);
    }
}

// ---------------------------------------------------------------------------
// 8. CubeHash16/32-512 (r = 16 rounds per 32-byte block, 10r init/final rounds).
// ---------------------------------------------------------------------------
static void cubehash_rounds(u32 x[32], int n) {
    for (int r = 0; r < n; ++r) {
        for (int i = 0; i < 16; ++i) x[i + 16] += x[i];
        for (int i = 0; i < 16; ++i) x[i] = rotl32(x[i], 7);
        for (int i = 0; i < 8; ++i) { u32 t = x[i]; x[i] = x[i + 8]; x[i + 8] = t; }
        for (int i = 0; i < 16; ++i) x[i] ^= x[i + 16];
        for (int i = 16; i < 32; ++i) if (!(i & 2)) { u32 t = x[i]; x[i] = x[i + 2]; x[i + 2] = t; }
        for (int i = 0; i < 16; ++i) x[i + 16] += x[i];
        for (int i = 0; i < 16; ++i) x[i] = rotl32(x[i], 11);
        for (int i = 0; i < 16; ++i) if (!(i & 4)) { u32 t = x[i]; x[i] = x[i + 4]; x[i + 4] = t; }
        for (int i = 0; i < 16; ++i) x[i] ^= x[i + 16];
        for (int i = 16; i < 32; ++i) if (!(i & 1)) { u32 t = x[i]; x[i] = x[i + 1]; x[i + 1] = t; }
    }
}
void cubehash512_iv(u32 x[32]) {
    for (int i = 0; i < 32; ++i) x[i] = 0;
    x[0] = 64; x[1] = 32; x[2] = 16;
    cubehash_rounds(x, 160);
}
void cubehash512(const u8* msg, size_t len, u8 out[64]) {
    u32 x[32];
    cubehash512_iv(x);
    size_t off = 0;
    while (len - off >= 32) {
        for (int i = 0; i < 8; ++i) x[i] ^= ld32le(msg + off + 4 * i);
        cubehash_rounds(x, 16);
        off += 32;
    }
    u8 buf[32];
    memset(buf, 0, sizeof buf);
    memcpy(buf, msg + off, len - off);
    buf[len - off] = 0x80;
    for (int i = 0; i < 8; ++i) x[i] ^= ld32le(buf + 4 * i);
    cubehash_rounds(x, 16);
    x[31] ^= 1;
    cubehash_rounds(x, 160);
    for (int i = 0; i < 16; ++i) st32le(out + 4 * i, x[i]);
}

// ---------------------------------------------------------------------------
// 9. SHAvite-3-512: 4-branch Feistel of 4-AES-round F functions, 14 rounds,
//    448-word message expansion with counter injection.
// ---------------------------------------------------------------------------
static void shavite_F(u32 x[4], const u32* k) {
    for (int r = 0; r < 4; ++r) {
        for (int i = 0; i < 4; ++i) x[i] ^= k[4 * r + i];
        aes_round_words(x);
    }
}
void shavite512_compress(u32 h[16], const u8 blk[128], const u32 cnt[4]) {
    init_sbox();
    u32 rk[448];
    for (int i = 0; i < 32; ++i) rk[i] = ld32le(blk + 4 * i);
    for (int r = 1; r < 14; ++r) {
        int b = 32 * r;
        if (r & 1) {
            for (int g = 0; g < 8; ++g) {
                int i = b + 4 * g;
                u32 t[4] = {rk[i - 31], rk[i - 30], rk[i - 29], rk[i - 32]};
                aes_round_words(t);
                for (int k = 0; k < 4; ++k) rk[i + k] = t[k] ^ rk[i - 4 + k];
                if (i == 32) { rk[32] ^= cnt[0]; rk[33] ^= cnt[1]; rk[34] ^= cnt[2]; rk[35] ^= ~cnt[3]; }
                if (i == 164) { rk[164] ^= cnt[3]; rk[165] ^= cnt[2]; rk[166] ^= cnt[1]; rk[167] ^= ~cnt[0]; }
                if (i == 316) { rk[316] ^= cnt[2]; rk[317] ^= cnt[3]; rk[318] ^= cnt[0]; rk[319] ^= ~cnt[1]; }
                if (i == 440) { rk[440] ^= cnt[1]; rk[441] ^= cnt[0]; rk[442] ^= cnt[3]; rk[443] ^= ~cnt[2]; }
            }
        } else {
            for (int k = 0; k < 32; ++k) rk[b + k] = rk[b + k - 32] ^ rk[b + k - 7];
        }
    }
    u32 A[4], B[4], C[4], D[4];
    for (int i = 0; i < 4; ++i) { A[i] = h[i]; B[i] = h[4 + i]; C[i] = h[8 + i]; D[i] = h[12 + i]; }
    for (int r = 0; r < 14; ++r) {
        u32 x[4];
        memcpy(x, B, sizeof x);
        shavite_F(x, rk + 32 * r);
        for (int i = 0; i < 4; ++i) A[i] ^= x[i];
        memcpy(x, D, sizeof x);
        shavite_F(x, rk + 32 * r + 16);
        for (int i = 0; i < 4; ++i) C[i] ^= x[i];
        u32 t[4];
        memcpy(t, D, sizeof t);
        memcpy(D, C, sizeof t);
        memcpy(C, B, sizeof t);
        memcpy(B, A, sizeof t);
        memcpy(A, t, sizeof t);
    }
    for (int i = 0; i < 4; ++i) { h[i] ^= A[i]; h[4 + i] ^= B[i]; h[8 + i] ^= C[i]; h[12 + i] ^= D[i]; }
}
static const u32 SHAVITE_IV[16] = {0x72FCCDD8, 0x79CA4727, 0x128A077B, 0x40D55AEC, 0xD1901A06, 0x430AE307,
                                   0xB29F5CD1, 0xDF07FBFC, 0x8E45D73D, 0x681AB538, 0xBDE86578, 0xDD577E47,
                                   0xE275EADE, 0x502D9FCD, 0xB9357178, 0x022A4B9A};
void shavite512(const u8* msg, size_t len, u8 out[64]) {
    init_sbox();
    u32 h[16];
    memcpy(h, SHAVITE_IV, sizeof h);
    u64 bits = 0;
    size_t off = 0;
    while (len - off >= 128) {
        bits += 1024;
        u32 cnt[4] = {(u32)bits, (u32)(bits >> 32), 0, 0};
        shavite512_compress(h, msg + off, cnt);
        off += 128;
    }
    size_t rem = len - off;
    u64 total = (u64)len * 8;
    u8 buf[256];
    memset(buf, 0, sizeof buf);
    if (rem) memcpy(buf, msg + off, rem);  // msg may be null when len == 0
    buf[rem] = 0x80;
    auto tail = [&](u8* b) {
        st32le(b + 110, (u32)total); st32le(b + 114, (u32)(total >> 32));
        st32le(b + 118, 0); st32le(b + 122, 0);
        b[126] = 0x00; b[127] = 0x02;
    };
    if (rem + 1 <= 110) {
        tail(buf);
        u32 cnt[4] = {rem ? (u32)total : 0u, rem ? (u32)(total >> 32) : 0u, 0, 0};
        shavite512_compress(h, buf, cnt);
    } else {
        u32 cnt[4] = {(u32)total, (u32)(total >> 32), 0, 0};
        shavite512_compress(h, buf, cnt);
        memset(buf, 0, 128);
        tail(buf);
        u32 z[4] = {0, 0, 0, 0};
        shavite512_compress(h, buf, z);
    }
    for (int i = 0; i < 16; ++i) st32le(out + 4 * i, h[i]);
}

// ---------------------------------------------------------------------------
// 10. SIMD-512: NTT over F_257 (alpha = 41), concatenated code (185 / 233),
//     4 rounds x 8 steps of a 4-branch Feistel on 32 words + 4 feed-forward steps.
// ---------------------------------------------------------------------------
static inline int mod257(int x) { x %= 257; return x < 0 ? x + 257 : x; }
static int simd_pow(int b, int e) {
    int r = 1;
    b = mod257(b);
    while (e) { if (e & 1) r = r * b % 257; b = b * b % 257; e >>= 1; }
    return r;
}
int simd_root = 41;  // evaluation root of the message NTT (self-test knob)
static void simd_expand(const u8 blk[128], bool final, int q[256]) {
    // y_i = sum_j blk_j root^(ij); root^256 = 1 (Fermat), so the exponent is taken mod 256.
    int pr[256], p41[256];
    pr[0] = p41[0] = 1;
    for (int k = 1; k < 256; ++k) { pr[k] = pr[k - 1] * mod257(simd_root) % 257; p41[k] = p41[k - 1] * 41 % 257; }
    for (int i = 0; i < 256; ++i) {
        int acc = 0;  // < 128 * 255 * 256
        for (int j = 0; j < 128; ++j)
            if (blk[j]) acc += blk[j] * pr[(i * j) & 255];
        int tw = p41[(255 * i) % 256];
        if (final) tw += p41[(253 * i) % 256];
        int v = mod257(acc + tw);
        q[i] = v <= 128 ? v : v - 257;
    }
}
static inline u32 simd_IF(u32 x, u32 y, u32 z) { return ((y ^ z) & x) ^ z; }
static inline u32 simd_MAJ(u32 x, u32 y, u32 z) { return (x & y) | ((x | y) & z); }
static void simd_step(u32 S[4][8], const u32 w[8], bool maj, int r, int s, int pp) {
    u32 tA[8];
    for (int j = 0; j < 8; ++j) tA[j] = rotl32(S[0][j], r);
    for (int j = 0; j < 8; ++j) {
        u32 f = maj ? simd_MAJ(S[0][j], S[1][j], S[2][j]) : simd_IF(S[0][j], S[1][j], S[2][j]);
        u32 tt = S[3][j] + w[j] + f;
        S[0][j] = rotl32(tt, s) + tA[j ^ pp];
        S[3][j] = S[2][j];
        S[2][j] = S[1][j];
        S[1][j] = tA[j];
    }
}
void simd512_compress(u32 state[32], const u8 blk[128], bool final) {
    int q[256];
    simd_expand(blk, final, q);
    auto inner = [](int l, int h, int mm) -> u32 { return ((u32)(l * mm) & 0xFFFFu) + ((u32)(h * mm) << 16); };
    u32 W[32][8];
    static const int SB[32] = {4, 6, 0, 2, 7, 5, 3, 1, 15, 11, 12, 8, 9, 13, 10, 14,
                               17, 18, 23, 20, 22, 21, 16, 19, 30, 24, 25, 31, 27, 29, 28, 26};
    for (int st = 0; st < 32; ++st) {
        int sb = SB[st];
        int o1, o2, mm;
        if (st < 16) { o1 = 0; o2 = 1; mm = 185; }
        else if (st < 24) { o1 = -256; o2 = -128; mm = 233; }
        else { o1 = -383; o2 = -255; mm = 233; }
        for (int j = 0; j < 8; ++j) W[st][j] = inner(q[16 * sb + 2 * j + o1], q[16 * sb + 2 * j + o2], mm);
    }
    u32 S[4][8], H[4][8];
    for (int b = 0; b < 4; ++b)
        for (int j = 0; j < 8; ++j) { H[b][j] = state[8 * b + j]; S[b][j] = H[b][j] ^ ld32le(blk + 4 * (8 * b + j)); }
    static const int PP[7] = {1, 6, 2, 3, 5, 7, 4};
    static const int RS[4][4] = {{3, 23, 17, 27}, {28, 19, 22, 7}, {29, 9, 15, 5}, {4, 13, 10, 25}};
    for (int rd = 0; rd < 4; ++rd) {
        const int* p = RS[rd];
        for (int k = 0; k < 8; ++k) {
            int r = p[k & 3], s = p[(k + 1) & 3];
            simd_step(S, W[8 * rd + k], k >= 4, r, s, PP[(k + rd) % 7]);
        }
    }
    simd_step(S, H[0], false, 4, 13, PP[4]);
    simd_step(S, H[1], false, 13, 10, PP[5]);
    simd_step(S, H[2], false, 10, 25, PP[6]);
    simd_step(S, H[3], false, 25, 4, PP[0]);
    for (int b = 0; b < 4; ++b)
        for (int j = 0; j < 8; ++j) state[8 * b + j] = S[b][j];
}
static const u32 SIMD_IV[32] = {
    0x0BA16B95, 0x72F999AD, 0x9FECC2AE, 0xBA3264FC, 0x5E894929, 0x8E9F30E5, 0x2F1DAA37, 0xF0F2C558,
    0xAC506643, 0xA90635A5, 0xE25B878B, 0xAAB7878F, 0x88817F7A, 0x0A02892B, 0x559A7550, 0x598F657E,
    0x7EEF60A1, 0x6B70E3E8, 0x9C1714D1, 0xB958E2A8, 0xAB02675E, 0xED1C014F, 0xCD8D65BB, 0xFDB7A257,
    0x09254899, 0xD699C7BC, 0x9019B6DC, 0x2B9022E4, 0x8FA14956, 0x21BF9BD3, 0xB94D0943, 0x6FFDDC22};
const u32* simd512_published_iv() { return SIMD_IV; }
void simd512(const u8* msg, size_t len, u8 out[64]) {
    u32 st[32];
    memcpy(st, SIMD_IV, sizeof st);
    size_t off = 0;
    while (len - off >= 128) { simd512_compress(st, msg + off, false); off += 128; }
    u8 buf[128];
    if (len - off > 0) {
        memset(buf, 0, sizeof buf);
        memcpy(buf, msg + off, len - off);
        simd512_compress(st, buf, false);
    }
    memset(buf, 0, sizeof buf);
    u64 bits = (u64)len * 8;
    st32le(buf, (u32)bits);
    st32le(buf + 4, (u32)(bits >> 32));
    simd512_compress(st, buf, true);
    for (int i = 0; i < 16; ++i) st32le(out + 4 * i, st[i]);
}

// ---------------------------------------------------------------------------
// 11. ECHO-512: 16 x 128-bit words, BIG.SubWords (2 AES rounds, counter key),
//     BIG.ShiftRows, BIG.MixColumns, 10 rounds, 1024-bit chaining.
// ---------------------------------------------------------------------------
static void echo512_compress(u8 V[8][16], const u8 blk[128], u64 counter) {
    u8 W[16][16];
    for (int i = 0; i < 8; ++i) { memcpy(W[i], V[i], 16); memcpy(W[8 + i], blk + 16 * i, 16); }
    u64 k = counter;
    for (int r = 0; r < 10; ++r) {
        for (int i = 0; i < 16; ++i) {
            u8 key[16];
            memset(key, 0, 16);
            st64le(key, k);
            aes_round(W[i], key);
            aes_round(W[i], nullptr);
            ++k;
        }
        u8 T[16][16];
        for (int c = 0; c < 4; ++c)
            for (int rr = 0; rr < 4; ++rr) memcpy(T[4 * c + rr], W[4 * ((c + rr) & 3) + rr], 16);
        for (int c = 0; c < 4; ++c)
            for (int b = 0; b < 16; ++b) {
                u8 a0 = T[4 * c][b], a1 = T[4 * c + 1][b], a2 = T[4 * c + 2][b], a3 = T[4 * c + 3][b];
                W[4 * c + 0][b] = (u8)(xt(a0) ^ xt(a1) ^ a1 ^ a2 ^ a3);
                W[4 * c + 1][b] = (u8)(a0 ^ xt(a1) ^ xt(a2) ^ a2 ^ a3);
                W[4 * c + 2][b] = (u8)(a0 ^ a1 ^ xt(a2) ^ xt(a3) ^ a3);
                W[4 * c + 3][b] = (u8)(xt(a0) ^ a0 ^ a1 ^ a2 ^ xt(a3));
            }
    }
    for (int i = 0; i < 8; ++i)
        for (int b = 0; b < 16; ++b) V[i][b] ^= blk[16 * i + b] ^ W[i][b] ^ W[i + 8][b];
}
void echo512(const u8* msg, size_t len, u8 out[64]) {
    init_sbox();
    u8 V[8][16];
    memset(V, 0, sizeof V);
    for (int i = 0; i < 8; ++i) V[i][1] = 0x02;  // 512 as 128-bit LE
    u64 bits = 0;
    size_t off = 0;
    while (len - off >= 128) { bits += 1024; echo512_compress(V, msg + off, bits); off += 128; }
    size_t rem = len - off;
    u64 total = (u64)len * 8;
    u8 buf[256];
    memset(buf, 0, sizeof buf);
    if (rem) memcpy(buf, msg + off, rem);  // msg may be null when len == 0
    buf[rem] = 0x80;
    auto tail = [&](u8* b) { b[110] = 0x00; b[111] = 0x02; st64le(b + 112, total); st64le(b + 120, 0); };
    if (rem + 1 <= 110) {
        tail(buf);
        echo512_compress(V, buf, rem ? total : 0);
    } else {
        echo512_compress(V, buf, total);
        memset(buf, 0, 128);
        tail(buf);
        echo512_compress(V, buf, 0);
    }
    for (int i = 0; i < 4; ++i) memcpy(out + 16 * i, V[i], 16);
}

// ---------------------------------------------------------------------------
// Chain
// ---------------------------------------------------------------------------
typedef void (*hash_fn)(const u8*, size_t, u8*);
static const hash_fn STAGES[11] = {blake512, bmw512, groestl512, skein512, jh512, keccak512,
                                   luffa512, cubehash512, shavite512, simd512, echo512};

void stage(int i, const u8* msg, size_t len, u8 out[64]) {
    init_sbox();
    jh_init_constants();
    STAGES[i](msg, len, out);
}

void x11(const u8* msg, size_t len, u8 out[32], u8* trace /* 11*64 or null */) {
    init_sbox();
    jh_init_constants();
    u8 a[64], b[64];
    STAGES[0](msg, len, a);
    if (trace) memcpy(trace, a, 64);
    for (int i = 1; i < 11; ++i) {
        STAGES[i](a, 64, b);
        memcpy(a, b, 64);
        if (trace) memcpy(trace + 64 * i, a, 64);
    }
    memcpy(out, a, 32);
}

}  // namespace x11
}  // namespace otedama

#ifdef X11_SELFTEST
#include <cstdio>
static void hex(const char* name, const uint8_t* p, size_t n) {
    printf("%s ", name);
    for (size_t i = 0; i < n; ++i) printf("%02x", p[i]);
    printf("\n");
}
int main() {
    using namespace otedama::x11;
    static const char* names[11] = {"blake", "bmw", "groestl", "skein", "jh", "keccak", "luffa", "cubehash", "shavite", "simd", "echo"};
    u8 out[64];
    for (int i = 0; i < 11; ++i) { stage(i, (const u8*)"", 0, out); hex(names[i], out, 64); }
    u64 iv[8];
    skein512_iv(iv);
    printf("skein_iv %016llx %016llx\n", (unsigned long long)iv[0], (unsigned long long)iv[1]);
    u8 H[128];
    jh512_iv(H);
    hex("jh_iv", H, 16);
    u32 c[32];
    cubehash512_iv(c);
    printf("cube_iv %08x %08x %08x %08x\n", c[0], c[1], c[2], c[3]);
    keccak512_pad((const u8*)"", 0, out, 0x06);
    hex("sha3_512", out, 16);
    const u8* sb = aes_sbox();
    printf("sbox %02x %02x %02x\n", sb[0], sb[1], sb[0x53]);
    return 0;
}
#endif
