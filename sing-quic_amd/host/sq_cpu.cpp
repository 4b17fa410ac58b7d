// sq_cpu.cpp -- the product's CPU transform (sq_cpu.h).
//
// Per packet it computes what SalamanderPacketConn / XPlusPacketConn compute
// per call (hysteria2/salamander.go:42-70, hysteria/xplus.go:46-75): a key
// from psk || salt, then the keystream XOR, with the quirk table of
// include/sqobfs.h.  Unlike the reference it hashes from the keyring's
// per-PSK midstate (one compression per packet for PSKs up to 120 / 39 B)
// and XORs a word at a time.
#include "sq_cpu.h"

#include <immintrin.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <atomic>
#include <mutex>

namespace sq {
namespace cpu {
namespace {

inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

constexpr uint64_t kB2IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                               0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                               0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                               0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
// RFC 7693 section 2.7 (rounds 10 and 11 reuse rows 0 and 1)
constexpr uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

inline void b2_g(uint64_t *v, int a, int b, int c, int d, uint64_t x, uint64_t y) {
  v[a] = v[a] + v[b] + x;
  v[d] = rotr64(v[d] ^ v[a], 32);
  v[c] = v[c] + v[d];
  v[b] = rotr64(v[b] ^ v[c], 24);
  v[a] = v[a] + v[b] + y;
  v[d] = rotr64(v[d] ^ v[a], 16);
  v[c] = v[c] + v[d];
  v[b] = rotr64(v[b] ^ v[c], 63);
}

constexpr uint32_t kS2K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

inline uint64_t ld64le(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);  // x86-64: little endian
  return v;
}
inline uint32_t ld32be(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

void b2_init256(uint64_t h[8]) {
  for (int i = 0; i < 8; i++) h[i] = kB2IV[i];
  h[0] ^= 0x01010020ULL;  // digest 32, key 0, fanout 1, depth 1
}

void s2_init(uint32_t st[8]) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(st, iv, sizeof iv);
}

constexpr uint32_t kBadLen = 0xFFFFFFFEu;   // sq_kernels.hip kBadLen
constexpr uint64_t kMaxPacket = 1ull << 26;  // sq_kernels.hip kMaxPacket

}  // namespace

namespace {

// BLAKE2b compression with AVX2: the state as four rows of four 64-bit
// words, G on the four columns at once, then on the diagonals (rows b, c, d
// rotated by 1, 2, 3 lanes); rotations by 32 / 24 / 16 are byte shuffles,
// by 63 a shift pair.
__attribute__((target("avx2"))) void b2_compress_avx2(uint64_t h[8], const uint64_t m[16],
                                                       uint64_t t, bool last) {
  const __m256i r24 = _mm256_setr_epi8(3, 4, 5, 6, 7, 0, 1, 2, 11, 12, 13, 14, 15, 8, 9, 10,
                                       3, 4, 5, 6, 7, 0, 1, 2, 11, 12, 13, 14, 15, 8, 9, 10);
  const __m256i r16 = _mm256_setr_epi8(2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 12, 13, 14, 15, 8, 9,
                                       2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 12, 13, 14, 15, 8, 9);
  const __m256i h0 = _mm256_loadu_si256((const __m256i *)&h[0]);
  const __m256i h1 = _mm256_loadu_si256((const __m256i *)&h[4]);
  __m256i a = h0, b = h1;
  __m256i c = _mm256_loadu_si256((const __m256i *)&kB2IV[0]);
  __m256i d = _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)&kB2IV[4]),
                               _mm256_set_epi64x(0, last ? -1ll : 0, 0, (long long)t));
  // (a macro: a lambda would not inherit the function's target)
#define SQ_B2G_AVX2(x, y)                                                      \
  do {                                                                         \
    a = _mm256_add_epi64(_mm256_add_epi64(a, b), (x));                         \
    d = _mm256_shuffle_epi32(_mm256_xor_si256(d, a), _MM_SHUFFLE(2, 3, 0, 1)); \
    c = _mm256_add_epi64(c, d);                                                \
    b = _mm256_shuffle_epi8(_mm256_xor_si256(b, c), r24);                      \
    a = _mm256_add_epi64(_mm256_add_epi64(a, b), (y));                         \
    d = _mm256_shuffle_epi8(_mm256_xor_si256(d, a), r16);                      \
    c = _mm256_add_epi64(c, d);                                                \
    const __m256i e_ = _mm256_xor_si256(b, c);                                 \
    b = _mm256_or_si256(_mm256_srli_epi64(e_, 63), _mm256_add_epi64(e_, e_));  \
  } while (0)
  for (int r = 0; r < 12; r++) {
    const uint8_t *z = kSigma[r];
    SQ_B2G_AVX2(_mm256_set_epi64x((long long)m[z[6]], (long long)m[z[4]], (long long)m[z[2]],
                                  (long long)m[z[0]]),
                _mm256_set_epi64x((long long)m[z[7]], (long long)m[z[5]], (long long)m[z[3]],
                                  (long long)m[z[1]]));
    b = _mm256_permute4x64_epi64(b, 0x39);  // diagonals: lane j holds b[j+1], c[j+2], d[j+3]
    c = _mm256_permute4x64_epi64(c, 0x4E);
    d = _mm256_permute4x64_epi64(d, 0x93);
    SQ_B2G_AVX2(_mm256_set_epi64x((long long)m[z[14]], (long long)m[z[12]], (long long)m[z[10]],
                                  (long long)m[z[8]]),
                _mm256_set_epi64x((long long)m[z[15]], (long long)m[z[13]], (long long)m[z[11]],
                                  (long long)m[z[9]]));
    b = _mm256_permute4x64_epi64(b, 0x93);
    c = _mm256_permute4x64_epi64(c, 0x4E);
    d = _mm256_permute4x64_epi64(d, 0x39);
  }
  _mm256_storeu_si256((__m256i *)&h[0], _mm256_xor_si256(h0, _mm256_xor_si256(a, c)));
  _mm256_storeu_si256((__m256i *)&h[4], _mm256_xor_si256(h1, _mm256_xor_si256(b, d)));
#undef SQ_B2G_AVX2
}

void b2_compress_portable(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last);

using B2Fn = void (*)(uint64_t *, const uint64_t *, uint64_t, bool);
// SQOBFS_CPU_PORTABLE=1 (tests): the portable compressions on any CPU
bool force_portable() {
  const char *e = getenv("SQOBFS_CPU_PORTABLE");
  return e && *e == '1';
}

B2Fn pick_b2() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") && !force_portable() ? b2_compress_avx2
                                                              : b2_compress_portable;
}

}  // namespace

void b2_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  static const B2Fn fn = pick_b2();
  fn(h, m, t, last);
}

namespace {
void b2_compress_portable(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  uint64_t v[16];
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = kB2IV[i];
  }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t *s = kSigma[r];
    b2_g(v, 0, 4, 8, 12, m[s[0]], m[s[1]]);
    b2_g(v, 1, 5, 9, 13, m[s[2]], m[s[3]]);
    b2_g(v, 2, 6, 10, 14, m[s[4]], m[s[5]]);
    b2_g(v, 3, 7, 11, 15, m[s[6]], m[s[7]]);
    b2_g(v, 0, 5, 10, 15, m[s[8]], m[s[9]]);
    b2_g(v, 1, 6, 11, 12, m[s[10]], m[s[11]]);
    b2_g(v, 2, 7, 8, 13, m[s[12]], m[s[13]]);
    b2_g(v, 3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}
}  // namespace

namespace {

// SHA-256 compression with the x86 SHA extensions (four rounds per
// sha256rnds2 pair, the schedule by sha256msg1 / sha256msg2); used when the
// CPU has them (AMD Zen, Intel since Ice Lake), picked once at first use.
__attribute__((target("sha,sse4.1"))) void s2_compress_shani(uint32_t st[8],
                                                             const uint32_t m[16]) {
  __m128i t = _mm_loadu_si128((const __m128i *)&st[0]);  // A B C D
  __m128i s1 = _mm_loadu_si128((const __m128i *)&st[4]); // E F G H
  t = _mm_shuffle_epi32(t, 0xB1);
  s1 = _mm_shuffle_epi32(s1, 0x1B);
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);     // A B E F (the instruction's order)
  s1 = _mm_blend_epi16(s1, t, 0xF0);          // C D G H
  const __m128i abef = s0, cdgh = s1;
  __m128i w[4];
  for (int i = 0; i < 16; i++) {
    __m128i x;
    if (i < 4) {
      x = _mm_loadu_si128((const __m128i *)&m[4 * i]);  // (the words, already decoded)
    } else {
      x = _mm_sha256msg1_epu32(w[(i - 4) & 3], w[(i - 3) & 3]);
      x = _mm_add_epi32(x, _mm_alignr_epi8(w[(i - 1) & 3], w[(i - 2) & 3], 4));
      x = _mm_sha256msg2_epu32(x, w[(i - 1) & 3]);
    }
    w[i & 3] = x;
    __m128i mk = _mm_add_epi32(x, _mm_loadu_si128((const __m128i *)&kS2K[4 * i]));
    s1 = _mm_sha256rnds2_epu32(s1, s0, mk);
    mk = _mm_shuffle_epi32(mk, 0x0E);
    s0 = _mm_sha256rnds2_epu32(s0, s1, mk);
  }
  s0 = _mm_add_epi32(s0, abef);
  s1 = _mm_add_epi32(s1, cdgh);
  t = _mm_shuffle_epi32(s0, 0x1B);
  s1 = _mm_shuffle_epi32(s1, 0xB1);
  _mm_storeu_si128((__m128i *)&st[0], _mm_blend_epi16(t, s1, 0xF0));  // A B C D
  _mm_storeu_si128((__m128i *)&st[4], _mm_alignr_epi8(s1, t, 8));     // E F G H
}

void s2_compress_portable(uint32_t st[8], const uint32_t m[16]);

using S2Fn = void (*)(uint32_t *, const uint32_t *);
S2Fn pick_s2() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1") && !force_portable()
             ? s2_compress_shani
             : s2_compress_portable;
}

}  // namespace

void s2_compress(uint32_t st[8], const uint32_t m[16]) {
  static const S2Fn fn = pick_s2();
  fn(st, m);
}

namespace {
void s2_compress_portable(uint32_t st[8], const uint32_t m[16]) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++) w[i] = m[i];
  for (int i = 16; i < 64; i++) {
    const uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
  for (int i = 0; i < 64; i++) {
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t t1 = h + S1 + ((e & f) ^ (~e & g)) + kS2K[i] + w[i];
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t t2 = S0 + ((a & b) ^ (a & c) ^ (b & c));
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}
}  // namespace

void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3],
                    uint32_t out[16]) {
  const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                           key[0],      key[1],      key[2],      key[3],
                           key[4],      key[5],      key[6],      key[7],
                           counter,     nonce[0],    nonce[1],    nonce[2]};
  uint32_t x[16];
  memcpy(x, in, sizeof x);
  auto qr = [&](int a, int b, int c, int d) {
    x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);
    x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);
    x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);
    x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
  };
  for (int r = 0; r < 10; r++) {
    qr(0, 4, 8, 12);
    qr(1, 5, 9, 13);
    qr(2, 6, 10, 14);
    qr(3, 7, 11, 15);
    qr(0, 5, 10, 15);
    qr(1, 6, 11, 12);
    qr(2, 7, 8, 13);
    qr(3, 4, 9, 14);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

void psk_prepare(int kind, const uint8_t *psk, uint32_t L, PskEntry *e) {
  memset(e, 0, sizeof *e);
  uint8_t tm[256];
  memset(tm, 0, sizeof tm);
  e->psk_len = L;
  e->kind = (uint32_t)kind;
  if (kind == SQOBFS_SALAMANDER) {
    // every PSK-only 128-byte block is followed by salt bytes, so it is never
    // BLAKE2b's final block (RFC 7693 section 3.3)
    uint64_t h[8];
    b2_init256(h);
    const uint32_t nfull = L / 128;
    for (uint32_t bk = 0; bk < nfull; bk++) {
      uint64_t m[16];
      for (int j = 0; j < 16; j++) m[j] = ld64le(psk + 128 * bk + 8 * j);
      b2_compress(h, m, 128ull * (bk + 1), false);
    }
    const uint32_t tail = L - 128 * nfull, tot = tail + kSalamanderSalt;
    if (tail) memcpy(tm, psk + 128 * nfull, tail);
    memcpy(e->h, h, sizeof h);
    for (int j = 0; j < 32; j++) e->m[j] = ld64le(tm + 8 * j);
    e->nblocks = tot > 128 ? 2 : 1;
    e->salt_pos = tail;
    e->t_first = 128ull * nfull + 128;
    e->t_last = 128ull * nfull + tot;
  } else {
    // SHA-256: 0x80 pad and the 64-bit big-endian bit length
    uint32_t st[8];
    s2_init(st);
    const uint32_t nfull = L / 64;
    for (uint32_t bk = 0; bk < nfull; bk++) {
      uint32_t m[16];
      for (int j = 0; j < 16; j++) m[j] = ld32be(psk + 64 * bk + 4 * j);
      s2_compress(st, m);
    }
    const uint32_t tail = L - 64 * nfull, used = tail + kXPlusSalt + 1 + 8;
    const uint32_t nb = used > 64 ? 2 : 1;
    if (tail) memcpy(tm, psk + 64 * nfull, tail);
    tm[tail + kXPlusSalt] = 0x80;
    const uint64_t bits = ((uint64_t)L + kXPlusSalt) * 8;
    for (int i = 0; i < 8; i++) tm[64 * nb - 1 - i] = (uint8_t)(bits >> (8 * i));
    uint32_t *h32 = reinterpret_cast<uint32_t *>(e->h);
    for (int i = 0; i < 8; i++) h32[i] = st[i];
    uint32_t *m32 = reinterpret_cast<uint32_t *>(e->m);
    for (int j = 0; j < 32; j++) m32[j] = ld32be(tm + 4 * j);
    e->nblocks = nb;
    e->salt_pos = tail;
  }
}

void derive_key(const PskEntry &e, const uint8_t *salt, uint8_t key[32]) {
  if (e.kind == SQOBFS_SALAMANDER) {
    // the final block(s): the entry's template (PSK tail, zero padded) with
    // the salt at salt_pos; on a little-endian host the words are the bytes
    uint8_t blk[256];
    memcpy(blk, e.m, sizeof blk);
    memcpy(blk + e.salt_pos, salt, kSalamanderSalt);
    uint64_t h[8], m[16];
    memcpy(h, e.h, sizeof h);
    for (uint32_t b = 0; b < e.nblocks; b++) {
      memcpy(m, blk + 128 * b, 128);
      const bool last = b + 1 == e.nblocks;
      b2_compress(h, m, last ? e.t_last : e.t_first, last);
    }
    memcpy(key, h, 32);
  } else {
    // big-endian words: byte i of the block is bits 24 - 8 (i % 4) of word i / 4
    uint32_t m[32];
    memcpy(m, e.m, sizeof m);
    for (uint32_t k = 0; k < (uint32_t)kXPlusSalt; k++) {
      const uint32_t i = e.salt_pos + k;
      m[i / 4] |= (uint32_t)salt[k] << (24 - 8 * (i % 4));
    }
    uint32_t st[8];
    memcpy(st, e.h, sizeof st);
    for (uint32_t b = 0; b < e.nblocks; b++) s2_compress(st, m + 16 * b);
    for (int i = 0; i < 8; i++) {
      key[4 * i] = (uint8_t)(st[i] >> 24);
      key[4 * i + 1] = (uint8_t)(st[i] >> 16);
      key[4 * i + 2] = (uint8_t)(st[i] >> 8);
      key[4 * i + 3] = (uint8_t)st[i];
    }
  }
}


// ---- multi-buffer BLAKE2b: L one-block messages at once, one per 64-bit
// vector lane (every packet's key is one compression for PSKs up to 120 B),
// so a batch's keys cost ~1/L of a compression each instead of one.
// L = 8 with AVX-512 (rotations are vprorq), 4 with AVX2.  SoA in and out:
// h[i][l] = chaining word i of message l, m[j][l] = its message word j,
// t[l] = its byte counter; key[i][l] = word i of its 32-byte digest.
namespace {
template <int L>
struct B2Lanes {
  uint64_t h[8][L], m[16][L], t[L];
  uint64_t key[4][L];
};

#define SQ_B2MB_ROR(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
#define SQ_B2MB_G(a, b, c, d, x, y)                  \
  do {                                               \
    v[a] = v[a] + v[b] + (x);                        \
    v[d] = SQ_B2MB_ROR(v[d] ^ v[a], 32);             \
    v[c] = v[c] + v[d];                              \
    v[b] = SQ_B2MB_ROR(v[b] ^ v[c], 24);             \
    v[a] = v[a] + v[b] + (y);                        \
    v[d] = SQ_B2MB_ROR(v[d] ^ v[a], 16);             \
    v[c] = v[c] + v[d];                              \
    v[b] = SQ_B2MB_ROR(v[b] ^ v[c], 63);             \
  } while (0)
#define SQ_B2MB_BODY(V)                                                         \
  V v[16], mm[16];                                                             \
  for (int i = 0; i < 8; i++) {                                                \
    memcpy(&v[i], J.h[i], sizeof(V));                                          \
    v[i + 8] = (V){} + kB2IV[i];                                               \
  }                                                                            \
  V tt;                                                                        \
  memcpy(&tt, J.t, sizeof(V));                                                 \
  v[12] ^= tt;                                                                 \
  v[14] = ~v[14]; /* every message here is its own final block */              \
  for (int j = 0; j < 16; j++) memcpy(&mm[j], J.m[j], sizeof(V));              \
  /* (macros: a lambda would not inherit the function's target) */           \
  for (int r = 0; r < 12; r++) {                                               \
    const uint8_t *z = kSigma[r];                                              \
    SQ_B2MB_G(0, 4, 8, 12, mm[z[0]], mm[z[1]]);                                \
    SQ_B2MB_G(1, 5, 9, 13, mm[z[2]], mm[z[3]]);                                \
    SQ_B2MB_G(2, 6, 10, 14, mm[z[4]], mm[z[5]]);                               \
    SQ_B2MB_G(3, 7, 11, 15, mm[z[6]], mm[z[7]]);                               \
    SQ_B2MB_G(0, 5, 10, 15, mm[z[8]], mm[z[9]]);                               \
    SQ_B2MB_G(1, 6, 11, 12, mm[z[10]], mm[z[11]]);                             \
    SQ_B2MB_G(2, 7, 8, 13, mm[z[12]], mm[z[13]]);                              \
    SQ_B2MB_G(3, 4, 9, 14, mm[z[14]], mm[z[15]]);                              \
  }                                                                            \
  for (int i = 0; i < 4; i++) {                                                \
    V hi;                                                                      \
    memcpy(&hi, J.h[i], sizeof(V));                                            \
    const V k = hi ^ v[i] ^ v[i + 8];                                          \
    memcpy(J.key[i], &k, sizeof(V));                                           \
  }

typedef uint64_t u64x8 __attribute__((vector_size(64)));
typedef uint64_t u64x4 __attribute__((vector_size(32)));
__attribute__((target("avx512f"))) void b2_mb8_avx512(B2Lanes<8> &J) { SQ_B2MB_BODY(u64x8) }
__attribute__((target("avx2"))) void b2_mb4_avx2(B2Lanes<4> &J) { SQ_B2MB_BODY(u64x4) }
#undef SQ_B2MB_BODY
#undef SQ_B2MB_G
#undef SQ_B2MB_ROR

// lanes per multi-buffer call on this CPU (0: none, per-message compressions)
// SQOBFS_CPU_MB=avx2 (tests): the AVX2 multi-buffer width on an AVX-512 host
int pick_b2_lanes() {
  __builtin_cpu_init();
  if (force_portable()) return 0;
  const char *e = getenv("SQOBFS_CPU_MB");
  const bool avx2_only = e && strcmp(e, "avx2") == 0;
  if (__builtin_cpu_supports("avx512f") && !avx2_only) return 8;
  return __builtin_cpu_supports("avx2") ? 4 : 0;
}
int b2_lanes() {
  static const int l = pick_b2_lanes();
  return l;
}

// The keys of n <= 8 packets whose entries are one-block (nblocks == 1):
// salts[k] = packet k's salt (8 bytes), keys[k] = its key.
template <int L>
void b2_keys_mb(const PskEntry *const *es, const uint8_t (*salts)[16], uint32_t n,
                uint8_t (*keys)[32], void (*fn)(B2Lanes<L> &)) {
  for (uint32_t k0 = 0; k0 < n; k0 += L) {
    B2Lanes<L> J;
    for (int l = 0; l < L; l++) {
      const uint32_t k = k0 + l < n ? k0 + l : n - 1;  // (a short group repeats its last)
      const PskEntry &e = *es[k];
      uint8_t blk[128];
      memcpy(blk, e.m, sizeof blk);
      memcpy(blk + e.salt_pos, salts[k], kSalamanderSalt);
      for (int i = 0; i < 8; i++) J.h[i][l] = e.h[i];
      for (int j = 0; j < 16; j++) J.m[j][l] = ld64le(blk + 8 * j);
      J.t[l] = e.t_last;
    }
    fn(J);
    for (int l = 0; l < L && k0 + l < n; l++)
      for (int i = 0; i < 4; i++) memcpy(keys[k0 + l] + 8 * i, &J.key[i][l], 8);
  }
}
}  // namespace

// ---- multi-buffer SHA-256 for XPlus: L one-block messages at once, one
// per 32-bit lane (every key is one compression for PSKs up to 39 B); L = 16
// with AVX-512, 8 with AVX2.  SoA: st[i][l], m[j][l] (big-endian words).
namespace {
template <int L>
struct S2Lanes {
  uint32_t st[8][L], m[16][L];
};

#define SQ_S2MB_ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
#define SQ_S2MB_BODY(V)                                                            \
  V w[16], a, b, c, d, e, f, g, h, st0[8];                                        \
  for (int i = 0; i < 8; i++) memcpy(&st0[i], J.st[i], sizeof(V));                \
  for (int j = 0; j < 16; j++) memcpy(&w[j], J.m[j], sizeof(V));                  \
  a = st0[0]; b = st0[1]; c = st0[2]; d = st0[3];                                 \
  e = st0[4]; f = st0[5]; g = st0[6]; h = st0[7];                                 \
  for (int i = 0; i < 64; i++) {                                                  \
    if (i >= 16) {                                                                \
      const V x15 = w[(i - 15) & 15], x2 = w[(i - 2) & 15];                       \
      const V s0 = SQ_S2MB_ROR(x15, 7) ^ SQ_S2MB_ROR(x15, 18) ^ (x15 >> 3);       \
      const V s1 = SQ_S2MB_ROR(x2, 17) ^ SQ_S2MB_ROR(x2, 19) ^ (x2 >> 10);        \
      w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;                          \
    }                                                                             \
    const V S1 = SQ_S2MB_ROR(e, 6) ^ SQ_S2MB_ROR(e, 11) ^ SQ_S2MB_ROR(e, 25);     \
    const V t1 = h + S1 + ((e & f) ^ (~e & g)) + kS2K[i] + w[i & 15];             \
    const V S0 = SQ_S2MB_ROR(a, 2) ^ SQ_S2MB_ROR(a, 13) ^ SQ_S2MB_ROR(a, 22);     \
    const V t2 = S0 + ((a & b) ^ (a & c) ^ (b & c));                              \
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;            \
  }                                                                               \
  const V out[8] = {a + st0[0], b + st0[1], c + st0[2], d + st0[3],               \
                    e + st0[4], f + st0[5], g + st0[6], h + st0[7]};              \
  for (int i = 0; i < 8; i++) memcpy(J.st[i], &out[i], sizeof(V));

typedef uint32_t u32x16 __attribute__((vector_size(64)));
typedef uint32_t u32x8 __attribute__((vector_size(32)));
__attribute__((target("avx512f"))) void s2_mb16_avx512(S2Lanes<16> &J) { SQ_S2MB_BODY(u32x16) }
__attribute__((target("avx2"))) void s2_mb8_avx2(S2Lanes<8> &J) { SQ_S2MB_BODY(u32x8) }
#undef SQ_S2MB_BODY
#undef SQ_S2MB_ROR

// The keys of n one-block XPlus packets (salts[k]: 16 bytes)
template <int L>
void s2_keys_mb(const PskEntry *const *es, const uint8_t (*salts)[16], uint32_t n,
                uint8_t (*keys)[32], void (*fn)(S2Lanes<L> &)) {
  for (uint32_t k0 = 0; k0 < n; k0 += L) {
    S2Lanes<L> J;
    for (int l = 0; l < L; l++) {
      const uint32_t k = k0 + l < n ? k0 + l : n - 1;  // (a short group repeats its last)
      const PskEntry &e = *es[k];
      uint32_t m[16];
      memcpy(m, e.m, sizeof m);
      for (uint32_t q = 0; q < (uint32_t)kXPlusSalt; q++) {
        const uint32_t i = e.salt_pos + q;
        m[i / 4] |= (uint32_t)salts[k][q] << (24 - 8 * (i % 4));
      }
      const uint32_t *h32 = reinterpret_cast<const uint32_t *>(e.h);
      for (int i = 0; i < 8; i++) J.st[i][l] = h32[i];
      for (int j = 0; j < 16; j++) J.m[j][l] = m[j];
    }
    fn(J);
    for (int l = 0; l < L && k0 + l < n; l++)
      for (int i = 0; i < 8; i++) {
        const uint32_t x = J.st[i][l];
        keys[k0 + l][4 * i] = (uint8_t)(x >> 24);
        keys[k0 + l][4 * i + 1] = (uint8_t)(x >> 16);
        keys[k0 + l][4 * i + 2] = (uint8_t)(x >> 8);
        keys[k0 + l][4 * i + 3] = (uint8_t)x;
      }
  }
}
}  // namespace

void derive_keys(const PskEntry *const *es, const uint8_t (*salts)[16], uint32_t n,
                 uint8_t (*keys)[32]) {
  // one-block entries through the multi-buffer compressions (BLAKE2b
  // Salamander, SHA-256 XPlus), two-block PSKs one at a time
  const PskEntry *one[kKeyBatch];
  uint8_t osalt[kKeyBatch][16];
  uint32_t idx[kKeyBatch], m = 0;
  const int lanes = b2_lanes();  // (8: AVX-512, 4: AVX2, 0: neither)
  const int kind = n ? (int)es[0]->kind : 0;  // (one keyring: one kind)
  for (uint32_t k = 0; k < n; k++) {
    if (lanes && es[k]->nblocks == 1) {
      one[m] = es[k];
      memcpy(osalt[m], salts[k], 16);
      idx[m++] = k;
    } else {
      derive_key(*es[k], salts[k], keys[k]);
    }
  }
  if (!m) return;
  uint8_t ok[kKeyBatch][32];
  if (kind == SQOBFS_SALAMANDER) {
    if (lanes == 8) b2_keys_mb<8>(one, osalt, m, ok, b2_mb8_avx512);
    else b2_keys_mb<4>(one, osalt, m, ok, b2_mb4_avx2);
  } else {
    if (lanes == 8) s2_keys_mb<16>(one, osalt, m, ok, s2_mb16_avx512);
    else s2_keys_mb<8>(one, osalt, m, ok, s2_mb8_avx2);
  }
  for (uint32_t q = 0; q < m; q++) memcpy(keys[idx[q]], ok[q], 32);
}

// 32 bytes per iteration as four 64-bit words (the compiler widens the loop
// to vector registers); the key's period is 32, so the key words are fixed.
// Two builds of the same loop, AVX2 and baseline, picked once (a plain
// function pointer, not an ifunc: ifunc resolvers run before the sanitizer
// runtimes are up).
namespace {
template <int>
inline void xor_loop(uint8_t *dst, const uint8_t *src, size_t n, const uint8_t key[32]) {
  uint64_t k[4];
  memcpy(k, key, 32);
  size_t j = 0;
  for (; j + 32 <= n; j += 32) {
    uint64_t w[4];
    memcpy(w, src + j, 32);
    w[0] ^= k[0];
    w[1] ^= k[1];
    w[2] ^= k[2];
    w[3] ^= k[3];
    memcpy(dst + j, w, 32);
  }
  for (; j < n; j++) dst[j] = src[j] ^ key[j & 31];
}
__attribute__((target("avx2"))) void xor_avx2(uint8_t *dst, const uint8_t *src, size_t n,
                                              const uint8_t key[32]) {
  xor_loop<1>(dst, src, n, key);
}
void xor_base(uint8_t *dst, const uint8_t *src, size_t n, const uint8_t key[32]) {
  xor_loop<0>(dst, src, n, key);
}
using XorFn = void (*)(uint8_t *, const uint8_t *, size_t, const uint8_t *);
XorFn pick_xor() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") && !force_portable() ? xor_avx2 : xor_base;
}
}  // namespace

void xor_stream(uint8_t *dst, const uint8_t *src, size_t n, const uint8_t key[32]) {
  static const XorFn fn = pick_xor();
  fn(dst, src, n, key);
}

void salt_stream(const uint32_t key[8], uint64_t seq, uint8_t *out, size_t bytes) {
  const uint32_t nonce[3] = {0x626f7173u /* "sqob" */, (uint32_t)seq, (uint32_t)(seq >> 32)};
  uint32_t blk[16];
  for (size_t o = 0, c = 0; o < bytes; o += 64, c++) {
    chacha20_block(key, (uint32_t)c, nonce, blk);
    const size_t k = bytes - o < 64 ? bytes - o : 64;
    memcpy(out + o, blk, k);  // little-endian words are the keystream bytes
  }
}

int run_batch(int kind, int dir, const PskEntry *table, uint32_t count, const sqobfs_batch *b,
              const uint8_t *salts) {
  if (!b || !table || count == 0) return SQ_EINVAL;
  if (b->n == 0) return SQ_OK;
  if (!b->in || !b->in_off || !b->in_len || !b->out || !b->out_off || !b->out_len)
    return SQ_EINVAL;
  const size_t S = kind == SQOBFS_SALAMANDER ? kSalamanderSalt : kXPlusSalt;
  const bool obfs = dir == SQOBFS_OBFUSCATE;
  if (obfs && !salts && !b->salt) return SQ_EINVAL;
  // kKeyBatch packets at a time: first every key of the group (the salts
  // copied first: an in-place salt may sit where the output goes), then the
  // XORs.  Packets' buffers do not overlap one another's.
  enum : uint8_t { kDone, kObfs, kCopy, kDeobfs };
  for (uint32_t i0 = 0; i0 < b->n; i0 += kKeyBatch) {
    const uint32_t i1 = b->n - i0 < kKeyBatch ? b->n : i0 + kKeyBatch;
    uint8_t what[kKeyBatch];
    uint64_t caps[kKeyBatch];
    uint8_t sl[kKeyBatch][16];
    uint8_t keys[kKeyBatch][32];
    const PskEntry *es[kKeyBatch];
    uint8_t ks[kKeyBatch][16];
    uint32_t kidx[kKeyBatch], nk = 0;
    for (uint32_t i = i0; i < i1; i++) {
      const uint32_t q = i - i0;
      what[q] = kDone;
      const uint32_t pid = b->psk_id ? b->psk_id[i] : 0u;
      const uint64_t len = b->in_len[i];
      const uint64_t cap = (!obfs && kind == SQOBFS_XPLUS && b->in_cap && b->in_cap[i] > len)
                               ? b->in_cap[i] : len;
      caps[q] = cap;
      if (len > kMaxPacket || cap > kMaxPacket) {
        b->out_len[i] = kBadLen;
        continue;
      }
      if (pid >= count) {
        b->out_len[i] = SQOBFS_BAD_PSK;
        continue;
      }
      const uint8_t *in = b->in + b->in_off[i];
      if (obfs) {  // salamander.go:57-70, xplus.go:62-75: salt || payload ^ key
        memcpy(sl[q], salts ? salts + (size_t)i * S : b->salt + (size_t)i * S, S);
        what[q] = kObfs;
      } else if (kind == SQOBFS_SALAMANDER && len <= S) {
        what[q] = kCopy;  // salamander.go:47-49: returned as is
        continue;
      } else if (kind == SQOBFS_XPLUS && len < S) {
        b->out_len[i] = 0;  // xplus.go:50-52
        continue;
      } else {  // salamander.go:50-53, xplus.go:54-57: the salt is the wire's head
        memcpy(sl[q], in, S);
        what[q] = kDeobfs;
      }
      es[nk] = &table[pid];
      memcpy(ks[nk], sl[q], 16);
      kidx[nk++] = q;
    }
    uint8_t kk[kKeyBatch][32];
    derive_keys(es, ks, nk, kk);
    for (uint32_t k = 0; k < nk; k++) memcpy(keys[kidx[k]], kk[k], 32);
    for (uint32_t i = i0; i < i1; i++) {
      const uint32_t q = i - i0;
      const uint64_t len = b->in_len[i];
      const uint8_t *in = b->in + b->in_off[i];
      uint8_t *out = b->out + b->out_off[i];
      switch (what[q]) {
        case kObfs:
          xor_stream(out + S, in, len, keys[q]);
          memcpy(out, sl[q], S);
          b->out_len[i] = (uint32_t)(S + len);
          break;
        case kCopy:
          memmove(out, in, len);
          b->out_len[i] = (uint32_t)len;
          break;
        case kDeobfs:  // (XPlus XORs to len(p) = cap)
          xor_stream(out, in + S, caps[q] - S, keys[q]);
          b->out_len[i] = (uint32_t)(len - S);
          break;
        default:
          break;
      }
    }
  }
  return SQ_OK;
}

}  // namespace cpu
}  // namespace sq

// ---- the process's host salt generator (keyrings without a context):
// ChaCha20 keyed from getrandom(2) once, one sequence number per use
void sq_host_salt_take(uint32_t key[8], uint64_t *seq) {
  static std::once_flag once;
  static uint32_t k[8];
  static std::atomic<uint64_t> next{0};
  std::call_once(once, [] {
    uint8_t b[32];
    size_t got = 0;
    while (got < sizeof b) {
      const ssize_t r = getrandom(b + got, sizeof b - got, 0);
      if (r > 0) got += (size_t)r;
    }
    memcpy(k, b, sizeof k);
  });
  memcpy(key, k, sizeof k);
  *seq = next.fetch_add(1);
}
