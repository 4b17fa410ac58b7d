// sq_hash.h -- lane-parallel BLAKE2b / SHA-256 compression for gfx950.
//
// Each lane of a wave compresses a DIFFERENT packet's psk||salt block, so the
// 64 lanes run the same straight-line code with no cross-lane traffic.
// Everything is register-resident and fully unrolled: message words are
// indexed by compile-time constants only (no scratch).
//
// BLAKE2b (RFC 7693) replaces golang.org/x/crypto/blake2b.Sum256 as called at
// hysteria2/salamander.go:50,61,84,99.  64-bit words: adds lower to
// v_lshl_add_u64, rotations to v_alignbit_b32 pairs (rotate by 32 is a
// register swap).
// SHA-256 (FIPS 180-4) replaces crypto/sha256.Sum256 as called at
// hysteria/xplus.go:54,70,93,107.  Rotations are single v_alignbit_b32.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sq {

// ---------------------------------------------------------------- BLAKE2b

__device__ __forceinline__ uint64_t b2_pack(uint32_t lo, uint32_t hi) {
  return ((uint64_t)hi << 32) | lo;
}

// rotr64 by n in (0,32): two funnel shifts of the halves
template <int N>
__device__ __forceinline__ uint64_t b2_rotr_lt32(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return b2_pack(__builtin_amdgcn_alignbit(hi, lo, N),
                 __builtin_amdgcn_alignbit(lo, hi, N));
}
__device__ __forceinline__ uint64_t b2_rotr32(uint64_t x) {
  return (x >> 32) | (x << 32);
}
// rotr 63 == rotl 1 == swap halves then rotr 31
__device__ __forceinline__ uint64_t b2_rotr63(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return b2_pack(__builtin_amdgcn_alignbit(lo, hi, 31),
                 __builtin_amdgcn_alignbit(hi, lo, 31));
}

#define SQ_B2_G(a, b, c, d, x, y)            \
  do {                                       \
    v##a = v##a + v##b + (x);                \
    v##d = b2_rotr32(v##d ^ v##a);           \
    v##c = v##c + v##d;                      \
    v##b = b2_rotr_lt32<24>(v##b ^ v##c);    \
    v##a = v##a + v##b + (y);                \
    v##d = b2_rotr_lt32<16>(v##d ^ v##a);    \
    v##c = v##c + v##d;                      \
    v##b = b2_rotr63(v##b ^ v##c);           \
  } while (0)

// One round with the RFC 7693 section 2.7 schedule row given literally.
#define SQ_B2_ROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, \
                    s13, s14, s15)                                          \
  do {                                                                      \
    SQ_B2_G(0, 4, 8, 12, m[s0], m[s1]);                                     \
    SQ_B2_G(1, 5, 9, 13, m[s2], m[s3]);                                     \
    SQ_B2_G(2, 6, 10, 14, m[s4], m[s5]);                                    \
    SQ_B2_G(3, 7, 11, 15, m[s6], m[s7]);                                    \
    SQ_B2_G(0, 5, 10, 15, m[s8], m[s9]);                                    \
    SQ_B2_G(1, 6, 11, 12, m[s10], m[s11]);                                  \
    SQ_B2_G(2, 7, 8, 13, m[s12], m[s13]);                                   \
    SQ_B2_G(3, 4, 9, 14, m[s14], m[s15]);                                   \
  } while (0)

constexpr uint64_t kB2IV0 = 0x6a09e667f3bcc908ULL;
constexpr uint64_t kB2IV1 = 0xbb67ae8584caa73bULL;
constexpr uint64_t kB2IV2 = 0x3c6ef372fe94f82bULL;
constexpr uint64_t kB2IV3 = 0xa54ff53a5f1d36f1ULL;
constexpr uint64_t kB2IV4 = 0x510e527fade682d1ULL;
constexpr uint64_t kB2IV5 = 0x9b05688c2b3e6c1fULL;
constexpr uint64_t kB2IV6 = 0x1f83d9abfb41bd6bULL;
constexpr uint64_t kB2IV7 = 0x5be0cd19137e2179ULL;

// BLAKE2b compression F (RFC 7693 section 3.2).  t < 2^64 always here.
__device__ __forceinline__ void b2_compress(uint64_t h[8], const uint64_t m[16],
                                            uint64_t t, bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3];
  uint64_t v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = kB2IV0, v9 = kB2IV1, v10 = kB2IV2, v11 = kB2IV3;
  uint64_t v12 = kB2IV4 ^ t, v13 = kB2IV5;
  uint64_t v14 = last ? ~kB2IV6 : kB2IV6, v15 = kB2IV7;
  SQ_B2_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  SQ_B2_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3);
  SQ_B2_ROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4);
  SQ_B2_ROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8);
  SQ_B2_ROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13);
  SQ_B2_ROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9);
  SQ_B2_ROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11);
  SQ_B2_ROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10);
  SQ_B2_ROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5);
  SQ_B2_ROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0);
  SQ_B2_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  SQ_B2_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3);
  h[0] ^= v0 ^ v8;
  h[1] ^= v1 ^ v9;
  h[2] ^= v2 ^ v10;
  h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12;
  h[5] ^= v5 ^ v13;
  h[6] ^= v6 ^ v14;
  h[7] ^= v7 ^ v15;
}

// BLAKE2b-256 initial chaining value: IV ^ parameter block (digest 32, key 0,
// fanout 1, depth 1).
__device__ __host__ inline void b2_init256(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ULL ^ 0x01010020ULL;
  h[1] = 0xbb67ae8584caa73bULL;
  h[2] = 0x3c6ef372fe94f82bULL;
  h[3] = 0xa54ff53a5f1d36f1ULL;
  h[4] = 0x510e527fade682d1ULL;
  h[5] = 0x9b05688c2b3e6c1fULL;
  h[6] = 0x1f83d9abfb41bd6bULL;
  h[7] = 0x5be0cd19137e2179ULL;
}

// ---------------------------------------------------------------- SHA-256

__device__ __forceinline__ uint32_t s2_rotr(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

__device__ __forceinline__ void s2_compress(uint32_t st[8], const uint32_t m[16]) {
  constexpr uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1,
      0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3,
      0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
      0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
      0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
      0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
      0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
      0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
      0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = m[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    if (i >= 16) {
      const uint32_t x15 = w[(i - 15) & 15], x2 = w[(i - 2) & 15];
      const uint32_t s0 = s2_rotr(x15, 7) ^ s2_rotr(x15, 18) ^ (x15 >> 3);
      const uint32_t s1 = s2_rotr(x2, 17) ^ s2_rotr(x2, 19) ^ (x2 >> 10);
      w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
    }
    const uint32_t S1 = s2_rotr(e, 6) ^ s2_rotr(e, 11) ^ s2_rotr(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + K[i] + w[i & 15];
    const uint32_t S0 = s2_rotr(a, 2) ^ s2_rotr(a, 13) ^ s2_rotr(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
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

__device__ __host__ inline void s2_init(uint32_t st[8]) {
  st[0] = 0x6a09e667;
  st[1] = 0xbb67ae85;
  st[2] = 0x3c6ef372;
  st[3] = 0xa54ff53a;
  st[4] = 0x510e527f;
  st[5] = 0x9b05688c;
  st[6] = 0x1f83d9ab;
  st[7] = 0x5be0cd19;
}

// ---------------------------------------------------------------- ChaCha20

// RFC 8439 section 2.3 block function (20 rounds), one block per lane.
// Used as the device salt generator (SQOBFS_FLAG_DEVICE_SALT): it replaces
// the host RNG reads of salamander.go:60,83,98 (buf.WriteRandom) and
// xplus.go:67-69 (math/rand).  Rotations are v_alignbit_b32.
__device__ __forceinline__ uint32_t cc_rotl(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, 32 - n);
}
#define SQ_CC_QR(a, b, c, d)                  \
  a += b; d ^= a; d = cc_rotl(d, 16);         \
  c += d; b ^= c; b = cc_rotl(b, 12);         \
  a += b; d ^= a; d = cc_rotl(d, 8);          \
  c += d; b ^= c; b = cc_rotl(b, 7);

__device__ __forceinline__ void chacha20_block(const uint32_t (&key)[8], uint32_t counter,
                                               const uint32_t (&nonce)[3],
                                               uint32_t (&out)[16]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                     counter, nonce[0], nonce[1], nonce[2]};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = in[i];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    SQ_CC_QR(x[0], x[4], x[8], x[12])
    SQ_CC_QR(x[1], x[5], x[9], x[13])
    SQ_CC_QR(x[2], x[6], x[10], x[14])
    SQ_CC_QR(x[3], x[7], x[11], x[15])
    SQ_CC_QR(x[0], x[5], x[10], x[15])
    SQ_CC_QR(x[1], x[6], x[11], x[12])
    SQ_CC_QR(x[2], x[7], x[8], x[13])
    SQ_CC_QR(x[3], x[4], x[9], x[14])
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}
#undef SQ_CC_QR

}  // namespace sq
