/*
 * oracle.c -- CPU restatement of sing-quic's Salamander / XPlus obfuscation.
 * TEST INFRASTRUCTURE ONLY (see oracle.h for scope, citations, and why parity
 * with the Go reference is unpinned).  Plain C99 + pthreads, built by
 * oracle/Makefile into oracle/liboracle.so.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* BLAKE2b (RFC 7693 section 3)                                        */
/* ------------------------------------------------------------------ */

static const uint64_t b2_iv[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
    0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

/* RFC 7693 section 2.7: message word schedule, rounds 10 and 11 repeat 0 and 1 */
static const uint8_t b2_sigma[12][16] = {
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

static uint64_t rotr64(uint64_t x, unsigned n) {
  return (x >> n) | (x << (64 - n));
}

static uint64_t load64le(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

/* RFC 7693 section 3.1, the mixing function G */
#define B2_G(a, b, c, d, x, y)          \
  do {                                  \
    v[a] = v[a] + v[b] + (x);           \
    v[d] = rotr64(v[d] ^ v[a], 32);     \
    v[c] = v[c] + v[d];                 \
    v[b] = rotr64(v[b] ^ v[c], 24);     \
    v[a] = v[a] + v[b] + (y);           \
    v[d] = rotr64(v[d] ^ v[a], 16);     \
    v[c] = v[c] + v[d];                 \
    v[b] = rotr64(v[b] ^ v[c], 63);     \
  } while (0)

/* RFC 7693 section 3.2, compression function F */
static void b2_compress(uint64_t h[8], const uint8_t block[128], uint64_t t,
                        int last) {
  uint64_t v[16], m[16];
  for (int i = 0; i < 16; i++) m[i] = load64le(block + 8 * i);
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = b2_iv[i];
  }
  v[12] ^= t; /* low word of the 128-bit offset counter; high word stays 0 */
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t *s = b2_sigma[r];
    B2_G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    B2_G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    B2_G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    B2_G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    B2_G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    B2_G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    B2_G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    B2_G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

void or_blake2b(const uint8_t *in, size_t len, uint8_t *out, size_t outlen) {
  uint64_t h[8];
  uint8_t block[128];
  for (int i = 0; i < 8; i++) h[i] = b2_iv[i];
  /* parameter block: digest length, key length 0, fanout 1, depth 1 */
  h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
  size_t off = 0;
  /* every full block except the final one is compressed with last = 0 */
  while (len - off > 128) {
    b2_compress(h, in + off, (uint64_t)(off + 128), 0);
    off += 128;
  }
  memset(block, 0, sizeof block);
  memcpy(block, in + off, len - off);
  b2_compress(h, block, (uint64_t)len, 1);
  for (size_t i = 0; i < outlen; i++) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
}

void or_blake2b256(const uint8_t *in, size_t len, uint8_t out[32]) {
  or_blake2b(in, len, out, 32);
}

/* ------------------------------------------------------------------ */
/* SHA-256 (FIPS 180-4 section 6.2)                                    */
/* ------------------------------------------------------------------ */

static const uint32_t s2_k[64] = {
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

static uint32_t rotr32(uint32_t x, unsigned n) {
  return (x >> n) | (x << (32 - n));
}

static void s2_compress(uint32_t st[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
           ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5],
           g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + s2_k[i] + w[i];
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
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

void or_sha256(const uint8_t *in, size_t len, uint8_t out[32]) {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[128];
  size_t off = 0;
  while (len - off >= 64) {
    s2_compress(st, in + off);
    off += 64;
  }
  size_t rem = len - off;
  memset(blk, 0, sizeof blk);
  memcpy(blk, in + off, rem);
  blk[rem] = 0x80;
  size_t padlen = (rem + 1 + 8 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) blk[padlen - 1 - i] = (uint8_t)(bits >> (8 * i));
  s2_compress(st, blk);
  if (padlen == 128) s2_compress(st, blk + 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

/* ------------------------------------------------------------------ */
/* Key derivation: hash(psk || salt).  The reference builds this input  */
/* with append(password, salt...); here it is always a private copy     */
/* (SURVEY.md section 5 explains the aliasing hazard in the Go code).   */
/* ------------------------------------------------------------------ */

/* ---------------------------------------------------------------- ChaCha20
 * RFC 8439 section 2.3, restated byte-exactly (little-endian words).  The
 * device salt generator (SQOBFS_FLAG_DEVICE_SALT) replaces the host RNG of
 * salamander.go:60,83,98 (sing buf.WriteRandom) and xplus.go:67-69
 * (math/rand); this is its checker, pinned by RFC 8439 section 2.3.2 and by
 * OpenSSL's chacha20 keystream (tests/golden/chacha20.json). */
static uint32_t rotl32(uint32_t x, unsigned n) { return (x << n) | (x >> (32 - n)); }
static uint32_t load32le(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}
#define OR_QR(a, b, c, d)                   \
  do {                                      \
    a += b; d ^= a; d = rotl32(d, 16);      \
    c += d; b ^= c; b = rotl32(b, 12);      \
    a += b; d ^= a; d = rotl32(d, 8);       \
    c += d; b ^= c; b = rotl32(b, 7);       \
  } while (0)

void or_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                       uint8_t out[64]) {
  uint32_t in[16], x[16];
  in[0] = 0x61707865u; in[1] = 0x3320646eu; in[2] = 0x79622d32u; in[3] = 0x6b206574u;
  for (int i = 0; i < 8; i++) in[4 + i] = load32le(key + 4 * i);
  in[12] = counter;
  for (int i = 0; i < 3; i++) in[13 + i] = load32le(nonce + 4 * i);
  for (int i = 0; i < 16; i++) x[i] = in[i];
  for (int r = 0; r < 10; r++) {
    OR_QR(x[0], x[4], x[8], x[12]);
    OR_QR(x[1], x[5], x[9], x[13]);
    OR_QR(x[2], x[6], x[10], x[14]);
    OR_QR(x[3], x[7], x[11], x[15]);
    OR_QR(x[0], x[5], x[10], x[15]);
    OR_QR(x[1], x[6], x[11], x[12]);
    OR_QR(x[2], x[7], x[8], x[13]);
    OR_QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) {
    const uint32_t v = x[i] + in[i];
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(v >> (8 * k));
  }
}
#undef OR_QR

void or_chacha20_stream(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter0,
                        uint8_t *out, size_t len) {
  uint8_t blk[64];
  for (size_t pos = 0; pos < len; pos += 64) {
    or_chacha20_block(key, counter0 + (uint32_t)(pos / 64), nonce, blk);
    const size_t take = len - pos < 64 ? len - pos : 64;
    memcpy(out + pos, blk, take);
  }
}

void or_device_salts(const uint8_t key[32], uint64_t seq, uint32_t n, uint32_t S,
                     uint8_t *out) {
  uint8_t nonce[12] = {'s', 'q', 'o', 'b'};
  for (int k = 0; k < 8; k++) nonce[4 + k] = (uint8_t)(seq >> (8 * k));
  or_chacha20_stream(key, nonce, 0, out, (size_t)n * S);
}

/* ---------------------------------------------------------------- Poly1305
 * RFC 8439 section 2.5, restated with 130-bit arithmetic in 26-bit limbs
 * (the accumulator h, the clamped r; reduction modulo 2^130 - 5). */
void or_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]) {
  const uint32_t r0 = load32le(key + 0) & 0x3ffffff;
  const uint32_t r1 = (load32le(key + 3) >> 2) & 0x3ffff03;
  const uint32_t r2 = (load32le(key + 6) >> 4) & 0x3ffc0ff;
  const uint32_t r3 = (load32le(key + 9) >> 6) & 0x3f03fff;
  const uint32_t r4 = (load32le(key + 12) >> 8) & 0x00fffff;
  const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;
  while (len > 0) {
    uint8_t blk[17] = {0};
    const size_t take = len < 16 ? len : 16;
    memcpy(blk, msg, take);
    blk[take] = 1;  /* the 2^(8*take) bit */
    h0 += load32le(blk + 0) & 0x3ffffff;
    h1 += (load32le(blk + 3) >> 2) & 0x3ffffff;
    h2 += (load32le(blk + 6) >> 4) & 0x3ffffff;
    h3 += (load32le(blk + 9) >> 6) & 0x3ffffff;
    h4 += (load32le(blk + 12) >> 8) | ((uint32_t)blk[16] << 24);
    const uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 +
                        (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
    uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 +
                  (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
    uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 +
                  (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
    uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 +
                  (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
    uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 +
                  (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
    uint32_t c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff;
    d1 += c; c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff;
    d2 += c; c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff;
    d3 += c; c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff;
    d4 += c; c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff;
    h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
    h1 += c;
    msg += take;
    len -= take;
  }
  /* full carry, then h mod 2^130-5 (subtract p if h >= p) */
  uint32_t c = h1 >> 26; h1 &= 0x3ffffff;
  h2 += c; c = h2 >> 26; h2 &= 0x3ffffff;
  h3 += c; c = h3 >> 26; h3 &= 0x3ffffff;
  h4 += c; c = h4 >> 26; h4 &= 0x3ffffff;
  h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
  h1 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
  uint32_t g4 = h4 + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1;  /* all ones if h >= p */
  h0 = (h0 & ~mask) | (g0 & mask);
  h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask);
  h3 = (h3 & ~mask) | (g3 & mask);
  h4 = (h4 & ~mask) | (g4 & mask);
  /* h + s mod 2^128 */
  uint64_t f0 = ((h0) | (h1 << 26)) + (uint64_t)load32le(key + 16);
  uint64_t f1 = ((h1 >> 6) | (h2 << 20)) + (uint64_t)load32le(key + 20) + (f0 >> 32);
  uint64_t f2 = ((h2 >> 12) | (h3 << 14)) + (uint64_t)load32le(key + 24) + (f1 >> 32);
  uint64_t f3 = ((h3 >> 18) | (h4 << 8)) + (uint64_t)load32le(key + 28) + (f2 >> 32);
  const uint32_t w[4] = {(uint32_t)f0, (uint32_t)f1, (uint32_t)f2, (uint32_t)f3};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 4; k++) tag[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
}

/* RFC 8439 section 2.8: otk = block 0; ct = pt ^ keystream from counter 1;
 * mac_data = aad || pad16 || ct || pad16 || le64(aad_len) || le64(ct_len). */
void or_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                  size_t aad_len, const uint8_t *pt, size_t len, uint8_t *ct, uint8_t tag[16]) {
  uint8_t blk[64];
  or_chacha20_block(key, 0, nonce, blk);
  for (size_t pos = 0; pos < len; pos += 64) {
    uint8_t ks[64];
    or_chacha20_block(key, 1 + (uint32_t)(pos / 64), nonce, ks);
    for (size_t i = pos; i < len && i < pos + 64; i++) ct[i] = pt[i] ^ ks[i - pos];
  }
  const size_t pa = (aad_len + 15) / 16 * 16, pc = (len + 15) / 16 * 16;
  uint8_t *mac = (uint8_t *)calloc(pa + pc + 16, 1);
  memcpy(mac, aad, aad_len);
  memcpy(mac + pa, ct, len);
  for (int k = 0; k < 8; k++) {
    mac[pa + pc + k] = (uint8_t)((uint64_t)aad_len >> (8 * k));
    mac[pa + pc + 8 + k] = (uint8_t)((uint64_t)len >> (8 * k));
  }
  or_poly1305(blk, mac, pa + pc + 16, tag);
  free(mac);
}

/* ---- AES-128 (FIPS-197) and GCM (NIST SP 800-38D), for the
 * TLS_AES_128_GCM_SHA256 QUIC suite (RFC 9001 5.3, 5.4.3).  Byte-oriented
 * restatement: the S-box is computed from its definition (multiplicative
 * inverse in GF(2^8) mod x^8+x^4+x^3+x+1, then the affine map), GHASH
 * multiplies bit by bit (SP 800-38D Algorithm 1). */
static uint8_t aes_sbox[256];
static int aes_sbox_ready;

static uint8_t gf8_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}

static void aes_init_sbox(void) {
  if (aes_sbox_ready) return;
  for (int x = 0; x < 256; x++) {
    uint8_t inv = 0;  /* x^254 = x^-1, and 0 -> 0 */
    if (x) {
      uint8_t acc = 1, base = (uint8_t)x;
      for (int e = 254; e; e >>= 1) {
        if (e & 1) acc = gf8_mul(acc, base);
        base = gf8_mul(base, base);
      }
      inv = acc;
    }
    uint8_t b = inv, y = 0x63;
    for (int k = 0; k < 5; k++) y ^= (uint8_t)((b << k) | (b >> ((8 - k) & 7)));
    aes_sbox[x] = y;
  }
  aes_sbox_ready = 1;
}

uint8_t or_aes_sbox(uint8_t x) {
  aes_init_sbox();
  return aes_sbox[x];
}

/* FIPS-197 5.2: 11 round keys of 16 bytes */
void or_aes128_expand(const uint8_t key[16], uint8_t rk[176]) {
  aes_init_sbox();
  memcpy(rk, key, 16);
  uint8_t rcon = 1;
  for (int i = 4; i < 44; i++) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % 4 == 0) {
      const uint8_t t0 = t[0];
      t[0] = (uint8_t)(aes_sbox[t[1]] ^ rcon);
      t[1] = aes_sbox[t[2]];
      t[2] = aes_sbox[t[3]];
      t[3] = aes_sbox[t0];
      rcon = gf8_mul(rcon, 2);
    }
    for (int k = 0; k < 4; k++) rk[4 * i + k] = rk[4 * (i - 4) + k] ^ t[k];
  }
}

/* FIPS-197 5.1: state byte r + 4c = input byte r + 4c */
void or_aes128_encrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
  aes_init_sbox();
  uint8_t s[16];
  for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
  for (int round = 1; round <= 10; round++) {
    uint8_t t[16];
    for (int c = 0; c < 4; c++)      /* SubBytes + ShiftRows */
      for (int r = 0; r < 4; r++) t[r + 4 * c] = aes_sbox[s[r + 4 * ((c + r) & 3)]];
    if (round < 10) {                /* MixColumns */
      for (int c = 0; c < 4; c++) {
        const uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c] = gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3;
        s[4 * c + 1] = a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3;
        s[4 * c + 2] = a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3);
        s[4 * c + 3] = gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2);
      }
    } else {
      memcpy(s, t, 16);
    }
    for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
  }
  memcpy(out, s, 16);
}

/* SP 800-38D 6.3, Algorithm 1: X * Y in GF(2^128), bit 0 = MSB of byte 0 */
void or_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]) {
  uint8_t z[16] = {0}, v[16];
  memcpy(v, y, 16);
  for (int i = 0; i < 128; i++) {
    if ((x[i / 8] >> (7 - (i % 8))) & 1)
      for (int k = 0; k < 16; k++) z[k] ^= v[k];
    const int lsb = v[15] & 1;
    for (int k = 15; k > 0; k--) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
    v[0] >>= 1;
    if (lsb) v[0] ^= 0xe1;
  }
  memcpy(out, z, 16);
}

/* GHASH_H over aad (zero-padded) || ct (zero-padded) || be64(bits(aad)) ||
 * be64(bits(ct)) (SP 800-38D 7.1 step 5) */
static void gcm_ghash(const uint8_t h[16], const uint8_t *aad, size_t aad_len,
                      const uint8_t *ct, size_t len, uint8_t x[16]) {
  memset(x, 0, 16);
  const uint8_t *parts[2] = {aad, ct};
  const size_t lens[2] = {aad_len, len};
  for (int p = 0; p < 2; p++)
    for (size_t pos = 0; pos < lens[p]; pos += 16) {
      for (size_t k = 0; k < 16 && pos + k < lens[p]; k++) x[k] ^= parts[p][pos + k];
      or_gf128_mul(x, h, x);
    }
  uint8_t l[16];
  for (int k = 0; k < 8; k++) {
    l[7 - k] = (uint8_t)(((uint64_t)aad_len * 8) >> (8 * k));
    l[15 - k] = (uint8_t)(((uint64_t)len * 8) >> (8 * k));
  }
  for (int k = 0; k < 16; k++) x[k] ^= l[k];
  or_gf128_mul(x, h, x);
}

/* AES-128-GCM with a 96-bit nonce: J0 = nonce || be32(1), payload counter
 * blocks from be32(2), tag = E(K, J0) ^ GHASH (SP 800-38D 7.1).  ct may be
 * pt (in place).  Open: pass the ciphertext as pt with decrypt = 1; the tag
 * is then computed over the input. */
void or_gcm_crypt(const uint8_t key[16], const uint8_t nonce[12], const uint8_t *aad,
                  size_t aad_len, const uint8_t *in, size_t len, uint8_t *out, uint8_t tag[16],
                  int decrypt) {
  uint8_t rk[176], h[16] = {0}, j[16], ks[16], x[16];
  or_aes128_expand(key, rk);
  or_aes128_encrypt(rk, h, h);
  memcpy(j, nonce, 12);
  if (decrypt) gcm_ghash(h, aad, aad_len, in, len, x);
  for (size_t pos = 0; pos < len; pos += 16) {
    const uint32_t ctr = 2 + (uint32_t)(pos / 16);
    j[12] = (uint8_t)(ctr >> 24); j[13] = (uint8_t)(ctr >> 16);
    j[14] = (uint8_t)(ctr >> 8); j[15] = (uint8_t)ctr;
    or_aes128_encrypt(rk, j, ks);
    for (size_t k = 0; k < 16 && pos + k < len; k++) out[pos + k] = in[pos + k] ^ ks[k];
  }
  if (!decrypt) gcm_ghash(h, aad, aad_len, out, len, x);
  j[12] = j[13] = j[14] = 0;
  j[15] = 1;
  or_aes128_encrypt(rk, j, ks);
  for (int k = 0; k < 16; k++) tag[k] = x[k] ^ ks[k];
}

static void quic_nonce(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]) {
  memcpy(nonce, iv, 12);  /* RFC 9001 5.3: iv XOR left-padded big-endian pn */
  for (int k = 0; k < 8; k++) nonce[11 - k] ^= (uint8_t)(pn >> (8 * k));
}

/* RFC 9001 5.4.4: mask = ChaCha20(hp, counter = sample[0..4), nonce =
 * sample[4..16)) applied to 5 zero bytes; 5.4.3: mask = AES-ECB(hp, sample). */
static void quic_mask(int suite, const uint8_t *hp, const uint8_t sample[16], uint8_t mask[5]) {
  uint8_t blk[64];
  if (suite == OR_QUIC_AES128GCM) {
    uint8_t rk[176];
    or_aes128_expand(hp, rk);
    or_aes128_encrypt(rk, sample, blk);
  } else {
    or_chacha20_block(hp, load32le(sample), sample + 4, blk);
  }
  memcpy(mask, blk, 5);
}

/* The payload AEAD of either suite; open (decrypt = 1) MACs the input. */
static void quic_aead(int suite, const uint8_t *key, const uint8_t nonce[12], const uint8_t *aad,
                      size_t aad_len, const uint8_t *in, size_t len, uint8_t *out,
                      uint8_t tag[16], int decrypt) {
  if (suite == OR_QUIC_AES128GCM) {
    or_gcm_crypt(key, nonce, aad, aad_len, in, len, out, tag, decrypt);
    return;
  }
  uint8_t otk[64];
  or_chacha20_block(key, 0, nonce, otk);
  const size_t pa = (aad_len + 15) / 16 * 16, pc = (len + 15) / 16 * 16;
  uint8_t *mac = (uint8_t *)calloc(pa + pc + 16, 1);
  memcpy(mac, aad, aad_len);
  if (decrypt) memcpy(mac + pa, in, len);
  for (size_t pos = 0; pos < len; pos += 64) {
    uint8_t ks[64];
    or_chacha20_block(key, 1 + (uint32_t)(pos / 64), nonce, ks);
    for (size_t i = pos; i < len && i < pos + 64; i++) out[i] = in[i] ^ ks[i - pos];
  }
  if (!decrypt) memcpy(mac + pa, out, len);
  for (int k = 0; k < 8; k++) {
    mac[pa + pc + k] = (uint8_t)((uint64_t)aad_len >> (8 * k));
    mac[pa + pc + 8 + k] = (uint8_t)((uint64_t)len >> (8 * k));
  }
  or_poly1305(otk, mac, pa + pc + 16, tag);
  free(mac);
}

long or_quic_seal2(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                   uint64_t pn, const uint8_t *pkt, size_t len, size_t pn_offset, uint8_t *out) {
  if (len == 0) return -1;
  const size_t pn_len = (size_t)(pkt[0] & 3) + 1, hdr = pn_offset + pn_len;
  if (hdr > len || pn_offset + 4 + 16 > len + 16) return -1;
  uint8_t nonce[12];
  quic_nonce(iv, pn, nonce);
  uint8_t *tmp = (uint8_t *)malloc(len + 16);
  memcpy(tmp, pkt, hdr);
  quic_aead(suite, key, nonce, pkt, hdr, pkt + hdr, len - hdr, tmp + hdr, tmp + len, 0);
  uint8_t mask[5];
  quic_mask(suite, hp, tmp + pn_offset + 4, mask);
  tmp[0] ^= mask[0] & ((tmp[0] & 0x80) ? 0x0f : 0x1f);
  for (size_t i = 0; i < pn_len; i++) tmp[pn_offset + i] ^= mask[1 + i];
  memcpy(out, tmp, len + 16);
  free(tmp);
  return (long)(len + 16);
}

long or_quic_seal(const uint8_t key[32], const uint8_t iv[12], const uint8_t hp[32],
                  uint64_t pn, const uint8_t *pkt, size_t len, size_t pn_offset, uint8_t *out) {
  return or_quic_seal2(OR_QUIC_CHACHA20, key, iv, hp, pn, pkt, len, pn_offset, out);
}

/* RFC 9000 Appendix A.3 */
static uint64_t decode_pn(uint64_t largest, uint64_t truncated, unsigned nbits) {
  const uint64_t expected = largest + 1, win = 1ull << nbits, hwin = win / 2;
  const uint64_t mask = win - 1;
  const uint64_t cand = (expected & ~mask) | truncated;
  if (cand + hwin <= expected && cand < (1ull << 62) - win) return cand + win;
  if (cand > expected + hwin && cand >= win) return cand - win;
  return cand;
}

long or_quic_open2(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                   uint64_t largest_pn, const uint8_t *pkt, size_t len, size_t pn_offset,
                   uint8_t *out, uint64_t *pn_out) {
  if (len < 16 || pn_offset + 4 + 16 > len) return -1;
  uint8_t mask[5];
  quic_mask(suite, hp, pkt + pn_offset + 4, mask);
  uint8_t *tmp = (uint8_t *)malloc(len);
  memcpy(tmp, pkt, len);
  tmp[0] ^= mask[0] & ((tmp[0] & 0x80) ? 0x0f : 0x1f);
  const size_t pn_len = (size_t)(tmp[0] & 3) + 1, hdr = pn_offset + pn_len;
  uint64_t trunc = 0;
  for (size_t i = 0; i < pn_len; i++) {
    tmp[pn_offset + i] ^= mask[1 + i];
    trunc = (trunc << 8) | tmp[pn_offset + i];
  }
  if (hdr > len - 16) {
    free(tmp);
    return -1;
  }
  const uint64_t pn = decode_pn(largest_pn, trunc, (unsigned)(8 * pn_len));
  uint8_t nonce[12], tag[16];
  quic_nonce(iv, pn, nonce);
  const size_t clen = len - 16 - hdr;
  uint8_t *pt = (uint8_t *)malloc(clen ? clen : 1);
  quic_aead(suite, key, nonce, tmp, hdr, tmp + hdr, clen, pt, tag, 1);
  uint8_t diff = 0;
  for (int i = 0; i < 16; i++) diff |= tag[i] ^ tmp[len - 16 + i];
  memcpy(out, tmp, hdr);
  memcpy(out + hdr, pt, clen);
  free(pt);
  free(tmp);
  if (pn_out) *pn_out = pn;
  return diff ? -2 : (long)(len - 16);
}

long or_quic_open(const uint8_t key[32], const uint8_t iv[12], const uint8_t hp[32],
                  uint64_t largest_pn, const uint8_t *pkt, size_t len, size_t pn_offset,
                  uint8_t *out, uint64_t *pn_out) {
  return or_quic_open2(OR_QUIC_CHACHA20, key, iv, hp, largest_pn, pkt, len, pn_offset, out,
                       pn_out);
}

static void hash_psk_salt(int kind, const uint8_t *psk, size_t psk_len,
                          const uint8_t *salt, size_t salt_len,
                          uint8_t key[32]) {
  uint8_t small[256];
  uint8_t *buf = (psk_len + salt_len <= sizeof small)
                     ? small
                     : (uint8_t *)malloc(psk_len + salt_len);
  if (psk_len) memcpy(buf, psk, psk_len);
  memcpy(buf + psk_len, salt, salt_len);
  if (kind == OR_SALAMANDER)
    or_blake2b256(buf, psk_len + salt_len, key);
  else
    or_sha256(buf, psk_len + salt_len, key);
  if (buf != small) free(buf);
}

void or_salamander_key(const uint8_t *psk, size_t psk_len,
                       const uint8_t salt[8], uint8_t key[32]) {
  hash_psk_salt(OR_SALAMANDER, psk, psk_len, salt, OR_SALAMANDER_SALT, key);
}

void or_xplus_key(const uint8_t *psk, size_t psk_len, const uint8_t salt[16],
                  uint8_t key[32]) {
  hash_psk_salt(OR_XPLUS, psk, psk_len, salt, OR_XPLUS_SALT, key);
}

/* salamander.go:57-70 */
long or_salamander_write(const uint8_t *psk, size_t psk_len,
                         const uint8_t salt[8], const uint8_t *p, size_t len,
                         uint8_t *wire) {
  uint8_t key[32];
  memcpy(wire, salt, OR_SALAMANDER_SALT);           /* :60 WriteRandom(8) */
  or_salamander_key(psk, psk_len, salt, key);       /* :61 */
  for (size_t index = 0; index < len; index++)      /* :62-64 */
    wire[OR_SALAMANDER_SALT + index] = p[index] ^ key[index % 32];
  return (long)len;                                 /* :69 */
}

/* salamander.go:42-55 */
long or_salamander_read(const uint8_t *psk, size_t psk_len, uint8_t *p,
                        size_t n) {
  uint8_t key[32];
  if (n <= OR_SALAMANDER_SALT) return (long)n;      /* :47-49 */
  or_salamander_key(psk, psk_len, p, key);          /* :50 */
  for (size_t index = 0; index < n - OR_SALAMANDER_SALT; index++) /* :51-53 */
    p[index] = p[OR_SALAMANDER_SALT + index] ^ key[index % 32];
  return (long)(n - OR_SALAMANDER_SALT);            /* :54 */
}

/* salamander.go:81-93 */
long or_salamander_write_inplace(const uint8_t *psk, size_t psk_len,
                                 const uint8_t salt[8], uint8_t *p,
                                 size_t len) {
  uint8_t key[32];
  or_salamander_key(psk, psk_len, salt, key);       /* :84 */
  for (size_t i = 0; i < len; i++) p[i] ^= key[i % 32]; /* :85-87 */
  return (long)len;                                 /* :92 */
}

/* salamander.go:95-109, literally (line 104 included) */
int or_salamander_write_vectorised(const uint8_t *psk, size_t psk_len,
                                   const uint8_t salt[8], uint8_t **bufs,
                                   const size_t *lens, size_t nbufs) {
  uint8_t key[32];
  or_salamander_key(psk, psk_len, salt, key);       /* :99 */
  size_t bufferIndex = 0;                           /* :100 */
  for (size_t b = 0; b < nbufs; b++) {
    uint8_t *content = bufs[b];
    for (size_t index = 0; index < lens[b]; index++) {
      size_t ci = bufferIndex + index;              /* content[bufferIndex+index] */
      size_t ki = bufferIndex + index % 32;         /* key[bufferIndex+index%32] */
      if (ki >= 32) return OR_PANIC;                /* key is [32]byte */
      if (ci >= lens[b]) return OR_PANIC;           /* content slice bound */
      /* Go evaluates the range value c before the assignment */
      content[ci] = content[index] ^ key[ki];
    }
    bufferIndex += lens[b];                         /* :106 */
  }
  return 0;
}

/* xplus.go:62-75 */
long or_xplus_write(const uint8_t *psk, size_t psk_len,
                    const uint8_t salt[16], const uint8_t *p, size_t len,
                    uint8_t *wire) {
  uint8_t key[32];
  memcpy(wire, salt, OR_XPLUS_SALT);                /* :66-69 */
  or_xplus_key(psk, psk_len, salt, key);            /* :70 */
  for (size_t i = 0; i < len; i++)                  /* :71-73 */
    wire[OR_XPLUS_SALT + i] = p[i] ^ key[i % 32];
  return (long)(len + OR_XPLUS_SALT);               /* :74 returns inner n */
}

/* xplus.go:46-60 */
long or_xplus_read(const uint8_t *psk, size_t psk_len, uint8_t *p, size_t n,
                   size_t cap) {
  uint8_t key[32];
  if (n < OR_XPLUS_SALT) return 0;                  /* :50-52 */
  or_xplus_key(psk, psk_len, p, key);               /* :54 */
  for (size_t i = 0; i < cap - OR_XPLUS_SALT; i++)  /* :55-57 range p[16:] */
    p[i] = p[OR_XPLUS_SALT + i] ^ key[i % 32];
  return (long)(n - OR_XPLUS_SALT);                 /* :58 */
}

/* xplus.go:100-118 */
void or_xplus_write_vectorised(const uint8_t *psk, size_t psk_len,
                               const uint8_t salt[16], uint8_t **bufs,
                               const size_t *lens, size_t nbufs) {
  uint8_t key[32];
  or_xplus_key(psk, psk_len, salt, key);            /* :107 */
  size_t index = 0;
  for (size_t b = 0; b < nbufs; b++)
    for (size_t i = 0; i < lens[b]; i++) {          /* :110-114 */
      bufs[b][i] ^= key[index % 32];
      index++;
    }
}

/* ------------------------------------------------------------------ */
/* Batch restatement                                                    */
/* ------------------------------------------------------------------ */

typedef struct {
  int kind, dir;
  const or_psks *psks;
  const or_batch *b;
  uint32_t lo, hi;
  int err;
} or_job;

static void run_one(int kind, int dir, const or_psks *psks, const or_batch *b,
                    uint32_t i, uint8_t *scratch, size_t scratch_cap) {
  uint32_t pid = b->psk_id ? b->psk_id[i] : 0;
  const uint8_t *psk = psks->blob + psks->off[pid];
  size_t psk_len = psks->len[pid];
  const uint8_t *in = b->in + b->in_off[i];
  uint8_t *out = b->out + b->out_off[i];
  size_t n = b->in_len[i];
  size_t S = kind == OR_SALAMANDER ? OR_SALAMANDER_SALT : OR_XPLUS_SALT;
  (void)scratch_cap;
  if (dir == OR_OBFUSCATE) {
    const uint8_t *salt = b->salt + (size_t)i * S;
    if (kind == OR_SALAMANDER)
      or_salamander_write(psk, psk_len, salt, in, n, out);
    else
      or_xplus_write(psk, psk_len, salt, in, n, out);
    b->out_len[i] = (uint32_t)(n + S);
    return;
  }
  /* deobfuscate: the reference decodes in place in the read buffer; the
   * batch form copies the datagram to scratch, runs the in-place routine and
   * copies the valid result out. */
  size_t cap = (kind == OR_XPLUS && b->in_cap) ? b->in_cap[i] : n;
  memcpy(scratch, in, cap);
  long r;
  if (kind == OR_SALAMANDER) {
    r = or_salamander_read(psk, psk_len, scratch, n);
    memcpy(out, scratch, (size_t)r);
  } else {
    r = or_xplus_read(psk, psk_len, scratch, n, cap);
    if (n >= OR_XPLUS_SALT) memcpy(out, scratch, cap - OR_XPLUS_SALT);
  }
  b->out_len[i] = (uint32_t)r;
}

static void *run_shard(void *arg) {
  or_job *j = (or_job *)arg;
  size_t cap = 0;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    size_t c = (j->b->in_cap && j->kind == OR_XPLUS) ? j->b->in_cap[i]
                                                      : j->b->in_len[i];
    if (c > cap) cap = c;
  }
  uint8_t *scratch = (uint8_t *)malloc(cap + 1);
  if (!scratch) {
    j->err = -1;
    return NULL;
  }
  for (uint32_t i = j->lo; i < j->hi; i++)
    run_one(j->kind, j->dir, j->psks, j->b, i, scratch, cap);
  free(scratch);
  return NULL;
}

int or_batch_run(int kind, int dir, const or_psks *psks, const or_batch *b,
                 int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > b->n) nthreads = b->n ? (int)b->n : 1;
  or_job *jobs = (or_job *)calloc((size_t)nthreads, sizeof(or_job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  int err = 0;
  for (int t = 0; t < nthreads; t++) {
    jobs[t].kind = kind;
    jobs[t].dir = dir;
    jobs[t].psks = psks;
    jobs[t].b = b;
    jobs[t].lo = (uint32_t)((uint64_t)b->n * t / nthreads);
    jobs[t].hi = (uint32_t)((uint64_t)b->n * (t + 1) / nthreads);
  }
  if (nthreads == 1) {
    run_shard(&jobs[0]);
  } else {
    for (int t = 0; t < nthreads; t++)
      pthread_create(&th[t], NULL, run_shard, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  }
  for (int t = 0; t < nthreads; t++) err |= jobs[t].err;
  free(jobs);
  free(th);
  return err;
}

/* QUIC seal of a whole batch on nthreads host threads (single key): the
 * CPU timing leg of bench.py --quic. */
typedef struct {
  int suite;
  const uint8_t *key, *iv, *hp, *in;
  const uint64_t *in_off, *out_off, *pn;
  const uint32_t *in_len;
  const uint16_t *pn_offset;
  uint8_t *out;
  uint32_t lo, hi;
  long err;
} or_qjob;

static void *quic_shard(void *arg) {
  or_qjob *j = (or_qjob *)arg;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    const long r = or_quic_seal2(j->suite, j->key, j->iv, j->hp, j->pn[i],
                                 j->in + j->in_off[i], j->in_len[i], j->pn_offset[i],
                                 j->out + j->out_off[i]);
    if (r < 0) j->err = r;
  }
  return NULL;
}

int or_quic_seal_batch2(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                        const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                        const uint16_t *pn_offset, const uint64_t *pn, uint32_t n, uint8_t *out,
                        const uint64_t *out_off, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  or_qjob *jobs = (or_qjob *)calloc((size_t)nthreads, sizeof(or_qjob));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    or_qjob j = {suite, key, iv, hp, in, in_off, out_off, pn, in_len, pn_offset, out,
                 (uint32_t)((uint64_t)n * t / nthreads),
                 (uint32_t)((uint64_t)n * (t + 1) / nthreads), 0};
    jobs[t] = j;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, quic_shard, &jobs[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  int err = 0;
  for (int t = 0; t < nthreads; t++) err |= jobs[t].err != 0;
  free(jobs);
  free(th);
  return err ? -1 : 0;
}

int or_quic_seal_batch(const uint8_t key[32], const uint8_t iv[12], const uint8_t hp[32],
                       const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                       const uint16_t *pn_offset, const uint64_t *pn, uint32_t n, uint8_t *out,
                       const uint64_t *out_off, int nthreads) {
  return or_quic_seal_batch2(OR_QUIC_CHACHA20, key, iv, hp, in, in_off, in_len, pn_offset, pn,
                             n, out, out_off, nthreads);
}

uint64_t or_fnv64(const uint8_t *p, size_t n, uint64_t h) {
  if (!h) h = 0xcbf29ce484222325ULL;
  for (size_t i = 0; i < n; i++) {
    h ^= p[i];
    h *= 0x100000001b3ULL;
  }
  return h;
}
