// sq_quic_gcm.hip -- gfx950 QUIC packet protection, TLS_AES_128_GCM_SHA256
// (the suite every QUIC stack must implement).
//
// Replaces, for a whole ragged batch per launch, quic-go's per-packet
//   internal/handshake/aead.go              Seal / Open (AES-128-GCM)
//   internal/handshake/header_protector.go  aesHeaderProtector
// (quic-go v0.52.0-beta.1, go.mod:7; reached from the reference through
// quic.go:47-102; not in the reference tree).  The algorithms are FIPS-197
// (AES-128), NIST SP 800-38D (GCM with a 96-bit nonce: J0 = nonce || 1,
// payload counters from 2) and RFC 9001 sections 5.3 / 5.4.3 (nonce, AES
// header protection: mask = AES-ECB(hp, sample)).  The CPU checker is
// oracle/oracle.c (or_quic_seal2 / or_quic_open2), pinned by FIPS-197, the GCM
// specification's test cases, RFC 9001 A.3 and OpenSSL
// (tests/golden/quic_gcm.json).
//
// gfx950 has no carry-less multiply and no AES instructions, so both run as
// LDS table lookups, laid out for the LDS banking rules:
//   * AES rounds: T0 and T1 = rotl8 T0 (T2, T3 are 16-bit rotations of
//     them), 32 copies each, as 256 rows of 256 bytes (64 KiB).  Lane l
//     reads copy l & 31, so a ds_read_b32 (two 32-lane halves, bank = word
//     mod 32) is conflict-free whatever the state bytes are, and a lookup's
//     address is one v_perm of the state word.
//   * GHASH: multiplication by H uses per-position tables (32 nibble
//     positions x 16 entries x 16 B = 8 KiB): X * H is the XOR of 32
//     independent ds_read_b128, each in a 256-byte bank row (conflict-free).
//     Shoup's 4-bit tables of H^1 .. H^128 (32 KiB) let each chunk of the
//     cooperative pass multiply its partial GHASH by the power that places it
//     in the packet: GHASH is linear, so the packet's value is the XOR of
//     the chunk partials times H^m (ds_xor_b32 into the packet's record) --
//     no serial combine.
// Work decomposition, per wave of 16 packets (as the ChaCha20 kernel):
//   1. owner lane per packet: descriptor; for open, header protection and
//      the packet number; nonce; GHASH over the header (the AAD), times
//      H^(payload blocks);
//   2. all 64 lanes: the packets' 64-byte payload chunks as one flat space;
//      a lane runs 4 AES-CTR blocks, XORs, Horners its <= 4 ciphertext blocks
//      with H from 0, multiplies by H^m (m = payload blocks after the chunk),
//      XORs the result into the packet's accumulator, and stores realigned
//      output;
//   3. owner lane: the lengths block, E(K, J0), the tag; for seal, header
//      protection.
// Payloads above 2,048 B (chunk multipliers past H^128) are walked by their
// owner lane in phase 3 (plain Horner), so any length works.
// Single-key launches keep the round keys in the kernarg segment (scalar
// operands) and the GHASH tables in LDS.  Multi-key launches of a large
// batch first group the packets by key (a stable counting sort,
// gcm_group_*: a permutation of the packet indices and a table of steps of
// up to 12 units of one key); each workgroup then stages the key of its
// current step (IV and GHASH tables, 40 KiB) in LDS and runs the single-key
// code on it, its round keys read as scalars from the keyring entry.  Batches that are not grouped (few packets per key,
// more than 1,023 keys) read each packet's keyring entry from global
// memory.
#include <hip/hip_runtime.h>

#include "sq_bytes.h"
#include "sq_internal.h"
#include "sq_obfs_key.h"
#include "sq_quic.h"

namespace sq {

constexpr uint32_t kGBlock = 768;  // 12 waves: one block per CU (156 KB of LDS)
constexpr uint32_t kGWaves = kGBlock / kWave;
// Packets per wave (owner lanes).  32 with 12-wave workgroups (the LDS
// tables plus 32 records per wave fill 156 KB, 3 waves per SIMD) measured
// seal 3,246 -> 3,146 us and open 3,252 -> 3,056 us against 16 packets in
// 16-wave groups (4 waves per SIMD), three interleaved passes.
constexpr uint32_t kGPpw = 32;
static_assert(kGPpw <= 32, "chunk-list entries hold the packet in 5 bits (gcm_unit)");
constexpr uint32_t kGCoopMax = 16 * kGcmPow;   // 2048 B

// ---------------------------------------------------------------- AES-128

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

// readfirstlane of 32-bit values (the builtin returns int: without the
// cast a word >= 2^31 sign-extends when widened)
__device__ __forceinline__ uint32_t rfl32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
  return ((uint64_t)rfl32((uint32_t)(x >> 32)) << 32) | (uint64_t)rfl32((uint32_t)x);
}

// Where a launch's keys live (KM): 0 one key (round keys in the kernarg
// segment, GHASH tables in LDS), 1 per-packet keyring entries in global
// memory, 2 the workgroup's staged key (GHASH tables and IV in LDS, round
// keys read wave-uniform from its keyring entry).
// round key r (4 column words); KM 2 reads them wave-uniform into SGPRs, as
// the kernarg ones are
template <int KM>
__device__ __forceinline__ void round_key(const uint32_t *rk, int r, uint32_t (&k)[4]) {
  if (KM == 1) {
    const u32x4 v = gld<u32x4>((uint64_t)(rk + 4 * r));
    k[0] = v.x; k[1] = v.y; k[2] = v.z; k[3] = v.w;
  } else if (KM == 2) {
    // the staged key's entry in global memory, through the constant address
    // space at a wave-uniform address: scalar loads into SGPRs (read from
    // LDS they held VGPRs and made these kernels spill)
    typedef const __attribute__((address_space(4))) uint32_t *cptr;
    const cptr c = (cptr)(uintptr_t)uniform_u64((uint64_t)(uintptr_t)(rk + 4 * r));
    k[0] = c[0]; k[1] = c[1]; k[2] = c[2]; k[3] = c[3];
  } else {
    k[0] = rk[4 * r]; k[1] = rk[4 * r + 1]; k[2] = rk[4 * r + 2]; k[3] = rk[4 * r + 3];
  }
}

// The T-table image in LDS: 256 rows of 256 bytes; row x = 32 copies of
// T0[x] then 32 copies of T1[x] = rotl8 T0[x].  Lane l reads column l & 31,
// so a ds_read_b32 (bank = word mod 32 per 32-lane half) is conflict-free.
// The byte offset of (row = byte r of s, this lane's column) is one v_perm:
// byte 0 = the lane's column offset lo = 4 (l & 31), byte 1 = s.byte r.
__device__ __forceinline__ uint32_t trow(uint32_t s, uint32_t lo, int r) {
  return __builtin_amdgcn_perm(lo, s, 0x0C0C0004u | ((uint32_t)r << 8));
}
__device__ __forceinline__ uint32_t t0at(const uint32_t *tT, uint32_t a) {
  return *(const uint32_t *)((const char *)tT + a);
}
__device__ __forceinline__ uint32_t t1at(const uint32_t *tT, uint32_t a) {
  return *(const uint32_t *)((const char *)tT + a + 128);
}

// three-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96):
// the compiler emits two v_xor_b32 for a ^ b ^ c
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// FIPS-197 cipher on one block held as 4 little-endian column words.
// Round: column c = T0[s_c.b0] ^ T1[s_c+1.b1] ^ rotl16(T0[s_c+2.b2] ^
// T1[s_c+3.b3]) ^ rk (T2 = rotl16 T0, T3 = rotl16 T1; ShiftRows folded into
// the byte picks), computed as xor3(a0, a1, rotl16(xor3(a2, a3, rotr16 rk)))
// -- 3 VALU ops per column besides the 4 v_perm addresses; the key schedule
// holds rounds 1-9 already rotated (sq_api.hip gcm_key).  The last round
// takes the S-box byte (T0 byte 1, T1 bytes 2 and 3) instead.
// R0 > 1: s holds the state entering round R0 (aes_ctr_n).
template <int KM, int NB, int R0 = 1>
__device__ __forceinline__ void aes_encrypt_n(const uint32_t *rk, const uint32_t *tT, uint32_t lo,
                                              uint32_t (&s)[NB][4]) {
  uint32_t k[4];
  if (R0 == 1) {
    round_key<KM>(rk, 0, k);
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
      for (int c = 0; c < 4; c++) s[q][c] ^= k[c];
  }
#pragma unroll
  for (int r = R0; r < 10; r++) {
    uint32_t kr[4];  // (rotated by 16 in the key schedule)
    round_key<KM>(rk, r, kr);
    uint32_t t[NB][4];
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t a0 = t0at(tT, trow(s[q][c], lo, 0));
        const uint32_t a1 = t1at(tT, trow(s[q][(c + 1) & 3], lo, 1));
        const uint32_t a2 = t0at(tT, trow(s[q][(c + 2) & 3], lo, 2));
        const uint32_t a3 = t1at(tT, trow(s[q][(c + 3) & 3], lo, 3));
        t[q][c] = xor3(a0, a1, rotl(xor3(a2, a3, kr[c]), 16));
      }
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
      for (int c = 0; c < 4; c++) s[q][c] = t[q][c];
  }
  round_key<KM>(rk, 10, k);
  uint32_t t[NB][4];
#pragma unroll
  for (int q = 0; q < NB; q++)
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t a0 = t0at(tT, trow(s[q][c], lo, 0));
      const uint32_t a1 = t0at(tT, trow(s[q][(c + 1) & 3], lo, 1));
      const uint32_t a2 = t1at(tT, trow(s[q][(c + 2) & 3], lo, 2));
      const uint32_t a3 = t1at(tT, trow(s[q][(c + 3) & 3], lo, 3));
      // S-box bytes: T0 byte 1 (a0, a1), T1 bytes 2 and 3 (a2, a3), two v_perm
      // into complementary bytes, then one three-input XOR with the key
      t[q][c] = xor3(__builtin_amdgcn_perm(a1, a0, 0x0C0C0501u),
                     __builtin_amdgcn_perm(a3, a2, 0x07020C0Cu), k[c]);
    }
#pragma unroll
  for (int q = 0; q < NB; q++)
#pragma unroll
    for (int c = 0; c < 4; c++) s[q][c] = t[q][c];
}

// Counter blocks nonce || be32(c) with c < 256 (a cooperative chunk's
// blocks: c = 2 + block index <= 129) differ only in byte 15.  Round 1 then
// varies in one lookup (that byte, into column 0), round 2 in four (column
// 0's bytes, one into each column): the rest of both rounds is the same for
// every block of a packet.  aes_ctr_pre computes those parts once per chunk
// (27 lookups); aes_ctr_n then runs a block's rounds 1 and 2 in 5 lookups and
// 12 VALU instead of 32 and ~60, and rounds 3-10 as aes_encrypt_n.
struct CtrPre {
  uint32_t c0;     // round-1 column 0 without the counter byte's term
  uint32_t f[4];   // round-2 columns without column 0's terms
  uint32_t k15;    // round key 0, byte 15 (the counter byte's key byte)
};
template <int KM>
__device__ __forceinline__ void aes_ctr_pre(const uint32_t *rk, const uint32_t *tT, uint32_t lo,
                                            const uint32_t (&nonce)[3], CtrPre &P) {
  uint32_t k[4], kr[4];
  round_key<KM>(rk, 0, k);
  // round 0; word 3 = the counter's zero bytes 0..2 under the key (byte 3
  // varies: unused here)
  const uint32_t s[4] = {nonce[0] ^ k[0], nonce[1] ^ k[1], nonce[2] ^ k[2], k[3]};
  P.k15 = k[3] >> 24;
  round_key<KM>(rk, 1, kr);  // (rotated by 16)
  uint32_t c[4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t a0 = t0at(tT, trow(s[q], lo, 0));
    const uint32_t a1 = t1at(tT, trow(s[(q + 1) & 3], lo, 1));
    const uint32_t a2 = t0at(tT, trow(s[(q + 2) & 3], lo, 2));
    const uint32_t a3 = q == 0 ? 0u : t1at(tT, trow(s[(q + 3) & 3], lo, 3));
    c[q] = xor3(a0, a1, rotl(xor3(a2, a3, kr[q]), 16));
  }
  P.c0 = c[0];
  round_key<KM>(rk, 2, kr);
  // round 2 over {col0, c1, c2, c3}: column q reads col0's byte (4 - q) & 3
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t a0 = q == 0 ? 0u : t0at(tT, trow(c[q], lo, 0));
    const uint32_t a1 = q == 3 ? 0u : t1at(tT, trow(c[(q + 1) & 3], lo, 1));
    const uint32_t a2 = q == 2 ? 0u : t0at(tT, trow(c[(q + 2) & 3], lo, 2));
    const uint32_t a3 = q == 1 ? 0u : t1at(tT, trow(c[(q + 3) & 3], lo, 3));
    P.f[q] = xor3(a0, a1, rotl(xor3(a2, a3, kr[q]), 16));
  }
}
// keystream blocks for counters ctr[q] (< 256) under P's nonce and key
template <int KM, int NB>
__device__ __forceinline__ void aes_ctr_n(const uint32_t *rk, const uint32_t *tT, uint32_t lo,
                                          const CtrPre &P, const uint32_t (&ctr)[NB],
                                          uint32_t (&s)[NB][4]) {
#pragma unroll
  for (int q = 0; q < NB; q++) {
    // round 1: column 0 = c0 ^ T3[counter byte ^ key byte]
    const uint32_t x = (ctr[q] ^ P.k15) & 0xFFu;
    const uint32_t col0 = P.c0 ^ rotl(t1at(tT, __builtin_amdgcn_perm(lo, x, 0x0C0C0004u)), 16);
    // round 2: each column's one term from col0
    s[q][0] = P.f[0] ^ t0at(tT, trow(col0, lo, 0));
    s[q][1] = P.f[1] ^ rotl(t1at(tT, trow(col0, lo, 3)), 16);
    s[q][2] = P.f[2] ^ rotl(t0at(tT, trow(col0, lo, 2)), 16);
    s[q][3] = P.f[3] ^ t1at(tT, trow(col0, lo, 1));
  }
  aes_encrypt_n<KM, NB, 3>(rk, tT, lo, s);
}

template <int KM>
__device__ __forceinline__ void aes_encrypt(const uint32_t *rk, const uint32_t *tT, uint32_t lo,
                                            uint32_t (&s)[4]) {
  uint32_t b[1][4] = {{s[0], s[1], s[2], s[3]}};
  aes_encrypt_n<KM, 1>(rk, tT, lo, b);
#pragma unroll
  for (int c = 0; c < 4; c++) s[c] = b[0][c];
}

// ---------------------------------------------------------------- GHASH

// x <- x * H^k in GF(2^128) (SP 800-38D bit order), x as big-endian words
// (x[0] = bytes 0..3).  tab = the 16-entry 4-bit table of H^k; nibbles are
// consumed from the low end of the 128-bit integer, each step multiplying
// the accumulator by x^4 (shift right 4, fold the 4 bits shifted out back
// with the reduction polynomial).  Entry n of table k-1 is stored in slot
// n ^ sw, sw = (k-1) & 15: lanes multiplying by different powers then read
// different 16-byte slots of the bank row for the same nibble (no
// ds_read_b128 bank conflicts).
// One word (8 nibbles) at a time: its table reads depend only on x, so they
// are issued back to back (4 in flight); the shifts then run with the
// fold deferred to the end of the word -- the bits shifted out collect in z4
// (fold bits enter z0 at bit 21 or above and cannot reach z3's low nibble
// within 8 shifts), and fold(u) = u ^ u>>1 ^ u>>2 ^ u>>7 over z0:z1, the
// 4-bit fold (rem<<28 ^ rem<<27 ^ rem<<26 ^ rem<<21) applied to 32 bits at
// once.
template <bool GLOBAL>
__device__ __forceinline__ void gmul(uint32_t (&x)[4], const uint32_t *tab, uint32_t sw) {
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  uint32_t w = x[3], w2 = x[2], w1 = x[1], w0 = x[0];
  const char *t = (const char *)tab;
  const uint32_t sw16 = sw << 4;
  // one word per iteration, kept rolled (unrolled, the compiler hoists every
  // word's reads and spills)
#pragma unroll 1
  for (int i = 0; i < 4; i++) {
    const uint32_t w4 = w << 4;
    uint32_t z4 = 0;
#pragma unroll
    for (int h = 0; h < 8; h += 4) {  // (4 reads in flight: 8 made the kernels spill)
      u32x4 e[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int jj = h + j;
        const uint32_t off = ((((jj & 1) ? w : w4) >> (8 * (jj >> 1))) & 0xF0u) ^ sw16;
        if (GLOBAL) e[j] = gld<u32x4>((uint64_t)(t + off));
        else e[j] = *(const u32x4 *)(t + off);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (i | h | j) {
          z4 = __builtin_amdgcn_alignbit(z3, z4, 4);
          z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
          z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
          z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
          z0 >>= 4;
        }
        z0 ^= e[j].x; z1 ^= e[j].y; z2 ^= e[j].z; z3 ^= e[j].w;
      }
    }
    z0 = xor3(z0, xor3(z4, z4 >> 1, z4 >> 2), z4 >> 7);
    z1 ^= xor3(z4 << 31, z4 << 30, z4 << 25);
    w = w2;
    w2 = w1;
    w1 = w0;
  }
  x[0] = z0; x[1] = z1; x[2] = z2; x[3] = z3;
}

// x <- x * H with the position tables of H (pos: 32 nibble positions x 16
// entries x 16 B, one 256-byte bank row per position): the XOR of
// pos[j][nibble j of x] over the 32 nibbles (from the low end of the 128-bit
// integer) -- no shifts, no reduction steps.  The lookups do not depend on
// each other: they are issued 4 at a time back to back (16 VGPRs; 8 at a
// time made the kernels spill), then folded with three-input XORs.  In LDS
// (pos at a compile-time address below 56 KiB) the loop is unrolled: an
// address is the nibble times 16, the position an immediate offset; the
// rolled form (global tables) adds the word's base to every address.
// (Round 5's loop issued one read at a time and waited for it: 32 LDS round
// trips in a row per multiply.)
template <bool GLOBAL>
__device__ __forceinline__ void gmul_pos_rolled(uint32_t (&x)[4], const uint32_t *pos) {
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  uint32_t w = x[3], w2 = x[2], w1 = x[1], w0 = x[0];
  const char *base = (const char *)pos;
  // one word per iteration, kept rolled (unrolled, the compiler hoists every
  // word's reads and spills)
#pragma unroll 1
  for (int i = 0; i < 4; i++) {
    const uint32_t w4 = w << 4;
#pragma unroll
    for (int h = 0; h < 8; h += 4) {
      u32x4 e[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int jj = h + j;
        const uint32_t off = (((jj & 1) ? w : w4) >> (8 * (jj >> 1))) & 0xF0u;
        const char *p = base + 256 * jj + off;
        if (GLOBAL) e[j] = gld<u32x4>((uint64_t)p);
        else e[j] = *(const u32x4 *)p;
      }
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        z0 = xor3(z0, e[j].x, e[j + 1].x);
        z1 = xor3(z1, e[j].y, e[j + 1].y);
        z2 = xor3(z2, e[j].z, e[j + 1].z);
        z3 = xor3(z3, e[j].w, e[j + 1].w);
      }
    }
    base += 8 * 256;
    w = w2;
    w2 = w1;
    w1 = w0;
  }
  x[0] = z0; x[1] = z1; x[2] = z2; x[3] = z3;
}

template <bool GLOBAL>
__device__ __forceinline__ void gmul_pos(uint32_t (&x)[4], const uint32_t *pos) {
  if (GLOBAL) {  // (per-packet keys: the tables in global memory, 64-bit addresses)
    gmul_pos_rolled<true>(x, pos);
    return;
  }
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  const char *base = (const char *)pos;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint32_t w = x[3 - i];
#pragma unroll
    for (int h = 0; h < 8; h += 4) {
      // (an empty asm the next reads' addresses depend on, after the last
      // XORs: keeps the unrolled reads from being hoisted into 128 VGPRs)
      asm volatile("" : "+v"(w), "+v"(z0), "+v"(z1), "+v"(z2), "+v"(z3));
      const uint32_t w4 = w << 4;
      u32x4 e[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int jj = h + j;
        const uint32_t off = (((jj & 1) ? w : w4) >> (8 * (jj >> 1))) & 0xF0u;
        const char *p = base + 256 * (8 * i + jj) + off;
        e[j] = *(const u32x4 *)p;
      }
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        z0 = xor3(z0, e[j].x, e[j + 1].x);
        z1 = xor3(z1, e[j].y, e[j + 1].y);
        z2 = xor3(z2, e[j].z, e[j + 1].z);
        z3 = xor3(z3, e[j].w, e[j + 1].w);
      }
    }
  }
  x[0] = z0; x[1] = z1; x[2] = z2; x[3] = z3;
}

// y ^= 16 bytes held as little-endian words
__device__ __forceinline__ void ghash_absorb(uint32_t (&y)[4], const uint32_t (&m)[4]) {
#pragma unroll
  for (int w = 0; w < 4; w++) y[w] ^= __builtin_bswap32(m[w]);
}

// Key material of one packet: round keys, header-protection round keys,
// IV, and the GHASH tables (table k-1 = H^k).
template <int KM>
struct GKey {
  const uint32_t *rk, *hrk, *iv, *hpos, *htab;
  // x <- x * H^(4 k) (k = 1 .. kGcmPow4)
  __device__ __forceinline__ void mul_pow4(uint32_t (&x)[4], uint32_t k) const {
    gmul<KM == 1>(x, htab + 64 * (k - 1), (k - 1) & 15u);
  }
};

// ---------------------------------------------------------------- payload

// Payload bytes [0, nv) at src -> dst: CTR blocks ctr0, ctr0 + 1, ...; y
// absorbs every ciphertext block (y = (y ^ C) * H).  Full blocks move with
// one unaligned 16-byte load and store each (global accesses work at any
// byte address on gfx950 under the HSA runtime's unaligned mode: one
// global_load / global_store_dwordx4, no realignment funnels -- round 5's
// aligned loads and two barrel shifts per block cost ~45 VALU ops of the
// ~200 outside AES and GHASH); the last, partial block reads only the
// aligned blocks that hold valid bytes (load16: an unaligned read past the
// payload could cross into an unmapped page) and writes exactly its bytes
// (store16).  Blocks are loaded one pair ahead of the stores, so in place,
// or with the output a few bytes after the input (the fused layer's salt),
// a store never overwrites unread input.  first32 = ciphertext bytes 0..31
// (zero past nv).  OB (fused Salamander layer): output (seal) or input
// (open) bytes are also XORed with the packet's Salamander key; okr = the
// key rotated to the first byte at src / dst (block j uses half j & 1).
template <bool OPEN, int KM, bool OB>
__device__ __forceinline__ void gcm_run(const GKey<KM> &K, const uint32_t *tT, uint32_t tcol,
                                        const uint32_t (&nonce)[3], uint32_t ctr0, uint64_t src,
                                        uint64_t dst, uint32_t nv, uint32_t (&y)[4],
                                        uint32_t (&first32)[8], const uint32_t (&okr)[8]) {
#pragma unroll
  for (int j = 0; j < 8; j++) first32[j] = 0u;
  if (nv == 0) return;
  auto load_blk = [&](uint32_t i, uint32_t (&v)[4]) {
    const uint32_t o = 16 * i;
    if (o + 16 <= nv) {
      const u32x4 x = gld<u32x4_a1>(src + o);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else if (o < nv) {
      load16(src + o, src + nv, v);
    } else {
#pragma unroll
      for (int w = 0; w < 4; w++) v[w] = 0u;
    }
  };
  const uint32_t nchunk = (nv + 15) / 16;
  uint32_t in[2][4];
  load_blk(0, in[0]);
  load_blk(1, in[1]);
  // two counter blocks per iteration: their AES rounds interleave, so each
  // round has 32 independent T-table reads in flight instead of 16
  for (uint32_t j = 0; j < nchunk; j += 2) {
    uint32_t nx[2][4];
    load_blk(j + 2, nx[0]);  // (in flight during this pair's AES and GHASH)
    load_blk(j + 3, nx[1]);
    uint32_t s2[2][4] = {{nonce[0], nonce[1], nonce[2], __builtin_bswap32(ctr0 + j)},
                         {nonce[0], nonce[1], nonce[2], __builtin_bswap32(ctr0 + j + 1)}};
    aes_encrypt_n<KM, 2>(K.rk, tT, tcol, s2);
#pragma unroll
    for (int q = 0; q < 2; q++) {
      if (q == 1 && j + 1 >= nchunk) break;
      const int nb = (int)nv - 16 * (int)(j + q);  // valid bytes, >= 1
      uint32_t x[4], c[4], m[4];
#pragma unroll
      for (int w = 0; w < 4; w++) {
        m[w] = nb >= 16 ? 0xFFFFFFFFu : range_mask(0, nb, w);
        x[w] = in[q][w];
        if (OB && OPEN) x[w] ^= okr[4 * q + w] & m[w];  // (j is even)
        c[w] = (x[w] ^ s2[q][w]) & m[w];
      }
      const uint32_t(&g)[4] = OPEN ? x : c;
      ghash_absorb(y, g);
      gmul_pos<KM == 1>(y, K.hpos);
      if (j == 0) {
#pragma unroll
        for (int w = 0; w < 4; w++) first32[4 * q + w] = g[w];
      }
      uint32_t o[4];  // what goes to dst
#pragma unroll
      for (int w = 0; w < 4; w++) o[w] = (OB && !OPEN) ? c[w] ^ (okr[4 * q + w] & m[w]) : c[w];
      const uint64_t D = dst + 16ull * (j + q);
      if (nb >= 16) gst<u32x4_a1>(D, u32x4_a1{o[0], o[1], o[2], o[3]});
      else store16(D, o, (uint32_t)nb);
    }
#pragma unroll
    for (int w = 0; w < 4; w++) {
      in[0][w] = nx[0][w];
      in[1][w] = nx[1][w];
    }
  }
}

// The cooperative pass's share of a packet: nfull (1..4) FULL payload
// blocks, blocks blk0 .. blk0 + nfull - 1 at src / dst (the chunk's start).
// No partial block ever reaches it (a payload's last, partial block is its
// owner lane's, in phase 3), so the body is straight-line code: no masks,
// no byte-exact helpers, no divergent branches but the predicated loads and
// stores of a short chunk.  The blocks sit right-aligned in 4 slots (slot s
// holds block s - z, z = 4 - nfull; slots below z are zero and absorb
// nothing, so Horner over the 4 slots equals Horner over the nfull blocks).
// All four loads are issued before the first store (in place, and the fused
// open's output 8 bytes before its input, never overwrite unread input).
// y = the chunk's GHASH partial: Horner with H from y0 entering before its
// first block (the header's GHASH for a payload's first chunk, else zero).
// ct32 (seal): the packet's LDS words that receive ciphertext blocks 0 and 1
// (the first chunk may be short: block 1 can be the second chunk's).
// OB: as gcm_run (okr = the key rotated to the payload start).
template <bool OPEN, int KM, bool OB>
__device__ __forceinline__ void gcm_chunk(const GKey<KM> &K, const uint32_t *tT, uint32_t tcol,
                                          const uint32_t (&nonce)[3], uint32_t blk0,
                                          uint32_t nfull, uint64_t src, uint64_t dst,
                                          const uint32_t (&y0)[4], uint32_t (&y)[4],
                                          uint32_t *ct32, const uint32_t (&okr)[8]) {
  const uint32_t z = 4u - nfull;
  const uint64_t sz = src - 16ull * z, dz = dst - 16ull * z;  // slot s at sz + 16 s
  uint32_t in[4][4];
#pragma unroll
  for (int s = 0; s < 4; s++) {
    if (s == 3 || (uint32_t)s >= z) {
      const u32x4 v = gld<u32x4_a1>(sz + 16ull * s);
      in[s][0] = v.x; in[s][1] = v.y; in[s][2] = v.z; in[s][3] = v.w;
    } else {
#pragma unroll
      for (int w = 0; w < 4; w++) in[s][w] = 0u;
    }
  }
#pragma unroll
  for (int w = 0; w < 4; w++) y[w] = 0u;
  const uint32_t ctr = 2u + blk0 - z;  // slot 0's counter (live slots: <= 129)
  CtrPre P;
  aes_ctr_pre<KM>(K.rk, tT, tcol, nonce, P);
#pragma unroll
  for (int h = 0; h < 4; h += 2) {
    uint32_t s2[2][4];
    const uint32_t cq[2] = {ctr + h, ctr + h + 1};
    aes_ctr_n<KM, 2>(K.rk, tT, tcol, P, cq, s2);
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const int s = h + q;
      const uint32_t live = s == 3 || (uint32_t)s >= z ? 0xFFFFFFFFu : 0u;
      uint32_t x[4], c[4], kw[4];
#pragma unroll
      for (int w = 0; w < 4; w++) {
        // the half of the key of block blk0 + s - z: parity (blk0 + s + z) & 1
        kw[w] = OB ? bsel((blk0 + s + z) & 1u, okr[4 + w], okr[w]) : 0u;
        x[w] = (OB && OPEN) ? in[s][w] ^ kw[w] : in[s][w];
        c[w] = (x[w] ^ s2[q][w]) & live;
      }
      if (OPEN) {
#pragma unroll
        for (int w = 0; w < 4; w++) x[w] &= live;
      }
      const uint32_t(&g)[4] = OPEN ? x : c;
#pragma unroll
      for (int w = 0; w < 4; w++)  // (the Horner state entering block 0)
        y[w] = xor3(y[w], __builtin_bswap32(g[w]), (uint32_t)s == z ? y0[w] : 0u);
      gmul_pos<KM == 1>(y, K.hpos);
      if (s == 3 || (uint32_t)s >= z) {
        uint32_t o[4];
#pragma unroll
        for (int w = 0; w < 4; w++) o[w] = (OB && !OPEN) ? c[w] ^ kw[w] : c[w];
        gst<u32x4_a1>(dz + 16ull * s, u32x4_a1{o[0], o[1], o[2], o[3]});
        const uint32_t bi = blk0 + (uint32_t)s - z;  // the payload's block index
        if (!OPEN && ct32 && bi < 2u) *(u32x4 *)(ct32 + 4 * bi) = u32x4{c[0], c[1], c[2], c[3]};
      }
    }
  }
}

// 5 header-protection mask bytes (RFC 9001 5.4.3): AES-ECB(hp, sample)
template <int KM>
__device__ __forceinline__ void gcm_hp_mask(const GKey<KM> &K, const uint32_t *tT, uint32_t tcol,
                                            const uint32_t (&sample)[4], uint32_t &m0,
                                            uint32_t &m1) {
  uint32_t s[4] = {sample[0], sample[1], sample[2], sample[3]};
  aes_encrypt<KM>(K.hrk, tT, tcol, s);
  m0 = s[0];
  m1 = s[1] & 0xFFu;
}

// ---------------------------------------------------------------- kernel

struct alignas(16) GRec {
  uint64_t src, dst;   // payload start in the input / output
  uint32_t pl, pad0;   // payload bytes
  uint32_t np, kid;    // payload blocks (16 B); keyring index
  uint32_t nonce[3], pad;
  uint32_t x[4];       // GHASH accumulator (big-endian words), ds_xor target
  uint32_t yh[4];      // the header's GHASH (joins the first chunk's Horner)
  uint32_t ct32[8];    // ciphertext bytes 0..31 (the header-protection sample)
  uint32_t okr[8];     // fused Salamander layer: key rotated to the payload start
};

// STAGED: the workgroup's staged key (round keys, IV and GHASH tables in LDS)
template <bool MULTI, bool STAGED>
__device__ __forceinline__ GKey<MULTI ? 1 : (STAGED ? 2 : 0)> key_of(
    const QGParams &Q, uint32_t kid, const uint32_t *tP, const uint32_t *tH, const uint32_t *tK) {
  GKey<MULTI ? 1 : (STAGED ? 2 : 0)> K;
  if (MULTI) {
    const QuicGcmKeyDev *E = Q.keys + kid;
    K.rk = E->rk; K.hrk = E->hrk; K.iv = E->iv;
    K.hpos = &E->hpos[0][0][0]; K.htab = &E->htab[0][0][0];
  } else if (STAGED) {  // kid: the staged key
    K.rk = Q.keys[kid].rk; K.hrk = Q.keys[kid].hrk; K.iv = tK + 88;
    K.hpos = tP; K.htab = tH;
  } else {
    K.rk = Q.rk0; K.hrk = Q.hrk0;  // (kernarg: scalar loads)
    K.iv = Q.iv0; K.hpos = tP; K.htab = tH;
  }
  return K;
}

constexpr uint32_t kNoKey = 0xFFFFFFFFu;

// Copy keyring entry E's IV and GHASH tables into the block's LDS (every
// thread of the block takes part).
__device__ __forceinline__ void stage_key(const QuicGcmKeyDev *E, uint32_t *tP, uint32_t *tH,
                                          uint32_t *tK) {
  if (threadIdx.x < 3) tK[88 + threadIdx.x] = E->iv[threadIdx.x];  // (round keys: scalar loads)
  const uint32_t *src = &E->hpos[0][0][0];  // hpos then htab, contiguous
  for (uint32_t i = threadIdx.x; i < (32 + kGcmPow4) * 16; i += kGBlock) {
    const u32x4 v = gld<u32x4>((uint64_t)(src + 4 * i));
    if (i < 32 * 16) *(u32x4 *)(tP + 4 * i) = v;
    else *(u32x4 *)(tH + 4 * (i - 32 * 16)) = v;
  }
}

// One unit (up to kGPpw packets) of a wave: the three phases.  recs = the
// wave's records.  STAGED (with MULTI false): every packet of the unit uses
// the workgroup's staged key.
template <bool OPEN, bool MULTI, bool OB, bool STAGED>
__device__ __forceinline__ void gcm_unit(const QGParams &Q, uint64_t base, uint32_t cnt,
                                         uint32_t skid, uint32_t lane,
                                         const uint32_t *tT, uint32_t tcol, const uint32_t *tP,
                                         const uint32_t *tH, const uint32_t *tK, GRec *recs,
                                         uint16_t *clist) {
  constexpr int KM = MULTI ? 1 : (STAGED ? 2 : 0);
  // the unit's packets: positions [base, base + cnt) (grouped batches: of
  // the key order)
  const uint64_t i64 = base + lane;
  const bool owner = lane < kGPpw && lane < cnt;
  const uint32_t p = owner && Q.perm ? Q.perm[i64] : (uint32_t)i64;

  // ---- 1. owner lanes
  bool live = owner;
  uint64_t pn_dec = 0;  // open: decoded packet number (0 if rejected)
  uint32_t status = 0, len = 0, pno = 0, first = 0, pn_len = 0, hdr = 0, pl = 0,
           kid = STAGED ? skid : 0u;
  uint64_t src = 0, dst = 0;
  uint32_t nonce[3] = {0u, 0u, 0u}, rtag[4] = {0u, 0u, 0u, 0u}, y[4] = {0u, 0u, 0u, 0u};
  uint32_t hd[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, pnw = 0;  // packet bytes 0..31; seal: pn bytes
  // fused Salamander layer (OB): wire = salt8 || QUIC packet ^ okey
  uint64_t wire = 0;
  uint32_t okey[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, osalt[4] = {0u, 0u, 0u, 0u};
  if (live && MULTI) {
    kid = Q.key_id[p];
    if (kid >= Q.n_keys) {
      status = kQEKey;
      live = false;
      kid = 0;
      if (OPEN && Q.pn_out) Q.pn_out[p] = 0;  // rejected: pn_out 0 (as below)
    }
  }
  const GKey<KM> K = key_of<MULTI, STAGED>(Q, kid, tP, tH, tK);
  if (live) {
    src = (uint64_t)Q.in + Q.in_off[p];
    dst = (uint64_t)Q.out + Q.out_off[p];
    len = Q.in_len[p];
    pno = Q.pn_offset[p];
    uint64_t pn = Q.pn[p];
    uint32_t pnb[4] = {0u, 0u, 0u, 0u};
    if (OB) {
      if (!OPEN) {  // wire = salt || protected packet ^ key
        wire = dst;
        dst = wire + kSalamanderSalt;
        const uint32_t *sp = reinterpret_cast<const uint32_t *>(Q.osalt + 8ull * p);
        osalt[0] = sp[0];
        osalt[1] = sp[1];
      } else if (len >= (uint32_t)kSalamanderSalt && len <= kQMaxPacket) {
        wire = src;  // salt = the first 8 wire bytes (salamander.go:50)
        load16(src, src + kSalamanderSalt, osalt);
        src += kSalamanderSalt;
        len -= kSalamanderSalt;
      } else {
        len = 0;  // too short for a salt: rejected below
      }
      salamander_key(&Q.opsk, osalt, okey);
    }
    // packet byte k (de-obfuscated when the fused layer is on)
    auto hb = [&](uint32_t k) -> uint32_t {
      const uint32_t b = head_byte(hd, src, k);
      return (OB && OPEN && k >= 32) ? b ^ byte32(okey, k & 31) : b;
    };
    if (!OPEN) {
      if (len) load_head32(src, len, hd);
      first = hd[0] & 0xFFu;
      pn_len = (first & 3) + 1;
      hdr = pno + pn_len;
      if (len == 0 || len > kQMaxPacket || hdr > len || pno + 4 > len) {
        live = false;
      } else {
        pl = len - hdr;
        for (uint32_t i = 0; i < pn_len; i++) pnw |= hb(pno + i) << (8 * i);
      }
    } else if (len < 16 || len > kQMaxPacket || pno + 4 + 16 > len) {
      live = false;
    } else {
      uint32_t sample[4], m0, m1;
      load16(src + pno + 4, src + len, sample);
      load16(src + len - 16, src + len, rtag);  // before any in-place write
      load_head32(src, len, hd);
      if (OB) {  // de-obfuscate what was read: key byte of QUIC offset k is okey[k % 32]
        uint32_t k4[4];
        keywin(okey, (pno + 4) & 31, k4);
#pragma unroll
        for (int w = 0; w < 4; w++) sample[w] ^= k4[w];
        keywin(okey, (len - 16) & 31, k4);
#pragma unroll
        for (int w = 0; w < 4; w++) rtag[w] ^= k4[w];
        keywin(okey, 0, k4);
#pragma unroll
        for (int w = 0; w < 4; w++) hd[w] ^= k4[w];
        keywin(okey, 16, k4);
#pragma unroll
        for (int w = 0; w < 4; w++) hd[4 + w] ^= k4[w];
      }
      gcm_hp_mask<KM>(K, tT, tcol, sample, m0, m1);
      const uint32_t pfirst = hd[0] & 0xFFu;
      first = pfirst ^ (m0 & ((pfirst & 0x80) ? 0x0Fu : 0x1Fu));
      pn_len = (first & 3) + 1;
      hdr = pno + pn_len;
      if (hdr > len - 16) {
        live = false;
      } else {
        uint64_t trunc = 0;
        for (uint32_t i = 0; i < pn_len; i++) {
          pnb[i] = hb(pno + i) ^ mask_byte(m0, m1, 1 + i);
          trunc = (trunc << 8) | pnb[i];
        }
        pn = decode_pn(pn, trunc, 8 * pn_len);
        pn_dec = pn;
        pl = len - 16 - hdr;
      }
    }
    if (!live) status = kQEShort;
  // every owner lane writes its pn_out (0 when the packet was rejected)
  if (OPEN && owner && Q.pn_out) Q.pn_out[p] = pn_dec;
    if (live) {
      const uint32_t iv[3] = {K.iv[0], K.iv[1], K.iv[2]};
      quic_nonce_iv(iv, pn, nonce);
      // AAD = the unprotected header; seal copies it unchanged (protection
      // is applied in phase 3), open writes the unprotected header
      for (uint32_t q = 0; q < hdr; q += 16) {
        uint32_t w[4];
        head_block(hd, src, q, hdr, w);
        if (OB && OPEN && q >= 32) {
          uint32_t k4[4];
          keywin(okey, q & 31, k4);
#pragma unroll
          for (int j = 0; j < 4; j++) w[j] ^= k4[j] & range_mask(0, (int)(hdr - q), j);
        }
        if (OPEN) {
          if (q == 0) set_byte(w, 0, first);
          for (uint32_t i = 0; i < pn_len; i++) {
            const uint32_t pos = pno + i;
            if (pos >= q && pos < q + 16) set_byte(w, pos - q, pnb[i]);
          }
        }
        ghash_absorb(y, w);
        gmul_pos<MULTI>(y, K.hpos);
        if (OB && !OPEN) {  // the wire carries the (still unprotected) header ^ key
          uint32_t k4[4];
          keywin(okey, q & 31, k4);
#pragma unroll
          for (int j = 0; j < 4; j++) w[j] ^= k4[j];
        }
        if (OPEN || OB || dst != src) store16(dst + q, w, hdr - q < 16 ? hdr - q : 16);
      }
    }
  }
  const bool coop = live && pl <= kGCoopMax;
  const uint32_t np = (pl + 15) / 16;
  // chunks of the cooperative pass: the full blocks, 4 per chunk, aligned to
  // the last full one (the first chunk may be short; the last, partial block
  // is the owner's, phase 3).  The header's GHASH enters the first chunk's
  // Horner, so every chunk's partial is placed by a power of H^4.
  const uint32_t nblk = coop ? (pl / 16 + 3) / 4 : 0u;
  // The unit's chunks in k-major order (k = chunks from the payload's end):
  // entry f of clist = packet | k << 5 -- every packet's last chunk, then
  // every packet's second last, ... (phase 2 walks the list from its end).
  // The lanes of a step then mostly
  // share k, so their multiplies by H^4k read ONE Shoup table (a lane group
  // reading different tables met in the same banks: ~15 % of the LDS's
  // cycles were conflicts), and their accumulations go to different packets.
  uint32_t T = 0;  // (wave-uniform)
  for (uint32_t k = 0;; k++) {
    const uint64_t M = __ballot(nblk > k);  // (owner lanes only: bits 0..31)
    if (!M) break;
    if (nblk > k)
      clist[T + __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u)] = (uint16_t)(lane | (k << 5));
    T += (uint32_t)__popcll(M);
  }
  if (lane < kGPpw) {
    GRec &R = recs[lane];
    R.src = src + hdr;
    R.dst = dst + hdr;
    R.pl = pl;
    R.np = np;
    R.kid = kid;
#pragma unroll
    for (int i = 0; i < 3; i++) R.nonce[i] = nonce[i];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      R.x[i] = coop && nblk == 0 ? y[i] : 0u;
      R.yh[i] = y[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) R.ct32[i] = 0u;
    if (OB) {
      uint32_t k4[4];
      keywin(okey, hdr & 31, k4);
#pragma unroll
      for (int i = 0; i < 4; i++) R.okr[i] = k4[i];
      keywin(okey, (hdr + 16) & 31, k4);
#pragma unroll
      for (int i = 0; i < 4; i++) R.okr[4 + i] = k4[i];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- 2. cooperative payload pass over the chunk list
  for (uint32_t base = 0; base < T; base += kWave) {
    const uint32_t f = base + lane;
    if (f < T) {
      // (read from the end: a packet's chunks run in address order -- the
      // fused open writes its output 8 bytes before its input, so a chunk
      // must never run after the one behind it)
      const uint32_t e = clist[T - 1 - f], k = e >> 5;
      GRec &R = recs[e & 31u];
      const GKey<KM> KB = key_of<MULTI, STAGED>(Q, R.kid, tP, tH, tK);
      // chunk k from the end: full blocks [end - nfull, end), end = npf - 4 k
      const uint32_t npf = R.pl / 16, b = (npf + 3) / 4 - 1 - k;
      const uint32_t end = npf - 4 * k, nfull = end < 4 ? end : 4u;
      const uint32_t rn[3] = {R.nonce[0], R.nonce[1], R.nonce[2]};
      uint32_t yb[4], rokr[8], y0[4];
#pragma unroll
      for (int i = 0; i < 8; i++) rokr[i] = OB ? R.okr[i] : 0u;
#pragma unroll
      for (int i = 0; i < 4; i++) y0[i] = b == 0 ? R.yh[i] : 0u;
      gcm_chunk<OPEN, KM, OB>(KB, tT, tcol, rn, end - nfull, nfull,
                              R.src + 16ull * (end - nfull), R.dst + 16ull * (end - nfull), y0,
                              yb, R.ct32, rokr);
      if (k) KB.mul_pow4(yb, k);  // 4 k full blocks follow
#pragma unroll
      for (int i = 0; i < 4; i++) atomicXor(&R.x[i], yb[i]);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- 3. owner lanes: lengths block, tag, header protection
  if (!owner) return;
  if (!live) {
    Q.out_len[p] = status;
    return;
  }
  uint32_t ct32[8];
  if (coop) {
#pragma unroll
    for (int i = 0; i < 4; i++) y[i] = recs[lane].x[i];
#pragma unroll
    for (int i = 0; i < 8; i++) ct32[i] = recs[lane].ct32[i];
    const uint32_t nb = pl & 15u;
    if (nb) {  // the payload's last, partial block
      const uint32_t k = pl / 16;
      const uint64_t ps = src + hdr + 16ull * k;
      uint32_t x[4], c[4], ks[4] = {nonce[0], nonce[1], nonce[2], __builtin_bswap32(2u + k)};
      load16(ps, src + hdr + pl, x);
      aes_encrypt<KM>(K.rk, tT, tcol, ks);
      uint32_t kw[4];
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const uint32_t m = range_mask(0, (int)nb, w);
        kw[w] = OB ? recs[lane].okr[4 * (k & 1) + w] & m : 0u;
        if (OB && OPEN) x[w] ^= kw[w];
        c[w] = (x[w] ^ ks[w]) & m;
      }
      ghash_absorb(y, OPEN ? x : c);  // (the chunks' sum is placed up to the
      gmul_pos<MULTI>(y, K.hpos);      // last full block: times H once more)
      uint32_t o[4];
#pragma unroll
      for (int w = 0; w < 4; w++) o[w] = (OB && !OPEN) ? c[w] ^ kw[w] : c[w];
      store16(dst + hdr + 16ull * k, o, nb);
      if (!OPEN && k < 2) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
          if (k == 0) ct32[w] = c[w];
          else ct32[4 + w] = c[w];
        }
      }
    }
  } else {
    uint32_t rokr[8];
#pragma unroll
    for (int i = 0; i < 8; i++) rokr[i] = OB ? recs[lane].okr[i] : 0u;
    gcm_run<OPEN, KM, OB>(K, tT, tcol, nonce, 2, src + hdr, dst + hdr, pl, y, ct32, rokr);
  }
  // lengths block: be64(8 * hdr) || be64(8 * pl)
  y[1] ^= 8 * hdr;
  y[2] ^= pl >> 29;
  y[3] ^= 8 * pl;
  gmul_pos<MULTI>(y, K.hpos);
  uint32_t tag[4] = {nonce[0], nonce[1], nonce[2], __builtin_bswap32(1u)};
  aes_encrypt<KM>(K.rk, tT, tcol, tag);  // E(K, J0)
#pragma unroll
  for (int w = 0; w < 4; w++) tag[w] ^= __builtin_bswap32(y[w]);
  if (OPEN) {
    const bool ok = ((tag[0] ^ rtag[0]) | (tag[1] ^ rtag[1]) | (tag[2] ^ rtag[2]) |
                     (tag[3] ^ rtag[3])) == 0;
    Q.out_len[p] = ok ? len - 16 : kQEAuth;
    return;
  }
  if (OB) {
    uint32_t k4[4], t4[4];
    keywin(okey, len & 31, k4);
#pragma unroll
    for (int w = 0; w < 4; w++) t4[w] = tag[w] ^ k4[w];
    store16(dst + len, t4, 16);
    store16(wire, osalt, kSalamanderSalt);
  } else {
    store16(dst + len, tag, 16);
  }
  // header protection: sample = (ciphertext || tag)[4 - pn_len ..][0..16)
  const uint32_t so = 4 - pn_len;
  uint32_t sample[4];
  if (pl >= so + 16) {
#pragma unroll
    for (int j = 0; j < 4; j++) sample[j] = __builtin_amdgcn_alignbyte(ct32[j + 1], ct32[j], so);
  } else {  // short payload: the sample reaches into the tag
    const uint32_t t8[8] = {tag[0], tag[1], tag[2], tag[3], 0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 4; j++) sample[j] = 0u;
    for (uint32_t i = 0; i < 16; i++) {
      const uint32_t k = so + i;
      const uint32_t bb = k < pl ? byte32(ct32, k) : byte32(t8, k - pl);
      sample[i >> 2] |= bb << (8 * (i & 3));
    }
  }
  uint32_t m0, m1;
  gcm_hp_mask<KM>(K, tT, tcol, sample, m0, m1);
  const uint32_t kb0 = OB ? okey[0] & 0xFFu : 0u;
  gst<uint8_t>(dst, (uint8_t)(first ^ kb0 ^ (m0 & ((first & 0x80) ? 0x0Fu : 0x1Fu))));
  for (uint32_t i = 0; i < pn_len; i++) {
    const uint32_t bb = (pnw >> (8 * i)) & 0xFFu;
    const uint32_t kb = OB ? byte32(okey, (pno + i) & 31) : 0u;
    gst<uint8_t>(dst + pno + i, (uint8_t)(bb ^ kb ^ mask_byte(m0, m1, 1 + i)));
  }
  Q.out_len[p] = len + 16 + (OB ? kSalamanderSalt : 0u);
}

// The kernels' LDS, one image laid out by hand (the compiler's placement of
// separate arrays put the position tables past 64 KiB): the GHASH position
// tables of H at address 0 (8 KiB; a lookup's position is its immediate
// offset), the AES T-table image (64 KiB; a lookup's row and column come
// from one v_perm, the image's base is the immediate), the power tables
// (32 KiB), the staged key words (TK), then the waves' records.  TABLES
// false (per-packet keys from global memory): no position or power tables.
constexpr uint32_t kGList = kGPpw * kGcmPow4;  // chunk-list entries per wave
template <bool TABLES, uint32_t TK>
constexpr uint32_t kLdsWords = (TABLES ? 32 * 64 + kGcmPow4 * 64 : 0u) + 256 * 64 +
                               (TK + 3) / 4 * 4 + (uint32_t)sizeof(GRec) * kGWaves * kGPpw / 4 +
                               kGWaves * kGList / 2;
template <bool TABLES, uint32_t TK>
__device__ __forceinline__ void gcm_lds(uint32_t *lds, uint32_t *&tP, uint32_t *&tT, uint32_t *&tH,
                                        uint32_t *&tK, GRec (*&recs)[kGPpw],
                                        uint16_t (*&clists)[kGList]) {
  tP = lds;
  tT = lds + (TABLES ? 32 * 64 : 0);
  tH = tT + 256 * 64;
  tK = tH + (TABLES ? kGcmPow4 * 64 : 0);
  recs = reinterpret_cast<GRec(*)[kGPpw]>(tK + (TK + 3) / 4 * 4);
  clists = reinterpret_cast<uint16_t(*)[kGList]>(recs + kGWaves);
}

// The T-table image (every launch) and, single key, the key's GHASH tables,
// into LDS (single-key round keys stay in the kernarg segment: staged in LDS
// they measured 17 % slower, the keys then occupying VGPRs).
template <bool MULTI>
__device__ __forceinline__ void stage_common(const QGParams &Q, uint32_t *tT, uint32_t *tP,
                                             uint32_t *tH, uint32_t *tK) {
  for (uint32_t i = threadIdx.x; i < 256 * 64; i += kGBlock) {
    const uint32_t v = Q.t0[i >> 6];
    tT[i] = (i & 32) ? rotl(v, 8) : v;
  }
  if (!MULTI) {
    const uint32_t *src = &Q.keys[0].hpos[0][0][0];  // hpos then htab, contiguous
    for (uint32_t i = threadIdx.x; i < (32 + kGcmPow4) * 16; i += kGBlock) {
      const u32x4 v = gld<u32x4>((uint64_t)(src + 4 * i));
      if (i < 32 * 16) *(u32x4 *)(tP + 4 * i) = v;
      else *(u32x4 *)(tH + 4 * (i - 32 * 16)) = v;
    }
  }
}

// One key (MULTI false) or per-packet keys from the keyring in global memory
// (MULTI true, batches that are not grouped).
template <bool OPEN, bool MULTI, bool OB>
__global__ __launch_bounds__(kGBlock) void quic_gcm_kernel(const QGParams Q) {
  // one LDS image laid out by hand (gcm_lds): the GHASH position tables at
  // address 0, so a lookup's position is its immediate offset (< 64 KiB)
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords<!MULTI, 4>];
  uint32_t *tP, *tT, *tH, *tK;
  GRec(*recs)[kGPpw];
  uint16_t(*clists)[kGList];
  gcm_lds<!MULTI, 4>(lds, tP, tT, tH, tK, recs, clists);
  const uint64_t units = ((uint64_t)Q.n + kGPpw - 1) / kGPpw;
  stage_common<MULTI>(Q, tT, tP, tH, tK);
  __syncthreads();
  const uint32_t lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint32_t tcol = 4 * (lane & 31);  // this lane's T-table column (byte offset)
  const uint64_t stride = (uint64_t)gridDim.x * kGWaves;
  for (uint64_t u = (uint64_t)blockIdx.x * kGWaves + wv; u < units; u += stride) {
    const uint64_t base = u * kGPpw;
    const uint32_t cnt = Q.n - base < kGPpw ? (uint32_t)(Q.n - base) : kGPpw;
    gcm_unit<OPEN, MULTI, OB, false>(Q, base, cnt, 0u, lane, tT, tcol, tP, tH, tK, recs[wv],
                                     clists[wv]);
  }
}

// Grouped multi-key batches (Q.perm, Q.gmeta): the work is a list of steps,
// each up to kGWaves units of ONE key (a key's units in order, kGWaves per
// step; its last step partly idle).  The workgroups stride over the steps
// and stage a step's key in LDS (IV, GHASH tables) when it
// changes (block-uniform: the staging barriers); every wave then runs the
// single-key code on its unit.  Invalid key ids were rejected by the
// grouping and take no step.  (Round-4 measurements, 1M packets, 16 keys,
// one process: steps that could straddle a key boundary, with the straddling
// units deferred to a per-packet launch, ran that launch's one unit-time,
// 350-390 us, serially after the rest; each workgroup walking a contiguous
// range of units measured slower than striding.)
template <bool OPEN, bool OB>
__global__ __launch_bounds__(kGBlock) void quic_gcm_staged_kernel(const QGParams Q) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords<true, 92>];
  uint32_t *tP, *tT, *tH, *tK;  // tK[88..90]: the staged key's IV
  GRec(*recs)[kGPpw];
  uint16_t(*clists)[kGList];
  gcm_lds<true, 92>(lds, tP, tT, tH, tK, recs, clists);
  stage_common<true>(Q, tT, tP, tH, tK);
  __syncthreads();
  const uint32_t lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint32_t tcol = 4 * (lane & 31);
  // step table (gcm_group_scan): kstart[bins] | kcount[bins] | sfirst[bins],
  // sfirst[n_keys] = the number of steps
  const uint32_t bins = Q.n_keys + 1;
  const uint32_t *kstart = Q.gmeta, *kcount = Q.gmeta + bins, *sfirst = Q.gmeta + 2 * bins;
  const uint32_t nsteps = rfl32(sfirst[Q.n_keys]);
  uint32_t staged = kNoKey;
  for (uint32_t st = blockIdx.x; st < nsteps; st += gridDim.x) {
    // the step's key: the last k with sfirst[k] <= st (keys without packets
    // share their successor's sfirst)
    uint32_t lo = 0, hi = Q.n_keys;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (rfl32(sfirst[mid]) <= st) lo = mid;
      else hi = mid;
    }
    const uint32_t k = lo;
    if (k != staged) {  // (block-uniform)
      __syncthreads();  // every wave is done with the previous key
      stage_key(Q.keys + k, tP, tH, tK);
      __syncthreads();
      staged = k;
    }
    const uint32_t j = st - rfl32(sfirst[k]);
    const uint32_t cnt_k = rfl32(kcount[k]);
    const uint64_t first = ((uint64_t)j * kGWaves + wv) * kGPpw;  // within the key
    if (first >= cnt_k) continue;
    const uint32_t cnt = cnt_k - first < kGPpw ? (uint32_t)(cnt_k - first) : kGPpw;
    gcm_unit<OPEN, false, OB, true>(Q, (uint64_t)rfl32(kstart[k]) + first, cnt, k,
                                    lane, tT, tcol, tP, tH, tK, recs[wv], clists[wv]);
  }
}

// ---------------------------------------------------------------- key groups

// Multi-key batches are grouped by key when they have at least kGrpMinN
// packets, at most kGrpMaxKeys keys and at least kGrpPerKey packets per key
// on average (a key's last step is partly idle: ~6 of 12 units, so sparser
// keys waste more than the staging saves).  Counting sort in three
// launches: per-chunk key histograms (bin n_keys: ids out of range), one
// exclusive scan over them in key-major order that also builds the step
// table, and a stable scatter by one wave per chunk (ranks among equal keys
// from ballots over the key bits) that rejects the out-of-range ids.
constexpr uint32_t kGrpMinN = 2048;
constexpr uint32_t kGrpMaxKeys = 1023;  // bins = keys + 1 <= 1024 (one scan block)
constexpr uint32_t kGrpPerKey = 1024;
constexpr uint32_t kStepPackets = kGWaves * kGPpw;  // a step: 12 units of 32
constexpr uint32_t kGrpChunk = 4096;  // packets per histogram chunk
constexpr uint32_t kGrpBits = 11;     // bins <= kGrpMaxKeys + 1 <= 2^11

__global__ __launch_bounds__(256) void gcm_group_hist(const uint16_t *kid, uint32_t n,
                                                      uint32_t bins, uint32_t nch,
                                                      uint32_t *hist) {
  __shared__ uint32_t h[kGrpMaxKeys + 1];
  for (uint32_t i = threadIdx.x; i < bins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t c0 = (uint64_t)blockIdx.x * kGrpChunk;
  for (uint32_t i = threadIdx.x; i < kGrpChunk && c0 + i < n; i += blockDim.x) {
    const uint32_t k = kid[c0 + i];
    atomicAdd(&h[k < bins - 1 ? k : bins - 1], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < bins; i += blockDim.x) hist[(uint64_t)i * nch + blockIdx.x] = h[i];
}

// exclusive prefix sum of the histograms (total words, in place), then the
// step table meta = kstart[bins] | kcount[bins] | sfirst[bins]; one block of
// 1024 threads
__global__ __launch_bounds__(1024) void gcm_group_scan(uint32_t *hist, uint32_t total,
                                                       uint32_t n, uint32_t bins, uint32_t nch,
                                                       uint32_t *meta) {
  __shared__ uint32_t s[1024];
  const uint32_t t = threadIdx.x, seg = (total + 1023) / 1024;
  const uint64_t a = (uint64_t)t * seg, b = a + seg < total ? a + seg : total;
  uint32_t sum = 0;
  for (uint64_t i = a; i < b; i++) sum += hist[i];
  s[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t v = t >= d ? s[t - d] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  uint32_t run = s[t] - sum;
  for (uint64_t i = a; i < b; i++) {
    const uint32_t v = hist[i];
    hist[i] = run;
    run += v;
  }
  __syncthreads();  // (the block's global writes, visible to the block)
  // per key: start, count, steps; the steps' exclusive prefix (bin bins-1,
  // the invalid ids, takes none: its sfirst is the total)
  uint32_t kst = 0, kc = 0, steps = 0;
  if (t < bins) {
    kst = hist[(uint64_t)t * nch];
    kc = (t + 1 < bins ? hist[(uint64_t)(t + 1) * nch] : n) - kst;
    steps = t + 1 < bins ? (kc + kStepPackets - 1) / kStepPackets : 0u;
  }
  __syncthreads();
  s[t] = steps;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t v = t >= d ? s[t - d] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  if (t < bins) {
    meta[t] = kst;
    meta[bins + t] = kc;
    meta[2 * bins + t] = s[t] - steps;
  }
}

__global__ __launch_bounds__(64) void gcm_group_scatter(const uint16_t *kid, uint32_t n,
                                                        uint32_t bins, uint32_t nch,
                                                        const uint32_t *hist, uint32_t *perm,
                                                        uint32_t *out_len, uint64_t *pn_out) {
  __shared__ uint32_t base[kGrpMaxKeys + 1];
  __shared__ uint16_t kk[kGrpChunk];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < bins; i += kWave) base[i] = hist[(uint64_t)i * nch + blockIdx.x];
  const uint64_t c0 = (uint64_t)blockIdx.x * kGrpChunk;
  const uint32_t m = n - c0 < kGrpChunk ? (uint32_t)(n - c0) : kGrpChunk;
  for (uint32_t i = lane; i < m; i += kWave) {
    const uint32_t k = kid[c0 + i];
    kk[i] = (uint16_t)(k < bins - 1 ? k : bins - 1);
    if (k >= bins - 1) {  // an id past the keyring: rejected, as the kernels do
      out_len[c0 + i] = kQEKey;
      if (pn_out) pn_out[c0 + i] = 0;
    }
  }
  __syncthreads();
  const uint64_t below = (1ull << lane) - 1ull;
  for (uint32_t j = 0; j < m; j += kWave) {
    const uint32_t i = j + lane;
    const bool valid = i < m;
    const uint32_t k = valid ? kk[i] : 0u;
    // lanes holding the same key as this one
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (uint32_t bt = 0; bt < kGrpBits; bt++) {
      const uint64_t on = __ballot(valid && ((k >> bt) & 1u));
      peers &= ((k >> bt) & 1u) ? on : ~on;
    }
    const uint32_t b0 = valid ? base[k] : 0u;
    if (valid) perm[b0 + __popcll(peers & below)] = (uint32_t)(c0 + i);
    // the highest lane of each key advances its base (after every read)
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers >> lane) == 1ull) base[k] = b0 + (uint32_t)__popcll(peers);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the base writes land first
  }
}

static uint32_t grp_chunks(uint32_t n) { return (n + kGrpChunk - 1) / kGrpChunk; }

}  // namespace sq

extern "C" uint64_t sq_gcm_group_scratch(uint32_t n, uint32_t n_keys) {
  using namespace sq;
  if (n < kGrpMinN || n_keys == 0 || n_keys > kGrpMaxKeys || n / n_keys < kGrpPerKey)
    return 0;  // not grouped
  // perm[n] | hist[bins * chunks] | meta[3 * bins]
  return 4ull * n + 4ull * (n_keys + 1) * grp_chunks(n) + 12ull * (n_keys + 1);
}

extern "C" int sq_launch_gcm_group(const uint16_t *key_id, uint32_t n, uint32_t n_keys,
                                   int open, uint32_t *out_len, uint64_t *pn_out,
                                   void *scratch, const uint32_t **meta, void *stream) {
  using namespace sq;
  if (sq_gcm_group_scratch(n, n_keys) == 0) return 1;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t nch = grp_chunks(n), bins = n_keys + 1;
  uint32_t *perm = (uint32_t *)scratch;
  uint32_t *hist = perm + n;
  uint32_t *mt = hist + (uint64_t)bins * nch;
  *meta = mt;
  (void)hipGetLastError();  // (a stale error is not these launches': sq_kernels.hip launch_k)
  hipLaunchKernelGGL(gcm_group_hist, dim3(nch), dim3(256), 0, s, key_id, n, bins, nch, hist);
  hipLaunchKernelGGL(gcm_group_scan, dim3(1), dim3(1024), 0, s, hist, bins * nch, n, bins, nch, mt);
  hipLaunchKernelGGL(gcm_group_scatter, dim3(nch), dim3(kWave), 0, s, key_id, n, bins, nch,
                     (const uint32_t *)hist, perm, out_len, open ? pn_out : nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

namespace sq {

// resident workgroups of a kernel on the device (the persistent grid)
static uint64_t resident_blocks(const void *fn) {
  int dev = 0, per_cu = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kGBlock, 0);
  return (uint64_t)(per_cu < 1 ? 1 : per_cu) * (uint64_t)(cus < 1 ? 1 : cus);
}

template <bool OPEN, bool MULTI, bool OB>
static int launch_gcm(const QGParams *qp, hipStream_t s) {
  // queried once (thread-safe static init)
  static const uint64_t cap = resident_blocks((const void *)quic_gcm_kernel<OPEN, MULTI, OB>);
  static const uint64_t cap_st =
      resident_blocks((const void *)quic_gcm_staged_kernel<OPEN, OB>);
  const uint64_t waves = ((uint64_t)qp->n + kGPpw - 1) / kGPpw;
  const uint64_t want = (waves + kGWaves - 1) / kGWaves;
  (void)hipGetLastError();  // (a stale error is not this launch's: sq_kernels.hip launch_k)
  if (MULTI && qp->perm) {  // grouped: every valid packet is in a step
    hipLaunchKernelGGL((quic_gcm_staged_kernel<OPEN, OB>), dim3((uint32_t)(want < cap_st ? want : cap_st)),
                       dim3(kGBlock), 0, s, *qp);
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  hipLaunchKernelGGL((quic_gcm_kernel<OPEN, MULTI, OB>), dim3((uint32_t)(want < cap ? want : cap)),
                     dim3(kGBlock), 0, s, *qp);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace sq

extern "C" int sq_launch_quic_gcm(int open, const sq::QGParams *qp, void *stream) {
  using namespace sq;
  if (qp->n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool multi = qp->key_id != nullptr;
  if (qp->obfs) {
    if (open) return multi ? launch_gcm<true, true, true>(qp, s) : launch_gcm<true, false, true>(qp, s);
    return multi ? launch_gcm<false, true, true>(qp, s) : launch_gcm<false, false, true>(qp, s);
  }
  if (open) return multi ? launch_gcm<true, true, false>(qp, s) : launch_gcm<true, false, false>(qp, s);
  return multi ? launch_gcm<false, true, false>(qp, s) : launch_gcm<false, false, false>(qp, s);
}
