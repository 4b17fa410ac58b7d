// sq_quic.hip -- gfx950 QUIC packet protection, AEAD_CHACHA20_POLY1305
// (SURVEY.md 8(f) rank 4).
//
// Replaces, for a whole ragged batch per launch, quic-go's per-packet
//   internal/handshake/aead.go           Seal / Open of 1-RTT packets
//   internal/handshake/header_protector.go  chacha header protection
// (quic-go v0.52.0-beta.1, go.mod:7; reached from the reference through
// quic.go:47-102; not in the reference tree).  The algorithms are RFC 8439
// sections 2.5 / 2.8 (Poly1305, the AEAD) and RFC 9001 sections 5.3 / 5.4.4
// (nonce, ChaCha20 header protection); the packet-number decode is RFC 9000
// Appendix A.3.  The CPU checker is oracle/oracle.c (or_quic_seal / open),
// pinned by RFC 9001 Appendix A.5 and OpenSSL (tests/golden/quic.json).
//
// Decomposition (quic_kernel below): 32 packets per wave, three phases.
//   1. owner lane per packet: descriptor, header protection off (open), the
//      Poly1305 key block and the MAC over the header;
//   2. all 64 lanes: the packets' FULL 64-byte blocks (keystream counter
//      1..) as one flat space, one block per lane per step, so consecutive
//      lanes read and write consecutive bytes (unaligned 16-byte loads and
//      stores: no realignment, no partial stores); each lane's four
//      ciphertext chunks are Horner-ed into a partial MAC (26-bit limbs,
//      v_mad_u64_u32 products) and lane pairs fold theirs;
//   3. owner lane: the partials combined with powers of r, the payload's
//      tail (its last pl % 64 bytes: keystream block from the lane pairs,
//      byte-exact stores), the tag, and (seal) the header-protection mask
//      from the ciphertext sample.
// The owner phases' ChaCha20 blocks are shared by lanes l and l + 32
// (lane pairs).  Payloads past the cooperative range are walked by their
// owner lane with a streaming realigner (payload_pass): aligned 16-byte
// loads one step ahead, realigned in registers, aligned 16-byte stores.
#include <hip/hip_runtime.h>

#include "sq_bytes.h"
#include "sq_hash.h"
#include "sq_internal.h"
#include "sq_obfs_key.h"
#include "sq_quic.h"

namespace sq {

// Threads per workgroup.  Its waves share nothing, and a workgroup's slots
// free only when all of its waves have ended: 1-wave groups measured 1.3 %
// (seal) and 1.0 % (open) faster than 4-wave ones, 3 interleaved passes.
constexpr uint32_t kQBlock = 64;
constexpr uint32_t kQWaves = kQBlock / kWave;
// Packets per wave (owner lanes of phases 1 and 3).  32 with a 1,536-byte
// cooperative range (MTU-sized packets; longer ones take the owner lane's
// sequential pass) needs 20 KB of LDS per wave (8 waves per CU, 2 per
// SIMD; the 2,048-byte range needed 25 KB, 6 per CU) and halves the idle
// lanes of the owner phases: seal 1,570 -> 1,406 us against 16 packets and
// 2,048 B (24: 1,545; 40: 1,677).
constexpr uint32_t kQPpw = 32;
// Waves per SIMD the register allocation must allow.  With pairs the LDS
// admits 3; the fused seal needs 177 VGPRs uncapped (2 waves) and 168 with
// 40 bytes of spills at 3: 1,548 -> 1,467 us, every other kernel unchanged
// (two interleaved passes).
constexpr uint32_t kQMinWaves = 3;
constexpr uint32_t kQCoopMax = 1536;  // payloads up to this size take the cooperative pass
constexpr uint32_t kQMaxBlk = kQPpw * (kQCoopMax / 64);
// Pairs: every packet's flat blocks start at an even index, and the even
// lane of each pair of lanes folds its neighbour's partial MAC into its own
// (P_b r^k + P_b+1, k = the chunks of block b+1), so LDS holds one partial
// per two blocks: 13 KB per wave instead of 20 KB, 12 waves per CU instead of
// 8.
static_assert((kQCoopMax / 64) % 2 == 0, "pairs: a packet's padded block count stays in range");
constexpr uint32_t kQParts = kQMaxBlk / 2;

// ---------------------------------------------------------------- Poly1305

struct Poly {
  uint32_t r0, r1, r2, r3, r4, s1, s2, s3, s4;
  uint32_t h0, h1, h2, h3, h4;
};

// r = clamp(otk[0..16)), h = 0 (RFC 8439 2.5.1)
__device__ __forceinline__ void poly_init(Poly &P, const uint32_t (&otk)[16]) {
  P.r0 = otk[0] & 0x3ffffffu;
  P.r1 = __builtin_amdgcn_alignbit(otk[1], otk[0], 26) & 0x3ffff03u;
  P.r2 = __builtin_amdgcn_alignbit(otk[2], otk[1], 20) & 0x3ffc0ffu;
  P.r3 = __builtin_amdgcn_alignbit(otk[3], otk[2], 14) & 0x3f03fffu;
  P.r4 = (otk[3] >> 8) & 0x00fffffu;
  P.s1 = P.r1 * 5;
  P.s2 = P.r2 * 5;
  P.s3 = P.r3 * 5;
  P.s4 = P.r4 * 5;
  P.h0 = P.h1 = P.h2 = P.h3 = P.h4 = 0;
}

__device__ __forceinline__ uint64_t mul(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

// h = h * r mod 2^130 - 5 (partially reduced limbs)
__device__ __forceinline__ void poly_mul(Poly &P) {
  const uint32_t h0 = P.h0, h1 = P.h1, h2 = P.h2, h3 = P.h3, h4 = P.h4;
  const uint64_t d0 = mul(h0, P.r0) + mul(h1, P.s4) + mul(h2, P.s3) + mul(h3, P.s2) + mul(h4, P.s1);
  uint64_t d1 = mul(h0, P.r1) + mul(h1, P.r0) + mul(h2, P.s4) + mul(h3, P.s3) + mul(h4, P.s2);
  uint64_t d2 = mul(h0, P.r2) + mul(h1, P.r1) + mul(h2, P.r0) + mul(h3, P.s4) + mul(h4, P.s3);
  uint64_t d3 = mul(h0, P.r3) + mul(h1, P.r2) + mul(h2, P.r1) + mul(h3, P.r0) + mul(h4, P.s4);
  uint64_t d4 = mul(h0, P.r4) + mul(h1, P.r3) + mul(h2, P.r2) + mul(h3, P.r1) + mul(h4, P.r0);
  uint32_t c = (uint32_t)(d0 >> 26);
  P.h0 = (uint32_t)d0 & 0x3ffffffu;
  d1 += c; c = (uint32_t)(d1 >> 26); P.h1 = (uint32_t)d1 & 0x3ffffffu;
  d2 += c; c = (uint32_t)(d2 >> 26); P.h2 = (uint32_t)d2 & 0x3ffffffu;
  d3 += c; c = (uint32_t)(d3 >> 26); P.h3 = (uint32_t)d3 & 0x3ffffffu;
  d4 += c; c = (uint32_t)(d4 >> 26); P.h4 = (uint32_t)d4 & 0x3ffffffu;
  P.h0 += c * 5;
  c = P.h0 >> 26;
  P.h0 &= 0x3ffffffu;
  P.h1 += c;
}

// h = (h + m + 2^128) * r mod 2^130 - 5, one full 16-byte block
__device__ __forceinline__ void poly_block(Poly &P, const uint32_t (&m)[4]) {
  P.h0 += m[0] & 0x3ffffffu;
  P.h1 += __builtin_amdgcn_alignbit(m[1], m[0], 26) & 0x3ffffffu;
  P.h2 += __builtin_amdgcn_alignbit(m[2], m[1], 20) & 0x3ffffffu;
  P.h3 += __builtin_amdgcn_alignbit(m[3], m[2], 14) & 0x3ffffffu;
  P.h4 += (m[3] >> 8) | (1u << 24);
  poly_mul(P);
}

// tag = (h mod p) + s mod 2^128, s = otk[16..32)
__device__ __forceinline__ void poly_finish(Poly &P, const uint32_t (&otk)[16],
                                            uint32_t (&tag)[4]) {
  uint32_t h0 = P.h0, h1 = P.h1, h2 = P.h2, h3 = P.h3, h4 = P.h4;
  uint32_t c = h1 >> 26; h1 &= 0x3ffffffu;
  h2 += c; c = h2 >> 26; h2 &= 0x3ffffffu;
  h3 += c; c = h3 >> 26; h3 &= 0x3ffffffu;
  h4 += c; c = h4 >> 26; h4 &= 0x3ffffffu;
  h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffffu;
  h1 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffffu;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffffu;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffffu;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffffu;
  const uint32_t g4 = h4 + c - (1u << 26);
  const uint32_t sel = (g4 >> 31) - 1u;  // all ones if h >= p
  h0 = bsel(sel, g0, h0);
  h1 = bsel(sel, g1, h1);
  h2 = bsel(sel, g2, h2);
  h3 = bsel(sel, g3, h3);
  h4 = bsel(sel, g4, h4);
  uint64_t f = (uint64_t)(h0 | (h1 << 26)) + otk[4];
  tag[0] = (uint32_t)f;
  f = (uint64_t)((h1 >> 6) | (h2 << 20)) + otk[5] + (f >> 32);
  tag[1] = (uint32_t)f;
  f = (uint64_t)((h2 >> 12) | (h3 << 14)) + otk[6] + (f >> 32);
  tag[2] = (uint32_t)f;
  f = (uint64_t)((h3 >> 18) | (h4 << 8)) + otk[7] + (f >> 32);
  tag[3] = (uint32_t)f;
}

// ---------------------------------------------------------------- helpers

// nonce = iv XOR be96(pn) as little-endian words (RFC 9001 5.3)
__device__ __forceinline__ void quic_nonce(const QuicKeyDev &K, uint64_t pn, uint32_t (&n)[3]) {
  quic_nonce_iv(K.iv, pn, n);
}

// ------------------------------------------------- lane-pair ChaCha20 blocks
// The owner phases run one ChaCha20 block per packet at a time (the Poly1305
// key block; the header-protection mask block) on the 32 owner lanes while
// lanes 32-63 idle, and a wave instruction costs the same whatever its exec
// mask.  Lane pairs: owner lane l and lane l + 32 share the
// block.  The low lane holds state columns 0-1, the high lane columns 2-3
// (4 x 4 state, words x0..x15 row-major, RFC 8439 2.3).  The column round
// is local; the diagonal round runs on the pair's diagonals after a swap of
// 4 words with the partner (v_permlane32_swap, a VALU op: b = (b1, b0'),
// c = (c0', c1'), d = (d1', d0), where ' is the partner's) and swaps 4 back
// after it.  Per lane 40 quarter rounds and 80 word swaps instead of 80
// quarter rounds.
static_assert(kQPpw == kWave / 2, "lane pairs are lanes l and l + 32");

// the partner lane's x (lane l <-> lane l + 32); every lane must be active
__device__ __forceinline__ uint32_t xhalf(uint32_t x, bool hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return hi ? r[0] : r[1];
}

// the low lane's pointer in both lanes of a pair
template <typename T>
__device__ __forceinline__ T *xlow_ptr(T *p, bool hi) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = xhalf((uint32_t)v, hi), up = xhalf((uint32_t)(v >> 32), hi);
  return hi ? (T *)(((uint64_t)up << 32) | lo) : p;
}

#define SQ_CC_QR2(a, b, c, d)                 \
  a += b; d ^= a; d = cc_rotl(d, 16);         \
  c += d; b ^= c; b = cc_rotl(b, 12);         \
  a += b; d ^= a; d = cc_rotl(d, 8);          \
  c += d; b ^= c; b = cc_rotl(b, 7);

// One block over a lane pair.  key: the block's key (read in full by both
// lanes); counter, n0..n2: the low lane's (the high lane's are ignored).
// o = this lane's two columns of the output: low lane words
// 0,1,4,5,8,9,12,13, high lane 2,3,6,7,10,11,14,15.
__device__ __forceinline__ void chacha20_pair(const uint32_t (&key)[8], uint32_t counter,
                                              uint32_t n0, uint32_t n1, uint32_t n2, bool hi,
                                              uint32_t (&o)[8]) {
  const uint32_t y1 = xhalf(n1, hi), y2 = xhalf(n2, hi);
  uint32_t in[8];
  in[0] = hi ? 0x79622d32u : 0x61707865u;
  in[1] = hi ? 0x6b206574u : 0x3320646eu;
  in[2] = hi ? key[2] : key[0];
  in[3] = hi ? key[3] : key[1];
  in[4] = hi ? key[6] : key[4];
  in[5] = hi ? key[7] : key[5];
  in[6] = hi ? y1 : counter;
  in[7] = hi ? y2 : n0;
  uint32_t a0 = in[0], a1 = in[1], b0 = in[2], b1 = in[3], c0 = in[4], c1 = in[5], d0 = in[6],
           d1 = in[7];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    SQ_CC_QR2(a0, b0, c0, d0)
    SQ_CC_QR2(a1, b1, c1, d1)
    // diagonalise: low lane (x0, x5, x10, x15), (x1, x6, x11, x12); high
    // lane (x2, x7, x8, x13), (x3, x4, x9, x14)
    uint32_t e0 = b1, e1 = xhalf(b0, hi), f0 = xhalf(c0, hi), f1 = xhalf(c1, hi),
             g0 = xhalf(d1, hi), g1 = d0;
    SQ_CC_QR2(a0, e0, f0, g0)
    SQ_CC_QR2(a1, e1, f1, g1)
    b0 = xhalf(e1, hi); b1 = e0;
    c0 = xhalf(f0, hi); c1 = xhalf(f1, hi);
    d0 = g1; d1 = xhalf(g0, hi);
  }
  o[0] = a0 + in[0]; o[1] = a1 + in[1]; o[2] = b0 + in[2]; o[3] = b1 + in[3];
  o[4] = c0 + in[4]; o[5] = c1 + in[5]; o[6] = d0 + in[6]; o[7] = d1 + in[7];
}
#undef SQ_CC_QR2

// The header-protection mask of every live owner lane (hp_mask); with lane
// pairs, every lane of the wave must call it.
template <bool MULTI>
__device__ __forceinline__ void hp_mask_lanes(const QuicKeyDev *K, const uint32_t (&sample)[4],
                                              bool live, uint32_t lane, uint32_t &m0,
                                              uint32_t &m1) {
  (void)live;
  const bool hi = lane >= kWave / 2;
  const QuicKeyDev *KP = MULTI ? xlow_ptr(K, hi) : K;
  uint32_t o[8];
  chacha20_pair(KP->hp, sample[0], sample[1], sample[2], sample[3], hi, o);
  m0 = o[0];
  m1 = o[1] & 0xFFu;
}

// The Poly1305 one-time key, otk[0..8) = ChaCha20(key, 0, nonce) words 0-7,
// of every live owner lane; with lane pairs, every lane must call it.
template <bool MULTI>
__device__ __forceinline__ void otk_lanes(const QuicKeyDev *K, const uint32_t (&nonce)[3],
                                          bool live, uint32_t lane, uint32_t (&otk)[16]) {
  (void)live;
  const bool hi = lane >= kWave / 2;
  const QuicKeyDev *KP = MULTI ? xlow_ptr(K, hi) : K;
  uint32_t o[8];
  chacha20_pair(KP->key, 0u, nonce[0], nonce[1], nonce[2], hi, o);
  otk[0] = o[0];
  otk[1] = o[1];
  otk[2] = xhalf(o[0], hi);
  otk[3] = xhalf(o[1], hi);
  otk[4] = o[2];
  otk[5] = o[3];
  otk[6] = xhalf(o[2], hi);
  otk[7] = xhalf(o[3], hi);
}

// Payload pass shared by seal (MAC over the output) and open (MAC over the
// input): XOR `len` bytes from src with the keystream from counter 1, MAC
// the ciphertext side, store to dst.  A streaming realigner: one aligned
// 16-byte load of the input and one aligned 16-byte store of the output per
// chunk, whatever the alignments of src and dst (only the first and last
// output blocks are partial stores; only aligned blocks holding valid input
// bytes are read).  In place (src == dst) works: every input block is loaded
// before the output block at the same address is stored.  first32 receives
// ciphertext bytes 0..31 (zero past len) for the header-protection sample.
// OB (fused Salamander layer): the output (seal) or input (open) bytes are
// also XORed with the packet's Salamander key, okr = that key rotated to the
// payload's first byte (chunk j uses its half j & 1).
template <bool SEAL, bool OB>
__device__ __forceinline__ void payload_pass(const QuicKeyDev &K, const uint32_t (&nonce)[3],
                                             uint64_t src, uint64_t dst, uint32_t len, Poly &P,
                                             uint32_t (&first32)[8], const uint32_t (&okr)[8]) {
#pragma unroll
  for (int j = 0; j < 8; j++) first32[j] = 0u;
  if (len == 0) return;
  const uint32_t ib = (uint32_t)(src & 15), oa = (uint32_t)(dst & 15);
  const uint64_t S0 = src - ib, D0 = dst - oa;
  const uint64_t last = (src + len - 1) & ~15ull;  // last aligned block with valid bytes
  // aligned input block i (0 = the one holding src), zero past the end; the
  // address is clamped so the load is unconditional (no branch, exact waits)
  auto load_blk = [&](uint32_t i, uint32_t (&v)[4]) {
    const uint64_t A = S0 + 16ull * i;
    const u32x4 x = gld<u32x4>(A < last ? A : last);
    const bool ok = A <= last;
    v[0] = ok ? x.x : 0u; v[1] = ok ? x.y : 0u; v[2] = ok ? x.z : 0u; v[3] = ok ? x.w : 0u;
  };
  uint32_t in_prev[4], prev_c[4] = {0u, 0u, 0u, 0u};
  uint32_t cur[4][4], nxt[4][4];
  load_blk(0, in_prev);
#pragma unroll
  for (int q = 0; q < 4; q++) load_blk(1 + q, cur[q]);
  const uint32_t nchunk = (len + 15) / 16, nstep = (nchunk + 3) / 4;
  for (uint32_t st = 0; st < nstep; st++) {
    // the next step's 64 input bytes are in flight during this step's
    // ChaCha20 block and MAC
#pragma unroll
    for (int q = 0; q < 4; q++) load_blk(4 * st + 5 + q, nxt[q]);
    uint32_t ks[16];
    chacha20_block(K.key, 1 + st, nonce, ks);
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint32_t j = 4 * st + q;
      if (j < nchunk) {
        const uint32_t nb = len - 16 * j < 16 ? len - 16 * j : 16;
        uint32_t in[4], c[4];
        funnel(in_prev, cur[q], ib, in);
#pragma unroll
        for (int w = 0; w < 4; w++) {
          in_prev[w] = cur[q][w];
          in[w] &= range_mask(0, (int)nb, w);
          if (OB && !SEAL) in[w] ^= okr[4 * (q & 1) + w] & range_mask(0, (int)nb, w);
          c[w] = (in[w] ^ ks[4 * q + w]) & range_mask(0, (int)nb, w);
        }
        if (SEAL) poly_block(P, c);
        else poly_block(P, in);
        if (j < 2) {
#pragma unroll
          for (int w = 0; w < 4; w++) first32[4 * j + w] = SEAL ? c[w] : in[w];
        }
        if (OB && SEAL) {
#pragma unroll
          for (int w = 0; w < 4; w++) c[w] ^= okr[4 * (q & 1) + w] & range_mask(0, (int)nb, w);
        }
        // output block D0 + 16j: bytes [0, oa) from the previous chunk's
        // tail, [oa, 16) from this chunk's head
        uint32_t blk[4];
        funnel(prev_c, c, 16 - oa, blk);
        const uint32_t lo = j == 0 ? oa : 0u;
        const uint32_t hi = oa + len - 16 * j < 16 ? oa + len - 16 * j : 16u;
        if (lo == 0 && hi == 16) gst<u32x4>(D0 + 16ull * j, u32x4{blk[0], blk[1], blk[2], blk[3]});
        else store_partial(D0 + 16ull * j, blk, lo, hi);
#pragma unroll
        for (int w = 0; w < 4; w++) prev_c[w] = c[w];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int w = 0; w < 4; w++) cur[q][w] = nxt[q][w];
  }
  // the last chunk's tail spills into one more output block
  if (oa + len > 16 * nchunk) {
    const uint32_t zero[4] = {0u, 0u, 0u, 0u};
    uint32_t blk[4];
    funnel(prev_c, zero, 16 - oa, blk);
    store_partial(D0 + 16ull * nchunk, blk, 0, oa + len - 16 * nchunk);
  }
}

// lengths block of the AEAD MAC: le64(aad_len) || le64(ct_len)
__device__ __forceinline__ void poly_lengths(Poly &P, uint32_t aad, uint32_t ct) {
  const uint32_t m[4] = {aad, 0u, ct, 0u};
  poly_block(P, m);
}

// ---------------------------------------------------------------- kernels

// Multi-key launches never point K at the kernarg copy: a pointer that may
// be either kernarg or global memory makes the compiler copy the whole
// QParams to scratch (576 bytes per lane measured) to form a flat pointer.
template <bool MULTI>
__device__ __forceinline__ bool pick_key(const QParams &Q, uint32_t p, const QuicKeyDev *&K) {
  K = MULTI ? Q.keys : &Q.key0;
  if (!MULTI) return true;
  const uint32_t kid = Q.key_id[p];
  if (kid >= Q.n_keys) return false;
  K = Q.keys + kid;
  return true;
}

// Per-packet record in LDS for the cooperative payload pass (176 bytes).
struct alignas(16) QRec {
  uint64_t src, dst;      // payload start in the input / output
  uint32_t pl, start;     // payload bytes; first flat keystream block
  uint32_t kid, nblk;     // key index; keystream blocks (64 bytes each)
  uint32_t nonce[3];
  uint32_t r[5];          // Poly1305 r (26-bit limbs; the 5 r terms are formed on use)
  uint32_t r4[5];         // pairs: r^4
  uint32_t pad[7];
  uint32_t ct32[8];       // ciphertext bytes 0..31 (the header-protection sample)
  uint32_t okr[8];        // fused Salamander layer: key rotated to the payload start
};
static_assert(sizeof(QRec) == 176, "QRec layout");

// One full 64-byte block b of one packet (cooperative pass, any lane): four
// unaligned 16-byte loads (issued before the keystream block), XOR, the
// chunks' Horner from h = 0 with the packet's r (partial MAC), four
// unaligned 16-byte stores.  gfx950 under the HSA runtime's unaligned mode
// moves a 16-byte access at any byte address in one instruction, so the
// round-5 realignment (five aligned loads and funnel shifts in, funnels and
// a shared "junction" block between neighbouring lanes out, byte-exact
// partial stores at a packet's ends) is gone; only full blocks come here
// (a payload's tail is its owner's, phase 3).  All loads precede the
// stores: in place, and the fused open's output 8 bytes before its input,
// never overwrite unread input (a block's stores reach 8 bytes into the
// previous block, read by an earlier lane or step).
template <bool OPEN, bool OB>
__device__ __forceinline__ void coop_full(const QuicKeyDev &K, QRec &R, uint32_t b,
                                          uint32_t (&contrib)[5]) {
  const uint64_t S = R.src + 64ull * b, D = R.dst + 64ull * b;
  uint32_t in[4][4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const u32x4 v = gld<u32x4_a1>(S + 16ull * q);
    in[q][0] = v.x; in[q][1] = v.y; in[q][2] = v.z; in[q][3] = v.w;
  }
  uint32_t ks[16];
  chacha20_block(K.key, 1 + b, R.nonce, ks);
  Poly L;
  L.r0 = R.r[0]; L.r1 = R.r[1]; L.r2 = R.r[2]; L.r3 = R.r[3]; L.r4 = R.r[4];
  L.s1 = L.r1 * 5; L.s2 = L.r2 * 5; L.s3 = L.r3 * 5; L.s4 = L.r4 * 5;
  L.h0 = L.h1 = L.h2 = L.h3 = L.h4 = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t x[4], c[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
      // (the key's half of chunk q: byte offset 64 b + 16 q, mod 32)
      x[w] = (OB && OPEN) ? in[q][w] ^ R.okr[4 * (q & 1) + w] : in[q][w];
      c[w] = x[w] ^ ks[4 * q + w];
    }
    if (OPEN) poly_block(L, x);
    else poly_block(L, c);
    if (!OPEN && b == 0 && q < 2) {
#pragma unroll
      for (int w = 0; w < 4; w++) R.ct32[4 * q + w] = c[w];
    }
    if (OB && !OPEN) {
#pragma unroll
      for (int w = 0; w < 4; w++) c[w] ^= R.okr[4 * (q & 1) + w];
    }
    gst<u32x4_a1>(D + 16ull * q, u32x4_a1{c[0], c[1], c[2], c[3]});
  }
  contrib[0] = L.h0; contrib[1] = L.h1; contrib[2] = L.h2; contrib[3] = L.h3; contrib[4] = L.h4;
}

// ChaCha20 block `counter` under each owner lane's key and nonce, all 16
// words in the owner (low) lane (lane pairs: every lane must call it).
template <bool MULTI>
__device__ __forceinline__ void ks_lanes(const QuicKeyDev *K, uint32_t counter,
                                         const uint32_t (&nonce)[3], uint32_t lane,
                                         uint32_t (&ks)[16]) {
  const bool hi = lane >= kWave / 2;
  const QuicKeyDev *KP = MULTI ? xlow_ptr(K, hi) : K;
  uint32_t o[8];
  chacha20_pair(KP->key, counter, nonce[0], nonce[1], nonce[2], hi, o);
#pragma unroll
  for (int i = 0; i < 4; i++) {  // low lane: words 4i, 4i+1; high lane: 4i+2, 4i+3
    ks[4 * i] = o[2 * i];
    ks[4 * i + 1] = o[2 * i + 1];
    ks[4 * i + 2] = xhalf(o[2 * i], hi);
    ks[4 * i + 3] = xhalf(o[2 * i + 1], hi);
  }
}

// Seal (OPEN = false) or open (OPEN = true) a ragged batch: kQPpw (32) packets
// per wave.
//   1. owner lane (one per packet): descriptor, header protection removal
//      and packet number (open), nonce, Poly1305 key, MAC over the header;
//   2. all 64 lanes: the packets' 64-byte keystream blocks as one flat
//      space (prefix sum), one block per lane per step -- consecutive lanes
//      read and write consecutive 64 bytes of a packet (coalesced); each
//      lane leaves its block's partial MAC P_b in LDS;
//   3. owner lane: h = h * r^k_b + P_b over the blocks (Horner in 4-block
//      strides: 1 multiply per 64 bytes), the lengths block, the tag, and
//      (seal) header protection from the sample kept in LDS.
// Payloads above kQCoopMax bytes are walked by their owner lane in phase 3
// (the sequential payload_pass), so any length works.
template <bool OPEN, bool MULTI, bool OB>
__global__ __launch_bounds__(kQBlock, kQMinWaves) void quic_kernel(const QParams Q) {
  __shared__ QRec recs[kQWaves][kQPpw];
  __shared__ uint32_t parts[kQWaves][kQParts][5];
  const uint32_t lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint64_t p64 = ((uint64_t)blockIdx.x * kQWaves + wv) * kQPpw + lane;
  const bool owner = lane < kQPpw && p64 < Q.n;
  const uint32_t p = (uint32_t)p64;

  // ---- 1. owner lanes
  bool live = owner;
  uint64_t pn_dec = 0;  // open: decoded packet number (0 if rejected)
  uint32_t status = 0, len = 0, pno = 0, first = 0, pn_len = 0, hdr = 0, pl = 0;
  uint64_t src = 0, dst = 0;
  const QuicKeyDev *K = MULTI ? Q.keys : &Q.key0;
  uint32_t nonce[3] = {0u, 0u, 0u}, otk[16], rtag[4] = {0u, 0u, 0u, 0u};
  uint32_t hd[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, pnw = 0;  // packet bytes 0..31; seal: pn bytes
  // fused Salamander layer (OB): wire = salt8 || QUIC packet ^ okey
  uint64_t wire = 0;
  uint32_t okey[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, osalt[4] = {0u, 0u, 0u, 0u};
  Poly P;
  P.h0 = P.h1 = P.h2 = P.h3 = P.h4 = 0;
  P.r0 = P.r1 = P.r2 = P.r3 = P.r4 = P.s1 = P.s2 = P.s3 = P.s4 = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) otk[i] = 0u;
  if (live && !pick_key<MULTI>(Q, p, K)) {
    status = kQEKey;
    live = false;
    if (OPEN && Q.pn_out) Q.pn_out[p] = 0;  // rejected: pn_out 0 (as below)
  }
  const bool entered = live;
  uint64_t pn = 0;
  uint32_t pnb[4] = {0u, 0u, 0u, 0u}, hs[4] = {0u, 0u, 0u, 0u};  // open: pn bytes, hp sample
  // packet byte k (de-obfuscated when the fused layer is on)
  auto hb = [&](uint32_t k) -> uint32_t {
    const uint32_t b = head_byte(hd, src, k);
    return (OB && OPEN && k >= 32) ? b ^ byte32(okey, k & 31) : b;
  };
  if (live) {
    src = (uint64_t)Q.in + Q.in_off[p];
    dst = (uint64_t)Q.out + Q.out_off[p];
    len = Q.in_len[p];
    pno = Q.pn_offset[p];
    pn = Q.pn[p];
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
      load16(src + pno + 4, src + len, hs);
      load16(src + len - 16, src + len, rtag);  // before any in-place write
      load_head32(src, len, hd);
      if (OB) {  // de-obfuscate what was read: key byte of QUIC offset k is okey[k % 32]
        uint32_t k4[4];
        keywin(okey, (pno + 4) & 31, k4);
#pragma unroll
        for (int w = 0; w < 4; w++) hs[w] ^= k4[w];
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
    }
  }
  if (OPEN) {  // header protection off (every lane: lane pairs)
    uint32_t m0 = 0u, m1 = 0u;
    hp_mask_lanes<MULTI>(K, hs, live, lane, m0, m1);
    if (live) {
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
  }
  if (entered) {
    if (!live) status = kQEShort;
    // every owner lane writes its pn_out (0 when the packet was rejected)
    if (OPEN && Q.pn_out) Q.pn_out[p] = pn_dec;
  }
  if (live) quic_nonce(*K, pn, nonce);
  otk_lanes<MULTI>(K, nonce, live, lane, otk);  // every lane: lane pairs
  if (live) {
    poly_init(P, otk);
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
      poly_block(P, w);
      if (OB && !OPEN) {  // the wire carries the (still unprotected) header ^ key
        uint32_t k4[4];
        keywin(okey, q & 31, k4);
#pragma unroll
        for (int j = 0; j < 4; j++) w[j] ^= k4[j];
      }
      if (OPEN || OB || dst != src) store16(dst + q, w, hdr - q < 16 ? hdr - q : 16);
    }
  }
  const bool coop = live && pl <= kQCoopMax;
  const uint32_t nblk = coop ? pl / 64 : 0u;  // full blocks (the tail is phase 3's)
  const uint32_t nflat = (nblk + 1) & ~1u;
  uint32_t incl = nflat;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, kWave);
    if (lane >= (uint32_t)d) incl += y;
  }
  const uint32_t start = incl - nflat, T = __shfl(incl, kWave - 1, kWave);
  if (lane < kQPpw) {
    QRec &R = recs[wv][lane];
    R.src = src + hdr;
    R.dst = dst + hdr;
    R.pl = pl;
    R.start = start;
    R.kid = MULTI && live ? (uint32_t)(K - Q.keys) : 0u;
    R.nblk = nblk;
#pragma unroll
    for (int i = 0; i < 3; i++) R.nonce[i] = nonce[i];
    R.r[0] = P.r0; R.r[1] = P.r1; R.r[2] = P.r2; R.r[3] = P.r3; R.r[4] = P.r4;
    if (nblk) {
      // X.h = r^4 (X.r = r)
      Poly X = P;
      X.h0 = P.r0; X.h1 = P.r1; X.h2 = P.r2; X.h3 = P.r3; X.h4 = P.r4;
#pragma unroll
      for (uint32_t k = 2; k <= 4; k++) poly_mul(X);
      R.r4[0] = X.h0; R.r4[1] = X.h1; R.r4[2] = X.h2; R.r4[3] = X.h3; R.r4[4] = X.h4;
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

  // ---- 2. cooperative payload pass over the flat block space
  for (uint32_t base = 0; base < T; base += kWave) {
    const uint32_t f = base + lane;
    const uint32_t pp = q_locate(start, base, f < T ? f : T - 1);
    QRec &R = recs[wv][pp];
    const uint32_t b = f - R.start;
    uint32_t c5[5] = {0u, 0u, 0u, 0u, 0u};
    if (f < T && b < R.nblk) {  // (b == nblk: an odd packet's padding block)
      const QuicKeyDev &KB = MULTI ? Q.keys[R.kid] : Q.key0;
      coop_full<OPEN, OB>(KB, R, b, c5);
    }
    // the odd neighbour's partial (the same packet: pairs start even)
    uint32_t n5[5];
#pragma unroll
    for (int i = 0; i < 5; i++) n5[i] = __shfl_down(c5[i], 1, kWave);
    if (!(lane & 1) && f < T) {
      if (b + 1 < R.nblk) {
        // P_b r^4 + P_b+1
        const uint32_t *m = R.r4;
        Poly X;
        X.r0 = m[0]; X.r1 = m[1]; X.r2 = m[2]; X.r3 = m[3]; X.r4 = m[4];
        X.s1 = X.r1 * 5; X.s2 = X.r2 * 5; X.s3 = X.r3 * 5; X.s4 = X.r4 * 5;
        X.h0 = c5[0]; X.h1 = c5[1]; X.h2 = c5[2]; X.h3 = c5[3]; X.h4 = c5[4];
        poly_mul(X);
        c5[0] = X.h0 + n5[0]; c5[1] = X.h1 + n5[1]; c5[2] = X.h2 + n5[2];
        c5[3] = X.h3 + n5[3]; c5[4] = X.h4 + n5[4];
      }
#pragma unroll
      for (int i = 0; i < 5; i++) parts[wv][f >> 1][i] = c5[i];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- 3. owner lanes: combine, tag, header protection (seal with lane
  // pairs: every lane stays for the mask block)
  const bool fin = owner && live;
  if (owner && !live) Q.out_len[p] = status;
  // the payload's tail keystream (block nblk + 1; every lane: lane pairs)
  uint32_t tks[16];
  ks_lanes<MULTI>(K, 1 + nblk, nonce, lane, tks);
  if (OPEN && !fin) return;
  uint32_t ct32[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  uint32_t tag[4] = {0u, 0u, 0u, 0u}, sample[4] = {0u, 0u, 0u, 0u};
  if (fin) {
    if (coop) {
      // pairs: h = h r^c + E_j, c = 8 chunks for a whole pair, 4 for a
      // last pair of one block
      const QRec &Rq = recs[wv][lane];
      Poly R1;
      R1.r0 = P.r0; R1.r1 = P.r1; R1.r2 = P.r2; R1.r3 = P.r3; R1.r4 = P.r4;
      R1.s1 = P.s1; R1.s2 = P.s2; R1.s3 = P.s3; R1.s4 = P.s4;
      Poly X;
      X.r0 = Rq.r4[0]; X.r1 = Rq.r4[1]; X.r2 = Rq.r4[2]; X.r3 = Rq.r4[3]; X.r4 = Rq.r4[4];
      X.s1 = X.r1 * 5; X.s2 = X.r2 * 5; X.s3 = X.r3 * 5; X.s4 = X.r4 * 5;
      X.h0 = X.r0; X.h1 = X.r1; X.h2 = X.r2; X.h3 = X.r3; X.h4 = X.r4;
      poly_mul(X);  // r^8
      const bool one = nblk & 1;  // the last pair holds one block
      const uint32_t M0 = one ? Rq.r4[0] : X.h0, M1 = one ? Rq.r4[1] : X.h1,
                     M2 = one ? Rq.r4[2] : X.h2, M3 = one ? Rq.r4[3] : X.h3,
                     M4 = one ? Rq.r4[4] : X.h4;
      const uint32_t npair = nflat / 2;
      for (uint32_t j = 0; j < npair; j++) {
        const bool lastp = j + 1 == npair;
        P.r0 = lastp ? M0 : X.h0;
        P.r1 = lastp ? M1 : X.h1;
        P.r2 = lastp ? M2 : X.h2;
        P.r3 = lastp ? M3 : X.h3;
        P.r4 = lastp ? M4 : X.h4;
        P.s1 = P.r1 * 5; P.s2 = P.r2 * 5; P.s3 = P.r3 * 5; P.s4 = P.r4 * 5;
        poly_mul(P);
        const uint32_t *c5 = parts[wv][start / 2 + j];
        P.h0 += c5[0]; P.h1 += c5[1]; P.h2 += c5[2]; P.h3 += c5[3]; P.h4 += c5[4];
      }
      // restore r for the tail and the lengths block
      P.r0 = R1.r0; P.r1 = R1.r1; P.r2 = R1.r2; P.r3 = R1.r3; P.r4 = R1.r4;
      P.s1 = R1.s1; P.s2 = R1.s2; P.s3 = R1.s3; P.s4 = R1.s4;
#pragma unroll
      for (int i = 0; i < 8; i++) ct32[i] = Rq.ct32[i];
      // the tail: pl % 64 bytes after the full blocks, byte-exact, chunk by
      // chunk (the MAC pads the last chunk with zeros, RFC 8439 2.8)
      const uint32_t tail = pl - 64 * nblk;
      const uint64_t ts = src + hdr + 64ull * nblk, td = dst + hdr + 64ull * nblk;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        if (16 * q < tail) {
          const uint32_t nb = tail - 16 * q < 16 ? tail - 16 * q : 16u;
          uint32_t x[4], c[4], kw[4];
          load16(ts + 16 * q, ts + tail, x);
#pragma unroll
          for (int w = 0; w < 4; w++) {
            const uint32_t m = range_mask(0, (int)nb, w);
            kw[w] = OB ? Rq.okr[4 * (q & 1) + w] & m : 0u;
            if (OB && OPEN) x[w] ^= kw[w];
            c[w] = (x[w] ^ tks[4 * q + w]) & m;
          }
          if (OPEN) poly_block(P, x);
          else poly_block(P, c);
          if (!OPEN && nblk == 0 && q < 2) {
#pragma unroll
            for (int w = 0; w < 4; w++) ct32[4 * q + w] = c[w];
          }
          uint32_t o[4];
#pragma unroll
          for (int w = 0; w < 4; w++) o[w] = (OB && !OPEN) ? c[w] ^ kw[w] : c[w];
          store16(td + 16 * q, o, nb);
        }
      }
    } else {
      uint32_t okr[8];
#pragma unroll
      for (int i = 0; i < 8; i++) okr[i] = OB ? recs[wv][lane].okr[i] : 0u;
      payload_pass<!OPEN, OB>(*K, nonce, src + hdr, dst + hdr, pl, P, ct32, okr);
    }
    poly_lengths(P, hdr, pl);
    poly_finish(P, otk, tag);
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
    if (pl >= so + 16) {
#pragma unroll
      for (int j = 0; j < 4; j++) sample[j] = __builtin_amdgcn_alignbyte(ct32[j + 1], ct32[j], so);
    } else {  // short payload: the sample reaches into the tag
      const uint32_t t8[8] = {tag[0], tag[1], tag[2], tag[3], 0u, 0u, 0u, 0u};
      for (uint32_t i = 0; i < 16; i++) {
        const uint32_t k = so + i;
        const uint32_t bb = k < pl ? byte32(ct32, k) : byte32(t8, k - pl);
        sample[i >> 2] |= bb << (8 * (i & 3));
      }
    }
  }  // fin
  if (OPEN) return;
  uint32_t m0 = 0u, m1 = 0u;
  hp_mask_lanes<MULTI>(K, sample, fin, lane, m0, m1);  // every lane: lane pairs
  if (!fin) return;
  // protected header bytes; with the fused layer also ^ the key byte of
  // their position
  const uint32_t kb0 = OB ? okey[0] & 0xFFu : 0u;
  gst<uint8_t>(dst, (uint8_t)(first ^ kb0 ^ (m0 & ((first & 0x80) ? 0x0Fu : 0x1Fu))));
  for (uint32_t i = 0; i < pn_len; i++) {
    const uint32_t bb = (pnw >> (8 * i)) & 0xFFu;
    const uint32_t kb = OB ? byte32(okey, (pno + i) & 31) : 0u;
    gst<uint8_t>(dst + pno + i, (uint8_t)(bb ^ kb ^ mask_byte(m0, m1, 1 + i)));
  }
  Q.out_len[p] = len + 16 + (OB ? kSalamanderSalt : 0u);
}

}  // namespace sq

extern "C" int sq_launch_quic(int open, const sq::QParams *qp, void *stream) {
  using namespace sq;
  if (qp->n == 0) return 0;
  const uint64_t waves = ((uint64_t)qp->n + kQPpw - 1) / kQPpw;
  const dim3 grid((uint32_t)((waves + kQWaves - 1) / kQWaves));
  hipStream_t s = (hipStream_t)stream;
  const bool multi = qp->key_id != nullptr;
#define SQ_QL(O, M, B) hipLaunchKernelGGL((quic_kernel<O, M, B>), grid, dim3(kQBlock), 0, s, *qp)
  (void)hipGetLastError();  // (a stale error is not this launch's: sq_kernels.hip launch_k)
  if (qp->obfs) {
    if (open) { if (multi) SQ_QL(true, true, true); else SQ_QL(true, false, true); }
    else { if (multi) SQ_QL(false, true, true); else SQ_QL(false, false, true); }
  } else {
    if (open) { if (multi) SQ_QL(true, true, false); else SQ_QL(true, false, false); }
    else { if (multi) SQ_QL(false, true, false); else SQ_QL(false, false, false); }
  }
#undef SQ_QL
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
