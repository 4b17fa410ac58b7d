// sq_quic.h -- helpers shared by the QUIC packet-protection kernels
// (sq_quic.hip: ChaCha20-Poly1305; sq_quic_gcm.hip: AES-128-GCM): header and
// packet-number handling of RFC 9001 5.3-5.4 / RFC 9000 A.3, byte shuffles,
// and the flat-block -> packet lookup of the cooperative payload pass.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sq_bytes.h"
#include "sq_internal.h"

namespace sq {

constexpr uint32_t kQMaxPacket = 1u << 20;
constexpr uint32_t kQEKey = 0xFFFFFFFFu, kQEShort = 0xFFFFFFFEu, kQEAuth = 0xFFFFFFFDu;

// nonce = iv XOR be96(pn) as little-endian words (RFC 9001 5.3)
__device__ __forceinline__ void quic_nonce_iv(const uint32_t (&iv)[3], uint64_t pn,
                                              uint32_t (&n)[3]) {
  n[0] = iv[0];
  n[1] = iv[1] ^ __builtin_bswap32((uint32_t)(pn >> 32));
  n[2] = iv[2] ^ __builtin_bswap32((uint32_t)pn);
}

// mask byte k (0..4) of (m0, m1)
__device__ __forceinline__ uint32_t mask_byte(uint32_t m0, uint32_t m1, uint32_t k) {
  return k < 4 ? (m0 >> (8 * k)) & 0xFFu : m1;
}

// Set byte `pos` (0..15, runtime) of a 16-byte register value to b.
__device__ __forceinline__ void set_byte(uint32_t (&v)[4], uint32_t pos, uint32_t b) {
  const uint32_t sh = 8 * (pos & 3), w = pos >> 2;
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t nv = (v[j] & ~(0xFFu << sh)) | (b << sh);
    v[j] = bsel(j == w, nv, v[j]);
  }
}

// byte k (0..31, runtime) of an 8-word register image
__device__ __forceinline__ uint32_t byte32(const uint32_t (&v)[8], uint32_t k) {
  const uint32_t w = k >> 2;
  uint32_t a = bsel(w & 1, v[1], v[0]), b = bsel(w & 1, v[3], v[2]);
  uint32_t c = bsel(w & 1, v[5], v[4]), d = bsel(w & 1, v[7], v[6]);
  a = bsel(w & 2, b, a);
  c = bsel(w & 2, d, c);
  return (bsel(w & 4, c, a) >> (8 * (k & 3))) & 0xFFu;
}

// RFC 9000 Appendix A.3
__device__ __forceinline__ uint64_t decode_pn(uint64_t largest, uint64_t truncated, uint32_t nbits) {
  const uint64_t expected = largest + 1, win = 1ull << nbits, hwin = win / 2, mask = win - 1;
  const uint64_t cand = (expected & ~mask) | truncated;
  if (cand + hwin <= expected && cand < (1ull << 62) - win) return cand + win;
  if (cand > expected + hwin && cand >= win) return cand - win;
  return cand;
}

// 16 bytes starting at byte o (0..16) of the 32-byte concatenation lo || hi
__device__ __forceinline__ void funnel(const uint32_t (&lo)[4], const uint32_t (&hi)[4],
                                       uint32_t o, uint32_t (&out)[4]) {
  const uint32_t w[12] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3], 0u, 0u, 0u, 0u};
  win16(w, o, out);
}

// Packet owning flat block c (>= b0) of the window [b0, b0 + 64): the last
// lane l with start[l] <= c (starts are sorted over the lanes).
__device__ __forceinline__ uint32_t q_locate(uint32_t start, uint32_t b0, uint32_t c) {
  int pp = __popcll(__ballot(start <= b0)) - 1;
  uint64_t M = __ballot(start > b0 && start < b0 + kWave);
  while (M) {
    const int l = __ffsll((unsigned long long)M) - 1;
    M &= M - 1;
    pp += c >= (uint32_t)__builtin_amdgcn_readlane(start, l) ? 1 : 0;
  }
  return pp < 0 ? 0u : (uint32_t)pp;
}

// The first 32 bytes of a packet of len >= 1 bytes at src (zero past the
// end), as 8 little-endian words.  One round of loads (at most four aligned
// blocks, all independent) yields the first byte, the packet number and any
// header of up to 32 bytes, instead of a chain of dependent byte loads.
__device__ __forceinline__ void load_head32(uint64_t src, uint32_t len, uint32_t (&hd)[8]) {
  const uint64_t end = src + len;
  uint32_t a[4], b[4] = {0u, 0u, 0u, 0u};
  load16(src, end, a);
  if (len > 16) load16(src + 16, end, b);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    hd[j] = a[j];
    hd[4 + j] = b[j];
  }
}

// byte k of the packet: from hd when k < 32, else loaded
__device__ __forceinline__ uint32_t head_byte(const uint32_t (&hd)[8], uint64_t src, uint32_t k) {
  return k < 32 ? byte32(hd, k) : (uint32_t)gld<uint8_t>(src + k);
}

// header block at q (a multiple of 16) with the bytes past hdr zeroed (the
// AAD's zero padding): from hd when q < 32, else loaded
__device__ __forceinline__ void head_block(const uint32_t (&hd)[8], uint64_t src, uint32_t q,
                                           uint32_t hdr, uint32_t (&w)[4]) {
  if (q < 32) {
    const int nb = (int)(hdr - q < 16 ? hdr - q : 16);
#pragma unroll
    for (int j = 0; j < 4; j++) w[j] = bsel(q == 0, hd[j], hd[4 + j]) & range_mask(0, nb, j);
  } else {
    load16(src + q, src + hdr, w);
  }
}

}  // namespace sq
