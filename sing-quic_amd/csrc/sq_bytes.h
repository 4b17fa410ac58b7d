// sq_bytes.h -- byte-granular register/global-memory helpers shared by the
// gfx950 kernels (obfuscation: sq_kernels.hip; QUIC protection: sq_quic.hip).
// Packets have arbitrary offsets and lengths: these read only the 16-byte
// aligned blocks that hold valid bytes and write exactly the bytes asked for,
// with naturally aligned 1/2/4/8/16-byte stores.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sq {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// dword-aligned 16-byte access: still one global_load_dwordx4 on gfx950
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// byte-aligned 16-byte access: one global_load / global_store_dwordx4 as
// well (the HSA runtime runs gfx950 in unaligned mode); only for bytes that
// are all inside the buffer (a read past its end may cross into an
// unmapped page)
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));

// Global-address-space accessors.  Packet addresses are computed as integers;
// a plain cast would give FLAT pointers, whose loads/stores count in both
// vmcnt and lgkmcnt and force the compiler to drain every outstanding store
// before each LDS read (one full HBM round trip per loop iteration).
#define SQ_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T gld(uint64_t a) {
  return *(const SQ_GLOBAL T *)a;
}
template <typename T>
__device__ __forceinline__ void gst(uint64_t a, T v) {
  *(SQ_GLOBAL T *)a = v;
}

// ------------------------------------------------------------ byte helpers

// Bitwise select (v_bfi_b32).  Used instead of `c ? a[i] : b[i]`, which
// clang folds into a select of POINTERS and then spills the arrays to scratch.
__device__ __forceinline__ uint32_t bsel(bool c, uint32_t a, uint32_t b) {
  const uint32_t m = 0u - (uint32_t)c;
  return (a & m) | (b & ~m);
}

// 5 consecutive words w[q..q+4] out of N (q runtime, q+4 < N) by a 3-stage
// barrel of bit selects (no scratch, no per-index compare chains).
template <int N>
__device__ __forceinline__ void take5(const uint32_t (&w)[N], uint32_t q,
                                      uint32_t (&x)[5]) {
  static_assert(N >= 12, "take5 needs 12 words");
  uint32_t y[8], z[6];
  const bool b2 = q & 4, b1 = q & 2, b0 = q & 1;
#pragma unroll
  for (int j = 0; j < 8; j++) y[j] = bsel(b2, w[j + 4], w[j]);
#pragma unroll
  for (int j = 0; j < 6; j++) z[j] = bsel(b1, y[j + 2], y[j]);
#pragma unroll
  for (int j = 0; j < 5; j++) x[j] = bsel(b0, z[j + 1], z[j]);
}

// 16 bytes starting at byte o (0..31) of a 48-byte register image w[12].
__device__ __forceinline__ void win16(const uint32_t (&w)[12], uint32_t o,
                                      uint32_t (&out)[4]) {
  uint32_t x[5];
  take5(w, o >> 2, x);
  const uint32_t sh = o & 3;
#pragma unroll
  for (int j = 0; j < 4; j++) out[j] = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
}

// keystream bytes key[(r + k) % 32], k = 0..15, as 4 LE words
__device__ __forceinline__ void keywin(const uint32_t (&key)[8], uint32_t r,
                                       uint32_t (&out)[4]) {
  uint32_t w[12];
#pragma unroll
  for (int j = 0; j < 12; j++) w[j] = key[j & 7];
  win16(w, r & 31, out);
}

// mask of bytes [lo, hi) inside word j (bytes 4j .. 4j+3)
__device__ __forceinline__ uint32_t bytes_below(int k) {
  return k <= 0 ? 0u : (k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * k)) - 1u));
}
__device__ __forceinline__ uint32_t range_mask(int lo, int hi, int j) {
  return bytes_below(hi - 4 * j) & ~bytes_below(lo - 4 * j);
}

__device__ __forceinline__ uint32_t pick4(const uint32_t (&v)[4], uint32_t i) {
  const uint32_t a = bsel(i & 1, v[1], v[0]);
  const uint32_t b = bsel(i & 1, v[3], v[2]);
  return bsel(i & 2, b, a);
}

// Loads the 16-byte-aligned blocks that hold bytes [ps, pe) (1..16 bytes) and
// returns the 16 bytes at address X (ps-15 <= X <= ps, pe <= X+16).  Only
// blocks containing at least one valid byte are read, so a packet at the very
// edge of an allocation never faults.
__device__ __forceinline__ void load_window(uint64_t ps, uint64_t pe,
                                            uint64_t X, uint32_t (&out)[4]) {
  const uint64_t B0 = ps & ~15ull;
  const u32x4 v0 = gld<u32x4>(B0);
  u32x4 v1 = {0u, 0u, 0u, 0u};
  if (pe > B0 + 16) v1 = gld<u32x4>(B0 + 16);
  const uint32_t w[12] = {0u,   0u,   0u,   0u,   v0.x, v0.y,
                          v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  win16(w, (uint32_t)(X - B0 + 16), out);
}

// Store bytes [a, b) of the 16-byte value v to the 16-byte-aligned address A
// with naturally aligned 1/2/4/8/16-byte stores (at most 9, usually 1-3).
__device__ __forceinline__ void store_partial(uint64_t A, const uint32_t (&v)[4],
                                              uint32_t a, uint32_t b) {
  uint32_t pos = a;
  if ((pos & 1) && pos + 1 <= b) {
    gst<uint8_t>(A + pos, (uint8_t)(pick4(v, pos >> 2) >> (8 * (pos & 3))));
    pos += 1;
  }
  if ((pos & 2) && pos + 2 <= b) {
    gst<uint16_t>(A + pos, (uint16_t)(pick4(v, pos >> 2) >> (8 * (pos & 2))));
    pos += 2;
  }
  if ((pos & 4) && pos + 4 <= b) {
    gst<uint32_t>(A + pos, pick4(v, pos >> 2));
    pos += 4;
  }
  if ((pos & 8) && pos + 8 <= b) {
    gst<u32x2>(A + 8, u32x2{v[2], v[3]});
    pos += 8;
  }
  if (pos == 0 && b == 16) {
    gst<u32x4>(A, u32x4{v[0], v[1], v[2], v[3]});
    pos = 16;
  }
  if (pos + 8 <= b) {  // pos is 0 or 8 here
    const bool hi = pos & 8;
    gst<u32x2>(A + pos, u32x2{bsel(hi, v[2], v[0]), bsel(hi, v[3], v[1])});
    pos += 8;
  }
  if (pos + 4 <= b) {
    gst<uint32_t>(A + pos, pick4(v, pos >> 2));
    pos += 4;
  }
  if (pos + 2 <= b) {
    gst<uint16_t>(A + pos, (uint16_t)(pick4(v, pos >> 2) >> (8 * (pos & 2))));
    pos += 2;
  }
  if (pos + 1 <= b) {
    gst<uint8_t>(A + pos, (uint8_t)(pick4(v, pos >> 2) >> (8 * (pos & 3))));
  }
}

// 16 bytes at any address X of which only [X, end) are valid (end > X): the
// bytes past `end` read as zero.
__device__ __forceinline__ void load16(uint64_t X, uint64_t end, uint32_t (&out)[4]) {
  const uint64_t pe = end < X + 16 ? end : X + 16;
  load_window(X, pe, X, out);
  const int nb = (int)(pe - X);
#pragma unroll
  for (int j = 0; j < 4; j++) out[j] &= range_mask(0, nb, j);
}

// Store bytes v[0 .. nbytes) (1..16) at any address Y: at most two aligned
// blocks, each written byte-exactly.
__device__ __forceinline__ void store16(uint64_t Y, const uint32_t (&v)[4], uint32_t nbytes) {
  const uint64_t A0 = Y & ~15ull;
  const uint32_t sh = (uint32_t)(Y & 15);
  const uint32_t w[12] = {0u, 0u, 0u, 0u, v[0], v[1], v[2], v[3], 0u, 0u, 0u, 0u};
  uint32_t blk[4];
  win16(w, 16 - sh, blk);  // block A0, byte j = v[j - sh]
  const uint32_t e0 = sh + nbytes < 16 ? sh + nbytes : 16;
  store_partial(A0, blk, sh, e0);
  if (sh + nbytes > 16) {
    win16(w, 32 - sh, blk);  // block A0 + 16, byte j = v[16 - sh + j]
    store_partial(A0 + 16, blk, 0, sh + nbytes - 16);
  }
}

// byte i (0..15, runtime) of a 16-byte register value
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&v)[4], uint32_t i) {
  return (pick4(v, i >> 2) >> (8 * (i & 3))) & 0xFFu;
}

}  // namespace sq
