// Dev-only bandwidth probes (not part of the product): which HBM streaming
// pattern can the obfuscation kernel hope for on MI355X?
//   PAT 0  grid-stride 16 B/lane (every wave walks the whole buffer)
//   PAT 1  per-wave contiguous region of `region` bytes
//   PAT 2  pure read (XOR-reduce, one store per lane)      -- read ceiling
//   PAT 3  pure write                                      -- write ceiling
//   PAT 4  as 1, but chunks c with c % 85 in {0, 84} are not stored (the
//          boundary blocks of 1360-byte packets: holes in every line pair)
//   PAT 5  as 4, but the holes are stored first, in a separate pass of the
//          same wave before its stream (what the edges do)
//   PAT 6  the region as 1360-byte packets, 16 lanes per packet, 4 packets per
//          round; lane j of a group copies chunks j, j + 16, ... (U per round)
//          single-buffered per round
// POL bit0 = nontemporal loads, bit1 = nontemporal stores.  SRC_OFF = source
// misalignment in bytes (8 mimics Salamander's salt shift).
// build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o build/libsqprobe.so scripts/probe_copy.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
#define G __attribute__((address_space(1)))

template <int POL>
__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
  if (POL & 1) return __builtin_nontemporal_load((const G u32x4 *)p);
  return *(const G u32x4_a4 *)p;
}
template <int POL>
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) {
  if (POL & 2) __builtin_nontemporal_store(v, (G u32x4 *)p);
  else *(G u32x4 *)p = v;
}

template <int U, int POL, int SRC_OFF>
__device__ __forceinline__ void lane_groups(const uint8_t *src, uint8_t *dst, uint64_t b,
                                            uint64_t e) {
  const u32x4 k = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  const uint32_t lane = threadIdx.x & 63, g = lane / 16, j = lane % 16;
  for (uint64_t r0 = b; r0 < e; r0 += 4 * 85) {  // round: 4 packets of 85 chunks
    const uint64_t pk = r0 + 85 * g;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t c = pk + j + 16 * u;
      const bool in = j + 16 * u < 85 && c < e;
      c = in ? c : b;
      v[u] = ld<POL>(src + 16 * c + SRC_OFF);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t c = pk + j + 16 * u;
      if (j + 16 * u < 85 && c < e) st<POL>(dst + 16 * c, v[u] ^ k);
    }
  }
}

template <int PAT, int U, int POL, int SRC_OFF>
__global__ __launch_bounds__(256) void probe(const uint8_t *src, uint8_t *dst, uint64_t n,
                                             uint64_t rc) {
  const u32x4 k = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  uint64_t b, e, step, first;
  if (PAT == 1 || PAT == 4 || PAT == 5 || PAT == 6) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    b = wave * rc;
    e = b + rc < n ? b + rc : n;
    step = 64;
    first = b + (threadIdx.x & 63);
  } else {
    b = 0;
    e = n;
    step = (uint64_t)gridDim.x * blockDim.x;
    first = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  }
  if (b >= e) return;
  if (PAT == 6) {
    lane_groups<U, POL, SRC_OFF>(src, dst, b, e);
    return;
  }
  u32x4 acc = {0, 0, 0, 0};
  if (PAT == 5) {  // the hole chunks of this wave's region, up front
    for (uint64_t c = b + (threadIdx.x & 63) * 85; c < e; c += 64 * 85) {
      st<POL>(dst + 16 * c, ld<POL>(src + 16 * c + SRC_OFF) ^ k);
      if (c + 84 < e) st<POL>(dst + 16 * (c + 84), ld<POL>(src + 16 * (c + 84) + SRC_OFF) ^ k);
    }
  }
  for (uint64_t c0 = first; c0 < e; c0 += step * U) {
    u32x4 v[U];
    if (PAT != 3) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t c = c0 + u * step;
        c = c < e ? c : e - 1;
        v[u] = ld<POL>(src + 16 * c + SRC_OFF);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t c = c0 + u * step;
      if (PAT == 2) acc ^= v[u];
      else if (c < e && (PAT < 4 || (c % 85 != 0 && c % 85 != 84)))
        st<POL>(dst + 16 * c, PAT == 3 ? k + (uint32_t)c : v[u] ^ k);
    }
  }
  if (PAT == 2 && acc.x == 0x12345678u) st<0>(dst, acc);
}

static uint32_t g_lds = 0;  // dynamic LDS per block: caps blocks per CU
template <int PAT, int U, int POL, int OFF>
static void go(const void *s, void *d, uint64_t n, uint64_t rc, uint64_t g, hipStream_t st) {
  hipLaunchKernelGGL((probe<PAT, U, POL, OFF>), dim3(g), dim3(256), g_lds, st, (const uint8_t *)s,
                     (uint8_t *)d, n, rc);
}
extern "C" void probe_set_lds(uint32_t bytes) { g_lds = bytes; }

#define CASE(P, U, POL, OFF)                                                      \
  if (pat == P && u == U && pol == POL && off == OFF) {                           \
    go<P, U, POL, OFF>(src, dst, n, rc, g, s);                                    \
    return hipGetLastError() == hipSuccess ? 0 : -1;                              \
  }
#define POLS(P, U, OFF) CASE(P, U, 0, OFF) CASE(P, U, 1, OFF) CASE(P, U, 2, OFF) CASE(P, U, 3, OFF)

extern "C" int probe_run(int pat, int u, int pol, int off, const void *src, void *dst,
                         uint64_t bytes, uint64_t region_bytes, int grid, void *stream) {
  const uint64_t n = bytes / 16, rc = region_bytes / 16;
  hipStream_t s = (hipStream_t)stream;
  uint64_t g = grid;
  if (pat == 1 || pat == 4 || pat == 5 || pat == 6) g = ((n + rc - 1) / rc + 3) / 4;
  POLS(0, 4, 0) POLS(0, 8, 0) POLS(0, 4, 8) POLS(0, 16, 0)
  POLS(1, 4, 8) POLS(1, 8, 8) POLS(1, 16, 8)
  POLS(2, 4, 0) POLS(2, 8, 0) POLS(3, 4, 0) POLS(3, 8, 0)
  POLS(4, 16, 8) POLS(5, 16, 8) POLS(4, 8, 8) POLS(5, 8, 8) POLS(6, 6, 8)
  return -2;
}
