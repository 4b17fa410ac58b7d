// Dev-only probe (not part of the product): does the ORDER in which the
// waves of a workgroup walk their bytes change the HBM copy rate?
//   MODE 0  every wave streams its own contiguous region of R chunks
//           (what obfs_kernel does today: one region per wave)
//   MODE 1  the W waves of a block share one region of W*R chunks; per step
//           wave w takes U consecutive 1-KiB rows (block covers W*U rows)
//   MODE 2  as 1, but rows are dealt round-robin (row r -> wave r % W)
// Copy-XOR with nt loads and stores, source offset 8 B (the salt shift).
// build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o build/libsqprobe2.so scripts/probe_locality.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

template <int MODE, int U, int BS>
__global__ __launch_bounds__(BS) void probe2(const uint8_t *src, uint8_t *dst, uint64_t n,
                                             uint64_t R) {
  constexpr int W = BS / 64;
  const u32x4 k = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x / 64;
  uint64_t b, e;
  if (MODE == 0) {
    b = ((uint64_t)blockIdx.x * W + w) * R;
  } else {
    b = (uint64_t)blockIdx.x * W * R;
  }
  e = b + (MODE == 0 ? R : W * R);
  e = e < n ? e : n;
  if (b >= e) return;
  const uint64_t step = MODE == 0 ? 64 * U : 64 * U * W;
  for (uint64_t c0 = b; c0 < e; c0 += step) {
    uint64_t c[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (MODE == 0) c[u] = c0 + 64 * u + lane;
      else if (MODE == 1) c[u] = c0 + 64 * (w * U + u) + lane;
      else c[u] = c0 + 64 * (u * W + w) + lane;
    }
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t cc = c[u] < e ? c[u] : e - 1;
      v[u] = __builtin_nontemporal_load((const G u32x4 *)(src + 16 * cc + 8));
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (c[u] < e) __builtin_nontemporal_store(v[u] ^ k, (G u32x4 *)(dst + 16 * c[u]));
  }
}

// MODE 3/4: persistent lockstep grid (NB blocks, all resident), rounds of
// 64 segments of SEG bytes per wave.  MODE 3 deals segment k of wave j in
// round r as r*NW*64 + k*NW + j (resident waves stream adjacent segments at
// the same time); MODE 4 gives each wave 64 consecutive segments per round.
// DUMMY = dependent VALU ops per step (an interleaved hash round's cost).
template <int MODE, int U, int DUMMY>
__global__ __launch_bounds__(256) void probe_pers(const uint8_t *src, uint8_t *dst, uint64_t nseg,
                                                  uint32_t *sink) {
  constexpr uint32_t SEG = 1360, CPS = SEG / 16;  // 85 chunks per segment
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t NW = (uint64_t)gridDim.x * 4, j = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const u32x4 key = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  uint32_t acc = lane;
  for (uint64_t r = 0; r * NW * 64 < nseg; r++) {
    const uint32_t T = 64 * CPS;
    for (uint32_t c0 = 0; c0 < T; c0 += 64 * U) {
      uint64_t sa[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t c = c0 + 64 * u + lane;
        const uint32_t k = c / CPS, w = c - k * CPS;
        const uint64_t seg = MODE == 3 ? r * NW * 64 + k * NW + j : (r * NW + j) * 64 + k;
        ok[u] = c < T && seg < nseg;
        sa[u] = (ok[u] ? seg : 0) * SEG + 16 * w;
      }
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load((const G u32x4 *)(src + sa[u] + 8));
#pragma unroll
      for (int d = 0; d < DUMMY; d++) acc = __builtin_amdgcn_alignbit(acc, acc * 3u + d, 7);
#pragma unroll
      for (int u = 0; u < U; u++)
        if (ok[u]) __builtin_nontemporal_store(v[u] ^ key, (G u32x4 *)(dst + sa[u]));
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int MODE, int U, int DUMMY>
static int gop(const void *s, void *d, uint64_t bytes, int nb, hipStream_t st) {
  hipLaunchKernelGGL((probe_pers<MODE, U, DUMMY>), dim3(nb), dim3(256), 0, st, (const uint8_t *)s,
                     (uint8_t *)d, bytes / 1360, (uint32_t *)d);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int probe_pers_run(int mode, int u, int dummy, int nb, const void *src, void *dst,
                              uint64_t bytes, void *stream) {
  hipStream_t s = (hipStream_t)stream;
#define PC(M, U, D) \
  if (mode == M && u == U && dummy == D) return gop<M, U, D>(src, dst, bytes, nb, s);
  PC(3, 6, 0) PC(4, 6, 0) PC(3, 6, 200) PC(4, 6, 200) PC(3, 4, 0) PC(3, 8, 0)
  return -2;
}

// MODE 5: as MODE 0 (one region per wave, U KiB per step), but the loads are
// LDS-DMA (global_load_lds_dwordx4: no VGPR destination) into a per-wave
// LDS buffer, then ds_read_b128 + XOR + nt store.  AUX: load cache policy.
template <int U, int AUX>
__global__ __launch_bounds__(256) void probe_glds(const uint8_t *src, uint8_t *dst, uint64_t n,
                                                  uint64_t R) {
  __shared__ u32x4 buf[4][U][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const u32x4 k = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  const uint64_t b = ((uint64_t)blockIdx.x * 4 + w) * R;
  uint64_t e = b + R;
  e = e < n ? e : n;
  if (b >= e) return;
  for (uint64_t c0 = b; c0 < e; c0 += 64 * U) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t c = c0 + 64 * u + lane;
      c = c < e ? c : e - 1;
      __builtin_amdgcn_global_load_lds((const void *)(src + 16 * c + 8),
                                       (__attribute__((address_space(3))) void *)&buf[w][u][0],
                                       16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t c = c0 + 64 * u + lane;
      const u32x4 v = buf[w][u][lane];
      if (c < e) __builtin_nontemporal_store(v ^ k, (G u32x4 *)(dst + 16 * c));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

extern "C" int probe_glds_run(int u, int aux, const void *src, void *dst, uint64_t bytes,
                              uint64_t region_bytes, void *stream) {
  const uint64_t n = bytes / 16, R = region_bytes / 16;
  const uint64_t g = ((n + R - 1) / R + 3) / 4;
  hipStream_t s = (hipStream_t)stream;
#define GC(UU, AA)                                                                          \
  if (u == UU && aux == AA) {                                                              \
    hipLaunchKernelGGL((probe_glds<UU, AA>), dim3(g), dim3(256), 0, s, (const uint8_t *)src, \
                       (uint8_t *)dst, n, R);                                              \
    return hipGetLastError() == hipSuccess ? 0 : -1;                                       \
  }
  GC(4, 0) GC(4, 2) GC(8, 0) GC(8, 2) GC(6, 2)
  return -2;
}

template <int MODE, int U, int BS>
static int go(const void *s, void *d, uint64_t n, uint64_t R, hipStream_t st) {
  constexpr int W = BS / 64;
  const uint64_t regions = (n + R - 1) / R;
  const uint64_t g = (regions + W - 1) / W;
  hipLaunchKernelGGL((probe2<MODE, U, BS>), dim3(g), dim3(BS), 0, st, (const uint8_t *)s,
                     (uint8_t *)d, n, R);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

#define CASE(M, U, BS) \
  if (mode == M && u == U && bs == BS) return go<M, U, BS>(src, dst, n, rc, s);
#define MODES(U, BS) CASE(0, U, BS) CASE(1, U, BS) CASE(2, U, BS)

extern "C" int probe2_run(int mode, int u, int bs, const void *src, void *dst, uint64_t bytes,
                          uint64_t region_bytes, void *stream) {
  const uint64_t n = bytes / 16, rc = region_bytes / 16;
  hipStream_t s = (hipStream_t)stream;
  MODES(4, 256) MODES(6, 256) MODES(8, 256) MODES(4, 512) MODES(6, 512) MODES(4, 1024)
  return -2;
}
