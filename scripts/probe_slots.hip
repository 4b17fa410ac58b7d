// Dev-only probe (not part of the product): HBM rate of a copy over fixed
// slots, to tell apart what a slotted batch costs the obfuscation kernel.
// Each wave copies `per` consecutive slots of `stride` bytes; in each slot it
// reads blocks [0, nbr) and writes blocks [0, nbw) (16 B each; written blocks
// past nbr carry a constant: slot padding the caller declared scratch).
// build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o build/libsqslots.so scripts/probe_slots.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(128) void slots_kernel(const uint8_t *src, uint8_t *dst,
                                                    uint32_t nslot, uint32_t stride,
                                                    uint32_t nbr, uint32_t nbw, uint32_t per) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 2 + threadIdx.x / 64;
  const uint64_t s0 = (uint64_t)wave * per;
  if (s0 >= nslot) return;
  const uint32_t ns = (uint32_t)(nslot - s0 < per ? nslot - s0 : per);
  const uint32_t T = ns * nbw;
  const uint8_t *sb = src + s0 * stride;
  uint8_t *db = dst + s0 * stride;
  const u32x4 k = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  for (uint32_t c0 = 0; c0 < T; c0 += 64 * U) {
    u32x4 v[U];
    uint32_t off[U];
    bool st[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t c = c0 + u * 64 + lane;
      const uint32_t cc = c < T ? c : T - 1;
      const uint32_t q = cc / nbw, b = cc - q * nbw;
      off[u] = q * stride + 16 * b;
      st[u] = c < T;
      const bool rd = b < nbr;
      v[u] = rd ? __builtin_nontemporal_load((const u32x4 *)(sb + off[u])) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (st[u]) __builtin_nontemporal_store(v[u] ^ k, (u32x4 *)(db + off[u]));
  }
}

// Persistent variant: `gw` waves (a grid sized to the resident slots) loop
// over the units of `per` slots; mode 1: static striding (unit = wave + k *
// gw), mode 2: dynamic (each wave takes its next unit from a counter).
template <int U>
__global__ __launch_bounds__(128) void slots_persist(const uint8_t *src, uint8_t *dst,
                                                     uint32_t nslot, uint32_t stride,
                                                     uint32_t nbr, uint32_t nbw, uint32_t per,
                                                     uint32_t gw, int mode, uint32_t *ctr) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 2 + threadIdx.x / 64;
  const uint32_t units = (nslot + per - 1) / per;
  const u32x4 k = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
  uint32_t unit = wave;
  if (mode == 2) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(ctr, 1u);
    unit = __builtin_amdgcn_readfirstlane(t);
  }
  while (unit < units) {
    const uint64_t s0 = (uint64_t)unit * per;
    const uint32_t ns = (uint32_t)(nslot - s0 < per ? nslot - s0 : per);
    const uint32_t T = ns * nbw;
    const uint8_t *sb = src + s0 * stride;
    uint8_t *db = dst + s0 * stride;
    for (uint32_t c0 = 0; c0 < T; c0 += 64 * U) {
      u32x4 v[U];
      uint32_t off[U];
      bool st[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t c = c0 + u * 64 + lane;
        const uint32_t cc = c < T ? c : T - 1;
        const uint32_t q = cc / nbw, b = cc - q * nbw;
        off[u] = q * stride + 16 * b;
        st[u] = c < T;
        const bool rd = b < nbr;
        v[u] = rd ? __builtin_nontemporal_load((const u32x4 *)(sb + off[u])) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < U; u++)
        if (st[u]) __builtin_nontemporal_store(v[u] ^ k, (u32x4 *)(db + off[u]));
    }
    if (mode == 2) {
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(ctr, 1u);
      unit = __builtin_amdgcn_readfirstlane(t);
    } else {
      unit += gw;
    }
  }
}

// dynamic LDS per 2-wave workgroup: caps the resident waves like the
// obfuscation kernel's 22 KB (6 groups per CU = 3 waves per SIMD at 24 KB)
static uint32_t g_lds = 0;
extern "C" void slots_set_lds(uint32_t bytes) { g_lds = bytes; }

extern "C" int slots_persist_run(const void *src, void *dst, uint32_t nslot, uint32_t stride,
                                 uint32_t nbr, uint32_t nbw, uint32_t per, uint32_t gw, int mode,
                                 uint32_t *ctr, hipStream_t s) {
  if (nbr > nbw || 16 * nbw > stride || per == 0 || gw == 0 || (gw & 1)) return -1;
  if (mode == 2 && hipMemsetAsync(ctr, 0, 4, s) != hipSuccess) return -3;
  hipLaunchKernelGGL(slots_persist<4>, dim3(gw / 2), dim3(128), g_lds, s, (const uint8_t *)src,
                     (uint8_t *)dst, nslot, stride, nbr, nbw, per, gw, mode, ctr);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int slots_run(const void *src, void *dst, uint32_t nslot, uint32_t stride, uint32_t nbr,
                         uint32_t nbw, uint32_t per, int u, hipStream_t s) {
  if (nbr > nbw || 16 * nbw > stride || per == 0) return -1;
  const uint64_t waves = (nslot + per - 1) / per;
  const dim3 grid((uint32_t)((waves + 1) / 2)), block(128);
  if (u == 4)
    hipLaunchKernelGGL(slots_kernel<4>, grid, block, g_lds, s, (const uint8_t *)src, (uint8_t *)dst,
                       nslot, stride, nbr, nbw, per);
  else if (u == 8)
    hipLaunchKernelGGL(slots_kernel<8>, grid, block, g_lds, s, (const uint8_t *)src, (uint8_t *)dst,
                       nslot, stride, nbr, nbw, per);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
