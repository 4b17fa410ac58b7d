// microbenchmark: issue cost of 64-bit add forms on gfx950 (dev only)
#include <hip/hip_runtime.h>
#include <stdint.h>
template <int MODE>
__global__ void mb(uint64_t *out, uint64_t seed, long long *cyc) {
  uint64_t a[8];
  for (int i = 0; i < 8; i++) a[i] = seed * (i + threadIdx.x + 1);
  const long long t0 = clock64();
  for (int it = 0; it < 256; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (MODE == 0) a[i] = a[i] + a[(i + 1) & 7];                 // v_lshl_add_u64
      if (MODE == 1) {                                               // add_co / addc_co
        uint32_t lo, hi;
        asm volatile("v_add_co_u32 %0, vcc, %2, %3\n\tv_addc_co_u32 %1, vcc, %4, %5, vcc"
                     : "=v"(lo), "=v"(hi)
                     : "v"((uint32_t)a[i]), "v"((uint32_t)a[(i + 1) & 7]),
                       "v"((uint32_t)(a[i] >> 32)), "v"((uint32_t)(a[(i + 1) & 7] >> 32))
                     : "vcc");
        a[i] = ((uint64_t)hi << 32) | lo;
      }
      if (MODE == 2) a[i] = a[i] ^ a[(i + 1) & 7];                 // 2x v_xor_b32
      if (MODE == 3) a[i] = (a[i] >> 24) | (a[i] << 40);           // rotate: 2x alignbit
    }
  }
  const long long t1 = clock64();
  uint64_t x = 0;
  for (int i = 0; i < 8; i++) x ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
extern "C" int mb_run(int mode, int blocks, int threads, uint64_t *out, long long *cyc) {
  if (mode == 0) hipLaunchKernelGGL(mb<0>, dim3(blocks), dim3(threads), 0, 0, out, 12345, cyc);
  if (mode == 1) hipLaunchKernelGGL(mb<1>, dim3(blocks), dim3(threads), 0, 0, out, 12345, cyc);
  if (mode == 2) hipLaunchKernelGGL(mb<2>, dim3(blocks), dim3(threads), 0, 0, out, 12345, cyc);
  if (mode == 3) hipLaunchKernelGGL(mb<3>, dim3(blocks), dim3(threads), 0, 0, out, 12345, cyc);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
