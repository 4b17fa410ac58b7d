// Probe (GPU box): VALU issue rate of the integer ops the QUIC kernels are
// made of (v_add_u32, v_xor_b32, v_alignbit_b32 -- ChaCha20's quarter round;
// v_mad_u64_u32 -- Poly1305's limb products) against v_fma_f32, in
// wave-instructions per second for the whole chip.  Every wave runs 8
// independent chains per lane (no dependency stalls at 4+ waves per SIMD);
// the ISA of each loop body is checked by hand with --save-temps.
// build: hipcc --offload-arch=gfx950 -O3 -o probe_valu scripts/probe_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int kIters = 4096;

// 8 chains x (add, xor, alignbit) per iteration = 24 VALU per lane
__global__ void k_arx(uint32_t *out, uint32_t seed) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = seed + threadIdx.x + i; b[i] = seed ^ (i * 0x9e3779b9u); }
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a[i] += b[i];
      b[i] ^= a[i];
      b[i] = __builtin_amdgcn_alignbit(b[i], b[i], 25);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= a[i] ^ b[i];
  if (r == 0x12345678u) out[threadIdx.x] = r;
}

// 8 chains of v_mad_u64_u32 per iteration
__global__ void k_mad64(uint32_t *out, uint32_t seed) {
  uint64_t a[8];
  uint32_t m = seed | 1u;
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = (uint64_t)(uint32_t)a[i] * m + (a[i] >> 32);
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= a[i];
  if ((uint32_t)r == 0x12345678u) out[threadIdx.x] = (uint32_t)r;
}

// 8 chains of v_fma_f32 per iteration
__global__ void k_fma(uint32_t *out, uint32_t seed) {
  float a[8];
  const float m = 0.999f + seed * 1e-9f, c = 1e-7f;
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = (float)(threadIdx.x + i);
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = __builtin_fmaf(a[i], m, c);
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; i++) r += a[i];
  if (r == 1234.5f) out[threadIdx.x] = 1u;
}

template <typename K>
static void run(const char *name, K kern, int ops_per_iter, uint32_t *d) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  for (int wps : {4, 8}) {  // waves per SIMD
    const dim3 grid(cus * 4 * wps), block(64);
    hipLaunchKernelGGL(kern, grid, block, 0, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, grid, block, 0, 0, d, 2u + r);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double winstr = 5.0 * grid.x * (double)kIters * ops_per_iter;
    const double rate = winstr / (ms * 1e-3);
    const double clk = p.clockRate * 1e3;  // Hz
    printf("%-10s %d waves/SIMD: %.3f T wave-instr/s = %.2f cycles per wave-instr per SIMD "
           "(%d CUs, %.0f MHz)\n",
           name, wps, rate / 1e12, cus * 4 * clk / rate, cus, clk / 1e6);
  }
}

int main() {
  uint32_t *d;
  CHECK(hipMalloc(&d, 4096));
  run("add/xor/rot", k_arx, 24, d);
  run("mad_u64+mov", k_mad64, 16, d);  // 8 v_mad_u64_u32 + 8 v_mov_b32 per iteration
  run("pk_fma_f32", k_fma, 4, d);  // 4 v_pk_fma_f32 per iteration
  CHECK(hipFree(d));
  return 0;
}
