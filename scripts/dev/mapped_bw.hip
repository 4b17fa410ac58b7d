// Dev probe (GPU box): what a kernel moves over PCIe on page-locked host
// memory it reads and writes directly (zero copy), by allocation flag, size
// and grid -- the bound of the packet conn engine's GPU route (DESIGN.md
// 9.5).  In place (read + write each byte once, as the engine's launch),
// read only and write only; 16 B per lane, kU loads in flight per lane
// before its stores.  Prints one JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 -o build/mapped_bw scripts/dev/mapped_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int kU = 4;

__global__ void __launch_bounds__(256) inplace(uint4 *p, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * kU;
  for (size_t b = ((size_t)blockIdx.x * blockDim.x) * kU + threadIdx.x; b < n16; b += stride) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n16) v[u] = p[i];
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n16) p[i] = make_uint4(v[u].x ^ 0x5a5a5a5au, v[u].y ^ 1u, v[u].z, v[u].w ^ 7u);
    }
  }
}

__global__ void __launch_bounds__(256) readonly(const uint4 *p, size_t n16, uint32_t *sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * kU;
  uint32_t acc = 0;
  for (size_t b = ((size_t)blockIdx.x * blockDim.x) * kU + threadIdx.x; b < n16; b += stride) {
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n16) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) writeonly(uint4 *p, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// device in, mapped host out (the inbound bytes came by DMA)
__global__ void __launch_bounds__(256) dev2host(const uint4 *src, uint4 *dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * kU;
  for (size_t b = ((size_t)blockIdx.x * blockDim.x) * kU + threadIdx.x; b < n16; b += stride) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n16) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n16) dst[i] = make_uint4(v[u].x ^ 0x5a5a5a5au, v[u].y ^ 1u, v[u].z, v[u].w ^ 7u);
    }
  }
}

// Staged variants over one page-locked buffer of `bytes`, split into
// `chunks` pieces on `ns` streams (piece i on stream i % ns):
//   hybrid: H2D copy of the piece, then a kernel reading it from HBM and
//           writing the result to the host buffer directly;
//   staged: H2D copy, kernel in place in HBM, D2H copy.
int staged(int reps) {
  const size_t sizes[] = {1u << 20, 5530000, 22118400};
  const int chunk_opts[] = {1, 2, 4, 8};
  const size_t cap = sizes[2];
  void *h;
  CK(hipHostMalloc(&h, cap, hipHostMallocDefault));
  memset(h, 1, cap);
  void *hd;
  CK(hipHostGetDevicePointer(&hd, h, 0));
  void *d;
  CK(hipMalloc(&d, cap));
  hipStream_t st[2];
  for (auto &x : st) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t e0, e1, j[2];
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &x : j) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  for (int mode = 0; mode < 2; mode++)
    for (size_t bytes : sizes)
      for (int chunks : chunk_opts)
        for (int ns = 1; ns <= 2; ns++) {
          if (ns == 2 && chunks == 1) continue;
          const size_t piece = (bytes / chunks + 15) & ~(size_t)15;
          auto run = [&] {
            // both streams start after the previous repetition's end
            CK(hipEventRecord(j[0], st[0]));
            CK(hipStreamWaitEvent(st[1], j[0], 0));
            for (int c = 0; c < chunks; c++) {
              const size_t off = c * piece;
              if (off >= bytes) break;
              const size_t len = bytes - off < piece ? bytes - off : piece;
              hipStream_t s = st[c % ns];
              uint8_t *hp = (uint8_t *)h + off, *hdp = (uint8_t *)hd + off, *dp = (uint8_t *)d + off;
              CK(hipMemcpyAsync(dp, hp, len, hipMemcpyHostToDevice, s));
              const int g = (int)((len / 16 + 256 * kU - 1) / (256 * kU));
              if (mode == 0) {
                dev2host<<<g, 256, 0, s>>>((const uint4 *)dp, (uint4 *)hdp, len / 16);
              } else {
                inplace<<<g, 256, 0, s>>>((uint4 *)dp, len / 16);
                CK(hipMemcpyAsync(hp, dp, len, hipMemcpyDeviceToHost, s));
              }
            }
            CK(hipEventRecord(j[1], st[1]));
            CK(hipStreamWaitEvent(st[0], j[1], 0));
          };
          for (int w = 0; w < 3; w++) run();
          CK(hipStreamSynchronize(st[0]));
          CK(hipEventRecord(e0, st[0]));
          for (int r = 0; r < reps; r++) run();
          CK(hipEventRecord(e1, st[0]));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          const double us = ms * 1e3 / reps;
          printf("{\"alloc\": \"default\", \"bytes\": %zu, \"chunks\": %d, \"streams\": %d, "
                 "\"kernel\": \"%s\", \"us\": %.1f, \"GBps\": %.2f}\n",
                 bytes, chunks, ns, mode == 0 ? "hybrid" : "staged", us, bytes / us / 1e3);
          fflush(stdout);
        }
  CK(hipFree(d));
  CK(hipHostFree(h));
  return 0;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  if (argc > 2 && !strcmp(argv[2], "staged")) return staged(reps);
  struct Alloc {
    const char *name;
    unsigned flags;
    bool reg;
  } allocs[] = {{"default", hipHostMallocDefault, false},
                {"coherent", hipHostMallocCoherent, false},
                {"noncoherent", hipHostMallocNonCoherent, false},
                {"registered", 0, true}};
  const size_t sizes[] = {1u << 20, 5530000, 22118400, 88473600};
  const int grids[] = {256, 1024, 4096};
  uint32_t *sink;
  CK(hipMalloc(&sink, 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Alloc &a : allocs) {
    const size_t cap = sizes[3];
    void *h = nullptr;
    if (a.reg) {
      h = aligned_alloc(4096, cap);
      memset(h, 1, cap);
      CK(hipHostRegister(h, cap, hipHostRegisterMapped));
    } else {
      CK(hipHostMalloc(&h, cap, a.flags));
      memset(h, 1, cap);
    }
    void *d = nullptr;
    CK(hipHostGetDevicePointer(&d, h, 0));
    for (size_t bytes : sizes) {
      const size_t n16 = bytes / 16;
      for (int g : grids) {
        for (int k = 0; k < 3; k++) {
          const char *kn = k == 0 ? "inplace" : k == 1 ? "read" : "write";
          auto run = [&] {
            if (k == 0) inplace<<<g, 256, 0, s>>>((uint4 *)d, n16);
            else if (k == 1) readonly<<<g, 256, 0, s>>>((const uint4 *)d, n16, sink);
            else writeonly<<<g, 256, 0, s>>>((uint4 *)d, n16);
          };
          for (int w = 0; w < 3; w++) run();
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          for (int r = 0; r < reps; r++) run();
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          const double us = ms * 1e3 / reps;
          printf("{\"alloc\": \"%s\", \"bytes\": %zu, \"grid\": %d, \"kernel\": \"%s\", "
                 "\"us\": %.1f, \"GBps\": %.2f}\n",
                 a.name, bytes, g, kn, us, bytes / us / 1e3);
          fflush(stdout);
        }
      }
    }
    if (a.reg) {
      CK(hipHostUnregister(h));
      free(h);
    } else {
      CK(hipHostFree(h));
    }
  }
  return 0;
}
