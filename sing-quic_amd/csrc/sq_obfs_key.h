// sq_obfs_key.h -- per-packet Salamander key derivation, shared by the
// obfuscation kernel (sq_kernels.hip) and the fused QUIC-seal + Salamander
// path (sq_quic.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sq_hash.h"
#include "sq_internal.h"

namespace sq {

// Salamander: key = BLAKE2b-256(psk || salt8) (hysteria2/salamander.go:50).
__device__ __forceinline__ void salamander_key(const PskEntry *E,
                                               const uint32_t (&salt)[4],
                                               uint32_t (&key)[8]) {
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = E->h[i];
  const uint32_t nb = E->nblocks, t = E->salt_pos;
  const uint64_t sv = b2_pack(salt[0], salt[1]);
  const uint32_t w = t >> 3, sh = (t & 7) * 8;
  const uint64_t lo = sv << sh;
  const uint64_t hi = sh ? (sv >> (64 - sh)) : 0ull;
  for (uint32_t blk = 0; blk < nb; blk++) {
    uint64_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t idx = 16 * blk + j;
      uint64_t x = E->m[idx];
      x |= (idx == w) ? lo : 0ull;
      x |= (idx == w + 1) ? hi : 0ull;
      m[j] = x;
    }
    const bool last = blk + 1 == nb;
    b2_compress(h, m, last ? E->t_last : E->t_first, last);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    key[2 * i] = (uint32_t)h[i];
    key[2 * i + 1] = (uint32_t)(h[i] >> 32);
  }
}

}  // namespace sq
