// sq_cpu.h -- the product's CPU transform: Salamander / XPlus over a ragged
// batch in host memory, with the semantics of a device launch
// (include/sqobfs.h, "Semantics per packet i").
//
// Where it runs (never as a stand-in for a working GPU's bulk path):
//   * sqobfs_pconn engines without a GPU (sqobfs_keyring_create with ctx
//     NULL) -- the reference's constructors cannot fail
//     (hysteria2/salamander.go:24-40, hysteria/xplus.go:19-37), so neither
//     may NewSalamanderConn / NewXPlusPacketConn here;
//   * batches too small to repay a launch (a lone handshake or ACK datagram:
//     ~1 us of byte work against ~30 us for a launch round trip);
//   * a batch whose launch failed, and every batch after it.
// The reference does this byte work per datagram on the caller's goroutine
// (salamander.go:42-70, xplus.go:46-75); this code does the same per batch.
//
// Self-contained: its own BLAKE2b (RFC 7693), SHA-256 (FIPS 180-4) and
// ChaCha20 (RFC 8439); nothing from oracle/ (the test checker) is linked.
// Plain C++17, no HIP: the engine builds and runs without a GPU runtime
// (the sanitizer builds of tests/cpp, scripts/dev/cpu_sanitize.sh).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "sq_internal.h"
#include "sqobfs.h"

namespace sq {
namespace cpu {

// BLAKE2b compression F (RFC 7693 section 3.2) and SHA-256 compression.
void b2_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last);
void s2_compress(uint32_t st[8], const uint32_t m[16]);
// ChaCha20 block function (RFC 8439 section 2.3).
void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3],
                    uint32_t out[16]);

// The per-PSK hash state of one keyring entry, laid out exactly as the GPU's
// psk_prepare_kernel lays it out (sq_internal.h PskEntry), so host and device
// entries can be compared byte for byte.
void psk_prepare(int kind, const uint8_t *psk, uint32_t len, PskEntry *e);

// key = BLAKE2b-256(psk || salt8) (salamander.go:50,61) or
// SHA-256(psk || salt16) (xplus.go:54,70), from the entry's midstate.
void derive_key(const PskEntry &e, const uint8_t *salt, uint8_t key[32]);
// The keys of n <= kKeyBatch packets (es[k]'s PSK, salts[k] its salt, S
// bytes of 16); one-block entries by the multi-buffer compressions
// (BLAKE2b: 8 at once with AVX-512, 4 with AVX2; SHA-256: 16 / 8).  All
// entries of one call are of one kind (one keyring).
constexpr uint32_t kKeyBatch = 64;
void derive_keys(const PskEntry *const *es, const uint8_t (*salts)[16], uint32_t n,
                 uint8_t (*keys)[32]);

// dst[j] = src[j] ^ key[j % 32], j < n.  dst == src (in place) or disjoint,
// or dst below src (the reference's left shift by the salt, salamander.go:51).
void xor_stream(uint8_t *dst, const uint8_t *src, size_t n, const uint8_t key[32]);

// The n * S salts of one SQOBFS_FLAG_DEVICE_SALT batch: the same ChaCha20
// keystream the GPU generates (include/sqobfs.h), nonce "sqob" || le64(seq).
void salt_stream(const uint32_t key[8], uint64_t seq, uint8_t *out, size_t bytes);

// One host batch, single thread.  table[count]: the keyring's host entries.
// salts: obfuscate with SQOBFS_FLAG_DEVICE_SALT -- the batch's n * S salts
// (salt_stream), else NULL (b->salt is read).  Per-packet results as a
// launch: out_len = SQOBFS_BAD_PSK for a psk_id out of range, 0xFFFFFFFE for
// a length past 2^26 (sq_kernels.hip kBadLen).  SQ_OK or SQ_EINVAL.
int run_batch(int kind, int dir, const PskEntry *table, uint32_t count, const sqobfs_batch *b,
              const uint8_t *salts);

}  // namespace cpu
}  // namespace sq
