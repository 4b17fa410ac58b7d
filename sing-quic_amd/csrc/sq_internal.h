// sq_internal.h -- layouts shared by the host C-ABI (sq_api.hip) and the
// gfx950 kernels (sq_kernels.hip).  Not part of the public ABI.
#pragma once

#include <stdint.h>

namespace sq {

constexpr int kSalamanderSalt = 8;  // hysteria2/salamander.go:15
constexpr int kXPlusSalt = 16;      // hysteria/xplus.go:17
constexpr int kWave = 64;           // CDNA wavefront
// Obfuscation kernel unit: packets per wavefront (sqobfs_set_unit_packets);
// two more lanes hold the unit's neighbour packets.

constexpr uint32_t kDefaultUnitPackets = 26;
constexpr uint32_t kMaxUnitPackets = 62;
// Sized by bytes when the batch's lengths are known (sqobfs_unit_packets_for):
// about this many payload bytes per wavefront (~21.7 KB
// per wave streams best; per-packet keyring gathers want longer units).
// (multi-PSK: 23 packets of 1,350 B.  In-process sweeps on three boxes,
// profiles/r03/ab/unit_sweep_256psk_*: 23 within 1.2 % of each box's best
// in both directions; 24 -- ~32 KB, consecutive waves' spans close to a
// power of two apart -- the slowest point on two of the three boxes.)
constexpr uint64_t kUnitBytes = 21700, kUnitBytesMultiPsk = 31500;
// XPlus with one PSK: 16 packets of 1,200 B beat 18 by 0.7-1.7 % in both
// directions on three boxes (unit size)
constexpr uint64_t kUnitBytesXPlus = 19500;
// ... but at least this many wavefronts per launch when the batch is small
// (latency: a socket batch of 256 datagrams runs as 256 one-packet waves)
constexpr uint32_t kMinUnits = 2048;

// Per-PSK hash state, derived once per keyring on the GPU (psk_prepare).
//
// Both hashes are Merkle-Damgard-style over psk || salt, and the PSK is the
// same for every packet of a connection (the `password` field captured by
// NewSalamanderConn, hysteria2/salamander.go:19-40).  So every block made of
// PSK bytes only is compressed once here, and the per-packet kernel starts
// from the chaining value `h` with a message template `m` that already holds
// the PSK tail (and, for SHA-256, the 0x80 pad byte and the bit length).  The
// packet's salt is OR-ed into `m` at byte `salt_pos`, giving 1 compression
// per packet for PSKs up to 120 B (BLAKE2b) / 39 B (SHA-256), at most 2 for
// any PSK length.
struct alignas(16) PskEntry {
  uint64_t h[8];     // BLAKE2b chaining value | SHA-256: 8 u32 in h32()
  uint64_t m[32];    // final block(s): BLAKE2b 2x16 LE u64 words |
                     // SHA-256 2x16 BE u32 words packed in the first 128 B
  uint64_t t_first;  // BLAKE2b byte counter for block 1 when nblocks == 2
  uint64_t t_last;   // BLAKE2b byte counter for the final block
  uint32_t nblocks;  // 1 or 2 compressions per packet
  uint32_t salt_pos; // byte offset of the salt inside the final block(s)
  uint32_t psk_len;
  uint32_t kind;     // sqobfs_kind
};
static_assert(sizeof(PskEntry) == 352, "PskEntry layout");

// Kernel arguments.  psk0 is the keyring's entry 0 passed by value, so the
// single-PSK kernels read the hash state from the kernarg segment (scalar
// loads, wave-uniform) instead of gathering it per lane.
struct KParams {
  const uint8_t *in;
  const uint64_t *in_off;
  const uint32_t *in_len;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *out_len;
  const uint8_t *salt;
  const uint16_t *psk_id;
  const uint32_t *in_cap;
  const PskEntry *psk_table;
  uint8_t *salt_out;        // device salts: [n*S] copy of the generated salts, or NULL
  uint32_t n;
  uint32_t n_psk;
  uint32_t device_salt;     // 1: obfuscate salts from ChaCha20(salt_key, salt_nonce)
  uint32_t ppw;             // packets per wavefront (unit size), 1 .. 62; 0 = default
  uint32_t out_blocks;      // 1: SQOBFS_FLAG_OUT_BLOCKS (outputs own their 16-byte blocks)
  uint32_t out_lines;       // 1: SQOBFS_FLAG_OUT_LINES (... and their last 128-byte line)
  uint32_t xcd;             // 1: XCD-contiguous units (set by the launcher: large batches)
  uint32_t psk_hot_m;       // multi-PSK: words of entry block 0 any entry needs (the rest are 0)
  uint32_t psk_hot_iv;      // multi-PSK: 1 when no entry has PSK-only blocks (h = initial state)
  uint32_t salt_key[8];
  uint32_t salt_nonce[3];
  PskEntry psk0;
};

// QUIC 1-RTT keys of one connection as little-endian words (ChaCha20 state
// order): key, iv (nonce base), hp (header protection key).
struct QuicKeyDev {
  uint32_t key[8];
  uint32_t iv[3];
  uint32_t hp[8];
  uint32_t pad;
};
static_assert(sizeof(QuicKeyDev) == 80, "QuicKeyDev layout");

// QUIC packet protection launch (sq_quic.hip); key0 = keyring entry 0 by
// value (single-connection batches read it from the kernarg segment).
struct QParams {
  const uint8_t *in;
  const uint64_t *in_off;
  const uint32_t *in_len;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *out_len;
  const uint16_t *pn_offset;
  const uint64_t *pn;
  const uint16_t *key_id;
  uint64_t *pn_out;
  const QuicKeyDev *keys;
  uint32_t n;
  uint32_t n_keys;
  QuicKeyDev key0;
  // fused Salamander layer (sqobfs_quic_seal_salamander / _open_salamander):
  // the QUIC packet travels as salt8 || packet ^ BLAKE2b-256(psk || salt8)
  const uint8_t *osalt;  // seal: [n*8] salts (device)
  uint32_t obfs;         // 1: fused path
  uint32_t pad_;
  PskEntry opsk;         // the Salamander keyring's entry 0
};

// AES-128-GCM (TLS_AES_128_GCM_SHA256) connection keys on the device:
// AES-128 key schedules of the payload key and the header-protection key as
// little-endian column words (word 4r + c = bytes 4c..4c+3 of round key r),
// the IV, per-position tables of H (hpos[j][n] = n x^(4 (31 - j)) H: X * H is
// the XOR of hpos[j][nibble j of X], 32 independent lookups, no shifts), and
// 4-bit GHASH tables of H^4, H^8, .. H^(4 kGcmPow4) (Shoup's method; slot
// n ^ (j & 15) of table j = the nibble polynomial n times H^(4 (j + 1)), as
// big-endian words): the cooperative pass cuts a payload into 4-block chunks
// aligned to its last full block, so a chunk's partial GHASH is placed by a
// power of H^4.
constexpr uint32_t kGcmPow = 128;  // payload blocks of the cooperative pass (2,048 B)
constexpr uint32_t kGcmPow4 = kGcmPow / 4;
struct QuicGcmKeyDev {
  uint32_t rk[44];   // AES-128 key schedule, words 4..39 (rounds 1-9) rotated
  uint32_t hrk[44];  // by 16 bits (sq_quic_gcm.hip aes_encrypt_n); hrk: the HP key's
  uint32_t iv[3];
  uint32_t pad;
  uint32_t hpos[32][16][4];
  uint32_t htab[kGcmPow4][16][4];
};

// AES-128-GCM launch; rk0 / hrk0 / iv0 = keyring entry 0 (kernarg); t0 = the
// 256-word AES T-table (device, 1 KiB), staged into LDS by every block.
struct QGParams {
  const uint8_t *in;
  const uint64_t *in_off;
  const uint32_t *in_len;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *out_len;
  const uint16_t *pn_offset;
  const uint64_t *pn;
  const uint16_t *key_id;
  uint64_t *pn_out;
  const uint32_t *perm;  // multi-key: packet indices grouped by key (or null)
  const uint32_t *gmeta; // grouped: per key start | count | first step, steps
  const QuicGcmKeyDev *keys;
  const uint32_t *t0;
  uint32_t n;
  uint32_t n_keys;
  uint32_t rk0[44];
  uint32_t hrk0[44];
  uint32_t iv0[3];
  uint32_t obfs;         // 1: fused Salamander layer (as QParams)
  const uint8_t *osalt;  // seal: [n*8] salts (device)
  PskEntry opsk;         // the Salamander keyring's entry 0
};

}  // namespace sq

// host helpers implemented in sq_api.hip
// poll a stream for up to `us` microseconds: 0 = drained, 1 = still busy, <0 error
int sq_spin_wait(void *stream, uint32_t us);
// packets per wavefront of a device batch of n packets (lengths unknown)
uint32_t sq_unit_packets_default(uint32_t n);
// ---- the device interface of the host engines (pconn.cpp, udp_batch.cpp).
// Implemented by sq_api.hip; tests/cpp/sq_devstub.cpp implements the same
// functions over a CPU "device" for the sanitizer builds (no HIP at all).
// private streams of host engines (pconn.cpp) on a context's GPU
struct sqobfs_ctx;
int sq_ctx_stream_create(sqobfs_ctx *ctx, void **out);
void sq_ctx_stream_destroy(sqobfs_ctx *ctx, void *s);
int sq_ctx_stream_wait(sqobfs_ctx *ctx, void *s, uint32_t spin_us);
// wait without holding a core: sleep nap_us, then poll with short sleeps
// (an event with hipEventBlockingSync after ~2 ms)
int sq_ctx_stream_wait_blocking(sqobfs_ctx *ctx, void *s, uint32_t nap_us);
// a synchronised library stream about to be destroyed: drop it from the
// keyring's release fence (sqobfs_keyring_destroy)
struct sqobfs_keyring;
void sq_keyring_forget(const sqobfs_keyring *kr, void *s);
// page-locked host memory the context's GPU reads and writes at the same
// address (zero-copy batches); freed with sqobfs_host_free
int sq_host_alloc_mapped(sqobfs_ctx *ctx, size_t bytes, void **out);
// the keyring's host copy of its per-PSK state (sq_cpu.h), and its context
// (NULL for a host keyring)
const sq::PskEntry *sq_keyring_host(const sqobfs_keyring *kr, uint32_t *count);
sqobfs_ctx *sq_keyring_ctx(const sqobfs_keyring *kr);
// the keyring's multi-PSK gather words (sq_api.hip keyring_hot_words)
void sq_keyring_hot(const sqobfs_keyring *kr, uint32_t *hot_m, uint32_t *hot_iv);
// a device keyring whose entries are copies of host entries (sq_keyring_host
// of other keyrings; hot_m / hot_iv: the max / min of theirs): the engine's
// merged keyrings, one launch over several pconns' batches (pconn.cpp); the
// table is copied and waited for on `stream` (NULL: the context's stream)
int sq_keyring_from_entries(sqobfs_ctx *ctx, int kind, const sq::PskEntry *e, uint32_t count,
                            uint32_t hot_m, uint32_t hot_iv, void *stream,
                            sqobfs_keyring **out);
// one sequence number of the context's salt stream (SQOBFS_FLAG_DEVICE_SALT)
// and its key, for salts made on the host; ctx NULL: the process's host
// generator (sq_cpu.cpp)
void sq_salt_take(sqobfs_ctx *ctx, uint32_t key[8], uint64_t *seq);
// the process's host salt generator (sq_cpu.cpp): random key, own sequence
void sq_host_salt_take(uint32_t key[8], uint64_t *seq);
// sqobfs_close: ends the context's packet conn engine (pconn.cpp)
void sq_engine_ctx_closed(sqobfs_ctx *ctx);

// launchers implemented in sq_quic_gcm.hip
extern "C" int sq_launch_quic_gcm(int open, const sq::QGParams *qp, void *stream);
// Multi-key AES-128-GCM batches: the packet permutation that groups them by
// key (stable counting sort) and the per-key step table of the staged
// kernel; packets with an out-of-range key id are rejected there (out_len,
// pn_out) and take no step.  sq_gcm_group_scratch: the device scratch it
// needs (perm[n] | histograms | meta), 0 when such a batch is not grouped
// (too few packets per key, or too many keys).  sq_launch_gcm_group returns
// 1 when not grouped, 0 on success, < 0 on a launch error; *meta = the
// step table inside scratch.
extern "C" uint64_t sq_gcm_group_scratch(uint32_t n, uint32_t n_keys);
extern "C" int sq_launch_gcm_group(const uint16_t *key_id, uint32_t n, uint32_t n_keys,
                                   int open, uint32_t *out_len, uint64_t *pn_out,
                                   void *scratch, const uint32_t **meta, void *stream);

// launchers implemented in sq_quic.hip
extern "C" int sq_launch_quic(int open, const sq::QParams *qp, void *stream);

// launchers implemented in sq_kernels.hip
// the calling thread's next obfuscation launch records these events with its
// dispatch (sqobfs_debug_time_next_launch)
extern "C" void sq_time_next_launch(void *start, void *stop);
extern "C" int sq_launch_obfs(int kind, int dir, const sq::KParams *kp,
                              void *stream);
extern "C" int sq_launch_psk_prepare(int kind, const uint8_t *blob,
                                     const uint64_t *off, const uint32_t *len,
                                     uint32_t count, sq::PskEntry *out,
                                     void *stream);
