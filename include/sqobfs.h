/*
 * sqobfs.h -- C ABI of the MI355X-native Salamander / XPlus obfuscation path.
 *
 * Drop-in boundary for sing-quic's per-datagram obfuscation layer
 * (reference: /root/reference, Go module github.com/sagernet/sing-quic).
 * The reference exposes the layer only as net.PacketConn decorators; every
 * entry point below replaces the per-packet body of one of those methods with
 * a batched launch over a ragged batch of datagrams:
 *
 *   sqobfs_keyring_create        <- the `password []byte` / `key []byte` field
 *                                   captured by NewSalamanderConn
 *                                   (hysteria2/salamander.go:19-40) and
 *                                   NewXPlusPacketConn (hysteria/xplus.go:19-44)
 *   sqobfs_salamander_obfuscate  <- SalamanderPacketConn.WriteTo body
 *                                   (hysteria2/salamander.go:57-70) and
 *                                   VectorisedSalamanderPacketConn.WriteTo
 *                                   (salamander.go:81-93)
 *   sqobfs_salamander_deobfuscate<- SalamanderPacketConn.ReadFrom body
 *                                   (hysteria2/salamander.go:42-55)
 *   sqobfs_xplus_obfuscate       <- XPlusPacketConn.WriteTo body
 *                                   (hysteria/xplus.go:62-75) and
 *                                   VectorisedXPlusConn.WriteTo (xplus.go:86-98)
 *   sqobfs_xplus_deobfuscate     <- XPlusPacketConn.ReadFrom body
 *                                   (hysteria/xplus.go:46-60)
 *   sqobfs_run_host              <- the same four, for batches that live in
 *                                   host memory (socket buffers): stages
 *                                   through pinned memory, H2D, launch, D2H.
 *
 * Plain C types only (no HIP/torch types): a cgo / ctypes / JNI binding needs
 * nothing but this header (INTEGRATION.md shows the cgo stub).
 *
 * Semantics per packet i (S = 8 Salamander, 16 XPlus; key = BLAKE2b-256 or
 * SHA-256 of psk || salt):
 *   obfuscate:   out[out_off[i] .. +S)       = salt[i*S .. +S) (or the
 *                                              device salt, see
 *                                              SQOBFS_FLAG_DEVICE_SALT)
 *                out[out_off[i]+S+j]         = in[in_off[i]+j] ^ key[j % 32],
 *                                              j < in_len[i]
 *                out_len[i] = S + in_len[i]
 *   deobfuscate: n = in_len[i], wire = in[in_off[i] ..)
 *     Salamander n <= 8: the n raw bytes are copied to out (the reference
 *                returns n and leaves p untouched, salamander.go:47-49),
 *                out_len[i] = n.
 *     XPlus n < 16: nothing written, out_len[i] = 0 (xplus.go:50-52).
 *     otherwise out[out_off[i]+j] = wire[S+j] ^ key[j % 32] for
 *                j < m - S, where m = n for Salamander and
 *                m = in_cap ? in_cap[i] : n for XPlus (xplus.go:55 XORs up
 *                to len(p), the read buffer's length, not n);
 *                out_len[i] = n - S.
 * Memory rules: each packet's output bytes must not overlap any other
 * packet's output, and must either not overlap its own input or be exactly
 * in place (the payload's output address == its input address, e.g. a
 * headroom layout with out_off = in_off - S for obfuscate).  Offsets and
 * lengths are arbitrary (no alignment required); 16-byte-aligned outputs are
 * the fast case.  `salt` must be 4-byte aligned.
 */
#ifndef SQOBFS_H
#define SQOBFS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SQOBFS_ABI_VERSION 6

#define SQOBFS_SALAMANDER_SALT_LEN 8 /* hysteria2/salamander.go:15 */
#define SQOBFS_XPLUS_SALT_LEN 16     /* hysteria/xplus.go:17 */
#define SQOBFS_OBFS_TYPE_SALAMANDER "salamander" /* salamander.go:17 */

/* status codes (0 = OK, negative = error) */
#define SQ_OK 0
#define SQ_EINVAL (-1)   /* bad argument (NULL pointer, kind mismatch ...) */
#define SQ_ENOMEM (-2)   /* host or device allocation failed */
#define SQ_EDEVICE (-3)  /* HIP runtime / kernel launch error */
#define SQ_ENODEV (-4)   /* no such GPU */
#define SQ_EPSK (-5)     /* a psk_id was out of range (host-staged path) */
#define SQ_ETIMEDOUT (-6) /* a deadline passed (sqobfs_pconn_*: os.ErrDeadlineExceeded) */
#define SQ_ECLOSED (-7)   /* the endpoint is closed (sqobfs_pconn_*: net.ErrClosed) */
#define SQ_EIO (-8)       /* the wrapped conn's read failed (sqobfs_pconn_rx_fail) */
/* sqobfs_pconn_*: a socket call failed with errno e */
#define SQOBFS_ERRNO(e) (-1000 - (e))

/* batch flag (sqobfs_run_host): output bytes outside the packets' output
 * regions need not be preserved (skips copying the output range in) */
#define SQOBFS_FLAG_OUT_UNINIT 1u

/* batch flag (obfuscate only): generate every packet's salt on the GPU
 * instead of reading `salt` -- replaces the per-packet host RNG of
 * SalamanderPacketConn.WriteTo (buf.WriteRandom, salamander.go:60,83,98)
 * and XPlusPacketConn.WriteTo (math/rand under a mutex, xplus.go:67-69).
 * The salts of one launch are the ChaCha20 keystream (RFC 8439 block
 * function, 20 rounds):
 *     salts[0 .. n*S) = ChaCha20(key, nonce, counter 0..)[0 .. n*S)
 *     key   = the context's 32-byte salt key (random from getrandom(2) at
 *             sqobfs_open, or set by sqobfs_salt_key)
 *     nonce = "sqob" || le64(seq), seq = the context's launch sequence
 *             number, incremented by every launch that uses this flag
 * i.e. packet i's salt is bytes [(i % (64/S))*S, +S) of keystream block
 * i / (64/S).  A (key, seq) pair is never reused by a context, so salts are
 * unpredictable without the key and never repeat.  `salt` is ignored;
 * `salt_out`, if not NULL, receives the n*S generated salts. */
#define SQOBFS_FLAG_DEVICE_SALT 2u

/* batch flag: outputs own their 16-byte blocks.  The caller promises that no
 * 16-byte-aligned block of `out` that holds output bytes of packet i holds
 * input or output bytes of any other packet of the batch (true of slotted
 * layouts whose slots are multiples of 16 bytes: the Go Slots, the UDP
 * endpoint, sqobfs_pconn).  The launch may then write every such block whole:
 * the bytes of those blocks outside packet i's output (slot padding, and in
 * place the packet's own consumed salt) are left with unspecified values.
 * Every output byte is as without the flag. */
#define SQOBFS_FLAG_OUT_BLOCKS 4u

/* batch flag: outputs own their 128-byte lines to the end (implies
 * SQOBFS_FLAG_OUT_BLOCKS).  The caller also promises that the bytes from the
 * end of packet i's output to the next 128-byte boundary of `out` hold no
 * input or output bytes of any packet of the batch (slots whose stride is a
 * multiple of 128 and whose bases are 128-byte aligned: the Go Slots and the
 * packet conn engine's 2,048-byte slots).  The launch then writes every output
 * through to the end of its last 128-byte line: a line written in part is
 * merged by the memory controller with what HBM holds (a read-modify-write),
 * which costs a slotted batch ~15 % of the HBM rate.
 * Those padding bytes are left with unspecified values (copies of the
 * packet's last output block); every output byte is as without the flag. */
#define SQOBFS_FLAG_OUT_LINES 8u

/* out_len value written for a packet whose psk_id is out of range */
#define SQOBFS_BAD_PSK 0xFFFFFFFFu

enum sqobfs_kind { SQOBFS_SALAMANDER = 0, SQOBFS_XPLUS = 1 };
enum sqobfs_dir { SQOBFS_OBFUSCATE = 0, SQOBFS_DEOBFUSCATE = 1 };

typedef struct sqobfs_ctx sqobfs_ctx;
typedef struct sqobfs_keyring sqobfs_keyring;

/* A ragged batch of datagrams.  Structure-of-arrays, one entry per packet.
 * For the device entry points every pointer is a device pointer on the
 * context's GPU; for sqobfs_run_host every pointer is a host pointer. */
typedef struct sqobfs_batch {
  uint32_t n;               /* number of packets */
  uint32_t flags;           /* 0 or SQOBFS_FLAG_* */
  const uint8_t *in;        /* input base */
  const uint64_t *in_off;   /* [n] byte offset of packet i in `in` */
  const uint32_t *in_len;   /* [n] payload length (obfs) / datagram length n (deobfs) */
  uint8_t *out;             /* output base */
  const uint64_t *out_off;  /* [n] byte offset of packet i's output in `out` */
  uint32_t *out_len;        /* [n] written: output length per the rules above */
  const uint8_t *salt;      /* obfuscate: [n*S] salts (4-byte aligned); deobfs: unused */
  const uint16_t *psk_id;   /* [n] keyring index per packet, NULL = all use 0 */
  const uint32_t *in_cap;   /* XPlus deobfuscate only: [n] read-buffer length
                               len(p) >= in_len (xplus.go:55); NULL = in_len */
  uint8_t *salt_out;        /* SQOBFS_FLAG_DEVICE_SALT: [n*S] receives the
                               generated salts (4-byte aligned), or NULL */
} sqobfs_batch;

int sqobfs_abi_version(void);
/* Static string naming the compiled kernel configuration (target, unroll,
 * packets per wavefront, nt policy), e.g. for bench records. */
const char *sqobfs_build_info(void);
const char *sqobfs_strerror(int status);
int sqobfs_device_count(int *count);

/* One context per GPU.  Thread-safe: device launches only read immutable
 * state (and bump an atomic salt sequence number); sqobfs_run_host
 * serialises on an internal lock.  Every entry point makes the context's GPU
 * current for its own duration and restores the calling thread's current
 * device before returning (no per-thread side effect). */
int sqobfs_open(int device, sqobfs_ctx **out);
void sqobfs_close(sqobfs_ctx *ctx);
/* the context's own non-blocking HIP stream (as void*), for callers that
 * want a private stream; sqobfs_run_host uses it internally */
void *sqobfs_stream(sqobfs_ctx *ctx);
/* wait for all work on `stream` (NULL = the HIP null stream) */
int sqobfs_sync(sqobfs_ctx *ctx, void *stream);
/* sqobfs_sync polls the stream for up to `us` microseconds before it blocks
 * (default 0: block at once).  Polling holds the calling CPU for that long;
 * it shortens the wake-up after short launches. */
int sqobfs_set_sync_spin(sqobfs_ctx *ctx, uint32_t us);

/* Set the context's salt key and next launch sequence number for
 * SQOBFS_FLAG_DEVICE_SALT (replay / tests; sqobfs_open draws a random key and
 * starts at 0).  Not to be called concurrently with launches on the context. */
int sqobfs_salt_key(sqobfs_ctx *ctx, const uint8_t key[32], uint64_t next_seq);
/* The sequence number the next SQOBFS_FLAG_DEVICE_SALT launch will use. */
uint64_t sqobfs_salt_seq(const sqobfs_ctx *ctx);

/* Tuning: the obfuscation kernel's unit, the number of consecutive packets
 * one wavefront derives keys for and streams (1 .. 62; 0 = automatic).
 * Results are identical for every value; only the speed changes (DESIGN.md
 * section 5: ~21.7 KB of payload per wavefront streams best).  Automatic means
 * sized by bytes where the library sees the lengths (sqobfs_run_host, per
 * chunk) and the built-in default (26) for device batches, whose lengths
 * stay on the GPU: a caller that knows its batch sets
 * sqobfs_unit_packets_for(...) here.  Takes effect on later launches. */
int sqobfs_set_unit_packets(sqobfs_ctx *ctx, uint32_t packets);
/* the unit size device launches will use (the default when 0 was set) */
uint32_t sqobfs_unit_packets(const sqobfs_ctx *ctx);
/* The unit size for a batch of n packets holding `bytes` payload (or
 * datagram) bytes in total: about 21.7 KB per wavefront, 31.5 KB when packets
 * select keyring entries (psk_id != NULL), at least 2,048 wavefronts for
 * small batches, clamped to 1 .. 62. */
uint32_t sqobfs_unit_packets_for(uint64_t bytes, uint32_t n, int multi_psk);
/* The same for the keyring kind's kernel: XPlus with one PSK streams best at
 * ~19.5 KB per wavefront (16 packets of 1,200 B); Salamander as above
 * (sqobfs_unit_packets_for is this with SQOBFS_SALAMANDER). */
uint32_t sqobfs_unit_packets_for_kind(int kind, uint64_t bytes, uint32_t n, int multi_psk);

/* Upload `count` pre-shared keys (host memory: psk k = blob[off[k] .. +len[k]])
 * and derive each one's per-PSK hash state on the GPU.  kind selects the
 * hash (BLAKE2b for Salamander, SHA-256 for XPlus).  Any PSK length works,
 * including 0.  Synchronous.  Every keyring also keeps the host copy of that
 * state (sqobfs_cpu_run, the packet conn engine's CPU path).
 * ctx == NULL makes a HOST keyring: no GPU is touched (none need exist); it
 * serves sqobfs_cpu_run and packet conns opened without a context. */
int sqobfs_keyring_create(sqobfs_ctx *ctx, int kind, uint32_t count,
                          const uint8_t *blob, const uint64_t *off,
                          const uint32_t *len, sqobfs_keyring **out);
/* Does not block: the keyring's device memory is released in stream order
 * after the launches that used it (never waits for other keyrings' or
 * contexts' work).  The context must outlive its keyrings.  A caller's
 * stream the keyring was launched on must either outlive the keyring or be
 * released from it first with sqobfs_keyring_release_stream (the release is
 * ordered after the work on each stream still listed). */
void sqobfs_keyring_destroy(sqobfs_keyring *kr);
/* The caller is about to destroy `stream`, on which it launched with kr:
 * waits for the stream's work so far and drops it from kr's release fence,
 * so sqobfs_keyring_destroy never touches the destroyed handle.  SQ_OK also
 * when kr was never launched on it. */
int sqobfs_keyring_release_stream(const sqobfs_keyring *kr, void *stream);
int sqobfs_keyring_kind(const sqobfs_keyring *kr);
uint32_t sqobfs_keyring_count(const sqobfs_keyring *kr);
/* Test hook: compare the keyring's device hash state with its host copy
 * (entry by entry, byte for byte).  Returns the number of entries that
 * differ (0 = identical), or a negative status (SQ_EINVAL for a host
 * keyring). */
int sqobfs_debug_keyring_check(const sqobfs_keyring *kr);

/* The same transform on the CPU, synchronously, on the calling thread: a
 * batch in host memory with the semantics of a launch (every pointer a host
 * pointer; per-packet results identical to the GPU's, out_len codes
 * included).  SQOBFS_FLAG_DEVICE_SALT draws the salts from the keyring's
 * context generator (the same ChaCha20 stream, consuming one sequence number
 * as a launch does), or for a host keyring from a process generator keyed
 * from getrandom(2).  Works with no GPU present.  The byte work of the
 * reference's per-datagram ReadFrom / WriteTo (salamander.go:42-70,
 * xplus.go:46-75) for callers with few datagrams. */
int sqobfs_cpu_run(const sqobfs_keyring *kr, int dir, const sqobfs_batch *host_batch);

/* Device-resident batch launches: asynchronous on `stream` (a hipStream_t
 * passed as void*; NULL = the HIP null stream, as in HIP itself).  All batch
 * pointers are device pointers; the keyring's kind must match the entry
 * point. */
int sqobfs_salamander_obfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr,
                                const sqobfs_batch *b, void *stream);
int sqobfs_salamander_deobfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr,
                                  const sqobfs_batch *b, void *stream);
int sqobfs_xplus_obfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr,
                           const sqobfs_batch *b, void *stream);
int sqobfs_xplus_deobfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr,
                             const sqobfs_batch *b, void *stream);
/* the same, with kind/dir as arguments */
int sqobfs_launch(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir,
                  const sqobfs_batch *b, void *stream);

/* Host-memory batch, synchronous.  The batch is cut into pieces of
 * consecutive packets (up to 8 chunks of >= 4,096 packets, 16 when both
 * buffers are pinned; from 4 chunks on, the last chunk is cut in three)
 * whose copy-in (H2D), kernel and copy-out (D2H) run on three streams and
 * overlap.  Pinned caller buffers (sqobfs_host_alloc) are copied by DMA
 * directly; pageable ones go through pinned staging, and a pageable
 * output is copied out piece by piece while later pieces move.  Output
 * bytes outside the packets' output regions are preserved unless
 * flags has SQOBFS_FLAG_OUT_UNINIT.  With SQOBFS_FLAG_DEVICE_SALT every
 * piece is one launch with its own sequence number (salts of piece c =
 * keystream(seq_c) over the piece's packets, in packet order). */
int sqobfs_run_host(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir,
                    const sqobfs_batch *host_batch);

/* Pinned host memory for zero-copy staging by callers (socket buffers). */
int sqobfs_host_alloc(sqobfs_ctx *ctx, size_t bytes, void **out);
void sqobfs_host_free(sqobfs_ctx *ctx, void *p);

/* ------------------------------------------------------------------------
 * QUIC packet protection: AEAD_CHACHA20_POLY1305
 * and AEAD_AES_128_GCM, each with its header protection.
 *
 * The next per-datagram byte transform under the obfuscation layer: quic-go
 * (v0.52.0-beta.1, go.mod:7; not in the reference tree) seals every 1-RTT
 * packet (internal/handshake/aead.go) and applies header protection
 * (internal/handshake/header_protector.go) one packet at a time.  Here a
 * ragged batch of packets is protected / unprotected in one launch:
 *   seal:  nonce = iv XOR be96(pn)                         (RFC 9001 5.3)
 *          payload -> ChaCha20-Poly1305(key, nonce, aad = header)
 *                                                          (RFC 8439 2.8)
 *          sample = 16 bytes at pn_offset + 4 of the sealed packet;
 *          mask = ChaCha20(hp, counter = sample[0:4], nonce = sample[4:16]);
 *          first byte ^= mask[0] & (long header ? 0x0f : 0x1f),
 *          packet number bytes ^= mask[1 .. pn_len]        (RFC 9001 5.4)
 *   open:  the reverse; the packet number is decoded from its truncated
 *          form against the largest received one (RFC 9000 Appendix A.3)
 *          and the tag is verified.
 * AES-128-GCM (TLS_AES_128_GCM_SHA256) is the same with
 *          payload -> AES-128-GCM(key, nonce, aad = header)   (SP 800-38D)
 *          mask = AES-128-ECB(hp, sample)                  (RFC 9001 5.4.3)
 * The packet-number length is (first byte & 3) + 1 of the unprotected
 * header, as QUIC encodes it. */

/* One connection's 1-RTT keys (from the TLS key schedule: "quic key",
 * "quic iv", "quic hp", RFC 9001 5.1).  AES-128-GCM uses key[0..16) and
 * hp[0..16). */
typedef struct sqobfs_quic_key {
  uint8_t key[32];
  uint8_t iv[12];
  uint8_t hp[32];
} sqobfs_quic_key;

/* Cipher suites (the AEAD of the negotiated TLS 1.3 suite, RFC 9001 5.3) */
#define SQOBFS_QUIC_CHACHA20_POLY1305 0u /* TLS_CHACHA20_POLY1305_SHA256 */
#define SQOBFS_QUIC_AES_128_GCM 1u       /* TLS_AES_128_GCM_SHA256 */

typedef struct sqobfs_quic_keyring sqobfs_quic_keyring;

/* out_len values of packets that were not processed */
#define SQOBFS_QUIC_EKEY 0xFFFFFFFFu   /* key_id out of range */
#define SQOBFS_QUIC_ESHORT 0xFFFFFFFEu /* too short to sample / bad pn_offset */
#define SQOBFS_QUIC_EAUTH 0xFFFFFFFDu  /* open: tag mismatch (output undefined) */

/* A ragged batch of QUIC packets (device pointers).
 *   seal: in  = header || payload (in_len[i] bytes); out = protected
 *         header || ciphertext || 16-byte tag, out_len[i] = in_len[i] + 16.
 *   open: in  = protected packet incl. tag; out = unprotected header ||
 *         plaintext, out_len[i] = in_len[i] - 16; pn_out[i] (optional) =
 *         the decoded packet number.
 * out may be exactly in place (out_off == in_off; seal needs 16 bytes of
 * room after each packet) or disjoint from every input. */
typedef struct sqobfs_quic_batch {
  uint32_t n;
  uint32_t flags;              /* 0 */
  const uint8_t *in;
  const uint64_t *in_off;
  const uint32_t *in_len;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *out_len;
  const uint16_t *pn_offset;   /* [n] offset of the packet number field */
  const uint64_t *pn;          /* [n] seal: the packet number; open: the
                                  largest packet number received so far */
  const uint16_t *key_id;      /* [n] keyring index, NULL = all use 0 */
  uint64_t *pn_out;            /* open: [n] decoded packet numbers, or NULL */
} sqobfs_quic_batch;

/* A keyring holds connections of ONE suite (a batch is sealed / opened
 * with the keyring's suite).  sqobfs_quic_keyring_create is the
 * ChaCha20-Poly1305 form.  For AES-128-GCM the key schedules and the GHASH
 * tables (about 16.5 KiB per connection) are prepared here, once. */
int sqobfs_quic_keyring_create_suite(sqobfs_ctx *ctx, uint32_t suite, uint32_t count,
                                     const sqobfs_quic_key *keys, sqobfs_quic_keyring **out);
int sqobfs_quic_keyring_create(sqobfs_ctx *ctx, uint32_t count, const sqobfs_quic_key *keys,
                               sqobfs_quic_keyring **out);
void sqobfs_quic_keyring_destroy(sqobfs_quic_keyring *kr);
int sqobfs_quic_seal(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                     const sqobfs_quic_batch *b, void *stream);
int sqobfs_quic_open(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                     const sqobfs_quic_batch *b, void *stream);

/* QUIC protection and the Salamander layer in ONE pass (Hysteria2's send and
 * receive path: quic-go seals a packet, then SalamanderPacketConn.WriteTo
 * obfuscates the datagram, salamander.go:57-70; ReadFrom then Open on the
 * way in).  One read of the plaintext and one write of the wire datagram
 * instead of two kernels and an intermediate buffer.
 *   seal: in = header || payload (as sqobfs_quic_seal); out = the wire
 *         datagram salt[i] || (protected packet || tag) ^ K_i, K_i =
 *         BLAKE2b-256(psk || salt[i]) repeated, out_len[i] = in_len[i] + 24.
 *         salt: [n*8] device bytes.  out must not overlap in, except the
 *         in-place form out_off[i] == in_off[i] - 8 (8 bytes of headroom in
 *         front of each packet, as the vectorised Salamander writer).
 *   open: in = wire datagram (in_len[i] bytes, salt first); out = unprotected
 *         header || plaintext, out_len[i] = in_len[i] - 24 (or a
 *         SQOBFS_QUIC_E* code; datagrams shorter than the salt give
 *         SQOBFS_QUIC_ESHORT).  In place (out_off == in_off) works.
 * okr: a Salamander keyring (entry 0 is the connection's PSK); kr: a QUIC
 * keyring of either suite. */
int sqobfs_quic_seal_salamander(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                                const sqobfs_keyring *okr, const sqobfs_quic_batch *b,
                                const uint8_t *salt, void *stream);
int sqobfs_quic_open_salamander(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                                const sqobfs_keyring *okr, const sqobfs_quic_batch *b,
                                void *stream);

/* ------------------------------------------------------------------------
 * Several GPUs in one process (packets are independent, so a
 * batch shards into contiguous ranges with no exchange at all).
 */

/* Contiguous shards of nearly equal work: cut[k] = first packet of shard k
 * (k < parts), cut[parts] = n, balanced by cumulative bytes (in_len plus a
 * small per-packet constant), so ragged batches split evenly.  cut has
 * parts + 1 entries. */
int sqobfs_shard_cuts(uint32_t n, const uint32_t *in_len, uint32_t parts, uint32_t *cut);
/* One host-memory batch over nctx contexts (GPUs): shard k (sqobfs_shard_cuts)
 * runs sqobfs_run_host on ctxs[k] with krs[k] (keyrings of the same kind and
 * PSKs, one per context), each shard on its own host thread with its own
 * pinned staging and streams.  Returns the first error, after every shard
 * has finished.  With SQOBFS_FLAG_DEVICE_SALT each shard draws its salts from
 * its own context's generator. */
int sqobfs_run_host_sharded(uint32_t nctx, sqobfs_ctx *const *ctxs,
                            const sqobfs_keyring *const *krs, int dir, const sqobfs_batch *hb);
/* Device-resident shards: bs[k] lives on ctxs[k]'s GPU and is launched there
 * on the context's stream; returns after all shards complete (first error).
 * = sqobfs_shard_launch + sqobfs_shard_wait. */
int sqobfs_shard_run(uint32_t nctx, sqobfs_ctx *const *ctxs, const sqobfs_keyring *const *krs,
                     int dir, const sqobfs_batch *bs);
/* The same without waiting: every shard is queued on its context's stream,
 * one completion event is recorded per context, and the call returns at
 * once with a ticket.  A caller keeps several steps in flight (launch step
 * i + 1, then wait for step i) so no host round trip sits between one
 * step's kernels and the next's.  Contexts may share a GPU.  On a failed
 * launch the shards already queued are waited for and the error returned
 * (no ticket). */
typedef struct sqobfs_shard_ticket sqobfs_shard_ticket;
int sqobfs_shard_launch(uint32_t nctx, sqobfs_ctx *const *ctxs, const sqobfs_keyring *const *krs,
                        int dir, const sqobfs_batch *bs, sqobfs_shard_ticket **out);
/* 1 when every shard of the ticket is done, 0 while one still runs, or an
 * error status (the ticket stays valid: wait for it to release it). */
int sqobfs_shard_query(sqobfs_shard_ticket *t);
/* Wait for every shard (polling each context's stream for its
 * sqobfs_set_sync_spin time, then blocking), release the ticket, return the
 * first error. */
int sqobfs_shard_wait(sqobfs_shard_ticket *t);

/* Bytes of pinned staging sqobfs_run_host holds (it grows to the largest
 * batch span seen: the input and output byte ranges the batch touches, not
 * their offsets). */
size_t sqobfs_host_staging_bytes(const sqobfs_ctx *ctx);
/* Test hook: the next sqobfs_run_host whose pipeline reaches chunk `chunk`
 * fails there with SQ_EDEVICE, as a failed launch would (-1 = off). */
void sqobfs_debug_fail_chunk(int chunk);
/* Test hook: on != 0 makes multi-key AES-128-GCM launches skip the grouping
 * by key (the path taken when the grouping scratch cannot be allocated). */
void sqobfs_debug_gcm_ungrouped(int on);
/* Test hook: keyring tables (obfuscation and QUIC) and the AES-GCM grouping
 * scratch created from now on are carved from the caller's device region
 * [base, base + bytes) instead of the device allocator (base NULL: the
 * allocator again; blocks carved earlier stay valid and are never freed).
 * Returns the bytes carved from the previous region.  For placement tests
 * (tables at addresses whose low 32-bit word has bit 31 set). */
uint64_t sqobfs_debug_device_pool(void *base, uint64_t bytes);
/* Measurement hook (bench.py): the calling thread's next obfuscation launch
 * (sqobfs_launch / sqobfs_run_host chunk) records start_event / stop_event
 * (hipEvent_t, created with timing) with its own kernel dispatch
 * (hipExtLaunchKernel), so per-kernel times cost no marker packets between
 * kernels.  Either may be NULL; spent by the next sqobfs_launch call even
 * when it launches nothing (an empty or refused batch). */
void sqobfs_debug_time_next_launch(void *start_event, void *stop_event);

/* ------------------------------------------------------------------------
 * Batched UDP socket I/O (Linux) -- the host side of the path.
 *
 * The reference moves one datagram per syscall: every ReadFrom / WriteTo of
 * the decorators wraps one recvfrom / sendto of the inner PacketConn
 * (salamander.go:43,65,88; xplus.go:47,74,97), and port hopping runs one
 * goroutine per socket feeding a 1024-deep channel of 2048-byte buffers
 * (hysteria/hop.go:19,40-161, recvLoop).  These entry points move whole
 * batches with recvmmsg / sendmmsg, fan several sockets into one batch, and
 * hand the batch to the GPU in one launch.
 */

/* Socket address, plain C (no <sys/socket.h> needed by callers). */
typedef struct sqobfs_addr {
  uint16_t family;   /* AF_INET (2) or AF_INET6 (10) */
  uint16_t port;     /* host byte order */
  uint32_t scope_id; /* IPv6 scope id, 0 for IPv4 */
  uint8_t addr[16];  /* IPv4: first 4 bytes; IPv6: all 16 */
} sqobfs_addr;

/* Receive up to `max` datagrams from the sockets fds[0..nfds) (fan-in).
 * Waits up to timeout_ms (-1 = forever, 0 = no wait) for the first
 * datagram, then drains every readable socket without blocking, round-robin,
 * with recvmmsg.  Datagram k lands at slots + k*slot_bytes + headroom
 * (at most slot_bytes - headroom bytes; longer ones are truncated, as a
 * ReadFrom into a fixed buffer truncates).  Writes len[k], fd_index[k] (index
 * into fds) and from[k] (may be NULL), and *count.  Returns SQ_OK with
 * *count == 0 on timeout, SQ_EINVAL on bad arguments, or -errno. */
int sqobfs_udp_recv(const int *fds, uint32_t nfds, uint8_t *slots, uint32_t slot_bytes,
                    uint32_t headroom, uint32_t max, int timeout_ms, uint32_t *len,
                    uint16_t *fd_index, sqobfs_addr *from, uint32_t *count);

/* Send n datagrams on socket fd with sendmmsg: datagram k is
 * base[off[k] .. +len[k]) to to[k].  Blocks while the socket buffer is
 * full; *sent = datagrams handed to the kernel.  SQ_OK or -errno. */
int sqobfs_udp_send(int fd, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                    const sqobfs_addr *to, uint32_t n, uint32_t *sent);

/* An obfuscating batched UDP endpoint: the sockets of one hysteria /
 * hysteria2 connection (several with port hopping), the keyring, and pinned
 * receive / transmit slots of slot_bytes each (2048 as in hop.go:19). */
typedef struct sqobfs_udp_conn sqobfs_udp_conn;

/* One received and deobfuscated batch.  Message i: payload
 * base[off[i] .. +len[i]) (len = what the reference's ReadFrom returns:
 * n - S, the raw n bytes for a Salamander datagram of n <= 8, 0 for an XPlus
 * datagram of n < 16 -- callers skip len 0), received on fds[fd_index[i]]
 * from from[i].  Valid until the next sqobfs_udp_conn_read. */
typedef struct sqobfs_udp_view {
  uint32_t count;
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  const uint16_t *fd_index;
  const sqobfs_addr *from;
} sqobfs_udp_view;

int sqobfs_udp_conn_open(sqobfs_ctx *ctx, const sqobfs_keyring *kr, const int *fds,
                         uint32_t nfds, uint32_t slots, uint32_t slot_bytes,
                         sqobfs_udp_conn **out);
void sqobfs_udp_conn_close(sqobfs_udp_conn *c);
/* ReadFrom for a whole batch: receive (sqobfs_udp_recv over the conn's
 * sockets), deobfuscate on the GPU in one launch that reads and writes the
 * conn's page-locked, GPU-mapped slots directly (zero copy; payload decoded
 * in place behind the salt), return the view.  slot_bytes: multiple of 16. */
int sqobfs_udp_conn_read(sqobfs_udp_conn *c, int timeout_ms, sqobfs_udp_view *out);
/* Transmit slot i's payload area: the caller writes payload i here (up to
 * slot_bytes - S bytes) -- S bytes of headroom precede it for the salt, as
 * the vectorised writers prepend it (salamander.go:81-93, xplus.go:86-98). */
uint8_t *sqobfs_udp_conn_tx_payload(sqobfs_udp_conn *c, uint32_t i);
/* WriteTo for a whole batch: obfuscate tx slots 0..n-1 (payload lengths
 * len[i]) in place with device salts (SQOBFS_FLAG_DEVICE_SALT) in one GPU
 * launch, then sendmmsg datagram i = salt || payload ^ key to to[i] on
 * fds[fd_index].  *sent = datagrams sent. */
int sqobfs_udp_conn_write(sqobfs_udp_conn *c, uint32_t fd_index, uint32_t n,
                          const uint32_t *len, const sqobfs_addr *to, uint32_t *sent);

/* QUIC through the endpoint (Hysteria2's data path; the conn's keyring must
 * be Salamander): one launch per batch seals AND obfuscates
 * (sqobfs_quic_seal_salamander) or de-obfuscates AND opens
 * (sqobfs_quic_open_salamander), in the mapped slots.
 * write_quic: QUIC packet i (header || payload, len[i] bytes, at most
 *   slot_bytes - 24) is written by the caller at sqobfs_udp_conn_tx_payload(i);
 *   packet numbers pn[i], pn field at pn_offset (the connection's short
 *   header: 1 + DCID length); salts from getrandom.  *sent = datagrams
 *   sent, a prefix of the batch: when the kernel rejects a packet (too short
 *   for its packet number and sample), the packets before it are sent and
 *   the call returns SQ_EINVAL, so packet *sent is the rejected one.
 * read_quic: receive a batch, open it with packet numbers decoded against
 *   largest_pn; view.len[i] = the packet's length (header || plaintext, at
 *   view.base + view.off[i]) or a SQOBFS_QUIC_E* code; *pn_out (optional) =
 *   the decoded packet numbers.  Valid until the next read. */
int sqobfs_udp_conn_write_quic(sqobfs_udp_conn *c, const sqobfs_quic_keyring *qkr,
                               uint32_t fd_index, uint32_t n, const uint32_t *len,
                               uint16_t pn_offset, const uint64_t *pn, const sqobfs_addr *to,
                               uint32_t *sent);
int sqobfs_udp_conn_read_quic(sqobfs_udp_conn *c, const sqobfs_quic_keyring *qkr,
                              uint16_t pn_offset, uint64_t largest_pn, int timeout_ms,
                              sqobfs_udp_view *out, const uint64_t **pn_out);

/* UDP segmentation offloads (Linux UDP_SEGMENT / UDP_GRO).
 * sqobfs_udp_send_gso: as sqobfs_udp_send, but consecutive datagrams to the
 * same address whose lengths are equal (the last of a run may be shorter)
 * go out as ONE message with a UDP_SEGMENT control message (at most 64
 * datagrams / 65,000 bytes per message); the kernel (or the NIC) cuts it
 * into the original datagrams.  -EIO / -EINVAL when the socket or route
 * cannot segment. */
int sqobfs_udp_send_gso(int fd, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        const sqobfs_addr *to, uint32_t n, uint32_t *sent);

#define SQOBFS_UDP_TX_GSO 1u /* conn_write sends runs with UDP_SEGMENT */
#define SQOBFS_UDP_RX_GRO 2u /* conn_read receives coalesced datagrams (UDP_GRO) */
/* Enable offloads on an endpoint.  With RX_GRO the receive region is used
 * as 64 KiB buffers that each hold up to 64 coalesced datagrams, so the
 * view's off[] are no longer slot-aligned (needs slots >= 64 and
 * slots * slot_bytes >= 64 KiB).  TX_GSO falls back to one datagram per
 * message if the first GSO send is refused.  Returns the flags in effect
 * (>= 0) or SQ_EINVAL. */
int sqobfs_udp_conn_set_offload(sqobfs_udp_conn *c, uint32_t flags);

/* ------------------------------------------------------------------------
 * Obfuscating packet conn: the engine behind the Go decorators (go/sqobfs).
 *
 * The reference's SalamanderPacketConn / XPlusPacketConn (hysteria2/
 * salamander.go:19-109, hysteria/xplus.go:39-118) transform one datagram per
 * ReadFrom / WriteTo, synchronously.  A pconn keeps their per-call contract
 * -- ReadFrom returns one datagram with the reference's length rules,
 * WriteTo takes one -- and batches the byte work underneath:
 *   WriteTo  copies the payload into the transmit batch being filled and
 *            returns; a worker obfuscates the batch in ONE launch (device
 *            salts, in place behind S bytes of headroom) and sends it.
 *            The worker launches as soon as it is idle (or linger_us after
 *            the batch's first datagram), so a lone packet goes out at once
 *            and a burst that arrives during a launch becomes the next batch.
 *   ReadFrom returns the next datagram of a de-obfuscated receive batch; a
 *            worker receives and de-obfuscates whole batches in ONE launch.
 * Batches live in page-locked, GPU-mapped slots (zero copy, as
 * sqobfs_udp_conn).  Two modes:
 *   socket (fd >= 0): the pconn dup()s a UDP socket and moves the datagrams
 *            itself with recvmmsg / sendmmsg (a Go *net.UDPConn's fd);
 *   pump   (fd < 0):  the caller moves them over any PacketConn: its reader
 *            hands each received datagram to sqobfs_pconn_rx_push, its
 *            writer sends what sqobfs_pconn_tx_take returns.
 * Addresses are sqobfs_addr (socket mode) and an opaque 64-bit tag that rides
 * with every datagram (pump mode: the caller's handle on its own address
 * object).  All calls are thread-safe; read and write may block, and honour
 * the deadlines of sqobfs_pconn_set_deadline. */
typedef struct sqobfs_pconn sqobfs_pconn;

typedef struct sqobfs_pconn_opts {
  uint32_t batch;      /* datagrams per launch at most (0 = 256) */
  uint32_t slot_bytes; /* per-datagram slot, multiple of 16 (0 = 2048, hop.go:19);
                          longer received datagrams are cut to it, as a
                          ReadFrom into a buffer of that size cuts them */
  uint32_t tx_batches; /* transmit batches (0 = 8: while a launch flies, the
                          writers fill the next ones, and they all join the
                          following launch; a batch holds a pool block only
                          while it fills, flies or waits to be taken) */
  uint32_t rx_batches; /* receive batches (0 = 8; a block only while a batch
                          fills, flies or holds unread datagrams) */
  uint32_t linger_us;  /* an idle worker waits this long for a partly filled
                          batch to grow (0: launch at once) */
  uint32_t spin_us;    /* a worker polls a launch at most this long before it
                          blocks (0 = 200); the engine polls about twice the
                          launches' recent completion time, within that bound;
                          SQOBFS_PCONN_NEVER = never poll: the engine's
                          completer thread sleeps through most of the
                          kernel's expected time, then polls with short
                          sleeps, and the worker goes on with other batches
                          meanwhile (no core is held while the kernel runs,
                          at ~50 us more latency) */
  uint32_t flags;      /* socket mode: SQOBFS_UDP_TX_GSO (runs of equal-length
                          datagrams to one address go out as UDP_SEGMENT
                          messages; off by itself if the socket refuses) |
                          SQOBFS_UDP_RX_GRO (coalesced receives, split into
                          the batch) */
  uint32_t cpu_max;    /* batches whose cost (payload bytes + 1024 per
                          datagram, a key derivation's worth) is at most this
                          run on the CPU path instead of a launch (0 = the
                          engine's measured break-even: its recent launch
                          round trip x its recent CPU-path rate, within
                          16 KiB .. 4 MiB, ~80 KiB before any measurement,
                          sqobfs_engine_info.route_bytes; SQOBFS_PCONN_NEVER =
                          always launch while the GPU works).  With 0, under
                          sustained load -- the engine's batches would keep
                          more than a tenth of a core busy on the CPU path
                          (sqobfs_engine_info.loaded) -- a batch of more than
                          64 datagrams also launches, waiting without
                          polling, when its CPU-path time exceeds twice the
                          host CPU time a launched batch costs (measured,
                          sqobfs_engine_info.gpu_host_ns): the host pays the
                          launch and the sockets, not the bytes; bursts of up
                          to 64 stay on the CPU path */
  uint32_t inline_gap_us; /* socket mode: a write made when the transmit side
                          is idle and the previous write is at least this old
                          is obfuscated on the CPU and sent on the writer's own
                          thread, its send error returned by that same call, as
                          the reference's WriteTo does (0 = 100;
                          SQOBFS_PCONN_NEVER = every write is batched) */
} sqobfs_pconn_opts;
#define SQOBFS_PCONN_NEVER 0xFFFFFFFFu

typedef struct sqobfs_pconn_stats {
  uint64_t tx_datagrams, tx_batches; /* obfuscated and handed to the socket / taker */
  uint64_t rx_datagrams, rx_batches; /* received and de-obfuscated */
  uint64_t rx_truncated;             /* datagrams longer than a slot (cut) */
  uint64_t tx_send_errors;           /* datagrams the socket refused (batched sends) */
  uint32_t tx_max_batch, rx_max_batch;
  uint64_t cpu_batches;   /* batches (tx + rx) transformed on the CPU path */
  uint64_t inline_writes; /* datagrams sent on the writer's thread (inline_gap_us) */
  uint64_t gpu_failures;  /* batches whose launch failed (the device); the engine
                             then stays on the CPU path */
  uint64_t dropped;       /* datagrams lost with a launch that failed after it started */
  uint64_t gpu_refused;   /* batches whose launch was refused for the moment (no
                             memory for a stream, a descriptor block or a merged
                             keyring): redone on the CPU path, the GPU stays on
                             (ABI 6) */
} sqobfs_pconn_stats;

/* kr's kind picks Salamander or XPlus.  ctx and kr must outlive the pconn.
 * ctx == NULL (with a host keyring): no GPU; every batch runs on the CPU
 * path, with the same results -- so a drop-in constructor never fails for
 * want of a device (salamander.go:24-40 cannot fail). */
int sqobfs_pconn_open(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int fd,
                      const sqobfs_pconn_opts *opts, sqobfs_pconn **out);
/* Graceful stop (net.PacketConn.Close): later writes fail with SQ_ECLOSED;
 * datagrams already written are still obfuscated and sent (taken, in pump
 * mode) for up to 200 ms; then every blocked call returns SQ_ECLOSED and the
 * workers end.  Idempotent; may run concurrently with other calls. */
void sqobfs_pconn_shutdown(sqobfs_pconn *pc);
/* shutdown, then free everything; no call may be in progress or follow */
void sqobfs_pconn_close(sqobfs_pconn *pc);
/* WriteTo (salamander.go:57-70 / 81-93, xplus.go:62-75 / 86-98): queue the
 * payload p[0..len) for `to` (socket mode) with `tag`.  Returns SQ_OK, SQ_EINVAL
 * (longer than slot_bytes - S), SQ_ECLOSED, SQ_ETIMEDOUT (write deadline, while
 * every transmit batch is busy), or a send error: an inline write's own
 * (opts.inline_gap_us: the reference's behaviour), else that of an earlier
 * batched datagram, reported once by the next write. */
int sqobfs_pconn_write(sqobfs_pconn *pc, const uint8_t *p, uint32_t len, const sqobfs_addr *to,
                       uint64_t tag);
/* ReadFrom (salamander.go:42-55, xplus.go:46-60) into p[0..cap): *n is what
 * the reference's ReadFrom returns for a datagram of w bytes read into a
 * buffer of cap bytes, m = min(w, cap): Salamander m <= 8: the m raw bytes,
 * else the first m - 8 payload bytes; XPlus m < 16: 0, else the first m - 16
 * payload bytes (XPlus's XOR of p past the returned length, xplus.go:55, is
 * not reproduced: those bytes are not defined).  from / tag: the datagram's
 * source and tag (either may be NULL).  Blocks until a datagram, the read
 * deadline (SQ_ETIMEDOUT), shutdown (SQ_ECLOSED) or a receive error. */
int sqobfs_pconn_read(sqobfs_pconn *pc, uint8_t *p, uint32_t cap, uint32_t *n,
                      sqobfs_addr *from, uint64_t *tag);
#define SQOBFS_PCONN_READ 1u
#define SQOBFS_PCONN_WRITE 2u
/* SetReadDeadline / SetWriteDeadline / SetDeadline: `which` = READ | WRITE;
 * unix_ns = wall-clock time in ns since the epoch, 0 = none.  Wakes blocked
 * calls, which fail with SQ_ETIMEDOUT once the deadline has passed. */
int sqobfs_pconn_set_deadline(sqobfs_pconn *pc, uint32_t which, int64_t unix_ns);
/* pump mode: a datagram the caller read from the wrapped conn (copied; cut
 * to slot_bytes).  Blocks while every receive batch is full and unread. */
int sqobfs_pconn_rx_push(sqobfs_pconn *pc, const uint8_t *wire, uint32_t n,
                         const sqobfs_addr *from, uint64_t tag);
/* pump mode: the wrapped conn's read failed: readers get `status` (e.g.
 * SQ_EIO) once the queued datagrams are read -- one reader when `once` (a
 * per-datagram error such as an ICMP-reported refusal, after which the
 * wrapped conn reads on), every later reader otherwise. */
int sqobfs_pconn_rx_fail(sqobfs_pconn *pc, int status, int once);
/* pump mode: the next obfuscated batch to send.  Datagram i is
 * base[off[i] .. +len[i]) (salt || payload ^ key) for to[i] / tag[i].  Valid
 * until sqobfs_pconn_tx_done.  One taker at a time.  SQ_ETIMEDOUT after
 * timeout_ms (-1 = forever), SQ_ECLOSED after shutdown. */
typedef struct sqobfs_pconn_tx {
  uint32_t count;
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  const sqobfs_addr *to;
  const uint64_t *tag;
} sqobfs_pconn_tx;
int sqobfs_pconn_tx_take(sqobfs_pconn *pc, int timeout_ms, sqobfs_pconn_tx *out);
int sqobfs_pconn_tx_done(sqobfs_pconn *pc);
int sqobfs_pconn_stats_get(const sqobfs_pconn *pc, sqobfs_pconn_stats *out);
/* live sqobfs_host_alloc blocks in the process (leak checks) */
int64_t sqobfs_debug_host_allocs(void);

/* The engine.  Every pconn of a context (ctx NULL: of the process's host
 * engine) is served by ONE engine: a fixed pool of worker threads that
 * obfuscate / de-obfuscate and move the batches of all its pconns, one poller
 * thread that watches their sockets (epoll), with a context one completer
 * thread that waits for the launches that do not poll (bulk batches; spin_us
 * SQOBFS_PCONN_NEVER) and finishes their batches, so the launching worker is
 * free at once (launches in flight: at most 32, each on a HIP stream of the
 * engine's), and a
 * pool of batch blocks (page-locked and GPU-mapped with a context) that
 * pconns take while they fill, transmit or hold unread datagrams and give
 * back when done.  So opening more pconns -- a port-hopping client re-dials
 * one per hop, hysteria/hop.go:114 -- adds no threads, and memory follows the
 * datagrams in flight, not the number of pconns. */
typedef struct sqobfs_engine_info {
  uint32_t pconns;       /* open pconns */
  uint32_t threads;      /* engine threads (workers + poller, + completer with a
                            context) */
  uint32_t workers;
  uint32_t pool_blocks;  /* batch blocks allocated (in use + free) */
  uint64_t pool_bytes;
  uint32_t blocks_in_use;
  uint32_t gpu_disabled; /* 1 after a failed launch: every batch runs on the CPU */
  uint64_t route_bytes;  /* pconns with cpu_max 0: batches costing more go to
                            the GPU (0 without a context) */
  uint32_t launch_us;    /* recent launch round trip (EWMA) */
  uint32_t cpu_ns_per_kib; /* recent CPU-path time per KiB of cost (EWMA) */
  uint32_t load_permille;  /* transform demand: the CPU-path time its batches
                              would take, per mille of one core's time
                              (smoothed over 10 ms windows) */
  uint32_t loaded;         /* 1 while that stays above 100 (off below 50):
                              batches of more than 64 datagrams may launch */
  uint32_t gpu_host_ns;    /* host CPU time of a launched batch with a
                              non-polling wait (launch call + wait; EWMA) */
  uint32_t cpus;           /* CPUs the engine's threads are kept on (the L3
                              domain of the thread that started it; 0 = not
                              restricted: sqobfs_engine_set_affinity) */
  uint32_t group_max;      /* the most batches one launch takes
                              (sqobfs_engine_set_group) */
  uint64_t launches;       /* kernel launches of the engine */
  uint64_t group_launches; /* ... that carried the batches of several pconns */
  uint64_t group_batches;  /* batches carried by those */
  uint64_t async_launches; /* launches completed by the completer thread (ABI 6) */
  uint32_t streams;        /* launch streams made: the most launches that were in
                              flight at once (at most 32) */
  uint32_t reserved;
} sqobfs_engine_info;
/* ctx NULL: the host engine.  SQ_OK with zeros when it was never started. */
int sqobfs_engine_info_get(sqobfs_ctx *ctx, sqobfs_engine_info *out);
/* Worker threads of the context's engine (0 = 4); only before its first
 * pconn opens (SQ_EINVAL after). */
int sqobfs_engine_set_workers(sqobfs_ctx *ctx, uint32_t workers);
/* Where the engine's threads run: SQOBFS_ENGINE_AFFINITY_L3 (the default)
 * keeps the workers and the poller on the CPUs of the process's affinity that
 * share the L3 cache (the CCD) of the thread that starts the engine -- the
 * first pconn open -- so its hand-offs stay in one cache; _NONE leaves them
 * to the scheduler.  Only before the context's first pconn opens (SQ_EINVAL
 * after). */
#define SQOBFS_ENGINE_AFFINITY_NONE 0
#define SQOBFS_ENGINE_AFFINITY_L3 1
int sqobfs_engine_set_affinity(sqobfs_ctx *ctx, int mode);
/* Coalesced launches.  A Hysteria2 server wraps one socket
 * (hysteria2/service.go:117-120) but a port-hopping client one conn per hop
 * (hysteria/hop.go:40-63) over a generic PacketConn (client.go:184-186:
 * pump mode here), and a process may serve many: when a worker launches a
 * pconn's batch, the pconn's other full batches queued in that direction
 * join the launch, and when the pconn is in pump mode and leaves the
 * routing to the engine (cpu_max 0 or SQOBFS_PCONN_NEVER), so do the batches
 * other such pconns of the same scheme have queued in the same direction --
 * at most max_batches batches (0 = 32; 1 = every batch its own launch) and
 * 16,384 datagrams -- so one kernel, one wait and one launch's host cost
 * carry them all (batches are not gathered to make a launch none of them
 * would make alone).  Batches routed to a non-polling launch while one is
 * still in flight wait for it, and its completion launches them together
 * (the engine's natural batching under load).  Their PSKs may differ: the
 * launch then reads per-datagram PSK ids into a keyring the engine merges
 * from the pconns' keyrings.  Socket-mode pconns' tasks are not gathered by
 * another pconn's worker (their steps are socket calls that the workers keep
 * making in parallel).  Any time. */
int sqobfs_engine_set_group(sqobfs_ctx *ctx, uint32_t max_batches);
/* Free the pool's unused blocks; returns how many were freed. */
int sqobfs_engine_trim(sqobfs_ctx *ctx);
/* Test hook: the next `count` launches of every engine fail -- at submission
 * (at_completion == 0: nothing ran; the batch is redone on the CPU) or when
 * waited for (1: as a kernel that faulted; the batch is dropped) -- and the
 * engines switch to the CPU path, as after a real device failure. */
void sqobfs_debug_engine_fail(int count, int at_completion);
/* Test hook: the next `count` batch-block allocations of every engine fail
 * (as a failed page-locked allocation); a socket pconn's receive side
 * retries on a timer and recovers. */
void sqobfs_debug_pool_fail(int count);
/* Test hook: while on, the engines' workers start no task (queued tasks
 * wait; a running one finishes), so a test can queue the batches of several
 * pconns and see them coalesced when it turns the hold off. */
void sqobfs_debug_engine_hold(int on);

#ifdef __cplusplus
}
#endif
#endif /* SQOBFS_H */
