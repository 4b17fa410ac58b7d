// sq_kernels.hip -- gfx950 kernels for the Salamander / XPlus obfuscation path.
//
// One fused kernel per (scheme, direction, psk-mode).  It replaces the
// per-datagram bodies of
//   SalamanderPacketConn.WriteTo / ReadFrom   hysteria2/salamander.go:42-70
//   VectorisedSalamanderPacketConn.WriteTo    hysteria2/salamander.go:81-93
//   XPlusPacketConn.WriteTo / ReadFrom        hysteria/xplus.go:46-75
//   VectorisedXPlusConn.WriteTo               hysteria/xplus.go:86-98
// for a whole ragged batch of datagrams per launch.
//
// One wavefront = one unit of ppw (sqobfs_set_unit_packets; ~21.7 KB of payload)
// consecutive packets, lane l owning packet l; lanes ppw and ppw + 1 hold the
// packets just after and just before the unit (its boundary neighbours).
//   1. descriptor  offsets, lengths, salt (obfuscate: the salt array;
//                  deobfuscate: the first S wire bytes), the quirk table; the
//                  loads of the head / tail image windows.
//   2. key         each lane hashes its own packet's psk||salt (BLAKE2b-256
//                  or SHA-256) from the keyring's per-PSK midstate.
//   3. plan        every 16-byte-aligned output block is OWNED by the packet
//                  holding its first byte.  A packet's owned blocks are its
//                  interior blocks (16 payload bytes: load, XOR, store) and at
//                  most two special ones: the first (salt bytes) and the last
//                  (its tail plus the head of the next datagram when the two
//                  are adjacent), whose 16 bytes are precomputed from the
//                  packet's head / tail images and the next lane's head image.
//                  Bytes of blocks no datagram pair covers whole (gaps between
//                  outputs) are written byte-exactly up front by the owner.
//                  The owned blocks of the unit form one flat space; per
//                  packet an LDS record (offsets, keystream phases, special
//                  values) and, per 64 blocks, four bit rows (packet starts,
//                  special first / last blocks, blocks not loaded).
//   4. stream      the wave walks the flat space, 64 lanes x U blocks per
//                  step, 1 KiB per wave instruction: one dwordx4 load, XOR
//                  with the record's keystream, one aligned dwordx4 store.
//                  A block's record is a v_mbcnt over the start bits; a
//                  special block's loaded value is discarded for its
//                  precomputed one (its load is kept when its input block
//                  holds a payload byte, so the read stream has no holes).
// So for back-to-back datagrams (GSO buffers, the bench's dense layout) every
// output line is written once, whole, in address order, like a plain copy.
// Measured on copy probes: leaving the boundary blocks to a separate pass
// costs 7-12 % (holes) to 30 % (holes filled early) of the HBM rate, and
// splitting wave instructions into 256-byte pieces (16 lanes per packet)
// costs 40 %.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "sq_bytes.h"
#include "sq_hash.h"
#include "sq_internal.h"
#include "sq_obfs_key.h"

namespace sq {

// Streaming policy of the bulk loads / stores (bit 0: loads, bit 1:
// stores).  Payload bytes are touched exactly once, so nontemporal (`nt`)
// accesses keep them from displacing useful L2 lines.
constexpr int kNt = 3;
// Blocks per lane per step (double-buffered: U..2U KiB of loads in flight).
constexpr int kU = 4;
// Wavefronts per workgroup (see kWavesPerGroup).
constexpr int kWpb = 2;
// The first packet of a unit gives the blocks it owns in the 64-byte line
// its output starts in to the previous unit's wave (which holds it as its
// look-ahead lane), so no output line is written by two waves.
constexpr bool kDonate = true;
// Stream alignment (map path): the flat space starts (d_lo / 16) mod
// 2^kAlign slots in, so for back-to-back outputs every 1 KiB wave
// instruction covers whole 2^(kAlign+4)-byte lines (3: 128-byte L2 lines).
constexpr int kAlign = 3;
// Flat blocks a unit's block map covers (its role bytes live in LDS).
constexpr uint32_t kMapBlk = 4096;
// Multi-PSK kernels load each lane's keyring entry (chaining value and
// first message block) right after the descriptor, so the gather overlaps
// the plan step (192 VGPRs: 2 waves per SIMD, still 2-3 % faster on the
// 256-PSK batch in-process, profiles/r03/ab); round 2 loaded it in the hash
// itself.
constexpr bool kPskPre = true;
// (Round 6: the compile-time switches of these constants were folded into
// them; their variants are in git history and DESIGN.md section 5.)
// Timeline builds (scripts/dev/timeline.py, never shipped): lane 0 of every
// wave records the constant-rate clock at its phase boundaries.
#ifndef SQ_TIMELINE
#define SQ_TIMELINE 0
#endif


// XCD-contiguous units.  Workgroups are dispatched round-robin over the 8
// XCDs, so block b runs on XCD b % 8 and, unmapped, the XCDs share one
// moving window of the batch.  Remapped, each XCD walks its own contiguous
// eighth (its L2 and its address translation see one window 1/8 the size).
// Measured in one process on three boxes (DESIGN.md section 5,
// profiles/r03/ab/xcd): 16M x 1350 B batches (45 GB of buffers) -5 to -7 %,
// the 16M 256-PSK batch -2 to -5.5 %, 4M x 1350 B +1.9 % on one box and
// -5 % on another, 1M +1.3 to +2.9 % (the gain follows the address-
// translation load, which depends on the box's memory as well as the
// size).  So launches of at least kXcdMinUnits units (~5.7 GB of payload at
// the byte-sized units) remap (KParams.xcd).  Runs of 32-768 blocks per XCD
// inside 8-run windows instead of eighths gained less at 16M and nothing at
// 1M.
constexpr uint64_t kXcdMinUnits = 1u << 18;

static_assert(kU == 4 && kDefaultUnitPackets == 26 && kNt == 3 && kWpb == 2 && kDonate &&
                  kAlign == 3 && kMapBlk == 4096,
              "sqobfs_build_info states these");
extern "C" const char *sqobfs_build_info(void) {
  return "gfx950 obfs_kernel U=4 default_ppw=26 NT=3 wpb=2 donate=1 align=3 map=4096"
         " windows=buffer earlysalt=1 dppred=1 xcd=rule";
}

// default unit size (KParams.ppw == 0); any 1 .. kMaxUnitPackets works
constexpr uint32_t kPktPerWave = kDefaultUnitPackets;

#if SQ_TIMELINE
constexpr uint32_t kTlStamps = 6, kTlWaves = 1u << 20;
__device__ uint64_t g_timeline[kTlWaves * kTlStamps];
#define SQ_STAMP(k)                                                                   \
  do {                                                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                             \
    if (lane == 0 && unit < kTlWaves) g_timeline[unit * kTlStamps + (k)] = t_;         \
  } while (0)
#else
#define SQ_STAMP(k) \
  do {              \
  } while (0)
#endif
static_assert(kPktPerWave >= 1 && kPktPerWave <= kMaxUnitPackets && kMaxUnitPackets + 2 <= kWave,
              "unit + 2 neighbour lanes");

constexpr uint32_t kMaxPacket = 1u << 26;  // per-packet length bound (u32 block math)
constexpr uint32_t kBadPsk = 0xFFFFFFFFu;
constexpr uint32_t kBadLen = 0xFFFFFFFEu;

// ------------------------------------------------------------ key derivation

// XPlus: key = SHA-256(psk || salt16) (hysteria/xplus.go:54).
__device__ __forceinline__ void xplus_key(const PskEntry *E,
                                          const uint32_t (&salt)[4],
                                          uint32_t (&key)[8]) {
  const uint32_t *h32 = reinterpret_cast<const uint32_t *>(E->h);
  const uint32_t *m32 = reinterpret_cast<const uint32_t *>(E->m);
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = h32[i];
  const uint32_t nb = E->nblocks, t = E->salt_pos;
  const uint32_t w = t >> 2, sh = (t & 3) * 8;
  uint32_t c[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint32_t cur = k < 4 ? __builtin_bswap32(salt[k]) : 0u;
    const uint32_t prev = k > 0 ? __builtin_bswap32(salt[k - 1]) : 0u;
    c[k] = (cur >> sh) | (sh ? (prev << (32 - sh)) : 0u);
  }
  for (uint32_t blk = 0; blk < nb; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t idx = 16 * blk + j;
      uint32_t x = m32[idx];
#pragma unroll
      for (int k = 0; k < 5; k++) x |= (idx == w + k) ? c[k] : 0u;
      m[j] = x;
    }
    s2_compress(st, m);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) key[i] = __builtin_bswap32(st[i]);
}

// ------------------------------------------------------------ packet job

struct PacketJob {
  uint64_t src_pay;  // address of payload byte 0 in the input
  uint64_t dst_pay;  // address of payload byte 0 in the output
  uint64_t len;      // payload bytes to transform
  uint32_t pre;      // salt bytes written in front of dst_pay (obfs) or 0
};

// ------------------------------------------------------------ wave helpers

// Wave-uniform 64-bit min / max: within each row of 16 lanes by DPP moves
// (quad swaps, half-row mirror, row mirror: every lane then holds its row's
// result), then the four rows' results by readlane -- no LDS round trips.
// Every lane must be active.  Measured in one process against a shuffle
// (ds_bpermute) butterfly (round 4, profiles/r04/ab2): -0.15 to -0.6 % on
// every kernel, -2 % with device salts on the ragged batch.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xF, 0xF, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
template <bool MAX>
__device__ __forceinline__ uint64_t wave_ext64_dpp(uint64_t x) {
  auto pick = [](uint64_t a, uint64_t b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
  x = pick(x, dpp64<0xB1>(x));   // quad_perm [1,0,3,2]
  x = pick(x, dpp64<0x4E>(x));   // quad_perm [2,3,0,1]
  x = pick(x, dpp64<0x141>(x));  // row_half_mirror
  x = pick(x, dpp64<0x140>(x));  // row_mirror
  uint64_t r[4];
#pragma unroll
  for (int k = 0; k < 4; k++)
    r[k] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 16 * k) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 16 * k);
  return pick(pick(r[0], r[1]), pick(r[2], r[3]));
}
__device__ __forceinline__ uint64_t shfl64(uint64_t x, uint32_t src) {
  return b2_pack((uint32_t)__shfl((int)(uint32_t)x, (int)src, kWave),
                 (uint32_t)__shfl((int)(uint32_t)(x >> 32), (int)src, kWave));
}
__device__ __forceinline__ uint32_t shfl32(uint32_t x, uint32_t src) {
  return (uint32_t)__shfl((int)x, (int)src, kWave);
}

// ------------------------------------------------------------ per-packet steps

// Device salts (SQOBFS_FLAG_DEVICE_SALT): the salt of packet p is bytes
// [(p % (64/S))*S, +S) of ChaCha20 keystream block p / (64/S), so a batch's
// salts are the keystream's first n*S bytes.
//
// Quad ChaCha20 (RFC 8439 2.3): the 4 lanes of a quad hold one block's state
// column by column (lane i: words i, 4 + i, 8 + i, 12 + i).  The column
// round is one quarter round per lane; the diagonal round rotates rows 1-3
// across the quad by 1, 2, 3 lanes (DPP quad_perm), runs one quarter round
// and rotates them back.  Per lane 80 quarter rounds -> 20, plus 60 DPP
// moves.  Every lane of the wave must call it.
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
#define SQ_QQR(a, b, c, d)                                              \
  a += b; d ^= a; d = __builtin_amdgcn_alignbit(d, d, 16);            \
  c += d; b ^= c; b = __builtin_amdgcn_alignbit(b, b, 20);            \
  a += b; d ^= a; d = __builtin_amdgcn_alignbit(d, d, 24);            \
  c += d; b ^= c; b = __builtin_amdgcn_alignbit(b, b, 25);
__device__ __forceinline__ void chacha20_quad(const uint32_t (&key)[8], uint32_t counter,
                                              const uint32_t (&nonce)[3], uint32_t col,
                                              uint32_t (&o)[4]) {
  const uint32_t sigma = col == 0 ? 0x61707865u : col == 1 ? 0x3320646eu
                         : col == 2 ? 0x79622d32u : 0x6b206574u;
  // the key and nonce words are wave-uniform: read them as scalars and
  // select per lane (a per-lane index into the kernarg array became a
  // vector load from it, whose wait drained the descriptor loads too)
  uint32_t kw[8], nw[3];
#pragma unroll
  for (int i = 0; i < 8; i++) kw[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)key[i]);
#pragma unroll
  for (int i = 0; i < 3; i++) nw[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)nonce[i]);
  const bool c1 = col == 1, c2 = col == 2, c3 = col == 3;
  const uint32_t kb = c3 ? kw[3] : c2 ? kw[2] : c1 ? kw[1] : kw[0];
  const uint32_t kc = c3 ? kw[7] : c2 ? kw[6] : c1 ? kw[5] : kw[4];
  const uint32_t kd = c3 ? nw[2] : c2 ? nw[1] : c1 ? nw[0] : counter;
  uint32_t a = sigma, b = kb, c = kc, d = kd;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    SQ_QQR(a, b, c, d)
    // lane i: b of lane i + 1, c of i + 2, d of i + 3 (quad_perm)
    b = qperm<0x39>(b);
    c = qperm<0x4E>(c);
    d = qperm<0x93>(d);
    SQ_QQR(a, b, c, d)
    b = qperm<0x93>(b);
    c = qperm<0x4E>(c);
    d = qperm<0x39>(d);
  }
  o[0] = a + sigma;
  o[1] = b + kb;
  o[2] = c + kc;
  o[3] = d + kd;
}
#undef SQ_QQR

// The device salts of a wave's packets (lanes 0 .. ppw + 1: the unit and
// its two neighbours) by quads: quad q computes keystream block b0 + q (16
// blocks per pass; a unit of up to 62 packets needs one pass, XPlus units
// over 58 packets two), the blocks are staged in the wave's LDS scratch
// (1 KiB), and every lane reads its S bytes.  Every lane must call it.
template <uint32_t S>
__device__ __forceinline__ void device_salts_wave(const KParams &P, uint64_t first, uint32_t ppw,
                                                  uint32_t lane, uint32_t p, bool valid,
                                                  uint32_t *scratch, uint32_t (&salt)[4]) {
  constexpr uint32_t per_block = 64 / S;  // 8 Salamander, 4 XPlus
  const uint64_t lo = first ? first - 1 : 0;
  const uint64_t hi0 = first + ppw, hi = hi0 < P.n ? hi0 : P.n - 1;
  const uint32_t b0 = (uint32_t)(lo / per_block);
  const uint32_t nb = (uint32_t)(hi / per_block) - b0 + 1;  // wave-uniform
  const uint32_t q = lane >> 2, col = lane & 3;
  const uint32_t mb = p / per_block - b0;  // this lane's block, relative
  const uint32_t w0 = (p % per_block) * (S / 4);
  for (uint32_t pass = 0; pass * 16 < nb; pass++) {
    uint32_t x[4];
    chacha20_quad(P.salt_key, b0 + 16 * pass + q, P.salt_nonce, col, x);
#pragma unroll
    for (int r = 0; r < 4; r++) scratch[16 * q + 4 * r + col] = x[r];
    const uint32_t rb = mb - 16 * pass;
    if (valid && rb < 16) {
#pragma unroll
      for (uint32_t k = 0; k < S / 4; k++) salt[k] = scratch[16 * rb + w0 + k];
    }
  }
}

// ... and its copy to salt_out (SQOBFS_FLAG_DEVICE_SALT with salt_out)
template <uint32_t S>
__device__ __forceinline__ void device_salt_out(const KParams &P, uint32_t p,
                                                const uint32_t (&salt)[4]) {
  if (P.salt_out) {
    uint32_t *so = reinterpret_cast<uint32_t *>(P.salt_out + (uint64_t)p * S);
#pragma unroll
    for (uint32_t k = 0; k < S / 4; k++) so[k] = salt[k];
  }
}

// Step 1, descriptor, in two halves so the persistent kernel can prefetch
// it one work unit ahead.  fetch_desc issues the loads of packet p's batch
// entry (offsets, lengths, psk id, XPlus capacity, obfuscate salt);
// finalize_desc applies the quirk table of include/sqobfs.h and gives the
// packet's job (addresses and length of the XOR stream, salt bytes to
// prepend), its salt (deobfuscate: the first S wire bytes, a dependent
// load), whether it needs a key, and its out_len.
struct RawDesc {
  uint64_t ioff, ooff;
  uint32_t len, cap, pid;
  uint32_t salt[4];
};

template <int KIND, int DIR, bool MULTI>
__device__ __forceinline__ void fetch_desc(const KParams &P, uint32_t p, bool valid, uint32_t p0,
                                           RawDesc &d) {
  constexpr uint32_t S = KIND == 0 ? kSalamanderSalt : kXPlusSalt;
  // Unconditional loads (a lane without a packet reads the unit's first
  // entry, p0, in the lines the wave reads anyway, and drops it): loads
  // under a divergent branch made the compiler wait for all of them
  // (s_waitcnt vmcnt(0)) where the branches join, before the device salts
  // could run under them.
  if (DIR == 1) {  // (deobfuscate: no device salts to overlap; the branch
                   // measured 0.3-0.9 % faster, profiles/r05/ab/desc_*)
    d.ioff = d.ooff = 0;
    d.len = d.cap = d.pid = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) d.salt[k] = 0u;
    if (!valid) return;
    d.ioff = P.in_off[p];
    d.ooff = P.out_off[p];
    d.len = P.in_len[p];
    if (MULTI) d.pid = P.psk_id[p];
    if (KIND == 1 && P.in_cap) d.cap = P.in_cap[p];
    return;
  }
  const uint32_t q = valid ? p : p0;
  const uint64_t ioff = P.in_off[q], ooff = P.out_off[q];
  const uint32_t len = P.in_len[q];
  const uint32_t pid = MULTI ? (uint32_t)P.psk_id[q] : 0u;
  const uint32_t cap = (KIND == 1 && DIR == 1 && P.in_cap) ? P.in_cap[q] : 0u;
  d.ioff = valid ? ioff : 0;
  d.ooff = valid ? ooff : 0;
  d.len = valid ? len : 0u;
  d.pid = valid ? pid : 0u;
  d.cap = valid ? cap : 0u;
#pragma unroll
  for (int k = 0; k < 4; k++) d.salt[k] = 0u;
  if (DIR == 0 && !P.device_salt) {
    const uint32_t *sp = reinterpret_cast<const uint32_t *>(P.salt + (uint64_t)q * S);
#pragma unroll
    for (uint32_t k = 0; k < S / 4; k++) d.salt[k] = valid ? sp[k] : 0u;
  }
  // (device salts: device_salts_wave, while these loads fly)
}

template <int KIND, int DIR, bool MULTI>
__device__ __forceinline__ void finalize_desc(const KParams &P, uint32_t p, bool valid,
                                              const RawDesc &d, PacketJob &J,
                                              uint32_t (&salt)[4], bool &do_hash,
                                              const PskEntry *&E, uint32_t &olen) {
  constexpr uint32_t S = KIND == 0 ? kSalamanderSalt : kXPlusSalt;
  J = {0, 0, 0, 0};
  do_hash = false;
  // single PSK: the kernarg copy (scalar loads); several: the device table
  // (never a pointer that may be either: that forces a flat copy of P)
  E = MULTI ? P.psk_table : &P.psk0;
  olen = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) salt[k] = 0u;
  if (!valid) return;
  const uint64_t in_base = (uint64_t)P.in + d.ioff;
  const uint64_t out_base = (uint64_t)P.out + d.ooff;
  const uint32_t len = d.len;
  bool bad = false;
  if (MULTI) {
    if (d.pid >= P.n_psk) bad = true;
    else E = P.psk_table + d.pid;
  }
  const uint32_t cap = d.cap > len ? d.cap : len;  // xplus.go:55 XORs to len(p)
  if (len > kMaxPacket || cap > kMaxPacket) {
    olen = kBadLen;
  } else if (bad) {
    olen = kBadPsk;
  } else if (DIR == 0) {  // obfuscate: wire = salt || payload ^ key
    if (P.device_salt) {  // (computed by fetch_desc)
#pragma unroll
      for (uint32_t k = 0; k < S / 4; k++) salt[k] = d.salt[k];
      device_salt_out<S>(P, p, salt);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < S / 4; k++) salt[k] = d.salt[k];
    }
    J = {in_base, out_base + S, len, S};
    olen = S + len;
    do_hash = true;
  } else if (KIND == 0 && len <= S) {
    // salamander.go:47-49: short datagram returned as is -> copy (key 0)
    J = {in_base, out_base, len, 0};
    olen = len;
  } else if (KIND == 1 && len < S) {
    olen = 0;  // xplus.go:50-52: dropped as empty
  } else {  // deobfuscate: salt = first S wire bytes
    // (read with the head window, fetch_windows: one round trip after the
    // descriptor instead of two)
    J = {in_base + S, out_base, (uint64_t)cap - S, 0};
    olen = len - S;
    do_hash = true;
  }
}

// The words of a keyring entry one compression needs (kPskPre): loaded
// early, consumed by the hash.
struct PskHot {
  uint64_t h[8];   // BLAKE2b chaining value | SHA-256 state (first 32 bytes)
  uint64_t m[16];  // first final block: BLAKE2b 16 words | SHA-256 16 BE words
  uint64_t t_first, t_last;
  uint32_t nblocks, salt_pos;
};

// message words of the first block loaded early (timing builds vary it; the
// rest are read by the hash)
constexpr uint32_t kPskPreM = 16;
template <int KIND>
__device__ __forceinline__ void load_hot(const KParams &P, const PskEntry *E, PskHot &H) {
  // the keyring's uniform bounds (sq_api.hip keyring_hot_words): words no
  // entry needs are zero and not loaded, the chaining value of a keyring of
  // short PSKs is the initial state
  const uint32_t mw = P.psk_hot_m < kPskPreM ? P.psk_hot_m : kPskPreM;
  if (P.psk_hot_iv) {
    if (KIND == 0) {
      b2_init256(H.h);
    } else {
      uint32_t st[8];
      s2_init(st);
#pragma unroll
      for (int i = 0; i < 8; i++) H.h[i] = i < 4 ? b2_pack(st[2 * i], st[2 * i + 1]) : 0ull;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) H.h[i] = KIND == 0 || i < 4 ? E->h[i] : 0ull;
  }
#pragma unroll
  for (int i = 0; i < 16; i++)
    H.m[i] = (KIND == 0 || i < 8) && (uint32_t)i < mw ? E->m[i] : 0ull;
  H.t_first = KIND == 0 ? E->t_first : 0ull;
  H.t_last = KIND == 0 ? E->t_last : 0ull;
  H.nblocks = E->nblocks;
  H.salt_pos = E->salt_pos;
}

// Salamander key from a preloaded entry (the second block, PSK tails over
// 120 bytes, is read from the table)
__device__ __forceinline__ void salamander_key_hot(const PskHot &H, const PskEntry *E,
                                                   const uint32_t (&salt)[4], uint32_t (&key)[8]) {
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = H.h[i];
  const uint32_t nb = H.nblocks, t = H.salt_pos;
  const uint64_t sv = b2_pack(salt[0], salt[1]);
  const uint32_t w = t >> 3, sh = (t & 7) * 8;
  const uint64_t lo = sv << sh;
  const uint64_t hi = sh ? (sv >> (64 - sh)) : 0ull;
  for (uint32_t blk = 0; blk < nb; blk++) {
    uint64_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t idx = 16 * blk + j;
      uint64_t x = blk == 0 && j < kPskPreM ? H.m[j] : E->m[idx];  // (H.m: zero past mw)
      x |= (idx == w) ? lo : 0ull;
      x |= (idx == w + 1) ? hi : 0ull;
      m[j] = x;
    }
    const bool last = blk + 1 == nb;
    b2_compress(h, m, last ? H.t_last : H.t_first, last);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    key[2 * i] = (uint32_t)h[i];
    key[2 * i + 1] = (uint32_t)(h[i] >> 32);
  }
}

// XPlus key from a preloaded entry (second block from the table)
__device__ __forceinline__ void xplus_key_hot(const PskHot &H, const PskEntry *E,
                                              const uint32_t (&salt)[4], uint32_t (&key)[8]) {
  const uint32_t *m32 = reinterpret_cast<const uint32_t *>(E->m);
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    st[2 * i] = (uint32_t)H.h[i];
    st[2 * i + 1] = (uint32_t)(H.h[i] >> 32);
  }
  const uint32_t nb = H.nblocks, t = H.salt_pos;
  const uint32_t w = t >> 2, sh = (t & 3) * 8;
  uint32_t c[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint32_t cur = k < 4 ? __builtin_bswap32(salt[k]) : 0u;
    const uint32_t prev = k > 0 ? __builtin_bswap32(salt[k - 1]) : 0u;
    c[k] = (cur >> sh) | (sh ? (prev << (32 - sh)) : 0u);
  }
  for (uint32_t blk = 0; blk < nb; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t idx = 16 * blk + j;
      const uint64_t hv = H.m[j >> 1];
      uint32_t x = blk == 0 && (j >> 1) < kPskPreM ? (uint32_t)(j & 1 ? hv >> 32 : hv)
                                                     : m32[idx];
#pragma unroll
      for (int k = 0; k < 5; k++) x |= (idx == w + k) ? c[k] : 0u;
      m[j] = x;
    }
    s2_compress(st, m);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) key[i] = __builtin_bswap32(st[i]);
}

// Step 2, key: lane-parallel, one packet per lane.
template <int KIND, bool HOT>
__device__ __forceinline__ void derive_key(bool do_hash, const PskEntry *E, const PskHot &H,
                                           const uint32_t (&salt)[4], uint32_t (&key)[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) key[i] = 0u;
  if (do_hash) {
    if (HOT) {
      if (KIND == 0) salamander_key_hot(H, E, salt, key);
      else xplus_key_hot(H, E, salt, key);
    } else {
      if (KIND == 0) salamander_key(E, salt, key);
      else xplus_key(E, salt, key);
    }
  }
}

// ------------------------------------------------------------ one unit

// Lane roles: lanes 0 .. ppw-1 own packets first + lane; lane ppw holds the
// packet right after the unit and lane ppw + 1 the one right before it (the
// neighbours of its boundary blocks: they own and write nothing).
__device__ __forceinline__ uint32_t lane_packet(uint64_t first, uint32_t ppw, uint32_t lane,
                                                uint32_t n, bool &valid, bool &owner) {
  const int64_t base = (int64_t)first;
  int64_t p = -1;
  if (lane < ppw) p = base + lane;
  else if (lane == ppw) p = base + ppw;
  else if (lane == ppw + 1) p = base - 1;
  valid = p >= 0 && p < (int64_t)n;
  owner = valid && lane < ppw;
  return valid ? (uint32_t)p : 0u;
}

// Output range [rs, re) of a packet's job (empty: ne == false).
__device__ __forceinline__ void out_range(const PacketJob &J, uint64_t &rs, uint64_t &re,
                                          bool &ne) {
  ne = J.len != 0 || J.pre != 0;
  rs = J.dst_pay - J.pre;
  re = J.dst_pay + J.len;
}

__device__ __forceinline__ uint64_t up16(uint64_t a) { return (a + 15) & ~15ull; }

// The last partial output block [BL, re) needs payload bytes the 32-byte
// head image does not hold.
__device__ __forceinline__ bool tail_from_window(uint64_t rs, uint64_t re) {
  return (re & 15) && (re & ~15ull) > rs + 16;
}

// The input blocks the packet's images need, all loaded together: the head
// window (payload bytes [0, 32 - pre)) and the tail window (payload bytes of
// the last partial output block); deobfuscate also the block before the head
// when it holds salt bytes.
//
// The six loads are raw buffer loads against one wave-uniform resource based
// at the wave's lowest window block.  A block a packet does not need gets an
// offset past num_records, so it reads zero without a memory access: every
// load is unconditional, with no substitute reads and no masks.  (Round 3
// issued conditional global loads, whose phi copies the compiler resolved
// with a full `s_waitcnt vmcnt(0)` before the plan, or unconditional loads
// of a readable substitute block for two of the eight kernels.)  Measured in
// one process against round 3's loads (DESIGN.md section 5,
// profiles/r04/ab): ragged deobfuscate -1.2 % dense / -1.7 % in 16-byte
// slots (both now >= 0.70), configs[1] deobfuscate -1.0 %, the 256-PSK
// obfuscate -5.2 %, the other kernels -0.1 to -0.5 %.
// A lane whose blocks lie 4 GiB or more past the base (a ragged batch
// scattered over more than 4 GiB within one unit) loads those again with
// 64-bit global loads where the images are built (reload_windows).
struct Windows {
  u32x4 h0, h1, h2, t0, t1;
  u32x4 s0;     // deobfuscate: the block before h0 when it holds salt bytes
  uint32_t rl;  // the needed blocks out of the resource's range
};
constexpr uint32_t kWinH0 = 1, kWinH1 = 2, kWinH2 = 4, kWinT0 = 8, kWinT1 = 16, kWinS0 = 32;
constexpr uint32_t kWinOffNone = 0xFFFFFFF0u;  // past num_records: reads zero

// The window block addresses of a packet (need: bits kWin*).
struct WinAddr {
  uint64_t s0, h0, h1, h2, t0, t1;
  uint32_t need;
};

template <int DIR, uint32_t S>
__device__ __forceinline__ WinAddr window_addrs(const PacketJob &J, bool wire_salt) {
  uint64_t rs, re;
  bool ne;
  out_range(J, rs, re, ne);
  const uint64_t hw = !ne ? 0ull : (J.len < 32 - J.pre ? J.len : 32 - J.pre);
  const uint64_t B = J.src_pay & ~15ull, e = J.src_pay + hw;
  const bool c_h0 = hw != 0, c_h1 = c_h0 && e > B + 16, c_h2 = c_h0 && e > B + 32;
  const bool c_s0 = DIR == 1 && c_h0 && wire_salt && (J.src_pay & 15) < S;
  const bool c_t0 = ne && tail_from_window(rs, re);
  const uint64_t ta = J.src_pay + ((re & ~15ull) - J.dst_pay), te = J.src_pay + J.len;
  const uint64_t TB = ta & ~15ull;
  const bool c_t1 = c_t0 && te > TB + 16;
  WinAddr A;
  A.s0 = B - 16;
  A.h0 = B;
  A.h1 = B + 16;
  A.h2 = B + 32;
  A.t0 = TB;
  A.t1 = TB + 16;
  A.need = (c_h0 ? kWinH0 : 0u) | (c_h1 ? kWinH1 : 0u) | (c_h2 ? kWinH2 : 0u) |
           (c_t0 ? kWinT0 : 0u) | (c_t1 ? kWinT1 : 0u) | (c_s0 ? kWinS0 : 0u);
  return A;
}

// Every needed block lies at or after the packet's h0 (s0 when needed): a
// tail block follows its head.
template <int DIR, uint32_t S>
__device__ __forceinline__ void fetch_windows(const PacketJob &J, bool wire_salt, Windows &W) {
  const WinAddr A = window_addrs<DIR, S>(J, wire_salt);
  const uint64_t first = (A.need & kWinS0) ? A.s0 : A.h0;
  const uint64_t lo0 = wave_ext64_dpp<false>(A.need ? first : ~0ull);
  const uint64_t lo = lo0 == ~0ull ? 0ull : lo0;  // (no lane needs a block)
  const __amdgpu_buffer_rsrc_t R =
      __builtin_amdgcn_make_buffer_rsrc((void *)lo, 0, (int)kWinOffNone, 0x00020000);
  uint32_t rl = 0u;
  auto off = [&](uint64_t a, uint32_t bit) -> uint32_t {
    if (!(A.need & bit)) return kWinOffNone;
    const uint64_t o = a - lo;  // a >= lo for every needed block
    if (o >= kWinOffNone) {
      rl |= bit;
      return kWinOffNone;
    }
    return (uint32_t)o;
  };
  const uint32_t o_s0 = off(A.s0, kWinS0), o_h0 = off(A.h0, kWinH0), o_h1 = off(A.h1, kWinH1),
                 o_h2 = off(A.h2, kWinH2), o_t0 = off(A.t0, kWinT0), o_t1 = off(A.t1, kWinT1);
  W.s0 = DIR == 1 ? __builtin_amdgcn_raw_buffer_load_b128(R, o_s0, 0, 0) : u32x4{0u, 0u, 0u, 0u};
  W.h0 = __builtin_amdgcn_raw_buffer_load_b128(R, o_h0, 0, 0);
  W.h1 = __builtin_amdgcn_raw_buffer_load_b128(R, o_h1, 0, 0);
  W.h2 = __builtin_amdgcn_raw_buffer_load_b128(R, o_h2, 0, 0);
  W.t0 = __builtin_amdgcn_raw_buffer_load_b128(R, o_t0, 0, 0);
  W.t1 = __builtin_amdgcn_raw_buffer_load_b128(R, o_t1, 0, 0);
  W.rl = rl;
}

// The blocks fetch_windows could not reach, loaded where the images are
// built (wave-uniform test; never taken for units within 4 GiB).
template <int DIR, uint32_t S>
__device__ __forceinline__ void reload_windows(const PacketJob &J, bool wire_salt, Windows &W) {
  if (__ballot(W.rl != 0u) == 0) return;
  const WinAddr A = window_addrs<DIR, S>(J, wire_salt);
  if (W.rl & kWinS0) W.s0 = gld<u32x4>(A.s0);
  if (W.rl & kWinH0) W.h0 = gld<u32x4>(A.h0);
  if (W.rl & kWinH1) W.h1 = gld<u32x4>(A.h1);
  if (W.rl & kWinH2) W.h2 = gld<u32x4>(A.h2);
  if (W.rl & kWinT0) W.t0 = gld<u32x4>(A.t0);
  if (W.rl & kWinT1) W.t1 = gld<u32x4>(A.t1);
}

// LDS record of a packet with blocks in the flat space (96 B), stored at the
// packet's rank among such packets.  Flat block c of the unit, owned by this
// packet, is at input ssub + 16 c and output dsub + 16 c (buffer offsets
// soff + 16 c, doff + 16 c); its keystream is tab[c & 1], except the special
// blocks c == sidx (first, value tab[2]) and c >= eidx (last, and out_lines
// pad blocks: value tab[3]),
// whose loads are range-checked away.
struct alignas(16) ChunkRec {
  uint64_t ssub, dsub;
  uint32_t soff, doff, sidx, eidx;
  u32x4 tab[4];
};
static_assert(sizeof(ChunkRec) == 96, "ChunkRec layout");

// Block -> packet map of a unit whose flat space fits kMapBlocks: one byte
// per flat block, the owning packet's record index (bits 0-5) and the
// block's role (bit 6: special first block, bit 7: special last block).
// The stream reads one byte per block: no search, no cross-lane work.
constexpr uint32_t kMapBlocks = kMapBlk;  // 64 KiB of output per unit (4096)
constexpr uint32_t kRoleFirst = 64, kRoleLast = 128;
// slack for the steps the double-buffered loop issues past the end
constexpr uint32_t kMapSlack = 2 * kWave * kU + 64;
// record index of the phase slots (below): no packet (ranks are <= 62)
constexpr uint32_t kRankNone = kWave - 1;
constexpr uint32_t kOffPhase = 0xFFFFF000u;  // + 16 c (c < 64) stays past any span
struct WaveLds {
  ChunkRec rec[kWave];
  uint32_t cst[kWave];  // flat start of the packet of each rank
  uint8_t role[kMapBlocks + kMapSlack];
};

struct WaveBufs {
  __amdgpu_buffer_rsrc_t src, dst;
};

struct UnitStream {
  uint32_t cst;    // lane: flat start of the packet of rank `lane` (~0 past the last)
  uint32_t T;      // wave-uniform: blocks in the flat space
  bool fast;       // wave-uniform: buffer-resource streaming possible
  bool map;        // wave-uniform: the bit map covers the flat space
  WaveBufs B;
};

constexpr uint32_t kNoIdx = 0xFFFFFFFFu;
constexpr uint64_t kMaxSpan = 0xFFFFE000ull;
static_assert(kOffPhase >= kMaxSpan && kOffPhase + 16ull * kWave <= 0xFFFFFFF0ull,
              "phase-slot offsets must be out of range and must not wrap");

// Block geometry of a unit's packets, from their jobs alone.
struct Geo {
  uint64_t rs, re, B0;  // output range, first owned block
  uint32_t nblk;        // owned blocks [B0, B0 + 16 nblk)
  uint32_t npad;        // out_lines: pad blocks after them (to the 128-byte line's end)
  uint32_t rank;        // record index (packets with flat blocks only)
  uint32_t start;       // flat index of the first owned block
  bool flat;            // has blocks in the flat space
  bool ne;              // non-empty output
  bool hf;              // first owned block special (holds salt bytes)
  bool hl;              // last owned block partly this packet's (re unaligned)
  bool lfull;           // ... and written whole (the next datagram fills it)
  bool pfull;           // bytes [rs, B0) are in the previous packet's whole block
  bool obh;             // out_blocks head: the first block starts at rs rounded down
};

// Step 3a, the plan: block ownership and special-block roles (no key, no
// payload bytes needed), the flat prefix sum, the stream half of the LDS
// records, the block map and the buffer resources -- everything the first
// stream loads need.  Every lane of the wave runs it.
// With out_blocks (SQOBFS_FLAG_OUT_BLOCKS) every block an output touches is
// the packet's own: its last block is always written whole (bytes past re
// scratch), and its first block starts at rs rounded down (a special block
// whose bytes before rs are scratch) -- unless the salt would then spill into
// a second block (obfuscate with rs % 16 + S > 16), which keeps the
// byte-exact head.  Slotted layouts (outputs at 16-byte-aligned slot starts,
// or decoded in place behind the salt) never need it.
// With out_lines (SQOBFS_FLAG_OUT_LINES, implies out_blocks) the owner also
// writes the blocks from its last block to the end of that 128-byte line
// (pad blocks: not loaded, value the last block's, like the special last
// block), so no line is written in part.
__device__ __forceinline__ UnitStream plan_unit(const PacketJob &J, bool owner, uint32_t lane,
                                                uint32_t ppw, bool has_prev, bool ob, bool ol,
                                                WaveLds &L, Geo &G) {
  out_range(J, G.rs, G.re, G.ne);
  const uint64_t rs = G.rs, re = G.re;
  // in place (input overlaps its own output blocks): a neighbour in another
  // wave must not read or write across this packet's blocks
  const uint64_t oblo = rs & ~15ull, obhi = up16(re);
  const bool ovl = G.ne && J.len && J.src_pay < obhi && J.src_pay + J.len > oblo;
  // neighbours: next lane = next packet (lane ppw for the last one),
  // previous lane = previous packet (lane ppw + 1 for the first one)
  const uint32_t nl = (lane + 1) & (kWave - 1);
  const uint32_t pl = lane == 0 ? ppw + 1 : lane - 1;
  const uint64_t rs_n = shfl64(rs, nl), re_n = shfl64(re, nl);
  const uint64_t rs_p = shfl64(rs, pl), re_p = shfl64(re, pl);
  const uint32_t fl = (G.ne ? 1u : 0u) | (ovl ? 2u : 0u);
  const uint32_t fl_n = shfl32(fl, nl), fl_p = shfl32(fl, pl);

  G.obh = ob && (uint32_t)(rs & 15) + J.pre <= 16u;
  const uint64_t B0r = G.obh ? (rs & ~15ull) : up16(rs), E = up16(re), BL = re & ~15ull;
  const uint32_t nraw = (G.ne && E > B0r) ? (uint32_t)((E - B0r) >> 4) : 0u;
  const bool cross_n = lane == ppw - 1, cross_p = lane == 0;
  // leading bytes [rs, B0) covered by the previous packet's whole last block
  // (the same predicate as the previous lane's lfull)
  const bool p_hl = (fl_p & 1) && (re_p & 15) && up16(re_p) > up16(rs_p);
  G.pfull = !ob && p_hl && G.ne && re_p == rs && re >= B0r && !(cross_p && ovl);
  // Donation.  A unit's first packet p gives its blocks in the 64-byte line
  // its output starts in ([B0, LE)) to the previous unit's wave, which holds
  // p as its look-ahead lane (key, head image and job already there): every
  // output line is then written whole by one wave.  Both waves decide from
  // the same data (p's job and p-1's end); only when p continues past LE, is
  // not in place, and its leading bytes are a whole junction block or none.
  const bool ahead = lane == ppw, head = lane == 0 && has_prev;
  const uint64_t LE = (rs + 63) & ~63ull;
  const bool donate = kDonate && (ahead || head) && G.ne && !ovl && LE > B0r &&
                      B0r + 16ull * nraw > LE && (G.obh || (rs & 15) == 0 || G.pfull);
  const uint32_t don = donate ? (uint32_t)((LE - B0r) >> 4) : 0u;
  const uint64_t B0 = donate && head ? LE : B0r;
  G.B0 = B0;
  G.nblk = owner ? nraw - (donate ? don : 0u) : (donate ? don : 0u);
  const uint32_t nblk = G.nblk;
  G.hl = nblk && (re & 15) && !(donate && ahead);
  G.hf = nblk && B0 < J.dst_pay && !(G.hl && B0 == BL);
  // last block whole: the next datagram starts at re and fills the block
  // (or, with out_blocks, the bytes past re are scratch)
  G.lfull = G.hl && (ob || ((fl_n & 1) && rs_n == re && re_n >= E && !(cross_n && (fl_n & 2))));
  // out_lines: pad blocks [E, re rounded up to 128) after the owned ones
  const uint32_t npad =
      ol && owner && nblk ? (uint32_t)((((re + 127) & ~127ull) - E) >> 4) : 0u;
  G.npad = npad;

  // the flat block space: this packet's blocks [B0, B0 + 16 F)
  const uint32_t F = ((G.hl && !G.lfull) ? nblk - 1 : nblk) + npad;
  uint32_t incl = F;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, kWave);
    if (lane >= (uint32_t)d) incl += y;
  }
  UnitStream U;
  const uint32_t start0 = incl - F;
  G.flat = F != 0;
  const uint64_t fm = __ballot(G.flat);
  G.rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
  const uint32_t K = (uint32_t)__popcll(fm);
  const uint32_t T0 = __builtin_amdgcn_readfirstlane(__shfl(incl, kWave - 1, kWave));
  U.map = T0 + (1u << kAlign) <= kMapBlocks;
  // interior blocks [i_lo, i_hi): the only ones loaded
  const uint32_t i_lo = G.hf ? 1u : 0u, i_hi = G.hl ? nblk - 1 : nblk;
  const bool has_int = i_hi > i_lo;
  const uint64_t sabs = B0 + (J.src_pay - J.dst_pay);  // input of block B0
  const uint64_t s_first = sabs + 16ull * i_lo, s_end = sabs + 16ull * i_hi;
  // spans: output of every flat block, input of every interior block
  const uint64_t d_lo = wave_ext64_dpp<false>(F ? B0 : ~0ull);
  const uint64_t d_hi = wave_ext64_dpp<true>(F ? B0 + 16ull * F : 0ull);
  const uint64_t s_lo = wave_ext64_dpp<false>(has_int ? s_first : ~0ull);
  const uint64_t s_hi = wave_ext64_dpp<true>(has_int ? s_end : 0ull);
  const bool mis = has_int && (sabs & 3);
  const bool sok = s_hi <= s_lo || s_hi - s_lo <= kMaxSpan;
  U.fast = T0 != 0 && __ballot(mis) == 0 && d_hi - d_lo <= kMaxSpan && sok;
  // map path (buffer streaming only: the generic path walks [0, T) by
  // `locate`): shift the flat space so that slot c sits at d_lo's line phase
  const uint32_t phase = U.map && U.fast && kAlign
                             ? (uint32_t)(d_lo >> 4) & ((1u << kAlign) - 1u)
                             : 0u;
  const uint32_t start = start0 + phase;
  G.start = start;
  U.T = T0 + phase;
  const bool si = s_hi > s_lo;
  const uint64_t sb = si ? s_lo : d_lo;
  if (U.fast) {
    U.B.src = __builtin_amdgcn_make_buffer_rsrc((void *)sb, 0,
                                                (int)(si ? (uint32_t)(s_hi - s_lo) : 0u),
                                                0x00020000);
    U.B.dst = __builtin_amdgcn_make_buffer_rsrc((void *)d_lo, 0, (int)(uint32_t)(d_hi - d_lo),
                                                0x00020000);
  }
  if (U.map && lane < phase) L.role[lane] = (uint8_t)kRankNone;
  if (U.map && lane == kRankNone) {
    L.rec[kRankNone].soff = kOffPhase;
    L.rec[kRankNone].doff = kOffPhase;
  }
  if (G.flat) {
    ChunkRec &R = L.rec[G.rank];
    R.ssub = sabs - 16ull * start;
    R.dsub = B0 - 16ull * start;
    R.soff = (uint32_t)(sabs - sb) - 16u * start;
    R.doff = (uint32_t)(B0 - d_lo) - 16u * start;
    R.sidx = G.hf ? start : kNoIdx;
    // blocks c >= eidx take tab[3]: the special last block and the pad blocks
    const uint32_t eidx = G.lfull ? start + nblk - 1 : (npad ? start + nblk : kNoIdx);
    R.eidx = eidx;
    L.cst[G.rank] = start;
    if (U.map) {
      // the role bytes of this packet's flat blocks [start, start + F)
      uint8_t *rb = L.role;
      const uint32_t e = start + F, rk = G.rank;
      uint32_t c = start;
      for (; c < e && (c & 3); c++) rb[c] = (uint8_t)rk;
      for (; c + 4 <= e; c += 4) *reinterpret_cast<uint32_t *>(rb + c) = rk * 0x01010101u;
      for (; c < e; c++) rb[c] = (uint8_t)rk;
      if (G.hf) rb[start] = (uint8_t)(rk | kRoleFirst);
      for (c = eidx; c < e; c++) rb[c] = (uint8_t)(rk | kRoleLast);
    }
  }
  // records visible to the whole wave (same-wave LDS ops are ordered; this
  // is a compiler barrier plus the LDS drain)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  U.cst = lane < K ? L.cst[lane] : kNoIdx;
  return U;
}

// Step 3b, the contents (while the first stream loads are in flight): key,
// head / tail images, the special blocks' values and the keystreams (the
// store half of the records), and the byte-exact stores of bytes no
// datagram pair covers whole.  Every lane of the wave runs it.
template <int KIND, int DIR, bool MULTI>
__device__ __forceinline__ void fill_unit(const KParams &P, const PacketJob &J,
                                          const uint32_t (&salt)[4], bool do_hash, uint32_t pid,
                                          const PskHot &hot,
                                          const Windows &W, bool owner, uint32_t lane,
                                          bool ob, const Geo &G, WaveLds &L) {
  constexpr uint32_t S = KIND == 0 ? kSalamanderSalt : kXPlusSalt;
  constexpr uint32_t PW = DIR == 0 ? S / 4 : 0;  // salt words in front of the payload
  uint32_t key[8];
  uint32_t sl[4] = {salt[0], salt[1], salt[2], salt[3]};
  // every window register stays allocated until here: a component no image
  // uses would otherwise be handed to the plan while its load is in flight,
  // and overwriting it waits for the load
  if (DIR == 1)
    asm volatile("" ::"v"(W.h0), "v"(W.h1), "v"(W.h2), "v"(W.t0), "v"(W.t1), "v"(W.s0));
  else  // (obfuscate loads no salt block)
    asm volatile("" ::"v"(W.h0), "v"(W.h1), "v"(W.h2), "v"(W.t0), "v"(W.t1));
  const u32x4 wh0 = W.h0, wh1 = W.h1, wh2 = W.h2;
  if (DIR == 1) {  // the wire salt, from the head window
    const u32x4 ws0 = W.s0;
    const uint32_t w[12] = {ws0.x, ws0.y, ws0.z, ws0.w, wh0.x, wh0.y,
                            wh0.z, wh0.w, wh1.x, wh1.y, wh1.z, wh1.w};
    win16(w, (uint32_t)(J.src_pay & 15) + 16 - S, sl);
  }
  // single PSK: the kernarg copy (scalar loads); several: the device table
  derive_key<KIND, MULTI && kPskPre>(do_hash, MULTI ? P.psk_table + pid : &P.psk0, hot, sl,
                                        key);
  const uint64_t rs = G.rs, re = G.re;
  // head image: output bytes [rs, rs + 32) = salt || payload ^ key
  uint32_t hi[8];
  {
    const uint32_t o = (uint32_t)(J.src_pay & 15);
    const uint32_t w0[12] = {0u, 0u, 0u, 0u, wh0.x, wh0.y, wh0.z, wh0.w,
                             wh1.x, wh1.y, wh1.z, wh1.w};
    const uint32_t w1[12] = {wh0.x, wh0.y, wh0.z, wh0.w, wh1.x, wh1.y,
                             wh1.z, wh1.w, wh2.x, wh2.y, wh2.z, wh2.w};
    uint32_t pa[4], pb[4];
    win16(w0, o + 16, pa);
    win16(w1, o + 16, pb);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if ((uint32_t)i < PW) {
        hi[i] = salt[i];
      } else {
        const int k = i - (int)PW;
        hi[i] = (k < 4 ? pa[k] : pb[k - 4]) ^ key[k];
      }
    }
  }
  const uint32_t hx[12] = {hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7], 0u, 0u, 0u, 0u};
  // the same image 16 bytes later (blocks that start before rs: out_blocks)
  const uint32_t hp[12] = {0u, 0u, 0u, 0u, hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
  // tail image: bytes [BL, re) of the last partial output block
  const uint64_t BL = re & ~15ull;
  const uint32_t t = (uint32_t)(re & 15);
  uint32_t ti[4];
  if (tail_from_window(rs, re)) {
    const uint64_t ta = J.src_pay + (BL - J.dst_pay);
    const u32x4 wt0 = W.t0, wt1 = W.t1;
    const uint32_t w[12] = {0u, 0u, 0u, 0u, wt0.x, wt0.y, wt0.z, wt0.w,
                            wt1.x, wt1.y, wt1.z, wt1.w};
    uint32_t ks[4];
    win16(w, (uint32_t)(ta & 15) + 16, ti);
    keywin(key, (uint32_t)(BL - J.dst_pay) & 31u, ks);
#pragma unroll
    for (int j = 0; j < 4; j++) ti[j] ^= ks[j];
  } else if (BL < rs) {  // out_blocks: one block holds the whole output
    win16(hp, (uint32_t)(BL + 16 - rs), ti);
  } else {
    win16(hx, (uint32_t)(BL - rs) & 31u, ti);  // BL - rs <= 16 here (or no tail)
  }
  // the next packet's head image (its salt / first payload bytes)
  const uint32_t nl = (lane + 1) & (kWave - 1);
  uint32_t hn[4];
#pragma unroll
  for (int j = 0; j < 4; j++) hn[j] = shfl32(hi[j], nl);

  // byte-exact stores of the bytes no datagram pair covers whole
  if (owner && G.ne) {
    if ((rs & 15) && !G.pfull && !G.obh) {
      const uint64_t lend = re < G.B0 ? re : G.B0;
      const uint32_t v[4] = {hi[0], hi[1], hi[2], hi[3]};
      store16(rs, v, (uint32_t)(lend - rs));
    }
    if (G.hl && !G.lfull) store16(BL, ti, t);
  }

  // special blocks and keystreams
  uint32_t vf[4] = {0u, 0u, 0u, 0u}, vl[4] = {0u, 0u, 0u, 0u};
  if (G.hf) {
    if (G.B0 < rs) win16(hp, (uint32_t)(G.B0 + 16 - rs), vf);  // out_blocks
    else win16(hx, (uint32_t)(G.B0 - rs), vf);
  }
  if (G.lfull) {
    const uint32_t w[12] = {0u, 0u, 0u, 0u, hn[0], hn[1], hn[2], hn[3], 0u, 0u, 0u, 0u};
    uint32_t sh[4];
    win16(w, 16 - t, sh);
#pragma unroll
    for (int j = 0; j < 4; j++) vl[j] = (ti[j] & range_mask(0, (int)t, j)) | (ob ? 0u : sh[j]);
  }
  uint32_t k0[4], k1[4];
  const uint32_t ph = (uint32_t)(G.B0 - J.dst_pay) & 31u;
  keywin(key, ph, k0);
  keywin(key, (ph + 16) & 31u, k1);
  // tab[c & 1] is the keystream of flat block c
  const bool odd = G.start & 1;
  if (G.flat) {
    ChunkRec &R = L.rec[G.rank];
    R.tab[0] = u32x4{bsel(odd, k1[0], k0[0]), bsel(odd, k1[1], k0[1]),
                     bsel(odd, k1[2], k0[2]), bsel(odd, k1[3], k0[3])};
    R.tab[1] = u32x4{bsel(odd, k0[0], k1[0]), bsel(odd, k0[1], k1[1]),
                     bsel(odd, k0[2], k1[2]), bsel(odd, k0[3], k1[3])};
    R.tab[2] = u32x4{vf[0], vf[1], vf[2], vf[3]};
    R.tab[3] = u32x4{vl[0], vl[1], vl[2], vl[3]};
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------ stream

// Record of flat block c = b0 + lane (c < T) without the block map: the
// last rank r with cst[r] <= c.  b0 is wave-uniform, so this is two ballots,
// a popcount and a scalar walk over the (few) packets that start inside the
// 64-block window.  Always returns a valid record index (0..63), also for
// c >= T.
__device__ __forceinline__ uint32_t locate(uint32_t cst, uint32_t b0, uint32_t c) {
  int pp = __popcll(__ballot(cst <= b0)) - 1;
  uint64_t M = __ballot(cst > b0 && cst < b0 + kWave);
  while (M) {
    const int l = __ffsll((unsigned long long)M) - 1;
    M &= M - 1;
    const uint32_t sl = __builtin_amdgcn_readlane(cst, l);
    pp += c >= sl ? 1 : 0;
  }
  return (uint32_t)(pp < 0 ? 0 : pp);
}

// Buffer-resource streaming.  The wave's input and output spans each fit a
// 32-bit buffer range, described by one SGPR resource per direction.  A
// block past the end (or a special block's load) gets an offset beyond
// num_records: the hardware range check returns zeros for its load and
// drops its store.  So every load/store in the loop is unconditional, with
// no branches, and the compiler's waitcnt accounting stays exact (a
// conditional store makes it fall back to draining).
constexpr uint32_t kOffNone = 0xFFFFFFF0u;
// cache-policy bits of the stream's buffer ops (gfx950: sc0 = 1, nt = 2,
// sc1 = 16)
constexpr int kAuxLd = (kNt & 1) ? 2 : 0;  // nt
constexpr int kAuxSt = (kNt & 2) ? 2 : 0;

// One stream step in flight: U blocks per lane with their keystreams (or
// special values) and output offsets.
template <int U>
struct Step {
  u32x4 v[U];
  u32x4 k[U];
  uint32_t doff[U];
};

// Issue step `base` (a multiple of 64): per block its record (block map:
// one role byte; otherwise `locate`), role and offsets, then the U loads.
// A special block's load is range-checked away (it reads zero) and its
// "keystream" is its precomputed value.
template <int U, bool MAP>
__device__ __forceinline__ void stream_issue(const WaveLds &L, const WaveBufs &B, uint32_t cst,
                                             uint32_t T, uint32_t lane, uint32_t base,
                                             Step<U> &S) {
  uint32_t pp[U], off[U], rl[U];
  // every LDS read of the step first, then the arithmetic, then the loads
  if (MAP) {
#pragma unroll
    for (int u = 0; u < U; u++) rl[u] = L.role[base + u * kWave + lane];
#pragma unroll
    for (int u = 0; u < U; u++) pp[u] = rl[u] & (kWave - 1);  // (past T: garbage, in range)
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) pp[u] = locate(cst, base + u * kWave, base + u * kWave + lane);
  }
  uint64_t sd[U];
  uint32_t idx[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t c = base + u * kWave + lane;
    const ChunkRec &R = L.rec[pp[u]];
    // unconditional record reads (pp is always a valid index), then selects:
    // no divergent branches around the LDS reads
    sd[u] = *reinterpret_cast<const uint64_t *>(&R.soff);
    if (MAP) {
      idx[u] = (rl[u] & kRoleFirst) ? 2u : ((rl[u] & kRoleLast) ? 3u : (c & 1u));
    } else {
      const uint64_t se = *reinterpret_cast<const uint64_t *>(&R.sidx);
      idx[u] = c == (uint32_t)se ? 2u : (c >= (uint32_t)(se >> 32) ? 3u : (c & 1u));
    }
    S.k[u] = R.tab[idx[u]];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t c = base + u * kWave + lane;
    const bool in = c < T;
    S.doff[u] = in ? (uint32_t)(sd[u] >> 32) + 16u * c : kOffNone;
    off[u] = in && idx[u] < 2u ? (uint32_t)sd[u] + 16u * c : kOffNone;
  }
#pragma unroll
  for (int u = 0; u < U; u++) S.v[u] = __builtin_amdgcn_raw_buffer_load_b128(B.src, off[u], 0, kAuxLd);
}

template <int U>
__device__ __forceinline__ void stream_store(const WaveLds &L, const WaveBufs &B,
                                             const Step<U> &S) {
  (void)L;
#pragma unroll
  for (int u = 0; u < U; u++)
    __builtin_amdgcn_raw_buffer_store_b128(S.v[u] ^ S.k[u], B.dst, S.doff[u], 0, kAuxSt);
}

// Double-buffered stream loop.  The caller has issued step 0's loads into
// cur; each iteration issues step i+1's U loads before step i is XORed and
// stored, so a wave keeps U..2U KiB of reads outstanding.
template <int U, bool MAP>
__device__ __forceinline__ void stream_loop(const WaveLds &L, const WaveBufs &B, uint32_t cst,
                                            uint32_t T, uint32_t lane, Step<U> &cur) {
  constexpr uint32_t STEP = kWave * U;
  // unrolled by two with two named steps, so no register copies between them
  Step<U> nxt;
  for (uint32_t base = 0;; base += 2 * STEP) {
    stream_issue<U, MAP>(L, B, cst, T, lane, base + STEP, nxt);
    stream_store<U>(L, B, cur);
    if (base + STEP >= T) break;
    stream_issue<U, MAP>(L, B, cst, T, lane, base + 2 * STEP, cur);
    stream_store<U>(L, B, nxt);
    if (base + 2 * STEP >= T) break;
  }
}

// Fallback for waves whose spans exceed a 32-bit buffer range or whose
// input is not 4-byte aligned: global accesses, any alignment (two aligned
// 16-byte loads + byte funnel per block), one block per lane.
__device__ __noinline__ void stream_generic(const WaveLds &L, uint32_t cst, uint32_t T,
                                            uint32_t lane) {
  for (uint32_t b0 = 0; b0 < T; b0 += kWave) {
    const uint32_t c = b0 + lane < T - 1 ? b0 + lane : T - 1;
    const ChunkRec &R = L.rec[locate(cst, b0, c)];
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    u32x4 k = R.tab[c & 1];
    if (c == R.sidx) {
      k = R.tab[2];
    } else if (c >= R.eidx) {  // the special last block or a pad block
      k = R.tab[3];
    } else {
      const uint64_t sa = R.ssub + 16ull * c;
      load_window(sa, sa + 16, sa, w);
    }
    if (b0 + lane < T) gst<u32x4>(R.dsub + 16ull * c, u32x4{w[0], w[1], w[2], w[3]} ^ k);
  }
}

// ------------------------------------------------------------ the kernel

// WPB: wavefronts per workgroup (independent units; they share nothing).
template <int KIND, int DIR, bool MULTI, int U, int WPB>
__global__ __launch_bounds__(WPB * kWave) void obfs_kernel(const KParams P) {
  __shared__ WaveLds lds[WPB];
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wv = threadIdx.x / kWave;
  uint32_t lb = blockIdx.x;
  if (P.xcd) {  // eighths (a bijection of [0, gridDim.x) for any grid size)
    const uint32_t ng = gridDim.x, q = ng / 8, r = ng % 8, xcd = lb % 8, ix = lb / 8;
    lb = xcd < r ? xcd * (q + 1) + ix : r * (q + 1) + (xcd - r) * q + ix;
  }
  const uint64_t unit = (uint64_t)lb * WPB + wv;
  const uint32_t ppw = P.ppw;
  const uint64_t first = unit * ppw;
  if (first >= P.n) return;
  SQ_STAMP(0);
  bool valid, owner;
  const uint32_t p = lane_packet(first, ppw, lane, P.n, valid, owner);
  // 1. descriptor (deobfuscate: the salt load) and the image windows: loads
  RawDesc d;
  fetch_desc<KIND, DIR, MULTI>(P, p, valid, (uint32_t)first, d);
  constexpr uint32_t kSalt = KIND == 0 ? kSalamanderSalt : kXPlusSalt;
  // device salts depend on p alone: computed while the descriptor loads fly
  // (round 4: -2.6 % on configs[1] against computing them after the loads
  // land), by quads (round 5: -0.8 % configs[1], -1.9 % ragged against one
  // whole block per lane)
  if (DIR == 0 && P.device_salt)
    device_salts_wave<kSalt>(P, first, ppw, lane, p, valid,
                             reinterpret_cast<uint32_t *>(lds[wv].role), d.salt);
  PacketJob J;
  uint32_t salt[4];
  bool do_hash;
  const PskEntry *E;
  uint32_t olen;
  finalize_desc<KIND, DIR, MULTI>(P, p, valid, d, J, salt, do_hash, E, olen);
  PskHot hot;
  if constexpr (MULTI && kPskPre) {
    load_hot<KIND>(P, E, hot);  // in flight during the plan
  }
  SQ_STAMP(1);
  Windows W;
  fetch_windows<DIR, kSalt>(J, do_hash, W);
  if (owner) P.out_len[p] = olen;
  // 3a. plan
  Geo G;
  WaveLds &L = lds[wv];
  const bool ob = P.out_blocks != 0;
  const UnitStream S = plan_unit(J, owner, lane, ppw, first != 0, ob, P.out_lines != 0, L, G);
  SQ_STAMP(2);
  Step<U> cur;
  const uint32_t pid = MULTI && d.pid < P.n_psk ? d.pid : 0u;
  reload_windows<DIR, kSalt>(J, do_hash, W);
  // 2 + 3b. key and block contents
  fill_unit<KIND, DIR, MULTI>(P, J, salt, do_hash, pid, hot, W, owner, lane, ob, G, L);
  SQ_STAMP(3);
  // 4. the stream
  if (S.fast && S.map) {
    stream_issue<U, true>(L, S.B, S.cst, S.T, lane, 0, cur);
    stream_loop<U, true>(L, S.B, S.cst, S.T, lane, cur);
  } else if (S.fast) {
    stream_issue<U, false>(L, S.B, S.cst, S.T, lane, 0, cur);
    stream_loop<U, false>(L, S.B, S.cst, S.T, lane, cur);
  } else if (S.T != 0) {
    stream_generic(L, S.cst, S.T, lane);
  }
#if SQ_TIMELINE
  SQ_STAMP(4);
  // when the wave's last store has left (the end of its life)
  __builtin_amdgcn_s_waitcnt(0);
  SQ_STAMP(5);
#endif
}

// ------------------------------------------------------------ PSK prepare

__device__ __forceinline__ uint64_t ld64le(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
__device__ __forceinline__ uint32_t ld32be(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// One thread per PSK: compress the PSK-only leading blocks, lay out the final
// block template.  Runs once per keyring (connection setup), not per packet.
__global__ void psk_prepare_kernel(int kind, const uint8_t *blob, const uint64_t *off,
                                   const uint32_t *len, uint32_t count, PskEntry *out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint8_t *psk = blob + off[k];
  const uint32_t L = len[k];
  PskEntry E;
  uint8_t tm[256];
  for (int i = 0; i < 256; i++) tm[i] = 0;
  E.psk_len = L;
  E.kind = (uint32_t)kind;
  if (kind == 0) {
    // BLAKE2b: every PSK-only 128-byte block is followed by salt bytes, so it
    // is never the final block (RFC 7693 section 3.3).
    uint64_t h[8];
    b2_init256(h);
    const uint32_t nfull = L / 128;
    for (uint32_t bk = 0; bk < nfull; bk++) {
      uint64_t m[16];
      for (int j = 0; j < 16; j++) m[j] = ld64le(psk + 128 * bk + 8 * j);
      b2_compress(h, m, 128ull * (bk + 1), false);
    }
    const uint32_t tail = L - 128 * nfull;
    const uint32_t tot = tail + kSalamanderSalt;
    for (uint32_t i = 0; i < tail; i++) tm[i] = psk[128 * nfull + i];
    for (int i = 0; i < 8; i++) E.h[i] = h[i];
    for (int j = 0; j < 32; j++) E.m[j] = ld64le(tm + 8 * j);
    E.nblocks = tot > 128 ? 2 : 1;
    E.salt_pos = tail;
    E.t_first = 128ull * nfull + 128;
    E.t_last = 128ull * nfull + tot;
  } else {
    // SHA-256: Merkle-Damgard with 0x80 pad and 64-bit big-endian bit length
    uint32_t st[8];
    s2_init(st);
    const uint32_t nfull = L / 64;
    for (uint32_t bk = 0; bk < nfull; bk++) {
      uint32_t m[16];
      for (int j = 0; j < 16; j++) m[j] = ld32be(psk + 64 * bk + 4 * j);
      s2_compress(st, m);
    }
    const uint32_t tail = L - 64 * nfull;
    const uint32_t used = tail + kXPlusSalt + 1 + 8;
    const uint32_t nb = used > 64 ? 2 : 1;
    for (uint32_t i = 0; i < tail; i++) tm[i] = psk[64 * nfull + i];
    tm[tail + kXPlusSalt] = 0x80;
    const uint64_t bits = ((uint64_t)L + kXPlusSalt) * 8;
    for (int i = 0; i < 8; i++) tm[64 * nb - 1 - i] = (uint8_t)(bits >> (8 * i));
    uint32_t *h32 = reinterpret_cast<uint32_t *>(E.h);
    for (int i = 0; i < 16; i++) h32[i] = i < 8 ? st[i] : 0u;
    uint32_t *m32 = reinterpret_cast<uint32_t *>(E.m);
    for (int j = 0; j < 64; j++) m32[j] = j < 32 ? ld32be(tm + 4 * j) : 0u;
    E.nblocks = nb;
    E.salt_pos = tail;
    E.t_first = 0;
    E.t_last = 0;
  }
  out[k] = E;
}

// Wavefronts per workgroup.  A workgroup's slots are released only when all
// of its waves have ended, so a 4-wave group holds its finished waves' slots
// until its slowest sibling is done; 1-wave groups avoid that but leave the
// wave-to-SIMD placement to the dispatcher.  Measured per kernel in one
// process: 2-wave groups are the fastest or within
// 1.5 % of it for every kernel and direction (Salamander obfuscate 2.6 %
// faster than 4-wave groups, XPlus obfuscate 3.4 % faster than 1-wave ones).
template <int KIND, int DIR>
constexpr int kWavesPerGroup = kWpb;

// sqobfs_debug_time_next_launch: events the calling thread's next launch
// records with its own dispatch (no marker packets between kernels)
thread_local hipEvent_t t_time_ev[2] = {nullptr, nullptr};

template <int KIND, int DIR, bool MULTI, int U, int WPB>
static int launch_k(const KParams &P, hipStream_t s) {
  const uint64_t units = ((uint64_t)P.n + P.ppw - 1) / P.ppw;
  const uint64_t blocks = (units + WPB - 1) / WPB;
  // HIP keeps a failed call's error until it is read: clear one left by an
  // earlier call on this thread (the caller's), or it would be taken for
  // this launch's and the launch reported as refused although it ran
  (void)hipGetLastError();
  if (t_time_ev[0] || t_time_ev[1]) {
    hipEvent_t e0 = t_time_ev[0], e1 = t_time_ev[1];
    t_time_ev[0] = t_time_ev[1] = nullptr;
    hipExtLaunchKernelGGL((obfs_kernel<KIND, DIR, MULTI, U, WPB>), dim3((uint32_t)blocks),
                          dim3(WPB * kWave), 0, s, e0, e1, 0u, P);
  } else {
    hipLaunchKernelGGL((obfs_kernel<KIND, DIR, MULTI, U, WPB>), dim3((uint32_t)blocks),
                       dim3(WPB * kWave), 0, s, P);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int KIND, int DIR, bool MULTI>
static int launch_one(const KParams *kp, hipStream_t s) {
  constexpr int U = kU;
  KParams P = *kp;
  if (P.ppw == 0) P.ppw = kPktPerWave;
  if (P.ppw > kMaxUnitPackets) {
    t_time_ev[0] = t_time_ev[1] = nullptr;
    return -1;
  }
  const uint64_t units = ((uint64_t)P.n + P.ppw - 1) / P.ppw;
  P.xcd = units >= kXcdMinUnits ? 1u : 0u;
  return launch_k<KIND, DIR, MULTI, U, kWavesPerGroup<KIND, DIR>>(P, s);
}

}  // namespace sq

extern "C" void sq_time_next_launch(void *start, void *stop) {
  sq::t_time_ev[0] = (hipEvent_t)start;
  sq::t_time_ev[1] = (hipEvent_t)stop;
}

extern "C" int sq_launch_obfs(int kind, int dir, const sq::KParams *kp, void *stream) {
  using namespace sq;
  if (kp->n == 0) {
    t_time_ev[0] = t_time_ev[1] = nullptr;
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  const bool multi = kp->psk_id != nullptr;
  const int sel = (kind << 2) | (dir << 1) | (multi ? 1 : 0);
  switch (sel) {
    case 0: return launch_one<0, 0, false>(kp, s);
    case 1: return launch_one<0, 0, true>(kp, s);
    case 2: return launch_one<0, 1, false>(kp, s);
    case 3: return launch_one<0, 1, true>(kp, s);
    case 4: return launch_one<1, 0, false>(kp, s);
    case 5: return launch_one<1, 0, true>(kp, s);
    case 6: return launch_one<1, 1, false>(kp, s);
    case 7: return launch_one<1, 1, true>(kp, s);
  }
  return -1;
}

#if SQ_TIMELINE
extern "C" int sqobfs_debug_timeline(uint64_t *host, uint64_t words) {
  const uint64_t cap = (uint64_t)sq::kTlWaves * sq::kTlStamps;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sq::g_timeline),
                             (words < cap ? words : cap) * sizeof(uint64_t)) == hipSuccess
             ? 0
             : -3;
}
#endif

extern "C" int sq_launch_psk_prepare(int kind, const uint8_t *blob, const uint64_t *off,
                                     const uint32_t *len, uint32_t count, sq::PskEntry *out,
                                     void *stream) {
  if (count == 0) return 0;
  const uint32_t threads = 64;
  (void)hipGetLastError();  // (a stale error is not this launch's: launch_k)
  hipLaunchKernelGGL(sq::psk_prepare_kernel, dim3((count + threads - 1) / threads),
                     dim3(threads), 0, (hipStream_t)stream, kind, blob, off, len, count, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
