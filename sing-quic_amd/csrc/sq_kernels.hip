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
// Work decomposition (one wavefront = PPW = 32 packets, independent waves):
//   1. descriptor  lane l < PPW owns packet PPW*wave + l: reads its offsets,
//                  lengths and salt (obfs: salt array; deobfs: first S wire
//                  bytes).
//   2. key         lane l hashes its own packet's psk||salt (BLAKE2b-256 or
//                  SHA-256) starting from the keyring's per-PSK midstate:
//                  PPW different packets hashed in parallel.
//   3. split       each packet's output is cut at 16-byte boundaries of the
//                  DESTINATION address: "full" chunks (16 payload bytes) and
//                  at most ~3 "edge" chunks (salt bytes, unaligned head,
//                  tail).  A wave prefix-sum over full-chunk counts builds a
//                  flat chunk space for the wave's packets; each packet's
//                  addressing and its two 16-byte keystream phases go to LDS.
//   4. edges       the owner lane writes its packet's edge chunks (byte-exact
//                  masked stores; loads only 16-byte-aligned blocks that hold
//                  valid bytes, so nothing outside a packet is ever touched).
//   5. stream      the wave walks the flat chunk space, 64 lanes x U chunks
//                  per step: one dwordx4 load, XOR with the LDS keystream,
//                  one aligned dwordx4 store per chunk.  Chunk -> packet is a
//                  ballot/popcount on the prefix sums held in registers.
// Every payload byte is read once and every output byte written once; the
// key never leaves LDS/registers.  Measured HBM traffic is 1.05x the
// algorithmic bytes (boundary lines: DESIGN.md section 5).
#include <hip/hip_runtime.h>

#include "sq_bytes.h"
#include "sq_hash.h"
#include "sq_internal.h"
#include "sq_obfs_key.h"

namespace sq {

// Streaming policy of the bulk chunk loads / stores (SQ_NT bit 0: loads,
// bit 1: stores).  Payload bytes are touched exactly once, so nontemporal
// (`nt`) accesses keep them from displacing useful L2 lines.
#ifndef SQ_NT
#define SQ_NT 3
#endif
#ifndef SQ_U
#define SQ_U 6
#endif


// Timing-only ablation builds (scripts/ablate.sh; never the shipped .so):
// 1 = skip edge chunks, 2 = skip key derivation, 3 = skip the chunk stream,
// 4 = skip edges and key derivation.
#ifndef SQ_ABLATE
#define SQ_ABLATE 0
#endif
// Packets per wavefront (<= 64).  Fewer packets per wave = shorter, more
// numerous work units: a smaller address window in flight and a shorter
// tail, at the price of idle lanes during the per-lane key derivation.
#ifndef SQ_PPW
#define SQ_PPW 32
#endif
constexpr int kPktPerWave = SQ_PPW;
// Full chunks start and end on 64-byte line boundaries (1) or on 16-byte
// chunk boundaries (0).
#ifndef SQ_LINE_EDGES
#define SQ_LINE_EDGES 0
#endif
#ifndef SQ_TIMELINE
#define SQ_TIMELINE 0
#endif
// Wave priority experiment (timing builds): 1 = raise the priority of waves
// once they stream, 2 = raise it while they prepare (descriptor, hash, edges).
#ifndef SQ_PRIO
#define SQ_PRIO 0
#endif

#define SQ_STR2(x) #x
#define SQ_STR(x) SQ_STR2(x)
extern "C" const char *sqobfs_build_info(void) {
  return "gfx950 obfs_kernel U=" SQ_STR(SQ_U) " PPW=" SQ_STR(SQ_PPW) " NT=" SQ_STR(SQ_NT)
         " block=" SQ_STR(SQ_BLOCK) " ablate=" SQ_STR(SQ_ABLATE);
}

constexpr uint32_t kMaxPacket = 1u << 26;  // per-packet length bound (u32 chunk math)
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

// ------------------------------------------------------------ edge chunks

struct PacketJob {
  uint64_t src_pay;  // address of payload byte 0 in the input
  uint64_t dst_pay;  // address of payload byte 0 in the output
  uint64_t len;      // payload bytes to transform
  uint32_t pre;      // salt bytes written in front of dst_pay (obfs) or 0
};

// Output bytes [a, b) of the 16-byte output block at A (other bytes zero):
// salt bytes and/or payload bytes XOR keystream.  Reads only the 16-byte
// input blocks that hold payload bytes of the range.
__device__ __forceinline__ void block_val(const PacketJob &J, const uint32_t (&key)[8],
                                          const uint32_t (&salt)[4], uint64_t A, uint32_t a,
                                          uint32_t b, uint32_t (&val)[4]) {
#pragma unroll
  for (int j = 0; j < 4; j++) val[j] = 0u;
  const int64_t dp = (int64_t)(J.dst_pay - A);  // payload starts dp bytes into the block
  const uint32_t pay_lo = dp > (int64_t)a ? (uint32_t)(dp < 16 ? dp : 16) : a;
  if (pay_lo < b) {
    const uint64_t X = J.src_pay - (uint64_t)dp;  // input address of output byte A
    uint32_t win[4], ks[4];
    load_window(X + pay_lo, X + b, X, win);
    keywin(key, (uint32_t)(A - J.dst_pay) & 31u, ks);
#pragma unroll
    for (int j = 0; j < 4; j++) val[j] = (win[j] ^ ks[j]) & range_mask(pay_lo, b, j);
  }
  if (J.pre && dp > (int64_t)a) {
    const uint32_t se = dp < (int64_t)b ? (uint32_t)dp : b;  // salt bytes [a, se)
    const uint32_t w[12] = {0u, 0u, 0u, 0u, salt[0], salt[1], salt[2], salt[3], 0u, 0u, 0u, 0u};
    uint32_t sw[4];
    win16(w, (uint32_t)(16 + (int64_t)J.pre - dp), sw);
#pragma unroll
    for (int j = 0; j < 4; j++) val[j] |= sw[j] & range_mask(a, se, j);
  }
}

// Byte-exact store of output bytes [A0, A1) (any alignment, edge chunks of
// small packets and of packets without an adjacent neighbour).
__device__ __forceinline__ void edge_span(const PacketJob &J, const uint32_t (&key)[8],
                                          const uint32_t (&salt)[4], uint64_t A0,
                                          uint64_t A1) {
  for (uint64_t A = A0 & ~15ull; A < A1; A += 16) {
    const uint32_t a = (uint32_t)((A0 > A ? A0 : A) - A);
    const uint32_t b = (uint32_t)((A1 < A + 16 ? A1 : A + 16) - A);
    uint32_t val[4];
    block_val(J, key, salt, A, a, b, val);
    store_partial(A, val, a, b);
  }
}

// ------------------------------------------------------------ chunk stream

// LDS record per packet (48 B): input/output addressing for flat chunk c
// (addr = base + 16*c) and the keystream for even / odd c.
struct alignas(16) ChunkRec {
  uint64_t ssub, dsub;
  u32x4 ks[2];
};

// Packet owning flat chunk c = b0 + lane (c < T): the last lane l with
// start[l] <= c.  b0 is wave-uniform, so this is two ballots, a popcount and
// a scalar walk over the (few) packets that start inside the 64-chunk window.
// Always returns a valid record index (0..63), also for c >= T.
__device__ __forceinline__ uint32_t locate(uint32_t start, uint32_t b0, uint32_t c) {
  int pp = __popcll(__ballot(start <= b0)) - 1;
  uint64_t M = __ballot(start > b0 && start < b0 + kWave);
  while (M) {
    const int l = __ffsll((unsigned long long)M) - 1;
    M &= M - 1;
    const uint32_t sl = __builtin_amdgcn_readlane(start, l);
    pp += c >= sl ? 1 : 0;
  }
  return (uint32_t)pp;
}

// Buffer-resource streaming.  The wave's input and output spans (all its
// full chunks) each fit a 32-bit buffer range, described by one SGPR
// resource per direction.  A chunk past the end gets an offset beyond
// num_records: the hardware range check returns zeros for its load and
// drops its store.  So every load/store in the loop is unconditional, with
// no padding writes and no branches, and the compiler's waitcnt accounting
// stays exact (a conditional store makes it fall back to draining).
constexpr uint32_t kOffNone = 0xFFFFFFF0u;
// cache-policy bits of the stream's buffer ops (gfx950: sc0 = 1, nt = 2,
// sc1 = 16); SQ_AUXLD / SQ_AUXST override them in timing builds
#ifdef SQ_AUXLD
constexpr int kAuxLd = SQ_AUXLD;
#else
constexpr int kAuxLd = (SQ_NT & 1) ? 2 : 0;  // nt
#endif
#ifdef SQ_AUXST
constexpr int kAuxSt = SQ_AUXST;
#else
constexpr int kAuxSt = (SQ_NT & 2) ? 2 : 0;
#endif

struct WaveBufs {
  __amdgpu_buffer_rsrc_t src, dst;
  uint32_t sbase, dbase;  // low 32 bits of the span bases
};

__device__ __forceinline__ uint32_t src_off(const ChunkRec *wrec, const WaveBufs &B,
                                            uint32_t pp, uint32_t c, uint32_t T) {
  return c < T ? (uint32_t)wrec[pp].ssub - B.sbase + 16u * c : kOffNone;
}

template <int U>
__device__ __forceinline__ void stream_issue(const ChunkRec *wrec, const WaveBufs &B,
                                             uint32_t start, uint32_t T, uint32_t lane,
                                             uint32_t base, u32x4 (&v)[U], uint32_t (&pp)[U]) {
  uint32_t off[U];
  // all packet lookups (SALU + ballots) first, then all LDS reads, then all
  // loads: one LDS round trip per step instead of one per chunk
#pragma unroll
  for (int u = 0; u < U; u++) pp[u] = locate(start, base + u * kWave, base + u * kWave + lane);
#pragma unroll
  for (int u = 0; u < U; u++) off[u] = src_off(wrec, B, pp[u], base + u * kWave + lane, T);
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(B.src, off[u], 0, kAuxLd);
}

__device__ __forceinline__ void store_chunk(const ChunkRec *wrec, const WaveBufs &B,
                                            uint32_t pp, uint32_t c, uint32_t T, u32x4 v) {
  const ChunkRec &R = wrec[pp];
  const uint32_t off = c < T ? (uint32_t)R.dsub - B.dbase + 16u * c : kOffNone;
  __builtin_amdgcn_raw_buffer_store_b128(v ^ R.ks[c & 1], B.dst, off, 0, kAuxSt);
}

// Double-buffered stream loop.  The caller has issued step 0's loads into
// cur/cpp (before the edge chunks, so the two overlap); each iteration issues
// step i+1's U loads before step i is XORed and stored, so a wave keeps
// U..2U KiB of reads outstanding.  Loads past T are range-checked away.
template <int U>
__device__ __forceinline__ void stream_loop(const ChunkRec *wrec, const WaveBufs &B,
                                            uint32_t start, uint32_t T, uint32_t lane,
                                            u32x4 (&cur)[U], uint32_t (&cpp)[U]) {
  constexpr uint32_t STEP = kWave * U;
  for (uint32_t base = 0; base < T; base += STEP) {
    u32x4 nxt[U];
    uint32_t npp[U];
    stream_issue<U>(wrec, B, start, T, lane, base + STEP, nxt, npp);
#pragma unroll
    for (int u = 0; u < U; u++) store_chunk(wrec, B, cpp[u], base + u * kWave + lane, T, cur[u]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      cur[u] = nxt[u];
      cpp[u] = npp[u];
    }
  }
}

// Fallback for waves whose spans exceed a 32-bit buffer range or whose
// input chunks are not 4-byte aligned: global accesses, any alignment
// (two aligned 16-byte loads + byte funnel per chunk), one chunk per lane.
__device__ __noinline__ void stream_generic(const ChunkRec *wrec, uint32_t start, uint32_t T,
                                            uint32_t lane) {
  for (uint32_t b0 = 0; b0 < T; b0 += kWave) {
    const uint32_t c = min(b0 + lane, T - 1);
    const ChunkRec &R = wrec[locate(start, b0, c)];
    const uint64_t sa = R.ssub + 16ull * c;
    uint32_t w[4];
    if ((sa & 3) == 0) {
      const u32x4 x = gld<u32x4_a4>(sa);
      w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
    } else {
      load_window(sa, sa + 16, sa, w);
    }
    if (b0 + lane < T) gst<u32x4>(R.dsub + 16ull * c, u32x4{w[0], w[1], w[2], w[3]} ^ R.ks[c & 1]);
  }
}

// 64-bit wave min / max (butterfly), result wave-uniform.
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_xor((unsigned long long)x, d, kWave);
    x = y < x ? y : x;
  }
  return x;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t x) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_xor((unsigned long long)x, d, kWave);
    x = y > x ? y : x;
  }
  return x;
}
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  return b2_pack(__builtin_amdgcn_readfirstlane((uint32_t)x),
                 __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)));
}

// Timing-only timeline builds (SQ_TIMELINE=1, never the shipped .so): every
// stream wave records s_memrealtime (100 MHz) at start, at the start of its
// stream and at exit; scripts/timeline.py reads them back after one launch.
#if SQ_TIMELINE
constexpr uint64_t kTimelineWaves = 1u << 20;
__device__ uint64_t g_timeline[3 * kTimelineWaves];
extern "C" int sq_timeline_copy(uint64_t *host, uint64_t waves) {
  if (waves > kTimelineWaves) waves = kTimelineWaves;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_timeline), 3 * 8 * waves, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
struct TimelineRec {
  uint64_t t0, t1;
  __device__ ~TimelineRec() {
    if ((threadIdx.x & (kWave - 1)) == 0) {
      const uint64_t w = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
      if (w < kTimelineWaves) {
        g_timeline[3 * w] = t0;
        g_timeline[3 * w + 1] = t1;
        g_timeline[3 * w + 2] = __builtin_amdgcn_s_memrealtime();
      }
    }
  }
};
#define SQ_TL_START const uint64_t tl0_ = __builtin_amdgcn_s_memrealtime();
#define SQ_TL_STREAM TimelineRec tl_rec_{tl0_, __builtin_amdgcn_s_memrealtime()};
#else
#define SQ_TL_START
#define SQ_TL_STREAM
#endif

// ------------------------------------------------------------ per-packet steps

// Device salt of packet p (SQOBFS_FLAG_DEVICE_SALT): bytes [(p % (64/S))*S,
// +S) of ChaCha20 keystream block p / (64/S), so the batch's salts are the
// keystream's first n*S bytes.  Each lane computes its own packet's block
// (lanes sharing a block compute it redundantly: same instruction stream).
template <uint32_t S>
__device__ __forceinline__ void device_salt(const KParams &P, uint32_t p, uint32_t (&salt)[4]) {
  constexpr uint32_t per_block = 64 / S;  // 8 Salamander, 4 XPlus
  uint32_t blk[16];
  chacha20_block(P.salt_key, p / per_block, P.salt_nonce, blk);
  // word offset (p % per_block) * S/4: barrel-select S/4 words
  const uint32_t q = (p % per_block) * (S / 4);
  uint32_t y[16];
#pragma unroll
  for (int j = 0; j < 16; j++) y[j] = blk[j];
#pragma unroll
  for (int sh = 8; sh >= 1; sh >>= 1) {
    const bool b = q & sh;
#pragma unroll
    for (int j = 0; j + sh < 16; j++) y[j] = bsel(b, y[j + sh], y[j]);
  }
#pragma unroll
  for (uint32_t k = 0; k < S / 4; k++) salt[k] = y[k];
  if (P.salt_out) {
    uint32_t *so = reinterpret_cast<uint32_t *>(P.salt_out + (uint64_t)p * S);
#pragma unroll
    for (uint32_t k = 0; k < S / 4; k++) so[k] = salt[k];
  }
}

// Step 1, descriptor: packet p's job (addresses and length of the XOR
// stream, salt bytes to prepend), its salt (obfuscate: the salt array;
// deobfuscate: the first S wire bytes), whether it needs a key, and its
// out_len (the quirk table of include/sqobfs.h).
template <int KIND, int DIR, bool MULTI>
__device__ __forceinline__ void describe(const KParams &P, uint32_t p, bool valid, PacketJob &J,
                                         uint32_t (&salt)[4], bool &do_hash,
                                         const PskEntry *&E, uint32_t &olen) {
  constexpr uint32_t S = KIND == 0 ? kSalamanderSalt : kXPlusSalt;
  J = {0, 0, 0, 0};
  do_hash = false;
  E = &P.psk0;
  olen = 0;
  if (!valid) return;
  const uint64_t in_base = (uint64_t)P.in + P.in_off[p];
  const uint64_t out_base = (uint64_t)P.out + P.out_off[p];
  const uint32_t len = P.in_len[p];
  bool bad = false;
  if (MULTI) {
    const uint32_t pid = P.psk_id[p];
    if (pid >= P.n_psk) bad = true;
    else E = P.psk_table + pid;
  }
  uint32_t cap = len;
  if (KIND == 1 && DIR == 1 && P.in_cap) {
    const uint32_t c = P.in_cap[p];
    cap = c > len ? c : len;
  }
  if (len > kMaxPacket || cap > kMaxPacket) {
    olen = kBadLen;
  } else if (bad) {
    olen = kBadPsk;
  } else if (DIR == 0) {  // obfuscate: wire = salt || payload ^ key
    if (P.device_salt) {
      device_salt<S>(P, p, salt);
    } else {
      const uint32_t *sp = reinterpret_cast<const uint32_t *>(P.salt + (uint64_t)p * S);
#pragma unroll
      for (uint32_t k = 0; k < S / 4; k++) salt[k] = sp[k];
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
    uint32_t w[4];
    load_window(in_base, in_base + S, in_base, w);
#pragma unroll
    for (uint32_t k = 0; k < S / 4; k++) salt[k] = w[k];
    J = {in_base + S, out_base, (uint64_t)cap - S, 0};
    olen = len - S;
    do_hash = true;
  }
}

// Step 2, key: lane-parallel, one packet per lane.
template <int KIND>
__device__ __forceinline__ void derive_key(bool do_hash, const PskEntry *E,
                                           const uint32_t (&salt)[4], uint32_t (&key)[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) key[i] = 0u;
#if SQ_ABLATE == 2 || SQ_ABLATE == 4  // timing-only build: no key derivation
  if (do_hash) { key[0] = salt[0]; key[1] = salt[1]; do_hash = false; }
#endif
  if (do_hash) {
    if (KIND == 0) salamander_key(E, salt, key);
    else xplus_key(E, salt, key);
  }
}

// Steps 3-5 for the packets of one wave (one per lane, any subset of lanes
// may be idle with J.len == 0):
//   3. split every packet's output at 16-byte boundaries of the destination
//      into full chunks (a flat chunk space over the wave, by prefix sum) and
//      edges (salt bytes, unaligned head, tail);
//   4. write the edges (owner lane, byte-exact, plain stores);
//   5. stream the flat chunk space with nt loads and stores.
// The edge bytes of a boundary line and the nt stream stores of the rest of
// that line merge in L2: skipping the edges (SQ_ABLATE=1) leaves those lines
// partial and costs ~10 %.  SQ_LINE_EDGES=1 (timing builds) instead streams
// only whole 64-byte lines and writes the boundary lines as edges: no
// partial nt stores at all, but the longer edge phase costs ~3 % more than
// it saves.
template <int U>
__device__ __forceinline__ void transform(const PacketJob &J, const uint32_t (&key)[8],
                                          const uint32_t (&salt)[4], uint32_t lane,
                                          ChunkRec *wrec) {
  // ---- 3. split into full chunks (flat, streamed) and edges (owner lane)
  constexpr uint64_t kAl = SQ_LINE_EDGES ? 64 : 16;
  const uint64_t rs = J.dst_pay - J.pre, re = J.dst_pay + J.len;
  const uint64_t fa = (J.dst_pay + kAl - 1) & ~(kAl - 1), fb = re & ~(kAl - 1);
  const uint32_t F = (J.len && fb > fa) ? (uint32_t)((fb - fa) >> 4) : 0u;
  uint32_t incl = F;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, kWave);
    if (lane >= (uint32_t)d) incl += y;
  }
  const uint32_t start = incl - F;
  const uint32_t T = __shfl(incl, kWave - 1, kWave);
  const uint64_t s_first = J.src_pay + (fa - J.dst_pay);  // input of the first full chunk
  {
    uint32_t k0[4], k1[4];
    const uint32_t r0 = (uint32_t)(fa - J.dst_pay) & 31u;
    keywin(key, r0, k0);
    keywin(key, r0 + 16, k1);
    const bool odd = start & 1;
    ChunkRec R;
    R.ssub = s_first - 16ull * start;
    R.dsub = fa - 16ull * start;
    R.ks[0] = u32x4{bsel(odd, k1[0], k0[0]), bsel(odd, k1[1], k0[1]),
                    bsel(odd, k1[2], k0[2]), bsel(odd, k1[3], k0[3])};
    R.ks[1] = u32x4{bsel(odd, k0[0], k1[0]), bsel(odd, k0[1], k1[1]),
                    bsel(odd, k0[2], k1[2]), bsel(odd, k0[3], k1[3])};
    wrec[lane] = R;
  }
  // wave spans of the full chunks, for the two buffer resources
  const bool has = F != 0;
  const uint64_t s_lo = uniform64(wave_min64(has ? s_first : ~0ull));
  const uint64_t s_hi = uniform64(wave_max64(has ? s_first + 16ull * F : 0ull));
  const uint64_t d_lo = uniform64(wave_min64(has ? fa : ~0ull));
  const uint64_t d_hi = uniform64(wave_max64(has ? fb : 0ull));
  const bool mis = has && (s_first & 3);
  constexpr uint64_t kMaxSpan = 0xFFFFFF00ull;
  const bool fast = T != 0 && SQ_ABLATE != 3 && __ballot(mis) == 0 &&
                    s_hi - s_lo <= kMaxSpan && d_hi - d_lo <= kMaxSpan;
  // LDS records visible to the whole wave (same-wave LDS ops are ordered;
  // this is a compiler barrier plus the LDS drain)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  SQ_TL_STREAM
#if SQ_PRIO == 1
  __builtin_amdgcn_s_setprio(3);
#elif SQ_PRIO == 2
  __builtin_amdgcn_s_setprio(0);
#endif

  // ---- 4. edges: salt bytes and the partial lines at both ends.  They never
  // overlap the full chunks' input or output bytes.
  if (SQ_ABLATE != 1 && SQ_ABLATE != 4 && re > rs) {
    if (F) {
      edge_span(J, key, salt, rs, fa);
      edge_span(J, key, salt, fb, re);
    } else {
      edge_span(J, key, salt, rs, re);
    }
  }

  WaveBufs B;
  u32x4 cur[U];
  uint32_t cpp[U];
  if (fast) {
    B.src = __builtin_amdgcn_make_buffer_rsrc((void *)s_lo, 0, (int)(uint32_t)(s_hi - s_lo),
                                              0x00020000);
    B.dst = __builtin_amdgcn_make_buffer_rsrc((void *)d_lo, 0, (int)(uint32_t)(d_hi - d_lo),
                                              0x00020000);
    B.sbase = (uint32_t)s_lo;
    B.dbase = (uint32_t)d_lo;
    stream_issue<U>(wrec, B, start, T, lane, 0, cur, cpp);
  }

  // ---- 5. stream the flat full-chunk space
  if (fast) stream_loop<U>(wrec, B, start, T, lane, cur, cpp);
  else if (T != 0 && SQ_ABLATE != 3) stream_generic(wrec, start, T, lane);
}

// ------------------------------------------------------------ kernels

// The kernel: each wave owns kPktPerWave consecutive packets (descriptor ->
// key -> transform).  A two-pass variant (a key kernel with 64 hashes per
// wave, then short stream-only tiles of 4-32 packets per wave) was measured
// and dropped: its key pass alone took 74-85 us on configs[1] and the stream
// pass was no faster than this kernel's stream.
template <int KIND, int DIR, bool MULTI, int U>
__global__ __launch_bounds__(kBlock) void obfs_kernel(const KParams P) {
  __shared__ ChunkRec recs[kWavesPerBlock][kWave];
  SQ_TL_START
#if SQ_PRIO == 2
  __builtin_amdgcn_s_setprio(3);
#endif
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wv = threadIdx.x / kWave;
  const uint64_t p64 = ((uint64_t)blockIdx.x * kWavesPerBlock + wv) * kPktPerWave + lane;
  const bool valid = lane < (uint32_t)kPktPerWave && p64 < P.n;
  const uint32_t p = (uint32_t)p64;
  PacketJob J;
  uint32_t salt[4] = {0u, 0u, 0u, 0u};
  bool do_hash;
  const PskEntry *E;
  uint32_t olen;
  describe<KIND, DIR, MULTI>(P, p, valid, J, salt, do_hash, E, olen);
  if (valid) P.out_len[p] = olen;
  uint32_t key[8];
  derive_key<KIND>(do_hash, E, salt, key);
  transform<U>(J, key, salt, lane, recs[wv]);
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

template <int KIND, int DIR, bool MULTI>
static int launch_one(const KParams *kp, hipStream_t s) {
  constexpr int U = SQ_U;
  constexpr uint64_t per_block = (uint64_t)kWavesPerBlock * kPktPerWave;
  const uint64_t blocks = ((uint64_t)kp->n + per_block - 1) / per_block;
  hipLaunchKernelGGL((obfs_kernel<KIND, DIR, MULTI, U>), dim3((uint32_t)blocks), dim3(kBlock), 0,
                     s, *kp);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace sq

extern "C" int sq_launch_obfs(int kind, int dir, const sq::KParams *kp, void *stream) {
  using namespace sq;
  if (kp->n == 0) return 0;
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

extern "C" int sq_launch_psk_prepare(int kind, const uint8_t *blob, const uint64_t *off,
                                     const uint32_t *len, uint32_t count, sq::PskEntry *out,
                                     void *stream) {
  if (count == 0) return 0;
  const uint32_t threads = 64;
  hipLaunchKernelGGL(sq::psk_prepare_kernel, dim3((count + threads - 1) / threads),
                     dim3(threads), 0, (hipStream_t)stream, kind, blob, off, len, count, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
