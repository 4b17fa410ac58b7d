// sq_api.hip -- the C ABI declared in include/sqobfs.h.
//
// Contexts (one per GPU), keyrings (the PSK captured by NewSalamanderConn /
// NewXPlusPacketConn, hysteria2/salamander.go:24-40, hysteria/xplus.go:19-37),
// device-resident batch launches and the host-staged path.  Every device
// entry point runs its byte transform in sq_kernels.hip and reports a missing
// or failed GPU as an error.  The one host transform is the explicit CPU
// path (sqobfs_cpu_run, host keyrings; host/sq_cpu.cpp), which the packet
// conn engine picks for small batches and when there is no working GPU.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <sys/random.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/sqobfs.h"
#include "../host/sq_cpu.h"
#include "sq_internal.h"

struct sqobfs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // compute (and sqobfs_stream)
  hipStream_t h2d = nullptr;     // sqobfs_run_host copy-in
  hipStream_t d2h = nullptr;     // sqobfs_run_host copy-out
  hipStream_t rel = nullptr;     // keyring releases (stream-ordered frees)
  // sqobfs_sync: poll the stream this long before blocking (0 = block)
  std::atomic<uint32_t> spin_us{0};
  std::mutex mu;  // guards the staging buffers of sqobfs_run_host
  uint8_t *pinned = nullptr;
  size_t pinned_cap = 0;
  uint8_t *dev = nullptr;
  size_t dev_cap = 0;
  hipEvent_t ev[64] = {};  // pipeline events of sqobfs_run_host (kEvents)
  // SQOBFS_FLAG_DEVICE_SALT: ChaCha20 key and the next launch sequence number
  uint32_t salt_key[8] = {};
  std::atomic<uint64_t> salt_seq{0};
  // obfuscation kernel unit size (packets per wavefront); 0 = built-in default
  std::atomic<uint32_t> unit_packets{0};
  // multi-key AES-GCM grouping scratch, cached per library-owned stream (the
  // context's own and the engine's; grown as needed, freed with the stream or
  // the context).  gcm_mu is held while a grouped launch is enqueued, so
  // two threads on one stream cannot interleave their group / kernel pairs.
  std::mutex gcm_mu;
  std::unordered_map<hipStream_t, std::pair<void *, uint64_t>> gcm_scratch;
};

namespace {
constexpr uint32_t kHostChunks = 8;  // sqobfs_run_host pipeline depth
// test hook (sqobfs_debug_fail_chunk): the launch of that pipeline chunk
// fails as a device error would, once
std::atomic<int> g_fail_chunk{-1};
// test hook (sqobfs_debug_gcm_ungrouped): multi-key AES-GCM launches skip the
// grouping (as when its scratch cannot be allocated)
std::atomic<int> g_gcm_ungrouped{0};
// test hook (sqobfs_debug_device_pool): keyring tables and grouping scratch
// carved from a caller's device region (deterministic placement, e.g. at
// addresses whose low 32-bit word has bit 31 set) instead of the allocator.
// [lo, hi) stays known after the pool is turned off, so frees of carved
// blocks stay no-ops.
struct DebugPool {
  std::mutex mu;
  bool on = false;
  uint8_t *lo = nullptr, *hi = nullptr;
  uint64_t used = 0;
};
DebugPool g_dpool;
bool in_dpool(const void *p) {
  std::lock_guard<std::mutex> g(g_dpool.mu);
  return p && (const uint8_t *)p >= g_dpool.lo && (const uint8_t *)p < g_dpool.hi;
}
// Stream-ordered device allocation of the library's tables and scratch.
hipError_t tab_alloc(void **p, size_t bytes, hipStream_t s) {
  {
    std::lock_guard<std::mutex> g(g_dpool.mu);
    if (g_dpool.on) {
      const uint64_t off = (g_dpool.used + 255) & ~255ull;
      if (g_dpool.lo + off + bytes > g_dpool.hi) return hipErrorOutOfMemory;
      *p = g_dpool.lo + off;
      g_dpool.used = off + bytes;
      return hipSuccess;
    }
  }
  return hipMallocAsync(p, bytes, s);
}
void tab_free_async(void *p, hipStream_t s) {
  if (p && !in_dpool(p)) (void)hipFreeAsync(p, s);
}
void tab_free(void *p) {
  if (p && !in_dpool(p)) (void)hipFree(p);
}
// live sqobfs_host_alloc blocks (sqobfs_debug_host_allocs: leak checks)
std::atomic<int64_t> g_host_allocs{0};
constexpr uint32_t kEvents = 64;
static_assert(sizeof(((sqobfs_ctx *)nullptr)->ev) / sizeof(hipEvent_t) == kEvents, "event ring");
// three events per pipeline piece (copy-in, kernel, copy-out), none reused
// within a call: at most 2 kHostChunks - 1 + 3 pieces
static_assert(3 * (2 * kHostChunks + 2) <= kEvents, "run_host pieces");
}

// The streams a keyring's table was read on.  Destroying the keyring records
// an event on each of them (after every launch enqueued there so far, the
// keyring's last ones included) and frees its device memory in stream order
// after those events (hipFreeAsync on the context's release stream): the
// call neither blocks nor waits for launches that do not use the keyring
// (another connection's, another context's).  Launches only remember their
// stream -- a per-launch event would cost the stream ~5 us between kernels
// (profiles/r03/ab/event_cost.txt) -- so those streams must still exist at
// destroy time; the library's own streams forget themselves when they are
// synchronised and destroyed (sq_keyring_forget).
struct KeyringUses {
  std::mutex mu;
  std::vector<hipStream_t> streams;
  void note(hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu);
    for (hipStream_t x : streams)
      if (x == s) return;
    streams.push_back(s);
  }
  void forget(hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu);
    streams.erase(std::remove(streams.begin(), streams.end(), s), streams.end());
  }
  // the release stream waits for every stream's work so far
  void fence(hipStream_t rel) {
    std::lock_guard<std::mutex> lk(mu);
    for (hipStream_t s : streams) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess &&
          hipEventRecord(e, s) == hipSuccess) {
        (void)hipStreamWaitEvent(rel, e, 0);
      } else {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(s);  // no event: wait for the stream instead
      }
      if (e) (void)hipEventDestroy(e);
    }
    streams.clear();
  }
};

struct sqobfs_quic_keyring {
  sqobfs_ctx *ctx = nullptr;
  mutable KeyringUses uses;
  uint32_t suite = SQOBFS_QUIC_CHACHA20_POLY1305;
  uint32_t count = 0;
  sq::QuicKeyDev *table = nullptr;  // device (ChaCha20-Poly1305)
  sq::QuicKeyDev host0;             // entry 0, passed by value
  sq::QuicGcmKeyDev *gtable = nullptr;  // device (AES-128-GCM)
  uint32_t *t0 = nullptr;               // device AES T-table (256 words)
  uint32_t grk0[44], ghrk0[44], giv0[3];
};

// sqobfs_shard_launch: one completion event per context of the step
struct sqobfs_shard_ticket {
  struct Part {
    sqobfs_ctx *ctx;
    hipEvent_t ev;
  };
  std::vector<Part> parts;
};

struct sqobfs_keyring {
  sqobfs_ctx *ctx = nullptr;      // NULL: a host keyring (no device state)
  mutable KeyringUses uses;
  int kind = 0;
  uint32_t count = 0;
  sq::PskEntry *table = nullptr;  // device
  sq::PskEntry host0;             // entry 0, passed by value to the kernels
  uint32_t hot_m = 16;            // block-0 message words any entry needs
  uint32_t hot_iv = 0;            // 1: every entry starts from the hash's initial state
  std::vector<sq::PskEntry> host; // the same state made on the host (sq_cpu.h)
};

namespace {

int hip_status(hipError_t e) {
  if (e == hipSuccess) return SQ_OK;
  if (e == hipErrorOutOfMemory) return SQ_ENOMEM;
  if (e == hipErrorInvalidDevice || e == hipErrorNoDevice) return SQ_ENODEV;
  return SQ_EDEVICE;
}

#define SQ_TRY(x)                        \
  do {                                   \
    const int st_ = hip_status((x));     \
    if (st_ != SQ_OK) return st_;        \
  } while (0)

// Makes `device` current on the calling thread for one entry point and
// restores the caller's device on return: the ABI leaves no per-thread side
// effect (a Go host's goroutines migrate between OS threads, and a host
// running several GPUs keeps its own notion of the current one).
struct DeviceScope {
  int prev = -1;
  bool changed = false;
  int status = SQ_OK;
  explicit DeviceScope(int device) {
    if (hipGetDevice(&prev) != hipSuccess) {
      (void)hipGetLastError();
      prev = -1;
    }
    if (prev != device) {
      status = hip_status(hipSetDevice(device));
      changed = status == SQ_OK;
    }
  }
  ~DeviceScope() {
    if (changed && prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope &) = delete;
  DeviceScope &operator=(const DeviceScope &) = delete;
};

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

size_t salt_len(int kind) {
  return kind == SQOBFS_SALAMANDER ? SQOBFS_SALAMANDER_SALT_LEN : SQOBFS_XPLUS_SALT_LEN;
}

}  // namespace

// Polls `s` for up to `us` microseconds: SQ_OK when it drained, 1 when it is
// still busy (the caller then blocks), or an error.  Shared with the host
// side (udp_batch.cpp, pconn.cpp).
int sq_spin_wait(void *stream, uint32_t us) {
  if (us == 0) return 1;
  hipStream_t s = (hipStream_t)stream;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return SQ_OK;
    if (q != hipErrorNotReady) return hip_status(q);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(us)) return 1;
    cpu_relax();
  }
}

// A private non-blocking stream on the context's GPU (host engines:
// pconn.cpp), and its release.
int sq_ctx_stream_create(sqobfs_ctx *ctx, void **out) {
  *out = nullptr;
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  hipStream_t s = nullptr;
  const int st = hip_status(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (st == SQ_OK) {
    *out = (void *)s;
    std::lock_guard<std::mutex> g(ctx->gcm_mu);
    ctx->gcm_scratch[s] = {nullptr, 0};  // library-owned: its scratch may be cached
  }
  return st;
}

void sq_ctx_stream_destroy(sqobfs_ctx *ctx, void *s) {
  if (!s) return;
  DeviceScope ds_(ctx->device);
  (void)hipStreamSynchronize((hipStream_t)s);
  {
    std::lock_guard<std::mutex> g(ctx->gcm_mu);
    auto it = ctx->gcm_scratch.find((hipStream_t)s);
    if (it != ctx->gcm_scratch.end()) {
      tab_free(it->second.first);  // (the stream is idle)
      ctx->gcm_scratch.erase(it);
    }
  }
  (void)hipStreamDestroy((hipStream_t)s);
}

// Wait for `s`: poll up to spin_us, then block.
// A library stream that is about to be destroyed, synchronised: the
// keyring no longer needs to fence it.
void sq_keyring_forget(const sqobfs_keyring *kr, void *s) {
  if (kr) kr->uses.forget((hipStream_t)s);
}

int sq_ctx_stream_wait(sqobfs_ctx *ctx, void *s, uint32_t spin_us) {
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  const int st = sq_spin_wait(s, spin_us);
  if (st != 1) return st;
  return hip_status(hipStreamSynchronize((hipStream_t)s));
}

namespace {
// One blocking-sync event per thread and device (engine workers are
// long-lived threads on one context); destroyed when the thread ends.
struct BlockingEvents {
  hipEvent_t ev[64] = {};
  ~BlockingEvents() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};
thread_local BlockingEvents t_block_ev;
}  // namespace

int sq_ctx_stream_wait_blocking(sqobfs_ctx *ctx, void *s, uint32_t nap_us) {
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  hipStream_t hs = (hipStream_t)s;
  // Sleep nap_us (the caller's estimate of most of the kernel's time), then
  // poll with short sleeps: the thread holds no core meanwhile.  (An event
  // with hipEventBlockingSync measured ~33 us of host CPU per ~35 us launch:
  // the runtime spins before it sleeps.)  Past ~2 ms of polls, the blocking
  // event.
  auto nap = [](uint32_t us) {
    timespec ts = {0, (long)us * 1000};
    nanosleep(&ts, nullptr);
  };
  if (nap_us) nap(nap_us);
  for (int i = 0; i < 400; i++) {
    const hipError_t q = hipStreamQuery(hs);
    if (q == hipSuccess) return SQ_OK;
    if (q != hipErrorNotReady) return hip_status(q);
    nap(5);
  }
  if (ctx->device < 0 || ctx->device >= 64) return hip_status(hipStreamSynchronize(hs));
  hipEvent_t &e = t_block_ev.ev[ctx->device];
  if (!e && hipEventCreateWithFlags(&e, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess) {
    e = nullptr;
    return hip_status(hipStreamSynchronize(hs));
  }
  const int st = hip_status(hipEventRecord(e, hs));
  if (st != SQ_OK) return st;
  return hip_status(hipEventSynchronize(e));
}

int sq_host_alloc_mapped(sqobfs_ctx *ctx, size_t bytes, void **out) {
  const int st = sqobfs_host_alloc(ctx, bytes, out);
  if (st != SQ_OK) return st;
  void *dev = nullptr;  // the GPU's view of the block: the same address on ROCm
  DeviceScope ds_(ctx->device);
  if (hipHostGetDevicePointer(&dev, *out, 0) != hipSuccess || dev != *out) {
    (void)hipGetLastError();
    sqobfs_host_free(ctx, *out);
    *out = nullptr;
    return SQ_EDEVICE;
  }
  return SQ_OK;
}

const sq::PskEntry *sq_keyring_host(const sqobfs_keyring *kr, uint32_t *count) {
  *count = kr->count;
  return kr->host.data();
}

sqobfs_ctx *sq_keyring_ctx(const sqobfs_keyring *kr) { return kr->ctx; }

void sq_keyring_hot(const sqobfs_keyring *kr, uint32_t *hot_m, uint32_t *hot_iv) {
  *hot_m = kr->hot_m;
  *hot_iv = kr->hot_iv;
}

int sq_keyring_from_entries(sqobfs_ctx *ctx, int kind, const sq::PskEntry *e, uint32_t count,
                            uint32_t hot_m, uint32_t hot_iv, void *stream,
                            sqobfs_keyring **out) {
  *out = nullptr;
  if (!ctx || !e || count == 0) return SQ_EINVAL;
  sqobfs_keyring *kr = new (std::nothrow) sqobfs_keyring();
  if (!kr) return SQ_ENOMEM;
  kr->ctx = ctx;
  kr->kind = kind;
  kr->count = count;
  kr->hot_m = hot_m;
  kr->hot_iv = hot_iv;
  try {
    kr->host.assign(e, e + count);
  } catch (...) {
    delete kr;
    return SQ_ENOMEM;
  }
  kr->host0 = kr->host[0];
  DeviceScope ds_(ctx->device);
  int st = ds_.status;
  // the table is made on the caller's stream (the engine's launch stream),
  // so the wait does not queue behind the context stream's own work
  hipStream_t hs = stream ? (hipStream_t)stream : ctx->stream;
  // (the host entries are the device layout: sqobfs_debug_keyring_check)
  if (st == SQ_OK)
    st = hip_status(tab_alloc((void **)&kr->table, sizeof(sq::PskEntry) * count, hs));
  if (st == SQ_OK)
    st = hip_status(hipMemcpyAsync(kr->table, kr->host.data(), sizeof(sq::PskEntry) * count,
                                   hipMemcpyHostToDevice, hs));
  if (st == SQ_OK) st = hip_status(hipStreamSynchronize(hs));
  if (st != SQ_OK) {
    if (kr->table) {
      (void)hipStreamSynchronize(hs);
      tab_free_async(kr->table, hs);
      (void)hipStreamSynchronize(hs);
    }
    delete kr;
    return st;
  }
  *out = kr;
  return SQ_OK;
}

void sq_salt_take(sqobfs_ctx *ctx, uint32_t key[8], uint64_t *seq) {
  if (!ctx) {
    sq_host_salt_take(key, seq);
    return;
  }
  memcpy(key, ctx->salt_key, sizeof ctx->salt_key);
  *seq = ctx->salt_seq.fetch_add(1);
}

// Default unit (packets per wavefront) of a device batch whose lengths the
// library cannot see: the built-in default, but small batches are spread so
// that the launch has at least kMinUnits wavefronts (a 256-datagram socket
// batch is 256 one-packet waves over the CUs, not 10 waves of 26 packets).
uint32_t sq_unit_packets_default(uint32_t n) {
  const uint32_t spread = (n + sq::kMinUnits - 1) / sq::kMinUnits;
  return std::max<uint32_t>(1u, std::min<uint32_t>(sq::kDefaultUnitPackets, spread));
}

namespace {

// NULL is the HIP null stream (HIP convention; torch's default stream), so a
// caller's events and copies on that stream order with our kernels.
hipStream_t pick_stream(sqobfs_ctx *ctx, void *stream) {
  (void)ctx;
  return (hipStream_t)stream;
}

int check_batch_shape(const sqobfs_batch *b, int dir) {
  if (!b) return SQ_EINVAL;
  if (b->flags & ~(uint32_t)(SQOBFS_FLAG_OUT_UNINIT | SQOBFS_FLAG_DEVICE_SALT |
                             SQOBFS_FLAG_OUT_BLOCKS | SQOBFS_FLAG_OUT_LINES))
    return SQ_EINVAL;
  const bool dev_salt = b->flags & SQOBFS_FLAG_DEVICE_SALT;
  if (dev_salt && dir != SQOBFS_OBFUSCATE) return SQ_EINVAL;
  if (b->n == 0) return SQ_OK;
  if (!b->in || !b->in_off || !b->in_len || !b->out || !b->out_off || !b->out_len)
    return SQ_EINVAL;
  if (dir == SQOBFS_OBFUSCATE && !dev_salt) {
    if (!b->salt || ((uintptr_t)b->salt & 3)) return SQ_EINVAL;
  }
  if (dev_salt && ((uintptr_t)b->salt_out & 3)) return SQ_EINVAL;
  return SQ_OK;
}

// "sqob" || le64(seq): the ChaCha20 nonce of one device-salt launch
constexpr uint32_t kSaltDomain = 0x626f7173u;  // bytes 's' 'q' 'o' 'b'

sq::KParams make_params(sqobfs_ctx *ctx, const sqobfs_keyring *kr, const sqobfs_batch *b) {
  sq::KParams kp;
  memset(&kp, 0, sizeof kp);
  kp.in = b->in;
  kp.in_off = b->in_off;
  kp.in_len = b->in_len;
  kp.out = b->out;
  kp.out_off = b->out_off;
  kp.out_len = b->out_len;
  kp.salt = b->salt;
  kp.psk_id = b->psk_id;
  kp.in_cap = b->in_cap;
  kp.psk_table = kr->table;
  kp.n = b->n;
  kp.n_psk = kr->count;
  kp.psk0 = kr->host0;
  kp.psk_hot_m = kr->hot_m;
  kp.psk_hot_iv = kr->hot_iv;
  kp.ppw = ctx->unit_packets.load(std::memory_order_relaxed);
  kp.out_lines = (b->flags & SQOBFS_FLAG_OUT_LINES) ? 1u : 0u;
  kp.out_blocks = (b->flags & SQOBFS_FLAG_OUT_BLOCKS) || kp.out_lines ? 1u : 0u;
  if (b->flags & SQOBFS_FLAG_DEVICE_SALT) {
    const uint64_t seq = ctx->salt_seq.fetch_add(1);
    kp.device_salt = 1;
    kp.salt_out = b->salt_out;
    memcpy(kp.salt_key, ctx->salt_key, sizeof kp.salt_key);
    kp.salt_nonce[0] = kSaltDomain;
    kp.salt_nonce[1] = (uint32_t)seq;
    kp.salt_nonce[2] = (uint32_t)(seq >> 32);
  }
  return kp;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Range {
  size_t lo, hi;     // byte range touched in the caller's buffer
  uint32_t p0, p1;   // packets of the chunk
};

// What run_host's slot packing (slot_pack) needs to know of a batch,
// gathered in packet_spans' pass: whether packet i sits at in_off[0] + i si
// and out_off[0] + i so, and the widest input and output.
struct SlotScan {
  bool strided = false;   // (set by the caller when the layout may be strided)
  size_t si = 0, so = 0;  // candidate strides
  size_t wi = 0, wo = 0;  // widest input (with XPlus in_cap) and output
};

// The input and output byte ranges packets [p0, p1) of hb touch (empty
// ranges are {0, 0}), per the output-length rules of include/sqobfs.h; with
// a scan, its stride check and widths over the same packets (one pass: at
// 256K packets each pass over the descriptors costs ~0.1 ms before the
// pipeline's first copy).
void packet_spans(const sqobfs_batch *hb, int kind, int dir, uint32_t p0, uint32_t p1,
                  Range &ri, Range &ro, SlotScan *scan = nullptr) {
  const size_t S = salt_len(kind);
  ri = Range{SIZE_MAX, 0, p0, p1};
  ro = Range{SIZE_MAX, 0, p0, p1};
  bool strided = scan && scan->strided;
  size_t wi = 0, wo = 0;
  const uint64_t i0 = scan ? hb->in_off[0] : 0, o0 = scan ? hb->out_off[0] : 0;
  for (uint32_t i = p0; i < p1; i++) {
    const size_t len = hb->in_len[i];
    size_t cap = len;
    if (kind == SQOBFS_XPLUS && dir == SQOBFS_DEOBFUSCATE && hb->in_cap)
      cap = std::max<size_t>(len, hb->in_cap[i]);
    size_t osz;
    if (dir == SQOBFS_OBFUSCATE) osz = S + len;
    else if (kind == SQOBFS_SALAMANDER) osz = len <= S ? len : len - S;
    else osz = len < S ? 0 : cap - S;
    if (cap) {
      ri.lo = std::min<size_t>(ri.lo, hb->in_off[i]);
      ri.hi = std::max<size_t>(ri.hi, hb->in_off[i] + cap);
    }
    if (osz) {
      ro.lo = std::min<size_t>(ro.lo, hb->out_off[i]);
      ro.hi = std::max<size_t>(ro.hi, hb->out_off[i] + osz);
    }
    if (strided) {
      strided = hb->in_off[i] == i0 + scan->si * i && hb->out_off[i] == o0 + scan->so * i;
      wi = std::max(wi, cap);
      wo = std::max(wo, osz);
    }
  }
  if (ri.lo > ri.hi) ri.lo = ri.hi = 0;
  if (ro.lo > ro.hi) ro.lo = ro.hi = 0;
  if (scan) {
    scan->strided = strided;
    scan->wi = std::max(scan->wi, wi);
    scan->wo = std::max(scan->wo, wo);
  }
}

// byte range ra of buffer a and rb of buffer b overlap
bool spans_meet(const uint8_t *a, const Range &ra, const uint8_t *b, const Range &rb) {
  return ra.hi > ra.lo && rb.hi > rb.lo && a + ra.lo < b + rb.hi && b + rb.lo < a + ra.hi;
}

// Some part's output range overlaps another part's input or output range:
// the parts cannot run concurrently, each copying its whole span.
bool parts_clash(const sqobfs_batch *hb, const std::vector<Range> &rin,
                 const std::vector<Range> &rout) {
  const size_t k = rin.size();
  for (size_t x = 0; x < k; x++)
    for (size_t y = 0; y < k; y++)
      if (x != y && (spans_meet(hb->out, rout[x], hb->out, rout[y]) ||
                     spans_meet(hb->out, rout[x], hb->in, rin[y])))
        return true;
  return false;
}

bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory reports an error: clear it
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// memcpy of large pageable ranges on several host threads
void par_memcpy(void *dst, const void *src, size_t n) {
  constexpr size_t kPer = 8u << 20;
  const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  const unsigned nt = (unsigned)std::min<size_t>(hw, (n + kPer - 1) / kPer);
  if (nt <= 1) {
    memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++) {
    const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
    auto part = [=] { memcpy((uint8_t *)dst + lo, (const uint8_t *)src + lo, hi - lo); };
    try {
      th.emplace_back(part);
    } catch (...) {  // (no thread: that part on this one)
      part();
    }
  }
  for (auto &x : th) x.join();
}

// Fixed-stride slots (the Go Slots, socket batches): packet i's input at
// in_off[0] + i si and its output at out_off[0] + i so.  sqobfs_run_host then
// stages only the first wi / wo bytes of every slot, rows packed at pitches
// pi / po, with 2-D copies (hipMemcpy2DAsync moves rows of ~1.4 KB at the
// PCIe rate of a contiguous copy): a 2,048-byte slot
// holding a 1,358-byte datagram costs 1,358 bytes of PCIe each way, not
// 2,048.  Used when both buffers are page-locked, the strides hold the rows,
// the input and output spans are apart, output rows keep their phase modulo
// 16 / 128 (for SQOBFS_FLAG_OUT_BLOCKS / _LINES) and the packing saves at
// least an eighth of a span.
struct SlotPack {
  bool on = false;
  size_t si = 0, so = 0;    // caller's strides
  size_t wi = 0, wo = 0;    // bytes staged per slot (the widest input / output)
  size_t phi = 0, pho = 0;  // staged row offset of the input / output (address phase)
  size_t pi = 0, po = 0;    // staged pitches
};

// A scan candidate: a batch run_host may pack (page-locked buffers, at
// least 64 packets, host salts, increasing first offsets).
SlotScan slot_scan_start(const sqobfs_batch *hb, bool pinned) {
  SlotScan sc;
  if (!pinned || hb->n < 64 || (hb->flags & SQOBFS_FLAG_DEVICE_SALT)) return sc;
  if (hb->in_off[1] <= hb->in_off[0] || hb->out_off[1] <= hb->out_off[0]) return sc;
  sc.strided = true;
  sc.si = hb->in_off[1] - hb->in_off[0];
  sc.so = hb->out_off[1] - hb->out_off[0];
  return sc;
}

SlotPack slot_pack(const sqobfs_batch *hb, const SlotScan &sc, size_t in_lo, size_t in_hi,
                   size_t out_lo, size_t out_hi) {
  SlotPack sp;
  if (!sc.strided) return sp;
  sp.si = sc.si;
  sp.so = sc.so;
  sp.wi = sc.wi;
  sp.wo = sc.wo;
  const bool lines = hb->flags & SQOBFS_FLAG_OUT_LINES;
  const bool blocks = lines || (hb->flags & SQOBFS_FLAG_OUT_BLOCKS);
  const size_t oa = lines ? 128 : 16;
  if (sp.wi > sp.si || sp.wo > sp.so || (blocks && sp.so % oa)) return sp;
  // the input and output spans must be apart (no in-place slots)
  if (in_hi > in_lo && out_hi > out_lo && hb->in + in_lo < hb->out + out_hi &&
      hb->out + out_lo < hb->in + in_hi)
    return sp;
  sp.phi = ((uintptr_t)hb->in + hb->in_off[0]) & 15;
  sp.pho = ((uintptr_t)hb->out + hb->out_off[0]) & (oa - 1);
  sp.pi = align_up(sp.phi + sp.wi, 16);
  sp.po = align_up(sp.pho + sp.wo, oa);
  sp.on = 8 * (sp.pi + sp.po) <= 7 * (sp.si + sp.so);
  return sp;
}

}  // namespace

extern "C" {

int sqobfs_abi_version(void) { return SQOBFS_ABI_VERSION; }

const char *sqobfs_strerror(int status) {
  switch (status) {
    case SQ_OK: return "ok";
    case SQ_EINVAL: return "invalid argument";
    case SQ_ENOMEM: return "out of memory";
    case SQ_EDEVICE: return "HIP runtime or kernel launch error";
    case SQ_ENODEV: return "no such GPU";
    case SQ_EPSK: return "psk_id out of range";
    case SQ_ETIMEDOUT: return "deadline exceeded";
    case SQ_ECLOSED: return "closed";
    case SQ_EIO: return "the wrapped connection failed";
  }
  return "unknown status";
}

int sqobfs_device_count(int *count) {
  if (!count) return SQ_EINVAL;
  *count = 0;
  const hipError_t e = hipGetDeviceCount(count);
  if (e == hipErrorNoDevice) {
    *count = 0;
    return SQ_ENODEV;
  }
  return hip_status(e);
}

int sqobfs_open(int device, sqobfs_ctx **out) {
  if (!out) return SQ_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return SQ_ENODEV;
  DeviceScope ds_(device);
  if (ds_.status != SQ_OK) return ds_.status;
  sqobfs_ctx *c = new (std::nothrow) sqobfs_ctx();
  if (!c) return SQ_ENOMEM;
  c->device = device;
  {
    uint8_t k[32];
    size_t got = 0;
    while (got < sizeof k) {
      const ssize_t r = getrandom(k + got, sizeof k - got, 0);
      if (r < 0) {
        delete c;
        return SQ_EDEVICE;
      }
      got += (size_t)r;
    }
    memcpy(c->salt_key, k, sizeof k);
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->rel, hipStreamNonBlocking);
  if (e != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->h2d) (void)hipStreamDestroy(c->h2d);
    if (c->d2h) (void)hipStreamDestroy(c->d2h);
    delete c;
    return hip_status(e);
  }
  *out = c;
  return SQ_OK;
}

void sqobfs_close(sqobfs_ctx *ctx) {
  if (!ctx) return;
  sq_engine_ctx_closed(ctx);  // its packet conn engine's threads and blocks
  DeviceScope ds_(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->rel);  // keyrings released before the context
  for (auto &kv : ctx->gcm_scratch)
    tab_free(kv.second.first);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->dev) (void)hipFree(ctx->dev);
  (void)hipStreamDestroy(ctx->stream);
  (void)hipStreamDestroy(ctx->h2d);
  (void)hipStreamDestroy(ctx->d2h);
  (void)hipStreamDestroy(ctx->rel);
  for (auto &e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  delete ctx;
}

int sqobfs_salt_key(sqobfs_ctx *ctx, const uint8_t key[32], uint64_t next_seq) {
  if (!ctx || !key) return SQ_EINVAL;
  memcpy(ctx->salt_key, key, sizeof ctx->salt_key);  // little-endian words
  ctx->salt_seq.store(next_seq);
  return SQ_OK;
}

uint64_t sqobfs_salt_seq(const sqobfs_ctx *ctx) { return ctx ? ctx->salt_seq.load() : 0; }

int sqobfs_set_unit_packets(sqobfs_ctx *ctx, uint32_t packets) {
  if (!ctx || packets > sq::kMaxUnitPackets) return SQ_EINVAL;
  ctx->unit_packets.store(packets, std::memory_order_relaxed);
  return SQ_OK;
}

uint32_t sqobfs_unit_packets_for(uint64_t bytes, uint32_t n, int multi_psk) {
  return sqobfs_unit_packets_for_kind(SQOBFS_SALAMANDER, bytes, n, multi_psk);
}

uint32_t sqobfs_unit_packets_for_kind(int kind, uint64_t bytes, uint32_t n, int multi_psk) {
  if (n == 0) return sq::kDefaultUnitPackets;
  const uint64_t target = multi_psk ? sq::kUnitBytesMultiPsk
                          : kind == SQOBFS_XPLUS ? sq::kUnitBytesXPlus
                                                 : sq::kUnitBytes;
  const uint64_t u = bytes ? target * n / bytes : sq::kMaxUnitPackets;  // floor(target / mean)
  // and at least kMinUnits wavefronts for small batches
  const uint64_t spread = ((uint64_t)n + sq::kMinUnits - 1) / sq::kMinUnits;
  return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(std::min(u, spread), 1),
                                      sq::kMaxUnitPackets);
}

uint32_t sqobfs_unit_packets(const sqobfs_ctx *ctx) {
  // (device batches below kMinUnits * default packets are spread further:
  // sq_unit_packets_default)
  const uint32_t v = ctx ? ctx->unit_packets.load(std::memory_order_relaxed) : 0u;
  return v ? v : sq::kDefaultUnitPackets;
}

void *sqobfs_stream(sqobfs_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int sqobfs_sync(sqobfs_ctx *ctx, void *stream) {
  if (!ctx) return SQ_EINVAL;
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  hipStream_t s = pick_stream(ctx, stream);
  // Opt-in (sqobfs_set_sync_spin): poll before blocking.  hipStreamSynchronize's
  // blocking wake-up left the GPU idle ~80 us between synchronous
  // 1M-packet batches (bench --inproc 1: 0.56 ms per step against 0.48 ms for
  // queued launches), but a poll holds a CPU for its whole length, so only a
  // caller with a thread to spare turns it on.
  const uint32_t spin = ctx->spin_us.load(std::memory_order_relaxed);
  const int st = sq_spin_wait(s, spin);
  if (st != 1) return st;
  return hip_status(hipStreamSynchronize(s));
}

int sqobfs_set_sync_spin(sqobfs_ctx *ctx, uint32_t us) {
  if (!ctx) return SQ_EINVAL;
  ctx->spin_us.store(us, std::memory_order_relaxed);
  return SQ_OK;
}

namespace {

// What the multi-PSK kernels gather per packet from an entry (sq_kernels.hip
// load_hot), from the PSK lengths alone (the entry layout of
// psk_prepare_kernel): `m` = the message words of the first compressed
// block any entry has non-zero -- BLAKE2b: PSK tail || salt, zero padded,
// all 16 when the salt spills into a second block; SHA-256: all 8 (its
// length field ends the block) -- and `iv` = 1 when no PSK has a PSK-only
// leading block, so every chaining value is the hash's initial state and is
// not loaded.  Keyrings of short PSKs (the common 8-64 bytes) then gather
// ~96 instead of ~216 bytes per packet.
void keyring_hot_words(int kind, uint32_t count, const uint32_t *len, uint32_t &m,
                       uint32_t &iv) {
  m = 0;
  iv = 1;
  for (uint32_t k = 0; k < count; k++) {
    const uint32_t L = len[k];
    if (kind == SQOBFS_SALAMANDER) {
      const uint32_t tot = L % 128 + SQOBFS_SALAMANDER_SALT_LEN;
      m = std::max<uint32_t>(m, tot > 128 ? 16u : (tot + 7) / 8);
      if (L >= 128) iv = 0;
    } else {
      m = 8;
      if (L >= 64) iv = 0;
    }
  }
}

}  // namespace

int sqobfs_keyring_create(sqobfs_ctx *ctx, int kind, uint32_t count, const uint8_t *blob,
                          const uint64_t *off, const uint32_t *len, sqobfs_keyring **out) {
  if (!out || count == 0 || !off || !len) return SQ_EINVAL;
  if (kind != SQOBFS_SALAMANDER && kind != SQOBFS_XPLUS) return SQ_EINVAL;
  *out = nullptr;
  size_t blob_bytes = 0;
  for (uint32_t k = 0; k < count; k++) blob_bytes = std::max<size_t>(blob_bytes, off[k] + len[k]);
  if (blob_bytes && !blob) return SQ_EINVAL;
  sqobfs_keyring *kr = new (std::nothrow) sqobfs_keyring();
  if (!kr) return SQ_ENOMEM;
  kr->ctx = ctx;
  kr->kind = kind;
  kr->count = count;
  try {
    kr->host.resize(count);
  } catch (...) {
    delete kr;
    return SQ_ENOMEM;
  }
  for (uint32_t k = 0; k < count; k++)
    sq::cpu::psk_prepare(kind, blob ? blob + off[k] : nullptr, len[k], &kr->host[k]);
  if (!ctx) {  // a host keyring
    kr->host0 = kr->host[0];
    *out = kr;
    return SQ_OK;
  }
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) {
    delete kr;
    return ds_.status;
  }
  keyring_hot_words(kind, count, len, kr->hot_m, kr->hot_iv);
  uint8_t *d_blob = nullptr;
  uint64_t *d_off = nullptr;
  uint32_t *d_len = nullptr;
  hipError_t e = tab_alloc((void **)&kr->table, sizeof(sq::PskEntry) * count, ctx->stream);
  if (e == hipSuccess) e = hipMalloc(&d_blob, blob_bytes ? blob_bytes : 1);
  if (e == hipSuccess) e = hipMalloc(&d_off, sizeof(uint64_t) * count);
  if (e == hipSuccess) e = hipMalloc(&d_len, sizeof(uint32_t) * count);
  if (e == hipSuccess && blob_bytes)
    e = hipMemcpyAsync(d_blob, blob, blob_bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_off, off, sizeof(uint64_t) * count, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_len, len, sizeof(uint32_t) * count, hipMemcpyHostToDevice, ctx->stream);
  int st = hip_status(e);
  if (st == SQ_OK)
    st = sq_launch_psk_prepare(kind, d_blob, d_off, d_len, count, kr->table, ctx->stream);
  if (st == SQ_OK)
    st = hip_status(hipMemcpyAsync(&kr->host0, kr->table, sizeof(sq::PskEntry),
                                   hipMemcpyDeviceToHost, ctx->stream));
  if (st == SQ_OK) st = hip_status(hipStreamSynchronize(ctx->stream));
  if (d_blob) (void)hipFree(d_blob);
  if (d_off) (void)hipFree(d_off);
  if (d_len) (void)hipFree(d_len);
  if (st != SQ_OK) {
    (void)hipStreamSynchronize(ctx->stream);
    tab_free_async(kr->table, ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
    delete kr;
    return st;
  }
  *out = kr;
  return SQ_OK;
}

void sqobfs_keyring_destroy(sqobfs_keyring *kr) {
  if (!kr) return;
  if (!kr->ctx) {
    delete kr;
    return;
  }
  DeviceScope ds_(kr->ctx->device);
  // launches that used the table may still run: free it after them, in
  // stream order, without blocking (and without a device-wide sync)
  kr->uses.fence(kr->ctx->rel);
  tab_free_async(kr->table, kr->ctx->rel);
  delete kr;
}

int sqobfs_keyring_kind(const sqobfs_keyring *kr) { return kr ? kr->kind : SQ_EINVAL; }
uint32_t sqobfs_keyring_count(const sqobfs_keyring *kr) { return kr ? kr->count : 0; }

int sqobfs_keyring_release_stream(const sqobfs_keyring *kr, void *stream) {
  if (!kr) return SQ_EINVAL;
  if (!kr->ctx || !stream) return SQ_OK;  // host keyring / the null stream (never destroyed)
  DeviceScope ds_(kr->ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  const int st = hip_status(hipStreamSynchronize((hipStream_t)stream));
  kr->uses.forget((hipStream_t)stream);
  return st;
}

int sqobfs_debug_keyring_check(const sqobfs_keyring *kr) {
  if (!kr || !kr->ctx) return SQ_EINVAL;
  DeviceScope ds_(kr->ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  std::vector<sq::PskEntry> dev(kr->count);
  hipStream_t s = kr->ctx->stream;
  int st = hip_status(hipMemcpyAsync(dev.data(), kr->table, sizeof(sq::PskEntry) * kr->count,
                                     hipMemcpyDeviceToHost, s));
  if (st == SQ_OK) st = hip_status(hipStreamSynchronize(s));
  if (st != SQ_OK) return st;
  int bad = 0;
  for (uint32_t k = 0; k < kr->count; k++)
    if (memcmp(&dev[k], &kr->host[k], sizeof(sq::PskEntry)) != 0) bad++;
  return bad;
}

int sqobfs_cpu_run(const sqobfs_keyring *kr, int dir, const sqobfs_batch *b) {
  if (!kr || (dir != SQOBFS_OBFUSCATE && dir != SQOBFS_DEOBFUSCATE)) return SQ_EINVAL;
  int st = check_batch_shape(b, dir);
  if (st != SQ_OK || b->n == 0) return st;
  std::vector<uint8_t> salts;
  if (b->flags & SQOBFS_FLAG_DEVICE_SALT) {
    const size_t S = salt_len(kr->kind);
    uint32_t key[8];
    uint64_t seq;
    sq_salt_take(kr->ctx, key, &seq);
    try {
      salts.resize((size_t)b->n * S);
    } catch (...) {
      return SQ_ENOMEM;
    }
    sq::cpu::salt_stream(key, seq, salts.data(), salts.size());
    if (b->salt_out) memcpy(b->salt_out, salts.data(), salts.size());
  }
  return sq::cpu::run_batch(kr->kind, dir, kr->host.data(), kr->count, b,
                            salts.empty() ? nullptr : salts.data());
}

int sqobfs_launch(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir, const sqobfs_batch *b,
                  void *stream) {
  // a launch that returns before its kernel still spends the timing hook
  const auto unarmed = [](int r) {
    sq_time_next_launch(nullptr, nullptr);
    return r;
  };
  if (!ctx || !kr || kr->ctx != ctx) return unarmed(SQ_EINVAL);  // (host keyrings: sqobfs_cpu_run)
  if (dir != SQOBFS_OBFUSCATE && dir != SQOBFS_DEOBFUSCATE) return unarmed(SQ_EINVAL);
  const int st = check_batch_shape(b, dir);
  if (st != SQ_OK || b->n == 0) return unarmed(st);
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return unarmed(ds_.status);
  sq::KParams kp = make_params(ctx, kr, b);
  if (kp.ppw == 0) kp.ppw = sq_unit_packets_default(b->n);
  hipStream_t s = pick_stream(ctx, stream);
  const int st2 = sq_launch_obfs(kr->kind, dir, &kp, s);
  if (st2 == SQ_OK) kr->uses.note(s);
  return st2;
}

int sqobfs_salamander_obfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr,
                                const sqobfs_batch *b, void *stream) {
  if (!kr || kr->kind != SQOBFS_SALAMANDER) return SQ_EINVAL;
  return sqobfs_launch(ctx, kr, SQOBFS_OBFUSCATE, b, stream);
}
int sqobfs_salamander_deobfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr,
                                  const sqobfs_batch *b, void *stream) {
  if (!kr || kr->kind != SQOBFS_SALAMANDER) return SQ_EINVAL;
  return sqobfs_launch(ctx, kr, SQOBFS_DEOBFUSCATE, b, stream);
}
int sqobfs_xplus_obfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr, const sqobfs_batch *b,
                           void *stream) {
  if (!kr || kr->kind != SQOBFS_XPLUS) return SQ_EINVAL;
  return sqobfs_launch(ctx, kr, SQOBFS_OBFUSCATE, b, stream);
}
int sqobfs_xplus_deobfuscate(sqobfs_ctx *ctx, const sqobfs_keyring *kr, const sqobfs_batch *b,
                             void *stream) {
  if (!kr || kr->kind != SQOBFS_XPLUS) return SQ_EINVAL;
  return sqobfs_launch(ctx, kr, SQOBFS_DEOBFUSCATE, b, stream);
}

// ---------------------------------------------------------------- QUIC

// ---- AES-128-GCM key preparation (host, once per keyring): FIPS-197 key
// expansion, H = AES_K(0^128), and the 4-bit GHASH tables of H^1..H^128
// that sq_quic_gcm.hip reads.  Connection setup work, not per packet.
extern "C++" {
namespace {
uint8_t gf8_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  for (; b; b >>= 1) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
  }
  return r;
}

struct AesTables {
  uint8_t sbox[256];
  uint32_t t0[256];  // little-endian column (2s, s, s, 3s)
  AesTables() {
    for (int x = 0; x < 256; x++) {
      uint8_t inv = 0, base = (uint8_t)x, acc = 1;
      if (x) {
        for (int e = 254; e; e >>= 1) {
          if (e & 1) acc = gf8_mul(acc, base);
          base = gf8_mul(base, base);
        }
        inv = acc;
      }
      uint8_t y = 0x63;
      for (int k = 0; k < 5; k++) y ^= (uint8_t)((inv << k) | (inv >> ((8 - k) & 7)));
      sbox[x] = y;
      const uint32_t s1 = y, s2 = gf8_mul(y, 2), s3 = s2 ^ s1;
      t0[x] = s2 | (s1 << 8) | (s1 << 16) | (s3 << 24);
    }
  }
};
const AesTables &aes_tables() {
  static const AesTables t;
  return t;
}

uint32_t le32(const uint8_t *b) {
  return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

void aes128_expand(const uint8_t key[16], uint32_t rk[44]) {
  const uint8_t *sb = aes_tables().sbox;
  uint8_t w[176];
  memcpy(w, key, 16);
  uint8_t rcon = 1;
  for (int i = 4; i < 44; i++) {
    uint8_t t[4] = {w[4 * i - 4], w[4 * i - 3], w[4 * i - 2], w[4 * i - 1]};
    if (i % 4 == 0) {
      const uint8_t t0 = t[0];
      t[0] = (uint8_t)(sb[t[1]] ^ rcon);
      t[1] = sb[t[2]];
      t[2] = sb[t[3]];
      t[3] = sb[t0];
      rcon = gf8_mul(rcon, 2);
    }
    for (int k = 0; k < 4; k++) w[4 * i + k] = w[4 * i - 16 + k] ^ t[k];
  }
  for (int i = 0; i < 44; i++) rk[i] = le32(w + 4 * i);
}

// one block, same column-word form as the device
void aes128_block(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
  const uint32_t *T = aes_tables().t0;
  auto rot = [](uint32_t x, int n) { return (x << n) | (x >> (32 - n)); };
  uint32_t s[4];
  for (int c = 0; c < 4; c++) s[c] = le32(in + 4 * c) ^ rk[c];
  for (int r = 1; r <= 10; r++) {
    uint32_t t[4];
    for (int c = 0; c < 4; c++) {
      const uint32_t a0 = T[s[c] & 0xFF], a1 = T[(s[(c + 1) & 3] >> 8) & 0xFF];
      const uint32_t a2 = T[(s[(c + 2) & 3] >> 16) & 0xFF], a3 = T[s[(c + 3) & 3] >> 24];
      t[c] = r < 10 ? a0 ^ rot(a1, 8) ^ rot(a2, 16) ^ rot(a3, 24)
                    : ((a0 >> 8) & 0xFF) | (a1 & 0xFF00) | ((a2 << 8) & 0xFF0000) |
                          ((a3 << 16) & 0xFF000000u);
      t[c] ^= rk[4 * r + c];
    }
    memcpy(s, t, sizeof s);
  }
  for (int c = 0; c < 4; c++)
    for (int k = 0; k < 4; k++) out[4 * c + k] = (uint8_t)(s[c] >> (8 * k));
}

// GF(2^128) element as a big-endian 128-bit integer (hi, lo); bit 127 of the
// integer is the coefficient of x^0 (SP 800-38D bit order)
struct G128 {
  uint64_t hi, lo;
};
G128 g_load(const uint8_t b[16]) {
  G128 g{0, 0};
  for (int k = 0; k < 8; k++) g.hi = (g.hi << 8) | b[k];
  for (int k = 8; k < 16; k++) g.lo = (g.lo << 8) | b[k];
  return g;
}
G128 g_mulx(G128 v) {  // v * x
  const bool lsb = v.lo & 1;
  v.lo = (v.lo >> 1) | (v.hi << 63);
  v.hi >>= 1;
  if (lsb) v.hi ^= 0xE100000000000000ull;
  return v;
}
G128 g_mul(G128 x, G128 y) {  // SP 800-38D Algorithm 1
  G128 z{0, 0}, v = y;
  for (int i = 0; i < 128; i++) {
    const bool bit = i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
    if (bit) {
      z.hi ^= v.hi;
      z.lo ^= v.lo;
    }
    v = g_mulx(v);
  }
  return z;
}

void gcm_key(const sqobfs_quic_key &k, sq::QuicGcmKeyDev &d) {
  memset(&d, 0, sizeof d);
  aes128_expand(k.key, d.rk);
  aes128_expand(k.hp, d.hrk);
  for (int i = 0; i < 3; i++) d.iv[i] = le32(k.iv + 4 * i);
  const uint8_t zero[16] = {0};
  uint8_t hb[16];
  aes128_block(d.rk, zero, hb);
  // rounds 1-9 stored rotated by 16 bits: the kernel folds the round key
  // under its rotl16 (sq_quic_gcm.hip aes_encrypt_n)
  for (int i = 4; i < 40; i++) {
    d.rk[i] = (d.rk[i] >> 16) | (d.rk[i] << 16);
    d.hrk[i] = (d.hrk[i] >> 16) | (d.hrk[i] << 16);
  }
  const G128 h = g_load(hb);
  const G128 h4 = g_mul(g_mul(h, h), g_mul(h, h));
  // position tables of H: nibble j enters Shoup's Horner loop j-th and is
  // multiplied by x^4 (31 - j) more times
  for (int n = 0; n < 16; n++) {
    G128 v{0, 0};
    for (int b = 0; b < 4; b++) {  // n H: bit 8 >> b of n is x^b
      if (!(n & (8 >> b))) continue;
      G128 t = h;
      for (int i = 0; i < b; i++) t = g_mulx(t);
      v.hi ^= t.hi;
      v.lo ^= t.lo;
    }
    for (int j = 31; j >= 0; j--) {
      d.hpos[j][n][0] = (uint32_t)(v.hi >> 32);
      d.hpos[j][n][1] = (uint32_t)v.hi;
      d.hpos[j][n][2] = (uint32_t)(v.lo >> 32);
      d.hpos[j][n][3] = (uint32_t)v.lo;
      for (int k = 0; k < 4; k++) v = g_mulx(v);
    }
  }
  G128 p = h4;
  for (uint32_t pw = 0; pw < sq::kGcmPow4; pw++) {  // table pw: H^(4 (pw + 1))
    if (pw) p = g_mul(p, h4);
    G128 e[16] = {};
    e[8] = p;  // Shoup: entry 8 = H^k, 4 = H^k x, 2 = H^k x^2, 1 = H^k x^3
    e[4] = g_mulx(e[8]);
    e[2] = g_mulx(e[4]);
    e[1] = g_mulx(e[2]);
    for (int n = 1; n < 16; n++) {
      if (n == 1 || n == 2 || n == 4 || n == 8) continue;
      G128 v{0, 0};
      for (int b = 1; b < 16; b <<= 1)
        if (n & b) {
          v.hi ^= e[b].hi;
          v.lo ^= e[b].lo;
        }
      e[n] = v;
    }
    for (int n = 0; n < 16; n++) {  // slot n ^ (pw & 15): see gmul in sq_quic_gcm.hip
      const int sl = n ^ (int)(pw & 15);
      d.htab[pw][sl][0] = (uint32_t)(e[n].hi >> 32);
      d.htab[pw][sl][1] = (uint32_t)e[n].hi;
      d.htab[pw][sl][2] = (uint32_t)(e[n].lo >> 32);
      d.htab[pw][sl][3] = (uint32_t)e[n].lo;
    }
  }
}
}  // namespace
}  // extern "C++"

int sqobfs_quic_keyring_create_suite(sqobfs_ctx *ctx, uint32_t suite, uint32_t count,
                                     const sqobfs_quic_key *keys, sqobfs_quic_keyring **out) {
  if (out) *out = nullptr;
  if (!ctx || !out || count == 0 || !keys) return SQ_EINVAL;
  if (suite != SQOBFS_QUIC_CHACHA20_POLY1305 && suite != SQOBFS_QUIC_AES_128_GCM)
    return SQ_EINVAL;
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  sqobfs_quic_keyring *kr = new (std::nothrow) sqobfs_quic_keyring();
  if (!kr) return SQ_ENOMEM;
  kr->ctx = ctx;
  kr->suite = suite;
  kr->count = count;
  hipError_t e = hipSuccess;
  if (suite == SQOBFS_QUIC_CHACHA20_POLY1305) {
    std::vector<sq::QuicKeyDev> h(count);
    for (uint32_t k = 0; k < count; k++) {
      memset(&h[k], 0, sizeof h[k]);
      for (int i = 0; i < 8; i++) h[k].key[i] = le32(keys[k].key + 4 * i);
      for (int i = 0; i < 3; i++) h[k].iv[i] = le32(keys[k].iv + 4 * i);
      for (int i = 0; i < 8; i++) h[k].hp[i] = le32(keys[k].hp + 4 * i);
    }
    kr->host0 = h[0];
    e = tab_alloc((void **)&kr->table, sizeof(sq::QuicKeyDev) * count, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(kr->table, h.data(), sizeof(sq::QuicKeyDev) * count,
                         hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  } else {
    std::vector<sq::QuicGcmKeyDev> h(count);
    for (uint32_t k = 0; k < count; k++) gcm_key(keys[k], h[k]);
    memcpy(kr->grk0, h[0].rk, sizeof kr->grk0);
    memcpy(kr->ghrk0, h[0].hrk, sizeof kr->ghrk0);
    memcpy(kr->giv0, h[0].iv, sizeof kr->giv0);
    e = tab_alloc((void **)&kr->gtable, sizeof(sq::QuicGcmKeyDev) * count, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(kr->gtable, h.data(), sizeof(sq::QuicGcmKeyDev) * count,
                         hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = tab_alloc((void **)&kr->t0, sizeof(uint32_t) * 256, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(kr->t0, aes_tables().t0, sizeof(uint32_t) * 256, hipMemcpyHostToDevice,
                         ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  }
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(ctx->stream);
    tab_free_async(kr->table, ctx->stream);
    tab_free_async(kr->gtable, ctx->stream);
    tab_free_async(kr->t0, ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
    delete kr;
    return hip_status(e);
  }
  *out = kr;
  return SQ_OK;
}

int sqobfs_quic_keyring_create(sqobfs_ctx *ctx, uint32_t count, const sqobfs_quic_key *keys,
                               sqobfs_quic_keyring **out) {
  return sqobfs_quic_keyring_create_suite(ctx, SQOBFS_QUIC_CHACHA20_POLY1305, count, keys, out);
}

void sqobfs_quic_keyring_destroy(sqobfs_quic_keyring *kr) {
  if (!kr) return;
  DeviceScope ds_(kr->ctx->device);
  kr->uses.fence(kr->ctx->rel);  // as sqobfs_keyring_destroy: stream-ordered, no wait
  tab_free_async(kr->table, kr->ctx->rel);
  tab_free_async(kr->gtable, kr->ctx->rel);
  tab_free_async(kr->t0, kr->ctx->rel);
  delete kr;
}

static int quic_launch(int open, sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                       const sqobfs_quic_batch *b, void *stream,
                       const sqobfs_keyring *okr = nullptr, const uint8_t *salt = nullptr) {
  if (!ctx || !kr || kr->ctx != ctx || !b || b->flags) return SQ_EINVAL;
  if (okr && (okr->ctx != ctx || okr->kind != SQOBFS_SALAMANDER || (!open && !salt)))
    return SQ_EINVAL;
  if (b->n == 0) return SQ_OK;
  if (!b->in || !b->in_off || !b->in_len || !b->out || !b->out_off || !b->out_len ||
      !b->pn_offset || !b->pn)
    return SQ_EINVAL;
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  if (kr->suite == SQOBFS_QUIC_AES_128_GCM) {
    sq::QGParams g;
    memset(&g, 0, sizeof g);
    g.in = b->in;
    g.in_off = b->in_off;
    g.in_len = b->in_len;
    g.out = b->out;
    g.out_off = b->out_off;
    g.out_len = b->out_len;
    g.pn_offset = b->pn_offset;
    g.pn = b->pn;
    g.key_id = b->key_id;
    g.pn_out = open ? b->pn_out : nullptr;
    g.keys = kr->gtable;
    g.t0 = kr->t0;
    g.n = b->n;
    g.n_keys = kr->count;
    memcpy(g.rk0, kr->grk0, sizeof g.rk0);
    memcpy(g.hrk0, kr->ghrk0, sizeof g.hrk0);
    memcpy(g.iv0, kr->giv0, sizeof g.iv0);
    if (okr) {
      g.obfs = 1;
      g.osalt = salt;
      g.opsk = okr->host0;
    }
    hipStream_t s = pick_stream(ctx, stream);
    // multi-key: group the packets by key first (the kernel then runs each
    // workgroup's units on one staged key).  The scratch is stream-ordered:
    // cached per library-owned stream, else allocated for this launch; none
    // (allocation failed, or the test hook) runs the ungrouped kernel
    void *scratch = nullptr;
    bool cached = false;
    const uint64_t gbytes =
        b->key_id && !g_gcm_ungrouped.load() ? sq_gcm_group_scratch(b->n, kr->count) : 0;
    std::unique_lock<std::mutex> glk(ctx->gcm_mu, std::defer_lock);
    if (gbytes) {
      glk.lock();
      if (s == ctx->stream && !ctx->gcm_scratch.count(s)) ctx->gcm_scratch[s] = {nullptr, 0};
      auto it = ctx->gcm_scratch.find(s);
      if (it != ctx->gcm_scratch.end()) {
        auto &e = it->second;
        if (e.second < gbytes) {  // grow (the old block is freed in stream order)
          const uint64_t want = std::max<uint64_t>(gbytes, 2 * e.second);
          tab_free_async(e.first, s);
          e = {nullptr, 0};
          if (tab_alloc(&e.first, want, s) == hipSuccess) e.second = want;
          else e.first = nullptr;
        }
        scratch = e.first;
        cached = true;
      } else {
        glk.unlock();  // (a caller's stream: this launch's own scratch)
        if (tab_alloc(&scratch, gbytes, s) != hipSuccess) scratch = nullptr;
      }
    }
    if (scratch) {
      const int gs = sq_launch_gcm_group(b->key_id, b->n, kr->count, open, b->out_len,
                                         open ? b->pn_out : nullptr, scratch, &g.gmeta, s);
      if (gs < 0) {
        if (!cached) tab_free_async(scratch, s);
        return gs;
      }
      g.perm = (const uint32_t *)scratch;
    }
    const int st = sq_launch_quic_gcm(open, &g, s);
    if (scratch && !cached) tab_free_async(scratch, s);
    if (st == SQ_OK) {
      kr->uses.note(s);
      if (okr) okr->uses.note(s);
    }
    return st;
  }
  sq::QParams q;
  memset(&q, 0, sizeof q);
  q.in = b->in;
  q.in_off = b->in_off;
  q.in_len = b->in_len;
  q.out = b->out;
  q.out_off = b->out_off;
  q.out_len = b->out_len;
  q.pn_offset = b->pn_offset;
  q.pn = b->pn;
  q.key_id = b->key_id;
  q.pn_out = open ? b->pn_out : nullptr;
  q.keys = kr->table;
  q.n = b->n;
  q.n_keys = kr->count;
  q.key0 = kr->host0;
  if (okr) {
    q.obfs = 1;
    q.osalt = salt;
    q.opsk = okr->host0;
  }
  hipStream_t s = pick_stream(ctx, stream);
  const int st = sq_launch_quic(open, &q, s);
  if (st == SQ_OK) {
    kr->uses.note(s);
    if (okr) okr->uses.note(s);
  }
  return st;
}

int sqobfs_quic_seal_salamander(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                                const sqobfs_keyring *okr, const sqobfs_quic_batch *b,
                                const uint8_t *salt, void *stream) {
  if (!okr) return SQ_EINVAL;
  return quic_launch(0, ctx, kr, b, stream, okr, salt);
}

int sqobfs_quic_open_salamander(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr,
                                const sqobfs_keyring *okr, const sqobfs_quic_batch *b,
                                void *stream) {
  if (!okr) return SQ_EINVAL;
  return quic_launch(1, ctx, kr, b, stream, okr, nullptr);
}

int sqobfs_quic_seal(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr, const sqobfs_quic_batch *b,
                     void *stream) {
  return quic_launch(0, ctx, kr, b, stream);
}

int sqobfs_quic_open(sqobfs_ctx *ctx, const sqobfs_quic_keyring *kr, const sqobfs_quic_batch *b,
                     void *stream) {
  return quic_launch(1, ctx, kr, b, stream);
}

size_t sqobfs_host_staging_bytes(const sqobfs_ctx *ctx) { return ctx ? ctx->pinned_cap : 0; }

void sqobfs_debug_fail_chunk(int chunk) { g_fail_chunk.store(chunk); }

void sqobfs_debug_gcm_ungrouped(int on) { g_gcm_ungrouped.store(on ? 1 : 0); }

uint64_t sqobfs_debug_device_pool(void *base, uint64_t bytes) {
  std::lock_guard<std::mutex> g(g_dpool.mu);
  const uint64_t used = g_dpool.used;
  g_dpool.used = 0;
  g_dpool.on = base != nullptr && bytes != 0;
  if (g_dpool.on) {
    g_dpool.lo = (uint8_t *)base;
    g_dpool.hi = (uint8_t *)base + bytes;
  }
  return used;
}

void sqobfs_debug_time_next_launch(void *start_event, void *stop_event) {
  sq_time_next_launch(start_event, stop_event);
}

int sqobfs_host_alloc(sqobfs_ctx *ctx, size_t bytes, void **out) {
  if (!ctx || !out) return SQ_EINVAL;
  *out = nullptr;
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  const int st = hip_status(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  if (st == SQ_OK) g_host_allocs.fetch_add(1);
  return st;
}

void sqobfs_host_free(sqobfs_ctx *ctx, void *p) {
  (void)ctx;
  if (p) {
    (void)hipHostFree(p);
    g_host_allocs.fetch_sub(1);
  }
}

int64_t sqobfs_debug_host_allocs(void) { return g_host_allocs.load(); }

int sqobfs_run_host(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir,
                    const sqobfs_batch *hb) {
  if (!ctx || !kr || kr->ctx != ctx) return SQ_EINVAL;
  if (dir != SQOBFS_OBFUSCATE && dir != SQOBFS_DEOBFUSCATE) return SQ_EINVAL;
  int st = check_batch_shape(hb, dir);
  if (st != SQ_OK || hb->n == 0) return st;
  const uint32_t n = hb->n;
  const int kind = kr->kind;
  const size_t S = salt_len(kind);
  if (hb->psk_id)
    for (uint32_t i = 0; i < n; i++)
      if (hb->psk_id[i] >= kr->count) return SQ_EPSK;
  // caller memory that is already pinned (sqobfs_host_alloc, hipHostMalloc)
  // is copied by DMA directly; pageable memory goes through pinned staging.
  // With both pinned there are no host-side staging copies, and twice the
  // chunks halve the pipeline's fill and drain (the
  // duplex ceiling)
  const bool in_pinned = is_pinned(hb->in), out_pinned = is_pinned(hb->out);
  const uint32_t maxc = in_pinned && out_pinned ? 2 * kHostChunks : kHostChunks;
  const uint32_t nchunk = n < 4096 ? 1u : std::min<uint32_t>(maxc, (n + 4095) / 4096);
  // Pieces of the pipeline: nchunk equal chunks; from 4 chunks on, the last
  // one is cut into 1/2, 1/4 and 1/4, so the drain -- the last piece's kernel
  // and copy-out, with nothing left to copy in -- moves a quarter chunk
  // ("Where the e2e time goes")
  std::vector<uint32_t> cut{0};
  if (nchunk < 4) {
    for (uint32_t c = 1; c <= nchunk; c++) cut.push_back((uint32_t)((uint64_t)n * c / nchunk));
  } else {
    const uint64_t W = 4ull * nchunk;
    uint64_t acc = 0;
    for (uint32_t c = 0; c + 1 < nchunk; c++) cut.push_back((uint32_t)(n * (acc += 4) / W));
    for (const uint32_t w : {2u, 1u, 1u}) cut.push_back((uint32_t)(n * (acc += w) / W));
  }
  const uint32_t npiece = (uint32_t)cut.size() - 1;
  // ---- one pass over the descriptors: per piece the input / output byte
  // ranges it touches, and what slot packing needs to know
  std::vector<Range> rin(npiece), rout(npiece);
  // (one thread: spreading the pass over 8 threads measured 1-4 % slower
  // end to end at 256K packets)
  SlotScan scan = slot_scan_start(hb, in_pinned && out_pinned);
  for (uint32_t c = 0; c < npiece; c++)
    packet_spans(hb, kind, dir, cut[c], cut[c + 1], rin[c], rout[c], &scan);
  // Pieces run concurrently: if one piece's output bytes overlap another
  // piece's input or output bytes (in-place or interleaved layouts), run
  // the batch as a single piece instead.
  if (parts_clash(hb, rin, rout)) {
    Range ri{SIZE_MAX, 0, 0, n}, ro{SIZE_MAX, 0, 0, n};
    for (uint32_t c = 0; c < npiece; c++) {
      if (rin[c].hi > rin[c].lo) ri.lo = std::min(ri.lo, rin[c].lo), ri.hi = std::max(ri.hi, rin[c].hi);
      if (rout[c].hi > rout[c].lo) ro.lo = std::min(ro.lo, rout[c].lo), ro.hi = std::max(ro.hi, rout[c].hi);
    }
    if (ri.lo > ri.hi) ri.lo = ri.hi = 0;
    if (ro.lo > ro.hi) ro.lo = ro.hi = 0;
    rin.assign(1, ri);
    rout.assign(1, ro);
  }
  const uint32_t nrun = (uint32_t)rin.size();
  // staging covers only the spans the batch touches, [lo, hi) of each buffer
  size_t in_lo = SIZE_MAX, in_hi = 0, out_lo = SIZE_MAX, out_hi = 0;
  for (uint32_t c = 0; c < nrun; c++) {
    if (rin[c].hi > rin[c].lo) in_lo = std::min(in_lo, rin[c].lo), in_hi = std::max(in_hi, rin[c].hi);
    if (rout[c].hi > rout[c].lo)
      out_lo = std::min(out_lo, rout[c].lo), out_hi = std::max(out_hi, rout[c].hi);
  }
  if (in_lo > in_hi) in_lo = in_hi = 0;
  if (out_lo > out_hi) out_lo = out_hi = 0;
  const bool preserve = !(hb->flags & SQOBFS_FLAG_OUT_UNINIT);
  const bool dev_salt = hb->flags & SQOBFS_FLAG_DEVICE_SALT;
  const bool host_salt = dir == SQOBFS_OBFUSCATE && !dev_salt;

  // staging layout (device mirror of the host ranges; pinned copies only
  // for what is pageable)
  // each staged byte keeps its address modulo 16 (the kernel's 16-byte
  // blocks are the caller's: aligned outputs stay the fast case, and
  // SQOBFS_FLAG_OUT_BLOCKS's promise holds on the device copy); with
  // SQOBFS_FLAG_OUT_LINES output bytes keep their address modulo 128, and the
  // last output line's padding, which the kernel writes, is staged too
  const size_t A = 256;
  const bool lines = hb->flags & SQOBFS_FLAG_OUT_LINES;
  // fixed-stride slots: packed rows instead of the spans (slot_pack)
  const SlotPack sp = nrun == npiece ? slot_pack(hb, scan, in_lo, in_hi, out_lo, out_hi)
                                     : SlotPack{};
  size_t o = 0;
  const size_t o_in = sp.on ? 0 : o + (((uintptr_t)hb->in + in_lo) & 15);
  o = align_up(sp.on ? sp.pi * n : o_in + (in_hi - in_lo), A);
  const size_t o_out = sp.on ? o : o + (((uintptr_t)hb->out + out_lo) & (lines ? 127 : 15));
  o = align_up(sp.on ? o_out + sp.po * n : o_out + (out_hi - out_lo) + (lines ? 128 : 0), A);
  // The descriptors the kernels read, in two groups, each one block of
  // arrays and one copy: the first piece's (staged and copied before any
  // payload moves) and the rest's (staged while the first piece's payload
  // is on the link).  Staging all of them first held the pipeline's first
  // copy back by ~0.4 ms at 256K packets.
  struct DescGroup {
    uint32_t p0, p1;
    size_t base, inlen, outoff, salt, pid, cap, end;  // in_off at base
  };
  auto group_at = [&](uint32_t p0, uint32_t p1, size_t at) {
    DescGroup g;
    const size_t m = p1 - p0;
    g.p0 = p0;
    g.p1 = p1;
    g.base = at;
    size_t x = at + 8 * m;
    g.inlen = x = align_up(x, 16);
    x += 4 * m;
    g.outoff = x = align_up(x, 16);
    x += 8 * m;
    g.salt = x = align_up(x, 16);
    x += host_salt ? S * m : 0;
    g.pid = x = align_up(x, 16);
    x += hb->psk_id ? 2 * m : 0;
    g.cap = x = align_up(x, 16);
    x += hb->in_cap ? 4 * m : 0;
    g.end = x;
    return g;
  };
  DescGroup grp[2];
  grp[0] = group_at(rin[0].p0, rin[0].p1, o);
  o = align_up(grp[0].end, A);
  grp[1] = group_at(nrun > 1 ? rin[1].p0 : n, n, o);
  o = align_up(grp[1].end, A);
  const size_t o_outlen = o;   o = align_up(o + 4ull * n, A);
  const size_t o_saltout = o;  o = align_up(o + (dev_salt && hb->salt_out ? S * n : 0), A);
  const size_t total = o;

  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceScope ds_(ctx->device);
  if (ds_.status != SQ_OK) return ds_.status;
  if (ctx->pinned_cap < total) {
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_cap = 0;
    SQ_TRY(hipHostMalloc(&ctx->pinned, total, hipHostMallocDefault));
    ctx->pinned_cap = total;
  }
  if (ctx->dev_cap < total) {
    if (ctx->dev) (void)hipFree(ctx->dev);
    ctx->dev = nullptr;
    ctx->dev_cap = 0;
    SQ_TRY(hipMalloc(&ctx->dev, total));
    ctx->dev_cap = total;
  }
  for (auto &e : ctx->ev)
    if (!e) SQ_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  uint8_t *H = ctx->pinned, *D = ctx->dev;
  // staged image of buffer byte x: base + o + (x - lo)
  auto hin = [&](size_t x) { return H + o_in + (x - in_lo); };
  auto hout = [&](size_t x) { return H + o_out + (x - out_lo); };
  auto din = [&](size_t x) { return D + o_in + (x - in_lo); };
  auto dout = [&](size_t x) { return D + o_out + (x - out_lo); };
  // Every failure past this point drains the three streams first, so no
  // copy is still writing the caller's or the staging memory on return.
  auto drain = [&](int code) {
    (void)hipStreamSynchronize(ctx->h2d);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamSynchronize(ctx->d2h);
    (void)hipGetLastError();
    return code;
  };
#define SQ_TRY_DRAIN(x)                                    \
  do {                                                     \
    const int st_ = hip_status((x));                       \
    if (st_ != SQ_OK) return drain(st_);                   \
  } while (0)

  // a descriptor group: staged, then one copy on the copy-in stream
  auto stage_group = [&](const DescGroup &g) {
    const size_t m = g.p1 - g.p0;
    if (m == 0) return hipSuccess;
    if (sp.on) {  // packed rows: packet i's bytes at row i, phase kept
      uint64_t *io = (uint64_t *)(H + g.base), *oo = (uint64_t *)(H + g.outoff);
      for (uint32_t i = g.p0; i < g.p1; i++) {
        io[i - g.p0] = sp.pi * i + sp.phi;
        oo[i - g.p0] = sp.po * i + sp.pho;
      }
    } else {
      memcpy(H + g.base, hb->in_off + g.p0, 8 * m);
      memcpy(H + g.outoff, hb->out_off + g.p0, 8 * m);
    }
    memcpy(H + g.inlen, hb->in_len + g.p0, 4 * m);
    if (host_salt) memcpy(H + g.salt, hb->salt + S * g.p0, S * m);
    if (hb->psk_id) memcpy(H + g.pid, hb->psk_id + g.p0, 2 * m);
    if (hb->in_cap) memcpy(H + g.cap, hb->in_cap + g.p0, 4 * m);
    return hipMemcpyAsync(D + g.base, H + g.base, g.end - g.base, hipMemcpyHostToDevice, ctx->h2d);
  };
  // a landed piece's results to the caller: out_len (and salt_out) from
  // staging, and pageable output bytes; run while later pieces still move
  auto finish = [&](uint32_t c) {
    const uint32_t p0 = rin[c].p0, m = rin[c].p1 - rin[c].p0;
    memcpy(hb->out_len + p0, H + o_outlen + 4ull * p0, 4ull * m);
    if (dev_salt && hb->salt_out) memcpy(hb->salt_out + S * p0, H + o_saltout + S * p0, S * m);
    if (!out_pinned && rout[c].hi > rout[c].lo)
      par_memcpy(hb->out + rout[c].lo, hout(rout[c].lo), rout[c].hi - rout[c].lo);
  };

  // pageable output is copied out piece by piece while later pieces move;
  // with page-locked output only out_len (and salt_out) remain, one copy at
  // the end (per-piece copies and waits cost more than they overlap)
  const bool per_piece = !out_pinned && nrun > 1;
  // ---- pipeline: H2D(c) on h2d | kernel(c) on the compute stream | D2H(c)
  // on d2h, chained by events; piece c+1's copy-in overlaps piece c's
  // kernel and piece c-1's copy-out, and the host finishes each landed
  // piece while the later ones move.
  SQ_TRY_DRAIN(stage_group(grp[0]));
  uint32_t fin = 0;  // pieces finished on the host
  for (uint32_t c = 0; c < nrun; c++) {
    const Range &ri = rin[c], &ro = rout[c];
    const uint32_t rows = ri.p1 - ri.p0;
    if (c == 1) SQ_TRY_DRAIN(stage_group(grp[1]));
    if (sp.on) {  // rows [p0, p1): the first wi / wo bytes of each slot
      if (sp.wi && rows)
        SQ_TRY_DRAIN(hipMemcpy2DAsync(D + o_in + sp.pi * ri.p0 + sp.phi, sp.pi,
                                      hb->in + hb->in_off[ri.p0], sp.si, sp.wi, rows,
                                      hipMemcpyHostToDevice, ctx->h2d));
      if (preserve && sp.wo && rows)
        SQ_TRY_DRAIN(hipMemcpy2DAsync(D + o_out + sp.po * ri.p0 + sp.pho, sp.po,
                                      hb->out + hb->out_off[ri.p0], sp.so, sp.wo, rows,
                                      hipMemcpyHostToDevice, ctx->h2d));
    } else if (ri.hi > ri.lo) {
      const uint8_t *src = hb->in + ri.lo;
      if (!in_pinned) {
        par_memcpy(hin(ri.lo), src, ri.hi - ri.lo);
        src = hin(ri.lo);
      }
      SQ_TRY_DRAIN(hipMemcpyAsync(din(ri.lo), src, ri.hi - ri.lo, hipMemcpyHostToDevice,
                                  ctx->h2d));
    }
    if (!sp.on && preserve && ro.hi > ro.lo) {  // bytes between packets keep their value
      const uint8_t *src = hb->out + ro.lo;
      if (!out_pinned) {
        par_memcpy(hout(ro.lo), src, ro.hi - ro.lo);
        src = hout(ro.lo);
      }
      SQ_TRY_DRAIN(hipMemcpyAsync(dout(ro.lo), src, ro.hi - ro.lo, hipMemcpyHostToDevice,
                                  ctx->h2d));
    }
    hipEvent_t ev_in = ctx->ev[3 * c], ev_k = ctx->ev[3 * c + 1], ev_out = ctx->ev[3 * c + 2];
    SQ_TRY_DRAIN(hipEventRecord(ev_in, ctx->h2d));
    SQ_TRY_DRAIN(hipStreamWaitEvent(ctx->stream, ev_in, 0));
    const DescGroup &g = grp[c == 0 ? 0 : 1];
    const size_t k = ri.p0 - g.p0;  // the piece's first packet within its group
    sqobfs_batch db = *hb;
    db.n = rows;
    db.in = sp.on ? D + o_in : din(0);  // in_off[i] >= in_lo for every packet of the batch
    db.in_off = (const uint64_t *)(D + g.base) + k;
    db.in_len = (const uint32_t *)(D + g.inlen) + k;
    db.out = sp.on ? D + o_out : dout(0);
    db.out_off = (const uint64_t *)(D + g.outoff) + k;
    db.out_len = (uint32_t *)(D + o_outlen) + ri.p0;
    db.salt = host_salt ? D + g.salt + S * k : nullptr;
    db.salt_out = dev_salt && hb->salt_out ? D + o_saltout + S * ri.p0 : nullptr;
    db.psk_id = hb->psk_id ? (const uint16_t *)(D + g.pid) + k : nullptr;
    db.in_cap = hb->in_cap ? (const uint32_t *)(D + g.cap) + k : nullptr;
    if (db.n) {
      sq::KParams kp = make_params(ctx, kr, &db);
      if (kp.ppw == 0) {  // lengths are on the host: size the units by bytes
        uint64_t bytes = 0;
        for (uint32_t i = ri.p0; i < ri.p1; i++) bytes += hb->in_len[i];
        kp.ppw = sqobfs_unit_packets_for_kind(kr->kind, bytes, db.n, hb->psk_id != nullptr);
      }
      int fc = (int)c;
      st = g_fail_chunk.compare_exchange_strong(fc, -1) ? SQ_EDEVICE
                                                         : sq_launch_obfs(kind, dir, &kp, ctx->stream);
      if (st != SQ_OK) return drain(st);
    }
    SQ_TRY_DRAIN(hipEventRecord(ev_k, ctx->stream));
    SQ_TRY_DRAIN(hipStreamWaitEvent(ctx->d2h, ev_k, 0));
    if (c + 1 == nrun) kr->uses.note(ctx->stream);
    if (sp.on) {
      if (sp.wo && rows)
        SQ_TRY_DRAIN(hipMemcpy2DAsync(hb->out + hb->out_off[ri.p0], sp.so,
                                      D + o_out + sp.po * ri.p0 + sp.pho, sp.po, sp.wo, rows,
                                      hipMemcpyDeviceToHost, ctx->d2h));
    } else if (ro.hi > ro.lo) {
      uint8_t *dst = out_pinned ? hb->out + ro.lo : hout(ro.lo);
      SQ_TRY_DRAIN(hipMemcpyAsync(dst, dout(ro.lo), ro.hi - ro.lo, hipMemcpyDeviceToHost,
                                  ctx->d2h));
    }
    if (!per_piece) continue;
    if (rows) {
      SQ_TRY_DRAIN(hipMemcpyAsync(H + o_outlen + 4ull * ri.p0, D + o_outlen + 4ull * ri.p0,
                                  4ull * rows, hipMemcpyDeviceToHost, ctx->d2h));
      if (dev_salt && hb->salt_out)
        SQ_TRY_DRAIN(hipMemcpyAsync(H + o_saltout + S * ri.p0, D + o_saltout + S * ri.p0,
                                    S * rows, hipMemcpyDeviceToHost, ctx->d2h));
    }
    SQ_TRY_DRAIN(hipEventRecord(ev_out, ctx->d2h));
    // finish the pieces that have landed meanwhile, in order
    while (fin < c) {
      const hipError_t q = hipEventQuery(ctx->ev[3 * fin + 2]);
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        break;
      }
      SQ_TRY_DRAIN(q);
      finish(fin++);
    }
  }
  if (per_piece) {
    for (; fin < nrun; fin++) {
      SQ_TRY_DRAIN(hipEventSynchronize(ctx->ev[3 * fin + 2]));
      finish(fin);
    }
    SQ_TRY_DRAIN(hipStreamSynchronize(ctx->d2h));
    return SQ_OK;
  }
  SQ_TRY_DRAIN(hipMemcpyAsync(H + o_outlen, D + o_outlen, 4ull * n, hipMemcpyDeviceToHost, ctx->d2h));
  if (dev_salt && hb->salt_out)
    SQ_TRY_DRAIN(hipMemcpyAsync(H + o_saltout, D + o_saltout, S * n, hipMemcpyDeviceToHost, ctx->d2h));
  SQ_TRY_DRAIN(hipStreamSynchronize(ctx->d2h));
  if (!out_pinned)  // (one piece)
    for (uint32_t c = 0; c < nrun; c++)
      if (rout[c].hi > rout[c].lo)
        par_memcpy(hb->out + rout[c].lo, hout(rout[c].lo), rout[c].hi - rout[c].lo);
  memcpy(hb->out_len, H + o_outlen, 4ull * n);
  if (dev_salt && hb->salt_out) memcpy(hb->salt_out, H + o_saltout, S * n);
  return SQ_OK;
#undef SQ_TRY_DRAIN
}

// ---------------------------------------------------------------- shards

int sqobfs_shard_cuts(uint32_t n, const uint32_t *in_len, uint32_t parts, uint32_t *cut) {
  if (!cut || parts == 0 || (n && !in_len)) return SQ_EINVAL;
  // weight = bytes + a per-packet constant (descriptor, key derivation), so
  // runs of empty datagrams still spread
  constexpr uint64_t kPerPacket = 64;
  uint64_t tot = 0;
  for (uint32_t i = 0; i < n; i++) tot += in_len[i] + kPerPacket;
  cut[0] = 0;
  uint64_t acc = 0;
  uint32_t i = 0;
  for (uint32_t k = 1; k < parts; k++) {
    const uint64_t want = tot * k / parts;
    while (i < n && acc + in_len[i] + kPerPacket / 2 <= want) acc += in_len[i++] + kPerPacket;
    cut[k] = i;
  }
  cut[parts] = n;
  return SQ_OK;
}

namespace {
// packets [p0, p1) of b as a batch of their own (same buffers)
sqobfs_batch sub_batch(const sqobfs_batch &b, uint32_t p0, uint32_t p1, size_t S) {
  sqobfs_batch s = b;
  s.n = p1 - p0;
  s.in_off = b.in_off + p0;
  s.in_len = b.in_len + p0;
  s.out_off = b.out_off + p0;
  s.out_len = b.out_len + p0;
  if (b.salt) s.salt = b.salt + S * p0;
  if (b.psk_id) s.psk_id = b.psk_id + p0;
  if (b.in_cap) s.in_cap = b.in_cap + p0;
  if (b.salt_out) s.salt_out = b.salt_out + S * p0;
  return s;
}
}  // namespace

int sqobfs_run_host_sharded(uint32_t nctx, sqobfs_ctx *const *ctxs,
                            const sqobfs_keyring *const *krs, int dir, const sqobfs_batch *hb) {
  if (nctx == 0 || !ctxs || !krs || !hb) return SQ_EINVAL;
  for (uint32_t k = 0; k < nctx; k++)
    if (!ctxs[k] || !krs[k] || krs[k]->ctx != ctxs[k] || krs[k]->kind != krs[0]->kind)
      return SQ_EINVAL;
  if (nctx == 1) return sqobfs_run_host(ctxs[0], krs[0], dir, hb);
  const int st0 = check_batch_shape(hb, dir);
  if (st0 != SQ_OK || hb->n == 0) return st0;
  std::vector<uint32_t> cut(nctx + 1);
  const int sc = sqobfs_shard_cuts(hb->n, hb->in_len, nctx, cut.data());
  if (sc != SQ_OK) return sc;
  const size_t S = salt_len(krs[0]->kind);
  // Each shard copies its whole input / output span: when one shard's output
  // span meets another shard's span (interleaved, shuffled or in-place
  // layouts) they cannot run at once, and the batch runs on one context
  // (whose own chunking makes the same check).
  {
    std::vector<Range> rin(nctx), rout(nctx);
    for (uint32_t k = 0; k < nctx; k++)
      packet_spans(hb, krs[0]->kind, dir, cut[k], cut[k + 1], rin[k], rout[k]);
    if (parts_clash(hb, rin, rout)) return sqobfs_run_host(ctxs[0], krs[0], dir, hb);
  }
  std::vector<int> st(nctx, SQ_OK);
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < nctx; k++) {
    if (cut[k + 1] == cut[k]) continue;
    th.emplace_back([&, k] {
      const sqobfs_batch sb = sub_batch(*hb, cut[k], cut[k + 1], S);
      st[k] = sqobfs_run_host(ctxs[k], krs[k], dir, &sb);
    });
  }
  for (auto &t : th) t.join();
  for (int x : st)
    if (x != SQ_OK) return x;
  return SQ_OK;
}

int sqobfs_shard_launch(uint32_t nctx, sqobfs_ctx *const *ctxs, const sqobfs_keyring *const *krs,
                        int dir, const sqobfs_batch *bs, sqobfs_shard_ticket **out) {
  if (out) *out = nullptr;
  if (nctx == 0 || !ctxs || !krs || !bs || !out) return SQ_EINVAL;
  for (uint32_t k = 0; k < nctx; k++)
    if (!ctxs[k] || !krs[k] || krs[k]->ctx != ctxs[k]) return SQ_EINVAL;
  sqobfs_shard_ticket *t = new (std::nothrow) sqobfs_shard_ticket();
  if (!t) return SQ_ENOMEM;
  // launches are asynchronous: one host thread queues every shard on its
  // context's stream and records the context's completion event after it
  int st = SQ_OK;
  for (uint32_t k = 0; k < nctx && st == SQ_OK; k++) {
    st = sqobfs_launch(ctxs[k], krs[k], dir, &bs[k], ctxs[k]->stream);
    if (st != SQ_OK) break;
    DeviceScope ds_(ctxs[k]->device);
    hipEvent_t e = nullptr;
    st = hip_status(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (st == SQ_OK) {
      st = hip_status(hipEventRecord(e, ctxs[k]->stream));
      t->parts.push_back({ctxs[k], e});
      if (st != SQ_OK) t->parts.back().ev = nullptr, (void)hipEventDestroy(e);
    }
    if (st != SQ_OK) {
      // the shards queued so far: wait for them before reporting
      for (uint32_t j = 0; j <= k; j++) (void)sqobfs_sync(ctxs[j], ctxs[j]->stream);
    }
  }
  if (st != SQ_OK) {
    (void)sqobfs_shard_wait(t);
    return st;
  }
  *out = t;
  return SQ_OK;
}

int sqobfs_shard_query(sqobfs_shard_ticket *t) {
  if (!t) return SQ_EINVAL;
  for (auto &p : t->parts) {
    if (!p.ev) continue;
    DeviceScope ds_(p.ctx->device);
    const hipError_t q = hipEventQuery(p.ev);
    if (q == hipErrorNotReady) return 0;
    if (q != hipSuccess) return hip_status(q);
  }
  return 1;
}

int sqobfs_shard_wait(sqobfs_shard_ticket *t) {
  if (!t) return SQ_EINVAL;
  int st = SQ_OK;
  for (auto &p : t->parts) {
    if (!p.ev) continue;
    DeviceScope ds_(p.ctx->device);
    // poll (sqobfs_set_sync_spin) before blocking, as sqobfs_sync does
    const uint32_t spin = p.ctx->spin_us.load(std::memory_order_relaxed);
    int s2 = 1;
    if (spin) {
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipEventQuery(p.ev);
        if (q == hipSuccess) {
          s2 = SQ_OK;
          break;
        }
        if (q != hipErrorNotReady) {
          s2 = hip_status(q);
          break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin)) break;
        cpu_relax();
      }
    }
    if (s2 == 1) s2 = hip_status(hipEventSynchronize(p.ev));
    if (st == SQ_OK) st = s2;
    (void)hipEventDestroy(p.ev);
  }
  delete t;
  return st;
}

int sqobfs_shard_run(uint32_t nctx, sqobfs_ctx *const *ctxs, const sqobfs_keyring *const *krs,
                     int dir, const sqobfs_batch *bs) {
  sqobfs_shard_ticket *t = nullptr;
  const int st = sqobfs_shard_launch(nctx, ctxs, krs, dir, bs, &t);
  if (st != SQ_OK) return st;
  return sqobfs_shard_wait(t);
}

}  // extern "C"
