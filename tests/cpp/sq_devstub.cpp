// sq_devstub.cpp -- a CPU "device" behind the engine's device interface
// (sq_internal.h) and the few public entry points the engine and its tests
// call, so the packet conn engine (host/pconn.cpp) and the CPU path
// (host/sq_cpu.cpp) build and run with no HIP runtime at all: under ASan and
// TSan in this container (scripts/dev/cpu_sanitize.sh), where a GPU and a
// sanitized HIP runtime are not available.
//
// Test infrastructure, never shipped.  Streams are real threads: a launch is
// queued and transformed there (sq::cpu::run_batch), asynchronously, and a
// stream wait blocks until it is done -- the same hand-off between a worker
// and the "GPU" as on the MI355X, which is what the sanitizers should see.
// Device salts follow include/sqobfs.h's construction (ChaCha20 of the
// context key and launch sequence number), so wire checks hold as on a GPU.
#include <string.h>
#include <sys/random.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "sq_cpu.h"
#include "sq_internal.h"
#include "sqobfs.h"

namespace {
std::atomic<int64_t> g_allocs{0};

struct Stream {
  std::mutex mu;
  std::condition_variable cv, cv_done;
  std::deque<std::function<void()>> q;
  bool stop = false, busy = false;
  std::thread th;
  Stream() {
    th = std::thread([this] {
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        auto job = std::move(q.front());
        q.pop_front();
        busy = true;
        lk.unlock();
        job();
        lk.lock();
        busy = false;
        cv_done.notify_all();
      }
    });
  }
  void push(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu);
    q.push_back(std::move(f));
    cv.notify_one();
  }
  void drain() {
    std::unique_lock<std::mutex> lk(mu);
    cv_done.wait(lk, [&] { return q.empty() && !busy; });
  }
  ~Stream() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
};
}  // namespace

struct sqobfs_ctx {
  uint32_t key[8];
  std::atomic<uint64_t> seq{0};
};

struct sqobfs_keyring {
  sqobfs_ctx *ctx = nullptr;
  int kind = 0;
  uint32_t count = 0;
  std::vector<sq::PskEntry> host;
};

// ---- the engine's device interface
int sq_ctx_stream_create(sqobfs_ctx *, void **out) {
  *out = new (std::nothrow) Stream();
  return *out ? SQ_OK : SQ_ENOMEM;
}
void sq_ctx_stream_destroy(sqobfs_ctx *, void *s) {
  if (!s) return;
  static_cast<Stream *>(s)->drain();
  delete static_cast<Stream *>(s);
}
int sq_ctx_stream_wait(sqobfs_ctx *, void *s, uint32_t) {
  if (s) static_cast<Stream *>(s)->drain();
  return SQ_OK;
}
int sq_ctx_stream_wait_blocking(sqobfs_ctx *ctx, void *s, uint32_t) {
  return sq_ctx_stream_wait(ctx, s, 0);
}
void sq_keyring_forget(const sqobfs_keyring *, void *) {}
int sq_host_alloc_mapped(sqobfs_ctx *ctx, size_t bytes, void **out) {
  return sqobfs_host_alloc(ctx, bytes, out);
}
const sq::PskEntry *sq_keyring_host(const sqobfs_keyring *kr, uint32_t *count) {
  *count = kr->count;
  return kr->host.data();
}
sqobfs_ctx *sq_keyring_ctx(const sqobfs_keyring *kr) { return kr->ctx; }
void sq_keyring_hot(const sqobfs_keyring *, uint32_t *hot_m, uint32_t *hot_iv) {
  *hot_m = 16;
  *hot_iv = 0;
}
int sq_keyring_from_entries(sqobfs_ctx *ctx, int kind, const sq::PskEntry *e, uint32_t count,
                            uint32_t, uint32_t, void *, sqobfs_keyring **out) {
  *out = nullptr;
  if (!ctx || !e || !count) return SQ_EINVAL;
  sqobfs_keyring *kr = new (std::nothrow) sqobfs_keyring();
  if (!kr) return SQ_ENOMEM;
  kr->ctx = ctx;
  kr->kind = kind;
  kr->count = count;
  kr->host.assign(e, e + count);
  *out = kr;
  return SQ_OK;
}
void sq_salt_take(sqobfs_ctx *ctx, uint32_t key[8], uint64_t *seq) {
  if (!ctx) return sq_host_salt_take(key, seq);
  memcpy(key, ctx->key, sizeof ctx->key);
  *seq = ctx->seq.fetch_add(1);
}

extern "C" {

const char *sqobfs_strerror(int status) { return status == SQ_OK ? "ok" : "error (stub)"; }

int sqobfs_open(int device, sqobfs_ctx **out) {
  if (!out) return SQ_EINVAL;
  *out = nullptr;
  if (device != 0) return SQ_ENODEV;
  sqobfs_ctx *c = new (std::nothrow) sqobfs_ctx();
  if (!c) return SQ_ENOMEM;
  if (getrandom(c->key, sizeof c->key, 0) != (ssize_t)sizeof c->key) memset(c->key, 7, 32);
  *out = c;
  return SQ_OK;
}

void sqobfs_close(sqobfs_ctx *ctx) {
  if (!ctx) return;
  sq_engine_ctx_closed(ctx);
  delete ctx;
}

int sqobfs_keyring_create(sqobfs_ctx *ctx, int kind, uint32_t count, const uint8_t *blob,
                          const uint64_t *off, const uint32_t *len, sqobfs_keyring **out) {
  if (!out || !count || !off || !len) return SQ_EINVAL;
  sqobfs_keyring *kr = new (std::nothrow) sqobfs_keyring();
  if (!kr) return SQ_ENOMEM;
  kr->ctx = ctx;
  kr->kind = kind;
  kr->count = count;
  kr->host.resize(count);
  for (uint32_t k = 0; k < count; k++)
    sq::cpu::psk_prepare(kind, blob ? blob + off[k] : nullptr, len[k], &kr->host[k]);
  *out = kr;
  return SQ_OK;
}
void sqobfs_keyring_destroy(sqobfs_keyring *kr) { delete kr; }
int sqobfs_keyring_kind(const sqobfs_keyring *kr) { return kr ? kr->kind : SQ_EINVAL; }
uint32_t sqobfs_keyring_count(const sqobfs_keyring *kr) { return kr ? kr->count : 0; }

// the "kernel": the batch is copied (the caller's descriptor may go away),
// its salts drawn at launch time as the GPU's are, the bytes transformed on
// the stream's thread
int sqobfs_launch(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir, const sqobfs_batch *b,
                  void *stream) {
  if (!ctx || !kr || kr->ctx != ctx || !b) return SQ_EINVAL;
  if (b->n == 0) return SQ_OK;
  std::vector<uint8_t> salts;
  if (b->flags & SQOBFS_FLAG_DEVICE_SALT) {
    uint32_t key[8];
    uint64_t seq;
    sq_salt_take(ctx, key, &seq);
    salts.resize((size_t)b->n * (kr->kind == SQOBFS_SALAMANDER ? 8 : 16));
    sq::cpu::salt_stream(key, seq, salts.data(), salts.size());
  }
  const sqobfs_batch d = *b;
  auto job = [kr, dir, d, salts = std::move(salts)] {
    (void)sq::cpu::run_batch(kr->kind, dir, kr->host.data(), kr->count, &d,
                             salts.empty() ? nullptr : salts.data());
  };
  if (stream) static_cast<Stream *>(stream)->push(std::move(job));
  else job();
  return SQ_OK;
}

void *sqobfs_stream(sqobfs_ctx *) { return nullptr; }

int sqobfs_host_alloc(sqobfs_ctx *, size_t bytes, void **out) {
  if (!out) return SQ_EINVAL;
  *out = malloc(bytes ? bytes : 1);
  if (!*out) return SQ_ENOMEM;
  g_allocs.fetch_add(1);
  return SQ_OK;
}
void sqobfs_host_free(sqobfs_ctx *, void *p) {
  if (!p) return;
  free(p);
  g_allocs.fetch_sub(1);
}
int64_t sqobfs_debug_host_allocs(void) { return g_allocs.load(); }

int sqobfs_quic_seal_salamander(sqobfs_ctx *, const sqobfs_quic_keyring *,
                                const sqobfs_keyring *, const sqobfs_quic_batch *,
                                const uint8_t *, void *) {
  return SQ_ENODEV;
}
int sqobfs_quic_open_salamander(sqobfs_ctx *, const sqobfs_quic_keyring *,
                                const sqobfs_keyring *, const sqobfs_quic_batch *, void *) {
  return SQ_ENODEV;
}

}  // extern "C"
