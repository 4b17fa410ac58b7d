// sq_api.hip -- the C ABI declared in include/sqobfs.h.
//
// Contexts (one per GPU), keyrings (the PSK captured by NewSalamanderConn /
// NewXPlusPacketConn, hysteria2/salamander.go:24-40, hysteria/xplus.go:19-37),
// device-resident batch launches and the host-staged path.  No hashing or
// XOR happens on the host: every byte transform runs in sq_kernels.hip, and
// a missing/failed GPU is reported as an error, never worked around.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <new>

#include "../../include/sqobfs.h"
#include "sq_internal.h"

struct sqobfs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;  // guards the staging buffers of sqobfs_run_host
  uint8_t *pinned = nullptr;
  size_t pinned_cap = 0;
  uint8_t *dev = nullptr;
  size_t dev_cap = 0;
};

struct sqobfs_keyring {
  sqobfs_ctx *ctx = nullptr;
  int kind = 0;
  uint32_t count = 0;
  sq::PskEntry *table = nullptr;  // device
  sq::PskEntry host0;             // entry 0, passed by value to the kernels
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

size_t salt_len(int kind) {
  return kind == SQOBFS_SALAMANDER ? SQOBFS_SALAMANDER_SALT_LEN : SQOBFS_XPLUS_SALT_LEN;
}

// NULL is the HIP null stream (HIP convention; torch's default stream), so a
// caller's events and copies on that stream order with our kernels.
hipStream_t pick_stream(sqobfs_ctx *ctx, void *stream) {
  (void)ctx;
  return (hipStream_t)stream;
}

int check_batch_shape(const sqobfs_batch *b, int dir) {
  if (!b) return SQ_EINVAL;
  if (b->flags != 0) return SQ_EINVAL;
  if (b->n == 0) return SQ_OK;
  if (!b->in || !b->in_off || !b->in_len || !b->out || !b->out_off || !b->out_len)
    return SQ_EINVAL;
  if (dir == SQOBFS_OBFUSCATE) {
    if (!b->salt || ((uintptr_t)b->salt & 3)) return SQ_EINVAL;
  }
  return SQ_OK;
}

sq::KParams make_params(const sqobfs_keyring *kr, const sqobfs_batch *b) {
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
  return kp;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

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
  SQ_TRY(hipSetDevice(device));
  sqobfs_ctx *c = new (std::nothrow) sqobfs_ctx();
  if (!c) return SQ_ENOMEM;
  c->device = device;
  const hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return hip_status(e);
  }
  *out = c;
  return SQ_OK;
}

void sqobfs_close(sqobfs_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->dev) (void)hipFree(ctx->dev);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

void *sqobfs_stream(sqobfs_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int sqobfs_sync(sqobfs_ctx *ctx, void *stream) {
  if (!ctx) return SQ_EINVAL;
  SQ_TRY(hipSetDevice(ctx->device));
  return hip_status(hipStreamSynchronize(pick_stream(ctx, stream)));
}

int sqobfs_keyring_create(sqobfs_ctx *ctx, int kind, uint32_t count, const uint8_t *blob,
                          const uint64_t *off, const uint32_t *len, sqobfs_keyring **out) {
  if (!ctx || !out || count == 0 || !off || !len) return SQ_EINVAL;
  if (kind != SQOBFS_SALAMANDER && kind != SQOBFS_XPLUS) return SQ_EINVAL;
  *out = nullptr;
  size_t blob_bytes = 0;
  for (uint32_t k = 0; k < count; k++) blob_bytes = std::max<size_t>(blob_bytes, off[k] + len[k]);
  if (blob_bytes && !blob) return SQ_EINVAL;
  SQ_TRY(hipSetDevice(ctx->device));
  sqobfs_keyring *kr = new (std::nothrow) sqobfs_keyring();
  if (!kr) return SQ_ENOMEM;
  kr->ctx = ctx;
  kr->kind = kind;
  kr->count = count;
  uint8_t *d_blob = nullptr;
  uint64_t *d_off = nullptr;
  uint32_t *d_len = nullptr;
  hipError_t e = hipMalloc(&kr->table, sizeof(sq::PskEntry) * count);
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
    if (kr->table) (void)hipFree(kr->table);
    delete kr;
    return st;
  }
  *out = kr;
  return SQ_OK;
}

void sqobfs_keyring_destroy(sqobfs_keyring *kr) {
  if (!kr) return;
  (void)hipSetDevice(kr->ctx->device);
  (void)hipStreamSynchronize(kr->ctx->stream);
  if (kr->table) (void)hipFree(kr->table);
  delete kr;
}

int sqobfs_keyring_kind(const sqobfs_keyring *kr) { return kr ? kr->kind : SQ_EINVAL; }
uint32_t sqobfs_keyring_count(const sqobfs_keyring *kr) { return kr ? kr->count : 0; }

int sqobfs_launch(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir, const sqobfs_batch *b,
                  void *stream) {
  if (!ctx || !kr || kr->ctx != ctx) return SQ_EINVAL;
  if (dir != SQOBFS_OBFUSCATE && dir != SQOBFS_DEOBFUSCATE) return SQ_EINVAL;
  const int st = check_batch_shape(b, dir);
  if (st != SQ_OK || b->n == 0) return st;
  SQ_TRY(hipSetDevice(ctx->device));
  const sq::KParams kp = make_params(kr, b);
  return sq_launch_obfs(kr->kind, dir, &kp, pick_stream(ctx, stream));
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

int sqobfs_host_alloc(sqobfs_ctx *ctx, size_t bytes, void **out) {
  if (!ctx || !out) return SQ_EINVAL;
  *out = nullptr;
  SQ_TRY(hipSetDevice(ctx->device));
  return hip_status(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
}

void sqobfs_host_free(sqobfs_ctx *ctx, void *p) {
  (void)ctx;
  if (p) (void)hipHostFree(p);
}

int sqobfs_run_host(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int dir,
                    const sqobfs_batch *hb) {
  if (!ctx || !kr || kr->ctx != ctx) return SQ_EINVAL;
  if (dir != SQOBFS_OBFUSCATE && dir != SQOBFS_DEOBFUSCATE) return SQ_EINVAL;
  int st = check_batch_shape(hb, dir);
  if (st != SQ_OK || hb->n == 0) return st;
  const uint32_t n = hb->n;
  const int kind = kr->kind;
  const size_t S = salt_len(kind);
  // extents of the touched input / output ranges, and psk_id validation
  size_t in_ext = 0, out_ext = 0;
  for (uint32_t i = 0; i < n; i++) {
    const size_t len = hb->in_len[i];
    size_t cap = len;
    if (kind == SQOBFS_XPLUS && dir == SQOBFS_DEOBFUSCATE && hb->in_cap)
      cap = std::max<size_t>(len, hb->in_cap[i]);
    in_ext = std::max(in_ext, (size_t)hb->in_off[i] + cap);
    size_t osz;
    if (dir == SQOBFS_OBFUSCATE) osz = S + len;
    else if (kind == SQOBFS_SALAMANDER) osz = len <= S ? len : len - S;
    else osz = len < S ? 0 : cap - S;
    out_ext = std::max(out_ext, (size_t)hb->out_off[i] + osz);
    if (hb->psk_id && hb->psk_id[i] >= kr->count) return SQ_EPSK;
  }
  // one staging layout, mirrored in pinned host memory and on the device
  const size_t A = 256;
  size_t o = 0;
  const size_t o_in = o;       o = align_up(o + in_ext, A);
  const size_t o_out = o;      o = align_up(o + out_ext, A);
  const size_t o_inoff = o;    o = align_up(o + 8ull * n, A);
  const size_t o_inlen = o;    o = align_up(o + 4ull * n, A);
  const size_t o_outoff = o;   o = align_up(o + 8ull * n, A);
  const size_t o_outlen = o;   o = align_up(o + 4ull * n, A);
  const size_t o_salt = o;     o = align_up(o + (dir == SQOBFS_OBFUSCATE ? S * n : 0), A);
  const size_t o_pid = o;      o = align_up(o + (hb->psk_id ? 2ull * n : 0), A);
  const size_t o_cap = o;      o = align_up(o + (hb->in_cap ? 4ull * n : 0), A);
  const size_t total = o;

  std::lock_guard<std::mutex> lk(ctx->mu);
  SQ_TRY(hipSetDevice(ctx->device));
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
  uint8_t *H = ctx->pinned, *D = ctx->dev;
  if (in_ext) memcpy(H + o_in, hb->in, in_ext);
  if (out_ext) memcpy(H + o_out, hb->out, out_ext);  // preserve untouched bytes
  memcpy(H + o_inoff, hb->in_off, 8ull * n);
  memcpy(H + o_inlen, hb->in_len, 4ull * n);
  memcpy(H + o_outoff, hb->out_off, 8ull * n);
  if (dir == SQOBFS_OBFUSCATE) memcpy(H + o_salt, hb->salt, S * n);
  if (hb->psk_id) memcpy(H + o_pid, hb->psk_id, 2ull * n);
  if (hb->in_cap) memcpy(H + o_cap, hb->in_cap, 4ull * n);
  SQ_TRY(hipMemcpyAsync(D, H, total, hipMemcpyHostToDevice, ctx->stream));
  sqobfs_batch db = *hb;
  db.in = D + o_in;
  db.in_off = (const uint64_t *)(D + o_inoff);
  db.in_len = (const uint32_t *)(D + o_inlen);
  db.out = D + o_out;
  db.out_off = (const uint64_t *)(D + o_outoff);
  db.out_len = (uint32_t *)(D + o_outlen);
  db.salt = dir == SQOBFS_OBFUSCATE ? D + o_salt : nullptr;
  db.psk_id = hb->psk_id ? (const uint16_t *)(D + o_pid) : nullptr;
  db.in_cap = hb->in_cap ? (const uint32_t *)(D + o_cap) : nullptr;
  const sq::KParams kp = make_params(kr, &db);
  st = sq_launch_obfs(kind, dir, &kp, ctx->stream);
  if (st != SQ_OK) return st;
  SQ_TRY(hipMemcpyAsync(H + o_out, D + o_out, out_ext, hipMemcpyDeviceToHost, ctx->stream));
  SQ_TRY(hipMemcpyAsync(H + o_outlen, D + o_outlen, 4ull * n, hipMemcpyDeviceToHost,
                        ctx->stream));
  SQ_TRY(hipStreamSynchronize(ctx->stream));
  if (out_ext) memcpy(hb->out, H + o_out, out_ext);
  memcpy(hb->out_len, H + o_outlen, 4ull * n);
  return SQ_OK;
}

}  // extern "C"
