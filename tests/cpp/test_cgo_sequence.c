/* Replays, in C, the exact libsqobfs call sequence and memory ownership of
 * the Go binding's Slots (go/sqobfs/sqobfs.go; its Conn drives the engine
 * tested by tests/cpp/test_pconn.c) -- the Go code
 * cannot be compiled here (no Go toolchain), so this pins what it does:
 *
 *   Open            sqobfs_open
 *   NewKeyring      malloc'd private PSK copy + malloc'd off/len ->
 *                   sqobfs_keyring_create -> free all three
 *   NewSlots        sqobfs_host_alloc(2*cap*slot) (pinned: in slots, then
 *                   out slots); calloc'd sqobfs_batch; malloc'd in_off,
 *                   out_off, in_len, out_len, in_cap, salt; offsets filled
 *   WriteTo x k     payload copied into In(i), SetLen
 *   Run             Slots.Run(Obfuscate, n, deviceSalt): b->n, flags =
 *                   OUT_UNINIT | OUT_LINES (128-byte-multiple slots) or
 *                   OUT_BLOCKS (16-byte multiples) | DEVICE_SALT, in_cap = NULL ->
 *                   sqobfs_run_host
 *   reader          datagrams copied into In(i) of another Slots, SetLen ->
 *                   Slots.Run(Deobfuscate) -> Out(i)[:out_len[i]]
 *   Free / Close    free every array, the batch, sqobfs_host_free,
 *                   sqobfs_keyring_destroy, sqobfs_close
 *
 * The wire is checked with the oracle's restated ReadFrom (salamander.go:
 * 42-55, xplus.go:46-60): the GPU draws the salts, so decoding is the check.
 * Build: tests/test_host_mirror.py (gcc, -lsqobfs -loracle). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "sqobfs.h"

#define FAIL(...)                                 \
  do {                                            \
    fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
    fprintf(stderr, __VA_ARGS__);                 \
    fputc('\n', stderr);                          \
    exit(1);                                      \
  } while (0)
#define CHECK(x) \
  do {           \
    int st_ = (x); \
    if (st_ != SQ_OK) FAIL("%s -> %d (%s)", #x, st_, sqobfs_strerror(st_)); \
  } while (0)

typedef struct {
  sqobfs_ctx *ctx;
  int cap, slot;
  uint8_t *data; /* pinned: cap in slots, then cap out slots */
  sqobfs_batch *b;
  uint64_t *in_off, *out_off;
  uint32_t *in_len, *out_len, *in_cap;
  uint8_t *salt;
} Slots;

static sqobfs_keyring *new_keyring(sqobfs_ctx *ctx, int kind, const uint8_t *psk, size_t n) {
  uint8_t *blob = malloc(n + 1);
  memcpy(blob, psk, n);
  uint64_t *off = malloc(8);
  uint32_t *ln = malloc(4);
  *off = 0;
  *ln = (uint32_t)n;
  sqobfs_keyring *kr = NULL;
  CHECK(sqobfs_keyring_create(ctx, kind, 1, blob, off, ln, &kr));
  free(blob);  /* Go: deferred frees, after the call returned */
  free(off);
  free(ln);
  return kr;
}

static Slots new_slots(sqobfs_ctx *ctx, int cap, int slot) {
  Slots s = {ctx, cap, slot};
  void *p = NULL;
  CHECK(sqobfs_host_alloc(ctx, (size_t)2 * cap * slot, &p));
  s.data = p;
  s.b = calloc(1, sizeof(sqobfs_batch));
  s.in_off = malloc(8 * (size_t)cap);
  s.out_off = malloc(8 * (size_t)cap);
  s.in_len = malloc(4 * (size_t)cap);
  s.out_len = malloc(4 * (size_t)cap);
  s.in_cap = malloc(4 * (size_t)cap);
  s.salt = malloc(16 * (size_t)cap);
  for (int i = 0; i < cap; i++) {
    s.in_off[i] = (uint64_t)i * slot;
    s.out_off[i] = (uint64_t)(cap + i) * slot;
  }
  s.b->in = s.data;
  s.b->out = s.data;
  s.b->in_off = s.in_off;
  s.b->in_len = s.in_len;
  s.b->out_off = s.out_off;
  s.b->out_len = s.out_len;
  s.b->salt = s.salt;
  return s;
}

static uint8_t *in_slot(Slots *s, int i) { return s->data + (size_t)i * s->slot; }
static uint8_t *out_slot(Slots *s, int i) { return s->data + (size_t)(s->cap + i) * s->slot; }

static int run(Slots *s, const sqobfs_keyring *kr, int dir, int n, int device_salt) {
  s->b->n = (uint32_t)n;
  /* Slots.Run: output slots are read only up to out_len (OUT_UNINIT), and
   * 128-byte-multiple slots own their last lines (OUT_LINES), 16-byte
   * multiples their blocks (OUT_BLOCKS) */
  s->b->flags = SQOBFS_FLAG_OUT_UNINIT |
                (s->slot % 128 == 0   ? SQOBFS_FLAG_OUT_LINES
                 : s->slot % 16 == 0 ? SQOBFS_FLAG_OUT_BLOCKS
                                     : 0u) |
                ((dir == SQOBFS_OBFUSCATE && device_salt) ? SQOBFS_FLAG_DEVICE_SALT : 0u);
  s->b->in_cap = NULL;
  return sqobfs_run_host(s->ctx, kr, dir, s->b);
}

static void free_slots(Slots *s) {
  free(s->in_off);
  free(s->out_off);
  free(s->in_len);
  free(s->out_len);
  free(s->in_cap);
  free(s->salt);
  free(s->b);
  sqobfs_host_free(s->ctx, s->data);
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)rng_state;
}

static void one_kind(sqobfs_ctx *ctx, int kind) {
  const uint8_t psk[] = "sing-quic-mi355x-bench-psk";
  const size_t pl = sizeof psk - 1;
  const int S = kind == SQOBFS_SALAMANDER ? 8 : 16;
  const int cap = 256, slot = 2048;
  sqobfs_keyring *kr = new_keyring(ctx, kind, psk, pl);
  Slots tx = new_slots(ctx, cap, slot), rx = new_slots(ctx, cap, slot);
  static uint8_t payload[256][2048];
  for (int round = 0; round < 3; round++) {
    const int n = round == 0 ? cap : 1 + (int)(rnd() % cap);  /* full and linger-flushed batches */
    /* WriteTo x n: copy payloads into the transmit slots */
    for (int i = 0; i < n; i++) {
      const int L = (int)(rnd() % (slot - S + 1));
      for (int j = 0; j < L; j++) payload[i][j] = (uint8_t)rnd();
      memcpy(in_slot(&tx, i), payload[i], (size_t)L);
      tx.in_len[i] = (uint32_t)L;
    }
    CHECK(run(&tx, kr, SQOBFS_OBFUSCATE, n, 1));
    /* the wire: decodes with the reference's ReadFrom to the payload */
    for (int i = 0; i < n; i++) {
      const uint32_t w = tx.out_len[i];
      if (w != tx.in_len[i] + (uint32_t)S) FAIL("kind %d out_len %u for len %u", kind, w, tx.in_len[i]);
      uint8_t buf[4096];
      memcpy(buf, out_slot(&tx, i), w);
      const long m = kind == SQOBFS_SALAMANDER ? or_salamander_read(psk, pl, buf, w)
                                               : or_xplus_read(psk, pl, buf, w, w);
      if (m != (long)tx.in_len[i] || memcmp(buf, payload[i], (size_t)m))
        FAIL("kind %d packet %d does not decode", kind, i);
      /* the reader: this datagram arrives; plus a short one every 16 */
      memcpy(in_slot(&rx, i), out_slot(&tx, i), w);
      rx.in_len[i] = w;
      if (i % 16 == 15) rx.in_len[i] = (uint32_t)(rnd() % (unsigned)(S + 1));
    }
    CHECK(run(&rx, kr, SQOBFS_DEOBFUSCATE, n, 0));
    for (int i = 0; i < n; i++) {
      uint8_t ref[4096];
      const uint32_t dn = rx.in_len[i];
      memcpy(ref, in_slot(&rx, i), dn);
      const long m = kind == SQOBFS_SALAMANDER ? or_salamander_read(psk, pl, ref, dn)
                                               : or_xplus_read(psk, pl, ref, dn, dn);
      if ((long)rx.out_len[i] != m) FAIL("kind %d packet %d: out_len %u want %ld", kind, i, rx.out_len[i], m);
      if (m && memcmp(out_slot(&rx, i), ref, (size_t)m)) FAIL("kind %d packet %d payload", kind, i);
    }
  }
  free_slots(&tx);
  free_slots(&rx);
  sqobfs_keyring_destroy(kr);
}

int main(void) {
  sqobfs_ctx *ctx = NULL;
  CHECK(sqobfs_open(0, &ctx));
  one_kind(ctx, SQOBFS_SALAMANDER);
  one_kind(ctx, SQOBFS_XPLUS);
  sqobfs_close(ctx);
  printf("ok: cgo call sequence replayed (Salamander + XPlus, device salts, short datagrams)\n");
  return 0;
}
