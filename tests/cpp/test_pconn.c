/* Threaded tests of the obfuscating packet conn engine (sqobfs_pconn_*, the
 * core under go/sqobfs.Conn) over loopback UDP, checked against the oracle's
 * restatement of the reference decorators (oracle/oracle.c:
 * SalamanderPacketConn / XPlusPacketConn ReadFrom / WriteTo,
 * hysteria2/salamander.go:42-93, hysteria/xplus.go:46-98).
 *
 *   wire      socket mode: every datagram written is, byte for byte, the
 *             reference's WriteTo output for its (device) salt
 *   read      socket mode: every datagram a peer sends (oracle-obfuscated,
 *             short, cut by a small read buffer) reads back exactly as the
 *             reference's ReadFrom returns it
 *   roundtrip two pconns talking to each other, concurrent reader
 *   deadline  a deadline set while ReadFrom blocks unblocks it with
 *             SQ_ETIMEDOUT; a passed deadline fails at once, even with data
 *             queued (net.Conn semantics); clearing it restores reads
 *   shutdown  a blocked ReadFrom returns SQ_ECLOSED; Close with every
 *             receive batch full and no reader returns promptly; writes
 *             queued before Close still go out
 *   pump      the generic-PacketConn mode (tx_take / rx_push) with tags
 *   memory    every batch block is back in the engine's pool after every
 *             Close, and sqobfs_host_alloc blocks balance once it is trimmed
 *   syncerr   an inline write returns its own send error (the reference's
 *             WriteTo); with inline writes off, the next write reports it
 *   shared    8 pconns on one context: one engine (threads flat), blocks
 *             taken only while datagrams are in flight, wire == reference
 *   routing   small batches on the CPU path, bursts on the GPU
 *   fail      injected launch failures: a refused launch is redone on the
 *             CPU, a failed kernel's batch is dropped, and every datagram
 *             after either still reads / writes as the reference's
 *   load      the default routing under sustained load: bursts of <= 64
 *             datagrams stay on the CPU path; bulk traffic (the engine's
 *             transform demand above a tenth of a core) turns the load mode
 *             on, and then a batch of more than 64 launches when its
 *             CPU-path time exceeds a launch's measured host cost; every
 *             sampled wire datagram == the reference's WriteTo
 *   group     coalesced launches: the queued batches of six pconns with four
 *             PSKs go out in one launch per direction, every datagram the
 *             reference's under its own conn's PSK; with coalescing off, one
 *             launch per batch; and eight conns with writer, taker, pusher
 *             and reader threads on four workers (stress)
 *   poolfail  a receive batch block that cannot be allocated (with nothing
 *             unread to restart the socket task) is retried: the datagram
 *             still reads, within its deadline
 * Modes (argv[1]): "gpu" (default: a context on GPU 0; with the CPU device
 * of tests/cpp/sq_devstub.cpp in the sanitizer builds) and "nodev" (no
 * context: host keyrings, every batch on the CPU path -- the drop-in with no
 * GPU at all).
 * Build and run: tests/test_pconn.py (gcc, -lsqobfs -loracle -lpthread). */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "oracle.h"
#include "sqobfs.h"

#define FAIL(...)                                            \
  do {                                                       \
    fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);     \
    fprintf(stderr, __VA_ARGS__);                            \
    fputc('\n', stderr);                                     \
    exit(1);                                                 \
  } while (0)
#define CHECK(x)                                                           \
  do {                                                                     \
    int st_ = (x);                                                         \
    if (st_ != SQ_OK) FAIL("%s -> %d (%s)", #x, st_, sqobfs_strerror(st_)); \
  } while (0)
#define EXPECT(c, ...) \
  do {                 \
    if (!(c)) FAIL(__VA_ARGS__); \
  } while (0)

static const uint8_t PSK[] = "sing-quic-mi355x-bench-psk";
#define PL (sizeof PSK - 1)
#define MAXW 4096

static sqobfs_ctx *g_ctx; /* NULL: nodev mode */
static int g_nodev;
/* the async pass: every batch launches and waits without polling, so the
 * engine's completer lands it and finishes it (pump) or hands it back to a
 * worker (socket mode) while the launching worker goes on */
static int g_async;
static void async_opts(sqobfs_pconn_opts *o) {
  if (!g_async) return;
  o->cpu_max = SQOBFS_PCONN_NEVER;
  o->spin_us = SQOBFS_PCONN_NEVER;
  o->inline_gap_us = SQOBFS_PCONN_NEVER;
}

/* every block back in the engine's pool; trimmed, the pinned allocations
 * balance */
static void check_mem(int64_t a0) {
  sqobfs_engine_info info;
  CHECK(sqobfs_engine_info_get(g_ctx, &info));
  EXPECT(info.blocks_in_use == 0, "%u batch blocks still in use", info.blocks_in_use);
  sqobfs_engine_trim(g_ctx);
  EXPECT(sqobfs_debug_host_allocs() == a0, "host allocs %lld -> %lld", (long long)a0,
         (long long)sqobfs_debug_host_allocs());
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static int64_t unix_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}
static void sleep_ms(int ms) {
  struct timespec ts = {ms / 1000, (long)(ms % 1000) * 1000000};
  nanosleep(&ts, NULL);
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)rng_state;
}

static int udp_socket(uint16_t *port) {
  int fd = socket(AF_INET, SOCK_DGRAM, 0);
  if (fd < 0) FAIL("socket: %s", strerror(errno));
  int big = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
  struct sockaddr_in a;
  memset(&a, 0, sizeof a);
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(fd, (struct sockaddr *)&a, sizeof a)) FAIL("bind: %s", strerror(errno));
  socklen_t sl = sizeof a;
  getsockname(fd, (struct sockaddr *)&a, &sl);
  *port = ntohs(a.sin_port);
  return fd;
}

static sqobfs_addr loop_addr(uint16_t port) {
  sqobfs_addr x;
  memset(&x, 0, sizeof x);
  x.family = AF_INET;
  x.port = port;
  x.addr[0] = 127;
  x.addr[3] = 1;
  return x;
}

static void send_to(int fd, uint16_t port, const uint8_t *p, size_t n) {
  struct sockaddr_in a;
  memset(&a, 0, sizeof a);
  a.sin_family = AF_INET;
  a.sin_port = htons(port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (sendto(fd, p, n, 0, (struct sockaddr *)&a, sizeof a) != (ssize_t)n)
    FAIL("sendto: %s", strerror(errno));
}

/* recv with a timeout: -1 on timeout */
static long recv_to(int fd, uint8_t *buf, size_t cap, int ms) {
  struct pollfd p = {fd, POLLIN, 0};
  if (poll(&p, 1, ms) <= 0) return -1;
  return recv(fd, buf, cap, 0);
}

static sqobfs_keyring *keyring(int kind) {
  uint64_t off = 0;
  uint32_t len = PL;
  sqobfs_keyring *kr = NULL;
  CHECK(sqobfs_keyring_create(g_ctx, kind, 1, PSK, &off, &len, &kr));
  return kr;
}

static int salt_len(int kind) { return kind == SQOBFS_SALAMANDER ? 8 : 16; }

/* the reference's WriteTo for this salt: wire must equal it byte for byte */
static long ref_write(int kind, const uint8_t *salt, const uint8_t *p, size_t n, uint8_t *wire) {
  return kind == SQOBFS_SALAMANDER ? or_salamander_write(PSK, PL, salt, p, n, wire)
                                   : or_xplus_write(PSK, PL, salt, p, n, wire);
}

/* the reference's ReadFrom of datagram w (w_len bytes) into a buffer of cap
 * bytes: returns its n, and p[0..n) */
static long ref_read(int kind, const uint8_t *w, size_t w_len, size_t cap, uint8_t *p) {
  const size_t m = w_len < cap ? w_len : cap;
  static uint8_t buf[MAXW + 64];
  memset(buf, 0, sizeof buf);
  memcpy(buf, w, m);
  long r = kind == SQOBFS_SALAMANDER ? or_salamander_read(PSK, PL, buf, m)
                                     : or_xplus_read(PSK, PL, buf, m, cap < MAXW ? cap : MAXW);
  if (r > 0) memcpy(p, buf, (size_t)r);
  return r;
}

static uint32_t pick_len(int i, int S, uint32_t slot) {
  static const uint32_t edge[] = {0, 1, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129};
  const uint32_t ne = sizeof edge / sizeof edge[0];
  if ((uint32_t)i < ne) return edge[i];
  if (i % 97 == 0) return slot - (uint32_t)S; /* the largest payload a slot takes */
  if (i % 5 == 0) return 1200 + rnd() % 253;  /* QUIC-sized */
  return rnd() % (slot - (uint32_t)S + 1);
}

/* ------------------------------------------------------------ wire */
typedef struct {
  int fd, n;
  uint8_t (*wire)[MAXW];
  long *wlen;
} PeerRx;

static void *peer_rx(void *arg) {
  PeerRx *r = arg;
  for (int i = 0; i < r->n; i++) {
    r->wlen[i] = recv_to(r->fd, r->wire[i], MAXW, 5000);
    if (r->wlen[i] < 0) {
      r->n = i;
      break;
    }
  }
  return NULL;
}

static void t_wire(int kind, uint32_t offload) {
  const int S = salt_len(kind), N = 1500;
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(kind);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  sqobfs_pconn *pc = NULL;
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.flags = offload;
  async_opts(&o);
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o, &pc));
  static uint8_t pay[1500][MAXW], wire[1500][MAXW];
  static uint32_t plen[1500];
  static long wlen[1500];
  PeerRx r = {fp, N, wire, wlen};
  pthread_t th;
  pthread_create(&th, NULL, peer_rx, &r);
  const sqobfs_addr to = loop_addr(pp);
  for (int i = 0; i < N; i++) {
    plen[i] = pick_len(i, S, 2048);
    if (offload && i % 3) plen[i] = 1300; /* runs of equal lengths: GSO messages */
    for (uint32_t j = 0; j < plen[i]; j++) pay[i][j] = (uint8_t)rnd();
    CHECK(sqobfs_pconn_write(pc, pay[i], plen[i], &to, (uint64_t)i));
    if (i % 200 == 199) sleep_ms(2); /* bursts with gaps: small and large batches */
  }
  pthread_join(th, NULL);
  EXPECT(r.n == N, "kind %d: peer got %d of %d datagrams", kind, r.n, N);
  for (int i = 0; i < N; i++) {
    EXPECT(wlen[i] == (long)plen[i] + S, "kind %d dgram %d: wire %ld for payload %u", kind, i,
           wlen[i], plen[i]);
    uint8_t ref[MAXW];
    ref_write(kind, wire[i], pay[i], plen[i], ref); /* its salt, the reference's bytes */
    EXPECT(!memcmp(ref, wire[i], (size_t)wlen[i]), "kind %d dgram %d: wire differs", kind, i);
  }
  sqobfs_pconn_stats st;
  for (int k = 0; k < 500; k++) { /* (a batch is counted after its send returns) */
    CHECK(sqobfs_pconn_stats_get(pc, &st));
    if (st.tx_datagrams == (uint64_t)N) break;
    sleep_ms(1);
  }
  EXPECT(st.tx_datagrams == (uint64_t)N, "tx_datagrams %llu", (unsigned long long)st.tx_datagrams);
  printf("  wire kind %d%s%s: %d datagrams in %llu batches (max %u), wire == reference\n", kind,
         offload ? " (GSO)" : "", g_async ? " [async]" : "", N, (unsigned long long)st.tx_batches,
         st.tx_max_batch);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ read */
static void t_read(int kind) {
  const int S = salt_len(kind), N = 1200;
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(kind);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  sqobfs_pconn *pc = NULL;
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.batch = 64; /* several batches per burst */
  async_opts(&o);
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o, &pc));
  static uint8_t wire[1200][MAXW];
  static uint32_t wl[1200];
  int sent = 0;
  for (int burst = 0; sent < N; burst++) {
    const int k = burst % 3 == 0 ? 1 : 1 + (int)(rnd() % 150);
    const int base = sent;
    for (int j = 0; j < k && sent < N; j++, sent++) {
      const int i = sent;
      if (i % 9 == 4) { /* short datagrams: n <= 8 (Salamander), n < 16 (XPlus) */
        wl[i] = rnd() % (uint32_t)(S + 3);
        for (uint32_t b = 0; b < wl[i]; b++) wire[i][b] = (uint8_t)rnd();
      } else {
        uint8_t salt[16], pay[MAXW];
        for (int b = 0; b < 16; b++) salt[b] = (uint8_t)rnd();
        const uint32_t L = pick_len(i, S, 2048);
        for (uint32_t b = 0; b < L; b++) pay[b] = (uint8_t)rnd();
        ref_write(kind, salt, pay, L, wire[i]);
        wl[i] = L + (uint32_t)S;
      }
      send_to(fp, pa, wire[i], wl[i]);
    }
    /* read the burst back with varying buffer sizes (len(p)) */
    for (int i = base; i < sent; i++) {
      uint32_t cap = 4096;
      if (i % 13 == 6) cap = 1 + rnd() % 40;     /* cut inside / near the salt */
      else if (i % 11 == 3) cap = 64 + rnd() % 600;
      uint8_t got[MAXW], ref[MAXW];
      uint32_t n = 0;
      sqobfs_addr from;
      uint64_t tag;
      CHECK(sqobfs_pconn_read(pc, got, cap, &n, &from, &tag));
      const long want = ref_read(kind, wire[i], wl[i], cap, ref);
      EXPECT((long)n == want, "kind %d dgram %d (wire %u, cap %u): n %u want %ld", kind, i, wl[i],
             cap, n, want);
      EXPECT(!n || !memcmp(got, ref, n), "kind %d dgram %d: payload differs", kind, i);
      EXPECT(from.port == pp && from.family == AF_INET, "kind %d: source address", kind);
    }
  }
  sqobfs_pconn_stats st;
  CHECK(sqobfs_pconn_stats_get(pc, &st));
  printf("  read kind %d%s: %d datagrams in %llu batches (max %u), == reference ReadFrom\n", kind,
         g_async ? " [async]" : "", N, (unsigned long long)st.rx_batches, st.rx_max_batch);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ roundtrip */
typedef struct {
  sqobfs_pconn *pc;
  int kind, n, got, bad;
  uint32_t *plen;
  uint8_t (*pay)[2048];
} Reader;

static void *reader(void *arg) {
  Reader *r = arg;
  CHECK(sqobfs_pconn_set_deadline(r->pc, SQOBFS_PCONN_READ, unix_ns() + 5000000000ll));
  for (int i = 0; i < r->n; i++) {
    uint8_t buf[MAXW];
    uint32_t n;
    const int st = sqobfs_pconn_read(r->pc, buf, sizeof buf, &n, NULL, NULL);
    if (st != SQ_OK) break;
    if (r->kind == SQOBFS_SALAMANDER && r->plen[i] == 0) {
      /* an empty payload's datagram is the bare 8-byte salt, and
       * salamander.go:47-49 returns datagrams of n <= 8 as they are */
      if (n != 8) r->bad++;
    } else if (n != r->plen[i] || memcmp(buf, r->pay[i], n)) {
      r->bad++;
    }
    r->got++;
  }
  return NULL;
}

static void t_roundtrip(int kind, uint32_t offload) {
  const int S = salt_len(kind), N = 3000;
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(kind);
  uint16_t pa, pb;
  int fa = udp_socket(&pa), fb = udp_socket(&pb);
  sqobfs_pconn *A = NULL, *B = NULL;
  sqobfs_pconn_opts oa, ob;
  memset(&oa, 0, sizeof oa);
  memset(&ob, 0, sizeof ob);
  oa.flags = offload & SQOBFS_UDP_TX_GSO; /* A sends with GSO, B receives with GRO */
  ob.flags = offload & SQOBFS_UDP_RX_GRO;
  async_opts(&oa);
  async_opts(&ob);
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &oa, &A));
  CHECK(sqobfs_pconn_open(g_ctx, kr, fb, &ob, &B));
  static uint8_t pay[3000][2048];
  static uint32_t plen[3000];
  for (int i = 0; i < N; i++) {
    plen[i] = pick_len(i, S, 2048);
    if (offload && i % 4) plen[i] = 1350; /* equal-length runs: GSO out, GRO in */
    for (uint32_t j = 0; j < plen[i]; j++) pay[i][j] = (uint8_t)rnd();
  }
  Reader r = {B, kind, N, 0, 0, plen, pay};
  pthread_t th;
  pthread_create(&th, NULL, reader, &r);
  const sqobfs_addr to = loop_addr(pb);
  const double t0 = now_s();
  for (int i = 0; i < N; i++) {
    CHECK(sqobfs_pconn_write(A, pay[i], plen[i], &to, 0));
    if (i % 256 == 255) sleep_ms(1); /* stay inside the socket buffers */
  }
  pthread_join(th, NULL);
  const double dt = now_s() - t0;
  EXPECT(r.got == N && r.bad == 0, "kind %d roundtrip: got %d bad %d of %d", kind, r.got, r.bad, N);
  sqobfs_pconn_stats sa, sb;
  CHECK(sqobfs_pconn_stats_get(A, &sa));
  CHECK(sqobfs_pconn_stats_get(B, &sb));
  printf("  roundtrip kind %d%s%s: %d datagrams A -> B in %.1f ms (%llu tx / %llu rx batches, "
         "%llu on the CPU path)\n", kind, offload ? " (GSO -> GRO)" : "", g_async ? " [async]" : "",
         N, dt * 1e3, (unsigned long long)sa.tx_batches, (unsigned long long)sb.rx_batches,
         (unsigned long long)(sa.cpu_batches + sb.cpu_batches));
  if (g_async)
    EXPECT(sa.cpu_batches + sb.cpu_batches == 0, "async roundtrip: %llu batches on the CPU path",
           (unsigned long long)(sa.cpu_batches + sb.cpu_batches));
  sqobfs_pconn_close(A);
  sqobfs_pconn_close(B);
  close(fa);
  close(fb);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ deadlines */
typedef struct {
  sqobfs_pconn *pc;
  int st;
  double t;
} Blocked;

static void *blocked_read(void *arg) {
  Blocked *b = arg;
  uint8_t buf[MAXW];
  uint32_t n;
  const double t0 = now_s();
  b->st = sqobfs_pconn_read(b->pc, buf, sizeof buf, &n, NULL, NULL);
  b->t = now_s() - t0;
  return NULL;
}

static void t_deadline(void) {
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(SQOBFS_SALAMANDER);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  sqobfs_pconn *pc = NULL;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, NULL, &pc));
  /* 1. ReadFrom blocks; a deadline set meanwhile unblocks it */
  Blocked b = {pc, 1, 0};
  pthread_t th;
  pthread_create(&th, NULL, blocked_read, &b);
  sleep_ms(50);
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ, unix_ns() + 40 * 1000000ll));
  pthread_join(th, NULL);
  EXPECT(b.st == SQ_ETIMEDOUT, "blocked read returned %d, want SQ_ETIMEDOUT", b.st);
  EXPECT(b.t > 0.08 && b.t < 2.0, "blocked read took %.3f s", b.t);
  /* 2. a passed deadline fails at once, even with a datagram queued */
  uint8_t w[64], salt[8] = {1, 2, 3, 4, 5, 6, 7, 8}, p[32] = {9};
  ref_write(SQOBFS_SALAMANDER, salt, p, 32, w);
  send_to(fp, pa, w, 40);
  sleep_ms(50);
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ, unix_ns() - 1));
  uint8_t buf[MAXW];
  uint32_t n;
  double t0 = now_s();
  EXPECT(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL) == SQ_ETIMEDOUT,
         "passed deadline must fail");
  EXPECT(now_s() - t0 < 0.05, "passed deadline must fail at once");
  /* 3. cleared: the queued datagram reads */
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ, 0));
  CHECK(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL));
  EXPECT(n == 32 && !memcmp(buf, p, 32), "datagram after clearing the deadline");
  /* 4. write deadline (SetWriteDeadline): passed -> SQ_ETIMEDOUT, cleared -> ok */
  const sqobfs_addr to = loop_addr(pp);
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_WRITE, unix_ns() - 1));
  EXPECT(sqobfs_pconn_write(pc, p, 32, &to, 0) == SQ_ETIMEDOUT, "passed write deadline");
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ | SQOBFS_PCONN_WRITE, 0));
  CHECK(sqobfs_pconn_write(pc, p, 32, &to, 0));
  EXPECT(recv_to(fp, buf, sizeof buf, 2000) == 40, "write after clearing the deadline");
  /* 5. SetDeadline in the future does not disturb a read that completes */
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ, unix_ns() + 2000000000ll));
  send_to(fp, pa, w, 40);
  CHECK(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL));
  EXPECT(n == 32, "read under a future deadline");
  printf("  deadline: blocked ReadFrom unblocked after %.0f ms (deadline set at 50 + 40 ms)\n",
         b.t * 1e3);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ shutdown */
static void *shutdown_thread(void *arg) {
  sqobfs_pconn_shutdown((sqobfs_pconn *)arg);
  return NULL;
}

static void t_shutdown(void) {
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(SQOBFS_XPLUS);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  /* 1. Close wakes a blocked ReadFrom with SQ_ECLOSED */
  sqobfs_pconn *pc = NULL;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, NULL, &pc));
  Blocked b = {pc, 1, 0};
  pthread_t th;
  pthread_create(&th, NULL, blocked_read, &b);
  sleep_ms(30);
  double t0 = now_s();
  sqobfs_pconn_shutdown(pc);
  pthread_join(th, NULL);
  EXPECT(b.st == SQ_ECLOSED, "read after shutdown returned %d", b.st);
  EXPECT(now_s() - t0 < 1.0, "shutdown took %.3f s", now_s() - t0);
  uint8_t buf[MAXW];
  uint32_t n;
  EXPECT(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL) == SQ_ECLOSED, "read after close");
  const sqobfs_addr to = loop_addr(pp);
  EXPECT(sqobfs_pconn_write(pc, buf, 10, &to, 0) == SQ_ECLOSED, "write after close");
  sqobfs_pconn_close(pc);
  /* 2. Close while every receive batch is full and nobody reads */
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.batch = 32;
  o.rx_batches = 2;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o, &pc));
  uint8_t w[1216], salt[16] = {7}, p[1200] = {3};
  ref_write(SQOBFS_XPLUS, salt, p, 1200, w);
  for (int i = 0; i < 400; i++) send_to(fp, pa, w, sizeof w);
  sqobfs_pconn_stats st;
  for (int k = 0; k < 200; k++) {
    CHECK(sqobfs_pconn_stats_get(pc, &st));
    if (st.rx_batches >= 2) break; /* both receive batches ready, none read */
    sleep_ms(5);
  }
  EXPECT(st.rx_batches >= 2, "receive batches did not fill (%llu)",
         (unsigned long long)st.rx_batches);
  sleep_ms(20);
  t0 = now_s();
  sqobfs_pconn_close(pc);
  const double tc = now_s() - t0;
  EXPECT(tc < 1.0, "close with full receive batches took %.3f s", tc);
  /* drain the socket */
  while (recv_to(fa, buf, sizeof buf, 10) >= 0) {
  }
  /* 3. datagrams written just before Close still go out */
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, NULL, &pc));
  for (int i = 0; i < 100; i++) CHECK(sqobfs_pconn_write(pc, p, 1200, &to, 0));
  sqobfs_pconn_close(pc);
  int got = 0;
  while (recv_to(fp, buf, sizeof buf, 200) == 1216) got++;
  EXPECT(got == 100, "%d of 100 datagrams written before Close were sent", got);
  /* 4. two concurrent Close calls: neither cuts the other's drain short
   *    (the second call used to wake the workers early) */
  {
    sqobfs_pconn_opts o2;
    memset(&o2, 0, sizeof o2);
    o2.inline_gap_us = SQOBFS_PCONN_NEVER;
    CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o2, &pc));
    for (int i = 0; i < 300; i++) CHECK(sqobfs_pconn_write(pc, p, 1200, &to, 0));
    pthread_t t1, t2;
    pthread_create(&t1, NULL, shutdown_thread, pc);
    pthread_create(&t2, NULL, shutdown_thread, pc);
    pthread_join(t1, NULL);
    pthread_join(t2, NULL);
    sqobfs_pconn_close(pc);
    got = 0;
    while (recv_to(fp, buf, sizeof buf, 200) == 1216) got++;
    EXPECT(got == 300, "%d of 300 datagrams sent with two concurrent closes", got);
  }
  printf("  shutdown: blocked read -> SQ_ECLOSED; close with full rx batches %.1f ms; "
         "writes before close sent (also with two concurrent closes)\n", tc * 1e3);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ pump */
typedef struct {
  sqobfs_pconn *pc;
  int kind, count, bad;
  uint8_t (*pay)[2048];
  uint32_t *plen;
} Taker;

static void *taker(void *arg) {
  Taker *t = arg;
  for (;;) {
    sqobfs_pconn_tx v;
    const int st = sqobfs_pconn_tx_take(t->pc, 100, &v);
    if (st == SQ_ETIMEDOUT) continue;
    if (st != SQ_OK) break;
    for (uint32_t i = 0; i < v.count; i++) {
      const uint8_t *w = v.base + v.off[i];
      const uint64_t id = v.tag[i];
      uint8_t ref[MAXW];
      ref_write(t->kind, w, t->pay[id], t->plen[id], ref);
      if (v.len[i] != t->plen[id] + (uint32_t)salt_len(t->kind) || memcmp(ref, w, v.len[i]))
        t->bad++;
      t->count++;
    }
    CHECK(sqobfs_pconn_tx_done(t->pc));
  }
  return NULL;
}

static void t_pump(int kind) {
  const int S = salt_len(kind), N = 2000;
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(kind);
  sqobfs_pconn *pc = NULL;
  CHECK(sqobfs_pconn_open(g_ctx, kr, -1, NULL, &pc));
  static uint8_t pay[2000][2048];
  static uint32_t plen[2000];
  for (int i = 0; i < N; i++) {
    plen[i] = pick_len(i, S, 2048);
    for (uint32_t j = 0; j < plen[i]; j++) pay[i][j] = (uint8_t)rnd();
  }
  Taker t = {pc, kind, 0, 0, pay, plen};
  pthread_t th;
  pthread_create(&th, NULL, taker, &t);
  /* transmit: tags carry the caller's address handle */
  for (int i = 0; i < N; i++) CHECK(sqobfs_pconn_write(pc, pay[i], plen[i], NULL, (uint64_t)i));
  /* receive: pushed datagrams read back as the reference's ReadFrom */
  for (int i = 0; i < N; i++) {
    uint8_t salt[16], w[MAXW], got[MAXW], ref[MAXW];
    for (int b = 0; b < 16; b++) salt[b] = (uint8_t)rnd();
    ref_write(kind, salt, pay[i], plen[i], w);
    const uint32_t wl = (i % 17 == 5) ? (uint32_t)(rnd() % (unsigned)S) : plen[i] + (uint32_t)S;
    CHECK(sqobfs_pconn_rx_push(pc, w, wl, NULL, 1000000 + (uint64_t)i));
    uint32_t n;
    uint64_t tag;
    CHECK(sqobfs_pconn_read(pc, got, MAXW, &n, NULL, &tag));
    const long want = ref_read(kind, w, wl, MAXW, ref);
    EXPECT((long)n == want && (!n || !memcmp(got, ref, n)), "pump kind %d dgram %d", kind, i);
    EXPECT(tag == 1000000 + (uint64_t)i, "pump tag");
  }
  /* Close drains what was written (the taker still runs) */
  sqobfs_pconn_shutdown(pc);
  pthread_join(th, NULL);
  EXPECT(t.count == N && t.bad == 0, "pump kind %d: taken %d bad %d of %d", kind, t.count, t.bad, N);
  /* the wrapped conn failed: readers get its status */
  sqobfs_pconn_close(pc);
  CHECK(sqobfs_pconn_open(g_ctx, kr, -1, NULL, &pc));
  CHECK(sqobfs_pconn_rx_fail(pc, SQ_EIO, 1)); /* once: one reader sees it, reads go on */
  uint8_t buf[64], w[40], s8[16] = {5}, p8[32] = {6};
  uint32_t n;
  EXPECT(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL) == SQ_EIO, "rx_fail once");
  ref_write(kind, s8, p8, (size_t)(40 - S), w);
  CHECK(sqobfs_pconn_rx_push(pc, w, 40, NULL, 7));
  CHECK(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL));
  EXPECT(n == (uint32_t)(40 - S), "read after a once error");
  CHECK(sqobfs_pconn_rx_fail(pc, SQ_EIO, 0)); /* for good */
  EXPECT(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL) == SQ_EIO, "rx_fail status");
  EXPECT(sqobfs_pconn_read(pc, buf, sizeof buf, &n, NULL, NULL) == SQ_EIO, "rx_fail sticky");
  sqobfs_pconn_close(pc);
  printf("  pump kind %d: %d datagrams taken == reference WriteTo, %d pushed == ReadFrom\n", kind,
         N, N);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ syncerr */
static void t_syncerr(int kind) {
  const int S = salt_len(kind);
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(kind);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  const sqobfs_addr to = loop_addr(pp), bad = loop_addr(0); /* UDP to port 0: EINVAL */
  uint8_t p[100], w[MAXW], ref[MAXW];
  for (int i = 0; i < 100; i++) p[i] = (uint8_t)rnd();
  /* 1. inline (the default): the failing write itself returns the error, the
   *    next one is clean and its datagram is the reference's */
  sqobfs_pconn *pc = NULL;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, NULL, &pc));
  sleep_ms(2);
  int st = sqobfs_pconn_write(pc, p, 100, &bad, 0);
  EXPECT(st == SQOBFS_ERRNO(EINVAL), "kind %d: inline write to port 0 returned %d", kind, st);
  sleep_ms(2);
  CHECK(sqobfs_pconn_write(pc, p, 100, &to, 0));
  long n = recv_to(fp, w, sizeof w, 2000);
  EXPECT(n == 100 + S, "kind %d: inline datagram %ld", kind, n);
  ref_write(kind, w, p, 100, ref);
  EXPECT(!memcmp(ref, w, (size_t)n), "kind %d: inline wire differs", kind);
  sqobfs_pconn_stats sa;
  CHECK(sqobfs_pconn_stats_get(pc, &sa));
  EXPECT(sa.inline_writes == 2 && sa.tx_datagrams == 1, "inline stats %llu %llu",
         (unsigned long long)sa.inline_writes, (unsigned long long)sa.tx_datagrams);
  sqobfs_pconn_close(pc);
  /* 2. every write batched: the error of a sent batch is reported once, by
   *    the next write (which then queues nothing), and later writes work */
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.inline_gap_us = SQOBFS_PCONN_NEVER;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o, &pc));
  CHECK(sqobfs_pconn_write(pc, p, 100, &bad, 0));
  sleep_ms(50);
  st = sqobfs_pconn_write(pc, p, 100, &to, 0);
  EXPECT(st == SQOBFS_ERRNO(EINVAL), "kind %d: batched error reported by %d", kind, st);
  CHECK(sqobfs_pconn_write(pc, p, 100, &to, 0));
  n = recv_to(fp, w, sizeof w, 2000);
  EXPECT(n == 100 + S, "kind %d: batched datagram %ld", kind, n);
  EXPECT(recv_to(fp, w, sizeof w, 50) < 0, "the reporting write queued nothing");
  CHECK(sqobfs_pconn_stats_get(pc, &sa));
  EXPECT(sa.inline_writes == 0 && sa.tx_send_errors == 1, "batched stats");
  sqobfs_pconn_close(pc);
  printf("  syncerr kind %d: inline write -> its own EINVAL; batched -> the next write's\n", kind);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ shared */
typedef struct {
  sqobfs_pconn *pc;
  int kind, n, fp, bad, got;
  uint16_t port;
} Lane;

static void *lane_run(void *arg) {
  Lane *l = arg;
  const int S = salt_len(l->kind);
  const sqobfs_addr to = loop_addr(l->port);
  uint8_t p[1400], w[MAXW], ref[MAXW];
  for (int i = 0; i < l->n; i++) {
    const uint32_t L = 1 + (uint32_t)(i * 37 % 1399);
    for (uint32_t j = 0; j < L; j++) p[j] = (uint8_t)(i + j * 7 + l->port);
    CHECK(sqobfs_pconn_write(l->pc, p, L, &to, 0));
    const long n = recv_to(l->fp, w, sizeof w, 2000);
    if (n != (long)L + S) {
      l->bad++;
      continue;
    }
    ref_write(l->kind, w, p, L, ref);
    if (memcmp(ref, w, (size_t)n)) l->bad++;
    l->got++;
  }
  return NULL;
}

static void t_shared(void) {
  enum { K = 8, N = 300 };
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr[2] = {keyring(0), keyring(1)};
  sqobfs_pconn *one = NULL;
  uint16_t p1;
  int f1 = udp_socket(&p1);
  CHECK(sqobfs_pconn_open(g_ctx, kr[0], f1, NULL, &one));
  sqobfs_engine_info i1, i8, iend, peak;
  CHECK(sqobfs_engine_info_get(g_ctx, &i1));
  Lane ln[K];
  int fa[K];
  pthread_t th[K];
  for (int k = 0; k < K; k++) {
    uint16_t pa;
    fa[k] = udp_socket(&pa);
    ln[k].fp = udp_socket(&ln[k].port);
    ln[k].kind = k % 2;
    ln[k].n = N;
    ln[k].bad = ln[k].got = 0;
    sqobfs_pconn_opts o;
    memset(&o, 0, sizeof o);
    o.inline_gap_us = SQOBFS_PCONN_NEVER; /* through the engine's workers */
    CHECK(sqobfs_pconn_open(g_ctx, kr[k % 2], fa[k], &o, &ln[k].pc));
  }
  CHECK(sqobfs_engine_info_get(g_ctx, &i8));
  for (int k = 0; k < K; k++) pthread_create(&th[k], NULL, lane_run, &ln[k]);
  for (int k = 0; k < K; k++) pthread_join(th[k], NULL);
  CHECK(sqobfs_engine_info_get(g_ctx, &peak));
  for (int k = 0; k < K; k++) {
    EXPECT(ln[k].got == N && ln[k].bad == 0, "shared conn %d: got %d bad %d", k, ln[k].got,
           ln[k].bad);
    sqobfs_pconn_close(ln[k].pc);
    close(fa[k]);
    close(ln[k].fp);
  }
  CHECK(sqobfs_engine_info_get(g_ctx, &iend));
  EXPECT(i8.pconns == i1.pconns + (uint32_t)K, "pconns %u -> %u", i1.pconns, i8.pconns);
  /* workers + the poller, + the completer on a context */
  EXPECT(i8.threads == i1.threads && i8.threads == i1.workers + 1 + (g_ctx ? 1u : 0u),
         "threads %u with 1 conn, %u with 9 (workers %u)", i1.threads, i8.threads, i1.workers);
  EXPECT(peak.pool_blocks <= 2 * (uint32_t)K + 2, "pool grew to %u blocks for %d conns",
         peak.pool_blocks, K);
  EXPECT(iend.blocks_in_use == 0, "blocks in use after close: %u", iend.blocks_in_use);
  printf("  shared: 9 conns on one engine: %u threads (as with 1), pool %u blocks (%.1f MiB) "
         "after %d x %d datagrams, wire == reference\n", i8.threads, peak.pool_blocks,
         peak.pool_bytes / 1048576.0, K, N);
  sqobfs_pconn_close(one);
  close(f1);
  sqobfs_keyring_destroy(kr[0]);
  sqobfs_keyring_destroy(kr[1]);
  check_mem(a0);
}

/* ------------------------------------------------------------ routing */
static void t_routing(void) {
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(SQOBFS_SALAMANDER);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  sqobfs_pconn *pc = NULL;
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.inline_gap_us = SQOBFS_PCONN_NEVER;
  o.cpu_max = 65536; /* a fixed threshold here; the measured default below */
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o, &pc));
  const sqobfs_addr to = loop_addr(pp);
  static uint8_t pay[2000][1400];
  uint8_t w[MAXW], ref[MAXW];
  /* lone datagrams: CPU batches */
  for (int i = 0; i < 5; i++) {
    for (int j = 0; j < 1350; j++) pay[i][j] = (uint8_t)rnd();
    CHECK(sqobfs_pconn_write(pc, pay[i], 1350, &to, 0));
    EXPECT(recv_to(fp, w, sizeof w, 2000) == 1358, "lone datagram");
    ref_write(0, w, pay[i], 1350, ref);
    EXPECT(!memcmp(ref, w, 1358), "lone datagram wire");
  }
  sqobfs_pconn_stats a;
  for (int k = 0; k < 200; k++) { /* (the worker counts a batch after its send) */
    CHECK(sqobfs_pconn_stats_get(pc, &a));
    if (a.tx_datagrams == 5) break;
    sleep_ms(1);
  }
  EXPECT(a.cpu_batches == 5 && a.tx_batches == 5, "lone datagrams: %llu CPU of %llu batches",
         (unsigned long long)a.cpu_batches, (unsigned long long)a.tx_batches);
  /* a burst: batches grow past cpu_max and launch */
  for (int i = 0; i < 2000; i++) {
    for (int j = 0; j < 1350; j += 8) pay[i][j] = (uint8_t)rnd();
    CHECK(sqobfs_pconn_write(pc, pay[i], 1350, &to, 0));
  }
  int got = 0, bad = 0;
  for (int i = 0; i < 2000; i++) {
    const long n = recv_to(fp, w, sizeof w, 2000);
    if (n < 0) break;
    ref_write(0, w, pay[i], 1350, ref);
    if (n != 1358 || memcmp(ref, w, 1358)) bad++;
    got++;
  }
  sqobfs_pconn_stats b;
  for (int k = 0; k < 200; k++) {
    CHECK(sqobfs_pconn_stats_get(pc, &b));
    if (b.tx_datagrams == 2005) break;
    sleep_ms(1);
  }
  EXPECT(got == 2000 && bad == 0, "burst: got %d bad %d", got, bad);
  const uint64_t gpu = (b.tx_batches - a.tx_batches) - (b.cpu_batches - a.cpu_batches);
  EXPECT(gpu > 0, "the burst never launched (%llu batches, max %u)",
         (unsigned long long)(b.tx_batches - a.tx_batches), b.tx_max_batch);
  printf("  routing: 5 lone datagrams -> 5 CPU batches; a 2000-datagram burst -> %llu batches "
         "(%llu on the GPU, max %u)\n", (unsigned long long)(b.tx_batches - a.tx_batches),
         (unsigned long long)gpu, b.tx_max_batch);
  /* the measured break-even (cpu_max 0): within its bounds, from the
   * engine's launch round trip and CPU-path rate */
  sqobfs_engine_info ei;
  CHECK(sqobfs_engine_info_get(g_ctx, &ei));
  EXPECT(ei.route_bytes >= (16u << 10) && ei.route_bytes <= (4u << 20) && ei.launch_us > 0 &&
             ei.cpu_ns_per_kib > 0,
         "route %llu B (launch %u us, cpu %u ns/KiB)", (unsigned long long)ei.route_bytes,
         ei.launch_us, ei.cpu_ns_per_kib);
  printf("  measured break-even: %llu B (launch %u us, CPU path %u ns per KiB of cost)\n",
         (unsigned long long)ei.route_bytes, ei.launch_us, ei.cpu_ns_per_kib);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ load */
typedef struct {
  int fd;
  int stop; /* (atomic accesses) */
  long got, checked, bad;
} LoadPeer;

/* payload of datagram seq: its number, then bytes derived from it */
static void load_payload(uint32_t seq, uint8_t *p) {
  memcpy(p, &seq, 4);
  for (uint32_t j = 4; j < 1350; j++) p[j] = (uint8_t)(seq * 31u + j);
}

static void *load_peer(void *arg) {
  LoadPeer *r = arg;
  enum { M = 64 };
  static uint8_t buf[M][MAXW];
  struct mmsghdr h[M];
  struct iovec iov[M];
  for (;;) {
    for (int j = 0; j < M; j++) {
      iov[j].iov_base = buf[j];
      iov[j].iov_len = MAXW;
      memset(&h[j], 0, sizeof h[j]);
      h[j].msg_hdr.msg_iov = &iov[j];
      h[j].msg_hdr.msg_iovlen = 1;
    }
    struct pollfd p = {r->fd, POLLIN, 0};
    if (poll(&p, 1, 20) <= 0) {
      if (__atomic_load_n(&r->stop, __ATOMIC_ACQUIRE)) break;
      continue;
    }
    const int m = recvmmsg(r->fd, h, M, MSG_DONTWAIT, NULL);
    for (int j = 0; j < m; j++) {
      r->got++;
      if ((r->got & 7) && r->got > 64) continue; /* decode one in 8 (oracle byte loops) */
      uint8_t got[MAXW], want[1350];
      const long n = ref_read(0, buf[j], h[j].msg_len, MAXW, got);
      uint32_t seq = 0;
      if (n == 1350) memcpy(&seq, got, 4);
      load_payload(seq, want);
      r->checked++;
      if (n != 1350 || memcmp(got, want, 1350)) r->bad++;
    }
  }
  return NULL;
}

static void t_load(void) {
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(SQOBFS_SALAMANDER);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  int huge = 64 << 20;
  setsockopt(fp, SOL_SOCKET, SO_RCVBUF, &huge, sizeof huge);
  sqobfs_pconn *pc = NULL;
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.batch = 1024;
  o.flags = SQOBFS_UDP_TX_GSO;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, &o, &pc));
  const sqobfs_addr to = loop_addr(pp);
  LoadPeer r = {fp, 0, 0, 0, 0};
  pthread_t th;
  pthread_create(&th, NULL, load_peer, &r);
  uint8_t pay[1350];
  uint32_t seq = 0;
  sqobfs_engine_info ei;
  /* 1. bursts of 64 with gaps: the CPU path */
  sqobfs_pconn_stats s0, s1, s2, s3;
  CHECK(sqobfs_pconn_stats_get(pc, &s0));
  /* the break-even route moves with the measured CPU rate (a sanitizer
   * build's CPU path is ~10x slower and jittery): the expectation below
   * holds for the lowest route the phase saw */
  uint64_t route = UINT64_MAX;
  for (int b = 0; b < 20; b++) {
    CHECK(sqobfs_engine_info_get(g_ctx, &ei));
    if (ei.route_bytes < route) route = ei.route_bytes;
    for (int j = 0; j < 64; j++, seq++) {
      load_payload(seq, pay);
      CHECK(sqobfs_pconn_write(pc, pay, 1350, &to, 0));
    }
    CHECK(sqobfs_engine_info_get(g_ctx, &ei));
    if (ei.route_bytes < route) route = ei.route_bytes;
    sleep_ms(3);
  }
  sleep_ms(20);
  CHECK(sqobfs_pconn_stats_get(pc, &s1));
  CHECK(sqobfs_engine_info_get(g_ctx, &ei));
  if (ei.route_bytes < route) route = ei.route_bytes;
  EXPECT(s1.tx_datagrams - s0.tx_datagrams == 1280, "bursts: %llu of 1280 sent",
         (unsigned long long)(s1.tx_datagrams - s0.tx_datagrams));
  if (route >= 64ull * (1350 + 1024) && s1.tx_max_batch <= 64)  /* (no bursts merged) */
    EXPECT(s1.cpu_batches - s0.cpu_batches == s1.tx_batches - s0.tx_batches,
           "bursts of 64: %llu of %llu batches on the CPU path (route %llu B, load %u)",
           (unsigned long long)(s1.cpu_batches - s0.cpu_batches),
           (unsigned long long)(s1.tx_batches - s0.tx_batches), (unsigned long long)route,
           ei.load_permille);
  /* 2. sustained: 0.5 s as fast as the writer goes */
  int loaded = 0;
  uint32_t pm_max = 0, ns_min = 0xFFFFFFFFu;
  const double t0 = now_s();
  while (now_s() - t0 < 0.5) {
    for (int j = 0; j < 256; j++, seq++) {
      load_payload(seq, pay);
      CHECK(sqobfs_pconn_write(pc, pay, 1350, &to, 0));
    }
    CHECK(sqobfs_engine_info_get(g_ctx, &ei));
    loaded |= (int)ei.loaded;
    if (ei.load_permille > pm_max) pm_max = ei.load_permille;
    if (ei.cpu_ns_per_kib < ns_min) ns_min = ei.cpu_ns_per_kib;
  }
  sleep_ms(50);
  CHECK(sqobfs_pconn_stats_get(pc, &s2));
  const uint64_t nb = s2.tx_batches - s1.tx_batches, nc = s2.cpu_batches - s1.cpu_batches;
  /* (the sanitizer builds' CPU path runs ~10x slower and their writer cannot
   * offer bulk load: there the load mode is not required to turn on) */
  CHECK(sqobfs_engine_info_get(g_ctx, &ei));
  const int slow = ei.cpu_ns_per_kib > 1500;
  EXPECT(loaded || slow, "sustained load never turned the engine's load mode on (peak %u permille)",
         pm_max);
  /* loaded, a batch of more than 64 launches when its CPU-path time exceeds
   * a launch's host cost: the phase's largest batch must have launched when
   * it clearly did (x1.5, and the CPU path's lowest rate seen in the phase:
   * the EWMAs move during the phase -- one GPU run saw 23 ns/KiB early and
   * 78 late, where a 652-datagram batch estimated at the late rate "should"
   * have launched; a slow, contended writer may never fill a batch past 64;
   * in the sanitizer builds the load mode may turn on only after the
   * largest batch went) */
  if (ns_min > ei.cpu_ns_per_kib) ns_min = ei.cpu_ns_per_kib;
  const double est_max = (double)s2.tx_max_batch * (1350 + 1024) * ns_min / 1024.0;
  EXPECT(nb > nc || !loaded || slow || s2.tx_max_batch <= 64 || est_max < 1.5 * ei.gpu_host_ns,
         "sustained load: no batch launched (%llu batches, max %u: est %.1f us of CPU path "
         "against %.1f us per launch)", (unsigned long long)nb, s2.tx_max_batch, est_max * 1e-3,
         ei.gpu_host_ns * 1e-3);
  /* 3. bursts again after the load: on the CPU path (n <= 64) */
  sleep_ms(30);
  for (int b = 0; b < 10; b++) {
    for (int j = 0; j < 64; j++, seq++) {
      load_payload(seq, pay);
      CHECK(sqobfs_pconn_write(pc, pay, 1350, &to, 0));
    }
    sleep_ms(3);
  }
  sleep_ms(20);
  CHECK(sqobfs_pconn_stats_get(pc, &s3));
  if (route >= 64ull * (1350 + 1024) && !slow)  /* (a slow worker can merge two bursts) */
    EXPECT(s3.cpu_batches - s2.cpu_batches == s3.tx_batches - s2.tx_batches,
           "bursts after the load: %llu of %llu batches on the CPU path",
           (unsigned long long)(s3.cpu_batches - s2.cpu_batches),
           (unsigned long long)(s3.tx_batches - s2.tx_batches));
  sleep_ms(100);
  __atomic_store_n(&r.stop, 1, __ATOMIC_RELEASE);
  pthread_join(th, NULL);
  EXPECT(r.bad == 0 && r.checked > 100, "load: %ld of %ld decoded datagrams differ", r.bad,
         r.checked);
  EXPECT(r.got >= (long)seq / 2, "load: only %ld of %u datagrams arrived", r.got, seq);
  printf("  load: bursts of 64 on the CPU path; sustained %u datagrams -> %llu batches (max %u), "
         "%llu launched (peak demand %u permille of a core, loaded %d; CPU path %u ns/KiB, "
         "launch %u ns of host CPU); %ld arrived, %ld decoded == reference\n", seq,
         (unsigned long long)nb, s2.tx_max_batch, (unsigned long long)(nb - nc), pm_max, loaded,
         ei.cpu_ns_per_kib, ei.gpu_host_ns, r.got, r.checked);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ poolfail */
static void t_poolfail(int kind) {
  const int S = salt_len(kind);
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr = keyring(kind);
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  sqobfs_pconn *pc = NULL;
  CHECK(sqobfs_pconn_open(g_ctx, kr, fa, NULL, &pc));
  for (int round = 0; round < 3; round++) {
    /* round 0: the first allocation fails; 1: the next 5 do; 2: none */
    sqobfs_debug_pool_fail(round == 0 ? 1 : round == 1 ? 5 : 0);
    uint8_t salt[16], pay[1400], w[MAXW], got[MAXW], ref[MAXW];
    for (int b = 0; b < 16; b++) salt[b] = (uint8_t)rnd();
    const uint32_t L = 100 + 600 * (uint32_t)round;
    for (uint32_t b = 0; b < L; b++) pay[b] = (uint8_t)rnd();
    ref_write(kind, salt, pay, L, w);
    send_to(fp, pa, w, L + (uint32_t)S);
    CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ, unix_ns() + 3000000000ll));
    uint32_t n = 0;
    const double t0 = now_s();
    const int st = sqobfs_pconn_read(pc, got, MAXW, &n, NULL, NULL);
    EXPECT(st == SQ_OK, "poolfail kind %d round %d: read -> %d after %.2f s (the receive side "
           "did not recover from the failed allocation)", kind, round, st, now_s() - t0);
    const long want = ref_read(kind, w, L + (uint32_t)S, MAXW, ref);
    EXPECT((long)n == want && !memcmp(got, ref, n), "poolfail kind %d round %d: payload", kind,
           round);
  }
  sqobfs_debug_pool_fail(0);
  CHECK(sqobfs_pconn_set_deadline(pc, SQOBFS_PCONN_READ, 0));
  printf("  poolfail kind %d: reads recover from failed batch-block allocations\n", kind);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
  sqobfs_keyring_destroy(kr);
  check_mem(a0);
}

/* ------------------------------------------------------------ fail */
/* On a context of its own (a failure turns its engine to the CPU for good).
 * at_completion 0: the launch is refused -> the batch is redone on the CPU;
 * 1: the kernel "faults" after running -> the batch is dropped. */
/* ------------------------------------------------------------ group */
/* the reference decorators for any PSK */
static long ref_write_psk(int kind, const uint8_t *psk, size_t pl, const uint8_t *salt,
                          const uint8_t *p, size_t n, uint8_t *wire) {
  return kind == SQOBFS_SALAMANDER ? or_salamander_write(psk, pl, salt, p, n, wire)
                                   : or_xplus_write(psk, pl, salt, p, n, wire);
}
static long ref_read_psk(int kind, const uint8_t *psk, size_t pl, const uint8_t *w, size_t wl,
                         uint8_t *p) {
  static uint8_t buf[MAXW + 64];
  memset(buf, 0, sizeof buf);
  memcpy(buf, w, wl);
  long r = kind == SQOBFS_SALAMANDER ? or_salamander_read(psk, pl, buf, wl)
                                     : or_xplus_read(psk, pl, buf, wl, MAXW);
  if (r > 0) memcpy(p, buf, (size_t)r);
  return r;
}

/* Coalesced launches (sqobfs_engine_set_group): six pump pconns -- three on
 * one keyring, three on keyrings of other PSKs (5 B, 130 B: a PSK-only
 * BLAKE2b block, and empty) -- queue a transmit and a receive batch each
 * while the engine's one worker is held; released, it launches the six
 * transmit batches as one launch and the six receive batches as another
 * (per-datagram PSK ids into the engine's merged keyring), and every
 * datagram is the reference's WriteTo / ReadFrom under its own conn's PSK.
 * Then with coalescing off (group 1) the same traffic takes a launch per
 * batch.  short_psks: the fifth conn's PSK is 12 B instead of 130, so every
 * PSK of the merged keyring fits the first compressed block (the multi-PSK
 * kernels then skip loading the chaining values: hot_iv). */
static void t_group(int kind, int short_psks) {
  enum { K = 6, N = 40 };
  const int S = salt_len(kind);
  sqobfs_ctx *ctx = NULL;
  CHECK(sqobfs_open(0, &ctx));
  CHECK(sqobfs_engine_set_workers(ctx, 1));
  const int64_t a0 = sqobfs_debug_host_allocs();
  static uint8_t long_psk[130];
  for (int i = 0; i < 130; i++) long_psk[i] = (uint8_t)(i * 29 + 3);
  static const uint8_t psk_b[] = "hop-b";
  const uint8_t *psk[K] = {PSK, PSK, PSK, psk_b, long_psk, NULL};
  const uint32_t pl[K] = {PL, PL, PL, 5, short_psks ? 12u : 130u, 0};
  sqobfs_keyring *kr[K];
  for (int k = 0; k < K; k++) {
    if (k == 1 || k == 2) {
      kr[k] = kr[0];
      continue;
    }
    uint64_t off = 0;
    uint32_t len = pl[k];
    static const uint8_t none = 0;
    CHECK(sqobfs_keyring_create(ctx, kind, 1, psk[k] ? psk[k] : &none, &off, &len, &kr[k]));
  }
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.cpu_max = SQOBFS_PCONN_NEVER; /* every batch launches */
  sqobfs_pconn *pc[K];
  for (int k = 0; k < K; k++) CHECK(sqobfs_pconn_open(ctx, kr[k], -1, &o, &pc[k]));
  static uint8_t pay[K][N][1400], wire[K][N][1500];
  static uint32_t plen[K][N], wlen[K][N];
  for (int round = 0; round < 2; round++) {
    if (round == 1) CHECK(sqobfs_engine_set_group(ctx, 1)); /* coalescing off */
    sqobfs_engine_info i0, i1;
    CHECK(sqobfs_engine_info_get(ctx, &i0));
    uint64_t ran0[K];
    for (int k = 0; k < K; k++) {
      sqobfs_pconn_stats st;
      CHECK(sqobfs_pconn_stats_get(pc[k], &st));
      ran0[k] = st.tx_batches + st.rx_batches;
    }
    sqobfs_debug_engine_hold(1);
    for (int k = 0; k < K; k++)
      for (int i = 0; i < N; i++) {
        plen[k][i] = (uint32_t)(i < 17 ? pick_len(i, S, 1400) : rnd() % 1385);
        for (uint32_t j = 0; j < plen[k][i]; j++) pay[k][i][j] = (uint8_t)rnd();
        CHECK(sqobfs_pconn_write(pc[k], pay[k][i], plen[k][i], NULL, (uint64_t)i));
      }
    for (int k = 0; k < K; k++)
      for (int i = 0; i < N; i++) {
        uint8_t salt[16];
        for (int b = 0; b < 16; b++) salt[b] = (uint8_t)rnd();
        ref_write_psk(kind, psk[k], pl[k], salt, pay[k][i], plen[k][i], wire[k][i]);
        wlen[k][i] = plen[k][i] + (uint32_t)S;
        CHECK(sqobfs_pconn_rx_push(pc[k], wire[k][i], wlen[k][i], NULL, (uint64_t)i));
      }
    sleep_ms(20);
    for (int k = 0; k < K; k++) {
      sqobfs_pconn_stats st;
      CHECK(sqobfs_pconn_stats_get(pc[k], &st));
      EXPECT(st.tx_batches + st.rx_batches == ran0[k], "group: conn %d ran while held", k);
    }
    sqobfs_debug_engine_hold(0);
    for (int k = 0; k < K; k++) {
      int got = 0;
      while (got < N) {
        sqobfs_pconn_tx v;
        CHECK(sqobfs_pconn_tx_take(pc[k], 5000, &v));
        for (uint32_t i = 0; i < v.count; i++, got++) {
          const uint8_t *w = v.base + v.off[i];
          const uint64_t id = v.tag[i];
          uint8_t ref[MAXW];
          EXPECT(id == (uint64_t)got && v.len[i] == plen[k][id] + (uint32_t)S,
                 "group kind %d conn %d: datagram %d len %u", kind, k, got, v.len[i]);
          ref_write_psk(kind, psk[k], pl[k], w, pay[k][id], plen[k][id], ref);
          EXPECT(!memcmp(ref, w, v.len[i]), "group kind %d conn %d: wire %d differs", kind, k, got);
        }
        CHECK(sqobfs_pconn_tx_done(pc[k]));
      }
      for (int i = 0; i < N; i++) {
        uint8_t got_p[MAXW], ref[MAXW];
        uint32_t n;
        uint64_t tag;
        CHECK(sqobfs_pconn_read(pc[k], got_p, MAXW, &n, NULL, &tag));
        const long want = ref_read_psk(kind, psk[k], pl[k], wire[k][i], wlen[k][i], ref);
        EXPECT(tag == (uint64_t)i && (long)n == want && (!n || !memcmp(got_p, ref, n)),
               "group kind %d conn %d: read %d", kind, k, i);
      }
      sqobfs_pconn_stats st;
      CHECK(sqobfs_pconn_stats_get(pc[k], &st));
      EXPECT(st.cpu_batches == 0 && st.gpu_failures == 0, "group conn %d: %llu CPU batches", k,
             (unsigned long long)st.cpu_batches);
    }
    CHECK(sqobfs_engine_info_get(ctx, &i1));
    const uint64_t gl = i1.group_launches - i0.group_launches;
    const uint64_t gb = i1.group_batches - i0.group_batches;
    const uint64_t nl = i1.launches - i0.launches;
    if (round == 0)
      EXPECT(gl == 2 && gb == 2 * K && nl == 2 && i0.group_max == 32,
             "group kind %d: %llu launches, %llu coalesced carrying %llu batches (want 2, 2, %d)",
             kind, (unsigned long long)nl, (unsigned long long)gl, (unsigned long long)gb, 2 * K);
    else
      EXPECT(gl == 0 && nl == 2 * K && i1.group_max == 1,
             "group off kind %d: %llu launches, %llu coalesced", kind, (unsigned long long)nl,
             (unsigned long long)gl);
    printf("  group kind %d (%s, PSKs of %u/5/%u/0 B): %d conns x %d datagrams each way in %llu "
           "launches, wire == reference WriteTo / ReadFrom\n", kind, round ? "off" : "on",
           (unsigned)PL, pl[4], K, N, (unsigned long long)nl);
  }
  for (int k = 0; k < K; k++) sqobfs_pconn_close(pc[k]);
  for (int k = 0; k < K; k++)
    if (k != 1 && k != 2) sqobfs_keyring_destroy(kr[k]);
  sqobfs_engine_trim(ctx);
  EXPECT(sqobfs_debug_host_allocs() == a0, "group: host allocs");
  sqobfs_close(ctx);
}

/* More PSKs than one merged keyring holds: 300 pump pconns, a
 * keyring of its own PSK each, queue two transmit and two receive datagrams
 * while the engine's one worker is held; released, the coalesced launches
 * (32 batches each) fill the merged keyring past its 256 entries, so the
 * engine starts a new one mid-traffic.  Every datagram is the reference's
 * under its own conn's PSK. */
static void t_many_psks(int kind) {
  enum { K = 300, N = 2 };
  const int S = salt_len(kind);
  sqobfs_ctx *ctx = NULL;
  CHECK(sqobfs_open(0, &ctx));
  CHECK(sqobfs_engine_set_workers(ctx, 1));
  const int64_t a0 = sqobfs_debug_host_allocs();
  static uint8_t psk[K][12];
  static sqobfs_keyring *kr[K];
  static sqobfs_pconn *pc[K];
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.cpu_max = SQOBFS_PCONN_NEVER; /* every batch launches */
  o.batch = 4;
  for (int k = 0; k < K; k++) {
    for (int b = 0; b < 12; b++) psk[k][b] = (uint8_t)(k * 7 + b * 131 + (k >> 8));
    uint64_t off = 0;
    uint32_t len = 12;
    CHECK(sqobfs_keyring_create(ctx, kind, 1, psk[k], &off, &len, &kr[k]));
    CHECK(sqobfs_pconn_open(ctx, kr[k], -1, &o, &pc[k]));
  }
  static uint8_t pay[K][N][1400], wire[K][N][1500];
  static uint32_t plen[K][N], wlen[K][N];
  sqobfs_engine_info i0, i1;
  CHECK(sqobfs_engine_info_get(ctx, &i0));
  sqobfs_debug_engine_hold(1);
  for (int k = 0; k < K; k++)
    for (int i = 0; i < N; i++) {
      plen[k][i] = (uint32_t)(rnd() % 1385);
      for (uint32_t j = 0; j < plen[k][i]; j++) pay[k][i][j] = (uint8_t)rnd();
      CHECK(sqobfs_pconn_write(pc[k], pay[k][i], plen[k][i], NULL, (uint64_t)i));
      uint8_t salt[16];
      for (int b = 0; b < 16; b++) salt[b] = (uint8_t)rnd();
      ref_write_psk(kind, psk[k], 12, salt, pay[k][i], plen[k][i], wire[k][i]);
      wlen[k][i] = plen[k][i] + (uint32_t)S;
      CHECK(sqobfs_pconn_rx_push(pc[k], wire[k][i], wlen[k][i], NULL, (uint64_t)i));
    }
  sqobfs_debug_engine_hold(0);
  for (int k = 0; k < K; k++) {
    int got = 0;
    while (got < N) {
      sqobfs_pconn_tx v;
      CHECK(sqobfs_pconn_tx_take(pc[k], 5000, &v));
      for (uint32_t i = 0; i < v.count; i++, got++) {
        const uint8_t *w = v.base + v.off[i];
        const uint64_t id = v.tag[i];
        uint8_t ref[MAXW];
        EXPECT(id == (uint64_t)got && v.len[i] == plen[k][id] + (uint32_t)S,
               "many PSKs kind %d conn %d: datagram %d len %u", kind, k, got, v.len[i]);
        ref_write_psk(kind, psk[k], 12, w, pay[k][id], plen[k][id], ref);
        EXPECT(!memcmp(ref, w, v.len[i]), "many PSKs kind %d conn %d: wire %d differs", kind, k,
               got);
      }
      CHECK(sqobfs_pconn_tx_done(pc[k]));
    }
    for (int i = 0; i < N; i++) {
      uint8_t got_p[MAXW], ref[MAXW];
      uint32_t n;
      uint64_t tag;
      CHECK(sqobfs_pconn_read(pc[k], got_p, MAXW, &n, NULL, &tag));
      const long want = ref_read_psk(kind, psk[k], 12, wire[k][i], wlen[k][i], ref);
      EXPECT(tag == (uint64_t)i && (long)n == want && (!n || !memcmp(got_p, ref, n)),
             "many PSKs kind %d conn %d: read %d", kind, k, i);
    }
    sqobfs_pconn_stats st;
    CHECK(sqobfs_pconn_stats_get(pc[k], &st));
    EXPECT(st.cpu_batches == 0 && st.gpu_failures == 0, "many PSKs conn %d: %llu CPU batches", k,
           (unsigned long long)st.cpu_batches);
  }
  CHECK(sqobfs_engine_info_get(ctx, &i1));
  const uint64_t gl = i1.group_launches - i0.group_launches;
  const uint64_t gb = i1.group_batches - i0.group_batches;
  EXPECT(gb >= K && gl * 32 >= gb && gl >= 2 * K / 32, "many PSKs kind %d: %llu coalesced "
         "launches carrying %llu batches", kind, (unsigned long long)gl, (unsigned long long)gb);
  printf("  many PSKs kind %d: %d conns of distinct PSKs, %llu coalesced launches carrying %llu "
         "batches, wire == reference\n", kind, K, (unsigned long long)gl, (unsigned long long)gb);
  for (int k = 0; k < K; k++) sqobfs_pconn_close(pc[k]);
  for (int k = 0; k < K; k++) sqobfs_keyring_destroy(kr[k]);
  sqobfs_engine_trim(ctx);
  EXPECT(sqobfs_debug_host_allocs() == a0, "many PSKs: host allocs");
  sqobfs_close(ctx);
}

/* Coalesced launches under concurrency: eight pump pconns (three PSKs, a
 * keyring each, as the Go adapters make them) on the default four workers,
 * each with a writer, a taker, a pusher and a reader thread; every batch
 * launches (cpu_max NEVER), so the workers grab each other's queued tasks
 * while all of them run.  Every datagram taken or read is the reference's
 * under its conn's PSK, none is lost.  (Under TSan: the grab against the
 * tasks' own scheduling.) */
enum { GS_K = 8, GS_N = 1500 };
static const uint8_t *gs_psk(int k, uint32_t *len) {
  static const uint8_t a[] = "hop-alpha", b[] = "a-longer-hop-psk-for-the-second-keyring-0123";
  switch (k % 3) {
    case 0: *len = PL; return PSK;
    case 1: *len = sizeof a - 1; return a;
    default: *len = sizeof b - 1; return b;
  }
}
static uint32_t gs_pay(int k, int i, uint8_t *p) {
  const uint32_t L = 1 + (uint32_t)(k * 131 + i * 37) % 1300;
  for (uint32_t j = 0; j < L; j++) p[j] = (uint8_t)(k * 7 + i * 13 + (int)j);
  return L;
}
typedef struct {
  sqobfs_pconn *pc;
  int kind, k, got, bad;
} GsArg;
static void *gs_writer(void *arg) {
  GsArg *g = arg;
  uint8_t p[1400];
  for (int i = 0; i < GS_N; i++) {
    const uint32_t L = gs_pay(g->k, i, p);
    CHECK(sqobfs_pconn_write(g->pc, p, L, NULL, (uint64_t)i));
  }
  return NULL;
}
static void *gs_taker(void *arg) {
  GsArg *g = arg;
  uint32_t pl;
  const uint8_t *psk = gs_psk(g->k, &pl);
  while (g->got < GS_N) {
    sqobfs_pconn_tx v;
    const int st = sqobfs_pconn_tx_take(g->pc, 5000, &v);
    if (st != SQ_OK) break;
    for (uint32_t i = 0; i < v.count; i++, g->got++) {
      uint8_t p[1400], ref[MAXW];
      const uint32_t L = gs_pay(g->k, (int)v.tag[i], p);
      const uint8_t *w = v.base + v.off[i];
      ref_write_psk(g->kind, psk, pl, w, p, L, ref);
      if (v.len[i] != L + (uint32_t)salt_len(g->kind) || memcmp(ref, w, v.len[i])) g->bad++;
    }
    CHECK(sqobfs_pconn_tx_done(g->pc));
  }
  return NULL;
}
static void *gs_pusher(void *arg) {
  GsArg *g = arg;
  uint32_t pl;
  const uint8_t *psk = gs_psk(g->k, &pl);
  for (int i = 0; i < GS_N; i++) {
    uint8_t p[1400], salt[16], w[MAXW];
    const uint32_t L = gs_pay(g->k, i, p);
    for (int b = 0; b < 16; b++) salt[b] = (uint8_t)(i * 31 + b + g->k);
    ref_write_psk(g->kind, psk, pl, salt, p, L, w);
    CHECK(sqobfs_pconn_rx_push(g->pc, w, L + (uint32_t)salt_len(g->kind), NULL, (uint64_t)i));
  }
  return NULL;
}
static void *gs_reader(void *arg) {
  GsArg *g = arg;
  /* (a lost datagram fails the count, within the deadline, not by a hang) */
  CHECK(sqobfs_pconn_set_deadline(g->pc, SQOBFS_PCONN_READ, unix_ns() + 120 * 1000000000ll));
  for (; g->got < GS_N; g->got++) {
    uint8_t got[MAXW], p[1400];
    uint32_t n;
    uint64_t tag;
    const int st = sqobfs_pconn_read(g->pc, got, MAXW, &n, NULL, &tag);
    if (st != SQ_OK) break;
    const uint32_t L = gs_pay(g->k, (int)tag, p);
    if (n != L || memcmp(got, p, L) || tag != (uint64_t)g->got) g->bad++;
  }
  return NULL;
}
static void t_group_stress(int kind, int no_poll) {
  sqobfs_ctx *ctx = NULL;
  CHECK(sqobfs_open(0, &ctx));
  const int64_t a0 = sqobfs_debug_host_allocs();
  sqobfs_keyring *kr[GS_K];
  sqobfs_pconn *pc[GS_K];
  sqobfs_pconn_opts o;
  memset(&o, 0, sizeof o);
  o.cpu_max = SQOBFS_PCONN_NEVER;
  o.batch = 64;
  /* no_poll: every launch lands on the completer, which finishes the
   * batches while the workers go on launching others */
  if (no_poll) o.spin_us = SQOBFS_PCONN_NEVER;
  for (int k = 0; k < GS_K; k++) {
    uint64_t off = 0;
    uint32_t len;
    const uint8_t *psk = gs_psk(k, &len);
    CHECK(sqobfs_keyring_create(ctx, kind, 1, psk, &off, &len, &kr[k]));
    CHECK(sqobfs_pconn_open(ctx, kr[k], -1, &o, &pc[k]));
  }
  GsArg ga[4][GS_K];
  pthread_t th[4][GS_K];
  void *(*fn[4])(void *) = {gs_writer, gs_taker, gs_pusher, gs_reader};
  for (int r = 0; r < 4; r++)
    for (int k = 0; k < GS_K; k++) {
      ga[r][k] = (GsArg){pc[k], kind, k, 0, 0};
      pthread_create(&th[r][k], NULL, fn[r], &ga[r][k]);
    }
  for (int r = 0; r < 4; r++)
    for (int k = 0; k < GS_K; k++) pthread_join(th[r][k], NULL);
  sqobfs_engine_info ei;
  CHECK(sqobfs_engine_info_get(ctx, &ei));
  for (int k = 0; k < GS_K; k++) {
    EXPECT(ga[1][k].got == GS_N && ga[1][k].bad == 0, "group stress kind %d conn %d: taken %d, %d "
           "differ", kind, k, ga[1][k].got, ga[1][k].bad);
    EXPECT(ga[3][k].got == GS_N && ga[3][k].bad == 0, "group stress kind %d conn %d: read %d, %d "
           "differ", kind, k, ga[3][k].got, ga[3][k].bad);
    sqobfs_pconn_close(pc[k]);
    sqobfs_keyring_destroy(kr[k]);
  }
  EXPECT(!no_poll || ei.async_launches == ei.launches, "group stress: %llu of %llu launches "
         "landed by the completer", (unsigned long long)ei.async_launches,
         (unsigned long long)ei.launches);
  EXPECT(no_poll || ei.async_launches == 0, "group stress: polled launches on the completer");
  printf("  group stress kind %d%s: %d conns x %d datagrams each way on 4 workers == reference; "
         "%llu launches (%llu by the completer, %u streams), %llu coalesced (%llu batches)\n",
         kind, no_poll ? " [async]" : "", GS_K, GS_N, (unsigned long long)ei.launches,
         (unsigned long long)ei.async_launches, ei.streams, (unsigned long long)ei.group_launches,
         (unsigned long long)ei.group_batches);
  sqobfs_engine_trim(ctx);
  EXPECT(sqobfs_debug_host_allocs() == a0, "group stress: host allocs");
  sqobfs_close(ctx);
}

static void t_fail(int at_completion, int no_poll) {
  sqobfs_ctx *ctx = NULL;
  CHECK(sqobfs_open(0, &ctx));
  /* (this context's engine threads left to the scheduler; after its first
   * pconn the setting is refused) */
  CHECK(sqobfs_engine_set_affinity(ctx, SQOBFS_ENGINE_AFFINITY_NONE));
  const int64_t a0 = sqobfs_debug_host_allocs();
  for (int kind = 0; kind < 2; kind++) {
    const int S = salt_len(kind);
    uint64_t off = 0;
    uint32_t plen_psk = PL;
    sqobfs_keyring *kr = NULL;
    CHECK(sqobfs_keyring_create(ctx, kind, 1, PSK, &off, &plen_psk, &kr));
    sqobfs_pconn *pc = NULL;
    sqobfs_pconn_opts o;
    memset(&o, 0, sizeof o);
    o.cpu_max = SQOBFS_PCONN_NEVER; /* every batch launches while the GPU works */
    if (no_poll) o.spin_us = SQOBFS_PCONN_NEVER; /* (landed by the completer) */
    CHECK(sqobfs_pconn_open(ctx, kr, -1, &o, &pc));
    EXPECT(sqobfs_engine_set_affinity(ctx, SQOBFS_ENGINE_AFFINITY_L3) == SQ_EINVAL,
           "affinity changed after the engine started");
    sqobfs_engine_info ai;
    CHECK(sqobfs_engine_info_get(ctx, &ai));
    EXPECT(ai.cpus == 0, "AFFINITY_NONE engine restricted to %u CPUs", ai.cpus);
    static uint8_t pay[400][2048];
    static uint32_t plen[400];
    for (int i = 0; i < 400; i++) {
      plen[i] = pick_len(i, S, 2048);
      for (uint32_t j = 0; j < plen[i]; j++) pay[i][j] = (uint8_t)rnd();
    }
    /* transmit: 100 before the failure, the failure, 300 after */
    Taker t = {pc, kind, 0, 0, pay, plen};
    pthread_t th;
    pthread_create(&th, NULL, taker, &t);
    for (int i = 0; i < 100; i++) CHECK(sqobfs_pconn_write(pc, pay[i], plen[i], NULL, (uint64_t)i));
    sleep_ms(50);
    if (kind == 0) sqobfs_debug_engine_fail(1, at_completion);
    for (int i = 100; i < 400; i++) {
      CHECK(sqobfs_pconn_write(pc, pay[i], plen[i], NULL, (uint64_t)i));
      if (i % 50 == 0) sleep_ms(2);
    }
    sleep_ms(100);
    sqobfs_pconn_stats st;
    CHECK(sqobfs_pconn_stats_get(pc, &st));
    /* receive: pushed datagrams still read back as the reference's ReadFrom
     * (the engine is on the CPU now) */
    for (int i = 0; i < 300; i++) {
      uint8_t salt[16], w[MAXW], got[MAXW], ref[MAXW];
      for (int b = 0; b < 16; b++) salt[b] = (uint8_t)rnd();
      ref_write(kind, salt, pay[i], plen[i], w);
      CHECK(sqobfs_pconn_rx_push(pc, w, plen[i] + (uint32_t)S, NULL, (uint64_t)i));
      uint32_t n;
      CHECK(sqobfs_pconn_read(pc, got, MAXW, &n, NULL, NULL));
      const long want = ref_read(kind, w, plen[i] + (uint32_t)S, MAXW, ref);
      EXPECT((long)n == want && (!n || !memcmp(got, ref, n)), "after failure: read %d", i);
    }
    sqobfs_pconn_shutdown(pc);
    pthread_join(th, NULL);
    sqobfs_engine_info info;
    CHECK(sqobfs_engine_info_get(ctx, &info));
    EXPECT(t.bad == 0, "fail kind %d: %d taken datagrams differ", kind, t.bad);
    EXPECT(info.gpu_disabled == 1, "the engine did not switch to the CPU");
    EXPECT(kind == 1 || st.gpu_failures == 1, "failure not counted");
    if (at_completion)
      EXPECT(t.count + (int)st.dropped == 400 && (kind == 1 || st.dropped > 0),
             "fail kind %d: taken %d + dropped %llu != 400", kind, t.count,
             (unsigned long long)st.dropped);
    else
      EXPECT(t.count == 400 && st.dropped == 0, "fail kind %d: taken %d of 400", kind, t.count);
    EXPECT(st.gpu_refused == 0, "fail kind %d: %llu refusals counted", kind,
           (unsigned long long)st.gpu_refused);
    printf("  fail kind %d (%s%s): %d of 400 datagrams taken == reference (%llu dropped), "
           "%llu CPU batches; 300 reads after it == reference\n", kind,
           at_completion ? "kernel failed" : "launch refused", no_poll ? ", async" : "", t.count,
           (unsigned long long)st.dropped, (unsigned long long)st.cpu_batches);
    sqobfs_pconn_close(pc);
    sqobfs_keyring_destroy(kr);
  }
  sqobfs_engine_trim(ctx);
  EXPECT(sqobfs_debug_host_allocs() == a0, "fail: host allocs");
  sqobfs_close(ctx);
}

int main(int argc, char **argv) {
  g_nodev = argc > 1 && !strcmp(argv[1], "nodev");
  if (!g_nodev) CHECK(sqobfs_open(0, &g_ctx));
  const int64_t a0 = sqobfs_debug_host_allocs();
  for (int kind = 0; kind < 2; kind++) {
    t_wire(kind, 0);
    t_wire(kind, SQOBFS_UDP_TX_GSO);
    t_read(kind);
    t_roundtrip(kind, 0);
    t_roundtrip(kind, SQOBFS_UDP_TX_GSO | SQOBFS_UDP_RX_GRO);
    t_pump(kind);
    t_syncerr(kind);
    t_poolfail(kind);
  }
  t_deadline();
  t_shutdown();
  t_shared();
  if (!g_nodev) {
    t_routing();
    t_load();
    t_group(SQOBFS_SALAMANDER, 0);
    t_group(SQOBFS_XPLUS, 0);
    t_group(SQOBFS_SALAMANDER, 1);
    t_group(SQOBFS_XPLUS, 1);
    t_many_psks(SQOBFS_SALAMANDER);
    t_many_psks(SQOBFS_XPLUS);
    t_group_stress(SQOBFS_SALAMANDER, 0);
    t_group_stress(SQOBFS_XPLUS, 0);
    t_group_stress(SQOBFS_SALAMANDER, 1);
    t_group_stress(SQOBFS_XPLUS, 1);
    t_fail(0, 0);
    t_fail(1, 0);
    t_fail(0, 1);
    t_fail(1, 1);
    /* the async pass: socket and pump conns whose every batch is landed by
     * the completer */
    sqobfs_engine_info a0i, a1i;
    CHECK(sqobfs_engine_info_get(g_ctx, &a0i));
    g_async = 1;
    for (int kind = 0; kind < 2; kind++) {
      t_wire(kind, 0);
      t_wire(kind, SQOBFS_UDP_TX_GSO);
      t_read(kind);
      t_roundtrip(kind, 0);
      t_roundtrip(kind, SQOBFS_UDP_TX_GSO | SQOBFS_UDP_RX_GRO);
    }
    g_async = 0;
    CHECK(sqobfs_engine_info_get(g_ctx, &a1i));
    EXPECT(a1i.async_launches > a0i.async_launches + 100, "async pass: %llu completer launches",
           (unsigned long long)(a1i.async_launches - a0i.async_launches));
    printf("  async pass: %llu launches landed by the completer (%u streams)\n",
           (unsigned long long)(a1i.async_launches - a0i.async_launches), a1i.streams);
  }
  sqobfs_engine_info info;
  CHECK(sqobfs_engine_info_get(g_ctx, &info));
  EXPECT(info.gpu_disabled == 0, "the shared engine switched to the CPU");
  EXPECT(info.cpus == 0 || info.cpus >= 2, "engine kept on %u CPU", info.cpus);
  printf("  engine threads kept on %u CPUs (the L3 domain of the thread that started it; 0 = "
         "free)\n", info.cpus);
  if (g_ctx) sqobfs_close(g_ctx);
  EXPECT(sqobfs_debug_host_allocs() == a0, "host allocs after close");
  printf("ok: pconn engine [%s] (socket + pump modes, deadlines, shutdown, memory, sync errors, "
         "allocation failures, "
         "shared engine%s)\n", g_nodev ? "no device" : "device",
         g_nodev ? "" : ", routing, load routing, coalesced launches, launch failures");
  return 0;
}
