/* lat_bench.c -- per-datagram latency of the host-memory paths (DESIGN.md
 * section 9.5), against the reference's synchronous per-datagram WriteTo /
 * ReadFrom (hysteria2/salamander.go:42-70).
 *
 * For batches of 1, 16, 64 and 256 Salamander datagrams of 1350 B:
 *   run_host   sqobfs_run_host on page-locked slots (staged H2D | kernel | D2H),
 *              one call per batch: every datagram of the batch waits the whole
 *              call
 *   mapped     one launch on page-locked, GPU-mapped slots + stream wait (what
 *              sqobfs_udp_conn and sqobfs_pconn do per batch), and the same
 *              over unit sizes 1..26 packets per wave for the 256 batch
 *   endpoint   sqobfs_udp_conn_write of the batch to a loopback socket: from
 *              the call to the last datagram's arrival
 *   pconn      n back-to-back sqobfs_pconn_write calls (the Go Conn's
 *              WriteTo): per datagram, its write call to its arrival at a
 *              plain loopback socket; and the receive side, a peer's burst of
 *              n datagrams to each sqobfs_pconn_read's return
 *   cpu        the oracle's byte-loop WriteTo of one datagram (the
 *              reference's per-call work on one core, no socket)
 * Prints one JSON object (p50 / p99 in microseconds).  Built by
 * `make -C sing-quic_amd tools`; run by bench.py --latency.
 *
 * `lat_bench load [seconds [reps]]`: sustained load instead -- pconn A -> pconn B
 * over loopback (GSO / GRO, 1,024-datagram batches), a writer paced at a
 * fixed offered rate, for every routing mode: the process's CPU time
 * (getrusage: every engine thread of both ends, the writer and the reader)
 * per GiB of payload that arrived, and the batches each route took
 * ("CPU per GiB").
 *
 * `lat_bench hops [K [seconds [reps]]]`: K pump-mode pconns on one context
 * (a port-hopping client's conns over generic PacketConns; default options,
 * a keyring per conn as the Go adapters make), K writers together offering
 * 0.5, 1, 2 GiB/s and unpaced, K takers; the defaults (coalesced launches),
 * coalescing off (sqobfs_engine_set_group 1) and every batch on the CPU
 * path: CPU seconds per GiB, launches and batches per launch
 * (`lat_bench hops K secs reps unpaced`: the unpaced rate only).
 *
 * `lat_bench tput [runs]`: the default-routing GSO / GRO throughput run
 * (200,000 datagrams A -> B) repeated, each with its process CPU time,
 * involuntary context switches and the cgroup's CPU-quota throttling
 * (cpu.stat nr_throttled / throttled_usec) over the run: whether a slow run
 * was a throttled one, and how many L3 domains (CCDs) the process's threads
 * last ran on ("the small-batch regime").
 * `lat_bench tput [runs] pin`: the process (and so every engine thread it
 * starts) restricted to the CPUs that share the L3 of the CPU it starts
 * on, within its affinity. */
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
#include <dirent.h>
#include <sched.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "sqobfs.h"

/* oracle restatement of SalamanderPacketConn.WriteTo (checker / CPU timing) */
long or_salamander_write(const uint8_t *psk, size_t psk_len, const uint8_t salt[8],
                         const uint8_t *p, size_t len, uint8_t *wire);

#define CHECK(x)                                                                   \
  do {                                                                             \
    int st_ = (x);                                                                 \
    if (st_ != SQ_OK) {                                                            \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, st_,        \
              sqobfs_strerror(st_));                                               \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

static const uint8_t PSK[] = "sing-quic-mi355x-bench-psk";
#define PL (sizeof PSK - 1)
#define L 1350
#define SLOT 2048
#define MAXN 256

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmpd(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}
static double pct(double *v, int n, double q) {
  qsort(v, (size_t)n, sizeof *v, cmpd);
  int i = (int)(q * (n - 1) + 0.5);
  return v[i];
}

static int udp_socket(uint16_t *port) {
  int fd = socket(AF_INET, SOCK_DGRAM, 0);
  int big = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
  struct sockaddr_in a;
  memset(&a, 0, sizeof a);
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  bind(fd, (struct sockaddr *)&a, sizeof a);
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

static long recv_to(int fd, uint8_t *buf, size_t cap, int ms) {
  struct pollfd p = {fd, POLLIN, 0};
  if (poll(&p, 1, ms) <= 0) return -1;
  return recv(fd, buf, cap, 0);
}

static const int SIZES[] = {1, 16, 64, 256};
#define NS 4
static int iters_for(int n) { return n <= 16 ? 400 : n <= 64 ? 200 : 100; }

static void print_stat(const char *name, double *v, int n, int last) {
  const double p50 = pct(v, n, 0.5), p99 = pct(v, n, 0.99);
  printf("\"%s\": {\"p50_us\": %.1f, \"p99_us\": %.1f, \"samples\": %d}%s", name, p50, p99, n,
         last ? "" : ", ");
}

/* pconn throughput reader: reads until 300 ms pass without a datagram */
void *tput_reader(void *arg) {
  struct rd {
    sqobfs_pconn *pc;
    long got;
    double last_us;
  } *r = arg;
  static uint8_t buf[4096];
  for (;;) {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    sqobfs_pconn_set_deadline(r->pc, SQOBFS_PCONN_READ,
                              (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec + 300000000);
    uint32_t n;
    if (sqobfs_pconn_read(r->pc, buf, sizeof buf, &n, NULL, NULL) != SQ_OK) break;
    r->got++;
    r->last_us = now_us();
  }
  return NULL;
}

/* per-datagram latency through the packet conn engine (opts o, NULL =
 * defaults): WriteTo bursts -> arrival at a peer socket; peer bursts ->
 * ReadFrom */
static void pconn_lat(sqobfs_ctx *ctx, sqobfs_keyring *kr, const char *label,
                      const sqobfs_pconn_opts *o) {
  static double v[MAXN * 400];
  uint16_t pa, pp;
  int fa = udp_socket(&pa), fp = udp_socket(&pp);
  sqobfs_pconn *pc;
  CHECK(sqobfs_pconn_open(ctx, kr, fa, o, &pc));
  const sqobfs_addr to = loop_addr(pp);
  static uint8_t pay[L], buf[4096], wire[MAXN][L + 8];
  memset(pay, 5, L);
  static double tw[MAXN];
  printf("\"pconn_write%s\": {", label);
  for (int k = 0; k < NS; k++) {
    const int n = SIZES[k], it = iters_for(n) / 4 + 1;
    int m = 0;
    for (int i = 0; i < it + 5; i++) {
      for (int j = 0; j < n; j++) {
        tw[j] = now_us();
        CHECK(sqobfs_pconn_write(pc, pay, L, &to, 0));
      }
      for (int j = 0; j < n; j++) {
        if (recv_to(fp, buf, sizeof buf, 2000) < 0) exit(3);
        if (i >= 5) v[m++] = now_us() - tw[j];
      }
    }
    char nm[16];
    snprintf(nm, sizeof nm, "%d", n);
    print_stat(nm, v, m, k == NS - 1);
  }
  printf("}, ");
  /* receive side: obfuscated datagrams from the peer */
  for (int j = 0; j < MAXN; j++) {
    uint8_t salt[8] = {(uint8_t)j, 1, 2, 3, 4, 5, 6, 7};
    or_salamander_write(PSK, PL, salt, pay, L, wire[j]);
  }
  struct sockaddr_in a;
  memset(&a, 0, sizeof a);
  a.sin_family = AF_INET;
  a.sin_port = htons(pa);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  printf("\"pconn_read%s\": {", label);
  for (int k = 0; k < NS; k++) {
    const int n = SIZES[k], it = iters_for(n) / 4 + 1;
    int m = 0;
    for (int i = 0; i < it + 5; i++) {
      const double t0 = now_us();
      for (int j = 0; j < n; j++)
        sendto(fp, wire[j], L + 8, 0, (struct sockaddr *)&a, sizeof a);
      for (int j = 0; j < n; j++) {
        uint32_t got;
        CHECK(sqobfs_pconn_read(pc, buf, sizeof buf, &got, NULL, NULL));
        if (got != L) exit(4);
        if (i >= 5) v[m++] = now_us() - t0;
      }
    }
    char nm[16];
    snprintf(nm, sizeof nm, "%d", n);
    print_stat(nm, v, m, k == NS - 1);
  }
  printf("}, ");
  sqobfs_pconn_stats st;
  CHECK(sqobfs_pconn_stats_get(pc, &st));
  printf("\"pconn_stats%s\": {\"tx_datagrams\": %llu, \"tx_batches\": %llu, \"rx_datagrams\": "
         "%llu, \"rx_batches\": %llu, \"cpu_batches\": %llu, \"inline_writes\": %llu}, ",
         label, (unsigned long long)st.tx_datagrams, (unsigned long long)st.tx_batches,
         (unsigned long long)st.rx_datagrams, (unsigned long long)st.rx_batches,
         (unsigned long long)st.cpu_batches, (unsigned long long)st.inline_writes);
  sqobfs_pconn_close(pc);
  close(fa);
  close(fp);
}

/* the cgroup's CPU throttling counters (v2 cpu.stat; zeros when absent) */
static void cg_throttle(long long *nr, long long *usec) {
  *nr = *usec = 0;
  FILE *f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return;
  char k[64];
  long long v;
  while (fscanf(f, "%63s %lld", k, &v) == 2) {
    if (!strcmp(k, "nr_throttled")) *nr = v;
    if (!strcmp(k, "throttled_usec")) *usec = v;
  }
  fclose(f);
}

/* L3 (CCD) id of a CPU, -1 when unknown */
static int l3_of(int cpu) {
  char path[128];
  snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/id", cpu);
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  int id = -1;
  if (fscanf(f, "%d", &id) != 1) id = -1;
  fclose(f);
  return id;
}

/* distinct L3 domains the process's threads last ran on, and the threads */
static int l3_spread(int *threads) {
  int ids[64], nid = 0;
  *threads = 0;
  DIR *d = opendir("/proc/self/task");
  if (!d) return -1;
  struct dirent *e;
  while ((e = readdir(d))) {
    if (e->d_name[0] == '.') continue;
    char path[300], buf[1024];
    snprintf(path, sizeof path, "/proc/self/task/%s/stat", e->d_name);
    FILE *f = fopen(path, "r");
    if (!f) continue;
    const size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *p = strrchr(buf, ')'); /* fields after the command name */
    if (!p) continue;
    int field = 2, cpu = -1;
    for (const char *q = p + 1; *q; q++)
      if (*q == ' ' && ++field == 39) {
        cpu = atoi(q + 1);
        break;
      }
    if (cpu < 0) continue;
    (*threads)++;
    const int id = l3_of(cpu);
    int seen = 0;
    for (int i = 0; i < nid; i++) seen |= ids[i] == id;
    if (!seen && nid < 64) ids[nid++] = id;
  }
  closedir(d);
  return nid;
}

/* restrict the process to the allowed CPUs sharing this CPU's L3 */
static int pin_to_l3(void) {
  cpu_set_t cur, want;
  if (sched_getaffinity(0, sizeof cur, &cur)) return 0;
  const int me = sched_getcpu(), l3 = l3_of(me);
  CPU_ZERO(&want);
  int n = 0;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &cur) && l3_of(c) == l3) {
      CPU_SET(c, &want);
      n++;
    }
  if (n && sched_setaffinity(0, sizeof want, &want)) return 0;
  return n;
}

static double cpu_s(void) {
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec +
         ru.ru_stime.tv_usec * 1e-6;
}

/* One sustained-load run: `gib_s` of payload offered for `secs` seconds
 * (0: as fast as the writer goes). */
static void load_run(const char *name, sqobfs_ctx *c, sqobfs_keyring *k,
                     const sqobfs_pconn_opts *mode, double gib_s, double secs) {
  uint16_t pa, pb;
  int fa = udp_socket(&pa), fb = udp_socket(&pb);
  int huge = 64 << 20;
  setsockopt(fb, SOL_SOCKET, SO_RCVBUF, &huge, sizeof huge);
  setsockopt(fa, SOL_SOCKET, SO_SNDBUF, &huge, sizeof huge);
  sqobfs_pconn *A, *B;
  sqobfs_pconn_opts oa = *mode, ob = *mode;
  oa.flags = SQOBFS_UDP_TX_GSO;
  ob.flags = SQOBFS_UDP_RX_GRO;
  oa.batch = ob.batch = 1024;
  CHECK(sqobfs_pconn_open(c, k, fa, &oa, &A));
  CHECK(sqobfs_pconn_open(c, k, fb, &ob, &B));
  const sqobfs_addr to = loop_addr(pb);
  static uint8_t pay[L];
  memset(pay, 9, L);
  struct rd {
    sqobfs_pconn *pc;
    long got;
    double last_us;
  } r = {B, 0, 0};
  pthread_t th;
  extern void *tput_reader(void *);
  pthread_create(&th, NULL, tput_reader, &r);
  const double rate = gib_s > 0 ? gib_s * (double)(1 << 30) / L : 0; /* datagrams per s */
  const double c0 = cpu_s(), t0 = now_us();
  long n = 0;
  for (;;) {
    for (int j = 0; j < 64; j++, n++) CHECK(sqobfs_pconn_write(A, pay, L, &to, 0));
    const double now = now_us();
    if (now - t0 >= secs * 1e6) break;
    if (rate > 0) {
      const double due = t0 + n / rate * 1e6;
      if (due > now + 20) {
        struct timespec ts = {0, (long)((due - now) * 1000)};
        nanosleep(&ts, NULL);
      }
    }
  }
  pthread_join(th, NULL); /* (the reader stops 300 ms after the last arrival) */
  const double c1 = cpu_s();
  const double dt = (r.last_us - t0) * 1e-6;
  const double gib = r.got * (double)L / (1 << 30);
  sqobfs_pconn_stats sa, sb;
  CHECK(sqobfs_pconn_stats_get(A, &sa));
  CHECK(sqobfs_pconn_stats_get(B, &sb));
  sqobfs_engine_info ei;
  CHECK(sqobfs_engine_info_get(c, &ei));
  const unsigned long long bt = sa.tx_batches + sb.rx_batches, bc = sa.cpu_batches + sb.cpu_batches;
  printf("{\"mode\": \"%s\", \"offered_gib_s\": %.3f, \"sent\": %ld, \"received\": %ld, "
         "\"seconds\": %.3f, \"payload_gib_s\": %.3f, \"cpu_seconds\": %.3f, "
         "\"cpu_cores\": %.2f, \"cpu_s_per_gib\": %.3f, \"batches\": %llu, "
         "\"gpu_batches\": %llu, \"cpu_batches\": %llu, \"inline_writes\": %llu, "
         "\"tx_max_batch\": %u, \"rx_max_batch\": %u, \"load_permille\": %u, \"loaded\": %u, "
         "\"gpu_host_ns\": %u, \"cpu_ns_per_kib\": %u, \"launch_us\": %u}",
         name, gib_s, n, r.got, dt, gib / dt, c1 - c0, (c1 - c0) / dt, (c1 - c0) / gib, bt, bt - bc,
         bc, (unsigned long long)sa.inline_writes, sa.tx_max_batch, sb.rx_max_batch,
         ei.load_permille, ei.loaded, ei.gpu_host_ns, ei.cpu_ns_per_kib, ei.launch_us);
  fflush(stdout);
  sqobfs_pconn_close(A);
  sqobfs_pconn_close(B);
  close(fa);
  close(fb);
}

static int load_main(double secs, int reps) {
  sqobfs_ctx *ctx;
  CHECK(sqobfs_open(0, &ctx));
  uint64_t o0 = 0;
  uint32_t l0 = PL;
  sqobfs_keyring *kr, *hk;
  CHECK(sqobfs_keyring_create(ctx, SQOBFS_SALAMANDER, 1, PSK, &o0, &l0, &kr));
  CHECK(sqobfs_keyring_create(NULL, SQOBFS_SALAMANDER, 1, PSK, &o0, &l0, &hk));
  sqobfs_pconn_opts dflt, cpu, gpoll, gblock;
  memset(&dflt, 0, sizeof dflt);
  cpu = gpoll = gblock = dflt;
  cpu.cpu_max = 1u << 30;
  gpoll.cpu_max = gpoll.inline_gap_us = SQOBFS_PCONN_NEVER;
  gblock = gpoll;
  gblock.spin_us = SQOBFS_PCONN_NEVER;
  static const double rates_all[] = {0.25, 0.5, 1.0, 2.0, 0};
  static const double rates_bulk[] = {1.0, 2.0, 0};
  /* reps > 1: the bulk rates only, every mode but the polling one, the
   * (rate, mode) runs interleaved reps times (box noise between runs) */
  const double *rates = reps > 1 ? rates_bulk : rates_all;
  const int nr = reps > 1 ? 3 : 5;
  printf("{\"load\": [");
  int first = 1;
  for (int ri = 0; ri < nr; ri++)
    for (int rp = 0; rp < (reps > 1 ? reps : 1); rp++)
    for (int m = 0; m < 5; m++) {
      if (reps > 1 && m == 2) continue;
      if (!first) printf(", ");
      first = 0;
      static const char *const names[] = {"default", "cpu_only", "gpu_poll", "gpu_block",
                                          "no_device"};
      const sqobfs_pconn_opts *o = m == 0 ? &dflt : m == 1 ? &cpu : m == 2 ? &gpoll
                                   : m == 3 ? &gblock : &dflt;
      load_run(names[m], m == 4 ? NULL : ctx, m == 4 ? hk : kr, o, rates[ri], secs);
    }
  printf("]}\n");
  sqobfs_keyring_destroy(hk);
  sqobfs_keyring_destroy(kr);
  sqobfs_close(ctx);
  return 0;
}

/* One default-routing throughput run (the main table's pconn_throughput
 * _gso_gro line) with its CPU, context-switch and throttling counters. */
static void tput_run(sqobfs_ctx *ctx, sqobfs_keyring *kr, int run, int last) {
  uint16_t pa, pb;
  int fa = udp_socket(&pa), fb = udp_socket(&pb);
  sqobfs_pconn *A, *B;
  sqobfs_pconn_opts oa, ob;
  memset(&oa, 0, sizeof oa);
  memset(&ob, 0, sizeof ob);
  oa.flags = SQOBFS_UDP_TX_GSO;
  ob.flags = SQOBFS_UDP_RX_GRO;
  CHECK(sqobfs_pconn_open(ctx, kr, fa, &oa, &A));
  CHECK(sqobfs_pconn_open(ctx, kr, fb, &ob, &B));
  const sqobfs_addr to = loop_addr(pb);
  static uint8_t pay[L];
  memset(pay, 9, L);
  struct rd {
    sqobfs_pconn *pc;
    long got;
    double last_us;
  } r = {B, 0, 0};
  pthread_t th;
  extern void *tput_reader(void *);
  pthread_create(&th, NULL, tput_reader, &r);
  struct rusage u0, u1, w0, w1;
  long long nr0, us0, nr1, us1;
  cg_throttle(&nr0, &us0);
  getrusage(RUSAGE_SELF, &u0);
  getrusage(RUSAGE_THREAD, &w0);
  const long N = 200000;
  const double t0 = now_us();
  for (long i = 0; i < N; i++) {
    CHECK(sqobfs_pconn_write(A, pay, L, &to, 0));
    if ((i & 1023) == 1023) {
      struct timespec ts = {0, 200000};
      nanosleep(&ts, NULL);
    }
  }
  getrusage(RUSAGE_THREAD, &w1);
  pthread_join(th, NULL);
  getrusage(RUSAGE_SELF, &u1);
  cg_throttle(&nr1, &us1);
  int nthr;
  const int l3 = l3_spread(&nthr);
  const double dt = (r.last_us - t0) * 1e-6;
  sqobfs_pconn_stats sa, sb;
  CHECK(sqobfs_pconn_stats_get(A, &sa));
  CHECK(sqobfs_pconn_stats_get(B, &sb));
#define TV(a) ((a).tv_sec + (a).tv_usec * 1e-6)
  printf("{\"run\": %d, \"received\": %ld, \"seconds\": %.3f, \"datagrams_per_s\": %.0f, "
         "\"tx_batches\": %llu, \"rx_batches\": %llu, \"cpu_s\": %.3f, \"writer_cpu_s\": %.3f, "
         "\"nivcsw\": %ld, \"nvcsw\": %ld, \"writer_nivcsw\": %ld, \"throttled_periods\": %lld, "
         "\"throttled_ms\": %.1f, \"l3_domains\": %d, \"threads\": %d}%s\n",
         run, r.got, dt, r.got / dt, (unsigned long long)sa.tx_batches,
         (unsigned long long)sb.rx_batches,
         TV(u1.ru_utime) + TV(u1.ru_stime) - TV(u0.ru_utime) - TV(u0.ru_stime),
         TV(w1.ru_utime) + TV(w1.ru_stime) - TV(w0.ru_utime) - TV(w0.ru_stime),
         u1.ru_nivcsw - u0.ru_nivcsw, u1.ru_nvcsw - u0.ru_nvcsw, w1.ru_nivcsw - w0.ru_nivcsw,
         nr1 - nr0, (us1 - us0) * 1e-3, l3, nthr, last ? "" : ",");
#undef TV
  fflush(stdout);
  sqobfs_pconn_close(A);
  sqobfs_pconn_close(B);
  close(fa);
  close(fb);
}

static int tput_main(int runs, int pin) {
  const int pinned = pin ? pin_to_l3() : 0;
  long long nr, us;
  FILE *cs = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (cs) fclose(cs);
  cg_throttle(&nr, &us);
  sqobfs_ctx *ctx;
  CHECK(sqobfs_open(0, &ctx));
  uint64_t o0 = 0;
  uint32_t l0 = PL;
  sqobfs_keyring *kr;
  CHECK(sqobfs_keyring_create(ctx, SQOBFS_SALAMANDER, 1, PSK, &o0, &l0, &kr));
  printf("{\"pinned_cpus\": %d, \"cgroup_cpu_stat\": %s, \"tput_gso_gro\": [\n", pinned,
         cs ? "true" : "false");
  for (int i = 0; i < runs; i++) tput_run(ctx, kr, i, i == runs - 1);
  printf("]}\n");
  sqobfs_keyring_destroy(kr);
  sqobfs_close(ctx);
  return 0;
}

/* ---- hops: several pump-mode pconns on one context, coalesced launches */
typedef struct {
  sqobfs_pconn *pc;
  double rate, secs, t0; /* datagrams per s (0: unpaced) */
  long n, got;
  double last_us;
} Hop;

static void *hop_writer(void *arg) {
  Hop *h = arg;
  static const uint8_t pay[L] = {9};
  for (;;) {
    for (int j = 0; j < 64; j++, h->n++) CHECK(sqobfs_pconn_write(h->pc, pay, L, NULL, 0));
    const double now = now_us();
    if (now - h->t0 >= h->secs * 1e6) break;
    if (h->rate > 0) {
      const double due = h->t0 + h->n / h->rate * 1e6;
      if (due > now + 20) {
        struct timespec ts = {0, (long)((due - now) * 1000)};
        nanosleep(&ts, NULL);
      }
    }
  }
  return NULL;
}

/* the wrapped conn's side of pump mode: take each obfuscated batch (here:
 * count it) and hand it back, until 300 ms pass without one */
static void *hop_taker(void *arg) {
  Hop *h = arg;
  for (;;) {
    sqobfs_pconn_tx v;
    if (sqobfs_pconn_tx_take(h->pc, 300, &v) != SQ_OK) break;
    h->got += v.count;
    h->last_us = now_us();
    CHECK(sqobfs_pconn_tx_done(h->pc));
  }
  return NULL;
}

/* K pump-mode pconns (the Go adapter over a generic PacketConn: a hop
 * client's bufio.NewUnbindPacketConn, hysteria/client.go:184-186), each on a
 * keyring of its own with the same PSK (as the adapters make one per conn),
 * K writers together offering gib_s of payload (0: unpaced) for secs
 * seconds, K takers.  cpu_max: the conns' option (0: the default routing). */
static void hops_run(sqobfs_ctx *c, const char *name, int K, uint32_t group, uint32_t cpu_max,
                     double gib_s, double secs) {
  enum { KMAX = 32 };
  CHECK(sqobfs_engine_set_group(c, group));
  Hop h[KMAX];
  sqobfs_keyring *kr[KMAX];
  pthread_t tw[KMAX], tt[KMAX];
  uint64_t o0 = 0;
  uint32_t l0 = PL;
  for (int k = 0; k < K; k++) {
    CHECK(sqobfs_keyring_create(c, SQOBFS_SALAMANDER, 1, PSK, &o0, &l0, &kr[k]));
    sqobfs_pconn_opts o;
    memset(&o, 0, sizeof o);
    o.cpu_max = cpu_max;
    /* (dev sweep: transmit batches per conn) */
    if (getenv("HOPS_TXB")) o.tx_batches = (uint32_t)atoi(getenv("HOPS_TXB"));
    memset(&h[k], 0, sizeof h[k]);
    CHECK(sqobfs_pconn_open(c, kr[k], -1, &o, &h[k].pc));
    h[k].rate = gib_s > 0 ? gib_s * (double)(1 << 30) / L / K : 0;
    h[k].secs = secs;
  }
  sqobfs_engine_info e0, e1;
  CHECK(sqobfs_engine_info_get(c, &e0));
  const double c0 = cpu_s(), t0 = now_us();
  for (int k = 0; k < K; k++) {
    h[k].t0 = t0;
    pthread_create(&tt[k], NULL, hop_taker, &h[k]);
    pthread_create(&tw[k], NULL, hop_writer, &h[k]);
  }
  long sent = 0, got = 0;
  double last = t0;
  for (int k = 0; k < K; k++) {
    pthread_join(tw[k], NULL);
    pthread_join(tt[k], NULL);
    sent += h[k].n;
    got += h[k].got;
    if (h[k].last_us > last) last = h[k].last_us;
  }
  const double c1 = cpu_s();
  CHECK(sqobfs_engine_info_get(c, &e1));
  unsigned long long bt = 0, bc = 0;
  uint32_t maxb = 0;
  for (int k = 0; k < K; k++) {
    sqobfs_pconn_stats s;
    CHECK(sqobfs_pconn_stats_get(h[k].pc, &s));
    bt += s.tx_batches;
    bc += s.cpu_batches;
    if (s.tx_max_batch > maxb) maxb = s.tx_max_batch;
  }
  const double dt = (last - t0) * 1e-6, gib = got * (double)L / (1 << 30);
  const unsigned long long nl = e1.launches - e0.launches;
  const unsigned long long gl = e1.group_launches - e0.group_launches;
  const unsigned long long gb = e1.group_batches - e0.group_batches;
  printf("{\"mode\": \"%s\", \"conns\": %d, \"group\": %u, \"offered_gib_s\": %.3f, "
         "\"sent\": %ld, \"taken\": %ld, \"seconds\": %.3f, \"payload_gib_s\": %.3f, "
         "\"cpu_seconds\": %.3f, \"cpu_s_per_gib\": %.3f, \"batches\": %llu, "
         "\"max_batch\": %u, \"cpu_batches\": %llu, \"launches\": %llu, "
         "\"coalesced_launches\": %llu, \"coalesced_batches\": %llu, "
         "\"batches_per_launch\": %.2f, \"loaded\": %u, \"gpu_host_ns\": %u, "
         "\"cpu_ns_per_kib\": %u}",
         name, K, e1.group_max, gib_s, sent, got, dt, gib / dt, c1 - c0, (c1 - c0) / gib, bt,
         maxb, bc, nl, gl, gb, nl ? (double)(bt - bc) / nl : 0.0, e1.loaded, e1.gpu_host_ns,
         e1.cpu_ns_per_kib);
  fflush(stdout);
  for (int k = 0; k < K; k++) {
    sqobfs_pconn_close(h[k].pc);
    sqobfs_keyring_destroy(kr[k]);
  }
}

static int hops_main(int K, double secs, int reps, int unpaced_only) {
  if (K < 1 || K > 32) K = 8;
  sqobfs_ctx *ctx;
  CHECK(sqobfs_open(0, &ctx));
  static const double rates[] = {0.5, 1.0, 2.0, 0};
  printf("{\"hops\": [");
  int first = 1;
  for (int ri = unpaced_only ? 3 : 0; ri < 4; ri++)
    for (int rp = 0; rp < reps; rp++)
      for (int m = 0; m < 3; m++) {
        if (!first) printf(", ");
        first = 0;
        /* the defaults; coalescing off; every batch on the CPU path */
        static const char *const names[] = {"default", "group_off", "cpu_only"};
        hops_run(ctx, names[m], K, m == 1 ? 1u : 0u, m == 2 ? 1u << 30 : 0u, rates[ri], secs);
      }
  printf("]}\n");
  sqobfs_close(ctx);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && !strcmp(argv[1], "hops"))
    return hops_main(argc > 2 ? atoi(argv[2]) : 8, argc > 3 ? atof(argv[3]) : 1.5,
                     argc > 4 ? atoi(argv[4]) : 1, argc > 5 && !strcmp(argv[5], "unpaced"));
  if (argc > 1 && !strcmp(argv[1], "load"))
    return load_main(argc > 2 ? atof(argv[2]) : 1.5, argc > 3 ? atoi(argv[3]) : 1);
  if (argc > 1 && !strcmp(argv[1], "tput"))
    return tput_main(argc > 2 ? atoi(argv[2]) : 45, argc > 3 && !strcmp(argv[3], "pin"));
  sqobfs_ctx *ctx;
  CHECK(sqobfs_open(0, &ctx));
  uint64_t off0 = 0;
  uint32_t len0 = PL;
  sqobfs_keyring *kr;
  CHECK(sqobfs_keyring_create(ctx, SQOBFS_SALAMANDER, 1, PSK, &off0, &len0, &kr));
  static double v[MAXN * 400];
  printf("{");

  /* ---- run_host on page-locked slots (the Go Slots.Run path) */
  {
    uint8_t *data;
    CHECK(sqobfs_host_alloc(ctx, 2ull * MAXN * SLOT, (void **)&data));
    static uint64_t in_off[MAXN], out_off[MAXN];
    static uint32_t in_len[MAXN], out_len[MAXN];
    static uint8_t salt[8 * MAXN];
    for (int i = 0; i < MAXN; i++) {
      in_off[i] = (uint64_t)i * SLOT;
      out_off[i] = (uint64_t)(MAXN + i) * SLOT;
      in_len[i] = L;
    }
    memset(data, 7, 2ull * MAXN * SLOT);
    printf("\"run_host\": {");
    for (int k = 0; k < NS; k++) {
      const int n = SIZES[k], it = iters_for(n);
      sqobfs_batch b;
      memset(&b, 0, sizeof b);
      b.n = (uint32_t)n;
      b.flags = SQOBFS_FLAG_OUT_UNINIT;
      b.in = data;
      b.in_off = in_off;
      b.in_len = in_len;
      b.out = data;
      b.out_off = out_off;
      b.out_len = out_len;
      b.salt = salt;
      for (int w = 0; w < 20; w++) CHECK(sqobfs_run_host(ctx, kr, SQOBFS_OBFUSCATE, &b));
      for (int i = 0; i < it; i++) {
        const double t0 = now_us();
        CHECK(sqobfs_run_host(ctx, kr, SQOBFS_OBFUSCATE, &b));
        v[i] = now_us() - t0;
      }
      char nm[16];
      snprintf(nm, sizeof nm, "%d", n);
      print_stat(nm, v, it, k == NS - 1);
    }
    printf("}, ");
    sqobfs_host_free(ctx, data);
  }

  /* ---- one launch on mapped slots + wait, per unit size */
  {
    uint8_t *blk;
    const size_t slots = (size_t)MAXN * SLOT;
    CHECK(sqobfs_host_alloc(ctx, slots + (size_t)MAXN * 24, (void **)&blk));
    uint64_t *in_off = (uint64_t *)(blk + slots), *out_off = in_off + MAXN;
    uint32_t *len = (uint32_t *)(out_off + MAXN), *out_len = len + MAXN;
    for (int i = 0; i < MAXN; i++) {
      in_off[i] = (uint64_t)i * SLOT + 8;
      out_off[i] = (uint64_t)i * SLOT;
      len[i] = L;
    }
    void *s = sqobfs_stream(ctx);
    CHECK(sqobfs_set_sync_spin(ctx, 500));
    static const uint32_t units[] = {0, 1, 2, 4, 8, 16, 26};
    printf("\"mapped\": {");
    for (int u = 0; u < 7; u++) {
      CHECK(sqobfs_set_unit_packets(ctx, units[u]));
      if (units[u]) printf("\"unit_%u\": {", units[u]);
      else printf("\"unit_auto\": {");
      for (int k = 0; k < NS; k++) {
        const int n = SIZES[k], it = iters_for(n);
        if (units[u] && n != MAXN) continue; /* the sweep is for the 256 batch */
        sqobfs_batch b;
        memset(&b, 0, sizeof b);
        b.n = (uint32_t)n;
        b.flags = SQOBFS_FLAG_DEVICE_SALT;
        b.in = blk;
        b.in_off = in_off;
        b.in_len = len;
        b.out = blk;
        b.out_off = out_off;
        b.out_len = out_len;
        for (int w = 0; w < 20; w++) {
          CHECK(sqobfs_launch(ctx, kr, SQOBFS_OBFUSCATE, &b, s));
          CHECK(sqobfs_sync(ctx, s));
        }
        for (int i = 0; i < it; i++) {
          const double t0 = now_us();
          CHECK(sqobfs_launch(ctx, kr, SQOBFS_OBFUSCATE, &b, s));
          CHECK(sqobfs_sync(ctx, s));
          v[i] = now_us() - t0;
        }
        char nm[16];
        snprintf(nm, sizeof nm, "%d", n);
        print_stat(nm, v, it, units[u] || k == NS - 1);
      }
      printf("}%s", u == 6 ? "" : ", ");
    }
    printf("}, ");
    CHECK(sqobfs_set_unit_packets(ctx, 0));
    CHECK(sqobfs_set_sync_spin(ctx, 0));
    sqobfs_host_free(ctx, blk);
  }

  /* ---- endpoint: sqobfs_udp_conn_write to a loopback socket */
  {
    uint16_t pa, pp;
    int fa = udp_socket(&pa), fp = udp_socket(&pp);
    sqobfs_udp_conn *c;
    CHECK(sqobfs_udp_conn_open(ctx, kr, &fa, 1, MAXN, SLOT, &c));
    static sqobfs_addr to[MAXN];
    static uint32_t len[MAXN];
    for (int i = 0; i < MAXN; i++) {
      to[i] = loop_addr(pp);
      len[i] = L;
      memset(sqobfs_udp_conn_tx_payload(c, (uint32_t)i), 3, L);
    }
    uint8_t buf[4096];
    printf("\"endpoint\": {");
    for (int k = 0; k < NS; k++) {
      const int n = SIZES[k], it = iters_for(n) / 2;
      for (int i = 0; i < it + 10; i++) {
        uint32_t sent;
        const double t0 = now_us();
        CHECK(sqobfs_udp_conn_write(c, 0, (uint32_t)n, len, to, &sent));
        for (int j = 0; j < n; j++)
          if (recv_to(fp, buf, sizeof buf, 2000) < 0) exit(2);
        if (i >= 10) v[i - 10] = now_us() - t0;
      }
      char nm[16];
      snprintf(nm, sizeof nm, "%d", n);
      print_stat(nm, v, it, k == NS - 1);
    }
    printf("}, ");
    sqobfs_udp_conn_close(c);
    close(fa);
    close(fp);
  }

  /* ---- pconn: WriteTo bursts -> arrival; peer bursts -> ReadFrom, with the
   * engine's defaults (inline writes when idle, small batches on the CPU
   * path) and with every batch launched on the GPU (round 3's engine) */
  sqobfs_pconn_opts gpu_only;
  memset(&gpu_only, 0, sizeof gpu_only);
  gpu_only.cpu_max = SQOBFS_PCONN_NEVER;
  gpu_only.inline_gap_us = SQOBFS_PCONN_NEVER;
  pconn_lat(ctx, kr, "", NULL);
  pconn_lat(ctx, kr, "_gpu_only", &gpu_only);
  {  /* no GPU at all: a host keyring and the host engine */
    sqobfs_keyring *hk;
    uint64_t o0 = 0;
    uint32_t l0 = PL;
    CHECK(sqobfs_keyring_create(NULL, SQOBFS_SALAMANDER, 1, PSK, &o0, &l0, &hk));
    pconn_lat(NULL, hk, "_no_device", NULL);
    sqobfs_keyring_destroy(hk);
  }
  /* the GPU context's engine with every batch on the CPU path, and the
   * defaults again (after the no-device run: order effects) */
  sqobfs_pconn_opts cpu_only;
  memset(&cpu_only, 0, sizeof cpu_only);
  cpu_only.cpu_max = 1u << 30;
  pconn_lat(ctx, kr, "_cpu_only", &cpu_only);
  pconn_lat(ctx, kr, "_defaults_again", NULL);

  /* ---- pconn throughput: pconn A -> pconn B over loopback, one writer
   * thread (the Go Conn's WriteTo callers), one reader thread; without and
   * with UDP GSO (A) / GRO (B); with the engine's routing (defaults), every
   * batch launched (_gpu_only), every batch on the CPU path (_cpu_only) and
   * on the host engine (_no_device), with batches held up to 20 us for more
   * datagrams (_linger20); the defaults again last (order effects) */
  {
    sqobfs_keyring *hk;
    uint64_t o0 = 0;
    uint32_t l0 = PL;
    CHECK(sqobfs_keyring_create(NULL, SQOBFS_SALAMANDER, 1, PSK, &o0, &l0, &hk));
    static const char *const modes[] = {"", "_gpu_only", "_cpu_only", "_no_device",
                                        "_linger20", "_defaults_again"};
    for (int m = 0; m < 6; m++)
      for (int off = 0; off < 2; off++) {
        sqobfs_ctx *const c = m == 3 ? NULL : ctx;
        sqobfs_keyring *const k = m == 3 ? hk : kr;
        uint16_t pa, pb;
        int fa = udp_socket(&pa), fb = udp_socket(&pb);
        sqobfs_pconn *A, *B;
        sqobfs_pconn_opts oa, ob;
        memset(&oa, 0, sizeof oa);
        memset(&ob, 0, sizeof ob);
        oa.flags = off ? SQOBFS_UDP_TX_GSO : 0u;
        ob.flags = off ? SQOBFS_UDP_RX_GRO : 0u;
        if (m == 1) oa.cpu_max = ob.cpu_max = oa.inline_gap_us = ob.inline_gap_us = SQOBFS_PCONN_NEVER;
        if (m == 2) oa.cpu_max = ob.cpu_max = 1u << 30;
        if (m == 4) oa.linger_us = ob.linger_us = 20;
        CHECK(sqobfs_pconn_open(c, k, fa, &oa, &A));
        CHECK(sqobfs_pconn_open(c, k, fb, &ob, &B));
        const sqobfs_addr to = loop_addr(pb);
        static uint8_t pay[L];
        memset(pay, 9, L);
        struct rd {
          sqobfs_pconn *pc;
          long got;
          double last_us;
        } r = {B, 0, 0};
        pthread_t th;
        extern void *tput_reader(void *);
        pthread_create(&th, NULL, tput_reader, &r);
        const long N = 200000;
        const double t0 = now_us();
        for (long i = 0; i < N; i++) {
          CHECK(sqobfs_pconn_write(A, pay, L, &to, 0));
          if ((i & 1023) == 1023) {
            /* stay inside the loopback socket buffers (UDP drops, the test
             * counts what arrives) */
            struct timespec ts = {0, 200000};
            nanosleep(&ts, NULL);
          }
        }
        const double tw = now_us();
        CHECK(sqobfs_pconn_set_deadline(B, SQOBFS_PCONN_READ, 0));
        pthread_join(th, NULL);
        const double dt = (r.last_us - t0) * 1e-6;  /* to the last datagram's arrival */
        sqobfs_pconn_stats sa, sb;
        CHECK(sqobfs_pconn_stats_get(A, &sa));
        CHECK(sqobfs_pconn_stats_get(B, &sb));
        sqobfs_engine_info ei;
        CHECK(sqobfs_engine_info_get(c, &ei));
        printf("\"pconn_throughput%s%s\": {\"datagrams\": %ld, \"received\": %ld, \"seconds\": %.3f, "
               "\"write_seconds\": %.3f, \"datagrams_per_s\": %.0f, \"payload_gib_s\": %.3f, "
               "\"tx_batches\": %llu, \"rx_batches\": %llu, \"tx_cpu_batches\": %llu, "
               "\"rx_cpu_batches\": %llu, \"inline_writes\": %llu, \"route_bytes\": %llu, "
               "\"launch_us\": %u, \"cpu_ns_per_kib\": %u}, ",
               modes[m], off ? "_gso_gro" : "", N, r.got, dt, (tw - t0) * 1e-6, r.got / dt,
               r.got * (double)L / dt / (1 << 30), (unsigned long long)sa.tx_batches,
               (unsigned long long)sb.rx_batches, (unsigned long long)sa.cpu_batches,
               (unsigned long long)sb.cpu_batches, (unsigned long long)sa.inline_writes,
               (unsigned long long)ei.route_bytes, ei.launch_us, ei.cpu_ns_per_kib);
        fflush(stdout);
        sqobfs_pconn_close(A);
        sqobfs_pconn_close(B);
        close(fa);
        close(fb);
      }
    sqobfs_keyring_destroy(hk);
  }

  /* ---- the reference's per-datagram work, one core (oracle byte loops) */
  {
    static uint8_t pay[L], wire[L + 8];
    uint8_t salt[8] = {1};
    for (int i = 0; i < 2000; i++) {
      const double t0 = now_us();
      or_salamander_write(PSK, PL, salt, pay, L, wire);
      v[i] = now_us() - t0;
    }
    printf("\"cpu_oracle_write_1350B\": {\"p50_us\": %.2f, \"p99_us\": %.2f}", pct(v, 2000, 0.5),
           pct(v, 2000, 0.99));
  }
  printf("}\n");
  sqobfs_keyring_destroy(kr);
  sqobfs_close(ctx);
  return 0;
}
