// pconn.cpp -- the obfuscating packet conn engine (include/sqobfs.h,
// "Obfuscating packet conn" and "The engine"): the batching core under the
// Go decorators go/sqobfs.Conn, written here so that its behaviour
// (coalescing, deadlines, shutdown, memory, failure handling) is the same for
// every host language and is tested natively (tests/cpp/test_pconn.c, on the
// GPU and, over the CPU device of tests/cpp/sq_devstub.cpp, under ASan and
// TSan).
//
// Reference: SalamanderPacketConn / XPlusPacketConn (hysteria2/salamander.go:
// 19-109, hysteria/xplus.go:39-118) transform one datagram per ReadFrom /
// WriteTo call on the caller's goroutine, and cannot fail to be constructed.
// Here the per-call contract stays (one datagram in or out per call, the
// reference's return values) and the byte work moves into batches:
//
//   write()  -> fill batch --(full, or the engine is idle)--> worker:
//               obfuscate in place -> sendmmsg | tx_take
//   epoll -> worker: recvmmsg | rx_push -> rx batch -> deobfuscate in place
//               -> ready queue -> read() copies one datagram out
//
// ONE engine per context serves every pconn on it: a fixed pool of worker
// threads (each with its own HIP stream), one poller thread (epoll over the
// sockets) and a pool of batch blocks (page-locked, GPU-mapped) that pconns
// take while a batch fills, flies or waits to be read, and give back after.
// So pconns -- one per hop socket of a port-hopping client, hop.go:114 --
// cost no threads of their own, and pinned memory follows the datagrams in
// flight.
//
// Where the bytes are transformed, per batch:
//   * on the GPU, one launch, when the batch's cost (payload bytes + 1 KiB
//     per datagram) exceeds opts.cpu_max -- by default a measured
//     break-even: the engine's recent launch round trip times its recent
//     CPU-path rate (route_bytes), so a batch goes to the GPU when the CPU
//     would take longer than a launch -- or, under sustained load, when the
//     CPU path would cost the host more than a launch does; the batches
//     other pconns have queued then join that launch (run_task);
//   * on the CPU (sq_cpu.h) otherwise, and always without a context (no GPU:
//     the drop-in constructors never fail), and for good after a launch
//     fails (a batch whose launch was refused is redone on the CPU; one whose
//     kernel failed after it started is dropped, as a lost datagram);
//   * inline: a write made while the transmit side is idle (and the previous
//     write is opts.inline_gap_us old) is obfuscated and sent on the writer's
//     own thread, and its send error is that call's -- the reference's
//     behaviour, for handshakes, ACKs and keep-alives.
// Natural batching: a worker takes whatever has accumulated as soon as it is
// free, and the datagrams written during a launch form the next batch.
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/udp.h>
#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/prctl.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "sq_cpu.h"
#include "sq_internal.h"
#include "sq_sockaddr.h"
#include "sqobfs.h"

namespace {

constexpr uint32_t kDefBatch = 256, kDefSlot = 2048, kDefBatches = 8, kDefSpinUs = 200;
// routing (opts.cpu_max 0): the CPU path's cost estimate before it is
// measured, and the bounds of the measured break-even
constexpr uint32_t kDefCpuNsPerKiB = 500;
constexpr uint64_t kRouteMin = 16u << 10, kRouteMax = 4u << 20;
constexpr uint64_t kRouteSample = 8u << 10;  // CPU batches at least this costly update the rate
constexpr uint32_t kHashCost = 1024;      // one key derivation ~ 1 KiB of XOR on a core
// load-aware routing (cpu_max 0): the engine's transform demand -- the
// CPU-path time its batches would take per wall second, in per mille of one
// core, measured over windows of kLoadWindowNs -- above kLoadOnPermille turns
// "loaded" on (off again below kLoadOffPermille).  Loaded, the host's CPU
// time is what the routing saves, not a batch's latency: a batch of more
// than kLoadMinDgrams datagrams launches (and waits without polling) when
// its CPU-path time is more than twice what a launch costs the host (the
// margin: a launched batch also waits ~3x longer) -- the worker
// thread's own CPU time per launched batch, launch call and blocking wait,
// measured (gpu_host_ns) -- so bulk traffic costs the host the launch and
// the socket work, not the bytes
constexpr int64_t kLoadWindowNs = 10'000'000;
constexpr uint32_t kLoadOnPermille = 100, kLoadOffPermille = 50;
constexpr uint32_t kLoadMinDgrams = 64;
constexpr uint32_t kDefGpuHostNs = 20'000;  // before the first launch is measured
constexpr uint32_t kDefInlineGapUs = 100;
constexpr uint32_t kDefWorkers = 4, kMaxWorkers = 64;
constexpr uint32_t kMaxBatch = 1u << 16;
constexpr int64_t kDrainNs = 200'000'000;  // shutdown: time given to queued writes
constexpr int64_t kAttachRetryNs = 1'000'000;  // socket rx: retry a failed block allocation
constexpr uint32_t kMmsg = 256;            // messages per sendmmsg / recvmmsg call
constexpr uint32_t kGsoMaxSegs = 64;       // UDP_MAX_SEGMENTS of older kernels
constexpr uint32_t kGsoMaxBytes = 65000;   // one GSO send stays below 64 KiB of IP payload
constexpr uint32_t kGroBuf = 65536;        // one coalesced receive
constexpr size_t kCtlWords = (CMSG_SPACE(sizeof(uint16_t)) + 7) / 8;
// one launch over several pconns' batches (run_task): at most group_max
// batches (sqobfs_engine_set_group) and kGroupDgrams datagrams; a merged
// keyring is made anew past kMergedMax PSKs
constexpr uint32_t kDefGroup = 32, kMaxGroup = 64, kGroupDgrams = 16384, kMergedMax = 256;
// launches in flight at once per engine (one stream each); a worker that
// would start one more waits for a stream
constexpr uint32_t kMaxFlights = 32;
// non-polling launches in flight at once (run_task): past it, the batches
// routed to the GPU wait, prepared, and the next completion launches all of
// them together -- the natural batching of the GPU route
constexpr uint32_t kDefFlightCap = 1;
// datagrams waiting for the launch slot past which a bulk batch overflows to
// the CPU path (gpu_saturated).  lat_bench hops 8 unpaced, in-process
// against the CPU path: 8,192 / 4,096 / 2,048 waiting datagrams 0.7-1.2x its
// rate, 256 1.09-1.20x in four runs on three boxes at less host CPU per GiB,
// 128 0.9-1.27x
constexpr uint32_t kDefPendMax = 256;

// sqobfs_debug_engine_fail, sqobfs_debug_pool_fail, sqobfs_debug_engine_hold
std::atomic<int> g_fail_count{0};
std::atomic<int> g_fail_at_completion{0};
std::atomic<int> g_pool_fail{0};
std::atomic<bool> g_hold{false};

// take one unit of a test hook's countdown
bool take_one(std::atomic<int> &c) {
  for (int v = c.load(); v > 0;)
    if (c.compare_exchange_weak(v, v - 1)) return true;
  return false;
}

int64_t unix_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}
int64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}
int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}
std::chrono::system_clock::time_point wall_tp(int64_t ns) {
  return std::chrono::system_clock::time_point(
      std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::nanoseconds(ns)));
}
std::chrono::steady_clock::time_point mono_tp(int64_t ns) {
  return std::chrono::steady_clock::time_point(
      std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::nanoseconds(ns)));
}

// One batch's memory, from the engine pool: the slots, then per datagram
// two u64 and two u32 arrays (the kernel reads and writes them in place).
struct Block {
  void *mem = nullptr;
  size_t bytes = 0;
  uint32_t B = 0, slot = 0;
  uint8_t *slots = nullptr;
  uint64_t *in_off = nullptr, *out_off = nullptr;
  uint32_t *len = nullptr, *out_len = nullptr;
};

// One batch of a pconn.  Its block is taken from the pool when the batch
// starts filling (or receiving) and given back when it is free again.
struct PBatch {
  Block *blk = nullptr;
  uint32_t n = 0;       // datagrams in the batch
  uint32_t next = 0;    // rx: next datagram read() hands out
  int64_t first_ns = 0; // monotonic time of the first datagram (linger)
  std::vector<sqobfs_addr> addr;
  std::vector<uint64_t> tag;
  std::vector<uint8_t> head;  // rx: the first 16 wire bytes of each datagram
};

enum { kTx = 0, kRx = 1 };

struct Engine;

}  // namespace

struct sqobfs_pconn {
  Engine *eng = nullptr;
  sqobfs_ctx *ctx = nullptr;
  const sqobfs_keyring *kr = nullptr;
  const sq::PskEntry *psk0 = nullptr;  // the keyring's host entry 0 (inline writes)
  int kind = 0;
  uint32_t S = 0;
  uint64_t id = 0;  // the engine's handle (epoll data)
  int fd = -1;      // socket mode: our dup of the caller's socket
  int wake = -1;    // eventfd, readable after shutdown (wakes a blocked send)
  sqobfs_pconn_opts o{};
  std::vector<PBatch> tb, rb;

  // ---- under mu
  std::mutex mu;
  std::condition_variable cv_txs;   // writers: a tx batch freed; shutdown: drained
  std::condition_variable cv_rxr;   // readers: a batch is ready
  std::condition_variable cv_rxs;   // pushers: an rx batch freed
  std::condition_variable cv_take;  // pump taker: an obfuscated batch is ready
  std::deque<uint32_t> tfree, tq, ttaken, rfree, rq, rready;
  int tfill = -1, rfill = -1;
  bool tx_busy = false;      // a worker is transforming / sending a tx batch
  bool taken = false;        // pump: the front of ttaken is out with the taker
  bool inline_busy = false;  // a writer is sending inline
  bool rx_stall = false;     // socket rx waits for a free batch (read() reschedules)
  bool rx_dead = false;      // the socket failed for good: no more receives
  bool writes_closed = false;
  bool closed = false;
  int tx_err = 0;            // reported once by the next write
  int rx_err = 0;            // reported once the ready queue is empty
  bool rx_err_sticky = false;
  int64_t rdl = 0, wdl = 0;  // deadlines, unix ns (0 = none)
  int64_t last_write_ns = 0;
  sqobfs_pconn_stats st{};
  std::vector<uint8_t> ibuf;  // the inline writer's datagram

  // ---- under eng->mu
  bool sched[2] = {false, false};  // a tx / rx task is queued, timed or running
  bool timed[2] = {false, false};  // ... waiting for its linger deadline
  bool again[2] = {false, false};  // work arrived while it ran: run it once more
  uint32_t tasks = 0;

  // socket I/O scratch, used by the one task of each direction at a time
  std::vector<mmsghdr> tmsg, rmsg;
  std::vector<iovec> tiov, riov;
  std::vector<sockaddr_storage> tss, rss;
  std::vector<uint64_t> tctl, rctl;  // UDP_SEGMENT / UDP_GRO control messages
  std::vector<uint32_t> tfirst;      // first datagram of each transmit message
  bool gso = false, gro = false;     // offloads in effect (socket mode)

  bool socket_mode() const { return fd >= 0; }
  uint8_t *slot(PBatch &b, uint32_t i) { return b.blk->slots + (size_t)i * o.slot_bytes; }
};

namespace {

struct Job;
struct Flight;

struct Task {
  sqobfs_pconn *pc;
  int dir;               // kTx / kRx
  Flight *fin = nullptr;  // set: finish these landed socket-mode batches of the
                          // pconn, in order (completer_main)
};

// A keyring the engine made for coalesced launches over pconns with
// different keyrings: copies of their entry 0 (merged_keyring).
struct MergedKeyring {
  sqobfs_keyring *kr = nullptr;
  std::vector<sq::PskEntry> e;
  uint32_t hot_m = 0, hot_iv = 1;
  MergedKeyring() = default;
  MergedKeyring(const MergedKeyring &) = delete;
  MergedKeyring &operator=(const MergedKeyring &) = delete;
  ~MergedKeyring() {
    if (kr) sqobfs_keyring_destroy(kr);  // (stream-ordered after its launches)
  }
};

struct Engine {
  sqobfs_ctx *ctx = nullptr;  // NULL: the host engine (CPU only)
  uint32_t nworkers = kDefWorkers;
  std::mutex mu;
  std::condition_variable cv;       // workers: a task is queued / a timer changed / stop
  std::condition_variable cv_idle;  // a pconn's last task ended
  std::deque<Task> runq;
  std::vector<std::pair<int64_t, Task>> timers;  // linger deadlines (monotonic ns)
  std::unordered_map<uint64_t, sqobfs_pconn *> byid;
  uint64_t next_id = 1;
  uint32_t pconns = 0;
  bool stop = false;
  std::vector<std::thread> threads;
  int epfd = -1, wake = -1;
  // launches in flight (under cmu): the streams (made on demand, at most
  // kMaxFlights, each carrying one launch at a time) and the launches the
  // completer thread waits for, in launch order
  std::mutex cmu;
  std::condition_variable cv_flight;  // the completer: a launch was queued / stop
  std::condition_variable cv_stream;  // a worker: a stream was given back
  std::vector<void *> streams, sfree;
  std::deque<Flight *> flights;
  std::vector<Job> pending;  // routed to the GPU while flight_cap launches fly
  uint32_t pending_dgrams = 0;
  uint32_t pend_max = kDefPendMax;  // past it, bulk batches overflow to the CPU path
  // (round 6 swept both in lat_bench hops: flight caps 1 / 2 / 4 and
  // overflow at 0 / 2,048 / 4,096 / 8,192 datagrams)
  uint32_t nflight = 0;     // non-polling launches started and not yet landed
  uint32_t flight_cap = kDefFlightCap;
  bool cstop = false;
  std::atomic<uint64_t> async_launches{0};
  std::atomic<bool> gpu_off{false};
  std::atomic<uint32_t> launch_us{40};  // recent launch completion time (EWMA)
  std::atomic<uint32_t> cpu_ns_kib{kDefCpuNsPerKiB};  // recent CPU-path ns per KiB of cost (EWMA)
  // load-aware routing: demand in the current window, its start, the
  // smoothed demand (permille of the workers' time) and the state
  std::atomic<uint64_t> demand_ns{0};
  std::atomic<int64_t> win_t0{0};
  std::atomic<uint32_t> load_pm{0};
  std::atomic<bool> loaded{false};
  std::atomic<uint32_t> gpu_host_ns{kDefGpuHostNs};  // host CPU per launched batch (EWMA)
  // non-polling waits: the time from launch to the completion the wait saw
  // (EWMA, us); the wait sleeps 3/4 of it, then polls, so the estimate
  // tracks the kernel and not the wait's own sleep
  std::atomic<uint32_t> kern_us{30};
  // coalesced launches (run_task): the most batches one takes, the merged
  // keyrings of each scheme, and counts
  std::atomic<uint32_t> group_max{kDefGroup};
  std::mutex mkr_mu;
  std::shared_ptr<MergedKeyring> mkr[2];
  std::atomic<uint64_t> launches{0}, group_launches{0}, group_batches{0};

  // the CPUs the engine's threads run on (sqobfs_engine_set_affinity);
  // ncpus 0: not restricted
  cpu_set_t cpus;
  uint32_t ncpus = 0;

  std::mutex pool_mu;
  std::map<std::pair<uint32_t, uint32_t>, std::vector<Block *>> free_blocks;
  uint32_t blocks = 0, in_use = 0;
  uint64_t pool_bytes = 0;
};

// ---- waiting on a condition with a deadline (unix ns, 0 = none): returns
// false when the deadline has passed
template <class Pred>
bool wait_dl(std::unique_lock<std::mutex> &lk, std::condition_variable &cv, const int64_t &dl,
             Pred ready) {
  while (!ready()) {
    const int64_t d = dl;  // re-read: set_deadline may move it while we wait
    if (d) {
      if (unix_ns() >= d) return false;
      cv.wait_until(lk, wall_tp(d));
    } else {
      cv.wait(lk);
    }
  }
  return true;
}

// ---------------------------------------------------------------- registry

std::mutex g_eng_mu;
std::map<sqobfs_ctx *, Engine *> g_engines;     // ctx NULL: the host engine (never ended)
std::map<sqobfs_ctx *, uint32_t> g_workers_cfg;  // sqobfs_engine_set_workers
std::map<sqobfs_ctx *, int> g_affinity_cfg;      // sqobfs_engine_set_affinity
std::map<sqobfs_ctx *, uint32_t> g_group_cfg;    // sqobfs_engine_set_group

// L3 (CCD) id of a CPU from sysfs; -1 when unknown
int l3_of(int cpu) {
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/id", cpu);
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  int id = -1;
  if (fscanf(f, "%d", &id) != 1) id = -1;
  fclose(f);
  return id;
}

// The CPUs of the process's affinity that share the calling thread's L3:
// the engine's threads stay together, next to the thread that started it.
// Measured ("the small-batch regime"): threads spread over
// 2-4 CCDs of the GPU box ran 5 of 45 loopback throughput runs at 0.9-1.3
// M datagrams/s; kept on one L3, 0 of 45, and +26 % at the median.
uint32_t l3_cpus(cpu_set_t *out) {
  CPU_ZERO(out);
  cpu_set_t cur;
  if (sched_getaffinity(0, sizeof cur, &cur)) return 0;
  const int me = sched_getcpu(), l3 = me >= 0 ? l3_of(me) : -1;
  if (l3 < 0) return 0;
  uint32_t n = 0;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &cur) && l3_of(c) == l3) {
      CPU_SET(c, out);
      n++;
    }
  return n >= 2 ? n : 0;  // (one CPU: leave the threads free)
}

void engine_thread_pin(const Engine *E) {
  if (E->ncpus) (void)pthread_setaffinity_np(pthread_self(), sizeof E->cpus, &E->cpus);
  // the sleeps of non-polling launch waits wake within ~1 us, not the
  // default 50 us of timer slack
  (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
}

void worker_main(Engine *E);
void poller_main(Engine *E);
void completer_main(Engine *E);

Engine *engine_get(sqobfs_ctx *ctx, int *status) {
  std::lock_guard<std::mutex> g(g_eng_mu);
  auto it = g_engines.find(ctx);
  if (it != g_engines.end()) return it->second;
  Engine *E = new (std::nothrow) Engine();
  if (!E) {
    *status = SQ_ENOMEM;
    return nullptr;
  }
  E->ctx = ctx;
  auto c = g_workers_cfg.find(ctx);
  if (c != g_workers_cfg.end() && c->second) E->nworkers = c->second;
  auto a = g_affinity_cfg.find(ctx);
  const int aff = a != g_affinity_cfg.end() ? a->second : SQOBFS_ENGINE_AFFINITY_L3;
  if (aff == SQOBFS_ENGINE_AFFINITY_L3) E->ncpus = l3_cpus(&E->cpus);
  auto gc = g_group_cfg.find(ctx);
  if (gc != g_group_cfg.end()) E->group_max = gc->second;
  E->wake = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  E->epfd = epoll_create1(EPOLL_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = 0;  // id 0: the engine's wake fd
  if (E->wake < 0 || E->epfd < 0 || epoll_ctl(E->epfd, EPOLL_CTL_ADD, E->wake, &ev) != 0) {
    if (E->wake >= 0) close(E->wake);
    if (E->epfd >= 0) close(E->epfd);
    delete E;
    *status = SQ_ENOMEM;
    return nullptr;
  }
  try {
    E->streams.reserve(kMaxFlights);
    E->sfree.reserve(kMaxFlights);
    for (uint32_t w = 0; w < E->nworkers; w++) E->threads.emplace_back(worker_main, E);
    E->threads.emplace_back(poller_main, E);
    if (ctx) E->threads.emplace_back(completer_main, E);
  } catch (...) {
    {
      std::lock_guard<std::mutex> lk(E->mu);
      E->stop = true;
    }
    {
      std::lock_guard<std::mutex> lk(E->cmu);
      E->cstop = true;
    }
    E->cv.notify_all();
    E->cv_flight.notify_all();
    const uint64_t one = 1;
    (void)!write(E->wake, &one, sizeof one);
    for (auto &t : E->threads) t.join();
    close(E->wake);
    close(E->epfd);
    delete E;
    *status = SQ_ENOMEM;
    return nullptr;
  }
  g_engines[ctx] = E;
  return E;
}

// ---------------------------------------------------------------- block pool

Block *block_take(Engine *E, uint32_t B, uint32_t slot) {
  if (take_one(g_pool_fail)) return nullptr;  // (test hook: an allocation failure)
  std::lock_guard<std::mutex> g(E->pool_mu);
  auto &fl = E->free_blocks[{B, slot}];
  if (!fl.empty()) {
    Block *b = fl.back();
    fl.pop_back();
    E->in_use++;
    return b;
  }
  Block *b = new (std::nothrow) Block();
  if (!b) return nullptr;
  const size_t slots = (size_t)B * slot, arrays = (size_t)B * (8 + 8 + 4 + 4);
  b->bytes = slots + arrays;
  if (E->ctx) {
    if (sq_host_alloc_mapped(E->ctx, b->bytes, &b->mem) != SQ_OK) b->mem = nullptr;
  } else {
    b->mem = aligned_alloc(4096, (b->bytes + 4095) / 4096 * 4096);
  }
  if (!b->mem) {
    delete b;
    return nullptr;
  }
  uint8_t *p = (uint8_t *)b->mem;
  b->B = B;
  b->slot = slot;
  b->slots = p;
  p += slots;
  b->in_off = (uint64_t *)p;
  p += 8ull * B;
  b->out_off = (uint64_t *)p;
  p += 8ull * B;
  b->len = (uint32_t *)p;
  p += 4ull * B;
  b->out_len = (uint32_t *)p;
  E->blocks++;
  E->in_use++;
  E->pool_bytes += b->bytes;
  return b;
}

void block_free_mem(Engine *E, Block *b) {
  if (E->ctx) sqobfs_host_free(E->ctx, b->mem);
  else free(b->mem);
  delete b;
}

void block_give(Engine *E, Block *b) {
  std::lock_guard<std::mutex> g(E->pool_mu);
  E->in_use--;
  E->free_blocks[{b->B, b->slot}].push_back(b);
}

// A batch's block, with the slot offsets of its direction: tx -- payload
// behind S bytes of headroom, wire = salt || payload in place from the slot
// start (the vectorised writers' layout, salamander.go:81-93); rx -- wire at
// the slot start, payload decoded in place behind the salt.
bool batch_attach(sqobfs_pconn *pc, PBatch &b, bool tx) {
  if (!b.blk) {
    b.blk = block_take(pc->eng, pc->o.batch, pc->o.slot_bytes);
    if (!b.blk) return false;
  }
  for (uint32_t i = 0; i < pc->o.batch; i++) {
    const uint64_t s0 = (uint64_t)i * pc->o.slot_bytes;
    b.blk->in_off[i] = tx ? s0 + pc->S : s0;
    b.blk->out_off[i] = tx ? s0 : s0 + pc->S;
  }
  return true;
}

void batch_detach(sqobfs_pconn *pc, PBatch &b) {
  if (b.blk) block_give(pc->eng, b.blk);
  b.blk = nullptr;
  b.n = 0;
  b.next = 0;
}

// ---------------------------------------------------------------- scheduling

// Queue the pconn's task of direction d unless one is queued, timed or
// running; a running one is told to run once more (`again`), so work that
// arrives while it finishes is never left behind.  Caller holds eng->mu.
void schedule_locked(Engine *E, sqobfs_pconn *pc, int d) {
  if (pc->sched[d]) {
    if (pc->timed[d]) {  // more work than the linger waits for: run now
      for (size_t k = 0; k < E->timers.size(); k++)
        if (E->timers[k].second.pc == pc && E->timers[k].second.dir == d) {
          E->timers.erase(E->timers.begin() + (long)k);
          break;
        }
      pc->timed[d] = false;
      E->runq.push_back({pc, d});
      E->cv.notify_one();
    } else {
      pc->again[d] = true;
    }
    return;
  }
  pc->sched[d] = true;
  pc->tasks++;
  E->runq.push_back({pc, d});
  E->cv.notify_one();
}

// Caller holds pc->mu (lock order: pc->mu, then eng->mu).
void schedule(sqobfs_pconn *pc, int d) {
  std::lock_guard<std::mutex> lk(pc->eng->mu);
  schedule_locked(pc->eng, pc, d);
}

// The calling thread is one of the engine's workers (worker_main), and the
// tasks it has requeued without a wake-up since the count was last reset.
thread_local bool t_worker = false;
thread_local uint32_t t_requeued = 0;

// The running task of direction d is done with the work it found: requeue
// (more work), park until `due` (linger), or end.  Caller holds pc->mu.
void task_end(sqobfs_pconn *pc, int d, bool more, int64_t due = 0) {
  Engine *E = pc->eng;
  std::lock_guard<std::mutex> lk(E->mu);
  if (pc->again[d]) {  // scheduled while running: look at once
    pc->again[d] = false;
    more = true;
    due = 0;
  }
  if (more && !pc->closed) {
    if (due) {
      pc->timed[d] = true;
      E->timers.push_back({due, {pc, d}});
      E->cv.notify_one();  // (a sleeping worker's deadline may be later)
    } else {
      // no wake-up: the calling worker goes back to the run queue next and
      // takes it itself.  Waking another worker for it made every batch a
      // hand-off between two threads (a futex wake and a context switch per
      // batch), which kept batches small at high rates (waking
      // one only when other tasks wait ahead brought that back: the tx and
      // rx tasks of a busy pair of conns are queued together most of the
      // time).  No task starves: a sleeping worker means the queue was empty
      // when it slept, and every task queued since came with a wake-up or,
      // like this one, with the worker that queued it.  (Off a worker -- the
      // completer finishing a launch -- there is no such worker: wake one.
      // A worker that requeues several, after a coalesced launch, wakes
      // others for the rest: run_task.)
      E->runq.push_back({pc, d});
      if (t_worker) t_requeued++;
      else E->cv.notify_one();
    }
    return;
  }
  pc->sched[d] = false;
  pc->tasks--;
  if (pc->tasks == 0) E->cv_idle.notify_all();
}

// ---------------------------------------------------------------- transform

// One task's batch between the task's prepare and finish steps, so that one
// worker can transform the batches of several tasks with one launch.
struct Job {
  sqobfs_pconn *pc = nullptr;
  int dir = kTx;        // the task's direction: kTx obfuscates, kRx deobfuscates
  uint32_t idx = 0;     // its batch: pc->tb[idx] / pc->rb[idx]
  bool slotted = true;  // datagrams in slots (not packed in GRO buffers)
  uint64_t trunc = 0;   // socket receive: truncated datagrams
  uint64_t cost = 0;    // payload bytes + kHashCost per datagram
  int st = SQ_OK;
  // cpu: transformed on the CPU path; failed: its launch failed and the
  // engine stays on the CPU; refused: its launch was refused for the moment
  // (redone on the CPU path, the GPU still on)
  bool cpu = false, failed = false, refused = false;
  // the last of its task's batches in this transform: its finish ends or
  // requeues the task (a launch may carry several batches of one task)
  bool end_task = true;
  PBatch &batch() const { return dir == kTx ? pc->tb[idx] : pc->rb[idx]; }
  int op() const { return dir == kTx ? SQOBFS_OBFUSCATE : SQOBFS_DEOBFUSCATE; }
};

constexpr int kRefused = 1;  // gpu_run: nothing ran

// The measured break-even cost: the CPU path would take a launch's round
// trip on a batch of this cost.
uint64_t route_bytes(const Engine *E) {
  const uint64_t l = E->launch_us.load(std::memory_order_relaxed);
  const uint64_t c = std::max<uint32_t>(1u, E->cpu_ns_kib.load(std::memory_order_relaxed));
  return std::min(kRouteMax, std::max(kRouteMin, l * 1000u * 1024u / c));
}

// Account a batch's transform demand (its estimated CPU-path time, whatever
// route it takes) and, once a window has passed, update the engine's load.
void note_demand(Engine *E, uint64_t cost) {
  const uint64_t est = cost * E->cpu_ns_kib.load(std::memory_order_relaxed) / 1024u;
  E->demand_ns.fetch_add(est, std::memory_order_relaxed);
  const int64_t now = mono_ns();
  int64_t t0 = E->win_t0.load(std::memory_order_relaxed);
  if (t0 == 0) {
    E->win_t0.compare_exchange_strong(t0, now);
    return;
  }
  if (now - t0 < kLoadWindowNs || !E->win_t0.compare_exchange_strong(t0, now)) return;
  const uint64_t d = E->demand_ns.exchange(0, std::memory_order_relaxed);
  const uint64_t pm = std::min<uint64_t>(100000, d * 1000u / (uint64_t)(now - t0));
  const uint32_t old = E->load_pm.load(std::memory_order_relaxed);
  const uint32_t sm = (uint32_t)((old + 3 * pm) / 4);  // (a window's jitter, damped)
  E->load_pm.store(sm, std::memory_order_relaxed);
  if (sm >= kLoadOnPermille) E->loaded.store(true, std::memory_order_relaxed);
  else if (sm < kLoadOffPermille) E->loaded.store(false, std::memory_order_relaxed);
}

// Where a job's batch is transformed (module comment): true for the GPU.
// Sets j.cost and *bulk (launched because of load: its wait does not poll).
bool route_gpu(Engine *E, Job &j, bool *bulk) {
  const PBatch &b = j.batch();
  const Block &k = *b.blk;
  uint64_t cost = 0;
  for (uint32_t i = 0; i < b.n; i++) cost += k.len[i] + kHashCost;
  j.cost = cost;
  const uint32_t cmax = j.pc->o.cpu_max;
  if (cmax == 0 && E->ctx) note_demand(E, cost);
  // loaded (cpu_max 0): a batch of more than kLoadMinDgrams launches when
  // the CPU path would cost the host more than a launch does
  *bulk = cmax == 0 && b.n > kLoadMinDgrams && E->loaded.load(std::memory_order_relaxed) &&
          cost * E->cpu_ns_kib.load(std::memory_order_relaxed) / 1024u >
              2ull * E->gpu_host_ns.load(std::memory_order_relaxed);
  return E->ctx && !E->gpu_off.load(std::memory_order_relaxed) &&
         (cmax == SQOBFS_PCONN_NEVER || *bulk ||
          cost > (cmax == 0 ? route_bytes(E) : (uint64_t)cmax));
}

// A job's batch as a descriptor over its own block.
void block_batch(const Job &j, sqobfs_batch &d) {
  const PBatch &b = j.batch();
  const Block &k = *b.blk;
  memset(&d, 0, sizeof d);
  d.n = b.n;
  d.in = k.slots;
  d.in_off = k.in_off;
  d.in_len = k.len;
  d.out = k.slots;
  d.out_off = k.out_off;
  d.out_len = k.out_len;
}

// The engine's keyring for one launch over the jobs' batches when their
// pconns hold different keyrings: one entry per distinct PSK state (the
// pconns' keyring entry 0, compared by content, so a keyring freed and
// another made at its address cannot alias), kept and extended while it has
// room, made anew past kMergedMax entries.  pid[j] = job j's entry.  NULL,
// with *st, when it cannot be made.
std::shared_ptr<MergedKeyring> merged_keyring(Engine *E, const Job *jobs, uint32_t nj,
                                              uint16_t *pid, void *stream, int *st) {
  const int kind = jobs[0].pc->kind;
  const int ki = kind == SQOBFS_SALAMANDER ? 0 : 1;
  auto find = [](const MergedKeyring *m, const sq::PskEntry *x) -> int {
    if (m)
      for (size_t i = 0; i < m->e.size(); i++)
        if (!memcmp(&m->e[i], x, sizeof *x)) return (int)i;
    return -1;
  };
  std::lock_guard<std::mutex> g(E->mkr_mu);
  std::shared_ptr<MergedKeyring> cur = E->mkr[ki];
  uint32_t j = 0;
  for (; j < nj; j++) {
    const int i = find(cur.get(), jobs[j].pc->psk0);
    if (i < 0) break;
    pid[j] = (uint16_t)i;
  }
  if (j == nj) return cur;
  std::shared_ptr<MergedKeyring> m;
  try {
    m = std::make_shared<MergedKeyring>();
    if (cur && cur->e.size() + nj <= kMergedMax) {
      m->e = cur->e;
      m->hot_m = cur->hot_m;
      m->hot_iv = cur->hot_iv;
    }
    for (j = 0; j < nj; j++) {
      int i = find(m.get(), jobs[j].pc->psk0);
      if (i < 0) {
        m->e.push_back(*jobs[j].pc->psk0);
        i = (int)m->e.size() - 1;
        uint32_t hm, hi;
        sq_keyring_hot(jobs[j].pc->kr, &hm, &hi);
        m->hot_m = std::max(m->hot_m, hm);
        m->hot_iv = std::min(m->hot_iv, hi);
      }
      pid[j] = (uint16_t)i;
    }
  } catch (...) {
    *st = SQ_ENOMEM;
    return nullptr;
  }
  *st = sq_keyring_from_entries(E->ctx, kind, m->e.data(), (uint32_t)m->e.size(), m->hot_m,
                                m->hot_iv, stream, &m->kr);
  if (*st != SQ_OK) return nullptr;
  E->mkr[ki] = m;  // (the old one is destroyed when its last launch lets go)
  return m;
}

// A launch from its start to its completion (gpu_launch .. gpu_land).  A
// launch whose wait does not poll -- bulk under load, or spin_us NEVER -- is
// completed by the engine's completer thread (completer_main), so the worker
// that made it goes back to the run queue at once (other pconns' batches,
// socket calls, hand-offs) instead of sleeping through the kernel and its
// round trip (~85 us); a polled launch (the latency route) is waited for by
// its own worker, which spins on it anyway.
struct Flight {
  Job jobs[kMaxGroup];
  uint32_t nj = 0;
  Block *gb = nullptr;                // a coalesced launch's descriptor block
  std::shared_ptr<MergedKeyring> mk;  // ... and its merged keyring
  void *stream = nullptr;
  int64_t t0 = 0;          // launch time (monotonic ns)
  int64_t launch_cpu = 0;  // the launching thread's CPU time in the launch call
  bool block = false;      // its wait does not poll
  int inject = 0;          // sqobfs_debug_engine_fail: 2 = the kernel "fails"
};

// A stream for one launch: a free one, a new one (at most kMaxFlights), or
// the next one given back.  NULL, with *st, when none can be made.
void *stream_take(Engine *E, int *st) {
  std::unique_lock<std::mutex> lk(E->cmu);
  for (;;) {
    if (E->cstop) {
      *st = SQ_ECLOSED;
      return nullptr;
    }
    if (!E->sfree.empty()) {
      void *s = E->sfree.back();
      E->sfree.pop_back();
      return s;
    }
    if (E->streams.size() < kMaxFlights) {  // (capacity reserved: no reallocation)
      void *s = nullptr;
      *st = sq_ctx_stream_create(E->ctx, &s);
      if (*st != SQ_OK) return nullptr;
      E->streams.push_back(s);
      return s;
    }
    E->cv_stream.wait(lk);
  }
}

void stream_give(Engine *E, void *s) {
  {
    std::lock_guard<std::mutex> lk(E->cmu);
    E->sfree.push_back(s);  // (capacity reserved)
  }
  E->cv_stream.notify_one();
}

// Starts the launch of f's jobs' batches on a stream of its own.  One batch:
// over its own block.  Several (coalesced, run_task): over one descriptor
// built in a block of the pool, every datagram addressed from the lowest of
// their blocks (blocks are mapped at their host addresses, so one base
// reaches them all), with per-datagram PSK ids into a merged keyring when
// the pconns' keyrings differ.  Returns SQ_OK (in flight: gpu_land completes
// it) or kRefused (nothing ran: the batches are intact, for the CPU path).
// A device failure turns the GPU off for the engine; a refusal of this batch
// or this moment (no memory for a stream, a block or a keyring) leaves the
// next batch free to launch.
int gpu_launch(Engine *E, Flight &f) {
  auto refused = [E, &f](int st) {
    if (st == SQ_EDEVICE || st == SQ_ENODEV) E->gpu_off.store(true);
    if (f.gb) block_give(E, f.gb);
    f.gb = nullptr;
    f.mk.reset();
    if (f.stream) stream_give(E, f.stream);
    f.stream = nullptr;
    return kRefused;
  };
  const Job *jobs = f.jobs;
  const uint32_t nj = f.nj;
  int st = SQ_OK;
  f.stream = stream_take(E, &st);
  if (!f.stream) return refused(st);
  const int op = jobs[0].op();
  const sqobfs_keyring *kr = jobs[0].pc->kr;
  sqobfs_batch d;
  bool slotted = jobs[0].slotted;
  if (nj == 1) {
    block_batch(jobs[0], d);
  } else {
    f.gb = block_take(E, kGroupDgrams, 16);  // (psk ids in its slot region)
    if (!f.gb) return refused(SQ_ENOMEM);
    bool same = true;
    for (uint32_t j = 1; j < nj; j++) same = same && jobs[j].pc->kr == kr;
    uint16_t pid[kMaxGroup] = {};
    if (!same) {
      f.mk = merged_keyring(E, jobs, nj, pid, f.stream, &st);
      if (!f.mk) return refused(st);
      kr = f.mk->kr;
    }
    uint8_t *base = jobs[0].batch().blk->slots;
    for (uint32_t j = 1; j < nj; j++) base = std::min(base, jobs[j].batch().blk->slots);
    Block *gb = f.gb;
    uint16_t *ids = (uint16_t *)gb->slots;
    uint32_t n = 0;
    for (uint32_t j = 0; j < nj; j++) {
      const PBatch &b = jobs[j].batch();
      const Block &k = *b.blk;
      const uint64_t delta = (uint64_t)(k.slots - base);
      for (uint32_t i = 0; i < b.n; i++, n++) {
        gb->in_off[n] = delta + k.in_off[i];
        gb->out_off[n] = delta + k.out_off[i];
        gb->len[n] = k.len[i];
        ids[n] = pid[j];
      }
      slotted = slotted && jobs[j].slotted;
    }
    memset(&d, 0, sizeof d);
    d.n = n;
    d.in = base;
    d.in_off = gb->in_off;
    d.in_len = gb->len;
    d.out = base;
    d.out_off = gb->out_off;
    d.out_len = gb->out_len;
    d.psk_id = same ? nullptr : ids;
  }
  // slots are multiples of 16 bytes: every output owns its blocks, so the
  // kernel writes them whole (SQOBFS_FLAG_OUT_BLOCKS); GRO buffers pack the
  // datagrams back to back (no flag)
  d.flags = (slotted ? SQOBFS_FLAG_OUT_BLOCKS : 0u) |
            (op == SQOBFS_OBFUSCATE ? SQOBFS_FLAG_DEVICE_SALT : 0u);
  f.inject = take_one(g_fail_count) ? (g_fail_at_completion.load() ? 2 : 1) : 0;
  f.t0 = mono_ns();
  const int64_t c0 = thread_cpu_ns();
  st = f.inject == 1 ? SQ_EDEVICE : sqobfs_launch(E->ctx, kr, op, &d, f.stream);
  f.launch_cpu = thread_cpu_ns() - c0;
  if (st != SQ_OK) return refused(st);
  E->launches.fetch_add(1, std::memory_order_relaxed);
  if (nj > 1) {
    E->group_launches.fetch_add(1, std::memory_order_relaxed);
    E->group_batches.fetch_add(nj, std::memory_order_relaxed);
  }
  return SQ_OK;
}

// Waits for f's launch -- polling up to twice the recent round trip (at most
// spin_us), or, for a non-polling one, asleep through 3/4 of the kernel's
// expected time from its start, then polling with short sleeps -- and
// completes it: the engine's estimates, out_len back into each block of a
// coalesced launch, the descriptor block and the stream given back.
// Returns SQ_OK, or the error of a kernel that failed (the batches,
// transformed in place, are lost; the GPU is off for the engine).
int gpu_land(Engine *E, Flight &f) {
  const int64_t c0 = thread_cpu_ns();
  const uint32_t ew = E->launch_us.load(std::memory_order_relaxed);
  int st;
  if (f.block) {
    const int64_t due = f.t0 + (int64_t)E->kern_us.load(std::memory_order_relaxed) * 750;
    const int64_t now = mono_ns();
    st = sq_ctx_stream_wait_blocking(E->ctx, f.stream,
                                     due > now ? (uint32_t)((due - now) / 1000) : 0u);
  } else {
    const uint32_t spin = std::min<uint32_t>(f.jobs[0].pc->o.spin_us, 2 * ew + 20);
    st = sq_ctx_stream_wait(E->ctx, f.stream, spin);
  }
  if (f.inject == 2) st = SQ_EDEVICE;
  if (st == SQ_OK) {
    const uint32_t us = (uint32_t)std::min<int64_t>((mono_ns() - f.t0) / 1000, 100000);
    E->launch_us.store((7 * ew + us) / 8, std::memory_order_relaxed);
    if (f.block) {  // the host's cost of a launched batch (polled waits would count their spin)
      E->kern_us.store((7 * E->kern_us.load(std::memory_order_relaxed) + us) / 8,
                       std::memory_order_relaxed);
      const uint32_t hn =
          (uint32_t)std::min<int64_t>(f.launch_cpu + thread_cpu_ns() - c0, 10'000'000);
      const uint32_t eh = E->gpu_host_ns.load(std::memory_order_relaxed);
      E->gpu_host_ns.store((7 * eh + hn) / 8, std::memory_order_relaxed);
    }
    if (f.gb) {
      uint32_t n = 0;
      for (uint32_t j = 0; j < f.nj; j++) {
        const PBatch &b = f.jobs[j].batch();
        for (uint32_t i = 0; i < b.n; i++) b.blk->out_len[i] = f.gb->out_len[n++];
      }
    }
  } else {
    // the kernel ran, in place, and failed: the slots' state is unknown
    E->gpu_off.store(true);
  }
  if (f.gb) block_give(E, f.gb);
  f.gb = nullptr;
  f.mk.reset();
  stream_give(E, f.stream);
  f.stream = nullptr;
  return st;
}

// Queues a started non-polling launch for the completer; false when it
// cannot (the engine is stopping, or no memory): its worker lands it.
bool flight_queue(Engine *E, Flight *f) {
  {
    std::lock_guard<std::mutex> lk(E->cmu);
    if (E->cstop) return false;
    try {
      E->flights.push_back(f);
    } catch (...) {
      return false;
    }
  }
  E->async_launches.fetch_add(1, std::memory_order_relaxed);
  E->cv_flight.notify_one();
  return true;
}

// The CPU path (sq_cpu.h) of a job's batch: salts of the context's stream,
// as a launch's.
int cpu_run(Engine *E, const Job &j) {
  sqobfs_pconn *pc = j.pc;
  const PBatch &b = j.batch();
  sqobfs_batch d;
  block_batch(j, d);
  uint32_t count = 0;
  const sq::PskEntry *tab = sq_keyring_host(pc->kr, &count);
  uint8_t sbuf[64 * 16];
  std::vector<uint8_t> sv;
  uint8_t *salts = nullptr;
  if (j.dir == kTx) {
    const size_t bytes = (size_t)b.n * pc->S;
    salts = sbuf;
    if (bytes > sizeof sbuf) {
      sv.resize(bytes);
      salts = sv.data();
    }
    uint32_t key[8];
    uint64_t seq;
    sq_salt_take(E->ctx, key, &seq);
    sq::cpu::salt_stream(key, seq, salts, bytes);
  }
  const int64_t t0 = mono_ns();
  const int st = sq::cpu::run_batch(pc->kind, j.op(), tab, count, &d, salts);
  if (j.cost >= kRouteSample) {  // (smaller batches: timer noise)
    const uint64_t ns = (uint64_t)std::max<int64_t>(0, mono_ns() - t0);
    const uint32_t now = (uint32_t)std::min<uint64_t>(1u << 20, ns * 1024u / j.cost);
    const uint32_t ew = E->cpu_ns_kib.load(std::memory_order_relaxed);
    E->cpu_ns_kib.store((7 * ew + now) / 8, std::memory_order_relaxed);
  }
  return st;
}

// ---------------------------------------------------------------- sending

// sendmmsg of a transmitted batch.  With GSO, consecutive datagrams to one
// address whose lengths are equal (the last of a run may be shorter) go out
// as one message with a UDP_SEGMENT control message (at most 64 datagrams /
// 65,000 bytes), each datagram still its own iovec in its slot; a socket
// that refuses turns GSO off and the rest goes one datagram per message.  A
// datagram (message) the socket refuses is skipped -- UDP is best effort;
// the reference's per-datagram WriteTo would have returned its error -- and
// its error is reported by the next write.  SQ_ECLOSED when shutdown
// interrupts a wait for socket space.
int send_batch(sqobfs_pconn *pc, PBatch &b, uint32_t from, int *first_err, uint64_t *errors) {
  const Block &k = *b.blk;
  uint32_t nm = 0;
  for (uint32_t i = from; i < b.n;) {
    uint32_t j = i + 1;
    if (pc->gso) {
      const uint32_t g = k.out_len[i];
      uint32_t bytes = g;
      while (j < b.n && j - i < kGsoMaxSegs && g > 0 && k.out_len[j] <= g && k.out_len[j] > 0 &&
             bytes + k.out_len[j] <= kGsoMaxBytes &&
             memcmp(&b.addr[j], &b.addr[i], sizeof b.addr[i]) == 0) {
        bytes += k.out_len[j];
        j++;
        if (k.out_len[j - 1] < g) break;
      }
    }
    for (uint32_t q = i; q < j; q++) {
      pc->tiov[q].iov_base = pc->slot(b, q);
      pc->tiov[q].iov_len = k.out_len[q];
    }
    mmsghdr &h = pc->tmsg[nm];
    memset(&h, 0, sizeof h);
    socklen_t sl;
    sq::to_sockaddr(b.addr[i], &pc->tss[nm], &sl);
    h.msg_hdr.msg_name = &pc->tss[nm];
    h.msg_hdr.msg_namelen = sl;
    h.msg_hdr.msg_iov = &pc->tiov[i];
    h.msg_hdr.msg_iovlen = j - i;
    if (j - i > 1) {
      h.msg_hdr.msg_control = &pc->tctl[kCtlWords * nm];
      h.msg_hdr.msg_controllen = CMSG_SPACE(sizeof(uint16_t));
      cmsghdr *cm = CMSG_FIRSTHDR(&h.msg_hdr);
      cm->cmsg_level = SOL_UDP;
      cm->cmsg_type = UDP_SEGMENT;
      cm->cmsg_len = CMSG_LEN(sizeof(uint16_t));
      const uint16_t gs = (uint16_t)k.out_len[i];
      memcpy(CMSG_DATA(cm), &gs, sizeof gs);
    }
    pc->tfirst[nm++] = i;
    i = j;
  }
  uint32_t done = 0;
  while (done < nm) {
    const uint32_t c = std::min(nm - done, kMmsg);
    const int m = sendmmsg(pc->fd, &pc->tmsg[done], c, MSG_DONTWAIT);
    if (m < 0) {
      const int e = errno;
      if (e == EINTR) continue;
      if (e == EAGAIN || e == EWOULDBLOCK || e == ENOBUFS) {
        pollfd p[2] = {{pc->fd, POLLOUT, 0}, {pc->wake, POLLIN, 0}};
        (void)poll(p, 2, 100);
        if (p[1].revents & POLLIN) return SQ_ECLOSED;
        continue;
      }
      if (pc->gso && pc->tmsg[done].msg_hdr.msg_iovlen > 1 &&
          (e == EIO || e == EINVAL || e == ENOPROTOOPT || e == EOPNOTSUPP)) {
        pc->gso = false;  // no segmentation offload here: one datagram per message
        return send_batch(pc, b, pc->tfirst[done], first_err, errors);
      }
      if (!*first_err) *first_err = SQOBFS_ERRNO(e);
      *errors += pc->tmsg[done].msg_hdr.msg_iovlen;
      done++;  // this message failed: go on with the next
      continue;
    }
    done += (uint32_t)m;
  }
  return SQ_OK;
}

// Transform bookkeeping shared by the tasks (under pc->mu).
void note_transform(sqobfs_pconn *pc, const Job &j) {
  if (j.cpu) pc->st.cpu_batches++;
  if (j.failed) pc->st.gpu_failures++;
  if (j.refused) pc->st.gpu_refused++;
  if (j.st != SQ_OK && j.st != SQ_ECLOSED) pc->st.dropped += j.batch().n;
}

// ---------------------------------------------------------------- tasks
//
// A task runs in two steps around the transform of its batch: prepare (take
// the batch; false when the task ended without one) and finish (send or
// queue it, end or requeue the task).  run_task joins them, so that the
// batches of several tasks can share one launch.

// Transmit: the next queued batch (or the filling one, once its linger is
// due) -> transform -> sendmmsg (socket mode) or the pump taker.
bool tx_prepare(sqobfs_pconn *pc, Job &j) {
  std::unique_lock<std::mutex> lk(pc->mu);
  if (pc->closed) {
    task_end(pc, kTx, false);
    return false;
  }
  if (pc->tq.empty()) {
    if (pc->tfill >= 0 && pc->tb[pc->tfill].n > 0) {
      const int64_t due = pc->tb[pc->tfill].first_ns + (int64_t)pc->o.linger_us * 1000;
      if (pc->o.linger_us && !pc->writes_closed && mono_ns() < due) {
        task_end(pc, kTx, true, due);
        return false;
      }
      pc->tq.push_back((uint32_t)pc->tfill);
      pc->tfill = -1;
    } else {
      task_end(pc, kTx, false);
      return false;
    }
  }
  j.pc = pc;
  j.dir = kTx;
  j.idx = pc->tq.front();
  j.slotted = true;
  pc->tq.pop_front();
  pc->tx_busy = true;
  return true;
}

void tx_finish(Job &j) {
  sqobfs_pconn *pc = j.pc;
  PBatch &b = j.batch();
  int send_err = 0;
  uint64_t nerr = 0;
  if (j.st == SQ_OK && pc->socket_mode()) j.st = send_batch(pc, b, 0, &send_err, &nerr);
  std::unique_lock<std::mutex> lk(pc->mu);
  note_transform(pc, j);
  if (send_err && !pc->tx_err) pc->tx_err = send_err;
  pc->st.tx_send_errors += nerr;
  if (j.st == SQ_OK) {
    pc->st.tx_datagrams += b.n;
    pc->st.tx_batches++;
    pc->st.tx_max_batch = std::max(pc->st.tx_max_batch, b.n);
  }
  if (j.st == SQ_OK && !pc->socket_mode()) {
    pc->ttaken.push_back(j.idx);
    pc->cv_take.notify_one();
  } else {
    batch_detach(pc, b);
    pc->tfree.push_back(j.idx);
  }
  pc->cv_txs.notify_all();
  if (!j.end_task) return;  // (the task's last batch ends it)
  pc->tx_busy = false;
  const bool more = !pc->tq.empty() || (pc->tfill >= 0 && pc->tb[pc->tfill].n > 0);
  task_end(pc, kTx, more);
}

// Receive, pump mode: the batch the caller pushed -> deobfuscate -> ready.
bool rx_pump_prepare(sqobfs_pconn *pc, Job &j) {
  std::unique_lock<std::mutex> lk(pc->mu);
  if (pc->closed) {
    task_end(pc, kRx, false);
    return false;
  }
  if (pc->rq.empty()) {
    if (pc->rfill >= 0 && pc->rb[pc->rfill].n > 0) {
      const int64_t due = pc->rb[pc->rfill].first_ns + (int64_t)pc->o.linger_us * 1000;
      if (pc->o.linger_us && mono_ns() < due) {
        task_end(pc, kRx, true, due);
        return false;
      }
      pc->rq.push_back((uint32_t)pc->rfill);
      pc->rfill = -1;
    } else {
      task_end(pc, kRx, false);
      return false;
    }
  }
  j.pc = pc;
  j.dir = kRx;
  j.idx = pc->rq.front();
  j.slotted = true;
  pc->rq.pop_front();
  pc->rb[j.idx].next = 0;
  return true;
}

// (pump and socket receive) the batch is ready to read, or lost with a
// failed launch.  Caller holds pc->mu.
void rx_done(sqobfs_pconn *pc, Job &j) {
  PBatch &b = j.batch();
  note_transform(pc, j);
  if (j.st != SQ_OK) {
    batch_detach(pc, b);
    pc->rfree.push_back(j.idx);
    pc->cv_rxs.notify_all();
  } else {
    pc->st.rx_datagrams += b.n;
    pc->st.rx_batches++;
    pc->st.rx_max_batch = std::max(pc->st.rx_max_batch, b.n);
    pc->rready.push_back(j.idx);
    pc->cv_rxr.notify_all();
  }
}

void rx_pump_finish(Job &j) {
  sqobfs_pconn *pc = j.pc;
  std::unique_lock<std::mutex> lk(pc->mu);
  rx_done(pc, j);
  if (!j.end_task) return;  // (the task's last batch ends it)
  const bool more = !pc->rq.empty() || (pc->rfill >= 0 && pc->rb[pc->rfill].n > 0);
  task_end(pc, kRx, more);
}

void rearm(Engine *E, sqobfs_pconn *pc) {
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLONESHOT;
  ev.data.u64 = pc->id;
  (void)epoll_ctl(E->epfd, EPOLL_CTL_MOD, pc->fd, &ev);  // (ENOENT after close: fine)
}

// Receive, socket mode (the poller saw the socket readable): recvmmsg one
// batch -> deobfuscate -> ready; requeued while the socket has more, the
// socket re-armed when it is drained.
bool rx_socket_prepare(Engine *E, sqobfs_pconn *pc, Job &j) {
  std::unique_lock<std::mutex> lk(pc->mu);
  if (pc->closed || pc->rx_dead) {
    task_end(pc, kRx, false);
    return false;
  }
  if (pc->rfree.empty()) {  // every batch holds unread datagrams: read() restarts us
    pc->rx_stall = true;
    task_end(pc, kRx, false);
    return false;
  }
  const uint32_t idx = pc->rfree.front();
  pc->rfree.pop_front();
  PBatch &b = pc->rb[idx];
  if (!batch_attach(pc, b, false)) {
    pc->rfree.push_front(idx);
    if (!pc->rready.empty()) {
      pc->rx_stall = true;  // no memory now: the read() that frees a batch retries
      task_end(pc, kRx, false);
      return false;
    }
    // nothing to read, so no read() will come back here: retry on a timer
    // (the socket stays un-armed meanwhile; its datagrams wait in the kernel)
    task_end(pc, kRx, true, mono_ns() + kAttachRetryNs);
    return false;
  }
  lk.unlock();
  // GRO: the batch's slot region as 64 KiB buffers of up to 64 coalesced
  // datagrams each (so the batch arrays always have room)
  const uint32_t ngro = pc->gro ? std::max<uint32_t>(1, std::min<uint64_t>(
                                      (uint64_t)pc->o.batch * pc->o.slot_bytes / kGroBuf,
                                      pc->o.batch / kGsoMaxSegs))
                                : 0;
  const uint32_t want = pc->gro ? ngro : pc->o.batch;
  Block &k = *b.blk;
  for (uint32_t q = 0; q < want; q++) {
    pc->riov[q].iov_base = pc->gro ? k.slots + (size_t)q * kGroBuf : pc->slot(b, q);
    pc->riov[q].iov_len = pc->gro ? kGroBuf : pc->o.slot_bytes;
    memset(&pc->rmsg[q], 0, sizeof pc->rmsg[q]);
    pc->rmsg[q].msg_hdr.msg_iov = &pc->riov[q];
    pc->rmsg[q].msg_hdr.msg_iovlen = 1;
    pc->rmsg[q].msg_hdr.msg_name = &pc->rss[q];
    pc->rmsg[q].msg_hdr.msg_namelen = sizeof pc->rss[q];
    if (pc->gro) {
      pc->rmsg[q].msg_hdr.msg_control = &pc->rctl[8ull * q];
      pc->rmsg[q].msg_hdr.msg_controllen = 8 * sizeof(uint64_t);
    }
  }
  int m;
  do {
    m = recvmmsg(pc->fd, pc->rmsg.data(), want, MSG_DONTWAIT, nullptr);
  } while (m < 0 && errno == EINTR);
  if (m <= 0) {
    const int e = m < 0 ? errno : EAGAIN;
    lk.lock();
    batch_detach(pc, b);
    pc->rfree.push_front(idx);
    if (e != EAGAIN && e != EWOULDBLOCK) {
      // ICMP-reported errors are per datagram (the next read works);
      // anything else ends the receive side
      pc->rx_err = SQOBFS_ERRNO(e);
      const bool transient = e == ECONNREFUSED || e == EHOSTUNREACH || e == ENETUNREACH;
      pc->rx_err_sticky = !transient;
      pc->rx_dead = !transient;
      pc->cv_rxr.notify_all();
    }
    if (!pc->rx_dead) rearm(E, pc);
    task_end(pc, kRx, false);
    return false;
  }
  uint64_t trunc = 0;
  uint32_t n = 0;
  if (pc->gro) {
    // split every coalesced message into its datagrams (cmsg UDP_GRO gives
    // the segment size; the last may be shorter), decoded in place
    for (int q = 0; q < m; q++) {
      const uint32_t total = pc->rmsg[q].msg_len;
      uint32_t seg = total;
      for (cmsghdr *cm = CMSG_FIRSTHDR(&pc->rmsg[q].msg_hdr); cm;
           cm = CMSG_NXTHDR(&pc->rmsg[q].msg_hdr, cm))
        if (cm->cmsg_level == SOL_UDP && cm->cmsg_type == UDP_GRO) {
          int v;
          memcpy(&v, CMSG_DATA(cm), sizeof v);
          if (v > 0) seg = (uint32_t)v;
        }
      if (pc->rmsg[q].msg_hdr.msg_flags & MSG_TRUNC) trunc++;
      sqobfs_addr from;
      sq::from_sockaddr(pc->rss[q], &from);
      const uint64_t base = (uint64_t)q * kGroBuf;
      for (uint32_t o = 0; (o < total || (total == 0 && o == 0)) && n < pc->o.batch;
           o += seg ? seg : 1) {
        const uint32_t l = std::min(seg, total - o);
        k.in_off[n] = base + o;
        k.out_off[n] = base + o + pc->S;
        k.len[n] = l;
        memcpy(&b.head[16ull * n], k.slots + base + o, std::min<uint32_t>(16, l));
        b.addr[n] = from;
        b.tag[n] = 0;
        n++;
        if (total == 0) break;
      }
    }
  } else {
    for (int q = 0; q < m; q++) {
      k.len[q] = std::min<uint32_t>(pc->rmsg[q].msg_len, pc->o.slot_bytes);
      memcpy(&b.head[16ull * q], pc->slot(b, (uint32_t)q), 16);
      if (pc->rmsg[q].msg_hdr.msg_flags & MSG_TRUNC) trunc++;
      sq::from_sockaddr(pc->rss[q], &b.addr[q]);
      b.tag[q] = 0;
    }
    n = (uint32_t)m;
  }
  b.n = n;
  b.next = 0;
  j.pc = pc;
  j.dir = kRx;
  j.idx = idx;
  j.slotted = !pc->gro;
  j.trunc = trunc;
  return true;
}

void rx_socket_finish(Job &j) {
  sqobfs_pconn *pc = j.pc;
  std::unique_lock<std::mutex> lk(pc->mu);
  pc->st.rx_truncated += j.trunc;
  rx_done(pc, j);
  task_end(pc, kRx, true);  // the socket may hold more: look again (EAGAIN re-arms)
}

bool task_prepare(Engine *E, const Task &t, Job &j) {
  if (t.dir == kTx) return tx_prepare(t.pc, j);
  if (t.pc->socket_mode()) return rx_socket_prepare(E, t.pc, j);
  return rx_pump_prepare(t.pc, j);
}

// The next queued batch of a task whose first batch run_task prepared and
// launches: a transmit task's next full batch, a pump receive task's next
// pushed one, when it has at most `room` datagrams; false when there is
// none (socket receive: one recvmmsg per task run).
bool task_prepare_next(const Task &t, uint32_t room, Job &j) {
  sqobfs_pconn *pc = t.pc;
  if (t.dir == kRx && pc->socket_mode()) return false;
  std::lock_guard<std::mutex> lk(pc->mu);
  std::deque<uint32_t> &q = t.dir == kTx ? pc->tq : pc->rq;
  if (pc->closed || q.empty()) return false;
  std::vector<PBatch> &bs = t.dir == kTx ? pc->tb : pc->rb;
  if (bs[q.front()].n > room) return false;
  j.pc = pc;
  j.dir = t.dir;
  j.idx = q.front();
  j.slotted = true;
  q.pop_front();
  if (t.dir == kRx) bs[j.idx].next = 0;
  return true;
}

void task_finish(Job &j) {
  if (j.dir == kTx) tx_finish(j);
  else if (j.pc->socket_mode()) rx_socket_finish(j);
  else rx_pump_finish(j);
}

// A pconn whose batches may join another's launch: pump mode -- its tasks'
// prepare and finish steps are queue operations, so one worker runs several
// at no cost to the others -- and it leaves the routing to the engine
// (cpu_max 0 or SQOBFS_PCONN_NEVER).  Socket-mode tasks are not gathered:
// their steps are the recvmmsg / sendmmsg calls, which the workers must keep
// making in parallel (measured, lat_bench hops over 8 socket pairs: gathering
// them halved the unpaced rate, 9-10.7 -> 4.4-4.7 GiB/s, for no CPU saved).
bool groupable(const sqobfs_pconn *pc) {
  return !pc->socket_mode() && (pc->o.cpu_max == 0 || pc->o.cpu_max == SQOBFS_PCONN_NEVER);
}

// Takes off the run queue up to `max` queued tasks of direction dir of
// groupable pconns of this kind whose batches (at most o.batch datagrams
// each) fit in `room` datagrams; the calling worker runs them.
uint32_t grab_tasks(Engine *E, int dir, int kind, uint32_t room, Task *out, uint32_t max) {
  std::lock_guard<std::mutex> lk(E->mu);
  uint32_t n = 0;
  for (auto it = E->runq.begin(); it != E->runq.end() && n < max;) {
    const sqobfs_pconn *pc = it->pc;
    if (!it->fin && it->dir == dir && pc->kind == kind && groupable(pc) && pc->o.batch <= room) {
      room -= pc->o.batch;
      out[n++] = *it;
      it = E->runq.erase(it);
    } else {
      ++it;
    }
  }
  return n;
}

// One task.  When its batch launches, the batches other pconns have queued
// for the same scheme and direction join the launch (up to group_max
// batches, kGroupDgrams datagrams): bulk traffic over several pconns -- the
// hop conns of a port-hopping client, a server's conns on one context --
// costs one launch and one wait per group (measured, lat_bench hops, 8 pump
// conns unpaced: ~4 batches per launch, a quarter of the launches).  A batch
// that would not have launched on its own rides along: the launch is paid
// for.  Batches are not gathered to make a launch that none of them would
// make alone: gathered groups of small batches under paced load launched
// 4-13K times in 3 s for no CPU saved ("Coalesced launches").
// The non-polling GPU route is saturated: every launch slot flies and
// batches of pend_max datagrams or more already wait for the next one.
bool gpu_saturated(Engine *E) {
  std::lock_guard<std::mutex> lk(E->cmu);
  return E->pend_max && E->nflight >= E->flight_cap && E->pending_dgrams >= E->pend_max;
}

// Sets the outcome of the jobs' transform -- st: SQ_OK, a failed kernel's
// error, or kRefused (nothing ran: redone on the CPU path; gpu: a launch was
// tried) -- and runs their finish steps.
void jobs_finish(Engine *E, Job *jobs, uint32_t nj, int st, bool gpu) {
  for (uint32_t k = 0; k < nj; k++) {
    Job &j = jobs[k];
    if (st == kRefused) {
      // a refusal that turned the GPU off counts as a failure; one of the
      // moment (no stream, block or keyring memory) as a refusal
      j.failed = gpu && E->gpu_off.load(std::memory_order_relaxed);
      j.refused = gpu && !j.failed;
      j.cpu = true;
      j.st = cpu_run(E, j);
    } else {
      j.failed = st != SQ_OK;
      j.st = st;
    }
  }
  t_requeued = 0;
  for (uint32_t k = 0; k < nj; k++) task_finish(jobs[k]);
  // a worker that requeued several tasks after a coalesced launch takes one
  // of them itself and wakes a worker for each of the others, which would
  // otherwise run one after another here (their batches may go to the CPU
  // path, where nothing regroups them)
  if (t_worker)
    for (uint32_t k = 1; k < t_requeued; k++) E->cv.notify_one();
  t_requeued = 0;
}

// One task.  When its batch launches, the batches other pconns have queued
// for the same scheme and direction join the launch (up to group_max
// batches, kGroupDgrams datagrams): bulk traffic over several pconns -- the
// hop conns of a port-hopping client, a server's conns on one context --
// costs one launch and one wait per group (measured, lat_bench hops, 8 pump
// conns unpaced: ~4 batches per launch, a quarter of the launches).  A batch
// that would not have launched on its own rides along: the launch is paid
// for.  Batches are not gathered to make a launch that none of them would
// make alone: gathered groups of small batches under paced load launched
// 4-13K times in 3 s for no CPU saved ("Coalesced launches").
// A launch that waits without polling goes to the completer (Flight), and
// the worker returns to the run queue; the completed launch's batches are
// finished there, or back on a worker (t.fin: a socket-mode batch).
void run_task(Engine *E, const Task &t) {
  if (t.fin) {  // (their status set by the completer)
    Flight *f = t.fin;
    jobs_finish(E, f->jobs, f->nj, f->jobs[0].st, true);
    delete f;
    return;
  }
  Flight f;
  Job *jobs = f.jobs;
  if (!task_prepare(E, t, jobs[0])) return;
  bool bulk = false;
  bool gpu = route_gpu(E, jobs[0], &bulk);
  // the GPU route saturated -- a launch in flight and a full launch's worth
  // of batches already waiting for it -- a bulk batch runs on the CPU path
  // instead of waiting: the host's cores add to the GPU's rate
  if (gpu && bulk && gpu_saturated(E)) gpu = false;
  uint32_t nj = 1, nd = jobs[0].batch().n;
  // a launched task takes its other queued batches along (finished in
  // order, the last one ending the task): a conn whose writer filled
  // several batches during the previous launch sends them all in this one
  const uint32_t gmax = std::min(kMaxGroup, E->group_max.load(std::memory_order_relaxed));
  auto take_queued = [&](const Task &tk) {
    while (nj < gmax && nd < kGroupDgrams && task_prepare_next(tk, kGroupDgrams - nd, jobs[nj])) {
      bool b2;
      (void)route_gpu(E, jobs[nj], &b2);  // (its cost, and the engine's demand)
      jobs[nj - 1].end_task = false;
      nd += jobs[nj].batch().n;
      nj++;
    }
  };
  if (gpu) take_queued(t);
  if (gpu && nj < gmax && groupable(t.pc) && nd < kGroupDgrams) {
    Task more[kMaxGroup];
    const uint32_t m = grab_tasks(E, t.dir, t.pc->kind, kGroupDgrams - nd, more, gmax - nj);
    for (uint32_t k = 0; k < m; k++)
      if (task_prepare(E, more[k], jobs[nj])) {
        bool b2;
        (void)route_gpu(E, jobs[nj], &b2);  // (its cost, and the engine's demand)
        nd += jobs[nj].batch().n;
        nj++;
        take_queued(more[k]);
      }
  }
  f.nj = nj;
  int st = kRefused;
  if (gpu) {
    f.block = bulk || t.pc->o.spin_us == SQOBFS_PCONN_NEVER;
    if (f.block) {
      // at most flight_cap non-polling launches fly; past it the batches
      // wait, prepared, and the completion that frees a slot launches every
      // one of them at once (completer_main)
      std::lock_guard<std::mutex> lk(E->cmu);
      if (!E->cstop && E->nflight >= E->flight_cap) {
        try {
          E->pending.insert(E->pending.end(), jobs, jobs + nj);
          E->pending_dgrams += nd;
          return;
        } catch (...) {  // (no memory: launch it now, over the cap)
        }
      }
      E->nflight++;
    }
    st = gpu_launch(E, f);
    if (st == SQ_OK && f.block) {
      Flight *h = new (std::nothrow) Flight(std::move(f));
      if (h) {
        if (flight_queue(E, h)) return;
        f = std::move(*h);
        delete h;
      }
    }
    if (st == SQ_OK) st = gpu_land(E, f);
    if (f.block) {
      std::lock_guard<std::mutex> lk(E->cmu);
      E->nflight--;
    }
  }
  jobs_finish(E, jobs, nj, st, gpu);
}

void worker_main(Engine *E) {
  engine_thread_pin(E);
  t_worker = true;
  std::unique_lock<std::mutex> lk(E->mu);
  for (;;) {
    if (E->stop) return;
    int64_t next = 0;
    if (!E->timers.empty()) {
      const int64_t now = mono_ns();
      for (size_t k = 0; k < E->timers.size();) {
        if (E->timers[k].first <= now) {
          Task t = E->timers[k].second;
          t.pc->timed[t.dir] = false;
          E->runq.push_back(t);
          E->timers.erase(E->timers.begin() + (long)k);
        } else {
          next = next ? std::min(next, E->timers[k].first) : E->timers[k].first;
          k++;
        }
      }
    }
    // (held: no new task starts; a completed launch's finish still runs)
    if (E->runq.empty() || (g_hold.load(std::memory_order_relaxed) && !E->runq.front().fin)) {
      if (next) E->cv.wait_until(lk, mono_tp(next));
      else E->cv.wait(lk);
      continue;
    }
    const Task t = E->runq.front();
    E->runq.pop_front();
    lk.unlock();
    run_task(E, t);
    lk.lock();
  }
}

// Starts one launch over pending batches, the first pending batch's scheme
// and direction and every other pending batch that may join it (up to
// kMaxGroup batches and kGroupDgrams datagrams).  Caller holds cmu, with a
// slot counted in nflight for it; returns with cmu held.  The new flight is
// queued for the completer; a refused launch's batches run on the CPU path
// here, and its slot is given back.
void launch_pending(Engine *E, std::unique_lock<std::mutex> &lk) {
  Flight *f = new (std::nothrow) Flight();
  if (!f) {
    E->nflight--;  // (the batches stay pending for the next completion)
    return;
  }
  const int kind = E->pending[0].pc->kind, dir = E->pending[0].dir;
  uint32_t nd = 0;
  // whole tasks only (a task's batches are consecutive, its last one ends
  // it): a task split over two launches could finish out of order
  std::vector<Job> &P = E->pending;
  size_t w = 0;
  for (size_t i = 0; i < P.size();) {
    size_t e = i + 1;
    while (e < P.size() && !P[e - 1].end_task) e++;
    uint32_t n = 0;
    for (size_t q = i; q < e; q++) n += P[q].batch().n;
    if (P[i].pc->kind == kind && P[i].dir == dir && f->nj + (e - i) <= kMaxGroup &&
        (f->nj == 0 || nd + n <= kGroupDgrams)) {
      for (size_t q = i; q < e; q++) f->jobs[f->nj++] = P[q];
      nd += n;
    } else {
      for (size_t q = i; q < e; q++) P[w++] = P[q];
    }
    i = e;
  }
  P.resize(w);
  E->pending_dgrams -= std::min(E->pending_dgrams, nd);
  f->block = true;
  lk.unlock();
  int st = gpu_launch(E, *f);
  lk.lock();
  if (st == SQ_OK) {
    try {
      E->flights.push_back(f);
      E->async_launches.fetch_add(1, std::memory_order_relaxed);
      return;
    } catch (...) {
    }
    lk.unlock();
    st = gpu_land(E, *f);
    lk.lock();
  }
  E->nflight--;
  lk.unlock();
  jobs_finish(E, f->jobs, f->nj, st, true);
  delete f;
  lk.lock();
}

// The completer (engines of a context): takes the launches queued by
// run_task and launch_pending in launch order and lands each (gpu_land:
// asleep through most of the kernel, then short polls), then finishes its
// batches -- pump-mode ones here (queue hand-offs: the batch to the taker
// or the readers, the task requeued with a wake-up), socket-mode ones on a
// worker (the sendmmsg, or the next recvmmsg), queued at the front of the
// run queue -- and launches the batches that waited for the slot.  On stop
// it lands what is in flight and runs what is pending on the CPU path.
void completer_main(Engine *E) {
  engine_thread_pin(E);
  std::unique_lock<std::mutex> lk(E->cmu);
  for (;;) {
    E->cv_flight.wait(lk, [E] { return E->cstop || !E->flights.empty(); });
    if (E->flights.empty()) break;
    Flight *f = E->flights.front();
    E->flights.pop_front();
    lk.unlock();
    const int st = gpu_land(E, *f);
    // the batches that waited for the slot launch first, so the GPU works
    // on them while this thread finishes the landed ones
    lk.lock();
    E->nflight--;
    while (!E->pending.empty() && E->nflight < E->flight_cap && !E->cstop) {
      E->nflight++;
      launch_pending(E, lk);
    }
    lk.unlock();
    // a socket-mode pconn's batches (consecutive: one task's) go back to a
    // worker together, in order, as one finish (their sends use the pconn's
    // scratch, one batch after another)
    uint32_t keep = 0;  // pump-mode jobs, finished here
    for (uint32_t k = 0; k < f->nj;) {
      uint32_t e = k + 1;
      while (e < f->nj && f->jobs[e].pc == f->jobs[k].pc && f->jobs[e].dir == f->jobs[k].dir) e++;
      for (uint32_t q = k; q < e; q++) {
        f->jobs[q].failed = st != SQ_OK;
        f->jobs[q].st = st;
      }
      Flight *h = f->jobs[k].pc->socket_mode() ? new (std::nothrow) Flight() : nullptr;
      bool queued = false;
      if (h) {
        for (uint32_t q = k; q < e; q++) h->jobs[h->nj++] = f->jobs[q];
        std::lock_guard<std::mutex> g(E->mu);
        if (!E->stop) {
          try {
            E->runq.push_front(Task{h->jobs[0].pc, h->jobs[0].dir, h});
            queued = true;
          } catch (...) {
          }
        }
      }
      if (queued) {
        E->cv.notify_one();
      } else {
        delete h;
        for (uint32_t q = k; q < e; q++) f->jobs[keep++] = f->jobs[q];
      }
      k = e;
    }
    jobs_finish(E, f->jobs, keep, st, true);
    delete f;
    lk.lock();
    // (batches that became pending while this thread finished: the next
    // completion launches them, or now if the slot is free)
    while (!E->pending.empty() && E->nflight < E->flight_cap && !E->cstop) {
      E->nflight++;
      launch_pending(E, lk);
    }
  }
  // stopped: what still waits for a slot runs on the CPU path
  std::vector<Job> rest;
  rest.swap(E->pending);
  E->pending_dgrams = 0;
  lk.unlock();
  for (Job &j : rest) jobs_finish(E, &j, 1, kRefused, false);
}

void poller_main(Engine *E) {
  engine_thread_pin(E);
  epoll_event ev[64];
  for (;;) {
    const int n = epoll_wait(E->epfd, ev, 64, -1);
    if (n < 0 && errno != EINTR) return;
    std::lock_guard<std::mutex> lk(E->mu);
    if (E->stop) return;
    for (int i = 0; i < n; i++) {
      if (ev[i].data.u64 == 0) continue;  // the wake fd (stop)
      auto it = E->byid.find(ev[i].data.u64);
      if (it == E->byid.end()) continue;  // closed meanwhile
      schedule_locked(E, it->second, kRx);
    }
  }
}

void engine_end(Engine *E) {
  {
    std::lock_guard<std::mutex> lk(E->mu);
    E->stop = true;
  }
  {
    std::lock_guard<std::mutex> lk(E->cmu);
    E->cstop = true;
  }
  E->cv.notify_all();
  E->cv_flight.notify_all();
  E->cv_stream.notify_all();
  const uint64_t one = 1;
  (void)!write(E->wake, &one, sizeof one);
  for (auto &t : E->threads) t.join();
  for (auto &m : E->mkr) m.reset();  // (fenced on the streams: before they go)
  for (void *s : E->streams) sq_ctx_stream_destroy(E->ctx, s);
  for (auto &kv : E->free_blocks)
    for (Block *b : kv.second) block_free_mem(E, b);
  close(E->wake);
  close(E->epfd);
  delete E;
}

}  // namespace

// ---------------------------------------------------------------- engine ABI

void sq_engine_ctx_closed(sqobfs_ctx *ctx) {
  Engine *E = nullptr;
  {
    std::lock_guard<std::mutex> g(g_eng_mu);
    g_workers_cfg.erase(ctx);
    g_affinity_cfg.erase(ctx);
    g_group_cfg.erase(ctx);
    auto it = g_engines.find(ctx);
    if (it == g_engines.end()) return;
    E = it->second;
    g_engines.erase(it);
  }
  engine_end(E);  // (the context outlives its pconns: none is open)
}

extern "C" {

int sqobfs_engine_info_get(sqobfs_ctx *ctx, sqobfs_engine_info *out) {
  if (!out) return SQ_EINVAL;
  memset(out, 0, sizeof *out);
  std::lock_guard<std::mutex> g(g_eng_mu);
  auto it = g_engines.find(ctx);
  if (it == g_engines.end()) return SQ_OK;
  Engine *E = it->second;
  {
    std::lock_guard<std::mutex> lk(E->mu);
    out->pconns = E->pconns;
    out->threads = (uint32_t)E->threads.size();
    out->workers = E->nworkers;
  }
  std::lock_guard<std::mutex> pg(E->pool_mu);
  out->pool_blocks = E->blocks;
  out->pool_bytes = E->pool_bytes;
  out->blocks_in_use = E->in_use;
  out->gpu_disabled = E->gpu_off.load() ? 1u : 0u;
  out->route_bytes = E->ctx ? route_bytes(E) : 0u;
  out->launch_us = E->launch_us.load();
  out->cpu_ns_per_kib = E->cpu_ns_kib.load();
  out->load_permille = E->load_pm.load();
  out->loaded = E->loaded.load() ? 1u : 0u;
  out->gpu_host_ns = E->gpu_host_ns.load();
  out->cpus = E->ncpus;
  out->group_max = E->group_max.load();
  out->launches = E->launches.load();
  out->group_launches = E->group_launches.load();
  out->group_batches = E->group_batches.load();
  out->async_launches = E->async_launches.load();
  {
    std::lock_guard<std::mutex> cl(E->cmu);
    out->streams = (uint32_t)E->streams.size();
  }
  return SQ_OK;
}

int sqobfs_engine_set_workers(sqobfs_ctx *ctx, uint32_t workers) {
  if (workers > kMaxWorkers) return SQ_EINVAL;
  std::lock_guard<std::mutex> g(g_eng_mu);
  if (g_engines.count(ctx)) return SQ_EINVAL;
  g_workers_cfg[ctx] = workers;
  return SQ_OK;
}

int sqobfs_engine_set_affinity(sqobfs_ctx *ctx, int mode) {
  if (mode != SQOBFS_ENGINE_AFFINITY_NONE && mode != SQOBFS_ENGINE_AFFINITY_L3) return SQ_EINVAL;
  std::lock_guard<std::mutex> g(g_eng_mu);
  if (g_engines.count(ctx)) return SQ_EINVAL;
  g_affinity_cfg[ctx] = mode;
  return SQ_OK;
}

int sqobfs_engine_set_group(sqobfs_ctx *ctx, uint32_t max_batches) {
  if (max_batches > kMaxGroup) return SQ_EINVAL;
  const uint32_t v = max_batches ? max_batches : kDefGroup;
  std::lock_guard<std::mutex> g(g_eng_mu);
  g_group_cfg[ctx] = v;
  auto it = g_engines.find(ctx);
  if (it != g_engines.end()) it->second->group_max.store(v);
  return SQ_OK;
}

int sqobfs_engine_trim(sqobfs_ctx *ctx) {
  // g_eng_mu held throughout: a concurrent sqobfs_close ends (deletes) the
  // engine under it, so E stays valid while the blocks are freed
  std::lock_guard<std::mutex> g(g_eng_mu);
  auto it = g_engines.find(ctx);
  if (it == g_engines.end()) return 0;
  Engine *E = it->second;
  std::vector<Block *> drop;
  {
    std::lock_guard<std::mutex> pg(E->pool_mu);
    for (auto &kv : E->free_blocks) {
      drop.insert(drop.end(), kv.second.begin(), kv.second.end());
      kv.second.clear();
    }
    for (Block *b : drop) {
      E->blocks--;
      E->pool_bytes -= b->bytes;
    }
  }
  for (Block *b : drop) block_free_mem(E, b);
  return (int)drop.size();
}

void sqobfs_debug_engine_fail(int count, int at_completion) {
  g_fail_at_completion.store(at_completion ? 1 : 0);
  g_fail_count.store(count > 0 ? count : 0);
}

void sqobfs_debug_pool_fail(int count) { g_pool_fail.store(count > 0 ? count : 0); }

void sqobfs_debug_engine_hold(int on) {
  g_hold.store(on != 0);
  if (on) return;
  std::lock_guard<std::mutex> g(g_eng_mu);
  for (auto &kv : g_engines) {
    Engine *E = kv.second;
    { std::lock_guard<std::mutex> lk(E->mu); }  // (a worker between its check and its wait)
    E->cv.notify_all();
  }
}

// ---------------------------------------------------------------- pconn ABI

int sqobfs_pconn_open(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int fd,
                      const sqobfs_pconn_opts *opts, sqobfs_pconn **out) {
  if (out) *out = nullptr;
  if (!kr || !out || sq_keyring_ctx(kr) != ctx) return SQ_EINVAL;
  sqobfs_pconn_opts o{};
  if (opts) o = *opts;
  if (o.batch == 0) o.batch = kDefBatch;
  if (o.slot_bytes == 0) o.slot_bytes = kDefSlot;
  if (o.tx_batches == 0) o.tx_batches = kDefBatches;
  if (o.rx_batches == 0) o.rx_batches = kDefBatches;
  if (o.spin_us == 0) o.spin_us = kDefSpinUs;
  // (cpu_max 0 stays 0: the measured break-even, route_bytes)
  if (o.inline_gap_us == 0) o.inline_gap_us = kDefInlineGapUs;
  const int kind = sqobfs_keyring_kind(kr);
  const uint32_t S = kind == SQOBFS_SALAMANDER ? SQOBFS_SALAMANDER_SALT_LEN : SQOBFS_XPLUS_SALT_LEN;
  if (o.batch > kMaxBatch || o.slot_bytes % 16 || o.slot_bytes <= S ||
      (o.flags & ~(uint32_t)(SQOBFS_UDP_TX_GSO | SQOBFS_UDP_RX_GRO)) || o.tx_batches > 64 ||
      o.rx_batches > 64)
    return SQ_EINVAL;
  int st = SQ_OK;
  Engine *E = engine_get(ctx, &st);
  if (!E) return st;
  sqobfs_pconn *pc = new (std::nothrow) sqobfs_pconn();
  if (!pc) return SQ_ENOMEM;
  pc->eng = E;
  pc->ctx = ctx;
  pc->kr = kr;
  uint32_t count = 0;
  pc->psk0 = sq_keyring_host(kr, &count);
  pc->kind = kind;
  pc->S = S;
  pc->o = o;
  try {
    pc->tb.resize(o.tx_batches);
    pc->rb.resize(o.rx_batches);
    for (auto *v : {&pc->tb, &pc->rb})
      for (PBatch &b : *v) {
        b.addr.resize(o.batch);
        b.tag.resize(o.batch);
      }
    for (PBatch &b : pc->rb) b.head.resize(16ull * o.batch);
    if (fd >= 0) {
      pc->tmsg.resize(o.batch);
      pc->tiov.resize(o.batch);
      pc->tss.resize(o.batch);
      pc->tctl.assign(kCtlWords * o.batch, 0);
      pc->tfirst.resize(o.batch);
      pc->rmsg.resize(o.batch);
      pc->riov.resize(o.batch);
      pc->rss.resize(o.batch);
      pc->ibuf.resize(o.slot_bytes);
    }
  } catch (...) {
    delete pc;
    return SQ_ENOMEM;
  }
  for (uint32_t k = 0; k < o.tx_batches; k++) pc->tfree.push_back(k);
  for (uint32_t k = 0; k < o.rx_batches; k++) pc->rfree.push_back(k);
  pc->wake = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  if (pc->wake < 0) {
    delete pc;
    return SQ_ENOMEM;
  }
  if (fd >= 0) {
    pc->fd = fcntl(fd, F_DUPFD_CLOEXEC, 0);
    if (pc->fd < 0) {
      const int e = errno;
      close(pc->wake);
      delete pc;
      return SQOBFS_ERRNO(e);
    }
    pc->gso = o.flags & SQOBFS_UDP_TX_GSO;  // probed by the first send
    if ((o.flags & SQOBFS_UDP_RX_GRO) && o.batch >= kGsoMaxSegs &&
        (uint64_t)o.batch * o.slot_bytes >= kGroBuf) {
      const int one = 1;
      pc->gro = setsockopt(pc->fd, SOL_UDP, UDP_GRO, &one, sizeof one) == 0;
      if (pc->gro) pc->rctl.assign(8ull * o.batch, 0);
    }
  }
  {
    std::lock_guard<std::mutex> lk(E->mu);
    pc->id = E->next_id++;
    E->byid[pc->id] = pc;
    E->pconns++;
  }
  if (fd >= 0) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLONESHOT;
    ev.data.u64 = pc->id;
    if (epoll_ctl(E->epfd, EPOLL_CTL_ADD, pc->fd, &ev) != 0) {
      const int e = errno;
      {
        std::lock_guard<std::mutex> lk(E->mu);
        E->byid.erase(pc->id);
        E->pconns--;
      }
      close(pc->fd);
      close(pc->wake);
      delete pc;
      return SQOBFS_ERRNO(e);
    }
  }
  *out = pc;
  return SQ_OK;
}

void sqobfs_pconn_shutdown(sqobfs_pconn *pc) {
  if (!pc) return;
  Engine *E = pc->eng;
  bool closer = false;
  {
    std::unique_lock<std::mutex> lk(pc->mu);
    if (!pc->writes_closed) {
      closer = true;
      pc->writes_closed = true;
      // what was written goes out: the filling batch now (no linger), then
      // wait (bounded) until the transmit side has drained -- sent, or taken
      // and done by the pump taker
      if (pc->tfill >= 0 && pc->tb[pc->tfill].n > 0) {
        pc->tq.push_back((uint32_t)pc->tfill);
        pc->tfill = -1;
      }
      if (!pc->tq.empty()) schedule(pc, kTx);
      pc->cv_txs.notify_all();
      const int64_t until = mono_ns() + kDrainNs;
      while (pc->tx_busy || pc->inline_busy || !pc->tq.empty() || !pc->ttaken.empty()) {
        if (mono_ns() >= until) break;
        pc->cv_txs.wait_until(lk, mono_tp(std::min(until, mono_ns() + 5'000'000)));
      }
      pc->closed = true;
      for (auto *cv : {&pc->cv_txs, &pc->cv_rxr, &pc->cv_rxs, &pc->cv_take}) cv->notify_all();
    }
  }
  if (closer) {
    const uint64_t one = 1;
    (void)!write(pc->wake, &one, sizeof one);  // a send blocked on socket space
    if (pc->fd >= 0) (void)epoll_ctl(E->epfd, EPOLL_CTL_DEL, pc->fd, nullptr);
  }
  // every call (a concurrent second one too) returns once the pconn's tasks
  // have ended, so sqobfs_pconn_close may free it
  std::unique_lock<std::mutex> lk(E->mu);
  E->byid.erase(pc->id);
  for (size_t k = 0; k < E->timers.size();) {
    if (E->timers[k].second.pc == pc) {
      const int d = E->timers[k].second.dir;
      pc->timed[d] = false;
      pc->sched[d] = false;
      pc->tasks--;
      E->timers.erase(E->timers.begin() + (long)k);
    } else {
      k++;
    }
  }
  E->cv_idle.wait(lk, [&] { return pc->tasks == 0; });
}

void sqobfs_pconn_close(sqobfs_pconn *pc) {
  if (!pc) return;
  sqobfs_pconn_shutdown(pc);
  Engine *E = pc->eng;
  // its launches are all complete: the keyring need not fence the engine's
  // streams for them (sqobfs_keyring_destroy)
  {
    std::lock_guard<std::mutex> lk(E->cmu);
    for (void *s : E->streams) sq_keyring_forget(pc->kr, s);
  }
  {
    std::lock_guard<std::mutex> lk(E->mu);
    E->pconns--;
  }
  for (auto *v : {&pc->tb, &pc->rb})
    for (PBatch &b : *v) batch_detach(pc, b);
  if (pc->fd >= 0) close(pc->fd);
  if (pc->wake >= 0) close(pc->wake);
  delete pc;
}

int sqobfs_pconn_set_deadline(sqobfs_pconn *pc, uint32_t which, int64_t unix_ns_) {
  if (!pc || (which & ~(SQOBFS_PCONN_READ | SQOBFS_PCONN_WRITE)) || unix_ns_ < 0) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(pc->mu);
  if (which & SQOBFS_PCONN_READ) {
    pc->rdl = unix_ns_;
    pc->cv_rxr.notify_all();
  }
  if (which & SQOBFS_PCONN_WRITE) {
    pc->wdl = unix_ns_;
    pc->cv_txs.notify_all();
  }
  return SQ_OK;
}

namespace {

// The inline write (opts.inline_gap_us): obfuscate on this thread and send,
// waiting for socket space as a blocking WriteTo does (bounded by the write
// deadline and by shutdown).  Caller set inline_busy; returns the send's
// status.
int write_inline(sqobfs_pconn *pc, const uint8_t *p, uint32_t len, const sqobfs_addr *to) {
  uint32_t key8[8];
  uint64_t seq;
  sq_salt_take(pc->ctx, key8, &seq);
  uint8_t *w = pc->ibuf.data();
  sq::cpu::salt_stream(key8, seq, w, pc->S);
  uint8_t key[32];
  sq::cpu::derive_key(*pc->psk0, w, key);
  sq::cpu::xor_stream(w + pc->S, p, len, key);
  sockaddr_storage ss;
  socklen_t sl;
  sq::to_sockaddr(*to, &ss, &sl);
  for (;;) {
    const ssize_t r = sendto(pc->fd, w, pc->S + len, MSG_DONTWAIT, (sockaddr *)&ss, sl);
    if (r >= 0) return SQ_OK;
    const int e = errno;
    if (e == EINTR) continue;
    if (e != EAGAIN && e != EWOULDBLOCK && e != ENOBUFS) return SQOBFS_ERRNO(e);
    int ms = 100;
    {
      std::lock_guard<std::mutex> lk(pc->mu);
      if (pc->closed) return SQ_ECLOSED;
      if (pc->wdl) {
        const int64_t left = pc->wdl - unix_ns();
        if (left <= 0) return SQ_ETIMEDOUT;
        ms = (int)std::min<int64_t>(100, left / 1000000 + 1);
      }
    }
    pollfd q[2] = {{pc->fd, POLLOUT, 0}, {pc->wake, POLLIN, 0}};
    (void)poll(q, 2, ms);
    if (q[1].revents & POLLIN) return SQ_ECLOSED;
  }
}

}  // namespace

int sqobfs_pconn_write(sqobfs_pconn *pc, const uint8_t *p, uint32_t len, const sqobfs_addr *to,
                       uint64_t tag) {
  if (!pc || (len && !p) || (pc->socket_mode() && !to)) return SQ_EINVAL;
  if (len > pc->o.slot_bytes - pc->S) return SQ_EINVAL;
  std::unique_lock<std::mutex> lk(pc->mu);
  if (pc->writes_closed) return SQ_ECLOSED;
  // as a Go net.Conn: a passed deadline fails the call before anything else
  if (pc->wdl && unix_ns() >= pc->wdl) return SQ_ETIMEDOUT;
  if (pc->tx_err) {
    const int e = pc->tx_err;
    pc->tx_err = 0;
    return e;
  }
  const int64_t now = mono_ns();
  const int64_t gap = now - pc->last_write_ns;
  pc->last_write_ns = now;
  if (pc->socket_mode() && pc->o.inline_gap_us != SQOBFS_PCONN_NEVER && !pc->inline_busy &&
      pc->tfill < 0 && pc->tq.empty() && !pc->tx_busy &&
      gap >= (int64_t)pc->o.inline_gap_us * 1000) {
    bool idle;
    {
      std::lock_guard<std::mutex> el(pc->eng->mu);
      idle = !pc->sched[kTx];
    }
    if (idle) {
      pc->inline_busy = true;
      lk.unlock();
      const int st = write_inline(pc, p, len, to);
      lk.lock();
      pc->inline_busy = false;
      pc->st.inline_writes++;
      if (st == SQ_OK) pc->st.tx_datagrams++;
      pc->cv_txs.notify_all();
      return st;
    }
  }
  if (pc->tfill < 0) {
    const bool ok = wait_dl(lk, pc->cv_txs, pc->wdl, [&] {
      return pc->writes_closed || pc->tfill >= 0 || !pc->tfree.empty();
    });
    if (pc->writes_closed) return SQ_ECLOSED;
    if (!ok) return SQ_ETIMEDOUT;
    if (pc->tfill < 0) {  // (another writer may have opened one meanwhile)
      const uint32_t k = pc->tfree.front();
      if (!batch_attach(pc, pc->tb[k], true)) return SQ_ENOMEM;
      pc->tfree.pop_front();
      pc->tfill = (int)k;
      pc->tb[k].n = 0;
    }
  }
  PBatch &b = pc->tb[pc->tfill];
  const uint32_t i = b.n++;
  if (i == 0) b.first_ns = now;
  if (len) memcpy(pc->slot(b, i) + pc->S, p, len);
  b.blk->len[i] = len;
  if (to) b.addr[i] = *to;
  else memset(&b.addr[i], 0, sizeof b.addr[i]);
  b.tag[i] = tag;
  if (b.n == pc->o.batch) {
    pc->tq.push_back((uint32_t)pc->tfill);
    pc->tfill = -1;
    schedule(pc, kTx);
  } else if (i == 0) {
    schedule(pc, kTx);  // a free worker takes it at once (or after linger_us)
  }
  return SQ_OK;
}

int sqobfs_pconn_read(sqobfs_pconn *pc, uint8_t *p, uint32_t cap, uint32_t *n,
                      sqobfs_addr *from, uint64_t *tag) {
  if (n) *n = 0;
  if (!pc || !n || (cap && !p)) return SQ_EINVAL;
  std::unique_lock<std::mutex> lk(pc->mu);
  for (;;) {
    if (pc->closed) return SQ_ECLOSED;
    // as a Go net.Conn: a passed deadline fails the call even with data queued
    const int64_t d = pc->rdl;
    if (d && unix_ns() >= d) return SQ_ETIMEDOUT;
    if (!pc->rready.empty()) break;
    if (pc->rx_err) {
      const int e = pc->rx_err;
      if (!pc->rx_err_sticky) pc->rx_err = 0;
      return e;
    }
    if (d) {
      pc->cv_rxr.wait_until(lk, wall_tp(d));
    } else {
      pc->cv_rxr.wait(lk);
    }
  }
  const uint32_t idx = pc->rready.front();
  PBatch &b = pc->rb[idx];
  const Block &k = *b.blk;
  const uint32_t i = b.next++;
  // the reference reads the datagram into p (cut to len(p)) and decodes
  // what it got: m = min(wire, cap)
  const uint32_t w = k.len[i], m = std::min(w, cap), S = pc->S;
  uint32_t r = 0;
  const uint8_t *src = nullptr;
  if (pc->kind == SQOBFS_SALAMANDER && m <= S) {
    r = m;                       // salamander.go:47-49: returned as is
    src = &b.head[16ull * i];    // the raw bytes (the decode wrote the slot's head)
  } else if (pc->kind == SQOBFS_XPLUS && m < S) {
    r = 0;                  // xplus.go:50-52
  } else {
    r = m - S;              // the first m - S payload bytes
    src = k.slots + k.out_off[i];
  }
  if (r) memcpy(p, src, r);
  *n = r;
  if (from) *from = b.addr[i];
  if (tag) *tag = b.tag[i];
  if (b.next == b.n) {
    pc->rready.pop_front();
    batch_detach(pc, b);
    pc->rfree.push_back(idx);
    pc->cv_rxs.notify_all();
    if (pc->rx_stall) {  // the socket task waits for a free batch
      pc->rx_stall = false;
      schedule(pc, kRx);
    }
  }
  return SQ_OK;
}

int sqobfs_pconn_rx_push(sqobfs_pconn *pc, const uint8_t *wire, uint32_t n,
                         const sqobfs_addr *from, uint64_t tag) {
  if (!pc || pc->socket_mode() || (n && !wire)) return SQ_EINVAL;
  std::unique_lock<std::mutex> lk(pc->mu);
  if (pc->rfill < 0) {
    pc->cv_rxs.wait(lk, [&] { return pc->closed || !pc->rfree.empty() || pc->rfill >= 0; });
    if (pc->closed) return SQ_ECLOSED;
    if (pc->rfill < 0) {
      const uint32_t k = pc->rfree.front();
      if (!batch_attach(pc, pc->rb[k], false)) return SQ_ENOMEM;
      pc->rfree.pop_front();
      pc->rfill = (int)k;
      pc->rb[k].n = 0;
    }
  }
  if (pc->closed) return SQ_ECLOSED;
  PBatch &b = pc->rb[pc->rfill];
  const uint32_t i = b.n++;
  if (i == 0) b.first_ns = mono_ns();
  const uint32_t m = std::min(n, pc->o.slot_bytes);
  if (m < n) pc->st.rx_truncated++;
  if (m) memcpy(pc->slot(b, i), wire, m);
  memcpy(&b.head[16ull * i], pc->slot(b, i), 16);
  b.blk->len[i] = m;
  if (from) b.addr[i] = *from;
  else memset(&b.addr[i], 0, sizeof b.addr[i]);
  b.tag[i] = tag;
  if (b.n == pc->o.batch) {
    pc->rq.push_back((uint32_t)pc->rfill);
    pc->rfill = -1;
    schedule(pc, kRx);
  } else if (i == 0) {
    schedule(pc, kRx);
  }
  return SQ_OK;
}

int sqobfs_pconn_rx_fail(sqobfs_pconn *pc, int status, int once) {
  if (!pc || status >= 0) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(pc->mu);
  if (pc->rx_err && pc->rx_err_sticky) return SQ_OK;  // already failed for good
  pc->rx_err = status;
  pc->rx_err_sticky = !once;
  pc->cv_rxr.notify_all();
  return SQ_OK;
}

int sqobfs_pconn_tx_take(sqobfs_pconn *pc, int timeout_ms, sqobfs_pconn_tx *out) {
  if (!pc || !out || pc->socket_mode()) return SQ_EINVAL;
  memset(out, 0, sizeof *out);
  std::unique_lock<std::mutex> lk(pc->mu);
  if (pc->taken) return SQ_EINVAL;  // the previous batch was not done
  auto ready = [&] { return pc->closed || !pc->ttaken.empty(); };
  if (timeout_ms < 0) {
    pc->cv_take.wait(lk, ready);
  } else if (!pc->cv_take.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) {
    return SQ_ETIMEDOUT;
  }
  if (pc->ttaken.empty()) return SQ_ECLOSED;
  PBatch &b = pc->tb[pc->ttaken.front()];
  pc->taken = true;
  out->count = b.n;
  out->base = b.blk->slots;
  out->off = b.blk->out_off;
  out->len = b.blk->out_len;
  out->to = b.addr.data();
  out->tag = b.tag.data();
  return SQ_OK;
}

int sqobfs_pconn_tx_done(sqobfs_pconn *pc) {
  if (!pc) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(pc->mu);
  if (!pc->taken || pc->ttaken.empty()) return SQ_EINVAL;
  const uint32_t idx = pc->ttaken.front();
  pc->ttaken.pop_front();
  pc->taken = false;
  batch_detach(pc, pc->tb[idx]);
  pc->tfree.push_back(idx);
  pc->cv_txs.notify_all();
  return SQ_OK;
}

int sqobfs_pconn_stats_get(const sqobfs_pconn *pc, sqobfs_pconn_stats *out) {
  if (!pc || !out) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(const_cast<sqobfs_pconn *>(pc)->mu);
  *out = pc->st;
  return SQ_OK;
}

}  // extern "C"
