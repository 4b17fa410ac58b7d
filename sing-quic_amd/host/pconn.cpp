// pconn.cpp -- the obfuscating packet conn engine (include/sqobfs.h,
// "Obfuscating packet conn"): the batching core under the Go decorators
// go/sqobfs.Conn, written here so that its behaviour (coalescing, deadlines,
// shutdown, memory) is the same for every host language and is tested
// natively (tests/cpp/test_pconn.c).
//
// Reference: SalamanderPacketConn / XPlusPacketConn (hysteria2/salamander.go:
// 19-109, hysteria/xplus.go:39-118) transform one datagram per ReadFrom /
// WriteTo call on the caller's goroutine.  Here the per-call contract stays
// (one datagram in or out per call, the reference's return values) and the
// byte work moves into batches of page-locked, GPU-mapped slots, one kernel
// launch per batch:
//
//   write()  -> fill batch --(full, or the worker is idle)--> tx worker:
//               obfuscate in place (device salts) -> sendmmsg | tx_take
//   recvmmsg | rx_push -> rx batch -> rx worker: deobfuscate in place ->
//               ready queue -> read() copies one datagram out
//
// Natural batching: a worker takes whatever has accumulated as soon as it
// is idle, so a lone packet (a handshake, an ACK) is launched at once and
// the datagrams written during a launch form the next batch.  linger_us
// trades latency for larger batches when asked.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <netinet/udp.h>
#include <poll.h>
#include <string.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "sq_internal.h"
#include "sq_sockaddr.h"
#include "sqobfs.h"

namespace {

constexpr uint32_t kDefBatch = 256, kDefSlot = 2048, kDefBatches = 3, kDefSpinUs = 200;
constexpr uint32_t kMaxBatch = 1u << 16;
constexpr int64_t kDrainNs = 200'000'000;  // shutdown: time given to queued writes
constexpr uint32_t kMmsg = 256;            // messages per sendmmsg / recvmmsg call
constexpr uint32_t kGsoMaxSegs = 64;       // UDP_MAX_SEGMENTS of older kernels
constexpr uint32_t kGsoMaxBytes = 65000;   // one GSO send stays below 64 KiB of IP payload
constexpr uint32_t kGroBuf = 65536;        // one coalesced receive
constexpr size_t kCtlWords = (CMSG_SPACE(sizeof(uint16_t)) + 7) / 8;

int64_t unix_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
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

// One batch: its slots and descriptor arrays live in the mapped block (the
// kernel reads and writes them over PCIe), addresses and tags on the host.
struct PBatch {
  uint32_t n = 0;       // datagrams in the batch
  uint32_t next = 0;    // rx: next datagram read() hands out
  int64_t first_ns = 0; // monotonic time of the first datagram (linger)
  uint8_t *slots = nullptr;
  uint64_t *in_off = nullptr, *out_off = nullptr;
  uint32_t *len = nullptr, *out_len = nullptr;
  std::vector<sqobfs_addr> addr;
  std::vector<uint64_t> tag;
  std::vector<uint8_t> head;  // rx: the first 16 wire bytes of each datagram
};

}  // namespace

struct sqobfs_pconn {
  sqobfs_ctx *ctx = nullptr;
  const sqobfs_keyring *kr = nullptr;
  int kind = 0;
  uint32_t S = 0;
  int fd = -1;    // socket mode: our dup of the caller's socket
  int wake = -1;  // eventfd, readable after shutdown (wakes poll)
  sqobfs_pconn_opts o{};
  void *block = nullptr;
  void *txs = nullptr, *rxs = nullptr;  // private streams
  std::vector<PBatch> tb, rb;

  std::mutex mu;
  std::condition_variable cv_txw;   // tx worker: work arrived
  std::condition_variable cv_txs;   // writers: a tx batch freed; shutdown: drained
  std::condition_variable cv_rxw;   // pump rx worker: work arrived
  std::condition_variable cv_rxr;   // readers: a batch is ready
  std::condition_variable cv_rxs;   // rx worker / pushers: an rx batch freed
  std::condition_variable cv_take;  // pump taker: an obfuscated batch is ready
  std::deque<uint32_t> tfree, tq, ttaken, rfree, rq, rready;
  int tfill = -1, rfill = -1;
  bool tx_busy = false;      // tx worker is launching / sending a batch
  bool rx_busy = false;      // pump rx worker is launching
  bool taken = false;        // pump: the front of ttaken is out with the taker
  bool writes_closed = false;
  bool closed = false;
  int tx_err = 0;            // reported once by the next write
  int rx_err = 0;            // reported once the ready queue is empty
  bool rx_err_sticky = false;
  int64_t rdl = 0, wdl = 0;  // deadlines, unix ns (0 = none)
  sqobfs_pconn_stats st{};
  std::mutex join_mu;
  std::thread txw, rxw;
  // sendmmsg / recvmmsg scratch (owned by the tx / rx worker thread)
  std::vector<mmsghdr> tmsg, rmsg;
  std::vector<iovec> tiov, riov;
  std::vector<sockaddr_storage> tss, rss;
  std::vector<uint64_t> tctl, rctl;  // UDP_SEGMENT / UDP_GRO control messages
  std::vector<uint32_t> tfirst;      // first datagram of each transmit message
  bool gso = false, gro = false;     // offloads in effect (socket mode)

  bool socket_mode() const { return fd >= 0; }
  uint8_t *slot(PBatch &b, uint32_t i) { return b.slots + (size_t)i * o.slot_bytes; }
};

namespace {

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

int launch_wait(sqobfs_pconn *pc, void *stream, int dir, PBatch &b, bool slotted = true) {
  sqobfs_batch d;
  memset(&d, 0, sizeof d);
  d.n = b.n;
  // slots are multiples of 16 bytes: every output owns its blocks, so the
  // kernel writes them whole (SQOBFS_FLAG_OUT_BLOCKS); GRO buffers pack the
  // datagrams back to back (no flag)
  d.flags = (slotted ? SQOBFS_FLAG_OUT_BLOCKS : 0u) |
            (dir == SQOBFS_OBFUSCATE ? SQOBFS_FLAG_DEVICE_SALT : 0u);
  d.in = b.slots;
  d.in_off = b.in_off;
  d.in_len = b.len;
  d.out = b.slots;
  d.out_off = b.out_off;
  d.out_len = b.out_len;
  const int st = sqobfs_launch(pc->ctx, pc->kr, dir, &d, stream);
  if (st != SQ_OK) return st;
  return sq_ctx_stream_wait(pc->ctx, stream, pc->o.spin_us);
}

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
  // messages over datagrams [from, n)
  uint32_t nm = 0;
  for (uint32_t i = from; i < b.n;) {
    uint32_t j = i + 1;
    if (pc->gso) {
      const uint32_t g = b.out_len[i];
      uint32_t bytes = g;
      while (j < b.n && j - i < kGsoMaxSegs && g > 0 && b.out_len[j] <= g && b.out_len[j] > 0 &&
             bytes + b.out_len[j] <= kGsoMaxBytes &&
             memcmp(&b.addr[j], &b.addr[i], sizeof b.addr[i]) == 0) {
        bytes += b.out_len[j];
        j++;
        if (b.out_len[j - 1] < g) break;
      }
    }
    for (uint32_t k = i; k < j; k++) {
      pc->tiov[k].iov_base = pc->slot(b, k);
      pc->tiov[k].iov_len = b.out_len[k];
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
      const uint16_t gs = (uint16_t)b.out_len[i];
      memcpy(CMSG_DATA(cm), &gs, sizeof gs);
    }
    pc->tfirst[nm++] = i;
    i = j;
  }
  uint32_t done = 0;
  while (done < nm) {
    const uint32_t k = std::min(nm - done, kMmsg);
    const int m = sendmmsg(pc->fd, &pc->tmsg[done], k, MSG_DONTWAIT);
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

// ---- transmit worker: socket mode sends, pump mode hands to the taker
void tx_worker(sqobfs_pconn *pc) {
  std::unique_lock<std::mutex> lk(pc->mu);
  for (;;) {
    // wait for a queued batch, or promote the filling one (at once, or after
    // linger_us from its first datagram)
    for (;;) {
      if (pc->closed) return;
      if (!pc->tq.empty()) break;
      if (pc->tfill >= 0 && pc->tb[pc->tfill].n > 0) {
        const int64_t due = pc->tb[pc->tfill].first_ns + (int64_t)pc->o.linger_us * 1000;
        if (pc->o.linger_us == 0 || pc->writes_closed || mono_ns() >= due) {
          pc->tq.push_back((uint32_t)pc->tfill);
          pc->tfill = -1;
          break;
        }
        pc->cv_txw.wait_until(lk, mono_tp(due));
        continue;
      }
      pc->cv_txw.wait(lk);
    }
    const uint32_t idx = pc->tq.front();
    pc->tq.pop_front();
    pc->tx_busy = true;
    PBatch &b = pc->tb[idx];
    lk.unlock();
    int st = launch_wait(pc, pc->txs, SQOBFS_OBFUSCATE, b);
    int send_err = 0;
    uint64_t nerr = 0;
    if (st == SQ_OK && pc->socket_mode()) st = send_batch(pc, b, 0, &send_err, &nerr);
    lk.lock();
    pc->tx_busy = false;
    if (st != SQ_OK && st != SQ_ECLOSED && !pc->tx_err) pc->tx_err = st;
    if (send_err && !pc->tx_err) pc->tx_err = send_err;
    pc->st.tx_send_errors += nerr;
    if (st == SQ_OK) {
      pc->st.tx_datagrams += b.n;
      pc->st.tx_batches++;
      pc->st.tx_max_batch = std::max(pc->st.tx_max_batch, b.n);
    }
    if (st == SQ_OK && !pc->socket_mode()) {
      pc->ttaken.push_back(idx);
      pc->cv_take.notify_one();
    } else {
      b.n = 0;
      pc->tfree.push_back(idx);
      pc->cv_txs.notify_all();
    }
  }
}

// ---- receive worker, socket mode: recvmmsg a batch, deobfuscate, publish
void rx_worker_socket(sqobfs_pconn *pc) {
  for (;;) {
    uint32_t idx;
    {
      std::unique_lock<std::mutex> lk(pc->mu);
      pc->cv_rxs.wait(lk, [&] { return pc->closed || !pc->rfree.empty(); });
      if (pc->closed) return;
      idx = pc->rfree.front();
      pc->rfree.pop_front();
    }
    PBatch &b = pc->rb[idx];
    int m = 0;
    // GRO: the batch's slot region as 64 KiB buffers of up to 64 coalesced
    // datagrams each (so the batch arrays always have room)
    const uint32_t ngro = pc->gro ? std::max<uint32_t>(1, std::min<uint64_t>(
                                        (uint64_t)pc->o.batch * pc->o.slot_bytes / kGroBuf,
                                        pc->o.batch / kGsoMaxSegs))
                                  : 0;
    for (;;) {
      pollfd p[2] = {{pc->fd, POLLIN, 0}, {pc->wake, POLLIN, 0}};
      const int r = poll(p, 2, -1);
      if (r < 0 && errno == EINTR) continue;
      if (p[1].revents & POLLIN) return;  // shutdown
      const uint32_t want = pc->gro ? ngro : pc->o.batch;
      for (uint32_t j = 0; j < want; j++) {
        pc->riov[j].iov_base = pc->gro ? b.slots + (size_t)j * kGroBuf : pc->slot(b, j);
        pc->riov[j].iov_len = pc->gro ? kGroBuf : pc->o.slot_bytes;
        memset(&pc->rmsg[j], 0, sizeof pc->rmsg[j]);
        pc->rmsg[j].msg_hdr.msg_iov = &pc->riov[j];
        pc->rmsg[j].msg_hdr.msg_iovlen = 1;
        pc->rmsg[j].msg_hdr.msg_name = &pc->rss[j];
        pc->rmsg[j].msg_hdr.msg_namelen = sizeof pc->rss[j];
        if (pc->gro) {
          pc->rmsg[j].msg_hdr.msg_control = &pc->rctl[8ull * j];
          pc->rmsg[j].msg_hdr.msg_controllen = 8 * sizeof(uint64_t);
        }
      }
      m = recvmmsg(pc->fd, pc->rmsg.data(), want, MSG_DONTWAIT, nullptr);
      if (m > 0) break;
      const int e = m < 0 ? errno : EAGAIN;
      if (e == EAGAIN || e == EWOULDBLOCK || e == EINTR) continue;
      // ICMP-reported errors are per datagram (the next read works);
      // anything else ends the receive side
      std::lock_guard<std::mutex> lk(pc->mu);
      pc->rx_err = SQOBFS_ERRNO(e);
      const bool transient = e == ECONNREFUSED || e == EHOSTUNREACH || e == ENETUNREACH;
      pc->rx_err_sticky = !transient;
      pc->cv_rxr.notify_all();
      if (!transient) return;
    }
    uint64_t trunc = 0;
    uint32_t n = 0;
    if (pc->gro) {
      // split every coalesced message into its datagrams (cmsg UDP_GRO gives
      // the segment size; the last may be shorter), decoded in place
      for (int j = 0; j < m; j++) {
        const uint32_t total = pc->rmsg[j].msg_len;
        uint32_t seg = total;
        for (cmsghdr *cm = CMSG_FIRSTHDR(&pc->rmsg[j].msg_hdr); cm;
             cm = CMSG_NXTHDR(&pc->rmsg[j].msg_hdr, cm))
          if (cm->cmsg_level == SOL_UDP && cm->cmsg_type == UDP_GRO) {
            int v;
            memcpy(&v, CMSG_DATA(cm), sizeof v);
            if (v > 0) seg = (uint32_t)v;
          }
        if (pc->rmsg[j].msg_hdr.msg_flags & MSG_TRUNC) trunc++;
        sqobfs_addr from;
        sq::from_sockaddr(pc->rss[j], &from);
        const uint64_t base = (uint64_t)j * kGroBuf;
        for (uint32_t o = 0; (o < total || (total == 0 && o == 0)) && n < pc->o.batch;
             o += seg ? seg : 1) {
          const uint32_t l = std::min(seg, total - o);
          b.in_off[n] = base + o;
          b.out_off[n] = base + o + pc->S;
          b.len[n] = l;
          memcpy(&b.head[16ull * n], b.slots + base + o, std::min<uint32_t>(16, l));
          b.addr[n] = from;
          b.tag[n] = 0;
          n++;
          if (total == 0) break;
        }
      }
    } else {
      for (int j = 0; j < m; j++) {
        b.len[j] = std::min<uint32_t>(pc->rmsg[j].msg_len, pc->o.slot_bytes);
        memcpy(&b.head[16ull * j], pc->slot(b, (uint32_t)j), 16);
        if (pc->rmsg[j].msg_hdr.msg_flags & MSG_TRUNC) trunc++;
        sq::from_sockaddr(pc->rss[j], &b.addr[j]);
        b.tag[j] = 0;
      }
      n = (uint32_t)m;
    }
    b.n = n;
    b.next = 0;
    const int st = launch_wait(pc, pc->rxs, SQOBFS_DEOBFUSCATE, b, !pc->gro);
    std::lock_guard<std::mutex> lk(pc->mu);
    pc->st.rx_truncated += trunc;
    if (st != SQ_OK) {
      pc->rx_err = st;
      pc->rx_err_sticky = true;
      pc->cv_rxr.notify_all();
      return;
    }
    pc->st.rx_datagrams += b.n;
    pc->st.rx_batches++;
    pc->st.rx_max_batch = std::max(pc->st.rx_max_batch, b.n);
    pc->rready.push_back(idx);
    pc->cv_rxr.notify_all();
  }
}

// ---- receive worker, pump mode: the caller pushes datagrams; launch
// batches as the tx worker does
void rx_worker_pump(sqobfs_pconn *pc) {
  std::unique_lock<std::mutex> lk(pc->mu);
  for (;;) {
    for (;;) {
      if (pc->closed) return;
      if (!pc->rq.empty()) break;
      if (pc->rfill >= 0 && pc->rb[pc->rfill].n > 0) {
        const int64_t due = pc->rb[pc->rfill].first_ns + (int64_t)pc->o.linger_us * 1000;
        if (pc->o.linger_us == 0 || mono_ns() >= due) {
          pc->rq.push_back((uint32_t)pc->rfill);
          pc->rfill = -1;
          break;
        }
        pc->cv_rxw.wait_until(lk, mono_tp(due));
        continue;
      }
      pc->cv_rxw.wait(lk);
    }
    const uint32_t idx = pc->rq.front();
    pc->rq.pop_front();
    pc->rx_busy = true;
    PBatch &b = pc->rb[idx];
    b.next = 0;
    lk.unlock();
    const int st = launch_wait(pc, pc->rxs, SQOBFS_DEOBFUSCATE, b);
    lk.lock();
    pc->rx_busy = false;
    if (st != SQ_OK) {
      pc->rx_err = st;
      pc->rx_err_sticky = true;
      pc->cv_rxr.notify_all();
      return;
    }
    pc->st.rx_datagrams += b.n;
    pc->st.rx_batches++;
    pc->st.rx_max_batch = std::max(pc->st.rx_max_batch, b.n);
    pc->rready.push_back(idx);
    pc->cv_rxr.notify_all();
  }
}

void free_pconn(sqobfs_pconn *pc) {
  if (pc->txs) {
    sq_ctx_stream_destroy(pc->ctx, pc->txs);  // synchronises first
    sq_keyring_forget(pc->kr, pc->txs);
  }
  if (pc->rxs) {
    sq_ctx_stream_destroy(pc->ctx, pc->rxs);
    sq_keyring_forget(pc->kr, pc->rxs);
  }
  if (pc->block) sqobfs_host_free(pc->ctx, pc->block);
  if (pc->fd >= 0) close(pc->fd);
  if (pc->wake >= 0) close(pc->wake);
  delete pc;
}

}  // namespace

extern "C" {

int sqobfs_pconn_open(sqobfs_ctx *ctx, const sqobfs_keyring *kr, int fd,
                      const sqobfs_pconn_opts *opts, sqobfs_pconn **out) {
  if (out) *out = nullptr;
  if (!ctx || !kr || !out) return SQ_EINVAL;
  sqobfs_pconn_opts o{};
  if (opts) o = *opts;
  if (o.batch == 0) o.batch = kDefBatch;
  if (o.slot_bytes == 0) o.slot_bytes = kDefSlot;
  if (o.tx_batches == 0) o.tx_batches = kDefBatches;
  if (o.rx_batches == 0) o.rx_batches = kDefBatches;
  if (o.spin_us == 0) o.spin_us = kDefSpinUs;
  const int kind = sqobfs_keyring_kind(kr);
  const uint32_t S = kind == SQOBFS_SALAMANDER ? SQOBFS_SALAMANDER_SALT_LEN : SQOBFS_XPLUS_SALT_LEN;
  if (o.batch > kMaxBatch || o.slot_bytes % 16 || o.slot_bytes <= S ||
      (o.flags & ~(uint32_t)(SQOBFS_UDP_TX_GSO | SQOBFS_UDP_RX_GRO)) || o.tx_batches > 64 ||
      o.rx_batches > 64)
    return SQ_EINVAL;
  sqobfs_pconn *pc = new (std::nothrow) sqobfs_pconn();
  if (!pc) return SQ_ENOMEM;
  pc->ctx = ctx;
  pc->kr = kr;
  pc->kind = kind;
  pc->S = S;
  pc->o = o;
  if (fd >= 0) {
    pc->fd = fcntl(fd, F_DUPFD_CLOEXEC, 0);
    if (pc->fd < 0) {
      const int e = errno;
      delete pc;
      return SQOBFS_ERRNO(e);
    }
  }
  pc->wake = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  if (pc->wake < 0) {
    free_pconn(pc);
    return SQ_ENOMEM;
  }
  // one mapped block: all slots, then per batch 2 u64 + 2 u32 arrays
  const uint32_t nb = o.tx_batches + o.rx_batches, B = o.batch;
  const size_t slots = (size_t)B * o.slot_bytes, arrays = (size_t)B * (8 + 8 + 4 + 4);
  int st = sqobfs_host_alloc(ctx, (size_t)nb * (slots + arrays), &pc->block);
  void *dev = nullptr;  // the GPU's view of the block (the same address on ROCm)
  if (st == SQ_OK && (hipHostGetDevicePointer(&dev, pc->block, 0) != hipSuccess ||
                      dev != pc->block)) {
    (void)hipGetLastError();
    st = SQ_EDEVICE;
  }
  if (st == SQ_OK) st = sq_ctx_stream_create(ctx, &pc->txs);
  if (st == SQ_OK) st = sq_ctx_stream_create(ctx, &pc->rxs);
  if (st != SQ_OK) {
    free_pconn(pc);
    return st;
  }
  uint8_t *p = (uint8_t *)pc->block, *a = p + (size_t)nb * slots;
  pc->tb.resize(o.tx_batches);
  pc->rb.resize(o.rx_batches);
  for (uint32_t k = 0; k < nb; k++) {
    const bool tx = k < o.tx_batches;
    PBatch &b = tx ? pc->tb[k] : pc->rb[k - o.tx_batches];
    b.slots = p + (size_t)k * slots;
    b.in_off = (uint64_t *)a;   a += 8ull * B;
    b.out_off = (uint64_t *)a;  a += 8ull * B;
    b.len = (uint32_t *)a;      a += 4ull * B;
    b.out_len = (uint32_t *)a;  a += 4ull * B;
    b.addr.resize(B);
    b.tag.resize(B);
    if (!tx) b.head.resize(16ull * B);
    for (uint32_t i = 0; i < B; i++) {
      const uint64_t s0 = (uint64_t)i * o.slot_bytes;
      // tx: payload behind S bytes of headroom, wire = salt || payload in
      // place from the slot start (the vectorised writers' layout,
      // salamander.go:81-93); rx: wire at the slot start, payload decoded in
      // place behind the salt
      b.in_off[i] = tx ? s0 + S : s0;
      b.out_off[i] = tx ? s0 : s0 + S;
    }
    if (tx) pc->tfree.push_back(k);
    else pc->rfree.push_back(k - o.tx_batches);
  }
  if (pc->socket_mode()) {
    pc->tmsg.resize(B);
    pc->tiov.resize(B);
    pc->tss.resize(B);
    pc->tctl.assign(kCtlWords * B, 0);
    pc->tfirst.resize(B);
    pc->rmsg.resize(B);
    pc->riov.resize(B);
    pc->rss.resize(B);
    pc->gso = o.flags & SQOBFS_UDP_TX_GSO;  // probed by the first send
    if ((o.flags & SQOBFS_UDP_RX_GRO) && B >= kGsoMaxSegs &&
        (uint64_t)B * o.slot_bytes >= kGroBuf) {
      const int one = 1;
      pc->gro = setsockopt(pc->fd, SOL_UDP, UDP_GRO, &one, sizeof one) == 0;
      if (pc->gro) pc->rctl.assign(8ull * B, 0);
    }
  }
  try {
    pc->txw = std::thread(tx_worker, pc);
    pc->rxw = pc->socket_mode() ? std::thread(rx_worker_socket, pc) : std::thread(rx_worker_pump, pc);
  } catch (...) {
    sqobfs_pconn_shutdown(pc);
    free_pconn(pc);
    return SQ_ENOMEM;
  }
  *out = pc;
  return SQ_OK;
}

void sqobfs_pconn_shutdown(sqobfs_pconn *pc) {
  if (!pc) return;
  {
    std::unique_lock<std::mutex> lk(pc->mu);
    if (!pc->writes_closed) {
      pc->writes_closed = true;
      pc->cv_txw.notify_all();
      pc->cv_txs.notify_all();
      // what was written goes out: wait (bounded) until the transmit side
      // has drained -- sent, or taken and done by the pump taker
      const int64_t until = mono_ns() + kDrainNs;
      while (!pc->closed && (pc->tx_busy || !pc->tq.empty() || !pc->ttaken.empty() ||
                             (pc->tfill >= 0 && pc->tb[pc->tfill].n > 0))) {
        if (mono_ns() >= until) break;
        pc->cv_txs.wait_until(lk, mono_tp(std::min(until, mono_ns() + 5'000'000)));
      }
      pc->closed = true;
      for (auto *cv : {&pc->cv_txw, &pc->cv_txs, &pc->cv_rxw, &pc->cv_rxr, &pc->cv_rxs,
                       &pc->cv_take})
        cv->notify_all();
    }
  }
  if (pc->wake >= 0) {
    const uint64_t one = 1;
    (void)!write(pc->wake, &one, sizeof one);
  }
  std::lock_guard<std::mutex> jl(pc->join_mu);
  if (pc->txw.joinable()) pc->txw.join();
  if (pc->rxw.joinable()) pc->rxw.join();
}

void sqobfs_pconn_close(sqobfs_pconn *pc) {
  if (!pc) return;
  sqobfs_pconn_shutdown(pc);
  free_pconn(pc);
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
  if (pc->tfill < 0) {
    const bool ok = wait_dl(lk, pc->cv_txs, pc->wdl, [&] {
      return pc->writes_closed || pc->tfill >= 0 || !pc->tfree.empty();
    });
    if (pc->writes_closed) return SQ_ECLOSED;
    if (!ok) return SQ_ETIMEDOUT;
    if (pc->tfill < 0) {  // (another writer may have opened one meanwhile)
      pc->tfill = (int)pc->tfree.front();
      pc->tfree.pop_front();
      pc->tb[pc->tfill].n = 0;
    }
  }
  PBatch &b = pc->tb[pc->tfill];
  const uint32_t i = b.n++;
  if (i == 0) b.first_ns = mono_ns();
  if (len) memcpy(pc->slot(b, i) + pc->S, p, len);
  b.len[i] = len;
  if (to) b.addr[i] = *to;
  else memset(&b.addr[i], 0, sizeof b.addr[i]);
  b.tag[i] = tag;
  if (b.n == pc->o.batch) {
    pc->tq.push_back((uint32_t)pc->tfill);
    pc->tfill = -1;
    pc->cv_txw.notify_one();
  } else if (i == 0 && !pc->tx_busy) {
    pc->cv_txw.notify_one();  // an idle worker takes it at once (or lingers)
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
  const uint32_t i = b.next++;
  // the reference reads the datagram into p (cut to len(p)) and decodes
  // what it got: m = min(wire, cap)
  const uint32_t w = b.len[i], m = std::min(w, cap), S = pc->S;
  uint32_t r = 0;
  const uint8_t *src = nullptr;
  if (pc->kind == SQOBFS_SALAMANDER && m <= S) {
    r = m;                       // salamander.go:47-49: returned as is
    src = &b.head[16ull * i];    // the raw bytes (the decode wrote the slot's head)
  } else if (pc->kind == SQOBFS_XPLUS && m < S) {
    r = 0;                  // xplus.go:50-52
  } else {
    r = m - S;              // the first m - S payload bytes
    src = b.slots + b.out_off[i];
  }
  if (r) memcpy(p, src, r);
  *n = r;
  if (from) *from = b.addr[i];
  if (tag) *tag = b.tag[i];
  if (b.next == b.n) {
    pc->rready.pop_front();
    b.n = 0;
    pc->rfree.push_back(idx);
    pc->cv_rxs.notify_all();
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
      pc->rfill = (int)pc->rfree.front();
      pc->rfree.pop_front();
      pc->rb[pc->rfill].n = 0;
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
  b.len[i] = m;
  if (from) b.addr[i] = *from;
  else memset(&b.addr[i], 0, sizeof b.addr[i]);
  b.tag[i] = tag;
  if (b.n == pc->o.batch) {
    pc->rq.push_back((uint32_t)pc->rfill);
    pc->rfill = -1;
    pc->cv_rxw.notify_one();
  } else if (i == 0 && !pc->rx_busy) {
    pc->cv_rxw.notify_one();
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
  out->base = b.slots;
  out->off = b.out_off;
  out->len = b.out_len;
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
  pc->tb[idx].n = 0;
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
