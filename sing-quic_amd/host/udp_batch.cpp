// udp_batch.cpp -- batched UDP socket I/O feeding the GPU obfuscation path
// (include/sqobfs.h, "Batched UDP socket I/O").
//
// The reference moves one datagram per syscall: each ReadFrom / WriteTo of
// SalamanderPacketConn / XPlusPacketConn wraps one read / write of the inner
// PacketConn (hysteria2/salamander.go:43,65,88; hysteria/xplus.go:47,74,97),
// and port hopping runs one recvLoop goroutine per socket into a 1024-deep
// channel of 2048-byte buffers, dropping when it is full
// (hysteria/hop.go:19,40-161).  Here a batch is received with recvmmsg from
// all of a connection's sockets at once (fan-in, round-robin, nothing
// dropped: the kernel socket buffers queue), deobfuscated by one GPU launch
// on the pinned slots, and transmitted batches are obfuscated in place by
// one launch and sent with sendmmsg.
//
// Zero copy: the slots AND the batch arrays live in one page-locked block
// mapped into the GPU's address space, and the kernel reads and writes them
// over PCIe directly (sqobfs_launch on the mapped pointers, then a stream
// sync).  A socket batch is a few hundred KiB, so one launch + sync costs far
// less than the staged H2D | kernel | D2H of sqobfs_run_host.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "sqobfs.h"

namespace {

constexpr uint32_t kMmsgChunk = 256;     // messages per recvmmsg / sendmmsg call
constexpr uint32_t kFairPerRound = 64;   // per socket per fan-in round

void to_sockaddr(const sqobfs_addr &a, sockaddr_storage *ss, socklen_t *sl) {
  memset(ss, 0, sizeof *ss);
  if (a.family == AF_INET6) {
    auto *s6 = reinterpret_cast<sockaddr_in6 *>(ss);
    s6->sin6_family = AF_INET6;
    s6->sin6_port = htons(a.port);
    s6->sin6_scope_id = a.scope_id;
    memcpy(&s6->sin6_addr, a.addr, 16);
    *sl = sizeof(sockaddr_in6);
  } else {
    auto *s4 = reinterpret_cast<sockaddr_in *>(ss);
    s4->sin_family = AF_INET;
    s4->sin_port = htons(a.port);
    memcpy(&s4->sin_addr, a.addr, 4);
    *sl = sizeof(sockaddr_in);
  }
}

void from_sockaddr(const sockaddr_storage &ss, sqobfs_addr *a) {
  memset(a, 0, sizeof *a);
  if (ss.ss_family == AF_INET6) {
    const auto *s6 = reinterpret_cast<const sockaddr_in6 *>(&ss);
    a->family = AF_INET6;
    a->port = ntohs(s6->sin6_port);
    a->scope_id = s6->sin6_scope_id;
    memcpy(a->addr, &s6->sin6_addr, 16);
  } else if (ss.ss_family == AF_INET) {
    const auto *s4 = reinterpret_cast<const sockaddr_in *>(&ss);
    a->family = AF_INET;
    a->port = ntohs(s4->sin_port);
    memcpy(a->addr, &s4->sin_addr, 4);
  }
}

}  // namespace

struct sqobfs_udp_conn {
  sqobfs_ctx *ctx = nullptr;
  const sqobfs_keyring *kr = nullptr;
  std::vector<int> fds;
  uint32_t slots = 0, slot_bytes = 0, S = 0;
  void *block = nullptr;  // page-locked, GPU-mapped: slots + batch arrays
  uint8_t *rx = nullptr, *tx = nullptr;
  std::mutex rx_mu, tx_mu;
  // receive batch (in the mapped block)
  uint64_t *rx_in_off = nullptr, *rx_out_off = nullptr;
  uint32_t *rx_len = nullptr, *rx_out_len = nullptr;
  std::vector<uint16_t> rx_fd;
  std::vector<sqobfs_addr> rx_from;
  // transmit batch (in the mapped block)
  uint64_t *tx_in_off = nullptr, *tx_out_off = nullptr;
  uint32_t *tx_len = nullptr, *tx_out_len = nullptr;
  std::vector<uint32_t> tx_wire_len;
};

namespace {

// one launch on the mapped block + wait (the conn's batches are small)
int launch_sync(sqobfs_udp_conn *c, int dir, const sqobfs_batch &b) {
  void *s = sqobfs_stream(c->ctx);
  const int st = sqobfs_launch(c->ctx, c->kr, dir, &b, s);
  return st != SQ_OK ? st : sqobfs_sync(c->ctx, s);
}

}  // namespace

extern "C" {

int sqobfs_udp_recv(const int *fds, uint32_t nfds, uint8_t *slots, uint32_t slot_bytes,
                    uint32_t headroom, uint32_t max, int timeout_ms, uint32_t *len,
                    uint16_t *fd_index, sqobfs_addr *from, uint32_t *count) {
  if (count) *count = 0;
  if (!fds || nfds == 0 || nfds > 65535 || !slots || slot_bytes <= headroom || max == 0 ||
      !len || !fd_index || !count)
    return SQ_EINVAL;
  std::vector<pollfd> pfd(nfds);
  for (uint32_t i = 0; i < nfds; i++) pfd[i] = {fds[i], POLLIN, 0};
  int r;
  do {
    r = poll(pfd.data(), nfds, timeout_ms);
  } while (r < 0 && errno == EINTR);
  if (r < 0) return -errno;
  if (r == 0) return SQ_OK;  // timeout

  const uint32_t cap = slot_bytes - headroom;
  std::vector<mmsghdr> msg(kMmsgChunk);
  std::vector<iovec> iov(kMmsgChunk);
  std::vector<sockaddr_storage> ss(kMmsgChunk);
  std::vector<bool> live(nfds, true);
  uint32_t got = 0, nlive = nfds;
  int first_err = 0;
  while (got < max && nlive > 0) {
    for (uint32_t f = 0; f < nfds && got < max; f++) {
      if (!live[f]) continue;
      const uint32_t want = std::min({max - got, kFairPerRound, kMmsgChunk});
      for (uint32_t k = 0; k < want; k++) {
        iov[k].iov_base = slots + (size_t)(got + k) * slot_bytes + headroom;
        iov[k].iov_len = cap;
        memset(&msg[k], 0, sizeof msg[k]);
        msg[k].msg_hdr.msg_iov = &iov[k];
        msg[k].msg_hdr.msg_iovlen = 1;
        msg[k].msg_hdr.msg_name = &ss[k];
        msg[k].msg_hdr.msg_namelen = sizeof ss[k];
      }
      const int m = recvmmsg(fds[f], msg.data(), want, MSG_DONTWAIT, nullptr);
      if (m < 0) {
        if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR && !first_err)
          first_err = -errno;
        if (errno != EINTR) {
          live[f] = false;
          nlive--;
        }
        continue;
      }
      for (int k = 0; k < m; k++) {
        len[got + k] = std::min<uint32_t>(msg[k].msg_len, cap);
        fd_index[got + k] = (uint16_t)f;
        if (from) from_sockaddr(ss[k], &from[got + k]);
      }
      got += (uint32_t)m;
      if ((uint32_t)m < want) {  // drained for now
        live[f] = false;
        nlive--;
      }
    }
  }
  *count = got;
  return got == 0 && first_err ? first_err : SQ_OK;
}

int sqobfs_udp_send(int fd, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                    const sqobfs_addr *to, uint32_t n, uint32_t *sent) {
  if (sent) *sent = 0;
  if (n == 0) return SQ_OK;
  if (!base || !off || !len || !to || !sent) return SQ_EINVAL;
  std::vector<mmsghdr> msg(kMmsgChunk);
  std::vector<iovec> iov(kMmsgChunk);
  std::vector<sockaddr_storage> ss(kMmsgChunk);
  uint32_t done = 0;
  while (done < n) {
    const uint32_t k_n = std::min(n - done, kMmsgChunk);
    for (uint32_t k = 0; k < k_n; k++) {
      const uint32_t i = done + k;
      iov[k].iov_base = const_cast<uint8_t *>(base + off[i]);
      iov[k].iov_len = len[i];
      memset(&msg[k], 0, sizeof msg[k]);
      socklen_t sl;
      to_sockaddr(to[i], &ss[k], &sl);
      msg[k].msg_hdr.msg_iov = &iov[k];
      msg[k].msg_hdr.msg_iovlen = 1;
      msg[k].msg_hdr.msg_name = &ss[k];
      msg[k].msg_hdr.msg_namelen = sl;
    }
    const int m = sendmmsg(fd, msg.data(), k_n, 0);
    if (m < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {  // non-blocking socket: wait
        pollfd p = {fd, POLLOUT, 0};
        if (poll(&p, 1, -1) < 0 && errno != EINTR) {
          *sent = done;
          return -errno;
        }
        continue;
      }
      *sent = done;
      return -errno;
    }
    done += (uint32_t)m;
  }
  *sent = done;
  return SQ_OK;
}

int sqobfs_udp_conn_open(sqobfs_ctx *ctx, const sqobfs_keyring *kr, const int *fds,
                         uint32_t nfds, uint32_t slots, uint32_t slot_bytes,
                         sqobfs_udp_conn **out) {
  if (out) *out = nullptr;
  if (!ctx || !kr || !fds || nfds == 0 || nfds > 65535 || slots == 0 || !out) return SQ_EINVAL;
  const int kind = sqobfs_keyring_kind(kr);
  const uint32_t S = kind == SQOBFS_SALAMANDER ? SQOBFS_SALAMANDER_SALT_LEN
                                               : SQOBFS_XPLUS_SALT_LEN;
  if (slot_bytes <= S || slot_bytes % 16) return SQ_EINVAL;
  sqobfs_udp_conn *c = new (std::nothrow) sqobfs_udp_conn();
  if (!c) return SQ_ENOMEM;
  c->ctx = ctx;
  c->kr = kr;
  c->fds.assign(fds, fds + nfds);
  c->slots = slots;
  c->slot_bytes = slot_bytes;
  c->S = S;
  // one mapped block: rx slots | tx slots | 4 u64 arrays | 4 u32 arrays
  const size_t sb = (size_t)slots * slot_bytes, a64 = 8ull * slots, a32 = 4ull * slots;
  const size_t bytes = 2 * sb + 4 * a64 + 4 * a32;
  if (sqobfs_host_alloc(ctx, bytes, &c->block) != SQ_OK) {
    delete c;
    return SQ_ENOMEM;
  }
  void *dev = nullptr;  // the GPU's view of the block (the same address on ROCm)
  if (hipHostGetDevicePointer(&dev, c->block, 0) != hipSuccess || dev != c->block) {
    (void)hipGetLastError();
    sqobfs_host_free(ctx, c->block);
    delete c;
    return SQ_EDEVICE;
  }
  uint8_t *p = (uint8_t *)c->block;
  c->rx = p;                                 p += sb;
  c->tx = p;                                 p += sb;
  c->rx_in_off = (uint64_t *)p;              p += a64;
  c->rx_out_off = (uint64_t *)p;             p += a64;
  c->tx_in_off = (uint64_t *)p;              p += a64;
  c->tx_out_off = (uint64_t *)p;             p += a64;
  c->rx_len = (uint32_t *)p;                 p += a32;
  c->rx_out_len = (uint32_t *)p;             p += a32;
  c->tx_len = (uint32_t *)p;                 p += a32;
  c->tx_out_len = (uint32_t *)p;
  c->rx_fd.resize(slots);
  c->rx_from.resize(slots);
  c->tx_wire_len.resize(slots);
  for (uint32_t i = 0; i < slots; i++) {
    c->rx_in_off[i] = (uint64_t)i * slot_bytes;       // wire at the slot start
    c->rx_out_off[i] = (uint64_t)i * slot_bytes + S;  // payload decoded in place
    c->tx_in_off[i] = (uint64_t)i * slot_bytes + S;   // payload behind S of headroom
    c->tx_out_off[i] = (uint64_t)i * slot_bytes;      // wire = salt || payload, in place
  }
  *out = c;
  return SQ_OK;
}

void sqobfs_udp_conn_close(sqobfs_udp_conn *c) {
  if (!c) return;
  sqobfs_host_free(c->ctx, c->block);
  delete c;
}

int sqobfs_udp_conn_read(sqobfs_udp_conn *c, int timeout_ms, sqobfs_udp_view *out) {
  if (!c || !out) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(c->rx_mu);
  memset(out, 0, sizeof *out);
  uint32_t n = 0;
  int st = sqobfs_udp_recv(c->fds.data(), (uint32_t)c->fds.size(), c->rx, c->slot_bytes, 0,
                           c->slots, timeout_ms, c->rx_len, c->rx_fd.data(),
                           c->rx_from.data(), &n);
  if (st != SQ_OK || n == 0) return st;
  sqobfs_batch b;
  memset(&b, 0, sizeof b);
  b.n = n;
  b.in = c->rx;
  b.in_off = c->rx_in_off;
  b.in_len = c->rx_len;
  b.out = c->rx;
  b.out_off = c->rx_out_off;
  b.out_len = c->rx_out_len;
  st = launch_sync(c, SQOBFS_DEOBFUSCATE, b);
  if (st != SQ_OK) return st;
  out->count = n;
  out->base = c->rx;
  out->off = c->rx_out_off;
  out->len = c->rx_out_len;
  out->fd_index = c->rx_fd.data();
  out->from = c->rx_from.data();
  return SQ_OK;
}

uint8_t *sqobfs_udp_conn_tx_payload(sqobfs_udp_conn *c, uint32_t i) {
  if (!c || i >= c->slots) return nullptr;
  return c->tx + (size_t)i * c->slot_bytes + c->S;
}

int sqobfs_udp_conn_write(sqobfs_udp_conn *c, uint32_t fd_index, uint32_t n,
                          const uint32_t *len, const sqobfs_addr *to, uint32_t *sent) {
  if (sent) *sent = 0;
  if (!c || !sent || fd_index >= c->fds.size() || n > c->slots) return SQ_EINVAL;
  if (n == 0) return SQ_OK;
  if (!len || !to) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(c->tx_mu);
  for (uint32_t i = 0; i < n; i++) {
    if (len[i] > c->slot_bytes - c->S) return SQ_EINVAL;
    c->tx_len[i] = len[i];
    c->tx_wire_len[i] = len[i] + c->S;
  }
  sqobfs_batch b;
  memset(&b, 0, sizeof b);
  b.n = n;
  b.flags = SQOBFS_FLAG_DEVICE_SALT;
  b.in = c->tx;
  b.in_off = c->tx_in_off;
  b.in_len = c->tx_len;
  b.out = c->tx;
  b.out_off = c->tx_out_off;
  b.out_len = c->tx_out_len;
  const int st = launch_sync(c, SQOBFS_OBFUSCATE, b);
  if (st != SQ_OK) return st;
  return sqobfs_udp_send(c->fds[fd_index], c->tx, c->tx_out_off, c->tx_wire_len.data(), to, n,
                         sent);
}

}  // extern "C"
