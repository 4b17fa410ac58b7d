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
#include <netinet/in.h>
#include <netinet/udp.h>
#include <poll.h>
#include <string.h>
#include <sys/random.h>
#include <sys/socket.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "sq_internal.h"
#include "sq_sockaddr.h"
#include "sqobfs.h"

namespace {

constexpr uint32_t kMmsgChunk = 256;     // messages per recvmmsg / sendmmsg call
constexpr uint32_t kFairPerRound = 64;   // per socket per fan-in round
constexpr uint32_t kGsoMaxSegs = 64;     // UDP_MAX_SEGMENTS of older kernels
constexpr uint32_t kGsoMaxBytes = 65000; // one GSO send stays below 64 KiB of IP payload
constexpr uint32_t kGroBuf = 65536;      // one coalesced receive

using sq::from_sockaddr;
using sq::to_sockaddr;

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
  uint32_t offload = 0;  // SQOBFS_UDP_TX_GSO | SQOBFS_UDP_RX_GRO in effect
  // QUIC batch arrays (in the mapped block).  Transmit and receive have
  // their own (a reader and a writer thread run at once, under different
  // locks: sharing the packet-number array would let one direction seal
  // under the other's packet numbers, i.e. reuse an AEAD nonce).
  uint64_t *qpn_tx = nullptr;               // write_quic: packet numbers
  uint16_t *qpno_tx = nullptr;              // write_quic: pn offsets
  uint8_t *qsalt = nullptr;                 // write_quic: Salamander salts
  uint64_t *qpn_rx = nullptr, *qpn_out = nullptr;  // read_quic: largest pn / decoded
  uint16_t *qpno_rx = nullptr;              // read_quic: pn offsets
};

namespace {

// one launch on the mapped block + wait (the conn's batches are small: poll
// the stream for a while instead of paying the blocking wake-up)
constexpr uint32_t kLaunchSpinUs = 200;
int launch_sync(sqobfs_udp_conn *c, int dir, const sqobfs_batch &b) {
  void *s = sqobfs_stream(c->ctx);
  const int st = sqobfs_launch(c->ctx, c->kr, dir, &b, s);
  return st != SQ_OK ? st : sq_ctx_stream_wait(c->ctx, s, kLaunchSpinUs);
}

// sendmmsg of msg[0..n), waiting while the socket buffer is full.  Returns
// the number of messages handed to the kernel, or -errno if none was.
int send_all(int fd, mmsghdr *msg, uint32_t n, uint32_t *done_msgs) {
  uint32_t done = 0;
  while (done < n) {
    const int m = sendmmsg(fd, msg + done, n - done, 0);
    if (m < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd p = {fd, POLLOUT, 0};
        if (poll(&p, 1, -1) < 0 && errno != EINTR) break;
        continue;
      }
      *done_msgs = done;
      return -errno;
    }
    done += (uint32_t)m;
  }
  *done_msgs = done;
  return SQ_OK;
}

// (Re)set the receive batch offsets to the fixed slot layout.
void rx_fixed_offsets(sqobfs_udp_conn *c) {
  for (uint32_t i = 0; i < c->slots; i++) {
    c->rx_in_off[i] = (uint64_t)i * c->slot_bytes;
    c->rx_out_off[i] = (uint64_t)i * c->slot_bytes + c->S;
  }
}

// Fan-in receive with UDP GRO: recvmmsg into 64 KiB buffers laid over the
// rx region; a coalesced message holds several datagrams of gso_size bytes
// (the last may be shorter, cmsg UDP_GRO).  Writes the batch offsets.
int recv_gro(sqobfs_udp_conn *c, int timeout_ms, uint32_t *count) {
  *count = 0;
  const uint32_t nfds = (uint32_t)c->fds.size();
  std::vector<pollfd> pfd(nfds);
  for (uint32_t i = 0; i < nfds; i++) pfd[i] = {c->fds[i], POLLIN, 0};
  int r;
  do {
    r = poll(pfd.data(), nfds, timeout_ms);
  } while (r < 0 && errno == EINTR);
  if (r < 0) return -errno;
  if (r == 0) return SQ_OK;
  const uint64_t region = (uint64_t)c->slots * c->slot_bytes;
  // at most kGsoMaxSegs datagrams per buffer, so the batch arrays (slots
  // entries) always have room for a whole buffer
  const uint32_t nbuf = std::max<uint32_t>(
      1, std::min<uint64_t>(region / kGroBuf, c->slots / kGsoMaxSegs));
  std::vector<mmsghdr> msg(nbuf);
  std::vector<iovec> iov(nbuf);
  std::vector<sockaddr_storage> ss(nbuf);
  std::vector<uint64_t> ctl(nbuf * 8);
  std::vector<bool> live(nfds, true);
  uint32_t got = 0, used = 0, nlive = nfds;
  int first_err = 0;
  while (used < nbuf && nlive > 0) {
    for (uint32_t f = 0; f < nfds && used < nbuf; f++) {
      if (!live[f]) continue;
      const uint32_t want = nbuf - used;
      for (uint32_t k = 0; k < want; k++) {
        iov[k].iov_base = c->rx + (size_t)(used + k) * kGroBuf;
        iov[k].iov_len = kGroBuf;
        memset(&msg[k], 0, sizeof msg[k]);
        msg[k].msg_hdr.msg_iov = &iov[k];
        msg[k].msg_hdr.msg_iovlen = 1;
        msg[k].msg_hdr.msg_name = &ss[k];
        msg[k].msg_hdr.msg_namelen = sizeof ss[k];
        msg[k].msg_hdr.msg_control = &ctl[8 * k];
        msg[k].msg_hdr.msg_controllen = 8 * sizeof(uint64_t);
      }
      const int m = recvmmsg(c->fds[f], msg.data(), want, MSG_DONTWAIT, nullptr);
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
        const uint32_t total = msg[k].msg_len;
        uint32_t seg = total;
        for (cmsghdr *cm = CMSG_FIRSTHDR(&msg[k].msg_hdr); cm;
             cm = CMSG_NXTHDR(&msg[k].msg_hdr, cm))
          if (cm->cmsg_level == SOL_UDP && cm->cmsg_type == UDP_GRO) {
            int v;
            memcpy(&v, CMSG_DATA(cm), sizeof v);
            if (v > 0) seg = (uint32_t)v;
          }
        const uint64_t base = (uint64_t)(used + k) * kGroBuf;
        sqobfs_addr from;
        from_sockaddr(ss[k], &from);
        for (uint32_t o = 0; o < total || (total == 0 && o == 0); o += seg ? seg : 1) {
          const uint32_t l = std::min(seg, total - o);
          c->rx_in_off[got] = base + o;
          c->rx_out_off[got] = base + o + c->S;
          c->rx_len[got] = l;
          c->rx_fd[got] = (uint16_t)f;
          c->rx_from[got] = from;
          got++;
          if (total == 0) break;
        }
      }
      used += (uint32_t)m;
      if ((uint32_t)m < want) {
        live[f] = false;
        nlive--;
      }
    }
  }
  *count = got;
  return got == 0 && first_err ? first_err : SQ_OK;
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

int sqobfs_udp_send_gso(int fd, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        const sqobfs_addr *to, uint32_t n, uint32_t *sent) {
  if (sent) *sent = 0;
  if (n == 0) return SQ_OK;
  if (!base || !off || !len || !to || !sent) return SQ_EINVAL;
  std::vector<mmsghdr> msg;
  std::vector<iovec> iov(n);
  std::vector<sockaddr_storage> ss;
  std::vector<uint64_t> ctl;
  std::vector<uint32_t> first;  // first datagram of each message
  msg.reserve(n);
  ss.reserve(n);
  first.reserve(n + 1);
  constexpr size_t kCtlWords = (CMSG_SPACE(sizeof(uint16_t)) + 7) / 8;  // 24 bytes
  ctl.reserve(kCtlWords * n);
  for (uint32_t i = 0; i < n;) {
    // a run to one destination: every datagram gso bytes, the last <= gso
    const uint32_t gso = len[i];
    uint32_t j = i + 1, bytes = gso;
    while (j < n && j - i < kGsoMaxSegs && gso > 0 && len[j] <= gso && len[j] > 0 &&
           bytes + len[j] <= kGsoMaxBytes && memcmp(&to[j], &to[i], sizeof to[i]) == 0) {
      bytes += len[j];
      j++;
      if (len[j - 1] < gso) break;
    }
    for (uint32_t k = i; k < j; k++) {
      iov[k].iov_base = const_cast<uint8_t *>(base + off[k]);
      iov[k].iov_len = len[k];
    }
    mmsghdr h;
    memset(&h, 0, sizeof h);
    ss.emplace_back();
    socklen_t sl;
    to_sockaddr(to[i], &ss.back(), &sl);
    h.msg_hdr.msg_name = &ss.back();
    h.msg_hdr.msg_namelen = sl;
    h.msg_hdr.msg_iov = &iov[i];
    h.msg_hdr.msg_iovlen = j - i;
    if (j - i > 1) {  // UDP_SEGMENT: the kernel cuts the message into gso-byte datagrams
      ctl.resize(ctl.size() + kCtlWords, 0);  // within the reservation: no reallocation
      h.msg_hdr.msg_control = &ctl[ctl.size() - kCtlWords];
      h.msg_hdr.msg_controllen = CMSG_SPACE(sizeof(uint16_t));
      cmsghdr *cm = CMSG_FIRSTHDR(&h.msg_hdr);
      cm->cmsg_level = SOL_UDP;
      cm->cmsg_type = UDP_SEGMENT;
      cm->cmsg_len = CMSG_LEN(sizeof(uint16_t));
      const uint16_t g = (uint16_t)gso;
      memcpy(CMSG_DATA(cm), &g, sizeof g);
    }
    msg.push_back(h);
    first.push_back(i);
    i = j;
  }
  first.push_back(n);
  uint32_t done_msgs = 0;
  int st = SQ_OK;
  for (uint32_t m0 = 0; m0 < msg.size() && st == SQ_OK;) {
    const uint32_t k_n = std::min<uint32_t>((uint32_t)msg.size() - m0, kMmsgChunk);
    uint32_t d = 0;
    st = send_all(fd, msg.data() + m0, k_n, &d);
    done_msgs = m0 + d;
    m0 += k_n;
  }
  *sent = first[done_msgs];
  return st;
}

int sqobfs_udp_conn_set_offload(sqobfs_udp_conn *c, uint32_t flags) {
  if (!c || (flags & ~(SQOBFS_UDP_TX_GSO | SQOBFS_UDP_RX_GRO))) return SQ_EINVAL;
  std::lock_guard<std::mutex> lr(c->rx_mu);
  std::lock_guard<std::mutex> lt(c->tx_mu);
  uint32_t on = flags & SQOBFS_UDP_TX_GSO;  // probed on the first send
  const bool gro_fits = c->slots >= kGsoMaxSegs && (uint64_t)c->slots * c->slot_bytes >= kGroBuf;
  const int want_gro = (flags & SQOBFS_UDP_RX_GRO) && gro_fits ? 1 : 0;
  bool gro_ok = true;
  for (int fd : c->fds)
    if (setsockopt(fd, SOL_UDP, UDP_GRO, &want_gro, sizeof want_gro) != 0) gro_ok = false;
  if (want_gro && gro_ok) on |= SQOBFS_UDP_RX_GRO;
  if (!(on & SQOBFS_UDP_RX_GRO)) {
    const int zero = 0;
    for (int fd : c->fds) (void)setsockopt(fd, SOL_UDP, UDP_GRO, &zero, sizeof zero);
    rx_fixed_offsets(c);
  }
  c->offload = on;
  return (int)on;
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
  // one mapped block: rx slots | tx slots | 7 u64 arrays | 4 u32 arrays |
  // salts (8 B each) | 2 u16 packet-number offset arrays
  const size_t sb = (size_t)slots * slot_bytes, a64 = 8ull * slots, a32 = 4ull * slots;
  const size_t bytes = 2 * sb + 7 * a64 + 4 * a32 + 8ull * slots + 4ull * slots;
  // page-locked and mapped: the GPU reads and writes it at the same address
  const int st = sq_host_alloc_mapped(ctx, bytes, &c->block);
  if (st != SQ_OK) {
    delete c;
    return st;
  }
  uint8_t *p = (uint8_t *)c->block;
  c->rx = p;                                 p += sb;
  c->tx = p;                                 p += sb;
  c->rx_in_off = (uint64_t *)p;              p += a64;
  c->rx_out_off = (uint64_t *)p;             p += a64;
  c->tx_in_off = (uint64_t *)p;              p += a64;
  c->tx_out_off = (uint64_t *)p;             p += a64;
  c->qpn_tx = (uint64_t *)p;                 p += a64;
  c->qpn_rx = (uint64_t *)p;                 p += a64;
  c->qpn_out = (uint64_t *)p;                p += a64;
  c->rx_len = (uint32_t *)p;                 p += a32;
  c->rx_out_len = (uint32_t *)p;             p += a32;
  c->tx_len = (uint32_t *)p;                 p += a32;
  c->tx_out_len = (uint32_t *)p;             p += a32;
  c->qsalt = p;                              p += 8ull * slots;
  c->qpno_tx = (uint16_t *)p;                p += 2ull * slots;
  c->qpno_rx = (uint16_t *)p;
  c->rx_fd.resize(slots);
  c->rx_from.resize(slots);
  c->tx_wire_len.resize(slots);
  rx_fixed_offsets(c);  // wire at the slot start, payload decoded in place behind it
  for (uint32_t i = 0; i < slots; i++) {
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
  int st = (c->offload & SQOBFS_UDP_RX_GRO)
               ? recv_gro(c, timeout_ms, &n)
               : sqobfs_udp_recv(c->fds.data(), (uint32_t)c->fds.size(), c->rx, c->slot_bytes,
                                 0, c->slots, timeout_ms, c->rx_len, c->rx_fd.data(),
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
  // fixed slots (multiples of 16 bytes): outputs own their blocks; GRO
  // buffers pack datagrams back to back, so not there
  if (!(c->offload & SQOBFS_UDP_RX_GRO)) b.flags = SQOBFS_FLAG_OUT_BLOCKS;
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
  b.flags = SQOBFS_FLAG_DEVICE_SALT | SQOBFS_FLAG_OUT_BLOCKS;  // slots of 16-byte multiples
  b.in = c->tx;
  b.in_off = c->tx_in_off;
  b.in_len = c->tx_len;
  b.out = c->tx;
  b.out_off = c->tx_out_off;
  b.out_len = c->tx_out_len;
  const int st = launch_sync(c, SQOBFS_OBFUSCATE, b);
  if (st != SQ_OK) return st;
  if (c->offload & SQOBFS_UDP_TX_GSO) {
    const int g = sqobfs_udp_send_gso(c->fds[fd_index], c->tx, c->tx_out_off,
                                      c->tx_wire_len.data(), to, n, sent);
    // no UDP GSO on this socket / route: fall back to one datagram per message
    if (g == SQ_OK || *sent > 0 || (g != -EIO && g != -EINVAL && g != -ENOPROTOOPT &&
                                    g != -EOPNOTSUPP))
      return g;
    c->offload &= ~SQOBFS_UDP_TX_GSO;
  }
  return sqobfs_udp_send(c->fds[fd_index], c->tx, c->tx_out_off, c->tx_wire_len.data(), to, n,
                         sent);
}

// ---- QUIC over the endpoint: the fused seal / open + Salamander kernels
// (sqobfs_quic_seal_salamander, sqobfs_quic_open_salamander) on the mapped
// slots, so one launch per batch does QUIC protection and obfuscation.

int sqobfs_udp_conn_write_quic(sqobfs_udp_conn *c, const sqobfs_quic_keyring *qkr,
                               uint32_t fd_index, uint32_t n, const uint32_t *len,
                               uint16_t pn_offset, const uint64_t *pn, const sqobfs_addr *to,
                               uint32_t *sent) {
  if (sent) *sent = 0;
  if (!c || !qkr || !sent || fd_index >= c->fds.size() || n > c->slots ||
      sqobfs_keyring_kind(c->kr) != SQOBFS_SALAMANDER)
    return SQ_EINVAL;
  if (n == 0) return SQ_OK;
  if (!len || !pn || !to) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(c->tx_mu);
  for (uint32_t i = 0; i < n; i++) {
    if (len[i] + 16 + c->S > c->slot_bytes) return SQ_EINVAL;
    c->tx_len[i] = len[i];
    c->qpn_tx[i] = pn[i];
    c->qpno_tx[i] = pn_offset;
  }
  // salts: 8 random bytes per datagram (salamander.go:60 buf.WriteRandom)
  for (size_t got = 0, want = 8ull * n; got < want;) {
    const ssize_t r = getrandom(c->qsalt + got, want - got, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    got += (size_t)r;
  }
  sqobfs_quic_batch b;
  memset(&b, 0, sizeof b);
  b.n = n;
  b.in = c->tx;
  b.in_off = c->tx_in_off;    // packet at slot + 8 ...
  b.in_len = c->tx_len;
  b.out = c->tx;
  b.out_off = c->tx_out_off;  // ... wire from the slot start (the in-place form)
  b.out_len = c->tx_out_len;
  b.pn_offset = c->qpno_tx;
  b.pn = c->qpn_tx;
  void *s = sqobfs_stream(c->ctx);
  int st = sqobfs_quic_seal_salamander(c->ctx, qkr, c->kr, &b, c->qsalt, s);
  if (st == SQ_OK) st = sq_ctx_stream_wait(c->ctx, s, kLaunchSpinUs);
  if (st != SQ_OK) return st;
  // *sent stays a prefix count (as for conn_write): the datagrams before the
  // first packet the kernel rejected (tx_out_len = SQOBFS_QUIC_E*) are sent,
  // and the call then fails with SQ_EINVAL, so packet *sent is the bad one
  uint32_t m = 0;
  while (m < n && c->tx_out_len[m] == len[m] + 16 + c->S) m++;
  for (uint32_t i = 0; i < m; i++) c->tx_wire_len[i] = c->tx_out_len[i];
  int g = SQ_OK;
  if (m && (c->offload & SQOBFS_UDP_TX_GSO)) {
    g = sqobfs_udp_send_gso(c->fds[fd_index], c->tx, c->tx_out_off, c->tx_wire_len.data(), to, m,
                            sent);
    if (!(g == SQ_OK || *sent > 0 || (g != -EIO && g != -EINVAL && g != -ENOPROTOOPT &&
                                      g != -EOPNOTSUPP)))
      c->offload &= ~SQOBFS_UDP_TX_GSO;
    else if (g != SQ_OK)
      return g;
  }
  if (m && !(c->offload & SQOBFS_UDP_TX_GSO)) {
    g = sqobfs_udp_send(c->fds[fd_index], c->tx, c->tx_out_off, c->tx_wire_len.data(), to, m,
                        sent);
    if (g != SQ_OK) return g;
  }
  return m < n ? SQ_EINVAL : SQ_OK;
}

int sqobfs_udp_conn_read_quic(sqobfs_udp_conn *c, const sqobfs_quic_keyring *qkr,
                              uint16_t pn_offset, uint64_t largest_pn, int timeout_ms,
                              sqobfs_udp_view *out, const uint64_t **pn_out) {
  if (!c || !qkr || !out || sqobfs_keyring_kind(c->kr) != SQOBFS_SALAMANDER) return SQ_EINVAL;
  std::lock_guard<std::mutex> lk(c->rx_mu);
  memset(out, 0, sizeof *out);
  if (pn_out) *pn_out = nullptr;
  uint32_t n = 0;
  int st = (c->offload & SQOBFS_UDP_RX_GRO)
               ? recv_gro(c, timeout_ms, &n)
               : sqobfs_udp_recv(c->fds.data(), (uint32_t)c->fds.size(), c->rx, c->slot_bytes,
                                 0, c->slots, timeout_ms, c->rx_len, c->rx_fd.data(),
                                 c->rx_from.data(), &n);
  if (st != SQ_OK || n == 0) return st;
  for (uint32_t i = 0; i < n; i++) {
    c->qpno_rx[i] = pn_offset;
    c->qpn_rx[i] = largest_pn;
  }
  sqobfs_quic_batch b;
  memset(&b, 0, sizeof b);
  b.n = n;
  b.in = c->rx;
  b.in_off = c->rx_in_off;
  b.in_len = c->rx_len;
  b.out = c->rx;
  b.out_off = c->rx_in_off;  // in place: the plaintext packet from the datagram start
  b.out_len = c->rx_out_len;
  b.pn_offset = c->qpno_rx;
  b.pn = c->qpn_rx;
  b.pn_out = c->qpn_out;
  void *s = sqobfs_stream(c->ctx);
  st = sqobfs_quic_open_salamander(c->ctx, qkr, c->kr, &b, s);
  if (st == SQ_OK) st = sq_ctx_stream_wait(c->ctx, s, kLaunchSpinUs);
  if (st != SQ_OK) return st;
  out->count = n;
  out->base = c->rx;
  out->off = c->rx_in_off;
  out->len = c->rx_out_len;
  out->fd_index = c->rx_fd.data();
  out->from = c->rx_from.data();
  if (pn_out) *pn_out = c->qpn_out;
  return SQ_OK;
}

}  // extern "C"
