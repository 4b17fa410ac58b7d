// Tests of the C++ PacketConn mirror (sing-quic_amd/host/) against the CPU
// oracle, over an in-memory fake socket (the reference has no tests; the
// fake follows HopPacketConn's datagram queue, hysteria/hop.go:139-161).
// Built and run by tests/test_gpu_host_mirror.py on the GPU box.
#include <stdio.h>
#include <string.h>

#include <deque>
#include <mutex>
#include <random>

#include "oracle.h"
#include "packet_conn.h"

using namespace sq;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      failures++;                                                       \
    }                                                                   \
  } while (0)

constexpr Error kErrEmpty = 1001;  // fake socket: nothing to read
constexpr Error kErrWrite = 1002;  // fake socket: injected write error

// In-memory datagram socket.
class FakeConn : public PacketConn {
 public:
  std::deque<std::vector<uint8_t>> q;
  std::mutex mu;
  bool fail_writes = false;
  Error ReadFrom(uint8_t *p, size_t cap, size_t *n, Addr *addr) override {
    std::lock_guard<std::mutex> lk(mu);
    *n = 0;
    if (q.empty()) return kErrEmpty;
    auto d = q.front();
    q.pop_front();
    *n = d.size() < cap ? d.size() : cap;
    memcpy(p, d.data(), *n);
    if (addr) *addr = Addr{"udp", "127.0.0.1:443"};
    return 0;
  }
  Error WriteTo(uint8_t *p, size_t len, const Addr &, size_t *n) override {
    std::lock_guard<std::mutex> lk(mu);
    *n = 0;
    if (fail_writes) return kErrWrite;
    q.emplace_back(p, p + len);
    *n = len;
    return 0;
  }
};

// Fake socket that also takes iovec-style writes (one datagram).
class FakeVecConn : public FakeConn, public VectorisedPacketWriter {
 public:
  Error WriteVectorisedPacket(const std::vector<std::vector<uint8_t> *> &bufs,
                              const Addr &) override {
    std::lock_guard<std::mutex> lk(mu);
    std::vector<uint8_t> d;
    for (auto *b : bufs) d.insert(d.end(), b->begin(), b->end());
    q.push_back(d);
    return 0;
  }
};

static std::vector<uint8_t> rnd(std::mt19937 &g, size_t n) {
  std::vector<uint8_t> v(n);
  for (auto &x : v) x = (uint8_t)g();
  return v;
}

static void test_salamander(std::mt19937 &g) {
  const std::vector<uint8_t> psk = {'p', 'a', 's', 's', 'w', 'o', 'r', 'd'};
  auto sock = std::make_shared<FakeConn>();
  auto conn = NewSalamanderConn(sock, psk);
  CHECK(dynamic_cast<VectorisedSalamanderPacketConn *>(conn.get()) == nullptr);
  for (size_t len : {0, 1, 7, 8, 9, 31, 32, 33, 1200, 1350, 1452}) {
    auto p = rnd(g, len);
    auto keep = p;
    size_t n = 99;
    CHECK(conn->WriteTo(p.data(), len, Addr{}, &n) == 0);
    CHECK(n == len);    // salamander.go:69 returns len(p)
    CHECK(p == keep);   // plain WriteTo leaves p untouched
    auto wire = sock->q.back();
    CHECK(wire.size() == len + 8);
    std::vector<uint8_t> want(len + 8);
    or_salamander_write(psk.data(), psk.size(), wire.data(), p.data(), len, want.data());
    CHECK(wire == want);
    // ReadFrom decodes in place (left shift by 8)
    std::vector<uint8_t> buf(2048, 0xEE);
    Addr a;
    CHECK(conn->ReadFrom(buf.data(), buf.size(), &n, &a) == 0);
    // an empty payload is an 8-byte datagram, which ReadFrom returns raw
    // (salamander.go:47-49): n = 8, the salt left in p
    CHECK(n == (len == 0 ? 8 : len));
    CHECK(memcmp(buf.data(), len == 0 ? wire.data() : p.data(), len == 0 ? 8 : len) == 0);
    CHECK(a.address == "127.0.0.1:443");
  }
  // salamander.go:47-49: n <= 8 is returned untouched
  for (size_t len = 0; len <= 8; len++) {
    auto d = rnd(g, len);
    sock->q.push_back(d);
    std::vector<uint8_t> buf(64, 0xCD);
    size_t n = 0;
    CHECK(conn->ReadFrom(buf.data(), buf.size(), &n, nullptr) == 0);
    CHECK(n == len);
    CHECK(memcmp(buf.data(), d.data(), len) == 0);
  }
  // errors of the inner socket are returned verbatim
  size_t n = 7;
  std::vector<uint8_t> buf(64);
  CHECK(conn->ReadFrom(buf.data(), buf.size(), &n, nullptr) == kErrEmpty);
  sock->fail_writes = true;
  CHECK(conn->WriteTo(buf.data(), 10, Addr{}, &n) == kErrWrite);
  CHECK(n == 0);
  sock->fail_writes = false;
}

static void test_salamander_vectorised(std::mt19937 &g) {
  const std::vector<uint8_t> psk = rnd(g, 40);
  auto sock = std::make_shared<FakeVecConn>();
  auto conn = NewSalamanderConn(sock, psk);
  auto *vc = dynamic_cast<VectorisedSalamanderPacketConn *>(conn.get());
  CHECK(vc != nullptr);
  // WriteTo mutates the caller's buffer (salamander.go:85-87)
  auto p = rnd(g, 500);
  auto orig = p;
  size_t n = 0;
  CHECK(conn->WriteTo(p.data(), p.size(), Addr{}, &n) == 0);
  CHECK(n == 500);
  auto wire = sock->q.back();
  std::vector<uint8_t> want(508);
  or_salamander_write(psk.data(), psk.size(), wire.data(), orig.data(), 500, want.data());
  CHECK(wire == want);
  CHECK(memcmp(p.data(), wire.data() + 8, 500) == 0);
  // multi-buffer: one continuous keystream (the evident intent of :95-109)
  auto b1 = rnd(g, 33), b2 = rnd(g, 70), b3 = rnd(g, 5);
  std::vector<uint8_t> cat = b1;
  cat.insert(cat.end(), b2.begin(), b2.end());
  cat.insert(cat.end(), b3.begin(), b3.end());
  CHECK(vc->WriteVectorisedPacket({&b1, &b2, &b3}, Addr{}) == 0);
  wire = sock->q.back();
  CHECK(wire.size() == 8 + cat.size());
  want.assign(8 + cat.size(), 0);
  or_salamander_write(psk.data(), psk.size(), wire.data(), cat.data(), cat.size(), want.data());
  CHECK(wire == want);
  // single first buffer: identical to the reference's literal loop
  auto only = rnd(g, 64);
  auto only_orig = only;
  CHECK(vc->WriteVectorisedPacket({&only}, Addr{}) == 0);
  wire = sock->q.back();
  std::vector<uint8_t> lit = only_orig;
  uint8_t *bp = lit.data();
  size_t bl = lit.size();
  CHECK(or_salamander_write_vectorised(psk.data(), psk.size(), wire.data(), &bp, &bl, 1) == 0);
  CHECK(lit == only);
}

static void test_xplus(std::mt19937 &g) {
  const std::vector<uint8_t> psk = rnd(g, 26);
  auto sock = std::make_shared<FakeConn>();
  auto conn = NewXPlusPacketConn(sock, psk);
  for (size_t len : {0, 1, 15, 16, 17, 1200}) {
    auto p = rnd(g, len);
    size_t n = 0;
    CHECK(conn->WriteTo(p.data(), len, Addr{}, &n) == 0);
    CHECK(n == len + 16);  // xplus.go:74 returns the inner n
    auto wire = sock->q.back();
    std::vector<uint8_t> want(len + 16);
    or_xplus_write(psk.data(), psk.size(), wire.data(), p.data(), len, want.data());
    CHECK(wire == want);
    // ReadFrom XORs the whole read buffer tail (xplus.go:55): compare the
    // entire buffer with the oracle
    std::vector<uint8_t> buf(len + 16 + 37);
    for (auto &x : buf) x = (uint8_t)g();
    std::vector<uint8_t> ref = buf;
    memcpy(ref.data(), wire.data(), wire.size());
    const long r = or_xplus_read(psk.data(), psk.size(), ref.data(), wire.size(), ref.size());
    CHECK(conn->ReadFrom(buf.data(), buf.size(), &n, nullptr) == 0);
    CHECK((long)n == r);
    CHECK(memcmp(buf.data(), ref.data(), ref.size() - 16) == 0);
  }
  // xplus.go:50-52: n < 16 -> 0
  sock->q.push_back(rnd(g, 15));
  std::vector<uint8_t> buf(64);
  size_t n = 9;
  CHECK(conn->ReadFrom(buf.data(), buf.size(), &n, nullptr) == 0);
  CHECK(n == 0);
}

static void test_xplus_vectorised(std::mt19937 &g) {
  const std::vector<uint8_t> psk = rnd(g, 50);  // two SHA-256 blocks
  auto sock = std::make_shared<FakeVecConn>();
  auto conn = NewXPlusPacketConn(sock, psk);
  auto *vc = dynamic_cast<VectorisedXPlusConn *>(conn.get());
  CHECK(vc != nullptr);
  auto b1 = rnd(g, 3), b2 = rnd(g, 90);
  auto o1 = b1, o2 = b2;
  CHECK(vc->WriteVectorisedPacket({&b1, &b2}, Addr{}) == 0);
  auto wire = sock->q.back();
  uint8_t *bp[2] = {o1.data(), o2.data()};
  size_t bl[2] = {o1.size(), o2.size()};
  or_xplus_write_vectorised(psk.data(), psk.size(), wire.data(), bp, bl, 2);
  CHECK(o1 == b1 && o2 == b2);
  CHECK(memcmp(wire.data() + 16, b1.data(), 3) == 0);
}

static void test_batches(std::mt19937 &g) {
  for (int kind = 0; kind < 2; kind++) {
    const std::vector<uint8_t> psk = rnd(g, 26);
    auto sock = std::make_shared<FakeConn>();
    std::shared_ptr<PacketConn> conn = kind == 0 ? NewSalamanderConn(sock, psk)
                                                 : NewXPlusPacketConn(sock, psk);
    std::vector<Datagram> in(1500);
    for (auto &d : in) d.data = rnd(g, g() % 1500);
    const Error e = kind == 0 ? static_cast<SalamanderPacketConn *>(conn.get())->WriteBatch(in)
                              : static_cast<XPlusPacketConn *>(conn.get())->WriteBatch(in);
    CHECK(e == 0);
    CHECK(sock->q.size() == in.size());
    std::vector<Datagram> out;
    const Error r = kind == 0
                        ? static_cast<SalamanderPacketConn *>(conn.get())->ReadBatch(out, 2000)
                        : static_cast<XPlusPacketConn *>(conn.get())->ReadBatch(out, 2000);
    CHECK(r == 0);
    CHECK(out.size() == in.size());
    for (size_t i = 0; i < in.size() && i < out.size(); i++) {
      if (kind == 0 && in[i].data.empty()) {
        CHECK(out[i].data.size() == 8);  // 8-byte datagram: returned raw (salt)
      } else {
        CHECK(out[i].data == in[i].data);
      }
    }
  }
}

int main() {
  std::mt19937 g(1234);
  test_salamander(g);
  test_salamander_vectorised(g);
  test_xplus(g);
  test_xplus_vectorised(g);
  test_batches(g);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("test_packet_conn: ok\n");
  return 0;
}
