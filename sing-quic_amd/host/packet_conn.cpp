// packet_conn.cpp -- C++ mirror of the reference's obfuscating PacketConn
// decorators (see packet_conn.h).  Every transform goes through the C ABI --
// sqobfs_run_host (gfx950 kernels) for batches worth a launch, sqobfs_cpu_run
// (the library's CPU path) for single datagrams, small batches and when no
// GPU can be opened; this file only moves bytes between sockets and batches.
#include "packet_conn.h"

#include <string.h>
#include <sys/random.h>

#include <chrono>

namespace sq {

namespace {

constexpr uint32_t kBadLen = 0xFFFFFFFEu;

// salt buffers must be 4-byte aligned for the batch ABI
struct alignas(16) SaltBuf {
  uint8_t b[16];
};

int check_len(uint32_t out_len) {
  return (out_len == kBadLen || out_len == SQOBFS_BAD_PSK) ? SQ_EINVAL : SQ_OK;
}

// wire[0 .. S+len) = salt || p ^ key  (one packet)
int obfuscate_one(Obfuscator &ob, const uint8_t *p, size_t len, const uint8_t *salt,
                  uint8_t *wire) {
  uint64_t in_off = 0, out_off = 0;
  uint32_t in_len = (uint32_t)len, out_len = 0;
  sqobfs_batch b;
  memset(&b, 0, sizeof b);
  b.n = 1;
  b.in = p ? p : wire;
  b.in_off = &in_off;
  b.in_len = &in_len;
  b.out = wire;
  b.out_off = &out_off;
  b.out_len = &out_len;
  b.salt = salt;
  const int st = ob.run(SQOBFS_OBFUSCATE, b);
  return st != SQ_OK ? st : check_len(out_len);
}

// decode datagram p[0:n) (read buffer of `cap` bytes) into p[0 : ...) in
// place, as ReadFrom does; returns the out_len the kernel computed
int deobfuscate_one_inplace(Obfuscator &ob, uint8_t *p, size_t n, size_t cap, uint32_t *out_len) {
  uint64_t in_off = 0, out_off = 0;
  uint32_t in_len = (uint32_t)n, in_cap = (uint32_t)cap;
  sqobfs_batch b;
  memset(&b, 0, sizeof b);
  b.n = 1;
  b.in = p;  // the host-staged path copies input and output ranges
  b.in_off = &in_off;  // separately, so decoding over the read buffer is fine
  b.in_len = &in_len;
  b.out = p;
  b.out_off = &out_off;
  b.out_len = out_len;
  b.in_cap = ob.kind() == SQOBFS_XPLUS ? &in_cap : nullptr;
  const int st = ob.run(SQOBFS_DEOBFUSCATE, b);
  return st != SQ_OK ? st : check_len(*out_len);
}

// Read up to `max` datagrams, decode them with one launch.
Error read_batch(PacketConn &conn, Obfuscator &ob, std::vector<Datagram> &out, size_t max,
                 size_t buf_size) {
  out.clear();
  if (max == 0) return 0;
  std::vector<uint8_t> buf(max * buf_size);
  std::vector<uint64_t> in_off;
  std::vector<uint32_t> in_len;
  std::vector<Addr> addrs;
  Error err = 0;
  for (size_t i = 0; i < max; i++) {
    size_t n = 0;
    Addr a;
    err = conn.ReadFrom(buf.data() + i * buf_size, buf_size, &n, &a);
    if (err) break;
    in_off.push_back(i * buf_size);
    in_len.push_back((uint32_t)n);
    addrs.push_back(a);
  }
  const uint32_t cnt = (uint32_t)in_len.size();
  if (cnt == 0) return err;
  const size_t S = ob.salt_len();
  std::vector<uint64_t> out_off(cnt);
  uint64_t pos = 0;
  for (uint32_t i = 0; i < cnt; i++) {
    out_off[i] = pos;
    pos += in_len[i] <= S ? in_len[i] : in_len[i] - S;  // upper bound of each output
  }
  std::vector<uint8_t> dec(pos + 1);
  std::vector<uint32_t> out_len(cnt);
  sqobfs_batch b;
  memset(&b, 0, sizeof b);
  b.n = cnt;
  b.in = buf.data();
  b.in_off = in_off.data();
  b.in_len = in_len.data();
  b.out = dec.data();
  b.out_off = out_off.data();
  b.out_len = out_len.data();
  const int st = ob.run(SQOBFS_DEOBFUSCATE, b);
  if (st != SQ_OK) return st;
  out.resize(cnt);
  for (uint32_t i = 0; i < cnt; i++) {
    out[i].data.assign(dec.begin() + out_off[i], dec.begin() + out_off[i] + out_len[i]);
    out[i].addr = addrs[i];
  }
  return 0;
}

// Obfuscate all datagrams with one launch, then write them one by one.
template <typename SaltFn>
Error write_batch(PacketConn &conn, Obfuscator &ob, const std::vector<Datagram> &in,
                  SaltFn salt_fn) {
  const uint32_t cnt = (uint32_t)in.size();
  if (cnt == 0) return 0;
  const size_t S = ob.salt_len();
  std::vector<uint64_t> in_off(cnt), out_off(cnt);
  std::vector<uint32_t> in_len(cnt), out_len(cnt);
  uint64_t ip = 0, op = 0;
  for (uint32_t i = 0; i < cnt; i++) {
    in_off[i] = ip;
    in_len[i] = (uint32_t)in[i].data.size();
    ip += in[i].data.size();
    out_off[i] = op;
    op += S + in[i].data.size();
  }
  std::vector<uint8_t> payload(ip + 1), wire(op + 1);
  for (uint32_t i = 0; i < cnt; i++)
    if (in_len[i]) memcpy(payload.data() + in_off[i], in[i].data.data(), in_len[i]);
  std::vector<uint32_t> salts32((cnt * S + 3) / 4);
  uint8_t *salts = reinterpret_cast<uint8_t *>(salts32.data());
  for (uint32_t i = 0; i < cnt; i++) salt_fn(salts + i * S);
  sqobfs_batch b;
  memset(&b, 0, sizeof b);
  b.n = cnt;
  b.in = payload.data();
  b.in_off = in_off.data();
  b.in_len = in_len.data();
  b.out = wire.data();
  b.out_off = out_off.data();
  b.out_len = out_len.data();
  b.salt = salts;
  const int st = ob.run(SQOBFS_OBFUSCATE, b);
  if (st != SQ_OK) return st;
  for (uint32_t i = 0; i < cnt; i++) {
    size_t n = 0;
    const Error err = conn.WriteTo(wire.data() + out_off[i], out_len[i], in[i].addr, &n);
    if (err) return err;
  }
  return 0;
}

std::shared_ptr<Obfuscator> make_ob(int kind, const std::vector<uint8_t> &psk, int device) {
  return std::make_shared<Obfuscator>(kind, psk.data(), psk.size(), device);
}

void crypto_random(uint8_t *b, size_t n) {
  // sing's buf.WriteRandom (salamander.go:60,83,98) draws from crypto/rand
  size_t got = 0;
  while (got < n) {
    const ssize_t r = getrandom(b + got, n - got, 0);
    if (r > 0) got += (size_t)r;
  }
}

}  // namespace

// ---------------------------------------------------------------- Obfuscator

Obfuscator::Obfuscator(int kind, const uint8_t *psk, size_t psk_len, int device) : kind_(kind) {
  // no GPU: a host keyring, every batch on the CPU path (the reference's
  // constructors cannot fail, salamander.go:24-40, xplus.go:19-37)
  if (sqobfs_open(device, &ctx_) != SQ_OK) ctx_ = nullptr;
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)psk_len;
  static const uint8_t empty = 0;
  status_ = sqobfs_keyring_create(ctx_, kind, 1, psk_len ? psk : &empty, &off, &len, &kr_);
}

Obfuscator::~Obfuscator() {
  if (kr_) sqobfs_keyring_destroy(kr_);
  if (ctx_) sqobfs_close(ctx_);
}

int Obfuscator::run(int dir, const sqobfs_batch &b) {
  if (status_ != SQ_OK) return status_;
  // a batch worth a launch goes to the GPU (cost as the packet conn engine
  // counts it: payload bytes + 1 KiB per datagram): above the measured
  // break-even -- the recent staged round trip (sqobfs_run_host) times the
  // recent CPU-path rate, as the engine's route_bytes; a single datagram
  // costs ~1 us on the CPU path against a ~50 us staged round trip
  uint64_t cost = 0;
  for (uint32_t i = 0; i < b.n; i++) cost += b.in_len[i] + 1024u;
  const uint64_t g = gpu_us_.load(std::memory_order_relaxed);
  const uint64_t c = std::max<uint32_t>(1u, cpu_ns_kib_.load(std::memory_order_relaxed));
  const uint64_t route = std::min<uint64_t>(16u << 20, std::max<uint64_t>(16u << 10, g * 1024000u / c));
  const auto t0 = std::chrono::steady_clock::now();
  auto ewma = [&](std::atomic<uint32_t> &a, uint64_t v) {
    const uint32_t o = a.load(std::memory_order_relaxed);
    a.store((uint32_t)((7ull * o + std::min<uint64_t>(v, 1u << 30)) / 8), std::memory_order_relaxed);
  };
  if (!ctx_ || gpu_failed_.load(std::memory_order_relaxed) || cost <= route) {
    const int st = sqobfs_cpu_run(kr_, dir, &b);
    if (cost >= (8u << 10))  // (smaller batches: timer noise)
      ewma(cpu_ns_kib_, (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now() - t0).count() * 1024u / cost);
    return st;
  }
  const int st = sqobfs_run_host(ctx_, kr_, dir, &b);
  if (st == SQ_EDEVICE || st == SQ_ENODEV)
    gpu_failed_.store(true, std::memory_order_relaxed);  // later batches: the CPU
  if (st == SQ_OK)
    ewma(gpu_us_, (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                      std::chrono::steady_clock::now() - t0).count());
  return st;
}

// ---------------------------------------------------------------- Salamander

SalamanderPacketConn::SalamanderPacketConn(std::shared_ptr<PacketConn> conn,
                                           std::vector<uint8_t> password, int device)
    : conn_(std::move(conn)), password_(std::move(password)) {
  ob_ = make_ob(SQOBFS_SALAMANDER, password_, device);
}

void SalamanderPacketConn::random_salt(uint8_t *salt) { crypto_random(salt, 8); }

Error SalamanderPacketConn::ReadFrom(uint8_t *p, size_t cap, size_t *n, Addr *addr) {
  *n = 0;
  size_t got = 0;
  const Error err = conn_->ReadFrom(p, cap, &got, addr);  // salamander.go:43
  *n = got;
  if (err) return err;
  if (got <= 8) return 0;  // :47-49
  uint32_t out_len = 0;
  const int st = deobfuscate_one_inplace(*ob_, p, got, got, &out_len);  // :50-53
  if (st != SQ_OK) return st;
  *n = out_len;  // :54, n - 8
  return 0;
}

Error SalamanderPacketConn::WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) {
  *n = 0;
  SaltBuf salt;
  random_salt(salt.b);  // :60
  std::vector<uint8_t> wire(len + 8);
  const int st = obfuscate_one(*ob_, p, len, salt.b, wire.data());  // :61-64
  if (st != SQ_OK) return st;
  size_t w = 0;
  const Error err = conn_->WriteTo(wire.data(), wire.size(), addr, &w);  // :65
  if (err) return err;
  *n = len;  // :69
  return 0;
}

Error SalamanderPacketConn::ReadBatch(std::vector<Datagram> &out, size_t max, size_t buf_size) {
  return read_batch(*conn_, *ob_, out, max, buf_size);
}

Error SalamanderPacketConn::WriteBatch(const std::vector<Datagram> &in) {
  return write_batch(*conn_, *ob_, in, [](uint8_t *s) { crypto_random(s, 8); });
}

VectorisedSalamanderPacketConn::VectorisedSalamanderPacketConn(
    std::shared_ptr<PacketConn> conn, std::shared_ptr<VectorisedPacketWriter> writer,
    std::vector<uint8_t> password, int device)
    : SalamanderPacketConn(std::move(conn), std::move(password), device),
      writer_(std::move(writer)) {}

Error VectorisedSalamanderPacketConn::WriteTo(uint8_t *p, size_t len, const Addr &addr,
                                              size_t *n) {
  *n = 0;
  SaltBuf salt;
  random_salt(salt.b);  // salamander.go:82-83
  std::vector<uint8_t> wire(len + 8);
  const int st = obfuscate_one(*ob_, p, len, salt.b, wire.data());  // :84
  if (st != SQ_OK) return st;
  if (len) memcpy(p, wire.data() + 8, len);  // :85-87, in place on the caller's p
  std::vector<uint8_t> header(salt.b, salt.b + 8), body(p, p + len);
  const Error err = writer_->WriteVectorisedPacket({&header, &body}, addr);  // :88
  if (err) return err;
  *n = len;  // :92
  return 0;
}

Error VectorisedSalamanderPacketConn::WriteVectorisedPacket(
    const std::vector<std::vector<uint8_t> *> &buffers, const Addr &dst) {
  SaltBuf salt;
  random_salt(salt.b);  // :96-98
  std::vector<uint8_t> cat;
  for (auto *b : buffers) cat.insert(cat.end(), b->begin(), b->end());
  std::vector<uint8_t> wire(cat.size() + 8);
  const int st = obfuscate_one(*ob_, cat.data(), cat.size(), salt.b, wire.data());  // :99
  if (st != SQ_OK) return st;
  size_t pos = 8;  // one continuous keystream (see header: line 104)
  for (auto *b : buffers) {
    if (!b->empty()) memcpy(b->data(), wire.data() + pos, b->size());
    pos += b->size();
  }
  std::vector<uint8_t> header(salt.b, salt.b + 8);
  std::vector<std::vector<uint8_t> *> all{&header};
  all.insert(all.end(), buffers.begin(), buffers.end());
  return writer_->WriteVectorisedPacket(all, dst);  // :108
}

std::shared_ptr<PacketConn> NewSalamanderConn(std::shared_ptr<PacketConn> conn,
                                              std::vector<uint8_t> password, int device) {
  // salamander.go:25: bufio.CreateVectorisedPacketWriter(conn)
  if (auto w = std::dynamic_pointer_cast<VectorisedPacketWriter>(conn))
    return std::make_shared<VectorisedSalamanderPacketConn>(conn, w, std::move(password), device);
  return std::make_shared<SalamanderPacketConn>(conn, std::move(password), device);
}

// ---------------------------------------------------------------- XPlus

XPlusPacketConn::XPlusPacketConn(std::shared_ptr<PacketConn> conn, std::vector<uint8_t> key,
                                 int device)
    : conn_(std::move(conn)), key_(std::move(key)) {
  ob_ = make_ob(SQOBFS_XPLUS, key_, device);
  // xplus.go:26,34: rand.New(rand.NewSource(time.Now().UnixNano()))
  rand_.seed((uint64_t)std::chrono::system_clock::now().time_since_epoch().count());
}

void XPlusPacketConn::random_salt(uint8_t *salt) {
  std::lock_guard<std::mutex> lk(rand_access_);  // xplus.go:67-69
  for (int i = 0; i < 16; i += 8) {
    const uint64_t r = rand_();
    memcpy(salt + i, &r, 8);
  }
}

Error XPlusPacketConn::ReadFrom(uint8_t *p, size_t cap, size_t *n, Addr *addr) {
  *n = 0;
  size_t got = 0;
  const Error err = conn_->ReadFrom(p, cap, &got, addr);  // xplus.go:47
  if (err) {
    *n = got;
    return err;
  }
  if (got < 16) return 0;  // :50-52, n = 0, no error
  uint32_t out_len = 0;
  const int st = deobfuscate_one_inplace(*ob_, p, got, cap, &out_len);  // :54-57 over p[16:cap)
  if (st != SQ_OK) return st;
  *n = out_len;  // :58, n - 16
  return 0;
}

Error XPlusPacketConn::WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) {
  *n = 0;
  SaltBuf salt;
  random_salt(salt.b);  // :66-69
  std::vector<uint8_t> wire(len + 16);
  const int st = obfuscate_one(*ob_, p, len, salt.b, wire.data());  // :70-73
  if (st != SQ_OK) return st;
  return conn_->WriteTo(wire.data(), wire.size(), addr, n);  // :74, inner n
}

Error XPlusPacketConn::ReadBatch(std::vector<Datagram> &out, size_t max, size_t buf_size) {
  return read_batch(*conn_, *ob_, out, max, buf_size);
}

Error XPlusPacketConn::WriteBatch(const std::vector<Datagram> &in) {
  return write_batch(*conn_, *ob_, in, [this](uint8_t *s) { random_salt(s); });
}

VectorisedXPlusConn::VectorisedXPlusConn(std::shared_ptr<PacketConn> conn,
                                         std::shared_ptr<VectorisedPacketWriter> writer,
                                         std::vector<uint8_t> key, int device)
    : XPlusPacketConn(std::move(conn), std::move(key), device), writer_(std::move(writer)) {}

Error VectorisedXPlusConn::WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) {
  *n = 0;
  SaltBuf salt;
  random_salt(salt.b);  // xplus.go:87-92
  std::vector<uint8_t> wire(len + 16);
  const int st = obfuscate_one(*ob_, p, len, salt.b, wire.data());  // :93
  if (st != SQ_OK) return st;
  if (len) memcpy(p, wire.data() + 16, len);  // :94-96, in place
  std::vector<uint8_t> header(salt.b, salt.b + 16), body(p, p + len);
  const Error err = writer_->WriteVectorisedPacket({&header, &body}, addr);  // :97
  if (err) return err;
  // sing's bufio.WriteVectorisedPacket (not in the tree) reports the bytes
  // of the datagram; like XPlusPacketConn.WriteTo that is len(p) + 16
  *n = len + 16;
  return 0;
}

Error VectorisedXPlusConn::WriteVectorisedPacket(const std::vector<std::vector<uint8_t> *> &buffers,
                                                 const Addr &dst) {
  SaltBuf salt;
  random_salt(salt.b);  // :101-106
  std::vector<uint8_t> cat;
  for (auto *b : buffers) cat.insert(cat.end(), b->begin(), b->end());
  std::vector<uint8_t> wire(cat.size() + 16);
  const int st = obfuscate_one(*ob_, cat.data(), cat.size(), salt.b, wire.data());  // :107
  if (st != SQ_OK) return st;
  size_t pos = 16;  // running keystream index over all buffers (:108-115)
  for (auto *b : buffers) {
    if (!b->empty()) memcpy(b->data(), wire.data() + pos, b->size());
    pos += b->size();
  }
  std::vector<uint8_t> header(salt.b, salt.b + 16);
  std::vector<std::vector<uint8_t> *> all{&header};
  all.insert(all.end(), buffers.begin(), buffers.end());
  return writer_->WriteVectorisedPacket(all, dst);  // :116-117
}

std::shared_ptr<PacketConn> NewXPlusPacketConn(std::shared_ptr<PacketConn> conn,
                                               std::vector<uint8_t> key, int device) {
  if (auto w = std::dynamic_pointer_cast<VectorisedPacketWriter>(conn))  // xplus.go:20
    return std::make_shared<VectorisedXPlusConn>(conn, w, std::move(key), device);
  return std::make_shared<XPlusPacketConn>(conn, std::move(key), device);
}

}  // namespace sq
