// packet_conn.h -- C++ mirror of sing-quic's obfuscating PacketConn
// decorators, layered on the C ABI of include/sqobfs.h.
//
// The reference is Go (no Go toolchain exists in this image), so this is the
// host side the task calls for when the reference's language is absent: the
// same names, argument meaning and error behaviour as
//   hysteria2/salamander.go  NewSalamanderConn / SalamanderPacketConn /
//                            VectorisedSalamanderPacketConn
//   hysteria/xplus.go        NewXPlusPacketConn / XPlusPacketConn /
//                            VectorisedXPlusConn
// with every byte transform executed through the C ABI: batches worth a
// launch by the gfx950 kernels, single datagrams and small batches by the
// library's CPU path (sqobfs_cpu_run), which also serves every call when no
// GPU can be opened -- so, like the reference's, the constructors never fail
// for want of a device.  The batch methods (ReadBatch / WriteBatch) are the
// intended use: one GPU launch per batch of datagrams (recvmmsg/sendmmsg
// style); the per-packet methods keep call sites written against the
// reference compiling unchanged.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "sqobfs.h"

namespace sq {

// net.Addr stand-in: the decorators only pass it through.
struct Addr {
  std::string network;
  std::string address;
};

// Errors: 0 = nil.  Inner-socket errors are passed through verbatim
// (salamander.go:43-46,65-68; xplus.go:47-49,74); GPU failures surface as
// the negative sqobfs status codes.
using Error = int;

// net.PacketConn (the subset the decorators use).
class PacketConn {
 public:
  virtual ~PacketConn() = default;
  // reads one datagram into p[0:cap); n = bytes read
  virtual Error ReadFrom(uint8_t *p, size_t cap, size_t *n, Addr *addr) = 0;
  // writes p[0:len) as one datagram; n = bytes written.  p is mutable as
  // in Go: the vectorised decorators XOR the caller's buffer in place
  // (salamander.go:85-87, xplus.go:94-96).
  virtual Error WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) = 0;
  virtual Error Close() { return 0; }
};

// N.VectorisedPacketWriter: one datagram from several buffers.
class VectorisedPacketWriter {
 public:
  virtual ~VectorisedPacketWriter() = default;
  virtual Error WriteVectorisedPacket(const std::vector<std::vector<uint8_t> *> &buffers,
                                      const Addr &dst) = 0;
};

// A datagram in a batch call.
struct Datagram {
  std::vector<uint8_t> data;  // ReadBatch: filled with the decoded payload
  Addr addr;
};

// GPU state shared by the decorators: one context + keyring.
class Obfuscator {
 public:
  Obfuscator(int kind, const uint8_t *psk, size_t psk_len, int device = 0);
  ~Obfuscator();
  Obfuscator(const Obfuscator &) = delete;
  Obfuscator &operator=(const Obfuscator &) = delete;

  int kind() const { return kind_; }
  size_t salt_len() const { return kind_ == SQOBFS_SALAMANDER ? 8 : 16; }
  // host batch: sqobfs_run_host when it is worth a launch, else (and with
  // no GPU, or after a failed launch) sqobfs_cpu_run; returns sqobfs status
  int run(int dir, const sqobfs_batch &b);
  int status() const { return status_; }
  bool has_gpu() const { return ctx_ != nullptr && !gpu_failed_.load(std::memory_order_relaxed); }

 private:
  int kind_;
  int status_ = SQ_OK;
  std::atomic<bool> gpu_failed_{false};  // (run() from concurrent ReadFrom / WriteTo)
  // routing (run): recent staged round trip (us) and CPU-path ns per KiB of
  // cost, EWMAs; ~120 KiB break-even before either is measured
  std::atomic<uint32_t> gpu_us_{60};
  std::atomic<uint32_t> cpu_ns_kib_{500};
  sqobfs_ctx *ctx_ = nullptr;
  sqobfs_keyring *kr_ = nullptr;
};

// hysteria2/salamander.go:19-22
class SalamanderPacketConn : public PacketConn {
 public:
  SalamanderPacketConn(std::shared_ptr<PacketConn> conn, std::vector<uint8_t> password,
                       int device = 0);
  // salamander.go:42-55: decodes in place; n <= 8 returned untouched
  Error ReadFrom(uint8_t *p, size_t cap, size_t *n, Addr *addr) override;
  // salamander.go:57-70: copies salt || p^key, returns len(p)
  Error WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) override;
  Error Close() override { return conn_->Close(); }
  // salamander.go:72-74
  PacketConn *Upstream() const { return conn_.get(); }

  // batch forms: one GPU launch for the whole batch
  Error ReadBatch(std::vector<Datagram> &out, size_t max, size_t buf_size = 2048);
  Error WriteBatch(const std::vector<Datagram> &in);

 protected:
  void random_salt(uint8_t *salt);
  std::shared_ptr<PacketConn> conn_;
  std::vector<uint8_t> password_;
  std::shared_ptr<Obfuscator> ob_;
};

// hysteria2/salamander.go:76-109
class VectorisedSalamanderPacketConn : public SalamanderPacketConn,
                                       public VectorisedPacketWriter {
 public:
  VectorisedSalamanderPacketConn(std::shared_ptr<PacketConn> conn,
                                 std::shared_ptr<VectorisedPacketWriter> writer,
                                 std::vector<uint8_t> password, int device = 0);
  // salamander.go:81-93: XORs p IN PLACE (caller's buffer) and writes
  // [salt, p] through the vectorised writer; returns len(p)
  Error WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) override;
  // salamander.go:95-109.  The reference's line 104 mis-indexes every buffer
  // after a non-empty first one (Go panics); this implements the evident
  // intent -- one continuous keystream over the concatenation, as XPlus
  // does (xplus.go:108-115) -- and documents the divergence.
  Error WriteVectorisedPacket(const std::vector<std::vector<uint8_t> *> &buffers,
                              const Addr &dst) override;

 private:
  std::shared_ptr<VectorisedPacketWriter> writer_;
};

// hysteria/xplus.go:39-44
class XPlusPacketConn : public PacketConn {
 public:
  XPlusPacketConn(std::shared_ptr<PacketConn> conn, std::vector<uint8_t> key, int device = 0);
  // xplus.go:46-60: n < 16 -> 0; XORs the whole buffer tail p[16:cap)
  Error ReadFrom(uint8_t *p, size_t cap, size_t *n, Addr *addr) override;
  // xplus.go:62-75: returns the inner WriteTo's n (= len(p) + 16)
  Error WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) override;
  Error Close() override { return conn_->Close(); }
  PacketConn *Upstream() const { return conn_.get(); }  // xplus.go:77-79

  Error ReadBatch(std::vector<Datagram> &out, size_t max, size_t buf_size = 2048);
  Error WriteBatch(const std::vector<Datagram> &in);

 protected:
  void random_salt(uint8_t *salt);  // xplus.go:67-69, math/rand under a mutex
  std::shared_ptr<PacketConn> conn_;
  std::vector<uint8_t> key_;
  std::shared_ptr<Obfuscator> ob_;
  std::mutex rand_access_;
  std::mt19937_64 rand_;
};

// hysteria/xplus.go:81-118
class VectorisedXPlusConn : public XPlusPacketConn, public VectorisedPacketWriter {
 public:
  VectorisedXPlusConn(std::shared_ptr<PacketConn> conn,
                      std::shared_ptr<VectorisedPacketWriter> writer, std::vector<uint8_t> key,
                      int device = 0);
  // xplus.go:86-98: XORs p in place, writes [salt, p]
  Error WriteTo(uint8_t *p, size_t len, const Addr &addr, size_t *n) override;
  Error WriteVectorisedPacket(const std::vector<std::vector<uint8_t> *> &buffers,
                              const Addr &dst) override;  // xplus.go:100-118

 private:
  std::shared_ptr<VectorisedPacketWriter> writer_;
};

// salamander.go:17
constexpr const char *ObfsTypeSalamander = SQOBFS_OBFS_TYPE_SALAMANDER;

// Constructors with the reference's selection rule (salamander.go:24-40,
// xplus.go:19-37): the vectorised variant when the inner conn also
// implements VectorisedPacketWriter.
std::shared_ptr<PacketConn> NewSalamanderConn(std::shared_ptr<PacketConn> conn,
                                              std::vector<uint8_t> password, int device = 0);
std::shared_ptr<PacketConn> NewXPlusPacketConn(std::shared_ptr<PacketConn> conn,
                                               std::vector<uint8_t> key, int device = 0);

}  // namespace sq
