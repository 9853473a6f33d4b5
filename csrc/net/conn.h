// Byte-stream connections of the chat plane: raw TCP, the Noise XX secure
// channel (libp2p "/noise"), and multistream-select 1.0.0 negotiation.
//
// Every layer is a Conn, so an upgraded connection can run over a TCP socket or
// over a circuit-relay-v2 stream (relay.h) with identical code.
#pragma once
#include <atomic>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "crypto.h"
#include "util.h"

namespace p2p {

class Conn {
 public:
  virtual ~Conn() = default;
  // Blocking read of up to n bytes; returns 0 on EOF.  Throws NetError on error/timeout.
  virtual size_t read_some(uint8_t* buf, size_t n) = 0;
  virtual void write_all(const uint8_t* buf, size_t n) = 0;
  virtual void close_write() {}
  virtual void close() = 0;
  // Read deadline in ms from now (0 = none) for subsequent reads.
  virtual void set_read_timeout(int ms) { (void)ms; }
  virtual std::string remote_addr() const { return ""; }

  void write_all(const Bytes& b) { write_all(b.data(), b.size()); }
  void write_all(const std::string& s) { write_all((const uint8_t*)s.data(), s.size()); }
  void read_exact(uint8_t* buf, size_t n);
  Bytes read_exact(size_t n) {
    Bytes b(n);
    read_exact(b.data(), n);
    return b;
  }
  // Reads until EOF (bounded by max; throws if exceeded).
  Bytes read_all(size_t max);
};
using ConnPtr = std::shared_ptr<Conn>;

// Read-buffered view over a Conn, so that bytes pipelined after a negotiation
// message (lazy multistream) are not lost.  Itself a Conn.
class BufConn : public Conn {
 public:
  explicit BufConn(ConnPtr c) : c_(std::move(c)) {}
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override;
  void write_all(const uint8_t* buf, size_t n) override { c_->write_all(buf, n); }
  void close_write() override { c_->close_write(); }
  void close() override { c_->close(); }
  void set_read_timeout(int ms) override { c_->set_read_timeout(ms); }
  std::string remote_addr() const override { return c_->remote_addr(); }
  uint8_t read_byte();
  uint64_t read_uvarint();
  Bytes read_frame(size_t max);  // uvarint length-prefixed
  void unread(const uint8_t* b, size_t n) { pending_.insert(pending_.begin(), b, b + n); }
  const ConnPtr& inner() const { return c_; }

 private:
  ConnPtr c_;
  Bytes pending_;
};

void write_frame(Conn& c, const Bytes& payload);  // uvarint length-prefixed

// ---------------------------------------------------------------- TCP
class TcpConn : public Conn {
 public:
  explicit TcpConn(int fd, std::string remote = "");
  ~TcpConn() override;
  static std::shared_ptr<TcpConn> dial(const std::string& host, int port, int timeout_ms);
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override;
  void write_all(const uint8_t* buf, size_t n) override;
  void close_write() override;
  void close() override;
  void set_read_timeout(int ms) override { timeout_ms_ = ms; }
  std::string remote_addr() const override { return remote_; }
  int fd() const { return fd_; }

 private:
  std::atomic<int> fd_;  // -1 once close() ran; readers/writers check it
  int own_fd_;           // released only by the destructor: no fd reuse under a reader
  int timeout_ms_ = 0;
  std::string remote_;
  std::mutex wmu_;
};

class TcpListener {
 public:
  TcpListener(const std::string& host, int port);  // port 0 = ephemeral
  ~TcpListener();
  std::shared_ptr<TcpConn> accept();  // nullptr once closed
  int port() const { return port_; }
  const std::string& host() const { return host_; }
  void close();

 private:
  std::atomic<int> fd_;
  int own_fd_ = -1;  // released by the destructor (close() only shuts it down)
  int port_ = 0;
  std::string host_;
};

// Local interface addresses (IPv4) for address advertisement.
std::vector<std::string> local_ipv4_addrs(bool include_loopback = true);

// ---------------------------------------------------------------- multistream
extern const char* kMultistreamProto;  // "/multistream/1.0.0"
// Initiator: propose `proto`; throws NetError("protocol not supported") on "na".
void ms_select(BufConn& c, const std::string& proto);
// Proposes protos in order (falling through on "na"); returns the accepted one.
std::string ms_select_any(BufConn& c, const std::vector<std::string>& protos);
// Responder: returns the agreed protocol; throws if the peer gives up.
std::string ms_handle(BufConn& c, const std::set<std::string>& protos);

// ---------------------------------------------------------------- Noise XX
// libp2p Noise: Noise_XX_25519_ChaChaPoly_SHA256, empty prologue, signed
// static-key payload ("noise-libp2p-static-key:" || static pub), 2-byte
// big-endian frame lengths, stream muxer list in the payload extensions.
// The libp2p Noise handshake payload (NoiseHandshakePayload protobuf: identity_key = 1,
// identity_sig = 2 over "noise-libp2p-static-key:" || static_pub, extensions = 4 with the
// early-muxer list) exactly as the handshake sends it; exposed for wire fixtures.
Bytes noise_handshake_payload(const PrivateKey& id_key, const Bytes& static_pub);

class NoiseConn : public Conn {
 public:
  // Runs the handshake over `c`.  Initiator: `expected` (if non-empty) must match
  // the responder's identity.  Throws NetError on any failure.
  static std::shared_ptr<NoiseConn> handshake(ConnPtr c, const PrivateKey& id_key, bool initiator,
                                              const PeerId& expected = PeerId());
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override;
  void write_all(const uint8_t* buf, size_t n) override;
  void close_write() override { c_->close_write(); }
  void close() override { c_->close(); }
  void set_read_timeout(int ms) override { c_->set_read_timeout(ms); }
  std::string remote_addr() const override { return c_->remote_addr(); }
  const PeerId& remote_peer() const { return remote_; }
  const PublicKey& remote_key() const { return remote_key_; }

 private:
  ConnPtr c_;
  PeerId remote_;
  PublicKey remote_key_;
  Bytes k_send_, k_recv_;
  uint64_t n_send_ = 0, n_recv_ = 0;
  Bytes rbuf_;
  size_t rpos_ = 0;
  std::mutex wmu_;
};

}  // namespace p2p
