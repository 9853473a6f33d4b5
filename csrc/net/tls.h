// libp2p TLS 1.3 security transport (`/tls/1.0.0`) on OpenSSL 3.
//
// The second of go-libp2p's default secure channels (the reference host is built
// with go-libp2p defaults, `go/cmd/node/main.go:137-144`).  Per the
// libp2p TLS spec:
//   * each side presents a fresh self-signed X.509 certificate (ECDSA P-256 key)
//     carrying the extension 1.3.6.1.4.1.53594.1.1 =
//       SignedKey ::= SEQUENCE { publicKey OCTET STRING, signature OCTET STRING }
//     where publicKey is the host's libp2p PublicKey protobuf and signature is the
//     host key's signature over "libp2p-tls-handshake:" || DER(cert SubjectPublicKeyInfo);
//   * TLS 1.3 only, mutual authentication, no CA: the peer is authenticated by
//     that extension, its PeerID is derived from the embedded key;
//   * ALPN carries early muxer negotiation: the client offers
//     ["yamux/1.0.0", "libp2p"]; a server that selects "yamux/1.0.0" skips the
//     multistream round for the muxer ("libp2p" = negotiate it in-band).
//
// The record layer runs over memory BIOs so that a yamux reader thread blocked
// waiting for bytes never holds the SSL object: the socket I/O happens outside
// the SSL lock and writers serialise on their own mutex (an SSL object must not
// be entered by two threads at once).
#pragma once
#include <memory>
#include <mutex>
#include <string>

#include "conn.h"
#include "crypto.h"

namespace p2p {

extern const char* kTlsProto;  // "/tls/1.0.0"

class TlsConn : public Conn {
 public:
  // Runs the TLS 1.3 handshake over `c` (client when `initiator`).  `expected`
  // (initiator, if non-empty) must match the server's identity.  Throws NetError.
  static std::shared_ptr<TlsConn> handshake(ConnPtr c, const PrivateKey& id_key, bool initiator,
                                            const PeerId& expected = PeerId());
  ~TlsConn() override;
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override;
  void write_all(const uint8_t* buf, size_t n) override;
  void close_write() override;
  void close() override { c_->close(); }
  void set_read_timeout(int ms) override { c_->set_read_timeout(ms); }
  std::string remote_addr() const override { return c_->remote_addr(); }
  const PeerId& remote_peer() const { return remote_; }
  const PublicKey& remote_key() const { return remote_key_; }
  // ALPN-selected muxer ("yamux/1.0.0") or "" when the muxer is negotiated in-band.
  const std::string& early_muxer() const { return muxer_; }

 private:
  TlsConn() = default;
  void flush_locked_out(std::unique_lock<std::mutex>& ssl_lk);  // wbio -> socket
  bool feed();                                                   // socket -> rbio

  ConnPtr c_;
  void* ctx_ = nullptr;  // SSL_CTX*
  void* ssl_ = nullptr;  // SSL*
  void* rbio_ = nullptr;
  void* wbio_ = nullptr;
  std::mutex ssl_mu_;  // guards the SSL object and both BIOs
  std::mutex wmu_;     // orders encrypted bytes on the socket (taken before ssl_mu_)
  PeerId remote_;
  PublicKey remote_key_;
  std::string muxer_;
  bool eof_ = false;
};

// Certificate extension helpers (exposed for tests / codecs).
Bytes tls_signed_key_der(const Bytes& pubkey_pb, const Bytes& sig);
bool tls_parse_signed_key(const Bytes& der, Bytes* pubkey_pb, Bytes* sig);
// The libp2p certificate of `id` (fresh P-256 key; EVP_PKEY** / X509** as void**),
// and authentication of a peer certificate (X509*) -> its libp2p key and PeerID.
// Shared with the QUIC transport, whose TLS handshake carries the same certificate.
void tls_make_cert(const PrivateKey& id, void** key_out, void** cert_out);
void tls_verify_peer_cert(void* x509, PublicKey* key, PeerId* id);

}  // namespace p2p
