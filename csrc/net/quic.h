// QUIC v1 transport for libp2p (`/udp/<port>/quic-v1`, RFC 9000 / 9001), the
// second listener of the reference host (`go/cmd/node/main.go:140`).
//
// libp2p over QUIC needs no separate security or muxer negotiation: the TLS 1.3
// handshake runs inside QUIC (ALPN "libp2p", the same self-signed certificate
// with the libp2p SignedKey extension as `/tls/1.0.0`, tls.h) and every libp2p
// stream is a native bidirectional QUIC stream on which multistream-select picks
// the application protocol.
//
// Design (one UDP socket per transport, one thread):
//   * QuicTransport owns the socket and a receive thread that demultiplexes
//     datagrams by destination connection id (8-byte ids chosen by each side),
//     creates a server connection for a fresh 1200-byte Initial, and ticks every
//     connection's timers (PTO retransmission, idle timeout, keep-alive PING).
//   * QuicConn is a MuxSession.  Packet protection is RFC 9001: Initial keys
//     from the client's first destination id, AES-128-GCM payload protection,
//     AES-ECB header protection, 4-byte packet numbers, three packet-number
//     spaces with their own ACK state.
//   * TLS: OpenSSL 3.0 has no QUIC API, so the handshake runs on an ordinary TLS
//     1.3 SSL object over memory BIOs and the connection translates between its
//     records and QUIC CRYPTO frames.  The traffic secrets come from the keylog
//     callback; outgoing encrypted records are opened with the writer's own
//     secret to recover the handshake bytes of each encryption level, incoming
//     CRYPTO bytes are sealed into records under the peer's secret.  The QUIC
//     packet keys derive from the same secrets ("quic key/iv/hp").  Middlebox
//     compatibility mode and session tickets are off (QUIC forbids both), the
//     quic_transport_parameters extension (0x39) is a custom TLS extension.
//   * Loss recovery is PTO-based: every ack-eliciting packet keeps its frames;
//     when the probe timeout fires the frames go back to the send queue and are
//     re-sent in new packets (stream and CRYPTO frames are offset-addressed, so
//     a re-send is idempotent).  Flow control: connection and stream credit with
//     MAX_DATA / MAX_STREAM_DATA / MAX_STREAMS updates as the reader consumes.
//
// Not implemented (not needed between libp2p peers on a LAN/loopback): Retry,
// version negotiation, 0-RTT, connection migration, key update, ECN, congestion
// control beyond the flow-control windows.
#pragma once
#include <netinet/in.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "crypto.h"
#include "mux.h"

namespace p2p {

class QuicConn;

// RFC 9000 §16 variable-length integer (exposed for frame-level tests).
void quic_put_varint(Bytes& b, uint64_t v);
class QuicTransport;

class QuicStream : public MuxStream {
 public:
  QuicStream(std::shared_ptr<QuicConn> c, uint64_t id);
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override;
  void write_all(const uint8_t* buf, size_t n) override;
  void close_write() override;  // FIN
  void close() override;        // FIN + discard further input
  void reset() override;        // RESET_STREAM + STOP_SENDING
  void set_read_timeout(int ms) override { timeout_ms_ = ms; }
  std::string remote_addr() const override;
  uint64_t id() const { return id_; }

 private:
  friend class QuicConn;
  std::shared_ptr<QuicConn> c_;
  uint64_t id_;
  int timeout_ms_ = 0;
  // ---- guarded by the connection mutex
  std::map<uint64_t, Bytes> ooo_;  // out-of-order received segments by offset
  Bytes rbuf_;
  size_t rpos_ = 0;
  uint64_t recv_off_ = 0;            // next in-order offset
  uint64_t recv_high_ = 0;           // highest offset received (flow-control accounting)
  uint64_t fin_off_ = ~0ull;         // final size once the FIN arrived
  uint64_t consumed_ = 0, recv_limit_ = 0;
  Bytes sq_;                         // queued, not yet packetised (from sq_head_)
  size_t sq_head_ = 0;
  size_t queued() const { return sq_.size() - sq_head_; }
  uint64_t send_off_ = 0;            // stream offset of sq_[0]
  uint64_t max_send_ = 0;            // peer's credit for this stream
  bool fin_pending_ = false, fin_sent_ = false, local_closed_ = false;
  bool reset_ = false, stop_sending_ = false;
};

struct QuicKeys {
  bool ok = false;
  uint8_t key[16], iv[12], hp[16];
};
// RFC 9001 §5.2 Initial secrets for a client destination connection id
// (exposed for the Appendix A test vectors).
void quic_initial_keys(const Bytes& dcid, QuicKeys* client, QuicKeys* server);

class QuicConn : public MuxSession, public std::enable_shared_from_this<QuicConn> {
 public:
  static constexpr size_t kCidLen = 8;
  QuicConn(std::shared_ptr<QuicTransport> t, bool client, const sockaddr_in& peer,
           const PrivateKey& key);
  ~QuicConn() override;

  void start(std::function<void(StreamPtr)> on_stream,
             std::function<void()> on_close = nullptr) override;
  StreamPtr open_stream() override;
  void close() override;
  bool closed() const override { return closed_; }
  long ping(int timeout_ms) override;
  size_t num_streams() override;
  std::string transport() const override { return "quic-v1"; }

  const PeerId& remote_peer() const { return remote_; }
  std::string remote_addr() const;
  bool established() const { return established_; }
  uint64_t retransmitted() const { return retx_count_; }

  // TLS callbacks (OpenSSL keylog / custom extension 0x39); mutex held by the caller.
  void tls_keylog(const char* line);
  Bytes tp_encode() const { return transport_params(); }
  void tp_parse(const uint8_t* p, size_t n) { parse_transport_params(p, n); }
  // test hooks: queue one raw 1-RTT frame (protocol-violation tests); the close reason
  void send_raw_frame_for_test(const Bytes& frame);
  std::string error_text();

 private:
  friend class QuicTransport;
  friend class QuicStream;
  enum { INITIAL = 0, HANDSHAKE = 1, APP = 2 };
  struct SentPkt {
    std::chrono::steady_clock::time_point t;
    std::vector<Bytes> frames;  // retransmittable frames (raw encodings)
    size_t bytes = 0;           // datagram bytes (congestion accounting)
  };
  struct Space {
    uint64_t next_pn = 0;
    QuicKeys tx, rx;
    std::set<uint64_t> recvd;
    uint64_t recv_floor = 0;
    bool ack_pending = false;
    std::map<uint64_t, SentPkt> sent;
    std::deque<Bytes> queued;  // control frames and retransmissions
    Bytes crypto_pending;      // handshake bytes not yet framed
    uint64_t crypto_send_off = 0;
    std::map<uint64_t, Bytes> crypto_in;
    uint64_t crypto_in_off = 0;
    size_t crypto_in_bytes = 0;      // buffered out-of-order CRYPTO bytes (capped)
    std::vector<Bytes> undecryptable;  // packets that arrived before their keys
  };
  struct Events {  // callbacks run after the connection mutex is released
    std::vector<StreamPtr> streams;
    bool accepted = false, closed = false;
  };

  // -- called by the transport thread / dialer
  // key_cid: the client DCID the Initial keys derive from (after a Retry: the Retry's
  // SCID; default odcid); retry_scid: server side, the SCID of the Retry it sent
  void begin(const Bytes& dcid, const Bytes& scid, const Bytes& odcid,
             const Bytes& key_cid = Bytes(), const Bytes& retry_scid = Bytes());
  void on_retry(const Bytes& scid, const Bytes& token);
  void on_datagram(const uint8_t* d, size_t n);
  void tick(std::chrono::steady_clock::time_point now);
  bool wait_established(int timeout_ms);
  std::vector<Bytes> local_cids() const { return {scid_, odcid_}; }

  // -- internals (mutex held)
  void handle_packet(Bytes pkt, size_t pn_off, int space, bool long_hdr, Events& ev);
  void process_frames(int space, const uint8_t* p, size_t n, bool* elicit, Events& ev);
  void on_ack(int space, const uint8_t* p, size_t n, size_t* pos, bool ecn);
  void on_crypto(int space, uint64_t off, const uint8_t* data, size_t len, Events& ev);
  void on_stream_frame(uint64_t id, uint64_t off, const uint8_t* data, size_t len, bool fin,
                       Events& ev);
  std::shared_ptr<QuicStream> peer_stream(uint64_t id, Events& ev);
  void tls_drive(Events& ev);
  void tls_collect_output();
  void tls_feed(int level, const uint8_t* data, size_t len);
  void on_handshake_complete(Events& ev);
  void install_keys();
  void flush();
  void send_packet(int space, const Bytes& payload, bool elicit, std::vector<Bytes> frames);
  Bytes ack_frame(int space);
  void credit_after_read(QuicStream* s, size_t n);
  void maybe_remove(QuicStream* s);
  void fail(const std::string& why, uint64_t code, Events& ev);
  void close_locked(uint64_t code, bool app, Events& ev, bool send = true);
  void run(Events& ev);
  Bytes transport_params() const;
  void parse_transport_params(const uint8_t* p, size_t n);

  std::weak_ptr<QuicTransport> tr_;
  int fd_;
  bool client_;
  sockaddr_in peer_;
  const PrivateKey& key_;
  Bytes dcid_, scid_, odcid_;
  bool dcid_switched_ = false;
  // Retry (RFC 9000 §8.1.2 / §17.2.5): client -- the token echoed in every later Initial
  // and the Retry's SCID (checked against the server's retry_source_connection_id);
  // server -- the SCID of the Retry it sent (its transport parameter 0x10)
  bool retry_seen_ = false;
  Bytes retry_token_, retry_scid_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  Space sp_[3];
  // TLS
  void* ctx_ = nullptr;
  void* ssl_ = nullptr;
  void* rbio_ = nullptr;
  void* wbio_ = nullptr;
  Bytes tls_out_;  // unparsed records from the SSL write BIO
  Bytes sec_[2][2];  // [hs=0|app=1][client=0|server=1] traffic secrets
  int wr_epoch_ = 0;  // my write epoch in the record stream: 0 hs, 1 app
  uint64_t wr_seq_ = 0, rd_seq_[2] = {0, 0};
  bool tls_done_ = false;
  // transport parameters
  bool peer_tp_ = false;
  Bytes peer_odcid_;
  bool peer_has_retry_scid_ = false;
  Bytes peer_retry_scid_;
  uint64_t peer_max_data_ = 0, peer_sd_local_ = 0, peer_sd_remote_ = 0, peer_max_bidi_ = 0;
  uint64_t peer_idle_ms_ = 0;
  // state
  std::atomic<bool> closed_{false};
  std::atomic<bool> established_{false};
  bool confirmed_ = false, started_ = false, accepted_ = false;
  std::string error_;
  PeerId remote_;
  PublicKey remote_key_;
  // streams
  std::map<uint64_t, std::shared_ptr<QuicStream>> streams_;
  std::set<uint64_t> send_ready_;
  std::vector<StreamPtr> pending_inbound_;
  uint64_t next_local_idx_ = 0, next_remote_idx_ = 0;
  uint64_t remote_closed_ = 0, max_remote_streams_ = 0;
  uint64_t sent_data_ = 0, recv_consumed_ = 0, recv_max_data_ = 0;
  uint64_t recv_total_ = 0;  // sum of every stream's recv_high_ (connection flow control)
  std::function<void(StreamPtr)> on_stream_;
  std::function<void()> on_close_;
  // recovery
  double srtt_ms_ = 0, rttvar_ms_ = 0, latest_rtt_ms_ = 0;
  int pto_count_ = 0;
  std::atomic<uint64_t> retx_count_{0};
  std::chrono::steady_clock::time_point last_recv_, last_send_;
  std::map<uint64_t, bool> pings_;  // app packet number -> acked
  // NewReno congestion control (RFC 9002 §7)
  uint64_t cwnd_ = 0, ssthresh_ = ~0ull, bytes_in_flight_ = 0;
  std::chrono::steady_clock::time_point recovery_start_{};
  std::atomic<uint64_t> congestion_events_{0};
  void on_packet_acked(const SentPkt& p);
  void on_packets_lost(int space, std::chrono::steady_clock::time_point newest_lost_sent);
  void detect_lost(int space, uint64_t largest_acked, std::chrono::steady_clock::time_point now);
  // 1-RTT key update (RFC 9001 §6): current generation secrets, the key phase bit, the
  // previous generation's receive keys (late packets) and the next generation's
  Bytes app_sec_tx_, app_sec_rx_;
  QuicKeys rx_prev_, rx_next_;
  int key_phase_ = 0;
  uint64_t phase_first_pn_ = 0, phase_sent_ = 0;
  bool phase_acked_ = true;
  std::atomic<uint64_t> key_updates_{0};
  void update_tx_keys();
  void update_rx_keys();

 public:
  // Start a key update now (if the current phase is acknowledged); returns whether it did.
  bool force_key_update();
  uint64_t key_updates() const { return key_updates_; }
  uint64_t congestion_events() const { return congestion_events_; }
  uint64_t cwnd() const { return cwnd_; }
};
// Packets sent per key phase before an endpoint starts a key update (AES-128-GCM
// confidentiality limit is 2^23 packets; tests lower it).
void quic_set_key_update_interval(uint64_t packets);
using QuicConnPtr = std::shared_ptr<QuicConn>;

class QuicTransport : public std::enable_shared_from_this<QuicTransport> {
 public:
  // Binds a UDP socket on host:port (port 0 = ephemeral).  `key` must outlive it.
  static std::shared_ptr<QuicTransport> create(const std::string& host, int port,
                                               const PrivateKey& key);
  ~QuicTransport();
  int port() const { return port_; }
  const std::string& host() const { return host_; }
  // Inbound: called (in its own thread) for every connection whose handshake and
  // peer authentication completed.  Unset = dial-only transport.
  void set_accept(std::function<void(QuicConnPtr)> cb);
  // Outbound: handshake with host:port; `expected` (if non-empty) must match the
  // peer's identity.  Throws NetError.
  QuicConnPtr dial(const std::string& host, int port, const PeerId& expected, int timeout_ms);
  void close();
  // Test hook: drop this fraction of received datagrams (loss-recovery tests).
  void set_drop_rate(double r) { drop_rate_ = r; }
  long version_negotiations_sent() const { return vn_sent_; }
  // Address validation (RFC 9000 §8.1.2): answer every token-less client Initial with a
  // Retry and accept only Initials echoing a valid token (env P2P_QUIC_RETRY=1 at create).
  void set_require_retry(bool on) { require_retry_ = on; }
  long retries_sent() const { return retries_sent_; }
  long tokens_rejected() const { return tokens_rejected_; }

 private:
  friend class QuicConn;
  QuicTransport(const PrivateKey& key) : key_(key) {}
  void loop();
  void dispatch(const uint8_t* d, size_t n, const sockaddr_in& from);
  void send_version_negotiation(const uint8_t* d, size_t n, const sockaddr_in& to);
  void send_retry(const Bytes& odcid, const Bytes& client_scid, const sockaddr_in& to);
  bool check_token(const Bytes& token, const Bytes& dcid, const sockaddr_in& from,
                   Bytes* odcid) const;
  Bytes token_mac(const sockaddr_in& peer, const uint8_t* body, size_t n) const;
  void forget(const QuicConn* c);
  void register_cid(const Bytes& cid, const QuicConnPtr& c);

  const PrivateKey& key_;
  int fd_ = -1;
  int port_ = 0;
  std::string host_;
  std::mutex mu_;
  std::map<Bytes, QuicConnPtr> by_cid_;
  std::function<void(QuicConnPtr)> accept_;
  std::thread th_;
  std::atomic<bool> closed_{false};
  std::atomic<int> busy_{0};
  double drop_rate_ = 0;
  std::atomic<long> vn_sent_{0};
  std::atomic<bool> require_retry_{false};
  Bytes token_key_;  // random per transport: Retry tokens are only valid at this server
  std::atomic<long> retries_sent_{0}, tokens_rejected_{0};
};
// RFC 9001 §5.8 Retry integrity tag over the Retry pseudo-packet (odcid + the Retry
// packet without its tag); exposed for the RFC 9001 Appendix A.4 vector test.
Bytes quic_retry_tag(const Bytes& odcid, const uint8_t* retry, size_t len);

}  // namespace p2p
