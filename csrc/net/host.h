// libp2p host: identity, listeners, connection upgrade (multistream -> Noise ->
// multistream -> yamux), peerstore, protocol handlers, identify + ping, and
// dialing through circuit-relay-v2 (relay.h).  Mirrors the subset of the
// go-libp2p host the reference uses (`go/cmd/node/main.go:137-172,243-245`).
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "conn.h"
#include "multiaddr.h"
#include "quic.h"
#include "rcmgr.h"
#include "yamux.h"

namespace p2p {

extern const char* kIdentifyProto;  // "/ipfs/id/1.0.0"
extern const char* kPingProto;      // "/ipfs/ping/1.0.0"
extern const char* kNoiseProto;     // "/noise"
extern const char* kYamuxProto;     // "/yamux/1.0.0"

struct StreamCtx {
  StreamPtr stream;
  std::shared_ptr<BufConn> io;  // read/write through this (keeps pipelined bytes)
  PeerId peer;
  std::string protocol;
  bool relayed = false;
  std::shared_ptr<ResourceManager::Stream> rc;  // resource-manager reservation
};
using StreamHandler = std::function<void(StreamCtx&)>;

struct PeerInfo {
  PeerId id;
  std::vector<Multiaddr> addrs;
};

class Host {
 public:
  explicit Host(PrivateKey key, std::string agent = "p2p-llm-chat-amd/0.1.0");
  ~Host();
  const PeerId& id() const { return id_; }
  const PrivateKey& key() const { return key_; }
  std::string agent() const { return agent_; }

  // Listen on /ip4/<host>/tcp/<port> or /ip4/<host>/udp/<port>/quic-v1 (port 0 =
  // ephemeral).  Other transports are skipped with a log line.
  void listen(const Multiaddr& ma);
  // h.Addrs(): listen addrs with 0.0.0.0 expanded to interface addresses, plus
  // relay circuit addresses of active reservations.
  std::vector<Multiaddr> addrs();
  void add_advertised_addr(const Multiaddr& ma);

  void set_stream_handler(const std::string& proto, StreamHandler h);
  void remove_stream_handler(const std::string& proto);
  std::vector<std::string> protocols();

  // Peerstore
  void add_addrs(const PeerId& p, const std::vector<Multiaddr>& addrs);
  std::vector<Multiaddr> peer_addrs(const PeerId& p);
  std::vector<PeerId> peers();            // peers with a live connection
  bool connected(const PeerId& p);

  // Connect (reuse an existing session, else dial known addrs in order,
  // including /p2p-circuit addresses).  Throws NetError.
  SessionPtr connect(const PeerId& p, const std::vector<Multiaddr>& addrs, int timeout_ms);
  // Open a stream and negotiate `proto` on it.
  StreamCtx new_stream(const PeerId& p, const std::string& proto, int timeout_ms);
  long ping(const PeerId& p, int timeout_ms);

  // Upgrade a raw (TCP or relayed) connection and register the session.
  SessionPtr upgrade_outbound(ConnPtr raw, const PeerId& expected, bool relayed);
  SessionPtr upgrade_inbound(ConnPtr raw, bool relayed);

  // Identify results for a peer (protocols / listen addrs / agent).
  std::vector<std::string> peer_protocols(const PeerId& p);
  std::string peer_agent(const PeerId& p);
  // Transport of the live session: "tcp", "quic-v1" or "p2p-circuit" ("" = none).
  std::string peer_transport(const PeerId& p);

  // Called after identify completes for a peer (protocols, listen addrs); the
  // DHT uses it to fill its routing table like go-libp2p-kad-dht does.
  std::function<void(const PeerId&, const std::vector<std::string>&, const std::vector<Multiaddr>&)>
      on_identified;

  // Relay dialer hook (installed by RelayClient).
  std::function<SessionPtr(const Multiaddr& relay, const PeerId& target, int timeout_ms)> relay_dialer;

  // Secure channels: outbound proposals in this order, inbound accepts any of them.
  // Names: "noise" (/noise), "tls" (/tls/1.0.0).  Default {"noise", "tls"}.
  void set_security(const std::vector<std::string>& order);
  std::vector<std::string> security() const { return security_; }

  // Connection manager (go-libp2p's default host runs connmgr with low 160 / high 192
  // / 1 min grace): once more than `high` sessions are live, the least recently used
  // ones that are past the grace period and carry no open stream are closed until
  // `low` remain.  A trimmed peer is simply re-dialed on its next message.
  void set_conn_limits(int low, int high, int grace_ms);

  // Dial ranking: go-libp2p dials QUIC addresses ahead of TCP ones (its dial
  // ranker delays TCP while a QUIC dial is pending); off = keep address order.
  void set_prefer_quic(bool on) { prefer_quic_ = on; }
  long trimmed() const { return trimmed_; }

  // Resource manager (rcmgr.h): limits default to go-libp2p-like values with RCMGR_*
  // environment overrides; inbound streams / connections over a limit are reset.
  ResourceManager& resources() { return *rcmgr_; }


  void close();
  bool closed() const { return closed_; }

 private:
  void accept_loop(std::shared_ptr<TcpListener> l);
  std::shared_ptr<QuicTransport> quic_for_dial();
  void handle_stream(StreamPtr s, PeerId peer, bool relayed);
  void add_session(const PeerId& p, SessionPtr s, bool relayed, bool inbound);
  void run_identify(const PeerId& p, SessionPtr s);
  void touch(const PeerId& p);
  void trim_connections(const PeerId& keep);
  void identify_handler(StreamCtx& ctx);

  PrivateKey key_;
  PeerId id_;
  std::string agent_;
  std::vector<std::string> security_{"/noise", "/tls/1.0.0"};  // protocol ids, preference order
  std::mutex mu_;
  std::map<std::string, StreamHandler> handlers_;
  std::map<PeerId, std::vector<Multiaddr>> peerstore_;
  std::map<PeerId, SessionPtr> sessions_;
  struct ConnUse {
    std::chrono::steady_clock::time_point opened, used;
  };
  std::map<PeerId, ConnUse> conn_use_;
  int conn_low_ = 160, conn_high_ = 192, conn_grace_ms_ = 60000;
  std::atomic<long> trimmed_{0};
  std::map<PeerId, std::vector<std::string>> peer_protos_;
  std::map<PeerId, std::string> peer_agents_;
  std::map<PeerId, std::string> peer_transport_;
  std::vector<std::shared_ptr<TcpListener>> listeners_;
  std::shared_ptr<QuicTransport> quic_;  // the QUIC listener, or a dial-only socket
  bool prefer_quic_ = true;
  std::shared_ptr<ResourceManager> rcmgr_;
  std::vector<Multiaddr> listen_addrs_;
  std::vector<Multiaddr> extra_addrs_;
  std::vector<std::thread> threads_;
  std::atomic<bool> closed_{false};
  std::atomic<int> busy_{0};  // detached threads that use `this` (drained by close())
  struct Busy {
    Host* h;
    explicit Busy(Host* x) : h(x) { h->busy_++; }
    ~Busy() { h->busy_--; }
  };
};

}  // namespace p2p
