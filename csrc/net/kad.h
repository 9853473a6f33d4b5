// Minimal Kademlia DHT speaking libp2p's `/ipfs/kad/1.0.0` wire protocol
// (inventory A5).
//
// The reference constructs `dht.New(ctx, h, dht.Mode(dht.ModeAuto))` and never
// uses the handle (`go/cmd/node/main.go:150-154`): the DHT's only observable
// effect is that the node answers kad queries once it acts as a DHT server.
// This implements that surface natively:
//   * server: FIND_NODE / PING, plus in-memory GET_VALUE/PUT_VALUE and
//     ADD_PROVIDER/GET_PROVIDERS (records are never validated, like a
//     namespace-less kad store) on varint-length-prefixed protobuf messages;
//   * routing table: 256 k-buckets (k = 20) over XOR distance of
//     sha256(peer id multihash); peers are added when identify shows they
//     speak the kad protocol (what go-libp2p-kad-dht does), or explicitly;
//   * client: single FIND_NODE query and an iterative lookup (alpha = 3).
#pragma once
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "host.h"

namespace p2p {

extern const char* kKadProto;  // "/ipfs/kad/1.0.0"

enum class KadMode { Off, Client, Server };

struct KadPeer {
  PeerId id;
  std::vector<Multiaddr> addrs;
  int connection = 0;  // ConnectionType: 0 not connected, 1 connected
};

// Wire message (subset of dht.pb Message).
struct KadMessage {
  enum Type { PUT_VALUE = 0, GET_VALUE = 1, ADD_PROVIDER = 2, GET_PROVIDERS = 3, FIND_NODE = 4, PING = 5 };
  int type = FIND_NODE;
  Bytes key;
  Bytes record_key, record_value;  // Record{key=1, value=2}
  bool has_record = false;
  std::vector<KadPeer> closer, providers;
  Bytes encode() const;
  static KadMessage decode(const Bytes& b);
};

// XOR distance helpers over sha256 keyspace.
Bytes kad_key(const Bytes& raw);                       // sha256(raw)
int kad_common_prefix_len(const Bytes& a, const Bytes& b);
bool kad_closer(const Bytes& target, const Bytes& a, const Bytes& b);  // d(a) < d(b)

class Kad {
 public:
  static constexpr int K = 20;
  static constexpr int ALPHA = 3;

  Kad(std::shared_ptr<Host> host, KadMode mode);
  ~Kad();
  KadMode mode() const { return mode_; }

  // Routing table
  bool add_peer(const PeerId& p, const std::vector<Multiaddr>& addrs);
  void remove_peer(const PeerId& p);
  size_t size();
  std::vector<KadPeer> closest(const Bytes& key, int n, const PeerId* exclude = nullptr);

  // Client
  std::vector<KadPeer> find_node(const PeerId& peer, const Bytes& key, int timeout_ms = 5000);
  bool ping(const PeerId& peer, int timeout_ms = 5000);
  // Iterative lookup of the k closest peers to key (queries the network).
  std::vector<KadPeer> lookup(const Bytes& key, int timeout_ms = 10000);
  // Finds a peer's addresses through the DHT (lookup(peer) + exact match).
  bool find_peer(const PeerId& target, std::vector<Multiaddr>* addrs, int timeout_ms = 10000);
  // Self-lookup to populate the table from the bootstrap peers.
  void bootstrap(int timeout_ms = 10000);

  // Local store (served to queries)
  void put_local(const Bytes& key, const Bytes& value);
  bool get_local(const Bytes& key, Bytes* value);

 private:
  void handle(StreamCtx& c);
  KadMessage respond(const KadMessage& req, const PeerId& from);
  KadMessage request(const PeerId& peer, const KadMessage& m, int timeout_ms);

  std::shared_ptr<Host> host_;
  KadMode mode_;
  Bytes self_key_;
  std::mutex mu_;
  std::vector<std::vector<KadPeer>> buckets_;  // [256], most recently seen last
  std::map<Bytes, Bytes> values_;
  std::map<Bytes, std::vector<KadPeer>> providers_;
};

}  // namespace p2p
