// The chat application layer: ChatMessage (`go/cmd/node/proto/message.go:23-29`),
// the /p2p-llm-chat/1.0.0 one-message-per-stream protocol, Inbox
// (`go/cmd/node/main.go:97-128`), DirectoryClient (`:50-95`), the Directory
// service (`go/cmd/directory/main.go`) and the Node that wires the libp2p host,
// the HTTP API (`:213-283`) and the suggest-reply engine hook together.
#pragma once
#include <atomic>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "host.h"
#include "http.h"
#include "json.h"
#include "kad.h"
#include "natpmp.h"
#include "upnp.h"
#include "relay.h"

namespace p2p {

extern const char* kChatProto;  // "/p2p-llm-chat/1.0.0"
constexpr size_t kMaxChatMessage = 1 << 20;  // the reference reads unbounded (`:160`)

struct ChatMessage {
  std::string id, from_user, to_user, content, timestamp;
  Json to_json() const;  // Go field order: id, from_user, to_user, content, timestamp
  // Go json.Unmarshal semantics for the fields we care about; throws JsonError.
  static ChatMessage from_json(const Json& j);
};

class Inbox {
 public:
  explicit Inbox(std::string persist_path = "", size_t cap = 0);
  void push(const ChatMessage& m);
  // after == "": copy of everything; else messages strictly after the one with id==after;
  // unknown id -> empty (non-destructive, like the reference).
  std::vector<ChatMessage> drain(const std::string& after);
  size_t size();

 private:
  std::mutex mu_;
  std::deque<ChatMessage> q_;  // newest cap_ messages (O(1) trim at the front)
  std::string path_;
  size_t cap_;
};

class DirectoryClient {
 public:
  DirectoryClient(std::string base_url, int timeout_ms = 5000)
      : base_(std::move(base_url)), timeout_ms_(timeout_ms) {}
  void register_user(const std::string& username, const std::string& peer_id,
                     const std::vector<std::string>& addrs);  // throws on non-200
  // throws on transport error / non-200
  void lookup(const std::string& username, std::string* peer_id, std::vector<std::string>* addrs);

 private:
  std::string base_;
  int timeout_ms_;
};

struct DirectoryRecord {
  std::string peer_id;
  std::vector<std::string> addrs;
  int64_t last_ms = 0;
};

class DirectoryService {
 public:
  explicit DirectoryService(int ttl_s = 0) : ttl_s_(ttl_s) {}
  void install(HttpServer& srv);
  size_t size();

 private:
  std::mutex mu_;
  std::map<std::string, DirectoryRecord> data_;
  int ttl_s_;
};

struct NodeConfig {
  std::string username = "userA";
  std::string http_addr = "127.0.0.1:8081";
  std::string directory_url = "http://127.0.0.1:8080";
  std::string bootstrap;         // comma-separated multiaddrs
  std::string relays;            // comma-separated relay multiaddrs (opt-in)
  std::vector<std::string> listen = {"/ip4/0.0.0.0/tcp/0", "/ip4/0.0.0.0/udp/0/quic-v1"};
  std::string key_type = "rsa";  // reference: RSA-2048, regenerated each run
  std::string identity_file;     // opt-in persistence (libp2p PrivateKey protobuf)
  std::string inbox_file;        // opt-in JSONL persistence
  size_t inbox_cap = 100000;     // INBOX_CAP: newest messages kept (0 = unbounded, as the reference)
  std::string engine_url;        // forward /api/generate here when no in-process engine
  std::string llm_model = "llama3.1";
  std::string ui_file;           // optional browser UI served at GET / and GET /ui
  int register_interval_s = 0;   // 0 = register once (reference); >0 = refresh timer
  bool strict_sender = false;    // reject messages whose from_user != directory name of the peer
  bool access_log = true;
  // Kademlia (`/ipfs/kad/1.0.0`): "auto"/"server" answer queries, "client" only
  // queries, "off" disables.  The reference's dht.ModeAuto (main.go:151) is inert
  // without AutoNAT; we serve by default (no AutoNAT here) -- documented deviation.
  std::string dht_mode = "auto";
  // NAT port mapping (reference: libp2p.NATPortMap(), main.go:143): "off" (default here:
  // loopback tests/CI), "on" (default gateway) or an explicit "ip[:port]" NAT-PMP gateway
  std::string nat_pmp = "off";
  // UPnP-IGD port mapping (the other half of NATPortMap): "off", "on" (SSDP multicast),
  // "ip:port" (unicast M-SEARCH to that responder) or the device description URL
  std::string upnp = "off";
  // Secure channels, outbound preference order ("noise", "tls" = /tls/1.0.0); inbound
  // accepts every listed one.  go-libp2p's default host offers both (TLS first).
  std::string security = "noise,tls";
  // connection manager watermarks (go-libp2p default connmgr: 160 / 192, 1 min grace)
  int conn_low = 160, conn_high = 192, conn_grace_ms = 60000;
  // Dial ranking when a peer has QUIC and TCP addresses: "quic" (go-libp2p's
  // ranker: QUIC first) or "order" (as advertised)
  std::string dial_prefer = "quic";
  static NodeConfig from_env();
};

// Engine hook: Ollama /api/generate request JSON -> response JSON (in-process engine).
using GenerateHook = std::function<Json(const Json& req)>;
// Streaming engine hook: emit(chunk) per token batch (false = client gone); returns
// the final `done: true` object.
using GenerateStreamHook =
    std::function<Json(const Json& req, const std::function<bool(const Json&)>& emit)>;

class Node {
 public:
  explicit Node(NodeConfig cfg);
  ~Node();
  // Builds the host, registers with the directory (throws like log.Fatal), dials
  // bootstrap peers and starts the HTTP API.  Non-blocking.
  void start();
  void wait();  // blocks until stop()
  void stop();
  int http_port() const { return http_.port(); }
  std::string peer_id() const { return host_ ? host_->id().to_base58() : ""; }
  std::vector<std::string> addrs() const { return addrs_; }
  void set_generate_hook(GenerateHook h);
  void set_generate_stream_hook(GenerateStreamHook h);
  Inbox& inbox() { return inbox_; }
  std::shared_ptr<Host> host() { return host_; }
  Kad* kad() { return kad_.get(); }
  // POST /send semantics; returns (status, json body)
  std::pair<int, Json> send(const std::string& to, const std::string& content);
  Json metrics_json();

 private:
  void on_chat(StreamCtx& c);
  void setup_nat();
  void install_routes();
  Json generate(const Json& req);
  NodeConfig cfg_;
  std::shared_ptr<Host> host_;
  std::unique_ptr<RelayClient> relay_client_;
  std::unique_ptr<Kad> kad_;
  std::unique_ptr<NatPmp> nat_;
  std::unique_ptr<UpnpIgd> upnp_;
  std::unique_ptr<DirectoryClient> dir_;
  Inbox inbox_;
  HttpServer http_;
  std::vector<std::string> addrs_;
  std::mutex hook_mu_;
  GenerateHook hook_;
  GenerateStreamHook stream_hook_;
  std::thread refresher_;
  std::atomic<bool> stopping_{false};
  std::mutex stop_mu_;  // a second stop() caller blocks until the first finished
  std::atomic<long> n_sent_{0}, n_recv_{0}, n_suggest_{0}, n_send_fail_{0};
};

}  // namespace p2p
