#include "chat.h"

#include <algorithm>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <fstream>
#include <sstream>

namespace p2p {

const char* kChatProto = "/p2p-llm-chat/1.0.0";

// ================================================================ ChatMessage
Json ChatMessage::to_json() const {
  Json j = Json::object();
  j.set("id", id);
  j.set("from_user", from_user);
  j.set("to_user", to_user);
  j.set("content", content);
  j.set("timestamp", timestamp);
  return j;
}

static std::string go_type(const Json& v) {
  switch (v.type()) {
    case Json::Bool: return "bool";
    case Json::Number: return "number";
    case Json::Array: return "array";
    case Json::Object: return "object";
    default: return "string";
  }
}

static std::string str_field(const Json& j, const char* k, const char* go_struct) {
  const Json& v = j.get(k);
  if (v.is_null()) return "";
  if (!v.is_string())
    throw JsonError(std::string("json: cannot unmarshal ") + go_type(v) +
                    " into Go struct field " + go_struct + "." + k + " of type string");
  return v.str();
}

ChatMessage ChatMessage::from_json(const Json& j) {
  if (!j.is_object()) throw JsonError("json: cannot unmarshal " + go_type(j) +
                                      " into Go value of type proto.ChatMessage");
  ChatMessage m;
  m.id = str_field(j, "id", "ChatMessage");
  m.from_user = str_field(j, "from_user", "ChatMessage");
  m.to_user = str_field(j, "to_user", "ChatMessage");
  m.content = str_field(j, "content", "ChatMessage");
  const Json& ts = j.get("timestamp");
  if (ts.is_null()) {
    m.timestamp = "0001-01-01T00:00:00Z";  // Go zero time
  } else {
    if (!ts.is_string()) throw JsonError("json: cannot unmarshal into time.Time");
    parse_rfc3339(ts.str());  // validates like time.Time.UnmarshalJSON
    m.timestamp = ts.str();
  }
  return m;
}

// ================================================================ Inbox
Inbox::Inbox(std::string persist_path, size_t cap) : path_(std::move(persist_path)), cap_(cap) {
  if (path_.empty()) return;
  std::ifstream f(path_);
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty()) continue;
    try {
      q_.push_back(ChatMessage::from_json(Json::parse(line)));
    } catch (...) {
    }
  }
  while (cap_ && q_.size() > cap_) q_.pop_front();
}

void Inbox::push(const ChatMessage& m) {
  std::lock_guard<std::mutex> lk(mu_);
  q_.push_back(m);
  while (cap_ && q_.size() > cap_) q_.pop_front();
  if (!path_.empty()) {
    FILE* f = fopen(path_.c_str(), "a");
    if (f) {
      std::string s = m.to_json().dump() + "\n";
      fwrite(s.data(), 1, s.size(), f);
      fclose(f);
    }
  }
}

std::vector<ChatMessage> Inbox::drain(const std::string& after) {
  std::lock_guard<std::mutex> lk(mu_);
  if (after.empty()) return std::vector<ChatMessage>(q_.begin(), q_.end());
  std::vector<ChatMessage> out;
  bool found = false;
  for (auto& m : q_) {
    if (m.id == after) {
      found = true;
      continue;
    }
    if (found) out.push_back(m);
  }
  return out;
}

size_t Inbox::size() {
  std::lock_guard<std::mutex> lk(mu_);
  return q_.size();
}

// ================================================================ Directory client
void DirectoryClient::register_user(const std::string& username, const std::string& peer_id,
                                    const std::vector<std::string>& addrs) {
  Json body = Json::object();
  body.set("username", username);
  body.set("peer_id", peer_id);
  body.set("addrs", Json::array_of(addrs));
  HttpResult r = http_request("POST", base_ + "/register", body.dump(), "application/json",
                              timeout_ms_);
  if (r.status != 200) throw NetError("register failed: " + r.body);
}

void DirectoryClient::lookup(const std::string& username, std::string* peer_id,
                             std::vector<std::string>* addrs) {
  HttpResult r = http_request("GET", base_ + "/lookup?username=" + url_encode(username), "", "",
                              timeout_ms_);
  if (r.status != 200) throw NetError("lookup failed: " + r.body);
  Json j = Json::parse(r.body);
  *peer_id = j.get_string("peer_id");
  addrs->clear();
  const Json& a = j.get("addrs");
  if (a.is_array())
    for (auto& x : a.items())
      if (x.is_string()) addrs->push_back(x.str());
}

// ================================================================ Directory service
static std::string bind_error(const std::string& body, const std::exception& e) {
  if (body.find_first_not_of(" \t\r\n") == std::string::npos) return "EOF";
  return e.what();
}

void DirectoryService::install(HttpServer& srv) {
  srv.route("POST", "/register", [this](const HttpRequest& req, HttpResponse& res) {
    std::string username, peer_id;
    std::vector<std::string> addrs;
    try {
      Json j = Json::parse(req.body);
      if (!j.is_object()) throw JsonError("json: cannot unmarshal " + go_type(j) +
                                          " into Go value of type struct");
      username = str_field(j, "username", "Username");
      peer_id = str_field(j, "peer_id", "PeerID");
      const Json& a = j.get("addrs");
      if (!a.is_null()) {
        if (!a.is_array()) throw JsonError("json: cannot unmarshal " + go_type(a) +
                                           " into Go struct field .addrs of type []string");
        for (auto& x : a.items()) {
          if (!x.is_string()) throw JsonError("json: cannot unmarshal " + go_type(x) +
                                              " into Go struct field .addrs of type string");
          addrs.push_back(x.str());
        }
      }
    } catch (const std::exception& e) {
      res.text(400, bind_error(req.body, e));
      return;
    }
    if (username.empty() || peer_id.empty()) {
      res.text(400, "missing fields");
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      data_[username] = DirectoryRecord{peer_id, addrs, unix_ms()};
    }
    Json ok = Json::object();
    ok.set("ok", true);
    res.json(200, ok, true);
  });
  srv.route("GET", "/lookup", [this](const HttpRequest& req, HttpResponse& res) {
    std::string u = req.param("username");
    if (u.empty()) {
      res.text(400, "username required");
      return;
    }
    DirectoryRecord rec;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = data_.find(u);
      if (it == data_.end() || (ttl_s_ > 0 && unix_ms() - it->second.last_ms > ttl_s_ * 1000LL)) {
        res.text(404, "not found");
        return;
      }
      rec = it->second;
    }
    Json j = Json::object();
    j.set("peer_id", rec.peer_id);
    j.set("addrs", rec.addrs.empty() && false ? Json() : Json::array_of(rec.addrs));
    res.json(200, j, true);
  });
  srv.route("GET", "/health", [this](const HttpRequest&, HttpResponse& res) {
    Json j = Json::object();
    j.set("ok", true);
    j.set("users", (long)size());
    res.json(200, j, true);
  });
}

size_t DirectoryService::size() {
  std::lock_guard<std::mutex> lk(mu_);
  return data_.size();
}

// ================================================================ Node
NodeConfig NodeConfig::from_env() {
  NodeConfig c;
  c.username = env_or("MYNAMEIS", c.username);
  c.http_addr = env_or("HTTP_ADDR", c.http_addr);
  c.directory_url = env_or("DIRECTORY_URL", c.directory_url);
  c.bootstrap = env_or("BOOTSTRAP_ADDRS", "");
  c.relays = env_or("RELAY_ADDRS", "");
  c.key_type = env_or("KEY_TYPE", c.key_type);
  c.identity_file = env_or("IDENTITY_FILE", "");
  c.inbox_file = env_or("INBOX_FILE", "");
  c.inbox_cap = (size_t)atoll(env_or("INBOX_CAP", std::to_string(c.inbox_cap)).c_str());
  c.engine_url = env_or("ENGINE_URL", "");
  c.llm_model = env_or("LLM_MODEL", c.llm_model);
  c.ui_file = env_or("UI_FILE", "");
  c.register_interval_s = atoi(env_or("REGISTER_INTERVAL", "0").c_str());
  c.strict_sender = env_or("STRICT_SENDER", "0") == "1";
  c.access_log = env_or("GIN_MODE", "debug") != "quiet";
  c.dht_mode = env_or("DHT_MODE", c.dht_mode);
  c.nat_pmp = env_or("NAT_PMP", c.nat_pmp);
  c.security = env_or("SECURITY", c.security);
  c.upnp = env_or("UPNP", c.upnp);
  c.conn_low = atoi(env_or("CONN_LOW", std::to_string(c.conn_low)).c_str());
  c.conn_high = atoi(env_or("CONN_HIGH", std::to_string(c.conn_high)).c_str());
  c.conn_grace_ms = (int)(atof(env_or("CONN_GRACE", "60").c_str()) * 1000);
  c.dial_prefer = env_or("DIAL_PREFER", c.dial_prefer);
  std::string la = env_or("LISTEN_ADDRS", "");
  if (la == "none") {
    c.listen.clear();  // relay-only node
  } else if (!la.empty()) {
    c.listen.clear();
    std::stringstream ss(la);
    std::string t;
    while (std::getline(ss, t, ','))
      if (!t.empty()) c.listen.push_back(t);
  }
  return c;
}

static std::vector<std::string> split_csv(const std::string& s) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, ',')) {
    size_t a = t.find_first_not_of(" \t"), b = t.find_last_not_of(" \t");
    if (a == std::string::npos) continue;
    out.push_back(t.substr(a, b - a + 1));
  }
  return out;
}

static PrivateKey load_or_make_identity(const NodeConfig& cfg) {
  KeyType kt = cfg.key_type == "ed25519" ? KeyType::Ed25519 : KeyType::RSA;
  if (!cfg.identity_file.empty()) {
    std::ifstream f(cfg.identity_file, std::ios::binary);
    if (f) {
      Bytes b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      return PrivateKey::unmarshal(b);
    }
    PrivateKey k = PrivateKey::generate(kt, 2048);
    std::ofstream o(cfg.identity_file, std::ios::binary);
    Bytes b = k.marshal();
    o.write((const char*)b.data(), (std::streamsize)b.size());
    return k;
  }
  return PrivateKey::generate(kt, 2048);  // fresh identity every run, like the reference
}

Node::Node(NodeConfig cfg)
    : cfg_(std::move(cfg)), inbox_(cfg_.inbox_file, cfg_.inbox_cap), http_("GIN") {}

Node::~Node() { stop(); }

void Node::set_generate_stream_hook(GenerateStreamHook h) {
  std::lock_guard<std::mutex> lk(hook_mu_);
  stream_hook_ = std::move(h);
}

void Node::set_generate_hook(GenerateHook h) {
  std::lock_guard<std::mutex> lk(hook_mu_);
  hook_ = std::move(h);
}

void Node::on_chat(StreamCtx& c) {
  Bytes data;
  try {
    c.io->set_read_timeout(30000);
    data = c.io->read_all(kMaxChatMessage);
  } catch (const std::exception& e) {
    logf("read stream: %s", e.what());
    c.stream->reset();
    return;
  }
  c.stream->close();
  ChatMessage m;
  try {
    m = ChatMessage::from_json(Json::parse(to_string(data)));
  } catch (const std::exception& e) {
    logf("unmarshal: %s", e.what());
    return;
  }
  if (cfg_.strict_sender) {
    try {
      std::string pid;
      std::vector<std::string> addrs;
      dir_->lookup(m.from_user, &pid, &addrs);
      if (pid != c.peer.to_base58()) {
        logf("dropping message: from_user %s does not match peer %s", m.from_user.c_str(),
             c.peer.to_base58().c_str());
        return;
      }
    } catch (...) {
      logf("dropping message: cannot verify sender %s", m.from_user.c_str());
      return;
    }
  }
  inbox_.push(m);
  n_recv_++;
  logf("📩 Received from %s: %s", m.from_user.c_str(), m.content.c_str());
}

void Node::start() {
  PrivateKey key = load_or_make_identity(cfg_);
  host_ = std::make_shared<Host>(key);
  host_->set_security(split_csv(cfg_.security));
  host_->set_conn_limits(cfg_.conn_low, cfg_.conn_high, cfg_.conn_grace_ms);
  host_->set_prefer_quic(cfg_.dial_prefer == "quic");
  if (cfg_.dht_mode != "off") {
    // created before any listener/dial so identify results feed the routing table
    kad_ = std::make_unique<Kad>(host_, cfg_.dht_mode == "client" ? KadMode::Client : KadMode::Server);
  }
  for (auto& l : cfg_.listen) host_->listen(Multiaddr::parse(l));
  if ((cfg_.nat_pmp != "off" && !cfg_.nat_pmp.empty()) || (cfg_.upnp != "off" && !cfg_.upnp.empty()))
    setup_nat();
  relay_client_ = std::make_unique<RelayClient>(host_);
  host_->set_stream_handler(kChatProto, [this](StreamCtx& c) { on_chat(c); });
  for (auto& r : split_csv(cfg_.relays)) {
    try {
      relay_client_->reserve(Multiaddr::parse(r));
      logf("🔁 reserved relay slot via %s", r.c_str());
    } catch (const std::exception& e) {
      logf("relay reservation failed (%s): %s", r.c_str(), e.what());
    }
  }
  dir_ = std::make_unique<DirectoryClient>(cfg_.directory_url, 5000);
  std::string pid = host_->id().to_base58();
  addrs_.clear();
  for (auto& a : host_->addrs()) addrs_.push_back(a.str() + "/p2p/" + pid);
  dir_->register_user(cfg_.username, pid, addrs_);  // fatal on failure (caller exits)
  logf("👤 %s PeerID=%s", cfg_.username.c_str(), pid.c_str());
  for (auto& b : split_csv(cfg_.bootstrap)) {
    try {
      Multiaddr ma = Multiaddr::parse(b);
      PeerId id;
      Multiaddr bare = ma.without_peer(&id);
      if (id.empty()) throw NetError("invalid p2p multiaddr");
      host_->connect(id, {bare}, 10000);
      logf("✅ connected to bootstrap %s", id.to_base58().c_str());
      if (kad_) kad_->add_peer(id, {bare});
    } catch (const std::exception& e) {
      logf("connect: %s (%s)", e.what(), b.c_str());
    }
  }
  if (cfg_.register_interval_s > 0) {
    refresher_ = std::thread([this] {
      while (!stopping_) {
        for (int i = 0; i < cfg_.register_interval_s * 10 && !stopping_; ++i)
          std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (stopping_) break;
        try {
          std::string p = host_->id().to_base58();
          std::vector<std::string> a;
          for (auto& x : host_->addrs()) a.push_back(x.str() + "/p2p/" + p);
          dir_->register_user(cfg_.username, p, a);
        } catch (const std::exception& e) {
          logf("directory refresh failed: %s", e.what());
        }
      }
    });
  }
  install_routes();
  http_.set_access_log(cfg_.access_log);
  http_.start(cfg_.http_addr);
  logf("📡 HTTP listening on %s", cfg_.http_addr.c_str());
}

void Node::wait() { http_.serve_forever(); }

// NATPortMap (reference main.go:143): NAT-PMP first (NAT_PMP), else UPnP-IGD (UPNP);
// every TCP listen port is mapped, the external address advertised + registered.
void Node::setup_nat() {
  auto tcp_ports = [this] {
    std::vector<int> ports;
    for (auto& a : host_->addrs()) {
      std::string h;
      int port = 0;
      if (!a.tcp_host_port(&h, &port) || a.has(MA_P2P_CIRCUIT)) continue;
      if (std::find(ports.begin(), ports.end(), port) == ports.end()) ports.push_back(port);
    }
    return ports;
  };
  auto advertise = [this](const char* how, const std::string& ext, int port, const NatMapping& m) {
    host_->add_advertised_addr(
        Multiaddr::parse("/ip4/" + ext + "/tcp/" + std::to_string(m.external_port)));
    logf("%s: mapped tcp %d -> %s:%d", how, port, ext.c_str(), m.external_port);
  };
  if (cfg_.nat_pmp != "off" && !cfg_.nat_pmp.empty()) {
    nat_ = std::make_unique<NatPmp>(cfg_.nat_pmp == "on" ? "" : cfg_.nat_pmp, 1000);
    const std::string ext = nat_->ok() ? nat_->external_address() : "";
    if (ext.empty()) {
      logf("NAT-PMP: gateway %s did not answer", nat_->ok() ? nat_->gateway().c_str() : "(none)");
      nat_.reset();
    } else {
      std::vector<NatMapping> maps;
      for (int port : tcp_ports()) {
        NatMapping m;
        if (nat_->map_tcp(port, port, 3600, &m)) {
          maps.push_back(m);
          advertise("NAT-PMP", ext, port, m);
        }
      }
      nat_->keep_alive(maps);
      return;
    }
  }
  if (cfg_.upnp != "off" && !cfg_.upnp.empty()) {
    upnp_ = std::make_unique<UpnpIgd>(cfg_.upnp == "on" ? "" : cfg_.upnp, 2000);
    const std::string ext = upnp_->discover() ? upnp_->external_address() : "";
    if (ext.empty()) {
      logf("UPnP: no internet gateway device answered");
      upnp_.reset();
      return;
    }
    std::vector<NatMapping> maps;
    for (int port : tcp_ports()) {
      NatMapping m;
      if (upnp_->map_tcp(port, port, 3600, &m)) {
        maps.push_back(m);
        advertise("UPnP", ext, port, m);
      }
    }
    upnp_->keep_alive(maps);
  }
}

void Node::stop() {
  std::lock_guard<std::mutex> lk(stop_mu_);
  if (stopping_.exchange(true)) return;
  if (nat_) nat_->stop();  // before http_.stop(): that releases wait() and main may exit
  if (upnp_) upnp_->stop();
  http_.stop();
  if (refresher_.joinable()) refresher_.join();
  if (host_) host_->close();
  kad_.reset();  // after close(): no identify/handler thread can reach it any more
}

static Json err(const std::string& e) {
  Json j = Json::object();
  j.set("error", e);
  return j;
}

std::pair<int, Json> Node::send(const std::string& to, const std::string& content) {
  std::string pid_s;
  std::vector<std::string> addr_s;
  try {
    dir_->lookup(to, &pid_s, &addr_s);
  } catch (...) {
    n_send_fail_++;
    return {404, err("user not found")};
  }
  PeerId pid;
  try {
    pid = PeerId::decode(pid_s);
  } catch (...) {
    n_send_fail_++;
    return {400, err("bad peer id")};
  }
  std::vector<Multiaddr> addrs;
  for (auto& a : addr_s) {
    try {
      addrs.push_back(Multiaddr::parse(a));
    } catch (...) {
    }
  }
  const int kTimeout = 5000;  // one 5 s context for connect + stream + write (`:235`)
  auto t0 = std::chrono::steady_clock::now();
  try {
    if (pid != host_->id()) host_->connect(pid, addrs, kTimeout);  // errors ignored (`:243`)
  } catch (...) {
  }
  int left = kTimeout - (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::steady_clock::now() - t0)
                            .count();
  StreamCtx s;
  try {
    if (pid == host_->id()) throw NetError("failed to dial: dial to self attempted");
    if (!host_->connected(pid)) throw NetError("failed to dial " + pid.to_base58() + ": no good addresses");
    s = host_->new_stream(pid, kChatProto, std::max(left, 500));
  } catch (const std::exception& e) {
    n_send_fail_++;
    return {500, err(std::string("open stream failed: ") + e.what())};
  }
  ChatMessage m;
  m.id = uuid4();
  m.from_user = cfg_.username;
  m.to_user = to;
  m.content = content;
  m.timestamp = rfc3339_now_local();
  try {
    s.io->write_all(m.to_json().dump());
  } catch (const std::exception& e) {
    s.stream->reset();
    n_send_fail_++;
    return {500, err(std::string("write failed: ") + e.what())};
  }
  s.stream->close();
  n_sent_++;
  Json ok = Json::object();
  ok.set("status", "sent");
  ok.set("id", m.id);
  return {200, ok};
}

Json Node::generate(const Json& req) {
  GenerateHook h;
  {
    std::lock_guard<std::mutex> lk(hook_mu_);
    h = hook_;
  }
  n_suggest_++;
  if (h) return h(req);
  if (!cfg_.engine_url.empty()) {
    HttpResult r = http_request("POST", cfg_.engine_url + "/api/generate", req.dump(),
                                "application/json", 60000);
    if (r.status != 200) throw NetError("engine returned " + std::to_string(r.status));
    return Json::parse(r.body);
  }
  throw NetError("no LLM engine attached (run the node through p2p_llm_chat_go_amd.net.node "
                 "or set ENGINE_URL)");
}

Json Node::metrics_json() {
  Json j = Json::object();
  j.set("messages_sent_total", (long)n_sent_);
  j.set("messages_received_total", (long)n_recv_);
  j.set("send_failures_total", (long)n_send_fail_);
  j.set("suggest_requests_total", (long)n_suggest_);
  j.set("inbox_size", (long)inbox_.size());
  j.set("connected_peers", (long)(host_ ? host_->peers().size() : 0));
  j.set("connections_trimmed_total", (long)(host_ ? host_->trimmed() : 0));
  if (host_) {
    const Json rc = host_->resources().stats();
    for (auto& kv : rc.fields()) j.set("rcmgr_" + kv.first, kv.second);
  }
  return j;
}

static const char* kSuggestTemplate =
    "You are a helpful assistant. Draft a concise, friendly reply to the following message:\n\n"
    "%s\n\nReply:";

void Node::install_routes() {
  http_.route("POST", "/send", [this](const HttpRequest& req, HttpResponse& res) {
    std::string to, content;
    try {
      Json j = Json::parse(req.body);
      if (!j.is_object()) throw JsonError("json: cannot unmarshal " + go_type(j) +
                                          " into Go value of type main.SendBody");
      to = str_field(j, "to_username", "SendBody");
      content = str_field(j, "content", "SendBody");
    } catch (const std::exception& e) {
      res.json(400, err(bind_error(req.body, e)), true);
      return;
    }
    auto r = send(to, content);
    res.json(r.first, r.second, true);
  });
  http_.route("GET", "/inbox", [this](const HttpRequest& req, HttpResponse& res) {
    Json arr = Json::array();
    for (auto& m : inbox_.drain(req.param("after"))) arr.push(m.to_json());
    res.json(200, arr);
  });
  http_.route("GET", "/me", [this](const HttpRequest&, HttpResponse& res) {
    // NOTE: the reference returns string(h.ID()) (raw multihash bytes); base58 here.
    Json j = Json::object();
    j.set("username", cfg_.username);
    j.set("peer_id", host_->id().to_base58());
    j.set("addrs", Json::array_of(addrs_));
    res.json(200, j, true);
  });
  // ---- superset: LLM co-pilot endpoints served by the in-process engine ----
  http_.route("POST", "/api/generate", [this](const HttpRequest& req, HttpResponse& res) {
    Json j;
    try {
      j = Json::parse(req.body);
    } catch (const std::exception& e) {
      res.json(400, err(e.what()), true);
      return;
    }
    bool stream = j.get_bool("stream", true);  // Ollama default: streaming
    GenerateStreamHook sh;
    {
      std::lock_guard<std::mutex> lk(hook_mu_);
      sh = stream_hook_;
    }
    if (stream && sh) {  // token-by-token NDJSON from the in-process engine
      n_suggest_++;
      res.set_header("Content-Type", "application/x-ndjson");
      res.stream = [sh, j](const std::function<bool(const std::string&)>& w) {
        try {
          Json fin = sh(j, [&](const Json& c) { return w(c.dump() + "\n"); });
          w(fin.dump() + "\n");
        } catch (const std::exception& e) {
          w(err(e.what()).dump() + "\n");
        }
      };
      return;
    }
    Json out;
    try {
      out = generate(j);
    } catch (const std::exception& e) {
      res.json(500, err(e.what()), true);
      return;
    }
    if (!stream) {
      res.json(200, out);
      return;
    }
    res.set_header("Content-Type", "application/x-ndjson");
    res.stream = [out](const std::function<bool(const std::string&)>& w) {
      Json first = Json::object();
      first.set("model", out.get_string("model"));
      first.set("created_at", out.get_string("created_at"));
      first.set("response", out.get_string("response"));
      first.set("done", false);
      if (!w(first.dump() + "\n")) return;
      Json last = out;
      last.set("response", "");
      w(last.dump() + "\n");
    };
  });
  http_.route("POST", "/api/chat", [this](const HttpRequest& req, HttpResponse& res) {
    Json j;
    try {
      j = Json::parse(req.body);
      j.set("endpoint", "chat");
      GenerateStreamHook sh;
      {
        std::lock_guard<std::mutex> lk(hook_mu_);
        sh = stream_hook_;
      }
      if (j.get_bool("stream", true) && sh) {
        n_suggest_++;
        res.set_header("Content-Type", "application/x-ndjson");
        res.stream = [sh, j](const std::function<bool(const std::string&)>& w) {
          try {
            Json fin = sh(j, [&](const Json& c) { return w(c.dump() + "\n"); });
            w(fin.dump() + "\n");
          } catch (const std::exception& e) {
            w(err(e.what()).dump() + "\n");
          }
        };
        return;
      }
      Json out = generate(j);
      res.json(200, out);
    } catch (const std::exception& e) {
      res.json(500, err(e.what()), true);
    }
  });
  http_.route("GET", "/api/tags", [this](const HttpRequest&, HttpResponse& res) {
    Json m = Json::object();
    m.set("name", cfg_.llm_model + ":latest");
    m.set("model", cfg_.llm_model + ":latest");
    Json arr = Json::array();
    arr.push(m);
    Json j = Json::object();
    j.set("models", arr);
    res.json(200, j);
  });
  http_.route("POST", "/suggest", [this](const HttpRequest& req, HttpResponse& res) {
    // {"id": "<inbox message id>"} or {"message": "..."}; optional "send": true replies
    // to the original sender (the UI's "Send AI reply" button, web/streamlit_app.py:175-190).
    Json j;
    try {
      j = Json::parse(req.body.empty() ? "{}" : req.body);
    } catch (const std::exception& e) {
      res.json(400, err(e.what()), true);
      return;
    }
    std::string text = j.get_string("message");
    std::string reply_to;
    if (text.empty() && !j.get_string("id").empty()) {
      for (auto& m : inbox_.drain("")) {
        if (m.id == j.get_string("id")) {
          text = m.content;
          reply_to = m.from_user;
        }
      }
      if (text.empty()) {
        res.json(404, err("message not found"), true);
        return;
      }
    }
    std::string prompt = kSuggestTemplate;  // "...message:\n\n%s\n\nReply:" (no length cap)
    const size_t ph = prompt.find("%s");
    if (ph != std::string::npos) prompt.replace(ph, 2, text);
    Json g = Json::object();
    g.set("model", j.get_string("model", cfg_.llm_model));
    g.set("prompt", prompt);
    g.set("stream", false);
    if (j.has("options")) g.set("options", j.get("options"));
    Json out;
    try {
      out = generate(g);
    } catch (const std::exception& e) {
      res.json(503, err(std::string("LLM unavailable: ") + e.what()), true);
      return;
    }
    std::string sug = out.get_string("response");
    size_t a = sug.find_first_not_of(" \t\r\n"), b = sug.find_last_not_of(" \t\r\n");
    sug = a == std::string::npos ? "" : sug.substr(a, b - a + 1);
    Json r = Json::object();
    r.set("suggestion", sug);
    for (auto* k : {"eval_count", "eval_duration", "prompt_eval_count", "prompt_eval_duration",
                    "total_duration"})
      if (out.has(k)) r.set(k, out.get(k));
    if (j.get_bool("send", false) && !reply_to.empty()) {
      auto s = send(reply_to, sug);
      r.set("sent", s.first == 200);
      if (s.first == 200) r.set("sent_id", s.second.get_string("id"));
    }
    res.json(200, r);
  });
  http_.route("GET", "/peers", [this](const HttpRequest&, HttpResponse& res) {
    Json arr = Json::array();
    for (auto& p : host_->peers()) {
      Json e = Json::object();
      e.set("peer_id", p.to_base58());
      e.set("agent", host_->peer_agent(p));
      e.set("transport", host_->peer_transport(p));
      Json pr = Json::array();
      for (auto& x : host_->peer_protocols(p)) pr.push(x);
      e.set("protocols", pr);
      arr.push(e);
    }
    res.json(200, arr);
  });
  // DHT (superset of the reference API): routing table and peer lookup
  http_.route("GET", "/dht/peers", [this](const HttpRequest&, HttpResponse& res) {
    Json arr = Json::array();
    if (kad_) {
      for (auto& p : kad_->closest(kad_key(host_->id().bytes()), 1 << 20)) {
        Json e = Json::object();
        e.set("peer_id", p.id.to_base58());
        Json a = Json::array();
        for (auto& x : p.addrs) a.push(x.str());
        e.set("addrs", a);
        arr.push(e);
      }
    }
    res.json(200, arr);
  });
  http_.route("GET", "/dht/find", [this](const HttpRequest& req, HttpResponse& res) {
    if (!kad_) {
      res.json(503, err("dht disabled"));
      return;
    }
    PeerId target;
    try {
      target = PeerId::decode(req.param("peer"));
    } catch (...) {
      res.json(400, err("bad peer id"));
      return;
    }
    std::vector<Multiaddr> addrs;
    if (!kad_->find_peer(target, &addrs, 5000)) {
      res.json(404, err("peer not found"));
      return;
    }
    Json j = Json::object();
    j.set("peer_id", target.to_base58());
    Json a = Json::array();
    for (auto& x : addrs) a.push(x.str());
    j.set("addrs", a);
    res.json(200, j);
  });
  http_.route("GET", "/health", [](const HttpRequest&, HttpResponse& res) {
    Json j = Json::object();
    j.set("ok", true);
    res.json(200, j, true);
  });
  if (!cfg_.ui_file.empty()) {
    auto ui = [this](const HttpRequest&, HttpResponse& res) {
      std::ifstream f(cfg_.ui_file);
      if (!f) {
        res.text(404, "ui not found");
        return;
      }
      std::stringstream ss;
      ss << f.rdbuf();
      res.status = 200;
      res.body = ss.str();
      res.set_header("Content-Type", "text/html; charset=utf-8");
    };
    http_.route("GET", "/", ui);
    http_.route("GET", "/ui", ui);
  }
  http_.route("GET", "/metrics", [this](const HttpRequest&, HttpResponse& res) {
    std::string out;
    Json m = metrics_json();
    GenerateHook h;
    {
      std::lock_guard<std::mutex> lk(hook_mu_);
      h = hook_;
    }
    if (h) {
      try {
        Json q = Json::object();
        q.set("endpoint", "metrics");
        Json e = h(q);
        for (auto& kv : e.fields()) m.set("engine_" + kv.first, kv.second);
      } catch (...) {
      }
    }
    for (auto& kv : m.fields()) {
      if (!kv.second.is_number()) continue;
      out += "p2p_" + kv.first + " " + kv.second.dump() + "\n";
    }
    res.status = 200;
    res.body = out;
    res.set_header("Content-Type", "text/plain; version=0.0.4");
  });
}

}  // namespace p2p
