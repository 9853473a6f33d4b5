#include "host.h"
#include "tls.h"

#include <string.h>

#include <algorithm>
#include <chrono>

namespace p2p {

const char* kIdentifyProto = "/ipfs/id/1.0.0";
const char* kPingProto = "/ipfs/ping/1.0.0";
const char* kNoiseProto = "/noise";
const char* kYamuxProto = "/yamux/1.0.0";

static constexpr int kUpgradeTimeoutMs = 10000;

Host::Host(PrivateKey key, std::string agent)
    : key_(std::move(key)), id_(PeerId::from_public_key(key_.public_key())),
      agent_(std::move(agent)),
      rcmgr_(std::make_shared<ResourceManager>(ResourceLimits::from_env())) {
  set_stream_handler(kIdentifyProto, [this](StreamCtx& c) { identify_handler(c); });
  set_stream_handler(kPingProto, [](StreamCtx& c) {
    uint8_t buf[32];
    c.io->set_read_timeout(60000);
    while (true) {
      size_t got = 0;
      while (got < 32) {
        size_t r = c.io->read_some(buf + got, 32 - got);
        if (r == 0) {
          c.stream->close();
          return;
        }
        got += r;
      }
      c.io->write_all(buf, 32);
    }
  });
}

Host::~Host() { close(); }

void Host::close() {
  if (closed_.exchange(true)) return;
  std::vector<std::shared_ptr<TcpListener>> ls;
  std::map<PeerId, SessionPtr> ss;
  {
    std::lock_guard<std::mutex> lk(mu_);
    ls = listeners_;
    ss = sessions_;
  }
  for (auto& l : ls) l->close();
  for (auto& kv : ss) kv.second->close();
  std::shared_ptr<QuicTransport> q;
  {
    std::lock_guard<std::mutex> lk(mu_);
    q = quic_;
  }
  if (q) q->close();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  // let detached reader / handler / identify threads that reference this host finish
  for (int i = 0; i < 500 && busy_.load() > 0; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
}

void Host::listen(const Multiaddr& ma) {
  std::string host;
  int port = 0;
  if (ma.quic_host_port(&host, &port)) {
    std::lock_guard<std::mutex> lk(mu_);
    if (quic_) {
      logf("one QUIC listener per host; skipping %s", ma.str().c_str());
      return;
    }
    quic_ = QuicTransport::create(host, port, key_);
    quic_->set_accept([this](QuicConnPtr c) {
      if (closed_) {
        c->close();
        return;
      }
      Busy b(this);
      try {
        add_session(c->remote_peer(), c, false, true);
      } catch (const std::exception&) {
        c->close();
      }
    });
    listen_addrs_.push_back(
        Multiaddr::parse("/ip4/" + host + "/udp/" + std::to_string(quic_->port()) + "/quic-v1"));
    return;
  }
  if (ma.has(MA_QUIC_V1) || ma.has(MA_QUIC) || ma.has(MA_UDP)) {
    logf("transport not available (only /ip4/.../udp/.../quic-v1 is): %s", ma.str().c_str());
    return;
  }
  if (!ma.tcp_host_port(&host, &port)) throw NetError("listen: unsupported address " + ma.str());
  auto l = std::make_shared<TcpListener>(host, port);
  Multiaddr bound = Multiaddr::parse((host.find(':') != std::string::npos ? "/ip6/" : "/ip4/") +
                                     host + "/tcp/" + std::to_string(l->port()));
  {
    std::lock_guard<std::mutex> lk(mu_);
    listeners_.push_back(l);
    listen_addrs_.push_back(bound);
  }
  threads_.emplace_back([this, l] { accept_loop(l); });
}

std::vector<Multiaddr> Host::addrs() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<Multiaddr> out;
  for (auto& a : listen_addrs_) {
    std::string h;
    int port;
    if (a.tcp_host_port(&h, &port) && (h == "0.0.0.0")) {
      for (auto& ip : local_ipv4_addrs(true))
        out.push_back(Multiaddr::parse("/ip4/" + ip + "/tcp/" + std::to_string(port)));
    } else if (a.quic_host_port(&h, &port) && (h == "0.0.0.0")) {
      for (auto& ip : local_ipv4_addrs(true))
        out.push_back(Multiaddr::parse("/ip4/" + ip + "/udp/" + std::to_string(port) + "/quic-v1"));
    } else {
      out.push_back(a);
    }
  }
  for (auto& a : extra_addrs_) out.push_back(a);
  return out;
}

void Host::add_advertised_addr(const Multiaddr& ma) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& a : extra_addrs_)
    if (a == ma) return;
  extra_addrs_.push_back(ma);
}

void Host::set_stream_handler(const std::string& proto, StreamHandler h) {
  std::lock_guard<std::mutex> lk(mu_);
  handlers_[proto] = std::move(h);
}

void Host::remove_stream_handler(const std::string& proto) {
  std::lock_guard<std::mutex> lk(mu_);
  handlers_.erase(proto);
}

std::vector<std::string> Host::protocols() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  for (auto& kv : handlers_) out.push_back(kv.first);
  return out;
}

void Host::add_addrs(const PeerId& p, const std::vector<Multiaddr>& addrs) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& v = peerstore_[p];
  for (auto& a : addrs) {
    Multiaddr bare = a.without_peer();
    if (bare.has(MA_P2P_CIRCUIT)) bare = a;  // keep the relay's /p2p inside circuit addrs
    bool dup = false;
    for (auto& x : v) dup |= (x == bare);
    if (!dup) v.push_back(bare);
  }
}

std::vector<Multiaddr> Host::peer_addrs(const PeerId& p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = peerstore_.find(p);
  return it == peerstore_.end() ? std::vector<Multiaddr>{} : it->second;
}

std::vector<PeerId> Host::peers() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<PeerId> out;
  for (auto& kv : sessions_)
    if (!kv.second->closed()) out.push_back(kv.first);
  return out;
}

bool Host::connected(const PeerId& p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = sessions_.find(p);
  return it != sessions_.end() && !it->second->closed();
}

std::vector<std::string> Host::peer_protocols(const PeerId& p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = peer_protos_.find(p);
  return it == peer_protos_.end() ? std::vector<std::string>{} : it->second;
}

std::string Host::peer_transport(const PeerId& p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = sessions_.find(p);
  if (it == sessions_.end() || it->second->closed()) return "";
  auto t = peer_transport_.find(p);
  return t == peer_transport_.end() ? "" : t->second;
}

std::string Host::peer_agent(const PeerId& p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = peer_agents_.find(p);
  return it == peer_agents_.end() ? "" : it->second;
}

// ------------------------------------------------------------ upgrade
// The secured connection of an upgrade: a Noise or TLS channel, its peer, and the
// muxer TLS already agreed on through ALPN ("" = negotiate it with multistream).
struct Secured {
  ConnPtr conn;
  PeerId peer;
  std::string early_muxer;
};

static Secured secure(const std::string& proto, std::shared_ptr<BufConn> b, const PrivateKey& key,
                      bool initiator, const PeerId& expected) {
  if (proto == kTlsProto) {
    auto t = TlsConn::handshake(b, key, initiator, expected);
    return {t, t->remote_peer(), t->early_muxer()};
  }
  auto n = NoiseConn::handshake(b, key, initiator, expected);
  return {n, n->remote_peer(), ""};
}

void Host::set_security(const std::vector<std::string>& order) {
  std::vector<std::string> ids;
  for (auto& n : order) {
    if (n == "noise" || n == kNoiseProto) ids.push_back(kNoiseProto);
    else if (n == "tls" || n == kTlsProto) ids.push_back(kTlsProto);
    else throw NetError("unknown security transport: " + n);
  }
  if (ids.empty()) throw NetError("no security transport configured");
  security_ = ids;
}

SessionPtr Host::upgrade_outbound(ConnPtr raw, const PeerId& expected, bool relayed) {
  raw->set_read_timeout(kUpgradeTimeoutMs);
  auto b1 = std::make_shared<BufConn>(raw);
  const std::string proto = ms_select_any(*b1, security_);
  Secured sec = secure(proto, b1, key_, true, expected);
  auto b2 = std::make_shared<BufConn>(sec.conn);
  if (sec.early_muxer.empty()) ms_select(*b2, kYamuxProto);
  raw->set_read_timeout(0);
  auto sess = std::make_shared<YamuxSession>(b2, true);
  add_session(sec.peer, sess, relayed, false);
  return sess;
}

SessionPtr Host::upgrade_inbound(ConnPtr raw, bool relayed) {
  raw->set_read_timeout(kUpgradeTimeoutMs);
  auto b1 = std::make_shared<BufConn>(raw);
  const std::string proto =
      ms_handle(*b1, std::set<std::string>(security_.begin(), security_.end()));
  Secured sec = secure(proto, b1, key_, false, PeerId());
  auto b2 = std::make_shared<BufConn>(sec.conn);
  if (sec.early_muxer.empty()) ms_handle(*b2, {kYamuxProto});
  raw->set_read_timeout(0);
  auto sess = std::make_shared<YamuxSession>(b2, false);
  add_session(sec.peer, sess, relayed, true);
  return sess;
}

void Host::set_conn_limits(int low, int high, int grace_ms) {
  std::lock_guard<std::mutex> lk(mu_);
  conn_high_ = std::max(1, high);
  conn_low_ = std::max(0, std::min(low, conn_high_));
  conn_grace_ms_ = std::max(0, grace_ms);
}

void Host::touch(const PeerId& p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = conn_use_.find(p);
  if (it != conn_use_.end()) it->second.used = std::chrono::steady_clock::now();
}

void Host::trim_connections(const PeerId& keep) {
  std::vector<SessionPtr> victims;
  {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<std::pair<std::chrono::steady_clock::time_point, PeerId>> cands;
    int live = 0;
    const auto now = std::chrono::steady_clock::now();
    for (auto& kv : sessions_) {
      if (kv.second->closed()) continue;
      ++live;
      auto u = conn_use_.find(kv.first);
      if (kv.first == keep || u == conn_use_.end() || kv.second->num_streams() > 0) continue;
      if (now - u->second.opened < std::chrono::milliseconds(conn_grace_ms_)) continue;
      cands.push_back({u->second.used, kv.first});
    }
    if (live <= conn_high_) return;
    std::sort(cands.begin(), cands.end());
    for (auto& c : cands) {
      if (live <= conn_low_) break;
      victims.push_back(sessions_[c.second]);
      sessions_.erase(c.second);
      conn_use_.erase(c.second);
      --live;
    }
  }
  for (auto& v : victims) {
    v->close();
    trimmed_++;
  }
}

void Host::add_session(const PeerId& p, SessionPtr s, bool relayed, bool inbound) {
  std::shared_ptr<ResourceManager::Conn> rc = rcmgr_->open_conn(p, inbound);
  if (!rc) {
    s->close();
    throw NetError("resource limit exceeded: connection from/to " + p.to_base58());
  }
  SessionPtr old;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = sessions_.find(p);
    // Prefer a direct connection over a relayed one; otherwise keep the newest.
    if (it != sessions_.end() && !it->second->closed()) old = it->second;
    sessions_[p] = s;
    peer_transport_[p] = relayed ? "p2p-circuit" : (s->transport() == "quic-v1" ? "quic-v1" : "tcp");
    const auto now = std::chrono::steady_clock::now();
    conn_use_[p] = ConnUse{now, now};
  }
  std::weak_ptr<MuxSession> ws = s;
  busy_++;  // released by the session's on_close
  s->start([this, p, relayed](StreamPtr st) {
             Busy b(this);
             handle_stream(st, p, relayed);
           },
           [this, p, ws, rc]() mutable {
             Busy b(this);
             busy_--;
             rc.reset();
             std::lock_guard<std::mutex> lk(mu_);
             auto it = sessions_.find(p);
             auto sp = ws.lock();
             if (it != sessions_.end() && (!sp || it->second == sp)) {
               sessions_.erase(it);
               conn_use_.erase(p);
             }
           });
  (void)old;  // the old session stays usable for its open streams and dies on its own
  trim_connections(p);
  busy_++;
  std::thread([this, p, s] {
    run_identify(p, s);
    busy_--;
  }).detach();
}

void Host::accept_loop(std::shared_ptr<TcpListener> l) {
  while (!closed_) {
    auto c = l->accept();
    if (!c) break;
    busy_++;
    std::thread([this, c] {
      try {
        upgrade_inbound(c, false);
      } catch (const std::exception& e) {
        c->close();
      }
      busy_--;
    }).detach();
  }
}

void Host::handle_stream(StreamPtr s, PeerId peer, bool relayed) {
  touch(peer);
  std::shared_ptr<ResourceManager::Stream> rc = rcmgr_->open_stream(peer, true);
  if (!rc) {  // system / transient / peer scope full
    s->reset();
    return;
  }
  auto io = std::make_shared<BufConn>(s);
  std::set<std::string> protos;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : handlers_) protos.insert(kv.first);
  }
  s->set_read_timeout(kUpgradeTimeoutMs);
  std::string proto;
  try {
    proto = ms_handle(*io, protos);
  } catch (...) {
    s->reset();
    return;
  }
  s->set_read_timeout(0);
  s->protocol = proto;
  StreamHandler h;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = handlers_.find(proto);
    if (it != handlers_.end()) h = it->second;
  }
  if (!h || !rc->set_protocol(proto)) {  // unknown protocol, or its scope is full
    s->reset();
    return;
  }
  StreamCtx ctx{s, io, peer, proto, relayed, rc};
  h(ctx);
}

// ------------------------------------------------------------ identify
// message Identify { bytes publicKey = 1; repeated bytes listenAddrs = 2;
//   repeated string protocols = 3; bytes observedAddr = 4; string protocolVersion = 5;
//   string agentVersion = 6; }
void Host::identify_handler(StreamCtx& c) {
  PbWriter w;
  w.bytes_field(5, std::string("ipfs/0.1.0"));
  w.bytes_field(6, agent_);
  w.bytes_field(1, key_.public_key().marshal());
  for (auto& a : addrs()) w.bytes_field(2, a.bytes());
  std::string host;
  int port = 0;
  std::string ra = c.io->remote_addr();
  size_t colon = ra.rfind(':');
  if (colon != std::string::npos && ra.find(':') == colon) {
    try {
      w.bytes_field(4, Multiaddr::parse("/ip4/" + ra.substr(0, colon) + "/tcp/" +
                                        ra.substr(colon + 1)).bytes());
    } catch (...) {
    }
  }
  (void)host;
  (void)port;
  for (auto& p : protocols()) w.bytes_field(3, p);
  write_frame(*c.io, w.buf);
  c.stream->close();
}

void Host::run_identify(const PeerId& p, SessionPtr s) {
  try {
    StreamPtr st = s->open_stream();
    auto io = std::make_shared<BufConn>(st);
    st->set_read_timeout(kUpgradeTimeoutMs);
    ms_select(*io, kIdentifyProto);
    Bytes msg = io->read_frame(1 << 16);
    st->close();
    std::vector<std::string> protos;
    std::vector<Multiaddr> listen;
    std::string agent;
    for (auto& f : pb_parse(msg)) {
      if (f.field == 3 && f.wire == 2) protos.push_back(to_string(f.bytes));
      if (f.field == 6 && f.wire == 2) agent = to_string(f.bytes);
      if (f.field == 2 && f.wire == 2) {
        try {
          listen.push_back(Multiaddr::from_bytes(f.bytes));
        } catch (...) {
        }
      }
    }
    add_addrs(p, listen);
    decltype(on_identified) cb;
    {
      std::lock_guard<std::mutex> lk(mu_);
      peer_protos_[p] = protos;
      peer_agents_[p] = agent;
      cb = on_identified;
    }
    if (cb) cb(p, protos, listen);
  } catch (...) {
  }
}

// ------------------------------------------------------------ dial
SessionPtr Host::connect(const PeerId& p, const std::vector<Multiaddr>& addrs, int timeout_ms) {
  if (closed_) throw NetError("host closed");
  if (p == id_) throw NetError("dial to self attempted");
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = sessions_.find(p);
    if (it != sessions_.end() && !it->second->closed()) {
      auto u = conn_use_.find(p);
      if (u != conn_use_.end()) u->second.used = std::chrono::steady_clock::now();
      return it->second;
    }
  }
  add_addrs(p, addrs);
  std::vector<Multiaddr> cands = peer_addrs(p);
  // direct addresses first (QUIC ahead of TCP when preferred), then relayed ones
  auto rank = [this](const Multiaddr& a) {
    if (a.has(MA_P2P_CIRCUIT)) return 2;
    return (prefer_quic_ && a.has(MA_QUIC_V1)) ? 0 : 1;
  };
  std::stable_sort(cands.begin(), cands.end(),
                   [&](const Multiaddr& a, const Multiaddr& b) { return rank(a) < rank(b); });
  if (cands.empty()) throw NetError("no addresses");
  std::string errs;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  for (auto& a : cands) {
    int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                   deadline - std::chrono::steady_clock::now())
                   .count();
    if (left <= 0) break;
    try {
      Multiaddr relay, target;
      if (a.split_circuit(&relay, &target)) {
        if (!relay_dialer) throw NetError("no relay transport");
        return relay_dialer(relay, p, left);
      }
      std::string h;
      int port;
      if (a.quic_host_port(&h, &port)) {
        auto c = quic_for_dial()->dial(h, port, p, std::min(left, 5000));
        add_session(p, c, false, false);
        return c;
      }
      if (!a.tcp_host_port(&h, &port)) {
        errs += " [" + a.str() + ": unsupported transport]";
        continue;
      }
      auto c = TcpConn::dial(h, port, std::min(left, 5000));
      try {
        return upgrade_outbound(c, p, false);
      } catch (...) {
        c->close();
        throw;
      }
    } catch (const std::exception& e) {
      errs += " [" + a.str() + ": " + e.what() + "]";
    }
  }
  throw NetError("failed to dial " + p.to_base58() + ":" + errs);
}

std::shared_ptr<QuicTransport> Host::quic_for_dial() {
  std::lock_guard<std::mutex> lk(mu_);
  // dial from the listening socket (one 4-tuple per peer, NAT-friendly like
  // go-libp2p's reuse); a host without a QUIC listener gets a dial-only socket
  if (!quic_) quic_ = QuicTransport::create("0.0.0.0", 0, key_);
  return quic_;
}

StreamCtx Host::new_stream(const PeerId& p, const std::string& proto, int timeout_ms) {
  SessionPtr s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = sessions_.find(p);
    if (it != sessions_.end() && !it->second->closed()) s = it->second;
  }
  if (!s) {
    if (p == id_) throw NetError("failed to dial: dial to self attempted");
    s = connect(p, {}, timeout_ms);
  }
  std::shared_ptr<ResourceManager::Stream> rc = rcmgr_->open_stream(p, false);
  if (!rc) throw NetError("resource limit exceeded: outbound stream to " + p.to_base58());
  StreamPtr st = s->open_stream();
  auto io = std::make_shared<BufConn>(st);
  st->set_read_timeout(timeout_ms);
  try {
    ms_select(*io, proto);
  } catch (...) {
    st->reset();
    throw;
  }
  st->set_read_timeout(0);
  st->protocol = proto;
  rc->set_protocol(proto);
  return StreamCtx{st, io, p, proto, false, rc};
}

long Host::ping(const PeerId& p, int timeout_ms) {
  StreamCtx c = new_stream(p, kPingProto, timeout_ms);
  uint8_t b[32], r[32];
  random_bytes(b, 32);
  auto t0 = std::chrono::steady_clock::now();
  c.io->write_all(b, 32);
  c.io->set_read_timeout(timeout_ms);
  c.io->read_exact(r, 32);
  long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(
                std::chrono::steady_clock::now() - t0)
                .count();
  c.stream->close();
  if (memcmp(b, r, 32) != 0) throw NetError("ping: payload mismatch");
  return us;
}

}  // namespace p2p
