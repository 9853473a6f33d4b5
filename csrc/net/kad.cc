// Minimal Kademlia DHT (see kad.h).  Wire format: each request/response is
// one uvarint-length-prefixed protobuf `Message` on a `/ipfs/kad/1.0.0`
// stream; a requester may send several requests on one stream.
#include "kad.h"

#include <algorithm>
#include <chrono>
#include <set>

namespace p2p {

const char* kKadProto = "/ipfs/kad/1.0.0";

static constexpr size_t kMaxMsg = 4 << 20;
static constexpr size_t kMaxValues = 4096;

// --------------------------------------------------------------- codec
static Bytes encode_peer(const KadPeer& p) {
  PbWriter w;
  w.bytes_field(1, p.id.bytes());
  for (auto& a : p.addrs) w.bytes_field(2, a.bytes());
  if (p.connection) w.varint_field(3, (uint64_t)p.connection);
  return w.buf;
}

static bool decode_peer(const Bytes& b, KadPeer* out) {
  KadPeer p;
  for (auto& f : pb_parse(b)) {
    if (f.field == 1 && f.wire == 2) {
      try {
        p.id = PeerId::from_bytes(f.bytes);
      } catch (...) {
        return false;
      }
    } else if (f.field == 2 && f.wire == 2) {
      try {
        p.addrs.push_back(Multiaddr::from_bytes(f.bytes));
      } catch (...) {
      }
    } else if (f.field == 3 && f.wire == 0) {
      p.connection = (int)f.varint;
    }
  }
  if (p.id.empty()) return false;
  *out = std::move(p);
  return true;
}

Bytes KadMessage::encode() const {
  PbWriter w;
  w.varint_field(1, (uint64_t)type);
  if (!key.empty()) w.bytes_field(2, key);
  if (has_record) {
    PbWriter r;
    r.bytes_field(1, record_key);
    r.bytes_field(2, record_value);
    w.bytes_field(3, r.buf);
  }
  for (auto& p : closer) w.bytes_field(8, encode_peer(p));
  for (auto& p : providers) w.bytes_field(9, encode_peer(p));
  return w.buf;
}

KadMessage KadMessage::decode(const Bytes& b) {
  KadMessage m;
  m.type = 0;
  for (auto& f : pb_parse(b)) {
    if (f.field == 1 && f.wire == 0) {
      m.type = (int)f.varint;
    } else if (f.field == 2 && f.wire == 2) {
      m.key = f.bytes;
    } else if (f.field == 3 && f.wire == 2) {
      m.has_record = true;
      for (auto& r : pb_parse(f.bytes)) {
        if (r.field == 1 && r.wire == 2) m.record_key = r.bytes;
        if (r.field == 2 && r.wire == 2) m.record_value = r.bytes;
      }
    } else if ((f.field == 8 || f.field == 9) && f.wire == 2) {
      KadPeer p;
      if (decode_peer(f.bytes, &p)) (f.field == 8 ? m.closer : m.providers).push_back(std::move(p));
    }
  }
  return m;
}

// --------------------------------------------------------------- keyspace
Bytes kad_key(const Bytes& raw) { return sha256(raw); }

int kad_common_prefix_len(const Bytes& a, const Bytes& b) {
  for (size_t i = 0; i < a.size() && i < b.size(); ++i) {
    uint8_t x = a[i] ^ b[i];
    if (x) return (int)i * 8 + __builtin_clz((unsigned)x) - 24;
  }
  return (int)std::min(a.size(), b.size()) * 8;
}

bool kad_closer(const Bytes& t, const Bytes& a, const Bytes& b) {
  for (size_t i = 0; i < t.size(); ++i) {
    uint8_t da = a[i] ^ t[i], db = b[i] ^ t[i];
    if (da != db) return da < db;
  }
  return false;
}

// --------------------------------------------------------------- Kad
Kad::Kad(std::shared_ptr<Host> host, KadMode mode)
    : host_(std::move(host)), mode_(mode), self_key_(kad_key(host_->id().bytes())), buckets_(257) {
  if (mode_ == KadMode::Off) return;
  if (mode_ == KadMode::Server)
    host_->set_stream_handler(kKadProto, [this](StreamCtx& c) { handle(c); });
  host_->on_identified = [this](const PeerId& p, const std::vector<std::string>& protos,
                                const std::vector<Multiaddr>& addrs) {
    if (std::find(protos.begin(), protos.end(), kKadProto) != protos.end()) add_peer(p, addrs);
  };
}

Kad::~Kad() {
  if (mode_ == KadMode::Server) host_->remove_stream_handler(kKadProto);
}

bool Kad::add_peer(const PeerId& p, const std::vector<Multiaddr>& addrs) {
  if (p == host_->id() || p.empty()) return false;
  Bytes k = kad_key(p.bytes());
  int cpl = kad_common_prefix_len(self_key_, k);
  std::lock_guard<std::mutex> lk(mu_);
  auto& b = buckets_[cpl];
  for (auto it = b.begin(); it != b.end(); ++it) {
    if (it->id == p) {
      KadPeer e = *it;
      if (!addrs.empty()) e.addrs = addrs;
      b.erase(it);
      b.push_back(std::move(e));  // most recently seen last
      return true;
    }
  }
  if ((int)b.size() >= K) return false;  // full bucket: keep the long-lived entries
  b.push_back(KadPeer{p, addrs, 0});
  return true;
}

void Kad::remove_peer(const PeerId& p) {
  int cpl = kad_common_prefix_len(self_key_, kad_key(p.bytes()));
  std::lock_guard<std::mutex> lk(mu_);
  auto& b = buckets_[cpl];
  b.erase(std::remove_if(b.begin(), b.end(), [&](const KadPeer& e) { return e.id == p; }), b.end());
}

size_t Kad::size() {
  std::lock_guard<std::mutex> lk(mu_);
  size_t n = 0;
  for (auto& b : buckets_) n += b.size();
  return n;
}

std::vector<KadPeer> Kad::closest(const Bytes& key, int n, const PeerId* exclude) {
  std::vector<std::pair<Bytes, KadPeer>> all;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& b : buckets_)
      for (auto& e : b)
        if (!exclude || e.id != *exclude) all.push_back({kad_key(e.id.bytes()), e});
  }
  std::sort(all.begin(), all.end(),
            [&](const auto& x, const auto& y) { return kad_closer(key, x.first, y.first); });
  std::vector<KadPeer> out;
  for (int i = 0; i < (int)all.size() && i < n; ++i) {
    KadPeer p = all[i].second;
    p.connection = host_->connected(p.id) ? 1 : 0;
    out.push_back(std::move(p));
  }
  return out;
}

void Kad::put_local(const Bytes& key, const Bytes& value) {
  std::lock_guard<std::mutex> lk(mu_);
  if (values_.size() >= kMaxValues && !values_.count(key)) return;
  values_[key] = value;
}

bool Kad::get_local(const Bytes& key, Bytes* value) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = values_.find(key);
  if (it == values_.end()) return false;
  *value = it->second;
  return true;
}

KadMessage Kad::respond(const KadMessage& req, const PeerId& from) {
  KadMessage r;
  r.type = req.type;
  r.key = req.key;
  switch (req.type) {
    case KadMessage::PING:
      break;
    case KadMessage::FIND_NODE:
      r.closer = closest(kad_key(req.key), K, &from);
      break;
    case KadMessage::PUT_VALUE:
      if (req.has_record) put_local(req.record_key.empty() ? req.key : req.record_key,
                                    req.record_value);
      r.has_record = req.has_record;
      r.record_key = req.record_key;
      r.record_value = req.record_value;
      break;
    case KadMessage::GET_VALUE: {
      Bytes v;
      if (get_local(req.key, &v)) {
        r.has_record = true;
        r.record_key = req.key;
        r.record_value = v;
      }
      r.closer = closest(kad_key(req.key), K, &from);
      break;
    }
    case KadMessage::ADD_PROVIDER: {
      std::lock_guard<std::mutex> lk(mu_);
      auto& v = providers_[req.key];
      for (auto& p : req.providers)
        if (p.id == from && v.size() < (size_t)K) v.push_back(p);  // only self-announcements
      break;
    }
    case KadMessage::GET_PROVIDERS: {
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = providers_.find(req.key);
        if (it != providers_.end()) r.providers = it->second;
      }
      r.closer = closest(kad_key(req.key), K, &from);
      break;
    }
    default:
      throw NetError("kad: unknown message type");
  }
  return r;
}

void Kad::handle(StreamCtx& c) {
  c.io->set_read_timeout(60000);
  // the requester is reachable: remember it (server-side table refresh)
  add_peer(c.peer, host_->peer_addrs(c.peer));
  try {
    for (;;) {
      Bytes msg = c.io->read_frame(kMaxMsg);
      KadMessage r = respond(KadMessage::decode(msg), c.peer);
      write_frame(*c.io, r.encode());
    }
  } catch (...) {
  }
  c.stream->close();
}

KadMessage Kad::request(const PeerId& peer, const KadMessage& m, int timeout_ms) {
  StreamCtx c = host_->new_stream(peer, kKadProto, timeout_ms);
  try {
    write_frame(*c.io, m.encode());
    c.io->set_read_timeout(timeout_ms);
    Bytes resp = c.io->read_frame(kMaxMsg);
    c.stream->close();
    return KadMessage::decode(resp);
  } catch (...) {
    c.stream->reset();
    throw;
  }
}

std::vector<KadPeer> Kad::find_node(const PeerId& peer, const Bytes& key, int timeout_ms) {
  KadMessage m;
  m.type = KadMessage::FIND_NODE;
  m.key = key;
  KadMessage r = request(peer, m, timeout_ms);
  if (r.type != KadMessage::FIND_NODE) throw NetError("kad: unexpected response type");
  return r.closer;
}

bool Kad::ping(const PeerId& peer, int timeout_ms) {
  KadMessage m;
  m.type = KadMessage::PING;
  try {
    return request(peer, m, timeout_ms).type == KadMessage::PING;
  } catch (...) {
    return false;
  }
}

std::vector<KadPeer> Kad::lookup(const Bytes& raw_key, int timeout_ms) {
  const Bytes target = kad_key(raw_key);
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  std::map<PeerId, KadPeer> known;
  std::set<PeerId> queried, failed;
  for (auto& p : closest(target, K)) known[p.id] = p;
  auto by_distance = [&]() {
    std::vector<KadPeer> v;
    for (auto& kv : known)
      if (!failed.count(kv.first)) v.push_back(kv.second);
    std::sort(v.begin(), v.end(), [&](const KadPeer& a, const KadPeer& b) {
      return kad_closer(target, kad_key(a.id.bytes()), kad_key(b.id.bytes()));
    });
    if ((int)v.size() > K) v.resize(K);
    return v;
  };
  for (;;) {
    if (std::chrono::steady_clock::now() > deadline) break;
    std::vector<KadPeer> batch;
    for (auto& p : by_distance()) {
      if (!queried.count(p.id) && p.id != host_->id()) batch.push_back(p);
      if ((int)batch.size() >= ALPHA) break;
    }
    if (batch.empty()) break;  // the K closest known peers have all been queried
    for (auto& p : batch) {
      queried.insert(p.id);
      int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                     deadline - std::chrono::steady_clock::now())
                     .count();
      if (left <= 0) break;
      try {
        host_->connect(p.id, p.addrs, std::min(left, 5000));
        for (auto& q : find_node(p.id, raw_key, std::min(left, 5000))) {
          if (q.id == host_->id()) continue;
          host_->add_addrs(q.id, q.addrs);
          if (!known.count(q.id)) known[q.id] = q;
        }
        add_peer(p.id, p.addrs);
      } catch (...) {
        failed.insert(p.id);
      }
    }
  }
  return by_distance();
}

bool Kad::find_peer(const PeerId& target, std::vector<Multiaddr>* addrs, int timeout_ms) {
  for (auto& p : closest(kad_key(target.bytes()), K)) {
    if (p.id == target && !p.addrs.empty()) {
      *addrs = p.addrs;
      return true;
    }
  }
  for (auto& p : lookup(target.bytes(), timeout_ms)) {
    if (p.id == target) {
      *addrs = p.addrs.empty() ? host_->peer_addrs(target) : p.addrs;
      return !addrs->empty();
    }
  }
  return false;
}

void Kad::bootstrap(int timeout_ms) { lookup(host_->id().bytes(), timeout_ms); }

}  // namespace p2p
