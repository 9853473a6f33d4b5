#include "multiaddr.h"

#include <arpa/inet.h>
#include <string.h>

#include <sstream>

namespace p2p {

namespace {
struct Proto {
  uint32_t code;
  const char* name;
  int size;  // bits; -1 = length-prefixed; 0 = no value
};
const Proto kProtos[] = {
    {MA_IP4, "ip4", 32},        {MA_TCP, "tcp", 16},       {MA_UDP, "udp", 16},
    {MA_IP6, "ip6", 128},       {MA_DNS, "dns", -1},       {MA_DNS4, "dns4", -1},
    {MA_DNS6, "dns6", -1},      {MA_P2P, "p2p", -1},       {MA_P2P_CIRCUIT, "p2p-circuit", 0},
    {MA_QUIC, "quic", 0},       {MA_QUIC_V1, "quic-v1", 0}, {MA_WS, "ws", 0},
    {MA_WSS, "wss", 0},         {MA_TLS, "tls", 0},        {MA_NOISE, "noise", 0},
};
const Proto* by_name(const std::string& n) {
  if (n == "ipfs") return by_name("p2p");
  for (auto& p : kProtos)
    if (n == p.name) return &p;
  return nullptr;
}
const Proto* by_code(uint32_t c) {
  for (auto& p : kProtos)
    if (c == p.code) return &p;
  return nullptr;
}

Bytes value_from_string(const Proto* p, const std::string& v) {
  switch (p->code) {
    case MA_IP4: {
      Bytes b(4);
      if (inet_pton(AF_INET, v.c_str(), b.data()) != 1) throw NetError("multiaddr: bad ip4 " + v);
      return b;
    }
    case MA_IP6: {
      Bytes b(16);
      if (inet_pton(AF_INET6, v.c_str(), b.data()) != 1) throw NetError("multiaddr: bad ip6 " + v);
      return b;
    }
    case MA_TCP:
    case MA_UDP: {
      char* end = nullptr;
      long port = strtol(v.c_str(), &end, 10);
      if (v.empty() || *end || port < 0 || port > 65535) throw NetError("multiaddr: bad port " + v);
      return Bytes{(uint8_t)(port >> 8), (uint8_t)port};
    }
    case MA_P2P:
      return PeerId::decode(v).bytes();
    default:
      return to_bytes(v);  // dns*
  }
}

std::string value_to_string(const Proto* p, const Bytes& b) {
  char buf[64];
  switch (p->code) {
    case MA_IP4:
      inet_ntop(AF_INET, b.data(), buf, sizeof(buf));
      return buf;
    case MA_IP6:
      inet_ntop(AF_INET6, b.data(), buf, sizeof(buf));
      return buf;
    case MA_TCP:
    case MA_UDP:
      return std::to_string((b[0] << 8) | b[1]);
    case MA_P2P:
      return base58_encode(b);
    default:
      return to_string(b);
  }
}
}  // namespace

Multiaddr Multiaddr::parse(const std::string& s) {
  if (s.empty() || s[0] != '/') throw NetError("multiaddr: must start with '/': " + s);
  std::vector<std::string> toks;
  std::stringstream ss(s.substr(1));
  std::string t;
  while (std::getline(ss, t, '/')) toks.push_back(t);
  if (!toks.empty() && toks.back().empty()) toks.pop_back();
  Multiaddr m;
  for (size_t i = 0; i < toks.size(); ++i) {
    const Proto* p = by_name(toks[i]);
    if (!p) throw NetError("multiaddr: unknown protocol " + toks[i]);
    MaComponent c{p->code, {}};
    if (p->size != 0) {
      if (++i >= toks.size()) throw NetError("multiaddr: missing value for " + std::string(p->name));
      c.value = value_from_string(p, toks[i]);
    }
    m.parts_.push_back(std::move(c));
  }
  if (m.parts_.empty()) throw NetError("multiaddr: empty");
  return m;
}

Multiaddr Multiaddr::from_bytes(const Bytes& b) {
  Multiaddr m;
  size_t pos = 0;
  while (pos < b.size()) {
    uint32_t code = (uint32_t)get_uvarint(b, &pos);
    const Proto* p = by_code(code);
    if (!p) throw NetError("multiaddr: unknown code " + std::to_string(code));
    MaComponent c{code, {}};
    size_t n = 0;
    if (p->size > 0) n = (size_t)p->size / 8;
    else if (p->size < 0) n = (size_t)get_uvarint(b, &pos);
    if (pos + n > b.size()) throw NetError("multiaddr: truncated");
    c.value.assign(b.begin() + pos, b.begin() + pos + n);
    pos += n;
    m.parts_.push_back(std::move(c));
  }
  return m;
}

std::string Multiaddr::str() const {
  std::string out;
  for (auto& c : parts_) {
    const Proto* p = by_code(c.code);
    out += "/";
    out += p ? p->name : "?";
    if (p && p->size != 0) {
      out += "/";
      out += value_to_string(p, c.value);
    }
  }
  return out;
}

Bytes Multiaddr::bytes() const {
  Bytes out;
  for (auto& c : parts_) {
    put_uvarint(out, c.code);
    const Proto* p = by_code(c.code);
    if (p && p->size < 0) put_uvarint(out, c.value.size());
    append(out, c.value);
  }
  return out;
}

Multiaddr Multiaddr::encapsulate(const Multiaddr& o) const {
  Multiaddr m = *this;
  m.parts_.insert(m.parts_.end(), o.parts_.begin(), o.parts_.end());
  return m;
}

Multiaddr Multiaddr::with_peer(const PeerId& id) const {
  Multiaddr m = *this;
  m.parts_.push_back({MA_P2P, id.bytes()});
  return m;
}

Multiaddr Multiaddr::without_peer(PeerId* id) const {
  Multiaddr m = *this;
  if (!m.parts_.empty() && m.parts_.back().code == MA_P2P) {
    if (id) *id = PeerId::from_bytes(m.parts_.back().value);
    m.parts_.pop_back();
  }
  return m;
}

bool Multiaddr::has(uint32_t code) const {
  for (auto& c : parts_)
    if (c.code == code) return true;
  return false;
}

bool Multiaddr::split_circuit(Multiaddr* relay, Multiaddr* target) const {
  for (size_t i = 0; i < parts_.size(); ++i) {
    if (parts_[i].code == MA_P2P_CIRCUIT) {
      relay->parts_.assign(parts_.begin(), parts_.begin() + i);
      target->parts_.assign(parts_.begin() + i + 1, parts_.end());
      return true;
    }
  }
  return false;
}

bool Multiaddr::tcp_host_port(std::string* host, int* port) const {
  if (parts_.size() < 2) return false;
  const auto& a = parts_[0];
  const auto& b = parts_[1];
  if (b.code != MA_TCP) return false;
  const Proto* p = by_code(a.code);
  if (!p) return false;
  if (a.code == MA_IP4 || a.code == MA_IP6 || a.code == MA_DNS || a.code == MA_DNS4 ||
      a.code == MA_DNS6) {
    *host = value_to_string(p, a.value);
    *port = (b.value[0] << 8) | b.value[1];
    return true;
  }
  return false;
}

bool Multiaddr::quic_host_port(std::string* host, int* port) const {
  if (parts_.size() < 3 || parts_[0].code != MA_IP4 || parts_[1].code != MA_UDP ||
      parts_[2].code != MA_QUIC_V1)
    return false;
  *host = value_to_string(by_code(MA_IP4), parts_[0].value);
  *port = (parts_[1].value[0] << 8) | parts_[1].value[1];
  return true;
}

}  // namespace p2p
