#include "conn.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>

namespace p2p {

// ================================================================ Conn helpers
void Conn::read_exact(uint8_t* buf, size_t n) {
  size_t got = 0;
  while (got < n) {
    size_t r = read_some(buf + got, n - got);
    if (r == 0) throw NetError("unexpected EOF");
    got += r;
  }
}

Bytes Conn::read_all(size_t max) {
  Bytes out;
  uint8_t tmp[16384];
  while (true) {
    size_t r = read_some(tmp, sizeof(tmp));
    if (r == 0) break;
    if (out.size() + r > max) throw NetError("message too large");
    out.insert(out.end(), tmp, tmp + r);
  }
  return out;
}

size_t BufConn::read_some(uint8_t* buf, size_t n) {
  if (!pending_.empty()) {
    size_t k = std::min(n, pending_.size());
    memcpy(buf, pending_.data(), k);
    pending_.erase(pending_.begin(), pending_.begin() + k);
    return k;
  }
  return c_->read_some(buf, n);
}

uint8_t BufConn::read_byte() {
  uint8_t b;
  read_exact(&b, 1);
  return b;
}

uint64_t BufConn::read_uvarint() {
  uint64_t v = 0;
  for (int i = 0, shift = 0; i < 10; ++i, shift += 7) {
    uint8_t b = read_byte();
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return v;
  }
  throw NetError("varint overflow");
}

Bytes BufConn::read_frame(size_t max) {
  uint64_t n = read_uvarint();
  if (n > max) throw NetError("frame too large");
  return read_exact((size_t)n);
}

void write_frame(Conn& c, const Bytes& payload) {
  Bytes b = uvarint(payload.size());
  append(b, payload);
  c.write_all(b);
}

// ================================================================ TCP
TcpConn::TcpConn(int fd, std::string remote) : fd_(fd), own_fd_(fd), remote_(std::move(remote)) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

TcpConn::~TcpConn() {
  close();
  if (own_fd_ >= 0) ::close(own_fd_);
}

static std::string sockaddr_str(const sockaddr* sa) {
  char host[INET6_ADDRSTRLEN] = {0};
  int port = 0;
  if (sa->sa_family == AF_INET) {
    auto* s4 = (const sockaddr_in*)sa;
    inet_ntop(AF_INET, &s4->sin_addr, host, sizeof(host));
    port = ntohs(s4->sin_port);
  } else if (sa->sa_family == AF_INET6) {
    auto* s6 = (const sockaddr_in6*)sa;
    inet_ntop(AF_INET6, &s6->sin6_addr, host, sizeof(host));
    port = ntohs(s6->sin6_port);
  }
  return std::string(host) + ":" + std::to_string(port);
}

std::shared_ptr<TcpConn> TcpConn::dial(const std::string& host, int port, int timeout_ms) {
  addrinfo hints = {}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  std::string ps = std::to_string(port);
  if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw NetError("dial: cannot resolve " + host);
  std::string err = "dial: connection failed";
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int rc = connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p = {fd, POLLOUT, 0};
      rc = poll(&p, 1, timeout_ms > 0 ? timeout_ms : -1);
      if (rc == 1) {
        int so = 0;
        socklen_t sl = sizeof(so);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl);
        rc = so == 0 ? 0 : -1;
        if (so) err = std::string("dial: ") + strerror(so);
      } else {
        rc = -1;
        err = "dial: timeout";
      }
    } else if (rc != 0) {
      err = std::string("dial: ") + strerror(errno);
    }
    if (rc == 0) {
      fcntl(fd, F_SETFL, fl);
      std::string remote = sockaddr_str(ai->ai_addr);
      freeaddrinfo(res);
      return std::make_shared<TcpConn>(fd, remote);
    }
    ::close(fd);
  }
  freeaddrinfo(res);
  throw NetError(err + " (" + host + ":" + ps + ")");
}

size_t TcpConn::read_some(uint8_t* buf, size_t n) {
  while (true) {
    int fd = fd_.load();
    if (fd < 0) return 0;
    if (timeout_ms_ > 0) {
      pollfd p = {fd, POLLIN, 0};
      int rc = poll(&p, 1, timeout_ms_);
      if (rc == 0) throw NetError("read timeout");
      if (rc < 0 && errno != EINTR) throw NetError(std::string("poll: ") + strerror(errno));
      if (rc < 0) continue;
    }
    ssize_t r = recv(fd, buf, n, 0);
    if (r >= 0) return (size_t)r;
    if (errno == EINTR) continue;
    if (errno == ECONNRESET || errno == EBADF || errno == ENOTCONN) return 0;
    throw NetError(std::string("recv: ") + strerror(errno));
  }
}

void TcpConn::write_all(const uint8_t* buf, size_t n) {
  std::lock_guard<std::mutex> lk(wmu_);
  size_t off = 0;
  while (off < n) {
    int fd = fd_.load();
    if (fd < 0) throw NetError("write on closed connection");
    ssize_t w = send(fd, buf + off, n - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw NetError(std::string("send: ") + strerror(errno));
    }
    off += (size_t)w;
  }
}

void TcpConn::close_write() {
  int fd = fd_.load();
  if (fd >= 0) shutdown(fd, SHUT_WR);
}

// shutdown() wakes a thread blocked in recv/send on this socket; the descriptor
// itself stays open until the destructor, so it cannot be reused by another
// socket while that thread still holds the old number.
void TcpConn::close() {
  int fd = fd_.exchange(-1);
  if (fd >= 0) shutdown(fd, SHUT_RDWR);
}

TcpListener::TcpListener(const std::string& host, int port) : fd_(-1), host_(host) {
  addrinfo hints = {}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  std::string ps = std::to_string(port);
  if (getaddrinfo(host.empty() ? nullptr : host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw NetError("listen: cannot resolve " + host);
  int fd = socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    freeaddrinfo(res);
    throw NetError("listen: socket failed");
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (bind(fd, res->ai_addr, res->ai_addrlen) != 0 || ::listen(fd, 128) != 0) {
    std::string e = strerror(errno);
    ::close(fd);
    freeaddrinfo(res);
    throw NetError("listen " + host + ":" + ps + ": " + e);
  }
  freeaddrinfo(res);
  sockaddr_storage ss = {};
  socklen_t sl = sizeof(ss);
  getsockname(fd, (sockaddr*)&ss, &sl);
  port_ = ss.ss_family == AF_INET ? ntohs(((sockaddr_in*)&ss)->sin_port)
                                  : ntohs(((sockaddr_in6*)&ss)->sin6_port);
  own_fd_ = fd;
  fd_ = fd;
}

TcpListener::~TcpListener() {
  close();
  if (own_fd_ >= 0) ::close(own_fd_);
}

std::shared_ptr<TcpConn> TcpListener::accept() {
  while (true) {
    int lfd = fd_.load();
    if (lfd < 0) return nullptr;
    sockaddr_storage ss = {};
    socklen_t sl = sizeof(ss);
    int fd = ::accept4(lfd, (sockaddr*)&ss, &sl, SOCK_CLOEXEC);
    if (fd >= 0) return std::make_shared<TcpConn>(fd, sockaddr_str((sockaddr*)&ss));
    if (errno == EINTR || errno == ECONNABORTED) continue;
    return nullptr;
  }
}

void TcpListener::close() {
  int fd = fd_.exchange(-1);
  if (fd >= 0) shutdown(fd, SHUT_RDWR);  // wakes accept(); the fd is closed by the destructor
}

std::vector<std::string> local_ipv4_addrs(bool include_loopback) {
  std::vector<std::string> out;
  ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return {"127.0.0.1"};
  for (ifaddrs* i = ifa; i; i = i->ifa_next) {
    if (!i->ifa_addr || i->ifa_addr->sa_family != AF_INET) continue;
    char buf[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &((sockaddr_in*)i->ifa_addr)->sin_addr, buf, sizeof(buf));
    std::string s = buf;
    if (!include_loopback && s.rfind("127.", 0) == 0) continue;
    bool dup = false;
    for (auto& o : out) dup |= (o == s);
    if (!dup) out.push_back(s);
  }
  freeifaddrs(ifa);
  if (out.empty()) out.push_back("127.0.0.1");
  return out;
}

// ================================================================ multistream
const char* kMultistreamProto = "/multistream/1.0.0";

static void ms_write(Conn& c, const std::string& line) { write_frame(c, to_bytes(line + "\n")); }

static std::string ms_read(BufConn& c) {
  Bytes f = c.read_frame(1024);
  if (f.empty() || f.back() != '\n') throw NetError("multistream: malformed message");
  return std::string(f.begin(), f.end() - 1);
}

void ms_select(BufConn& c, const std::string& proto) {
  // header + proposal pipelined in one write
  Bytes out = uvarint(strlen(kMultistreamProto) + 1);
  append(out, std::string(kMultistreamProto) + "\n");
  put_uvarint(out, proto.size() + 1);
  append(out, proto + "\n");
  c.write_all(out);
  std::string h = ms_read(c);
  if (h != kMultistreamProto) throw NetError("multistream: bad header " + h);
  std::string r = ms_read(c);
  if (r == proto) return;
  if (r == "na") throw NetError("protocol not supported: " + proto);
  throw NetError("multistream: unexpected response " + r);
}

std::string ms_select_any(BufConn& c, const std::vector<std::string>& protos) {
  if (protos.empty()) throw NetError("multistream: nothing to propose");
  Bytes out = uvarint(strlen(kMultistreamProto) + 1);
  append(out, std::string(kMultistreamProto) + "\n");
  put_uvarint(out, protos[0].size() + 1);
  append(out, protos[0] + "\n");
  c.write_all(out);
  std::string h = ms_read(c);
  if (h != kMultistreamProto) throw NetError("multistream: bad header " + h);
  for (size_t i = 0;;) {
    std::string r = ms_read(c);
    if (r == protos[i]) return r;
    if (r != "na") throw NetError("multistream: unexpected response " + r);
    if (++i == protos.size()) throw NetError("protocol not supported: " + protos[0]);
    ms_write(c, protos[i]);
  }
}

std::string ms_handle(BufConn& c, const std::set<std::string>& protos) {
  std::string h = ms_read(c);
  if (h != kMultistreamProto) throw NetError("multistream: bad header " + h);
  ms_write(c, kMultistreamProto);
  for (int tries = 0; tries < 32; ++tries) {
    std::string p = ms_read(c);
    if (protos.count(p)) {
      ms_write(c, p);
      return p;
    }
    if (p == "ls") {
      Bytes body;
      for (auto& x : protos) {
        put_uvarint(body, x.size() + 1);
        append(body, x + "\n");
      }
      Bytes msg = body;
      msg.push_back('\n');
      write_frame(c, msg);
      continue;
    }
    ms_write(c, "na");
  }
  throw NetError("multistream: too many proposals");
}

// ================================================================ Noise XX
namespace {
const char* kNoiseName = "Noise_XX_25519_ChaChaPoly_SHA256";
const char* kSigPrefix = "noise-libp2p-static-key:";
constexpr size_t kMaxNoiseMsg = 65535;

struct Symmetric {
  Bytes ck, h, k;
  uint64_t n = 0;
  bool has_key = false;

  void init() {
    h = to_bytes(kNoiseName);  // exactly HASHLEN (32) bytes -> used as-is
    ck = h;
    mix_hash(Bytes());  // empty prologue
  }
  void mix_hash(const Bytes& data) {
    Bytes t = h;
    append(t, data);
    h = sha256(t);
  }
  static void hkdf2(const Bytes& ck, const Bytes& ikm, Bytes* o1, Bytes* o2) {
    Bytes tk = hmac_sha256(ck, ikm);
    *o1 = hmac_sha256(tk, Bytes{0x01});
    Bytes t2 = *o1;
    t2.push_back(0x02);
    *o2 = hmac_sha256(tk, t2);
  }
  void mix_key(const Bytes& ikm) {
    Bytes nck, tk;
    hkdf2(ck, ikm, &nck, &tk);
    ck = nck;
    k = tk;
    n = 0;
    has_key = true;
  }
  Bytes encrypt_and_hash(const Bytes& pt) {
    Bytes ct = has_key ? chachapoly_encrypt(k, n++, h, pt) : pt;
    mix_hash(ct);
    return ct;
  }
  Bytes decrypt_and_hash(const Bytes& ct) {
    Bytes pt = has_key ? chachapoly_decrypt(k, n++, h, ct) : ct;
    mix_hash(ct);
    return pt;
  }
  void split(Bytes* k1, Bytes* k2) { hkdf2(ck, Bytes(), k1, k2); }
};

void noise_write_msg(Conn& c, const Bytes& m) {
  if (m.size() > kMaxNoiseMsg) throw NetError("noise: message too large");
  Bytes out{(uint8_t)(m.size() >> 8), (uint8_t)m.size()};
  append(out, m);
  c.write_all(out);
}

Bytes noise_read_msg(Conn& c) {
  uint8_t l[2];
  c.read_exact(l, 2);
  size_t n = ((size_t)l[0] << 8) | l[1];
  return c.read_exact(n);
}

Bytes make_payload(const PrivateKey& id_key, const Bytes& static_pub) {
  Bytes msg = to_bytes(kSigPrefix);
  append(msg, static_pub);
  PbWriter ext;
  ext.bytes_field(2, std::string("/yamux/1.0.0"));
  PbWriter w;
  w.bytes_field(1, id_key.public_key().marshal());
  w.bytes_field(2, id_key.sign(msg));
  w.bytes_field(4, ext.buf);
  return w.buf;
}

PublicKey verify_payload(const Bytes& payload, const Bytes& remote_static) {
  Bytes key_pb, sig;
  for (auto& f : pb_parse(payload)) {
    if (f.field == 1 && f.wire == 2) key_pb = f.bytes;
    if (f.field == 2 && f.wire == 2) sig = f.bytes;
  }
  if (key_pb.empty() || sig.empty()) throw NetError("noise: payload missing identity");
  PublicKey pk = PublicKey::unmarshal(key_pb);
  Bytes msg = to_bytes(kSigPrefix);
  append(msg, remote_static);
  if (!pk.verify(msg, sig)) throw NetError("noise: bad static key signature");
  return pk;
}
}  // namespace

Bytes noise_handshake_payload(const PrivateKey& id_key, const Bytes& static_pub) {
  return make_payload(id_key, static_pub);
}

std::shared_ptr<NoiseConn> NoiseConn::handshake(ConnPtr c, const PrivateKey& id_key,
                                                bool initiator, const PeerId& expected) {
  auto nc = std::shared_ptr<NoiseConn>(new NoiseConn());
  nc->c_ = c;
  Symmetric ss;
  ss.init();
  X25519Key s = X25519Key::generate();
  X25519Key e = X25519Key::generate();
  Bytes re, rs;
  Bytes k1, k2;
  if (initiator) {
    // -> e
    Bytes m1 = e.pub;
    ss.mix_hash(e.pub);
    append(m1, ss.encrypt_and_hash(Bytes()));
    noise_write_msg(*c, m1);
    // <- e, ee, s, es
    Bytes m2 = noise_read_msg(*c);
    if (m2.size() < 32 + 48) throw NetError("noise: short message 2");
    re.assign(m2.begin(), m2.begin() + 32);
    ss.mix_hash(re);
    ss.mix_key(x25519(e.priv, re));
    rs = ss.decrypt_and_hash(Bytes(m2.begin() + 32, m2.begin() + 80));
    ss.mix_key(x25519(e.priv, rs));
    Bytes payload = ss.decrypt_and_hash(Bytes(m2.begin() + 80, m2.end()));
    nc->remote_key_ = verify_payload(payload, rs);
    nc->remote_ = PeerId::from_public_key(nc->remote_key_);
    if (!expected.empty() && expected != nc->remote_)
      throw NetError("noise: peer id mismatch (dialed " + expected.to_base58() + ", got " +
                     nc->remote_.to_base58() + ")");
    // -> s, se
    Bytes m3 = ss.encrypt_and_hash(s.pub);
    ss.mix_key(x25519(s.priv, re));
    append(m3, ss.encrypt_and_hash(make_payload(id_key, s.pub)));
    noise_write_msg(*c, m3);
    ss.split(&k1, &k2);
    nc->k_send_ = k1;
    nc->k_recv_ = k2;
  } else {
    // -> e
    Bytes m1 = noise_read_msg(*c);
    if (m1.size() < 32) throw NetError("noise: short message 1");
    re.assign(m1.begin(), m1.begin() + 32);
    ss.mix_hash(re);
    ss.decrypt_and_hash(Bytes(m1.begin() + 32, m1.end()));
    // <- e, ee, s, es
    Bytes m2 = e.pub;
    ss.mix_hash(e.pub);
    ss.mix_key(x25519(e.priv, re));
    append(m2, ss.encrypt_and_hash(s.pub));
    ss.mix_key(x25519(s.priv, re));
    append(m2, ss.encrypt_and_hash(make_payload(id_key, s.pub)));
    noise_write_msg(*c, m2);
    // -> s, se
    Bytes m3 = noise_read_msg(*c);
    if (m3.size() < 48) throw NetError("noise: short message 3");
    rs = ss.decrypt_and_hash(Bytes(m3.begin(), m3.begin() + 48));
    ss.mix_key(x25519(e.priv, rs));
    Bytes payload = ss.decrypt_and_hash(Bytes(m3.begin() + 48, m3.end()));
    nc->remote_key_ = verify_payload(payload, rs);
    nc->remote_ = PeerId::from_public_key(nc->remote_key_);
    ss.split(&k1, &k2);
    nc->k_send_ = k2;
    nc->k_recv_ = k1;
  }
  return nc;
}

size_t NoiseConn::read_some(uint8_t* buf, size_t n) {
  while (rpos_ >= rbuf_.size()) {
    uint8_t l[2];
    size_t got = 0;
    while (got < 2) {
      size_t r = c_->read_some(l + got, 2 - got);
      if (r == 0) {
        if (got == 0) return 0;  // clean EOF between frames
        throw NetError("noise: truncated frame");
      }
      got += r;
    }
    size_t len = ((size_t)l[0] << 8) | l[1];
    Bytes ct = c_->read_exact(len);
    rbuf_ = chachapoly_decrypt(k_recv_, n_recv_++, Bytes(), ct);
    rpos_ = 0;
  }
  size_t k = std::min(n, rbuf_.size() - rpos_);
  memcpy(buf, rbuf_.data() + rpos_, k);
  rpos_ += k;
  return k;
}

void NoiseConn::write_all(const uint8_t* buf, size_t n) {
  std::lock_guard<std::mutex> lk(wmu_);
  constexpr size_t kMaxPt = kMaxNoiseMsg - 16;
  size_t off = 0;
  Bytes out;
  do {
    size_t k = std::min(kMaxPt, n - off);
    Bytes ct = chachapoly_encrypt(k_send_, n_send_++, Bytes(), Bytes(buf + off, buf + off + k));
    out.push_back((uint8_t)(ct.size() >> 8));
    out.push_back((uint8_t)ct.size());
    append(out, ct);
    off += k;
  } while (off < n);
  c_->write_all(out);
}

}  // namespace p2p
