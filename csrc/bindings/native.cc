// pybind11 module `_native`: the C++ chat plane (node, directory, relay) for
// in-process use with the GPU engine, plus codec entry points for unit tests.
// The GIL is released while C++ blocks; the engine hook re-acquires it.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <arpa/inet.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <thread>

#include "net/chat.h"
#include "net/quic.h"
#include "net/tls.h"
#include "net/relay.h"
#include "net/yamux.h"
#include "runtime/scheduler.h"

namespace py = pybind11;
using namespace p2p;

void bind_runtime(py::module_& m);      // runtime_bind.cc
void bind_engine_loop(py::module_& m);  // runtime_bind.cc

namespace {

py::bytes B(const Bytes& b) { return py::bytes((const char*)b.data(), b.size()); }
Bytes U(const py::bytes& b) {
  std::string s = b;
  return Bytes(s.begin(), s.end());
}

NodeConfig cfg_from_dict(const py::dict& d) {
  NodeConfig c = NodeConfig::from_env();
  auto S = [&](const char* k, std::string* v) {
    if (d.contains(k)) *v = py::str(d[k]);
  };
  S("username", &c.username);
  S("http_addr", &c.http_addr);
  S("directory_url", &c.directory_url);
  S("bootstrap", &c.bootstrap);
  S("relays", &c.relays);
  S("key_type", &c.key_type);
  S("security", &c.security);
  S("dial_prefer", &c.dial_prefer);
  S("identity_file", &c.identity_file);
  S("inbox_file", &c.inbox_file);
  S("engine_url", &c.engine_url);
  S("llm_model", &c.llm_model);
  S("ui_file", &c.ui_file);
  if (d.contains("register_interval")) c.register_interval_s = py::int_(d["register_interval"]);
  if (d.contains("strict_sender")) c.strict_sender = py::bool_(d["strict_sender"]);
  if (d.contains("access_log")) c.access_log = py::bool_(d["access_log"]);
  if (d.contains("listen")) c.listen = d["listen"].cast<std::vector<std::string>>();
  return c;
}

// Noise + yamux self-test over a socketpair: returns the echoed payload.
std::string secure_echo(const std::string& key_type, const std::string& payload,
                        const std::string& security) {
  const bool tls = security == "tls";
  std::string early;  // TLS ALPN muxer agreed by the client side
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) throw NetError("socketpair");
  KeyType kt = key_type == "rsa" ? KeyType::RSA : KeyType::Ed25519;
  PrivateKey ka = PrivateKey::generate(kt), kb = PrivateKey::generate(kt);
  PeerId idb = PeerId::from_public_key(kb.public_key());
  auto ca = std::make_shared<TcpConn>(sv[0]);
  auto cb = std::make_shared<TcpConn>(sv[1]);
  Bytes data(payload.begin(), payload.end());
  std::string err;
  std::thread srv([&] {
    try {
      auto b1 = std::make_shared<BufConn>(cb);
      ConnPtr sec;
      bool early_mux = false;
      if (ms_handle(*b1, {"/noise", kTlsProto}) == kTlsProto) {
        auto t = TlsConn::handshake(b1, kb, false);
        early_mux = !t->early_muxer().empty();
        sec = t;
      } else {
        sec = NoiseConn::handshake(b1, kb, false);
      }
      auto b2 = std::make_shared<BufConn>(sec);
      if (!early_mux) ms_handle(*b2, {"/yamux/1.0.0"});
      auto sess = std::make_shared<YamuxSession>(b2, false);
      std::mutex m;
      std::condition_variable cv;
      bool done = false;
      sess->start([&](StreamPtr s) {
        auto io = std::make_shared<BufConn>(s);
        ms_handle(*io, {"/echo/1.0.0"});
        Bytes all = io->read_all(64 << 20);
        io->write_all(all);
        s->close();
        std::lock_guard<std::mutex> lk(m);
        done = true;
        cv.notify_all();
      });
      std::unique_lock<std::mutex> lk(m);
      cv.wait_for(lk, std::chrono::seconds(20), [&] { return done; });
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      sess->close();
    } catch (const std::exception& e) {
      err = e.what();
    }
  });
  Bytes got;
  try {
    auto b1 = std::make_shared<BufConn>(ca);
    ConnPtr sec;
    if (tls) {
      ms_select(*b1, kTlsProto);
      auto t = TlsConn::handshake(b1, ka, true, idb);
      early = t->early_muxer();
      sec = t;
    } else {
      ms_select(*b1, "/noise");
      sec = NoiseConn::handshake(b1, ka, true, idb);
    }
    auto b2 = std::make_shared<BufConn>(sec);
    if (early.empty()) ms_select(*b2, "/yamux/1.0.0");
    auto sess = std::make_shared<YamuxSession>(b2, true);
    sess->start(nullptr);
    StreamPtr s = sess->open_stream();
    auto io = std::make_shared<BufConn>(s);
    ms_select(*io, "/echo/1.0.0");
    io->write_all(data);
    s->close_write();
    s->set_read_timeout(20000);
    got = io->read_all(64 << 20);
    s->close();
    sess->close();
  } catch (const std::exception& e) {
    srv.join();
    throw NetError(std::string("client: ") + e.what() + (err.empty() ? "" : " / server: " + err));
  }
  srv.join();
  if (!err.empty()) throw NetError("server: " + err);
  std::string res(got.begin(), got.end());
  if (tls && early != "yamux/1.0.0") throw NetError("tls: ALPN did not select the early muxer");
  return res;
}

// QUIC self-test on loopback: two transports, client dials, opens `streams`
// streams in parallel and each echoes `payload` through a multistream-negotiated
// "/echo/1.0.0" handler.  Returns {echo ok, client retransmitted frames, rtt us}.
std::tuple<bool, uint64_t, long, uint64_t, uint64_t> quic_echo(const std::string& kt,
                                                               const std::string& payload,
                                                               double drop_rate, int streams,
                                                               uint64_t ku_interval) {
  // ku_interval > 0: both endpoints start a 1-RTT key update every ku_interval packets
  quic_set_key_update_interval(ku_interval ? ku_interval : (1ull << 22));
  const KeyType t = kt == "rsa" ? KeyType::RSA : KeyType::Ed25519;
  PrivateKey ka = PrivateKey::generate(t), kb = PrivateKey::generate(t);
  const PeerId idb = PeerId::from_public_key(kb.public_key());
  const PeerId ida = PeerId::from_public_key(ka.public_key());
  auto srv = QuicTransport::create("127.0.0.1", 0, kb);
  auto cli = QuicTransport::create("127.0.0.1", 0, ka);
  srv->set_drop_rate(drop_rate);
  cli->set_drop_rate(drop_rate);
  std::string err;
  std::mutex em;
  srv->set_accept([&](QuicConnPtr c) {
    if (c->remote_peer() != ida) {
      std::lock_guard<std::mutex> lk(em);
      err = "server saw the wrong client identity";
    }
    c->start([&](StreamPtr s) {
      try {
        auto io = std::make_shared<BufConn>(s);
        ms_handle(*io, {"/echo/1.0.0"});
        s->set_read_timeout(30000);
        Bytes all = io->read_all(256 << 20);
        io->write_all(all);
        s->close();
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(em);
        err = std::string("server stream: ") + e.what();
      }
    });
  });
  bool ok = true;
  long rtt = -1;
  uint64_t retx = 0, kus = 0, cong = 0;
  try {
    auto c = cli->dial("127.0.0.1", srv->port(), idb, 10000);
    c->start(nullptr);
    std::vector<std::thread> th;
    std::vector<int> good(streams, 0);
    for (int i = 0; i < streams; ++i)
      th.emplace_back([&, i] {
        try {
          StreamPtr s = c->open_stream();
          auto io = std::make_shared<BufConn>(s);
          s->set_read_timeout(30000);
          ms_select(*io, "/echo/1.0.0");
          io->write_all(payload);
          s->close_write();
          Bytes got = io->read_all(256 << 20);
          s->close();
          good[i] = std::string(got.begin(), got.end()) == payload;
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> lk(em);
          err = std::string("client stream: ") + e.what();
        }
      });
    for (auto& t : th) t.join();
    for (int g : good) ok = ok && g;
    rtt = c->ping(2000);
    retx = c->retransmitted();
    kus = c->key_updates();
    cong = c->congestion_events();
    c->close();
  } catch (const std::exception& e) {
    cli->close();
    srv->close();
    throw NetError(std::string("quic client: ") + e.what() + (err.empty() ? "" : " / " + err));
  }
  cli->close();
  srv->close();
  quic_set_key_update_interval(1ull << 22);
  if (!err.empty()) throw NetError(err);
  return {ok, retx, rtt, kus, cong};
}

}  // namespace

namespace {
// In-memory connection for wire fixtures: reads come from a script (then EOF), writes
// are recorded byte for byte.
class MemConn : public Conn {
 public:
  explicit MemConn(Bytes script) : in_(std::move(script)) {}
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override {
    std::lock_guard<std::mutex> lk(mu_);
    const size_t k = std::min(n, in_.size() - pos_);
    std::copy(in_.begin() + pos_, in_.begin() + pos_ + k, buf);
    pos_ += k;
    return k;
  }
  void write_all(const uint8_t* buf, size_t n) override {
    std::lock_guard<std::mutex> lk(mu_);
    out_.insert(out_.end(), buf, buf + n);
  }
  void close() override {}
  Bytes written() {
    std::lock_guard<std::mutex> lk(mu_);
    return out_;
  }

 private:
  std::mutex mu_;
  Bytes in_, out_;
  size_t pos_ = 0;
};

Bytes ms_line(const std::string& s) {
  Bytes b = uvarint(s.size() + 1);
  append(b, s + "\n");
  return b;
}
}  // namespace

static p2p::Bytes hexb(const std::string& h) {
  p2p::Bytes b;
  for (size_t i = 0; i + 1 < h.size(); i += 2) b.push_back((uint8_t)std::stoi(h.substr(i, 2), nullptr, 16));
  return b;
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "native chat plane (libp2p subset, HTTP, directory, relay) + engine runtime";
  py::register_exception<NetError>(m, "NetError");
  py::register_exception<JsonError>(m, "JsonError");

  // ---- codecs ----
  m.def("uvarint", [](uint64_t v) { return B(uvarint(v)); });
  m.def("read_uvarint", [](const py::bytes& b) {
    Bytes x = U(b);
    size_t pos = 0;
    uint64_t v = get_uvarint(x, &pos);
    return py::make_tuple(v, pos);
  });
  m.def("base58_encode", [](const py::bytes& b) { return base58_encode(U(b)); });
  m.def("base58_decode", [](const std::string& s) { return B(base58_decode(s)); });
  m.def("multiaddr_to_bytes", [](const std::string& s) { return B(Multiaddr::parse(s).bytes()); });
  m.def("multiaddr_from_bytes", [](const py::bytes& b) { return Multiaddr::from_bytes(U(b)).str(); });
  m.def("multiaddr_normalize", [](const std::string& s) { return Multiaddr::parse(s).str(); });
  m.def("keygen", [](const std::string& t) {
    PrivateKey k = PrivateKey::generate(t == "rsa" ? KeyType::RSA : KeyType::Ed25519);
    PublicKey p = k.public_key();
    return py::make_tuple(B(k.marshal()), B(p.marshal()), PeerId::from_public_key(p).to_base58());
  });
  m.def("peer_id_from_public_key", [](const py::bytes& pb) {
    return PeerId::from_public_key(PublicKey::unmarshal(U(pb))).to_base58();
  });
  m.def("peer_id_decode", [](const std::string& s) { return B(PeerId::decode(s).bytes()); });
  m.def("sign", [](const py::bytes& priv, const py::bytes& msg) {
    return B(PrivateKey::unmarshal(U(priv)).sign(U(msg)));
  });
  m.def("verify", [](const py::bytes& pub, const py::bytes& msg, const py::bytes& sig) {
    return PublicKey::unmarshal(U(pub)).verify(U(msg), U(sig));
  });
  m.def("json_roundtrip", [](const std::string& s, bool sorted) {
    Json j = Json::parse(s);
    return sorted ? j.dump_sorted() : j.dump();
  }, py::arg("text"), py::arg("sorted") = false);
  m.def("parse_rfc3339", &parse_rfc3339);
  m.def("rfc3339_now", &rfc3339_now_local);
  m.def("uuid4", &uuid4);
  m.def("secure_echo", [](const std::string& kt, const py::bytes& payload,
                          const std::string& security) {
    std::string in = payload, out;
    {
      py::gil_scoped_release rel;
      out = secure_echo(kt, in, security);
    }
    return py::bytes(out);
  }, py::arg("key_type"), py::arg("payload"), py::arg("security") = "noise");
  // Fault injection (SURVEY §5 "drop connection mid-stream"): a throw-away host dials
  // `addr` (…/p2p/<id>), opens a /p2p-llm-chat/1.0.0 stream, writes `payload` and then
  // ends it with `mode`: "close" (FIN: a well-formed send, the reference's s.Close()) or
  // "reset" (RST before EOF: the receiver's io.ReadAll fails, go/cmd/node/main.go:160-164).
  m.def("chat_inject", [](const std::string& addr, const py::bytes& payload,
                          const std::string& mode) {
    std::string data = payload;
    py::gil_scoped_release rel;
    PeerId pid;
    Multiaddr ma = Multiaddr::parse(addr).without_peer(&pid);
    auto h = std::make_shared<Host>(PrivateKey::generate(KeyType::Ed25519));
    h->connect(pid, {ma}, 5000);
    StreamCtx s = h->new_stream(pid, kChatProto, 5000);
    s.io->write_all(data);
    if (mode == "reset") {
      std::this_thread::sleep_for(std::chrono::milliseconds(50));  // partial bytes arrive first
      s.stream->reset();
    } else {
      s.stream->close();
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    h->close();
  }, py::arg("addr"), py::arg("payload"), py::arg("mode") = "reset");
  m.def("quic_echo", [](const std::string& kt, const py::bytes& payload, double drop, int streams,
                        uint64_t ku_interval) {
    std::string in = payload;
    py::gil_scoped_release rel;
    return quic_echo(kt, in, drop, streams, ku_interval);
  }, py::arg("key_type"), py::arg("payload"), py::arg("drop_rate") = 0.0, py::arg("streams") = 1,
     py::arg("key_update_interval") = 0);
  // ---- wire fixtures: the exact bytes our implementation puts on the wire ----
  m.def("wire_ms_select", [](const std::string& proto) {
    // dialer side of multistream-select 1.0 (header + proposal pipelined), peer accepts
    Bytes script = ms_line(kMultistreamProto);
    append(script, ms_line(proto));
    auto mc = std::make_shared<MemConn>(script);
    BufConn bc(mc);
    ms_select(bc, proto);
    return B(mc->written());
  });
  m.def("wire_ms_handle", [](const std::vector<std::string>& proposals,
                             const std::vector<std::string>& supported) {
    // listener side: the dialer's header + proposals in order; returns what we answer
    Bytes script = ms_line(kMultistreamProto);
    for (auto& p : proposals) append(script, ms_line(p));
    auto mc = std::make_shared<MemConn>(script);
    BufConn bc(mc);
    std::string chosen;
    try {
      chosen = ms_handle(bc, std::set<std::string>(supported.begin(), supported.end()));
    } catch (const NetError&) {
    }
    return py::make_tuple(chosen, B(mc->written()));
  });
  m.def("wire_yamux_client_stream", [](const py::bytes& payload) {
    // a dialer session opens stream 1, writes one message, half-closes (the chat send)
    auto mc = std::make_shared<MemConn>(Bytes());
    auto sess = std::make_shared<YamuxSession>(mc, true);
    StreamPtr st = sess->open_stream();
    st->write_all(U(payload));
    st->close_write();
    return B(mc->written());
  });
  m.def("noise_handshake_payload", [](const py::bytes& priv, const py::bytes& static_pub) {
    return B(noise_handshake_payload(PrivateKey::unmarshal(U(priv)), U(static_pub)));
  });
  m.def("relay_voucher", [](const py::bytes& priv, const std::string& relay,
                            const std::string& peer, uint64_t expire) {
    return B(test_make_voucher(PrivateKey::unmarshal(U(priv)), PeerId::decode(relay),
                               PeerId::decode(peer), expire));
  });
  m.def("relay_voucher_verify", [](const py::bytes& env, const std::string& relay,
                                   const std::string& peer, uint64_t expire) {
    try {
      verify_voucher(U(env), PeerId::decode(relay), PeerId::decode(peer), expire);
      return true;
    } catch (const NetError&) {
      return false;
    }
  });
  m.def("relay_voucher_check", []() {
    // {good voucher verifies, wrong peer rejected, wrong expiry rejected, foreign signer
    // rejected, tampered signature rejected}
    PrivateKey rk = PrivateKey::generate(KeyType::Ed25519), pk = PrivateKey::generate(KeyType::Ed25519);
    PrivateKey other = PrivateKey::generate(KeyType::RSA);
    const PeerId relay = PeerId::from_public_key(rk.public_key());
    const PeerId peer = PeerId::from_public_key(pk.public_key());
    const PeerId stranger = PeerId::from_public_key(other.public_key());
    const Bytes v = test_make_voucher(rk, relay, peer, 1234567);
    auto ok = [&](const Bytes& env, const PeerId& r, const PeerId& p, uint64_t e) {
      try {
        verify_voucher(env, r, p, e);
        return true;
      } catch (const NetError&) {
        return false;
      }
    };
    Bytes tampered = v;
    tampered[tampered.size() - 3] ^= 0x40;
    return py::make_tuple(ok(v, relay, peer, 1234567), ok(v, relay, stranger, 1234567),
                          ok(v, relay, peer, 1234568),
                          ok(test_make_voucher(other, relay, peer, 1234567), relay, peer, 1234567),
                          ok(tampered, relay, peer, 1234567));
  });
  m.def("rcmgr_check", [](const std::string& transport, int peer_streams, int proto_streams,
                          int attempts) {
    // A server host with small resource limits; a client holds `attempts` streams of one
    // protocol open.  Returns (accepted, refused, a stream after release works, stats).
    int accepted = 0, refused = 0;
    bool reopened = false;
    std::string stats;
    {
    py::gil_scoped_release rel;
    auto srv = std::make_shared<Host>(PrivateKey::generate(KeyType::Ed25519));
    auto cli = std::make_shared<Host>(PrivateKey::generate(KeyType::Ed25519));
    ResourceLimits l;
    l.peer_streams_inbound = peer_streams;
    l.protocol_streams_inbound = proto_streams;
    srv->resources().set_limits(l);
    srv->set_stream_handler("/hold/1.0.0", [](StreamCtx& c) {
      uint8_t b = 0;
      c.io->set_read_timeout(20000);
      try {
        if (c.io->read_some(&b, 1) != 1) return;
        c.io->write_all(&b, 1);
        while (c.io->read_some(&b, 1) == 1) {
        }
      } catch (...) {
      }
      c.stream->close();
    });
    srv->listen(Multiaddr::parse(transport == "quic" ? "/ip4/127.0.0.1/udp/0/quic-v1"
                                                     : "/ip4/127.0.0.1/tcp/0"));
    std::vector<StreamCtx> held;
    try {
      cli->connect(srv->id(), srv->addrs(), 10000);
      auto open_one = [&]() {
        StreamCtx c = cli->new_stream(srv->id(), "/hold/1.0.0", 10000);
        uint8_t b = 7;
        c.io->write_all(&b, 1);
        c.io->set_read_timeout(10000);
        if (c.io->read_some(&b, 1) != 1 || b != 7) throw NetError("no echo");
        return c;
      };
      for (int i = 0; i < attempts; ++i) {
        try {
          held.push_back(open_one());
          ++accepted;
        } catch (const std::exception&) {
          ++refused;
        }
      }
      for (auto& c : held) c.stream->close();
      held.clear();
      for (int i = 0; i < 100 && !reopened; ++i) {  // the server releases as handlers end
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        try {
          StreamCtx c = open_one();
          c.stream->close();
          reopened = true;
        } catch (const std::exception&) {
        }
      }
    } catch (...) {
      cli->close();
      srv->close();
      throw;
    }
    stats = srv->resources().stats().dump();
    cli->close();
    srv->close();
    }
    return py::make_tuple(accepted, refused, reopened, stats);
  }, py::arg("transport") = "tcp", py::arg("peer_streams") = 4, py::arg("proto_streams") = 2048,
     py::arg("attempts") = 8);
  m.def("quic_version_negotiation", []() {
    // (server) a long-header first flight of an unknown version gets a Version Negotiation
    // packet: version 0, connection ids swapped, versions listing 1; a short datagram none.
    // (client) a VN that does not list v1 fails the dial at once with the server's list;
    // one that lists v1 is ignored (the dial runs into its timeout instead).
    // Returns (vn_ok, short_ignored, client_error, ignored_error).
    PrivateKey kb = PrivateKey::generate(KeyType::Ed25519), ka = PrivateKey::generate(KeyType::Ed25519);
    bool vn_ok = false, short_ignored = false;
    std::string cli_err, ign_err;
    {
      py::gil_scoped_release nogil;
      auto srv = QuicTransport::create("127.0.0.1", 0, kb);
      srv->set_accept([](QuicConnPtr c) { c->start([](StreamPtr) {}); });
      const int fd = ::socket(AF_INET, SOCK_DGRAM, 0);
      timeval tv{1, 0};
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
      sockaddr_in to{};
      to.sin_family = AF_INET;
      to.sin_port = htons((uint16_t)srv->port());
      inet_pton(AF_INET, "127.0.0.1", &to.sin_addr);
      auto probe = [&](size_t len) {
        Bytes pkt(len, 0);
        pkt[0] = 0xc0;
        const uint8_t ver[4] = {0x0a, 0x0a, 0x0a, 0x0a};  // a reserved version
        memcpy(&pkt[1], ver, 4);
        pkt[5] = 8;
        for (int i = 0; i < 8; ++i) pkt[6 + i] = (uint8_t)(0xd0 + i);  // DCID
        pkt[14] = 8;
        for (int i = 0; i < 8; ++i) pkt[15 + i] = (uint8_t)(0x50 + i);  // SCID
        ::sendto(fd, pkt.data(), pkt.size(), 0, (const sockaddr*)&to, sizeof(to));
        uint8_t buf[1500];
        const ssize_t r = ::recv(fd, buf, sizeof(buf), 0);
        return Bytes(buf, buf + (r > 0 ? r : 0));
      };
      const Bytes shortr = probe(200);
      short_ignored = shortr.empty();
      const Bytes v = probe(1200);
      if (v.size() >= 7 + 8 + 1 + 8 + 4 && (v[0] & 0x80) && v[1] == 0 && v[2] == 0 && v[3] == 0 &&
          v[4] == 0 && v[5] == 8 && v[6] == 0x50 && v[14] == 8 && v[15] == 0xd0) {
        for (size_t q = 23; q + 4 <= v.size(); q += 4)
          vn_ok |= v[q] == 0 && v[q + 1] == 0 && v[q + 2] == 0 && v[q + 3] == 1;
      }
      ::close(fd);
      srv->close();
      // client side: a fake server answering the first Initial with a VN
      auto fake = [&](bool list_v1, int timeout_ms) {
        const int sfd = ::socket(AF_INET, SOCK_DGRAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
        ::bind(sfd, (const sockaddr*)&a, sizeof(a));
        socklen_t al = sizeof(a);
        getsockname(sfd, (sockaddr*)&a, &al);
        setsockopt(sfd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        std::thread t([&, sfd] {
          uint8_t buf[1600];
          sockaddr_in from{};
          socklen_t fl = sizeof(from);
          const ssize_t r = ::recvfrom(sfd, buf, sizeof(buf), 0, (sockaddr*)&from, &fl);
          if (r < 7) return;
          const size_t dl = buf[5], sl = buf[6 + dl];
          Bytes vn{0x80, 0, 0, 0, 0, (uint8_t)sl};
          vn.insert(vn.end(), buf + 7 + dl, buf + 7 + dl + sl);
          vn.push_back((uint8_t)dl);
          vn.insert(vn.end(), buf + 6, buf + 6 + dl);
          const uint8_t other[4] = {0xff, 0x00, 0x00, 0x1d};
          vn.insert(vn.end(), other, other + 4);
          if (list_v1) {
            const uint8_t v1[4] = {0, 0, 0, 1};
            vn.insert(vn.end(), v1, v1 + 4);
          }
          ::sendto(sfd, vn.data(), vn.size(), 0, (const sockaddr*)&from, fl);
        });
        auto cli = QuicTransport::create("127.0.0.1", 0, ka);
        std::string err;
        try {
          cli->dial("127.0.0.1", ntohs(a.sin_port), PeerId(), timeout_ms);
        } catch (const std::exception& e) {
          err = e.what();
        }
        t.join();
        cli->close();
        ::close(sfd);
        return err;
      };
      cli_err = fake(false, 5000);
      ign_err = fake(true, 600);
    }
    return py::make_tuple(vn_ok, short_ignored, cli_err, ign_err);
  });
  m.def("quic_retry", []() {
    // (a) the RFC 9001 Appendix A.4 Retry integrity tag;
    // (b) a server requiring address validation answers the first Initial with a Retry and
    //     completes the handshake with the client echoing the token (both ends check the
    //     original/retry connection-id transport parameters);
    // (c) an Initial with a forged token is dropped;
    // (d) against a fake server: a Retry with a bad tag is ignored, a valid one makes the
    //     client resend its first flight to the Retry's SCID carrying the token.
    // Returns (vector_ok, handshake_ok, retries_sent, forged_rejected, bad_tag_ignored,
    //          resend_ok).
    const Bytes odcid = hexb("8394c8f03e515708");
    const Bytes rp = hexb("ff000000010008f067a5502a4262b5746f6b656e");
    const bool vector_ok = quic_retry_tag(odcid, rp.data(), rp.size()) ==
                           hexb("04a265ba2eff4d829058fb3f0f2496ba");
    bool handshake_ok = false, bad_tag_ignored = false, resend_ok = false;
    long retries = 0, rejected = 0;
    {
      py::gil_scoped_release nogil;
      PrivateKey kb = PrivateKey::generate(KeyType::Ed25519), ka = PrivateKey::generate(KeyType::Ed25519);
      auto srv = QuicTransport::create("127.0.0.1", 0, kb);
      srv->set_require_retry(true);
      srv->set_accept([](QuicConnPtr c) { c->start([](StreamPtr) {}); });
      auto cli = QuicTransport::create("127.0.0.1", 0, ka);
      try {
        auto c = cli->dial("127.0.0.1", srv->port(), PeerId::from_public_key(kb.public_key()), 5000);
        handshake_ok = c->established();
        c->close();
      } catch (const std::exception&) {
      }
      retries = srv->retries_sent();
      // (c) forged token
      const int fd = ::socket(AF_INET, SOCK_DGRAM, 0);
      sockaddr_in to{};
      to.sin_family = AF_INET;
      to.sin_port = htons((uint16_t)srv->port());
      inet_pton(AF_INET, "127.0.0.1", &to.sin_addr);
      Bytes pkt(1200, 0);
      pkt[0] = 0xc3;
      pkt[4] = 1;
      pkt[5] = 8;
      for (int i = 0; i < 8; ++i) pkt[6 + i] = (uint8_t)(0xa0 + i);
      pkt[14] = 8;
      for (int i = 0; i < 8; ++i) pkt[15 + i] = (uint8_t)(0xb0 + i);
      pkt[23] = 41;  // token length (1-byte varint), bytes of garbage follow
      for (int i = 0; i < 41; ++i) pkt[24 + i] = (uint8_t)(i * 7);
      ::sendto(fd, pkt.data(), pkt.size(), 0, (const sockaddr*)&to, sizeof(to));
      ::close(fd);
      for (int i = 0; i < 100 && srv->tokens_rejected() == 0; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      rejected = srv->tokens_rejected();
      cli->close();
      srv->close();
      // (d) fake server
      auto fake = [&](bool good_tag) {
        const int sfd = ::socket(AF_INET, SOCK_DGRAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
        ::bind(sfd, (const sockaddr*)&a, sizeof(a));
        socklen_t al = sizeof(a);
        getsockname(sfd, (sockaddr*)&a, &al);
        timeval tv{1, 0};
        setsockopt(sfd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        const Bytes rscid = hexb("5a5a5a5a5a5a5a5a"), token = hexb("746f6b656e2d31");
        bool resent = false, second = false;
        std::thread t([&, sfd] {
          uint8_t buf[1600];
          sockaddr_in from{};
          socklen_t fl = sizeof(from);
          const ssize_t r = ::recvfrom(sfd, buf, sizeof(buf), 0, (sockaddr*)&from, &fl);
          if (r < 7) return;
          const size_t dl = buf[5], sl = buf[6 + dl];
          const Bytes cdcid(buf + 6, buf + 6 + dl);
          Bytes rt{0xf0, 0, 0, 0, 1, (uint8_t)sl};
          rt.insert(rt.end(), buf + 7 + dl, buf + 7 + dl + sl);
          rt.push_back((uint8_t)rscid.size());
          rt.insert(rt.end(), rscid.begin(), rscid.end());
          rt.insert(rt.end(), token.begin(), token.end());
          Bytes tag = quic_retry_tag(cdcid, rt.data(), rt.size());
          if (!good_tag) tag[3] ^= 1;
          rt.insert(rt.end(), tag.begin(), tag.end());
          ::sendto(sfd, rt.data(), rt.size(), 0, (const sockaddr*)&from, fl);
          // the next Initial: (good tag) DCID = rscid + our token; (bad tag) unchanged
          for (int k = 0; k < 4; ++k) {
            const ssize_t r2 = ::recvfrom(sfd, buf, sizeof(buf), 0, (sockaddr*)&from, &fl);
            if (r2 < 7) break;
            const size_t dl2 = buf[5];
            const Bytes d2(buf + 6, buf + 6 + dl2);
            const size_t sl2 = buf[6 + dl2];
            size_t q = 7 + dl2 + sl2;
            const size_t tl = buf[q++];  // tokens here are < 64 bytes: 1-byte varint
            const Bytes tk(buf + q, buf + q + tl);
            second = true;
            resent = good_tag ? (d2 == rscid && tk == token) : (d2 == cdcid && tk.empty());
            break;
          }
        });
        auto cl = QuicTransport::create("127.0.0.1", 0, ka);
        try {
          cl->dial("127.0.0.1", ntohs(a.sin_port), PeerId(), 1500);
        } catch (const std::exception&) {
        }
        t.join();
        cl->close();
        ::close(sfd);
        return second && resent;
      };
      bad_tag_ignored = fake(false);
      resend_ok = fake(true);
    }
    return py::make_tuple(vector_ok, handshake_ok, retries, rejected, bad_tag_ignored, resend_ok);
  });
  m.def("quic_protocol_violation", [](const std::string& kind) {
    // a client sends a frame past the server's advertised limits; returns the client's
    // view of the close (the server must answer with the RFC 9000 error code)
    PrivateKey ka = PrivateKey::generate(KeyType::Ed25519), kb = PrivateKey::generate(KeyType::Ed25519);
    const PeerId idb = PeerId::from_public_key(kb.public_key());
    auto srv = QuicTransport::create("127.0.0.1", 0, kb);
    auto cli = QuicTransport::create("127.0.0.1", 0, ka);
    srv->set_accept([](QuicConnPtr c) { c->start([](StreamPtr) {}); });
    std::string why;
    bool closed = false;
    {
      py::gil_scoped_release nogil;
      auto c = cli->dial("127.0.0.1", srv->port(), idb, 10000);
      c->start(nullptr);
      Bytes f;
      if (kind == "stream") {  // STREAM (OFF|LEN) on our stream 0 at 64 MiB: past the 4 MiB window
        f.push_back(0x0e);
        quic_put_varint(f, 0);
        quic_put_varint(f, 64ull << 20);
        quic_put_varint(f, 16);
        f.insert(f.end(), 16, 0x61);
      } else if (kind == "conn") {  // many streams, each inside its window, together past MAX_DATA
        for (int i = 0; i < 5; ++i) {
          Bytes g{0x0e};
          quic_put_varint(g, (uint64_t)i << 2);
          quic_put_varint(g, (4ull << 20) - 16);
          quic_put_varint(g, 16);
          g.insert(g.end(), 16, 0x62);
          c->send_raw_frame_for_test(g);
        }
      } else {  // CRYPTO far ahead of the handshake stream
        f.push_back(0x06);
        quic_put_varint(f, 1ull << 30);
        quic_put_varint(f, 16);
        f.insert(f.end(), 16, 0x63);
      }
      if (!f.empty()) c->send_raw_frame_for_test(f);
      for (int i = 0; i < 200 && !c->closed(); ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      closed = c->closed();
      why = c->error_text();
      c->close();
      cli->close();
      srv->close();
    }
    return py::make_tuple(closed, why);
  });
  m.def("quic_initial_keys", [](const py::bytes& dcid) {
    QuicKeys c, s;
    quic_initial_keys(U(dcid), &c, &s);
    auto t = [](const QuicKeys& k) {
      return py::make_tuple(py::bytes((const char*)k.key, 16), py::bytes((const char*)k.iv, 12),
                            py::bytes((const char*)k.hp, 16));
    };
    return py::make_tuple(t(c), t(s));
  });
  m.def("chat_message_from_json", [](const std::string& s) {
    return ChatMessage::from_json(Json::parse(s)).to_json().dump();
  });
  m.def("set_log_quiet", &set_log_quiet);
  m.def("http_request", [](const std::string& method, const std::string& url,
                           const std::string& body, const std::string& ctype, int timeout_ms) {
    HttpResult r;
    {
      py::gil_scoped_release rel;
      r = http_request(method, url, body, ctype, timeout_ms);
    }
    return py::make_tuple(r.status, r.body);
  }, py::arg("method"), py::arg("url"), py::arg("body") = "", py::arg("content_type") = "",
        py::arg("timeout_ms") = 5000);

  // ---- node ----
  py::class_<Node>(m, "Node")
      .def(py::init([](py::dict d) { return new Node(cfg_from_dict(d)); }), py::arg("config") = py::dict())
      .def("start", &Node::start, py::call_guard<py::gil_scoped_release>())
      .def("wait", &Node::wait, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Node::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("http_port", &Node::http_port)
      .def_property_readonly("peer_id", &Node::peer_id)
      .def_property_readonly("addrs", &Node::addrs)
      .def("send", [](Node& n, const std::string& to, const std::string& content) {
        std::pair<int, Json> r;
        {
          py::gil_scoped_release rel;
          r = n.send(to, content);
        }
        return py::make_tuple(r.first, r.second.dump_sorted());
      })
      .def("inbox", [](Node& n, const std::string& after) {
        Json arr = Json::array();
        for (auto& x : n.inbox().drain(after)) arr.push(x.to_json());
        return arr.dump();
      }, py::arg("after") = "")
      .def("set_generate_hook", [](Node& n, py::function fn) {
        auto holder = std::make_shared<py::function>(std::move(fn));
        n.set_generate_hook([holder](const Json& req) -> Json {
          std::string out;
          {
            py::gil_scoped_acquire g;
            out = py::str((*holder)(req.dump()));
          }
          return Json::parse(out);
        });
      })
      .def("set_generate_stream_hook", [](Node& n, py::function fn) {
        // fn(req_text, emit) -> final_text, emit(chunk_text) -> bool (called under the GIL)
        auto holder = std::make_shared<py::function>(std::move(fn));
        n.set_generate_stream_hook(
            [holder](const Json& req, const std::function<bool(const Json&)>& emit) -> Json {
              std::string out;
              {
                py::gil_scoped_acquire g;
                py::cpp_function py_emit([&emit](const std::string& chunk) {
                  Json c = Json::parse(chunk);
                  py::gil_scoped_release rel;  // socket write without the GIL
                  return emit(c);
                });
                out = py::str((*holder)(req.dump(), py_emit));
              }
              return Json::parse(out);
            });
      })
      .def("metrics", [](Node& n) { return n.metrics_json().dump(); });

  // ---- directory ----
  py::class_<HttpServer>(m, "_HttpServer");
  struct Dir {
    DirectoryService svc;
    HttpServer srv{"GIN"};
    explicit Dir(int ttl) : svc(ttl) { svc.install(srv); }
  };
  py::class_<Dir>(m, "Directory")
      .def(py::init<int>(), py::arg("ttl") = 0)
      .def("start", [](Dir& d, const std::string& addr, bool log) {
        d.srv.set_access_log(log);
        return d.srv.start(addr);
      }, py::arg("addr") = "127.0.0.1:0", py::arg("access_log") = false)
      .def("stop", [](Dir& d) { d.srv.stop(); }, py::call_guard<py::gil_scoped_release>())
      .def("size", [](Dir& d) { return d.svc.size(); });

  // ---- relay ----
  struct Relay {
    std::shared_ptr<Host> h;
    std::unique_ptr<RelayService> svc;
  };
  py::class_<Relay>(m, "Relay")
      .def(py::init([](const std::string& listen) {
        auto r = new Relay();
        r->h = std::make_shared<Host>(PrivateKey::generate(KeyType::Ed25519), "p2p-relay");
        r->h->listen(Multiaddr::parse(listen));
        r->svc = std::make_unique<RelayService>(r->h);
        return r;
      }), py::arg("listen") = "/ip4/127.0.0.1/tcp/0")
      .def_property_readonly("peer_id", [](Relay& r) { return r.h->id().to_base58(); })
      .def("addrs", [](Relay& r) {
        std::vector<std::string> out;
        for (auto& a : r.h->addrs()) out.push_back(a.str() + "/p2p/" + r.h->id().to_base58());
        return out;
      })
      .def("reservations", [](Relay& r) { return r.svc->reservations(); })
      .def("stop", [](Relay& r) { r.h->close(); }, py::call_guard<py::gil_scoped_release>());

  bind_runtime(m);
  bind_engine_loop(m);
}
