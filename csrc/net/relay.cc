#include "relay.h"

#include <time.h>

#include <thread>

namespace p2p {

const char* kHopProto = "/libp2p/circuit/relay/0.2.0/hop";
const char* kStopProto = "/libp2p/circuit/relay/0.2.0/stop";

namespace {
enum { HOP_RESERVE = 0, HOP_CONNECT = 1, HOP_STATUS = 2 };
enum { STOP_CONNECT = 0, STOP_STATUS = 1 };

struct RelayMsg {
  int type = -1;
  PeerId peer;
  std::vector<Bytes> peer_addrs;
  uint64_t expire = 0;
  std::vector<Bytes> resv_addrs;
  Bytes voucher;  // Reservation.voucher: signed envelope of a ReservationVoucher
  uint32_t limit_duration = 0;
  uint64_t limit_data = 0;
  int status = 0;
};

Bytes peer_pb(const PeerId& id, const std::vector<Bytes>& addrs) {
  PbWriter w;
  w.bytes_field(1, id.bytes());
  for (auto& a : addrs) w.bytes_field(2, a);
  return w.buf;
}

Bytes limit_pb(uint32_t dur, uint64_t data) {
  PbWriter w;
  w.varint_field(1, dur);
  w.varint_field(2, data);
  return w.buf;
}

// HopMessage {type=1, peer=2, reservation=3, limit=4, status=5}
// StopMessage {type=1, peer=2, limit=3, status=4}
RelayMsg parse(const Bytes& b, bool hop) {
  RelayMsg m;
  for (auto& f : pb_parse(b)) {
    if (f.field == 1 && f.wire == 0) m.type = (int)f.varint;
    else if (f.field == 2 && f.wire == 2) {
      for (auto& g : pb_parse(f.bytes)) {
        if (g.field == 1 && g.wire == 2) m.peer = PeerId::from_bytes(g.bytes);
        if (g.field == 2 && g.wire == 2) m.peer_addrs.push_back(g.bytes);
      }
    } else if (hop && f.field == 3 && f.wire == 2) {
      for (auto& g : pb_parse(f.bytes)) {
        if (g.field == 1 && g.wire == 0) m.expire = g.varint;
        if (g.field == 2 && g.wire == 2) m.resv_addrs.push_back(g.bytes);
        if (g.field == 3 && g.wire == 2) m.voucher = g.bytes;
      }
    } else if (((hop && f.field == 4) || (!hop && f.field == 3)) && f.wire == 2) {
      for (auto& g : pb_parse(f.bytes)) {
        if (g.field == 1 && g.wire == 0) m.limit_duration = (uint32_t)g.varint;
        if (g.field == 2 && g.wire == 0) m.limit_data = g.varint;
      }
    } else if (((hop && f.field == 5) || (!hop && f.field == 4)) && f.wire == 0) {
      m.status = (int)f.varint;
    }
  }
  return m;
}

// ---- reservation vouchers (circuit relay v2 spec, "Reservation Vouchers") ----
// ReservationVoucher {relay=1 (peer id bytes), peer=2 (peer id bytes), expiration=3}
// carried in a libp2p signed envelope (RFC 0002): Envelope {public_key=1, payload_type=2,
// payload=3, signature=5}, signature over
//   uvarint(len(domain)) domain uvarint(len(type)) type uvarint(len(payload)) payload
// with domain "libp2p-relay-rsvp" and payload type = the two raw bytes {0x03, 0x02}: the
// multicodec number written big-endian as go-libp2p's circuitv2 proto.RecordCodec does
// (like the peer record's {0x03, 0x01}) -- NOT its uvarint encoding (0x82 0x06).
const char* kVoucherDomain = "libp2p-relay-rsvp";

Bytes voucher_type() { return Bytes{0x03, 0x02}; }

Bytes envelope_signed_data(const Bytes& type, const Bytes& payload) {
  Bytes d;
  const std::string dom = kVoucherDomain;
  put_uvarint(d, dom.size());
  d.insert(d.end(), dom.begin(), dom.end());
  put_uvarint(d, type.size());
  append(d, type);
  put_uvarint(d, payload.size());
  append(d, payload);
  return d;
}

Bytes voucher_payload(const PeerId& relay, const PeerId& peer, uint64_t expire) {
  PbWriter w;
  w.bytes_field(1, relay.bytes());
  w.bytes_field(2, peer.bytes());
  w.varint_field(3, expire);
  return w.buf;
}

Bytes make_voucher(const PrivateKey& key, const PeerId& relay, const PeerId& peer,
                   uint64_t expire) {
  const Bytes type = voucher_type();
  const Bytes payload = voucher_payload(relay, peer, expire);
  PbWriter env;
  env.bytes_field(1, key.public_key().marshal());
  env.bytes_field(2, type);
  env.bytes_field(3, payload);
  env.bytes_field(5, key.sign(envelope_signed_data(type, payload)));
  return env.buf;
}
}  // namespace

// Verifies a reservation voucher envelope: signed by the relay's key (the envelope key
// must hash to `relay`), payload type ReservationVoucher, relay/peer fields matching, and
// the expiration equal to the reservation's.  Throws NetError on any mismatch.
void verify_voucher(const Bytes& env, const PeerId& relay, const PeerId& peer, uint64_t expire) {
  Bytes pk, type, payload, sig;
  for (auto& f : pb_parse(env)) {
    if (f.wire != 2) continue;
    if (f.field == 1) pk = f.bytes;
    if (f.field == 2) type = f.bytes;
    if (f.field == 3) payload = f.bytes;
    if (f.field == 5) sig = f.bytes;
  }
  if (pk.empty() || sig.empty()) throw NetError("voucher: malformed envelope");
  const PublicKey key = PublicKey::unmarshal(pk);
  if (!(PeerId::from_public_key(key) == relay)) throw NetError("voucher: not signed by the relay");
  if (type != voucher_type()) throw NetError("voucher: wrong payload type");
  if (!key.verify(envelope_signed_data(type, payload), sig))
    throw NetError("voucher: bad signature");
  PeerId vr, vp;
  uint64_t exp = 0;
  for (auto& f : pb_parse(payload)) {
    if (f.field == 1 && f.wire == 2) vr = PeerId::from_bytes(f.bytes);
    if (f.field == 2 && f.wire == 2) vp = PeerId::from_bytes(f.bytes);
    if (f.field == 3 && f.wire == 0) exp = f.varint;
  }
  if (!(vr == relay) || !(vp == peer) || exp != expire)
    throw NetError("voucher: fields do not match the reservation");
}

Bytes test_make_voucher(const PrivateKey& key, const PeerId& relay, const PeerId& peer,
                        uint64_t expire) {
  return make_voucher(key, relay, peer, expire);
}

namespace {
Bytes hop_status(int status, const Bytes& extra = Bytes()) {
  PbWriter w;
  w.varint_field(1, HOP_STATUS);
  append(w.buf, extra);
  w.varint_field(5, (uint64_t)status);
  return w.buf;
}

void splice(std::shared_ptr<BufConn> from, std::shared_ptr<BufConn> to, uint64_t limit,
            StreamPtr a, StreamPtr b) {
  uint8_t buf[16384];
  uint64_t moved = 0;
  try {
    while (true) {
      size_t r = from->read_some(buf, sizeof(buf));
      if (r == 0) {
        to->close_write();
        return;
      }
      moved += r;
      if (limit && moved > limit) throw NetError("relay data limit");
      to->write_all(buf, r);
    }
  } catch (...) {
    a->reset();
    b->reset();
  }
}
}  // namespace

// ================================================================ hop service
RelayService::RelayService(std::shared_ptr<Host> h, RelayResources r) : h_(std::move(h)), res_(r) {
  h_->set_stream_handler(kHopProto, [this](StreamCtx& c) { on_hop(c); });
}

size_t RelayService::reservations() {
  std::lock_guard<std::mutex> lk(mu_);
  return resv_.size();
}

void RelayService::on_hop(StreamCtx& c) {
  c.io->set_read_timeout(30000);
  RelayMsg m;
  try {
    m = parse(c.io->read_frame(4096), true);
  } catch (...) {
    write_frame(*c.io, hop_status(RS_MALFORMED_MESSAGE));
    c.stream->close();
    return;
  }
  const int64_t now = (int64_t)time(nullptr);
  if (m.type == HOP_RESERVE) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = resv_.begin(); it != resv_.end();)
        it = it->second < now ? resv_.erase(it) : std::next(it);
      if (!resv_.count(c.peer) && (int)resv_.size() >= res_.max_reservations) {
        write_frame(*c.io, hop_status(RS_RESERVATION_REFUSED));
        c.stream->close();
        return;
      }
      resv_[c.peer] = now + res_.reservation_ttl_s;
    }
    PbWriter rv;
    const uint64_t expire = (uint64_t)(now + res_.reservation_ttl_s);
    rv.varint_field(1, expire);
    for (auto& a : h_->addrs()) rv.bytes_field(2, a.with_peer(h_->id()).bytes());
    rv.bytes_field(3, make_voucher(h_->key(), h_->id(), c.peer, expire));
    PbWriter extra;
    extra.bytes_field(3, rv.buf);
    extra.bytes_field(4, limit_pb(res_.limit_duration_s, res_.limit_data));
    write_frame(*c.io, hop_status(RS_OK, extra.buf));
    c.stream->close();
    logf("relay: reservation for %s", c.peer.to_base58().c_str());
    return;
  }
  if (m.type != HOP_CONNECT) {
    write_frame(*c.io, hop_status(RS_UNEXPECTED_MESSAGE));
    c.stream->close();
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = resv_.find(m.peer);
    if (it == resv_.end() || it->second < now) {
      write_frame(*c.io, hop_status(RS_NO_RESERVATION));
      c.stream->close();
      return;
    }
  }
  if (circuits_.load() >= res_.max_circuits) {
    write_frame(*c.io, hop_status(RS_RESOURCE_LIMIT_EXCEEDED));
    c.stream->close();
    return;
  }
  StreamCtx dst;
  try {
    dst = h_->new_stream(m.peer, kStopProto, 10000);
    PbWriter w;
    w.varint_field(1, STOP_CONNECT);
    w.bytes_field(2, peer_pb(c.peer, {}));
    w.bytes_field(3, limit_pb(res_.limit_duration_s, res_.limit_data));
    write_frame(*dst.io, w.buf);
    dst.io->set_read_timeout(10000);
    RelayMsg r = parse(dst.io->read_frame(4096), false);
    if (r.type != STOP_STATUS || r.status != RS_OK) throw NetError("stop refused");
    dst.io->set_read_timeout(0);
  } catch (...) {
    if (dst.stream) dst.stream->reset();
    write_frame(*c.io, hop_status(RS_CONNECTION_FAILED));
    c.stream->close();
    return;
  }
  PbWriter extra;
  extra.bytes_field(4, limit_pb(res_.limit_duration_s, res_.limit_data));
  write_frame(*c.io, hop_status(RS_OK, extra.buf));
  c.io->set_read_timeout(res_.limit_duration_s * 1000);
  dst.io->set_read_timeout(res_.limit_duration_s * 1000);
  circuits_++;
  auto src_io = c.io, dst_io = dst.io;
  auto sa = c.stream, sb = dst.stream;
  uint64_t lim = res_.limit_data;
  std::thread t([dst_io, src_io, lim, sa, sb] { splice(dst_io, src_io, lim, sa, sb); });
  splice(src_io, dst_io, lim, sa, sb);
  t.join();
  circuits_--;
}

// ================================================================ client
RelayClient::RelayClient(std::shared_ptr<Host> h) : h_(std::move(h)) {
  h_->set_stream_handler(kStopProto, [this](StreamCtx& c) { on_stop(c); });
  std::weak_ptr<Host> wh = h_;
  h_->relay_dialer = [this](const Multiaddr& relay, const PeerId& target, int timeout_ms) {
    return dial(relay, target, timeout_ms);
  };
}

int64_t RelayClient::reserve(const Multiaddr& relay_addr, int timeout_ms) {
  PeerId rid;
  Multiaddr bare = relay_addr.without_peer(&rid);
  if (rid.empty()) throw NetError("relay address needs /p2p/<relay id>");
  h_->connect(rid, {bare}, timeout_ms);
  StreamCtx c = h_->new_stream(rid, kHopProto, timeout_ms);
  PbWriter w;
  w.varint_field(1, HOP_RESERVE);
  write_frame(*c.io, w.buf);
  c.io->set_read_timeout(timeout_ms);
  RelayMsg r = parse(c.io->read_frame(8192), true);
  c.stream->close();
  if (r.type != HOP_STATUS || r.status != RS_OK)
    throw NetError("relay reservation refused (status " + std::to_string(r.status) + ")");
  // A voucher, when present, must verify (signed by the relay, for this reservation).  A
  // missing one is accepted with a warning: interop with every relay implementation is
  // not proven, and the reservation itself is authenticated by the secure channel.
  if (r.voucher.empty())
    logf("relay %s: reservation without a voucher (accepted)", rid.to_base58().c_str());
  else
    verify_voucher(r.voucher, rid, h_->id(), r.expire);
  h_->add_advertised_addr(
      Multiaddr::parse(bare.str() + "/p2p/" + rid.to_base58() + "/p2p-circuit"));
  return (int64_t)r.expire;
}

SessionPtr RelayClient::dial(const Multiaddr& relay_addr, const PeerId& target, int timeout_ms) {
  PeerId rid;
  Multiaddr bare = relay_addr.without_peer(&rid);
  if (rid.empty()) throw NetError("circuit address needs the relay's /p2p/<id>");
  h_->connect(rid, bare.empty() ? std::vector<Multiaddr>{} : std::vector<Multiaddr>{bare},
              timeout_ms);
  StreamCtx c = h_->new_stream(rid, kHopProto, timeout_ms);
  PbWriter w;
  w.varint_field(1, HOP_CONNECT);
  w.bytes_field(2, peer_pb(target, {}));
  write_frame(*c.io, w.buf);
  c.io->set_read_timeout(timeout_ms);
  RelayMsg r = parse(c.io->read_frame(8192), true);
  if (r.type != HOP_STATUS || r.status != RS_OK) {
    c.stream->reset();
    throw NetError("relay connect failed (status " + std::to_string(r.status) + ")");
  }
  c.io->set_read_timeout(0);
  return h_->upgrade_outbound(c.io, target, true);
}

void RelayClient::on_stop(StreamCtx& c) {
  c.io->set_read_timeout(10000);
  RelayMsg m;
  try {
    m = parse(c.io->read_frame(4096), false);
  } catch (...) {
    c.stream->reset();
    return;
  }
  PbWriter w;
  w.varint_field(1, STOP_STATUS);
  if (m.type != STOP_CONNECT || m.peer.empty()) {
    w.varint_field(4, RS_MALFORMED_MESSAGE);
    write_frame(*c.io, w.buf);
    c.stream->close();
    return;
  }
  w.varint_field(4, RS_OK);
  write_frame(*c.io, w.buf);
  c.io->set_read_timeout(0);
  try {
    h_->upgrade_inbound(c.io, true);
  } catch (...) {
    c.stream->reset();
  }
}

}  // namespace p2p
