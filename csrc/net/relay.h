// Circuit relay v2: the hop service (`go/cmd/relay/main.go:30-47`, which the
// reference ships but never wires) and the client side the node uses to
// reserve a slot on a relay, accept relayed connections (stop protocol) and
// dial peers through /p2p-circuit addresses.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "host.h"

namespace p2p {

extern const char* kHopProto;   // "/libp2p/circuit/relay/0.2.0/hop"
extern const char* kStopProto;  // "/libp2p/circuit/relay/0.2.0/stop"

enum RelayStatus : int {
  RS_OK = 100, RS_RESERVATION_REFUSED = 200, RS_RESOURCE_LIMIT_EXCEEDED = 201,
  RS_PERMISSION_DENIED = 202, RS_CONNECTION_FAILED = 203, RS_NO_RESERVATION = 204,
  RS_MALFORMED_MESSAGE = 400, RS_UNEXPECTED_MESSAGE = 401,
};

struct RelayResources {  // go-libp2p relayv2.DefaultResources()
  int reservation_ttl_s = 3600;
  int max_reservations = 128;
  int max_circuits = 16;
  int limit_duration_s = 120;
  uint64_t limit_data = 1 << 17;
};

// Reservation vouchers (signed envelopes, domain "libp2p-relay-rsvp"): verify throws
// NetError unless `env` is a ReservationVoucher for (relay, peer, expire) signed by relay.
void verify_voucher(const Bytes& env, const PeerId& relay, const PeerId& peer, uint64_t expire);
Bytes test_make_voucher(const PrivateKey& key, const PeerId& relay, const PeerId& peer,
                        uint64_t expire);

class RelayService {
 public:
  RelayService(std::shared_ptr<Host> h, RelayResources r = RelayResources());
  size_t reservations();
  size_t active_circuits() const { return circuits_; }

 private:
  void on_hop(StreamCtx& c);
  std::shared_ptr<Host> h_;
  RelayResources res_;
  std::mutex mu_;
  std::map<PeerId, int64_t> resv_;  // peer -> expiry (unix s)
  std::atomic<int> circuits_{0};
};

class RelayClient {
 public:
  explicit RelayClient(std::shared_ptr<Host> h);
  // Reserve a slot; on success the host advertises <relay>/p2p-circuit.  Returns expiry.
  int64_t reserve(const Multiaddr& relay_addr, int timeout_ms = 10000);
  SessionPtr dial(const Multiaddr& relay_addr, const PeerId& target, int timeout_ms);

 private:
  void on_stop(StreamCtx& c);
  std::shared_ptr<Host> h_;
};

}  // namespace p2p
