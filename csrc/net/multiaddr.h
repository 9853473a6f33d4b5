// multiaddr (string <-> binary) for the protocols a chat node meets:
// ip4, ip6, dns, dns4, dns6, tcp, udp, quic, quic-v1, p2p, p2p-circuit, ws, wss, tls, noise.
#pragma once
#include <string>
#include <vector>

#include "crypto.h"
#include "util.h"

namespace p2p {

enum : uint32_t {
  MA_IP4 = 4, MA_TCP = 6, MA_DNS = 53, MA_DNS4 = 54, MA_DNS6 = 55, MA_IP6 = 41, MA_UDP = 273,
  MA_P2P_CIRCUIT = 290, MA_P2P = 421, MA_TLS = 448, MA_NOISE = 454, MA_QUIC = 460,
  MA_QUIC_V1 = 461, MA_WS = 477, MA_WSS = 478,
};

struct MaComponent {
  uint32_t code;
  Bytes value;
};

class Multiaddr {
 public:
  Multiaddr() = default;
  static Multiaddr parse(const std::string& s);  // throws NetError
  static Multiaddr from_bytes(const Bytes& b);
  std::string str() const;
  Bytes bytes() const;
  const std::vector<MaComponent>& parts() const { return parts_; }
  bool empty() const { return parts_.empty(); }

  Multiaddr encapsulate(const Multiaddr& o) const;
  Multiaddr with_peer(const PeerId& id) const;  // appends /p2p/<id>
  // Strips a trailing /p2p/<id> (returns it through *id when present).
  Multiaddr without_peer(PeerId* id = nullptr) const;
  bool has(uint32_t code) const;
  // The address before the first /p2p-circuit and the target after it.
  bool split_circuit(Multiaddr* relay, Multiaddr* target) const;
  // For /ip4|ip6|dns*/.../tcp/<port>: host + port.
  bool tcp_host_port(std::string* host, int* port) const;
  // For /ip4/<a>/udp/<port>/quic-v1: host + port.
  bool quic_host_port(std::string* host, int* port) const;
  bool operator==(const Multiaddr& o) const { return bytes() == o.bytes(); }

 private:
  std::vector<MaComponent> parts_;
};

}  // namespace p2p
