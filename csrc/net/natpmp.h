// NAT-PMP (RFC 6886) port mapping: the reference enables go-libp2p's
// `libp2p.NATPortMap()` (`go/cmd/node/main.go:143`), which maps
// the node's TCP listen port on the home gateway and advertises the external
// address.  This is the NAT-PMP half of that (UPnP-IGD is not built): gateway
// discovery from the default route, external-address and TCP-mapping requests
// over UDP/5351 with the RFC's retry schedule, renewal at half the lifetime,
// and deletion on shutdown.
#pragma once
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace p2p {

struct NatMapping {
  int internal_port = 0;
  int external_port = 0;
  unsigned lifetime = 0;
};

class NatPmp {
 public:
  // gateway "ip" or "ip:port" (default: the IPv4 default route's gateway, port 5351)
  explicit NatPmp(std::string gateway = "", int timeout_ms = 1000);
  ~NatPmp();
  bool ok() const { return !gw_ip_.empty(); }
  std::string gateway() const { return gw_ip_ + ":" + std::to_string(gw_port_); }
  // Returns "" on failure.
  std::string external_address();
  // Maps TCP internal_port; false on failure or a non-zero result code.
  bool map_tcp(int internal_port, int suggested_external, unsigned lifetime, NatMapping* out);
  bool unmap_tcp(int internal_port);
  // Keeps the mappings alive (renew at lifetime/2) until stop(); unmaps on stop.
  void keep_alive(std::vector<NatMapping> maps);
  void stop();

  static std::string default_gateway();  // from /proc/net/route, "" if none

 private:
  bool request(const unsigned char* req, size_t n, unsigned char* resp, size_t resp_n,
               unsigned char want_op);
  std::string gw_ip_;
  int gw_port_ = 5351;
  int timeout_ms_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::vector<NatMapping> maps_;
};

}  // namespace p2p
