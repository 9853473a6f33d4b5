// UPnP Internet Gateway Device port mapping: the UPnP half of go-libp2p's
// `libp2p.NATPortMap()` (`go/cmd/node/main.go:143`; NAT-PMP is
// natpmp.h).  SSDP discovery (M-SEARCH to 239.255.255.250:1900, or unicast to a
// configured responder), the device description's WANIPConnection /
// WANPPPConnection control URL, and the SOAP actions GetExternalIPAddress,
// AddPortMapping (renewed at half the lease) and DeletePortMapping on shutdown.
#pragma once
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "natpmp.h"  // NatMapping

namespace p2p {

class UpnpIgd {
 public:
  // where: "" = SSDP multicast discovery; "ip:port" = unicast M-SEARCH to that
  // responder; "http://..." = the device description URL (no SSDP).
  explicit UpnpIgd(std::string where = "", int timeout_ms = 2000);
  ~UpnpIgd();
  // Finds the gateway's WAN connection service; false if none answered.
  bool discover();
  const std::string& control_url() const { return control_url_; }
  std::string external_address();  // "" on failure
  bool map_tcp(int internal_port, int external_port, unsigned lease_s, NatMapping* out);
  bool unmap_tcp(int external_port);
  void keep_alive(std::vector<NatMapping> maps);  // renew at lease/2; unmap on stop()
  void stop();

  // helpers (exposed for tests)
  static std::string xml_text(const std::string& xml, const std::string& tag, size_t from = 0);
  static std::string resolve_url(const std::string& base, const std::string& ref);

 private:
  bool soap(const std::string& action, const std::string& args, std::string* resp);
  std::string where_;
  int timeout_ms_;
  std::string location_, control_url_, service_type_, local_ip_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::vector<NatMapping> maps_;
};

}  // namespace p2p
