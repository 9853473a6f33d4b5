#include "natpmp.h"

#include <arpa/inet.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <fstream>
#include <sstream>

#include "util.h"

namespace p2p {

std::string NatPmp::default_gateway() {
  std::ifstream f("/proc/net/route");
  std::string line;
  std::getline(f, line);  // header
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::string iface, dest, gw;
    ss >> iface >> dest >> gw;
    if (dest == "00000000" && gw != "00000000" && gw.size() == 8) {
      const unsigned v = (unsigned)strtoul(gw.c_str(), nullptr, 16);  // little-endian
      char buf[32];
      snprintf(buf, sizeof(buf), "%u.%u.%u.%u", v & 255, (v >> 8) & 255, (v >> 16) & 255,
               (v >> 24) & 255);
      return buf;
    }
  }
  return "";
}

NatPmp::NatPmp(std::string gateway, int timeout_ms) : timeout_ms_(timeout_ms) {
  if (gateway.empty()) gateway = default_gateway();
  const size_t c = gateway.rfind(':');
  if (c != std::string::npos) {
    gw_port_ = atoi(gateway.c_str() + c + 1);
    gateway = gateway.substr(0, c);
  }
  gw_ip_ = gateway;
}

NatPmp::~NatPmp() { stop(); }

// RFC 6886 §3.1: retransmit at 250 ms doubling; we cap the total wait at timeout_ms.
bool NatPmp::request(const unsigned char* req, size_t n, unsigned char* resp, size_t resp_n,
                     unsigned char want_op) {
  if (gw_ip_.empty()) return false;
  const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return false;
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)gw_port_);
  if (inet_pton(AF_INET, gw_ip_.c_str(), &sa.sin_addr) != 1 ||
      connect(fd, (sockaddr*)&sa, sizeof(sa)) != 0) {
    close(fd);
    return false;
  }
  bool ok = false;
  int wait = 250, spent = 0;
  while (!ok && spent < timeout_ms_) {
    if (send(fd, req, n, 0) != (ssize_t)n) break;
    const int w = std::min(wait, timeout_ms_ - spent);
    pollfd p{fd, POLLIN, 0};
    if (poll(&p, 1, w) > 0) {
      const ssize_t got = recv(fd, resp, resp_n, 0);
      ok = got >= 8 && resp[0] == 0 && resp[1] == want_op;
    }
    spent += w;
    wait *= 2;
  }
  close(fd);
  return ok;
}

std::string NatPmp::external_address() {
  const unsigned char req[2] = {0, 0};
  unsigned char r[16] = {};
  if (!request(req, 2, r, sizeof(r), 128)) return "";
  if (((r[2] << 8) | r[3]) != 0) return "";
  char buf[32];
  snprintf(buf, sizeof(buf), "%u.%u.%u.%u", r[8], r[9], r[10], r[11]);
  return buf;
}

bool NatPmp::map_tcp(int internal_port, int suggested_external, unsigned lifetime,
                     NatMapping* out) {
  unsigned char req[12] = {0, 2, 0, 0};
  req[4] = (unsigned char)(internal_port >> 8);
  req[5] = (unsigned char)internal_port;
  req[6] = (unsigned char)(suggested_external >> 8);
  req[7] = (unsigned char)suggested_external;
  req[8] = (unsigned char)(lifetime >> 24);
  req[9] = (unsigned char)(lifetime >> 16);
  req[10] = (unsigned char)(lifetime >> 8);
  req[11] = (unsigned char)lifetime;
  unsigned char r[16] = {};
  if (!request(req, sizeof(req), r, sizeof(r), 130)) return false;
  if (((r[2] << 8) | r[3]) != 0) return false;
  if (out) {
    out->internal_port = (r[8] << 8) | r[9];
    out->external_port = (r[10] << 8) | r[11];
    out->lifetime = ((unsigned)r[12] << 24) | ((unsigned)r[13] << 16) | ((unsigned)r[14] << 8) | r[15];
  }
  return true;
}

bool NatPmp::unmap_tcp(int internal_port) { return map_tcp(internal_port, 0, 0, nullptr); }

void NatPmp::keep_alive(std::vector<NatMapping> maps) {
  std::lock_guard<std::mutex> lk(mu_);
  maps_ = std::move(maps);
  if (th_.joinable() || maps_.empty()) return;
  th_ = std::thread([this] {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      unsigned life = 3600;
      for (auto& m : maps_) life = std::min(life, std::max(m.lifetime, 2u));
      cv_.wait_for(lk, std::chrono::seconds(life / 2), [this] { return stop_; });
      if (stop_) break;
      for (auto& m : maps_) {
        NatMapping n;
        if (map_tcp(m.internal_port, m.external_port, m.lifetime ? m.lifetime : 3600, &n)) m = n;
      }
    }
  });
}

void NatPmp::stop() {
  std::vector<NatMapping> maps;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_) return;
    stop_ = true;
    maps = maps_;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  for (auto& m : maps) unmap_tcp(m.internal_port);
}

}  // namespace p2p
