// UPnP-IGD port mapping -- see upnp.h.
#include "upnp.h"

#include <arpa/inet.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>

#include "http.h"
#include "util.h"

namespace p2p {

namespace {

const char* kSearchTargets[] = {"urn:schemas-upnp-org:device:InternetGatewayDevice:1",
                                "urn:schemas-upnp-org:device:InternetGatewayDevice:2"};
const char* kServices[] = {"urn:schemas-upnp-org:service:WANIPConnection:2",
                           "urn:schemas-upnp-org:service:WANIPConnection:1",
                           "urn:schemas-upnp-org:service:WANPPPConnection:1"};

std::string lower_s(std::string s) {
  std::transform(s.begin(), s.end(), s.begin(), [](unsigned char c) { return (char)tolower(c); });
  return s;
}

// "LOCATION:" header of an SSDP response
std::string ssdp_location(const std::string& resp) {
  const std::string l = lower_s(resp);
  size_t p = l.find("\nlocation:");
  if (p == std::string::npos) return "";
  p += 10;
  size_t e = resp.find('\r', p);
  if (e == std::string::npos) e = resp.find('\n', p);
  std::string v = resp.substr(p, e == std::string::npos ? std::string::npos : e - p);
  v.erase(0, v.find_first_not_of(" \t"));
  while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.pop_back();
  return v;
}

// the local address the kernel would use to reach host:port
std::string local_ip_towards(const std::string& host, int port) {
  const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return "";
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  std::string out;
  if (inet_pton(AF_INET, host.c_str(), &sa.sin_addr) == 1 &&
      connect(fd, (sockaddr*)&sa, sizeof(sa)) == 0) {
    sockaddr_in me{};
    socklen_t sl = sizeof(me);
    if (getsockname(fd, (sockaddr*)&me, &sl) == 0) {
      char buf[INET_ADDRSTRLEN];
      inet_ntop(AF_INET, &me.sin_addr, buf, sizeof(buf));
      out = buf;
    }
  }
  close(fd);
  return out;
}

}  // namespace

std::string UpnpIgd::xml_text(const std::string& xml, const std::string& tag, size_t from) {
  // namespace-agnostic: <tag>, <ns:tag> or <tag attr...>
  size_t p = from;
  while (true) {
    p = xml.find(tag, p);
    if (p == std::string::npos) return "";
    const bool open_ok = p > 0 && (xml[p - 1] == '<' || xml[p - 1] == ':');
    const size_t after = p + tag.size();
    if (open_ok && after < xml.size() && (xml[after] == '>' || xml[after] == ' ')) {
      const size_t lt = xml.rfind('<', p);
      if (lt != std::string::npos && xml[lt + 1] != '/') {
        const size_t gt = xml.find('>', after);
        if (gt == std::string::npos) return "";
        const size_t end = xml.find('<', gt + 1);
        if (end == std::string::npos) return "";
        std::string v = xml.substr(gt + 1, end - gt - 1);
        v.erase(0, v.find_first_not_of(" \t\r\n"));
        while (!v.empty() && isspace((unsigned char)v.back())) v.pop_back();
        return v;
      }
    }
    p = after;
  }
}

std::string UpnpIgd::resolve_url(const std::string& base, const std::string& ref) {
  if (ref.rfind("http://", 0) == 0) return ref;
  const size_t hs = base.find("://");
  const size_t path = base.find('/', hs == std::string::npos ? 0 : hs + 3);
  const std::string origin = path == std::string::npos ? base : base.substr(0, path);
  if (!ref.empty() && ref[0] == '/') return origin + ref;
  const std::string dir = path == std::string::npos ? "/" : base.substr(path, base.rfind('/') - path + 1);
  return origin + dir + ref;
}

UpnpIgd::UpnpIgd(std::string where, int timeout_ms) : where_(std::move(where)), timeout_ms_(timeout_ms) {}

UpnpIgd::~UpnpIgd() { stop(); }

bool UpnpIgd::discover() {
  if (where_.rfind("http://", 0) == 0) {
    location_ = where_;
  } else {
    std::string host = "239.255.255.250";
    int port = 1900;
    if (!where_.empty()) split_host_port(where_, &host, &port);
    const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return false;
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host.c_str(), &sa.sin_addr) != 1) {
      close(fd);
      return false;
    }
    for (const char* st : kSearchTargets) {
      const std::string msg = std::string("M-SEARCH * HTTP/1.1\r\nHOST: 239.255.255.250:1900\r\n") +
                              "MAN: \"ssdp:discover\"\r\nMX: 1\r\nST: " + st + "\r\n\r\n";
      sendto(fd, msg.data(), msg.size(), 0, (sockaddr*)&sa, sizeof(sa));
    }
    int left = timeout_ms_;
    while (left > 0 && location_.empty()) {
      pollfd p{fd, POLLIN, 0};
      const int step = std::min(left, 250);
      if (poll(&p, 1, step) > 0) {
        char buf[2048];
        const ssize_t n = recv(fd, buf, sizeof(buf) - 1, 0);
        if (n > 0) location_ = ssdp_location(std::string(buf, (size_t)n));
      }
      left -= step;
    }
    close(fd);
    if (location_.empty()) return false;
  }
  HttpResult d;
  try {
    d = http_request("GET", location_, "", "", timeout_ms_);
  } catch (const std::exception&) {
    return false;
  }
  if (d.status != 200) return false;
  const std::string base = xml_text(d.body, "URLBase");
  for (const char* svc : kServices) {
    size_t p = d.body.find(std::string(">") + svc + "<");
    if (p == std::string::npos) continue;
    const std::string ctl = xml_text(d.body, "controlURL", p);
    if (ctl.empty()) continue;
    service_type_ = svc;
    control_url_ = resolve_url(base.empty() ? location_ : base, ctl);
    break;
  }
  if (control_url_.empty()) return false;
  // the address the gateway reaches us on (host part of the control URL)
  std::string hp = control_url_.substr(7);
  hp = hp.substr(0, hp.find('/'));
  std::string h;
  int port = 80;
  if (hp.find(':') != std::string::npos) split_host_port(hp, &h, &port);
  else h = hp;
  local_ip_ = local_ip_towards(h, port);
  return !local_ip_.empty();
}

bool UpnpIgd::soap(const std::string& action, const std::string& args, std::string* resp) {
  if (control_url_.empty()) return false;
  const std::string body =
      "<?xml version=\"1.0\"?>\r\n<s:Envelope xmlns:s=\"http://schemas.xmlsoap.org/soap/envelope/\" "
      "s:encodingStyle=\"http://schemas.xmlsoap.org/soap/encoding/\"><s:Body><u:" + action +
      " xmlns:u=\"" + service_type_ + "\">" + args + "</u:" + action + "></s:Body></s:Envelope>\r\n";
  try {
    HttpResult r = http_request("POST", control_url_, body, "text/xml; charset=\"utf-8\"", timeout_ms_,
                                {{"SOAPAction", "\"" + service_type_ + "#" + action + "\""}});
    if (resp) *resp = r.body;
    return r.status == 200;
  } catch (const std::exception&) {
    return false;
  }
}

std::string UpnpIgd::external_address() {
  std::string r;
  if (!soap("GetExternalIPAddress", "", &r)) return "";
  return xml_text(r, "NewExternalIPAddress");
}

bool UpnpIgd::map_tcp(int internal_port, int external_port, unsigned lease_s, NatMapping* out) {
  const std::string args =
      "<NewRemoteHost></NewRemoteHost><NewExternalPort>" + std::to_string(external_port) +
      "</NewExternalPort><NewProtocol>TCP</NewProtocol><NewInternalPort>" +
      std::to_string(internal_port) + "</NewInternalPort><NewInternalClient>" + local_ip_ +
      "</NewInternalClient><NewEnabled>1</NewEnabled><NewPortMappingDescription>p2p-llm-chat"
      "</NewPortMappingDescription><NewLeaseDuration>" + std::to_string(lease_s) +
      "</NewLeaseDuration>";
  if (!soap("AddPortMapping", args, nullptr)) return false;
  if (out) {
    out->internal_port = internal_port;
    out->external_port = external_port;
    out->lifetime = lease_s;
  }
  return true;
}

bool UpnpIgd::unmap_tcp(int external_port) {
  return soap("DeletePortMapping",
              "<NewRemoteHost></NewRemoteHost><NewExternalPort>" + std::to_string(external_port) +
                  "</NewExternalPort><NewProtocol>TCP</NewProtocol>",
              nullptr);
}

void UpnpIgd::keep_alive(std::vector<NatMapping> maps) {
  std::lock_guard<std::mutex> lk(mu_);
  maps_ = std::move(maps);
  if (th_.joinable() || maps_.empty()) return;
  th_ = std::thread([this] {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      unsigned lease = 3600;
      for (auto& m : maps_) lease = std::min(lease, std::max(m.lifetime, 2u));
      cv_.wait_for(lk, std::chrono::seconds(lease / 2), [this] { return stop_; });
      if (stop_) break;
      for (auto& m : maps_) map_tcp(m.internal_port, m.external_port, m.lifetime, nullptr);
    }
  });
}

void UpnpIgd::stop() {
  std::vector<NatMapping> maps;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_) return;
    stop_ = true;
    maps = maps_;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  for (auto& m : maps) unmap_tcp(m.external_port);
}

}  // namespace p2p
