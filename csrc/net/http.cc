#include "http.h"

#include <ctype.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <chrono>

namespace p2p {

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      o += (char)c;
    } else {
      o += '%';
      o += hex[c >> 4];
      o += hex[c & 15];
    }
  }
  return o;
}

std::string url_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '+') {
      o += ' ';
    } else if (s[i] == '%' && i + 2 < s.size() && isxdigit((unsigned char)s[i + 1]) &&
               isxdigit((unsigned char)s[i + 2])) {
      o += (char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16);
      i += 2;
    } else {
      o += s[i];
    }
  }
  return o;
}

static std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

static std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

static std::map<std::string, std::string> parse_query(const std::string& q) {
  std::map<std::string, std::string> out;
  size_t i = 0;
  while (i <= q.size()) {
    size_t amp = q.find('&', i);
    if (amp == std::string::npos) amp = q.size();
    std::string kv = q.substr(i, amp - i);
    if (!kv.empty()) {
      size_t eq = kv.find('=');
      std::string k = url_decode(kv.substr(0, eq));
      std::string v = eq == std::string::npos ? "" : url_decode(kv.substr(eq + 1));
      if (!out.count(k)) out[k] = v;  // first value wins (Go's Query().Get)
    }
    i = amp + 1;
  }
  return out;
}

std::string HttpRequest::header(const std::string& k) const {
  auto it = headers.find(lower(k));
  return it == headers.end() ? "" : it->second;
}

std::string HttpRequest::param(const std::string& k, const std::string& def) const {
  auto it = query.find(k);
  return it == query.end() ? def : it->second;
}

void HttpResponse::set_header(const std::string& k, const std::string& v) {
  for (auto& h : headers)
    if (lower(h.first) == lower(k)) {
      h.second = v;
      return;
    }
  headers.emplace_back(k, v);
}

void HttpResponse::json(int code, const Json& j, bool sorted_keys) {
  status = code;
  body = sorted_keys ? j.dump_sorted() : j.dump();
  set_header("Content-Type", "application/json; charset=utf-8");
}

void HttpResponse::text(int code, const std::string& s) {
  status = code;
  body = s;
  set_header("Content-Type", "text/plain; charset=utf-8");
}

static const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 408: return "Request Timeout";
    case 413: return "Payload Too Large";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
  }
  return "Status";
}

void split_host_port(const std::string& addr, std::string* host, int* port) {
  if (!addr.empty() && addr[0] == '[') {
    size_t rb = addr.find(']');
    *host = addr.substr(1, rb - 1);
    *port = atoi(addr.c_str() + rb + 2);
    return;
  }
  size_t c = addr.rfind(':');
  if (c == std::string::npos) throw NetError("address missing port: " + addr);
  *host = addr.substr(0, c);
  *port = atoi(addr.c_str() + c + 1);
  if (host->empty()) *host = "0.0.0.0";
}

// ================================================================ server
HttpServer::~HttpServer() { stop(); }

void HttpServer::route(const std::string& method, const std::string& path, HttpHandler h) {
  routes_[method + " " + path] = std::move(h);
}

int HttpServer::start(const std::string& addr) {
  std::string host;
  int port;
  split_host_port(addr, &host, &port);
  listener_ = std::make_shared<TcpListener>(host, port);
  port_ = listener_->port();
  accept_thread_ = std::thread([this] {
    while (!stopped_) {
      auto c = listener_->accept();
      if (!c) break;
      {
        std::lock_guard<std::mutex> lk(mu_);
        conns_.push_back(c);
        if (conns_.size() > 1024) {
          std::vector<std::weak_ptr<TcpConn>> keep;
          for (auto& w : conns_)
            if (!w.expired()) keep.push_back(w);
          conns_.swap(keep);
        }
      }
      active_++;
      std::thread([this, c] {
        conn_loop(c);
        active_--;
      }).detach();
    }
    std::lock_guard<std::mutex> lk(mu_);
    accept_exited_ = true;
    exit_cv_.notify_all();
  });
  return port_;
}

void HttpServer::serve_forever() {
  if (!listener_) return;  // never started
  std::unique_lock<std::mutex> lk(mu_);
  exit_cv_.wait(lk, [this] { return accept_exited_; });
}

void HttpServer::stop() {
  if (stopped_.exchange(true)) return;
  if (listener_) listener_->close();
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& w : conns_)
      if (auto c = w.lock()) c->close();
  }
  if (accept_thread_.joinable()) accept_thread_.join();
  for (int i = 0; i < 500 && active_.load() > 0; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
}

static std::string read_line(BufConn& c, size_t max = 16384) {
  std::string s;
  while (true) {
    uint8_t b;
    if (c.read_some(&b, 1) == 0) {
      if (s.empty()) throw NetError("eof");
      return s;
    }
    if (b == '\n') {
      if (!s.empty() && s.back() == '\r') s.pop_back();
      return s;
    }
    s += (char)b;
    if (s.size() > max) throw NetError("line too long");
  }
}

void HttpServer::conn_loop(std::shared_ptr<TcpConn> c) {
  BufConn bc(c);
  c->set_read_timeout(120000);
  try {
    while (!stopped_ && handle_one(bc, *c)) {
    }
  } catch (...) {
  }
  c->close();
}

bool HttpServer::handle_one(BufConn& bc, TcpConn& raw) {
  std::string line = read_line(bc);
  auto t0 = std::chrono::steady_clock::now();
  HttpRequest req;
  req.remote = raw.remote_addr();
  {
    size_t a = line.find(' '), b = line.rfind(' ');
    if (a == std::string::npos || b == a) throw NetError("bad request line");
    req.method = line.substr(0, a);
    std::string target = line.substr(a + 1, b - a - 1);
    req.version = line.substr(b + 1);
    size_t q = target.find('?');
    req.path = url_decode(target.substr(0, q));
    if (q != std::string::npos) req.query_string = target.substr(q + 1);
    req.query = parse_query(req.query_string);
  }
  while (true) {
    std::string h = read_line(bc);
    if (h.empty()) break;
    size_t colon = h.find(':');
    if (colon == std::string::npos) continue;
    req.headers[lower(trim(h.substr(0, colon)))] = trim(h.substr(colon + 1));
  }
  HttpResponse res;
  bool too_large = false;
  if (lower(req.header("transfer-encoding")).find("chunked") != std::string::npos) {
    while (true) {
      std::string sz = read_line(bc);
      size_t n = strtoul(sz.c_str(), nullptr, 16);
      if (n == 0) {
        while (!read_line(bc).empty()) {
        }
        break;
      }
      if (req.body.size() + n > max_body) throw NetError("body too large");
      Bytes chunk = bc.read_exact(n);
      req.body.append(chunk.begin(), chunk.end());
      read_line(bc);
    }
  } else if (!req.header("content-length").empty()) {
    size_t n = strtoull(req.header("content-length").c_str(), nullptr, 10);
    if (n > max_body) {
      too_large = true;
    } else {
      Bytes b = bc.read_exact(n);
      req.body.assign(b.begin(), b.end());
    }
  }
  bool keep = lower(req.header("connection")) != "close" && req.version == "HTTP/1.1";
  if (too_large) {
    res.text(413, "request body too large");
    keep = false;
  } else {
    auto it = routes_.find(req.method + " " + req.path);
    if (it == routes_.end()) {
      if (req.method == "HEAD") it = routes_.find("GET " + req.path);
    }
    if (it == routes_.end()) {
      res.text(404, "404 page not found");
    } else {
      try {
        it->second(req, res);
      } catch (const std::exception& e) {
        // gin Recovery middleware: 500 with empty body
        logf("[Recovery] panic recovered: %s", e.what());
        res = HttpResponse();
        res.status = 500;
      }
    }
  }
  std::string head = "HTTP/1.1 " + std::to_string(res.status) + " " + reason(res.status) + "\r\n";
  char date[64];
  time_t now = time(nullptr);
  struct tm gm;
  gmtime_r(&now, &gm);
  strftime(date, sizeof(date), "%a, %d %b %Y %H:%M:%S GMT", &gm);
  head += std::string("Date: ") + date + "\r\n";
  for (auto& h : res.headers) head += h.first + ": " + h.second + "\r\n";
  if (res.stream) {
    head += "Transfer-Encoding: chunked\r\n";
    head += keep ? "" : "Connection: close\r\n";
    head += "\r\n";
    raw.write_all(head);
    res.stream([&](const std::string& chunk) -> bool {
      if (chunk.empty()) return true;
      char hx[32];
      snprintf(hx, sizeof(hx), "%zx\r\n", chunk.size());
      try {
        raw.write_all(std::string(hx) + chunk + "\r\n");
        return true;
      } catch (...) {
        return false;
      }
    });
    raw.write_all(std::string("0\r\n\r\n"));
  } else {
    head += "Content-Length: " + std::to_string(res.body.size()) + "\r\n";
    if (!keep) head += "Connection: close\r\n";
    head += "\r\n";
    if (req.method != "HEAD") head += res.body;
    raw.write_all(head);
  }
  if (access_log_) {
    double us = (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now() - t0)
                    .count() /
                1000.0;
    char lat[32];
    if (us < 1000) snprintf(lat, sizeof(lat), "%.3fµs", us);
    else if (us < 1e6) snprintf(lat, sizeof(lat), "%.3fms", us / 1000);
    else snprintf(lat, sizeof(lat), "%.3fs", us / 1e6);
    char ts[32];
    struct tm lt;
    localtime_r(&now, &lt);
    strftime(ts, sizeof(ts), "%Y/%m/%d - %H:%M:%S", &lt);
    std::string ip = req.remote.substr(0, req.remote.rfind(':'));
    fprintf(stderr, "[%s] %s | %3d | %13s | %15s | %-7s \"%s\"\n", name_.c_str(), ts, res.status,
            lat, ip.c_str(), req.method.c_str(), req.path.c_str());
  }
  return keep;
}

// ================================================================ client
HttpResult http_request(const std::string& method, const std::string& url, const std::string& body,
                        const std::string& content_type, int timeout_ms,
                        const std::vector<std::pair<std::string, std::string>>& headers) {
  if (url.rfind("http://", 0) != 0) throw NetError("unsupported URL scheme: " + url);
  std::string rest = url.substr(7);
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  std::string target = slash == std::string::npos ? "/" : rest.substr(slash);
  std::string host;
  int port = 80;
  if (hostport.find(':') != std::string::npos) split_host_port(hostport, &host, &port);
  else host = hostport;
  auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  auto left = [&] {
    return (int)std::max<long>(1, std::chrono::duration_cast<std::chrono::milliseconds>(
                                      t_end - std::chrono::steady_clock::now())
                                      .count());
  };
  auto c = TcpConn::dial(host, port, left());
  std::string req = method + " " + target + " HTTP/1.1\r\nHost: " + hostport +
                    "\r\nUser-Agent: p2p-llm-chat-amd/0.1\r\nConnection: close\r\n";
  if (!body.empty() || method == "POST" || method == "PUT") {
    req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
    if (!content_type.empty()) req += "Content-Type: " + content_type + "\r\n";
  }
  for (auto& h : headers) req += h.first + ": " + h.second + "\r\n";
  req += "\r\n" + body;
  c->write_all(req);
  BufConn bc(c);
  HttpResult out;
  c->set_read_timeout(left());
  std::string status = read_line(bc);
  if (status.rfind("HTTP/1.", 0) != 0) throw NetError("bad HTTP response");
  out.status = atoi(status.c_str() + 9);
  while (true) {
    c->set_read_timeout(left());
    std::string h = read_line(bc);
    if (h.empty()) break;
    size_t colon = h.find(':');
    if (colon != std::string::npos) out.headers[lower(trim(h.substr(0, colon)))] = trim(h.substr(colon + 1));
  }
  c->set_read_timeout(left());
  if (lower(out.headers["transfer-encoding"]).find("chunked") != std::string::npos) {
    while (true) {
      c->set_read_timeout(left());
      size_t n = strtoul(read_line(bc).c_str(), nullptr, 16);
      if (n == 0) break;
      Bytes ch = bc.read_exact(n);
      out.body.append(ch.begin(), ch.end());
      read_line(bc);
    }
  } else if (out.headers.count("content-length")) {
    size_t n = strtoull(out.headers["content-length"].c_str(), nullptr, 10);
    Bytes b = bc.read_exact(n);
    out.body.assign(b.begin(), b.end());
  } else {
    Bytes b = bc.read_all(64 << 20);
    out.body.assign(b.begin(), b.end());
  }
  c->close();
  return out;
}

}  // namespace p2p
