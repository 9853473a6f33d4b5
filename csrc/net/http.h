// Minimal HTTP/1.1 server + client for the node API, the Directory and the
// Ollama-compatible generate endpoint (the reference uses gin and net/http:
// `go/cmd/node/main.go:57,72,214`, `go/cmd/directory/main.go:59`).
//
// Server: thread per connection, keep-alive, Content-Length and chunked request
// bodies, gin-style access log, streaming (chunked) responses for NDJSON.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "conn.h"
#include "json.h"

namespace p2p {

std::string url_encode(const std::string& s);
std::string url_decode(const std::string& s);

struct HttpRequest {
  std::string method, path, query_string, version;
  std::map<std::string, std::string> query;    // decoded
  std::map<std::string, std::string> headers;  // lower-case names
  std::string body;
  std::string remote;
  std::string header(const std::string& k) const;
  std::string param(const std::string& k, const std::string& def = "") const;
};

struct HttpResponse {
  int status = 200;
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
  // Streaming: if set, called with a chunk writer after the headers are sent
  // (Transfer-Encoding: chunked).  The writer returns false once the client is gone.
  std::function<void(const std::function<bool(const std::string&)>&)> stream;

  void json(int code, const Json& j, bool sorted_keys = false);  // gin c.JSON
  void text(int code, const std::string& s);                     // gin c.String
  void set_header(const std::string& k, const std::string& v);
};

using HttpHandler = std::function<void(const HttpRequest&, HttpResponse&)>;

class HttpServer {
 public:
  explicit HttpServer(std::string name = "GIN") : name_(std::move(name)) {}
  ~HttpServer();
  void route(const std::string& method, const std::string& path, HttpHandler h);
  // Binds "host:port" (port 0 = ephemeral); returns the bound port.  Non-blocking.
  int start(const std::string& addr);
  void serve_forever();  // blocks until stop()
  void stop();
  int port() const { return port_; }
  void set_access_log(bool on) { access_log_ = on; }
  size_t max_body = 8 << 20;

 private:
  void conn_loop(std::shared_ptr<TcpConn> c);
  bool handle_one(BufConn& bc, TcpConn& raw);
  std::string name_;
  std::map<std::string, HttpHandler> routes_;  // "METHOD path"
  std::shared_ptr<TcpListener> listener_;
  std::thread accept_thread_;
  std::atomic<bool> stopped_{false};
  std::atomic<int> active_{0};
  int port_ = 0;
  bool access_log_ = true;
  std::mutex mu_;
  std::vector<std::weak_ptr<TcpConn>> conns_;
  // serve_forever() waits on this instead of joining: stop() is the only joiner of
  // accept_thread_ (two concurrent joins of one std::thread are undefined behaviour)
  std::condition_variable exit_cv_;
  bool accept_exited_ = false;
};

struct HttpResult {
  int status = 0;
  std::string body;
  std::map<std::string, std::string> headers;
};

// Blocking request with an overall timeout (ms).  url: http://host:port/path?query
// Throws NetError on connection failure / timeout (like Go's client.Do error).
HttpResult http_request(const std::string& method, const std::string& url,
                        const std::string& body = "", const std::string& content_type = "",
                        int timeout_ms = 5000,
                        const std::vector<std::pair<std::string, std::string>>& headers = {});

// Splits "host:port" (also "[v6]:port", ":port").
void split_host_port(const std::string& addr, std::string* host, int* port);

}  // namespace p2p
