// Native request path across processes (loop_remote.h): LoopServer in a replica leader's
// process, RemoteLoops (a P2PLoopApi table) in the node's.
#include "runtime/loop_remote.h"

#include <errno.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <stdexcept>

#include "runtime/engine_loop.h"

namespace p2p {

namespace {

using Clock = std::chrono::steady_clock;

sockaddr_un abstract_addr(const std::string& name, socklen_t* len) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (name.size() + 1 > sizeof(a.sun_path)) throw std::runtime_error("socket name too long");
  a.sun_path[0] = 0;  // abstract namespace
  memcpy(a.sun_path + 1, name.data(), name.size());
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + name.size());
  return a;
}

bool send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t w = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += (size_t)w;
  }
  return true;
}

bool send_frame(int fd, const std::string& payload) {
  const uint32_t n = (uint32_t)payload.size();
  std::string f(reinterpret_cast<const char*>(&n), 4);
  f += payload;
  return send_all(fd, f);
}

// reads exactly n bytes; false on EOF / error
bool recv_all(int fd, char* p, size_t n) {
  size_t got = 0;
  while (got < n) {
    const ssize_t r = recv(fd, p + got, n - got, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    got += (size_t)r;
  }
  return true;
}

// 1: a frame was read into *out; 0: nothing arrived within timeout_s; -1: closed / error
int recv_frame(int fd, double timeout_s, std::string* out) {
  pollfd p{fd, POLLIN, 0};
  const int ms = timeout_s < 0 ? -1 : (int)(timeout_s * 1000.0);
  int r;
  do r = poll(&p, 1, ms);
  while (r < 0 && errno == EINTR);
  if (r == 0) return 0;
  if (r < 0) return -1;
  uint32_t n = 0;
  if (!recv_all(fd, (char*)&n, 4) || n > (64u << 20)) return -1;
  out->resize(n);
  if (n && !recv_all(fd, &(*out)[0], n)) return -1;
  return 1;
}

struct Put {
  std::string s;
  template <class T>
  Put& v(T x) {
    s.append(reinterpret_cast<const char*>(&x), sizeof(T));
    return *this;
  }
  Put& str(const std::string& x) {
    v<uint32_t>((uint32_t)x.size());
    s += x;
    return *this;
  }
  Put& ints(const int32_t* p, size_t n) {
    v<uint32_t>((uint32_t)n);
    s.append(reinterpret_cast<const char*>(p), n * 4);
    return *this;
  }
};

struct Get {
  const std::string& s;
  size_t i = 0;
  template <class T>
  T v() {
    if (i + sizeof(T) > s.size()) throw std::runtime_error("truncated loop frame");
    T x;
    memcpy(&x, s.data() + i, sizeof(T));
    i += sizeof(T);
    return x;
  }
  std::string str() {
    const uint32_t n = v<uint32_t>();
    if (i + n > s.size()) throw std::runtime_error("truncated loop frame");
    std::string x = s.substr(i, n);
    i += n;
    return x;
  }
  std::vector<int32_t> ints() {
    const uint32_t n = v<uint32_t>();
    if (i + (size_t)n * 4 > s.size()) throw std::runtime_error("truncated loop frame");
    std::vector<int32_t> x(n);
    if (n) memcpy(x.data(), s.data() + i, (size_t)n * 4);
    i += (size_t)n * 4;
    return x;
  }
};

}  // namespace

// ------------------------------------------------------------------ server
LoopServer::LoopServer(EngineLoop* loop, const std::string& name) : loop_(loop), name_(name) {}

LoopServer::~LoopServer() { stop(); }

void LoopServer::start() {
  socklen_t len;
  const sockaddr_un a = abstract_addr(name_, &len);
  lfd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw std::runtime_error(std::string("loop server socket: ") + strerror(errno));
  if (bind(lfd_, (const sockaddr*)&a, len) != 0 || listen(lfd_, 256) != 0) {
    const std::string e = strerror(errno);
    close(lfd_);
    lfd_ = -1;
    throw std::runtime_error("loop server bind @" + name_ + ": " + e);
  }
  stop_ = false;
  th_ = std::thread([this] { accept_loop(); });
}

void LoopServer::stop() {
  stop_ = true;
  if (lfd_ >= 0) shutdown(lfd_, SHUT_RDWR);
  if (th_.joinable()) th_.join();
  if (lfd_ >= 0) close(lfd_);
  lfd_ = -1;
  // request threads poll every 50 ms and see stop_
  for (int i = 0; i < 200 && active_.load() > 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
}

void LoopServer::accept_loop() {
  while (!stop_) {
    pollfd p{lfd_, POLLIN, 0};
    const int r = poll(&p, 1, 100);
    if (r <= 0) continue;
    const int fd = accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      if (stop_) break;
      continue;
    }
    active_++;
    std::thread([this, fd] {
      try {
        serve(fd);
      } catch (const std::exception&) {
      }
      close(fd);
      active_--;
    }).detach();
  }
}

// One request per connection: submit, then stream its tokens as the loop decodes them,
// then the final result.  The client closing the connection (or a 'C' frame) cancels it.
void LoopServer::serve(int fd) {
  std::string f;
  if (recv_frame(fd, 30.0, &f) != 1 || f.empty() || f[0] != 'S') return;
  Get g{f, 1};
  const int32_t n = g.v<int32_t>();
  if (n < 0 || (size_t)n * 4 + 1 > f.size()) return;
  std::vector<int> ids(n);
  for (int i = 0; i < n; ++i) ids[i] = g.v<int32_t>();
  const int max_new = g.v<int32_t>();
  const bool stop_on_eos = g.v<uint8_t>() != 0;
  LoopSampling s;
  s.temperature = g.v<float>();
  s.top_k = g.v<int32_t>();
  s.top_p = g.v<float>();
  s.seed = g.v<int64_t>();
  int64_t id;
  try {
    id = loop_->submit(ids, max_new, stop_on_eos, s);
  } catch (const std::exception& e) {
    send_frame(fd, Put().v<char>('A').v<int64_t>(-1).str(e.what()).s);
    return;
  }
  served_++;
  if (!send_frame(fd, Put().v<char>('A').v<int64_t>(id).s)) {
    loop_->cancel(id);
    loop_->release(id);
    return;
  }
  size_t have = 0;
  bool done = false;
  while (!done) {
    std::vector<int> t;
    try {
      t = loop_->wait_tokens(id, have, 0.05, &done);
    } catch (const std::exception&) {
      done = true;
    }
    if (!t.empty()) {
      std::vector<int32_t> t32(t.begin(), t.end());
      if (!send_frame(fd, Put().v<char>('T').ints(t32.data(), t32.size()).s)) {
        loop_->cancel(id);
        loop_->release(id);
        return;
      }
      have += t.size();
    }
    if (done) break;
    // the client: a cancel frame, or gone
    pollfd p{fd, POLLIN, 0};
    if (poll(&p, 1, 0) > 0) {
      std::string c;
      if (recv_frame(fd, 0.0, &c) != 1 || (!c.empty() && c[0] == 'C')) {
        loop_->cancel(id);
        loop_->release(id);  // dropped when it ends
        return;
      }
    }
    if (stop_) {
      loop_->cancel(id);
      loop_->release(id);
      return;
    }
  }
  LoopResult r;
  try {
    loop_->wait(id, 0.0, &r);
  } catch (const std::exception& e) {
    r.error = e.what();
  }
  loop_->release(id);
  std::vector<int32_t> t32(r.tokens.begin(), r.tokens.end());
  send_frame(fd, Put()
                     .v<char>('R')
                     .v<uint8_t>(r.done ? 1 : 0)
                     .v<int32_t>(r.prompt_eval_count)
                     .v<int64_t>(r.prompt_eval_ns)
                     .v<int64_t>(r.eval_ns)
                     .v<int64_t>(r.total_ns)
                     .v<int64_t>(r.ttft_ns)
                     .str(r.done_reason)
                     .str(r.error)
                     .ints(t32.data(), t32.size())
                     .s);
}

// ------------------------------------------------------------------ client
namespace {

struct RemoteReq {
  int fd = -1;
  int replica = 0;
  std::vector<int32_t> tokens;
  bool finished = false;  // the 'R' frame arrived (or the connection broke)
  P2PLoopResult res{};
  std::string error, reason;
};

struct RemoteLoops {
  struct Replica {
    std::string name;
    bool alive = true;
    long outstanding = 0, routed = 0;
    std::string why;
  };
  std::vector<Replica> reps;
  std::map<int64_t, std::shared_ptr<RemoteReq>> reqs;
  int64_t next = 1;
  std::mutex mu;

  std::shared_ptr<RemoteReq> get(int64_t h) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = reqs.find(h);
    return it == reqs.end() ? nullptr : it->second;
  }
};

int connect_to(const std::string& name) {
  socklen_t len;
  const sockaddr_un a = abstract_addr(name, &len);
  const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  if (connect(fd, (const sockaddr*)&a, len) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

// one frame from the server into the request's state; false when nothing came in time
bool pump(RemoteReq& q, double timeout_s) {
  if (q.finished) return false;
  std::string f;
  const int r = recv_frame(q.fd, timeout_s, &f);
  if (r == 0) return false;
  if (r < 0 || f.empty()) {
    q.finished = true;
    q.error = "engine replica connection lost (replica process gone?)";
    return true;
  }
  try {
    Get g{f, 1};
    if (f[0] == 'T') {
      const auto t = g.ints();
      q.tokens.insert(q.tokens.end(), t.begin(), t.end());
    } else if (f[0] == 'R') {
      q.finished = true;
      q.res.done = g.v<uint8_t>();
      q.res.prompt_eval_count = g.v<int32_t>();
      q.res.prompt_eval_ns = g.v<int64_t>();
      q.res.eval_ns = g.v<int64_t>();
      q.res.total_ns = g.v<int64_t>();
      q.res.ttft_ns = g.v<int64_t>();
      q.reason = g.str();
      q.error = g.str();
      q.tokens = g.ints();
    }
  } catch (const std::exception& e) {
    q.finished = true;
    q.error = e.what();
  }
  return true;
}

void set_err(const std::string& e, char* err, int errlen) {
  if (err && errlen > 0) {
    strncpy(err, e.c_str(), (size_t)errlen - 1);
    err[errlen - 1] = 0;
  }
}

int64_t r_submit(void* loop, const int32_t* ids, int n, int max_new, int stop_on_eos, float temp,
                 int top_k, float top_p, int64_t seed, char* err, int errlen) {
  RemoteLoops& L = *(RemoteLoops*)loop;
  const std::string frame = Put()
                                .v<char>('S')
                                .v<int32_t>(n)
                                .s +
                            std::string(reinterpret_cast<const char*>(ids), (size_t)n * 4) +
                            Put()
                                .v<int32_t>(max_new)
                                .v<uint8_t>(stop_on_eos ? 1 : 0)
                                .v<float>(temp)
                                .v<int32_t>(top_k)
                                .v<float>(top_p)
                                .v<int64_t>(seed)
                                .s;
  std::string last = "no live engine replica";
  for (size_t attempt = 0; attempt < L.reps.size(); ++attempt) {
    int ri = -1;
    {
      std::lock_guard<std::mutex> lk(L.mu);
      for (int i = 0; i < (int)L.reps.size(); ++i)  // least outstanding, then lowest index
        if (L.reps[i].alive && (ri < 0 || L.reps[i].outstanding < L.reps[ri].outstanding)) ri = i;
      if (ri < 0) break;
      L.reps[ri].outstanding++;
    }
    auto q = std::make_shared<RemoteReq>();
    q->replica = ri;
    q->fd = connect_to(L.reps[ri].name);
    std::string f;
    bool ok = q->fd >= 0 && send_frame(q->fd, frame) && recv_frame(q->fd, 60.0, &f) == 1 &&
              f.size() >= 9 && f[0] == 'A';
    if (ok) {
      Get g{f, 1};
      const int64_t rid = g.v<int64_t>();
      if (rid >= 0) {
        std::lock_guard<std::mutex> lk(L.mu);
        L.reps[ri].routed++;
        const int64_t h = L.next++;
        L.reqs[h] = q;
        return h;
      }
      // refused by the loop (admission, context, replica down): the reason, no retry
      last = g.str();
      close(q->fd);
      std::lock_guard<std::mutex> lk(L.mu);
      L.reps[ri].outstanding--;
      set_err(last, err, errlen);
      return -1;
    }
    if (q->fd >= 0) close(q->fd);
    std::lock_guard<std::mutex> lk(L.mu);  // unreachable replica: never routed to again
    L.reps[ri].outstanding--;
    L.reps[ri].alive = false;
    L.reps[ri].why = "replica " + std::to_string(ri) + " unreachable at @" + L.reps[ri].name;
    last = L.reps[ri].why;
  }
  set_err(last, err, errlen);
  return -1;
}

int r_wait(void* loop, int64_t h, double timeout_s, P2PLoopResult* out) {
  memset(out, 0, sizeof(*out));
  auto q = ((RemoteLoops*)loop)->get(h);
  if (!q) {
    out->error = strdup("unknown request");
    out->tokens = (int32_t*)malloc(4);
    return 0;
  }
  const auto t0 = Clock::now();
  while (!q->finished) {
    double left = -1.0;
    if (timeout_s >= 0) {
      left = timeout_s - std::chrono::duration<double>(Clock::now() - t0).count();
      if (left <= 0) break;
    }
    pump(*q, left < 0 ? 1.0 : std::min(left, 1.0));
  }
  *out = q->res;
  out->done = q->finished && q->error.empty() ? q->res.done : 0;
  out->n_tokens = (int)q->tokens.size();
  out->tokens = (int32_t*)malloc(sizeof(int32_t) * std::max<size_t>(1, q->tokens.size()));
  if (!q->tokens.empty()) memcpy(out->tokens, q->tokens.data(), q->tokens.size() * 4);
  strncpy(out->done_reason, q->reason.c_str(), sizeof(out->done_reason) - 1);
  out->error = (q->finished && !q->error.empty()) ? strdup(q->error.c_str()) : nullptr;
  return 0;
}

int r_wait_tokens(void* loop, int64_t h, size_t have, double timeout_s, int32_t** toks, int* n,
                  int* done) {
  auto q = ((RemoteLoops*)loop)->get(h);
  *toks = (int32_t*)malloc(4);
  *n = 0;
  *done = 1;
  if (!q) return 0;
  const auto t0 = Clock::now();
  while (q->tokens.size() <= have && !q->finished) {
    const double left = timeout_s - std::chrono::duration<double>(Clock::now() - t0).count();
    if (timeout_s >= 0 && left <= 0) break;
    pump(*q, timeout_s < 0 ? 1.0 : left);
  }
  // 'T' frames carry the tokens as decoded; the final 'R' list is the reply (EOS trimmed)
  const size_t m = q->tokens.size() > have ? q->tokens.size() - have : 0;
  if (m) {
    free(*toks);
    *toks = (int32_t*)malloc(m * 4);
    memcpy(*toks, q->tokens.data() + have, m * 4);
  }
  *n = (int)m;
  *done = q->finished ? 1 : 0;
  return 0;
}

void r_cancel(void* loop, int64_t h) {
  auto q = ((RemoteLoops*)loop)->get(h);
  if (q && !q->finished) send_frame(q->fd, Put().v<char>('C').s);
}

void r_release(void* loop, int64_t h) {
  RemoteLoops& L = *(RemoteLoops*)loop;
  std::shared_ptr<RemoteReq> q;
  {
    std::lock_guard<std::mutex> lk(L.mu);
    auto it = L.reqs.find(h);
    if (it == L.reqs.end()) return;
    q = it->second;
    L.reqs.erase(it);
    L.reps[q->replica].outstanding--;
  }
  if (!q->finished) send_frame(q->fd, Put().v<char>('C').s);  // cancelled on the replica
  close(q->fd);
}

int r_dead(void* loop, char* buf, int len) {
  RemoteLoops& L = *(RemoteLoops*)loop;
  std::string d;
  {
    std::lock_guard<std::mutex> lk(L.mu);
    bool any = false;
    for (auto& r : L.reps) any |= r.alive;
    if (!any) {
      d = "no live engine replica";
      for (auto& r : L.reps) d += "; " + r.why;
    }
  }
  if (buf && len > 0) {
    strncpy(buf, d.c_str(), (size_t)len - 1);
    buf[len - 1] = 0;
  }
  return (int)d.size();
}

void r_free(void* p) { free(p); }

const P2PLoopApi g_remote_api = {P2P_LOOP_API_VERSION, r_submit, r_wait, r_wait_tokens, r_cancel,
                                 r_release, r_dead, r_free};

}  // namespace

const P2PLoopApi* remote_loop_api() { return &g_remote_api; }

void* remote_loops_create(const std::vector<std::string>& names) {
  auto* L = new RemoteLoops;
  for (auto& n : names) {
    RemoteLoops::Replica r;
    r.name = n;
    L->reps.push_back(r);
  }
  return L;
}

void remote_loops_destroy(void* rl) { delete (RemoteLoops*)rl; }

std::vector<long> remote_loops_routed(void* rl) {
  RemoteLoops& L = *(RemoteLoops*)rl;
  std::lock_guard<std::mutex> lk(L.mu);
  std::vector<long> v;
  for (auto& r : L.reps) v.push_back(r.routed);
  return v;
}

}  // namespace p2p
