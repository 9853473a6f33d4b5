#include "yamux.h"

#include <string.h>

#include <chrono>

namespace p2p {

namespace {
enum : uint8_t { T_DATA = 0, T_WINDOW = 1, T_PING = 2, T_GOAWAY = 3 };
enum : uint16_t { F_SYN = 1, F_ACK = 2, F_FIN = 4, F_RST = 8 };
constexpr size_t kMaxInboundStreams = 1024;
}  // namespace

// ================================================================ stream
YamuxStream::YamuxStream(std::shared_ptr<YamuxSession> s, uint32_t id)
    : s_(std::move(s)), id_(id), recv_window_(YamuxSession::kInitialWindow),
      send_window_(YamuxSession::kInitialWindow) {}

YamuxStream::~YamuxStream() = default;

std::string YamuxStream::remote_addr() const { return s_->conn()->remote_addr(); }

size_t YamuxStream::read_some(uint8_t* buf, size_t n) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] {
    return rpos_ < rbuf_.size() || remote_fin_ || reset_ || local_closed_ || s_->closed();
  };
  if (timeout_ms_ > 0) {
    if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms_), ready))
      throw NetError("stream read timeout");
  } else {
    cv_.wait(lk, ready);
  }
  if (rpos_ < rbuf_.size()) {
    size_t k = std::min(n, rbuf_.size() - rpos_);
    memcpy(buf, rbuf_.data() + rpos_, k);
    rpos_ += k;
    if (rpos_ == rbuf_.size()) {
      rbuf_.clear();
      rpos_ = 0;
    }
    unacked_ += (uint32_t)k;
    uint32_t credit = 0;
    if (unacked_ >= YamuxSession::kInitialWindow / 2 && !remote_fin_) {
      credit = unacked_;
      unacked_ = 0;
      recv_window_ += credit;
    }
    lk.unlock();
    if (credit) s_->send_frame(T_WINDOW, 0, id_, credit);
    return k;
  }
  if (reset_) throw NetError("stream reset");
  return 0;  // EOF (remote FIN), local close, or session closed
}

void YamuxStream::write_all(const uint8_t* buf, size_t n) {
  size_t off = 0;
  while (off < n) {
    uint32_t k;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return send_window_ > 0 || reset_ || s_->closed(); });
      if (reset_) throw NetError("stream reset");
      if (s_->closed()) throw NetError("session closed");
      if (local_fin_) throw NetError("write after close");
      k = (uint32_t)std::min<size_t>({n - off, (size_t)send_window_, (size_t)YamuxSession::kMaxFrame});
      send_window_ -= k;
    }
    s_->send_frame(T_DATA, 0, id_, k, buf + off);
    off += k;
  }
}

void YamuxStream::close_write() {
  bool remove = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (local_fin_ || reset_) return;
    local_fin_ = true;
    remove = remote_fin_;
  }
  if (!s_->closed()) {
    try {
      s_->send_frame(T_WINDOW, F_FIN, id_, 0);
    } catch (...) {
    }
  }
  if (remove) s_->remove_stream(id_);
}

void YamuxStream::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    local_closed_ = true;
  }
  cv_.notify_all();
  close_write();
}

void YamuxStream::reset() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (reset_) return;
    reset_ = true;
  }
  cv_.notify_all();
  if (!s_->closed()) {
    try {
      s_->send_frame(T_WINDOW, F_RST, id_, 0);
    } catch (...) {
    }
  }
  s_->remove_stream(id_);
}

// ================================================================ session
YamuxSession::YamuxSession(ConnPtr conn, bool client)
    : conn_(std::move(conn)), client_(client), next_id_(client ? 1 : 2) {}

YamuxSession::~YamuxSession() {
  close();
  if (reader_.joinable()) {
    if (reader_.get_id() == std::this_thread::get_id()) reader_.detach();
    else reader_.join();
  }
}

void YamuxSession::start(std::function<void(StreamPtr)> on_stream, std::function<void()> on_close) {
  on_stream_ = std::move(on_stream);
  on_close_ = std::move(on_close);
  auto self = shared_from_this();
  reader_ = std::thread([self] { self->reader_loop(); });
  reader_.detach();
}

void YamuxSession::send_frame(uint8_t type, uint16_t flags, uint32_t id, uint32_t length,
                              const uint8_t* data) {
  uint8_t h[12];
  h[0] = 0;
  h[1] = type;
  h[2] = (uint8_t)(flags >> 8);
  h[3] = (uint8_t)flags;
  for (int i = 0; i < 4; ++i) h[4 + i] = (uint8_t)(id >> (24 - 8 * i));
  for (int i = 0; i < 4; ++i) h[8 + i] = (uint8_t)(length >> (24 - 8 * i));
  Bytes out(h, h + 12);
  if (type == T_DATA && data && length) out.insert(out.end(), data, data + length);
  std::lock_guard<std::mutex> lk(wmu_);
  if (closed_) throw NetError("session closed");
  conn_->write_all(out);
}

StreamPtr YamuxSession::open_stream() {
  if (closed_) throw NetError("session closed");
  YStreamPtr s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    uint32_t id = next_id_;
    next_id_ += 2;
    s = std::make_shared<YamuxStream>(shared_from_this(), id);
    streams_[id] = s;
  }
  send_frame(T_WINDOW, F_SYN, s->id(), 0);
  return s;
}

void YamuxSession::remove_stream(uint32_t id) {
  std::lock_guard<std::mutex> lk(mu_);
  streams_.erase(id);
}

size_t YamuxSession::num_streams() {
  std::lock_guard<std::mutex> lk(mu_);
  return streams_.size();
}

void YamuxSession::close() {
  bool was = closed_.exchange(true);
  if (was) return;
  try {
    uint8_t h[12] = {0, T_GOAWAY, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    conn_->write_all(h, 12);
  } catch (...) {
  }
  conn_->close();
  std::map<uint32_t, YStreamPtr> ss;
  {
    std::lock_guard<std::mutex> lk(mu_);
    ss.swap(streams_);
  }
  for (auto& kv : ss) kv.second->cv_.notify_all();
  pcv_.notify_all();
}

long YamuxSession::ping(int timeout_ms) {
  uint32_t id;
  {
    std::lock_guard<std::mutex> lk(pmu_);
    id = ++ping_id_;
    ping_done_[id] = false;
  }
  auto t0 = std::chrono::steady_clock::now();
  send_frame(T_PING, F_SYN, 0, id);
  std::unique_lock<std::mutex> lk(pmu_);
  bool ok = pcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms),
                          [&] { return ping_done_[id] || closed_; });
  bool done = ping_done_[id];
  ping_done_.erase(id);
  if (!ok || !done) return -1;
  return (long)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now() - t0)
      .count();
}

void YamuxSession::handle_flags(const YStreamPtr& s, uint16_t flags) {
  bool remove = false;
  {
    std::lock_guard<std::mutex> lk(s->mu_);
    if (flags & F_FIN) {
      s->remote_fin_ = true;
      remove = s->local_fin_;
    }
    if (flags & F_RST) {
      s->reset_ = true;
      remove = true;
    }
  }
  s->cv_.notify_all();
  if (remove) remove_stream(s->id());
}

void YamuxSession::reader_loop() {
  auto self = shared_from_this();
  try {
    while (!closed_) {
      uint8_t h[12];
      size_t got = 0;
      while (got < 12) {
        size_t r = conn_->read_some(h + got, 12 - got);
        if (r == 0) throw NetError("eof");
        got += r;
      }
      if (h[0] != 0) throw NetError("yamux: bad version");
      uint8_t type = h[1];
      uint16_t flags = (uint16_t)(h[2] << 8 | h[3]);
      uint32_t id = (uint32_t)h[4] << 24 | (uint32_t)h[5] << 16 | (uint32_t)h[6] << 8 | h[7];
      uint32_t len = (uint32_t)h[8] << 24 | (uint32_t)h[9] << 16 | (uint32_t)h[10] << 8 | h[11];
      if (type == T_PING) {
        if (flags & F_SYN) send_frame(T_PING, F_ACK, 0, len);
        if (flags & F_ACK) {
          std::lock_guard<std::mutex> lk(pmu_);
          if (ping_done_.count(len)) ping_done_[len] = true;
          pcv_.notify_all();
        }
        continue;
      }
      if (type == T_GOAWAY) throw NetError("goaway");
      if (type != T_DATA && type != T_WINDOW) throw NetError("yamux: bad frame type");
      Bytes payload;
      if (type == T_DATA && len) {
        if (len > kInitialWindow * 64) throw NetError("yamux: frame too large");
        payload = conn_->read_exact(len);
      }
      YStreamPtr s;
      bool is_new = false;
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = streams_.find(id);
        if (it != streams_.end()) {
          s = it->second;
        } else if (flags & F_SYN) {
          if (streams_.size() >= kMaxInboundStreams) {
            s = nullptr;
          } else {
            s = std::make_shared<YamuxStream>(self, id);
            streams_[id] = s;
            is_new = true;
          }
        }
      }
      if (!s) {
        if (flags & F_SYN) send_frame(T_WINDOW, F_RST, id, 0);
        continue;  // frame for an already closed stream
      }
      if (is_new) send_frame(T_WINDOW, F_ACK, id, 0);
      if (type == T_WINDOW) {
        std::lock_guard<std::mutex> lk(s->mu_);
        s->send_window_ += len;
      } else if (!payload.empty()) {
        std::lock_guard<std::mutex> lk(s->mu_);
        if (payload.size() > s->recv_window_) throw NetError("yamux: receive window exceeded");
        s->recv_window_ -= (uint32_t)payload.size();
        if (!s->local_closed_) s->rbuf_.insert(s->rbuf_.end(), payload.begin(), payload.end());
      }
      s->cv_.notify_all();
      if (flags & (F_FIN | F_RST)) handle_flags(s, flags);
      if (is_new && on_stream_) {
        auto cb = on_stream_;
        std::thread([cb, s] {
          try {
            cb(s);
          } catch (...) {
            s->reset();
          }
        }).detach();
      }
    }
  } catch (...) {
  }
  close();
  if (on_close_) on_close_();
}

}  // namespace p2p
