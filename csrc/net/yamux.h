// yamux stream multiplexer ("/yamux/1.0.0", the muxer go-libp2p negotiates):
// 12-byte big-endian frame header {version=0, type, flags, stream id, length},
// Data / WindowUpdate / Ping / GoAway frames, SYN/ACK/FIN/RST flags, 256 KiB
// initial per-stream receive window with credit returned as the reader
// consumes, odd stream ids for the dialer and even ids for the listener.
// Half-close (FIN) is what lets the chat receiver's read-to-EOF terminate
// (`go/cmd/node/main.go:160`).
#pragma once
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "conn.h"
#include "mux.h"

namespace p2p {

class YamuxSession;

class YamuxStream : public MuxStream {
 public:
  YamuxStream(std::shared_ptr<YamuxSession> s, uint32_t id);
  ~YamuxStream() override;
  using Conn::write_all;
  size_t read_some(uint8_t* buf, size_t n) override;
  void write_all(const uint8_t* buf, size_t n) override;
  void close_write() override;  // FIN
  void close() override;        // FIN + stop reading
  void reset() override;        // RST
  void set_read_timeout(int ms) override { timeout_ms_ = ms; }
  std::string remote_addr() const override;
  uint32_t id() const { return id_; }
  std::shared_ptr<YamuxSession> session() const { return s_; }

 private:
  friend class YamuxSession;
  std::shared_ptr<YamuxSession> s_;
  uint32_t id_;
  std::mutex mu_;
  std::condition_variable cv_;
  Bytes rbuf_;
  size_t rpos_ = 0;
  uint32_t recv_window_;
  uint32_t unacked_ = 0;  // consumed bytes not yet returned as window credit
  uint32_t send_window_;
  bool remote_fin_ = false, local_fin_ = false, reset_ = false, local_closed_ = false;
  int timeout_ms_ = 0;
};
using YStreamPtr = std::shared_ptr<YamuxStream>;

class YamuxSession : public MuxSession, public std::enable_shared_from_this<YamuxSession> {
 public:
  static constexpr uint32_t kInitialWindow = 256 * 1024;
  static constexpr uint32_t kMaxFrame = 64 * 1024;

  YamuxSession(ConnPtr conn, bool client);
  ~YamuxSession();
  // Starts the reader thread.  on_stream runs (in its own thread) for every inbound stream;
  // on_close runs once when the session dies.
  void start(std::function<void(StreamPtr)> on_stream,
             std::function<void()> on_close = nullptr) override;
  StreamPtr open_stream() override;
  void close() override;
  bool closed() const override { return closed_; }
  std::string transport() const override { return "yamux"; }
  // Round-trip ping; returns RTT in microseconds or -1 on timeout.
  long ping(int timeout_ms) override;
  size_t num_streams() override;
  const ConnPtr& conn() const { return conn_; }

 private:
  friend class YamuxStream;
  void reader_loop();
  void send_frame(uint8_t type, uint16_t flags, uint32_t id, uint32_t length,
                  const uint8_t* data = nullptr);
  void remove_stream(uint32_t id);
  void handle_flags(const YStreamPtr& s, uint16_t flags);

  ConnPtr conn_;
  bool client_;
  std::mutex wmu_;
  std::mutex mu_;
  std::map<uint32_t, YStreamPtr> streams_;
  uint32_t next_id_;
  std::atomic<bool> closed_{false};
  std::function<void(StreamPtr)> on_stream_;
  std::function<void()> on_close_;
  std::thread reader_;
  // ping state
  std::mutex pmu_;
  std::condition_variable pcv_;
  uint32_t ping_id_ = 0;
  std::map<uint32_t, bool> ping_done_;
};

}  // namespace p2p
