// Stream-muxer interface of a libp2p connection.  Two implementations: yamux
// over a secured byte stream (TCP + Noise/TLS, or a relayed circuit; yamux.h)
// and QUIC, whose streams are native (quic.h).  The host, identify, ping, the
// relay and the chat protocol only see these two types.
#pragma once
#include <functional>
#include <memory>
#include <string>

#include "conn.h"

namespace p2p {

class MuxStream : public Conn {
 public:
  virtual void reset() = 0;  // abort both directions
  std::string protocol;      // negotiated protocol (set by the host)
};
using StreamPtr = std::shared_ptr<MuxStream>;

class MuxSession {
 public:
  virtual ~MuxSession() = default;
  // Starts delivery: on_stream runs (in its own thread) for every inbound stream;
  // on_close runs once when the session dies.
  virtual void start(std::function<void(StreamPtr)> on_stream,
                     std::function<void()> on_close = nullptr) = 0;
  virtual StreamPtr open_stream() = 0;
  virtual void close() = 0;
  virtual bool closed() const = 0;
  // Round-trip liveness probe; returns RTT in microseconds or -1 on timeout.
  virtual long ping(int timeout_ms) = 0;
  virtual size_t num_streams() = 0;
  virtual std::string transport() const = 0;  // "tcp", "quic-v1", ...
};
using SessionPtr = std::shared_ptr<MuxSession>;

}  // namespace p2p
