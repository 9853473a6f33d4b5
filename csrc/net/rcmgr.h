// Resource manager (the go-libp2p host's rcmgr): scoped accounting of
// connections and streams with limits per scope, so one peer (or one protocol) cannot
// exhaust the node.  Scopes, as in go-libp2p's network resource manager:
//   system    -- every inbound / outbound connection and stream of the host
//   transient -- inbound streams still negotiating their protocol (multistream)
//   peer      -- the streams and connections of one remote peer
//   protocol  -- the inbound streams of one protocol id (e.g. /p2p-llm-chat/1.0.0)
// A reservation that would exceed any scope's limit is refused; the caller resets the
// stream or closes the connection.  Counts only (the reference's go-libp2p also tracks
// memory; this node bounds memory by its fixed windows: yamux 256 KiB, QUIC 4/16 MiB,
// the 1 MiB chat cap, INBOX_CAP).
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "crypto.h"
#include "json.h"

namespace p2p {

struct ResourceLimits {  // defaults: go-libp2p's scaled defaults for a small host
  int system_conns_inbound = 256, system_conns_outbound = 512;
  int system_streams_inbound = 4096, system_streams_outbound = 8192;
  int transient_streams = 256;
  int peer_conns = 8;
  int peer_streams_inbound = 512, peer_streams_outbound = 1024;
  int protocol_streams_inbound = 2048;
  static ResourceLimits from_env();  // RCMGR_<FIELD> overrides (e.g. RCMGR_PEER_STREAMS_INBOUND)
};

class ResourceManager : public std::enable_shared_from_this<ResourceManager> {
 public:
  explicit ResourceManager(ResourceLimits l = ResourceLimits()) : lim_(l) {}
  void set_limits(const ResourceLimits& l) {
    std::lock_guard<std::mutex> lk(mu_);
    lim_ = l;
  }

  // An accounted stream / connection: released when the handle is destroyed (handles
  // keep the manager alive, so a session outliving its host still releases cleanly).
  class Stream {
   public:
    ~Stream();
    // Moves the stream from the transient scope to `proto`'s scope (inbound only).
    bool set_protocol(const std::string& proto);

   private:
    friend class ResourceManager;
    std::shared_ptr<ResourceManager> rm_;
    PeerId peer_;
    std::string proto_;
    bool inbound_ = false, transient_ = false;
  };
  class Conn {
   public:
    ~Conn();

   private:
    friend class ResourceManager;
    std::shared_ptr<ResourceManager> rm_;
    PeerId peer_;
    bool inbound_ = false;
  };

  // null = refused (a limit of some scope would be exceeded)
  std::unique_ptr<Stream> open_stream(const PeerId& peer, bool inbound);
  std::unique_ptr<Conn> open_conn(const PeerId& peer, bool inbound);
  Json stats();
  ResourceLimits limits() {
    std::lock_guard<std::mutex> lk(mu_);
    return lim_;
  }

 private:
  struct Counts {
    int streams_in = 0, streams_out = 0, conns = 0;
  };
  ResourceLimits lim_;
  std::mutex mu_;
  Counts system_;
  int conns_in_ = 0, conns_out_ = 0, transient_ = 0;
  std::map<PeerId, Counts> peers_;
  std::map<std::string, int> protocols_;
  long refused_streams_ = 0, refused_conns_ = 0;
};

}  // namespace p2p
