#include "rcmgr.h"

#include <cstdlib>

namespace p2p {

ResourceLimits ResourceLimits::from_env() {
  ResourceLimits l;
  auto get = [](const char* name, int* v) {
    const char* s = getenv(name);
    if (s && *s) *v = atoi(s);
  };
  get("RCMGR_SYSTEM_CONNS_INBOUND", &l.system_conns_inbound);
  get("RCMGR_SYSTEM_CONNS_OUTBOUND", &l.system_conns_outbound);
  get("RCMGR_SYSTEM_STREAMS_INBOUND", &l.system_streams_inbound);
  get("RCMGR_SYSTEM_STREAMS_OUTBOUND", &l.system_streams_outbound);
  get("RCMGR_TRANSIENT_STREAMS", &l.transient_streams);
  get("RCMGR_PEER_CONNS", &l.peer_conns);
  get("RCMGR_PEER_STREAMS_INBOUND", &l.peer_streams_inbound);
  get("RCMGR_PEER_STREAMS_OUTBOUND", &l.peer_streams_outbound);
  get("RCMGR_PROTOCOL_STREAMS_INBOUND", &l.protocol_streams_inbound);
  return l;
}

std::unique_ptr<ResourceManager::Stream> ResourceManager::open_stream(const PeerId& peer,
                                                                      bool inbound) {
  std::lock_guard<std::mutex> lk(mu_);
  Counts& pc = peers_[peer];
  const bool ok = inbound ? (system_.streams_in < lim_.system_streams_inbound &&
                             transient_ < lim_.transient_streams &&
                             pc.streams_in < lim_.peer_streams_inbound)
                          : (system_.streams_out < lim_.system_streams_outbound &&
                             pc.streams_out < lim_.peer_streams_outbound);
  if (!ok) {
    ++refused_streams_;
    if (pc.streams_in == 0 && pc.streams_out == 0 && pc.conns == 0) peers_.erase(peer);
    return nullptr;
  }
  auto s = std::unique_ptr<Stream>(new Stream());
  s->rm_ = shared_from_this();
  s->peer_ = peer;
  s->inbound_ = inbound;
  if (inbound) {
    ++system_.streams_in;
    ++pc.streams_in;
    ++transient_;
    s->transient_ = true;
  } else {
    ++system_.streams_out;
    ++pc.streams_out;
  }
  return s;
}

bool ResourceManager::Stream::set_protocol(const std::string& proto) {
  if (!inbound_) return true;  // the protocol scope limits inbound streams only
  std::lock_guard<std::mutex> lk(rm_->mu_);
  int& n = rm_->protocols_[proto];
  if (n >= rm_->lim_.protocol_streams_inbound) {
    ++rm_->refused_streams_;
    return false;
  }
  ++n;
  proto_ = proto;
  if (transient_) {
    --rm_->transient_;
    transient_ = false;
  }
  return true;
}

ResourceManager::Stream::~Stream() {
  if (!rm_) return;
  std::lock_guard<std::mutex> lk(rm_->mu_);
  if (transient_) --rm_->transient_;
  if (!proto_.empty()) {
    auto it = rm_->protocols_.find(proto_);
    if (it != rm_->protocols_.end() && --it->second <= 0) rm_->protocols_.erase(it);
  }
  auto pit = rm_->peers_.find(peer_);
  if (inbound_) {
    --rm_->system_.streams_in;
    if (pit != rm_->peers_.end()) --pit->second.streams_in;
  } else {
    --rm_->system_.streams_out;
    if (pit != rm_->peers_.end()) --pit->second.streams_out;
  }
  if (pit != rm_->peers_.end() && pit->second.streams_in <= 0 && pit->second.streams_out <= 0 &&
      pit->second.conns <= 0)
    rm_->peers_.erase(pit);
}

std::unique_ptr<ResourceManager::Conn> ResourceManager::open_conn(const PeerId& peer, bool inbound) {
  std::lock_guard<std::mutex> lk(mu_);
  Counts& pc = peers_[peer];
  const bool ok = (inbound ? conns_in_ < lim_.system_conns_inbound
                           : conns_out_ < lim_.system_conns_outbound) &&
                  pc.conns < lim_.peer_conns;
  if (!ok) {
    ++refused_conns_;
    if (pc.streams_in == 0 && pc.streams_out == 0 && pc.conns == 0) peers_.erase(peer);
    return nullptr;
  }
  auto c = std::unique_ptr<Conn>(new Conn());
  c->rm_ = shared_from_this();
  c->peer_ = peer;
  c->inbound_ = inbound;
  ++(inbound ? conns_in_ : conns_out_);
  ++pc.conns;
  ++system_.conns;
  return c;
}

ResourceManager::Conn::~Conn() {
  if (!rm_) return;
  std::lock_guard<std::mutex> lk(rm_->mu_);
  --(inbound_ ? rm_->conns_in_ : rm_->conns_out_);
  --rm_->system_.conns;
  auto pit = rm_->peers_.find(peer_);
  if (pit != rm_->peers_.end() && --pit->second.conns <= 0 && pit->second.streams_in <= 0 &&
      pit->second.streams_out <= 0)
    rm_->peers_.erase(pit);
}

Json ResourceManager::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  Json j = Json::object();
  j.set("streams_inbound", (long)system_.streams_in);
  j.set("streams_outbound", (long)system_.streams_out);
  j.set("streams_transient", (long)transient_);
  j.set("conns_inbound", (long)conns_in_);
  j.set("conns_outbound", (long)conns_out_);
  j.set("peers", (long)peers_.size());
  j.set("refused_streams", refused_streams_);
  j.set("refused_conns", refused_conns_);
  return j;
}

}  // namespace p2p
