// Leader -> follower replay of the native engine loop's device operations (mirror.h).
#include "runtime/mirror.h"

#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "runtime/hip_dyn.h"

namespace p2p {

namespace {

void write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0 && errno == ENOTSOCK) w = write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("group channel write failed: ") + strerror(errno));
    }
    p += w;
    n -= (size_t)w;
  }
}

// false on a clean EOF before the first byte
bool read_exact(int fd, char* p, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = read(fd, p + got, n - got);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("group channel read failed: ") + strerror(errno));
    }
    if (r == 0) {
      if (got == 0) return false;
      throw std::runtime_error("group channel closed mid-frame");
    }
    got += (size_t)r;
  }
  return true;
}

struct Reader {
  const std::string& s;
  size_t i = 0;
  template <class T>
  T get() {
    if (i + sizeof(T) > s.size()) throw std::runtime_error("mirror frame truncated");
    T v;
    memcpy(&v, s.data() + i, sizeof(T));
    i += sizeof(T);
    return v;
  }
  const char* bytes(size_t n) {
    if (i + n > s.size()) throw std::runtime_error("mirror frame truncated");
    const char* p = s.data() + i;
    i += n;
    return p;
  }
  std::vector<int> ints() {
    const uint32_t n = get<uint32_t>();
    std::vector<int> v(n);
    if (n) memcpy(v.data(), bytes((size_t)n * 4), (size_t)n * 4);
    return v;
  }
};

}  // namespace

// ------------------------------------------------------------------ leader
void MirrorSender::head(char op, char kind, int a, int b, bool greedy) {
  put<char>(op);
  put<char>(kind);
  put<int32_t>(a);
  put<int32_t>(b);
  put<uint8_t>(greedy ? 1 : 0);
}

void MirrorSender::h2d(char kind, int a, int b, bool greedy, uint8_t field, const void* src,
                       size_t n) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  head('H', kind, a, b, greedy);
  put<uint8_t>(field);
  put<uint32_t>((uint32_t)n);
  append((const char*)src, n);
}

void MirrorSender::tokens(char kind, int a, int b, bool greedy, uint8_t src, uint32_t s0,
                          uint32_t k, uint32_t rows) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  head('T', kind, a, b, greedy);
  put<uint8_t>(src);
  put<uint32_t>(s0);
  put<uint32_t>(k);
  put<uint32_t>(rows);
}

void MirrorSender::memset0(char kind, int a, int b, bool greedy, uint8_t field, size_t n) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  head('M', kind, a, b, greedy);
  put<uint8_t>(field);
  put<uint32_t>((uint32_t)n);
}

void MirrorSender::launch(char kind, int a, int b, bool greedy, uint8_t which, uint32_t count) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  head('L', kind, a, b, greedy);
  put<uint8_t>(which);
  put<uint32_t>(count);
}

void MirrorSender::faults() {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  put<char>('F');
}

void MirrorSender::provide(char kind, int a, int b, bool greedy) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  head('V', kind, a, b, greedy);
}

void MirrorSender::eager(const std::vector<std::vector<int>>& prompts,
                         const std::vector<std::vector<int>>& pages, const std::vector<int>& starts,
                         const std::vector<LoopSampling>& samp, int pad_rows, bool want) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  put<char>('E');
  put<uint32_t>((uint32_t)prompts.size());
  put<int32_t>(pad_rows);
  put<uint8_t>(want ? 1 : 0);
  for (size_t i = 0; i < prompts.size(); ++i) {
    put<uint32_t>((uint32_t)prompts[i].size());
    append((const char*)prompts[i].data(), prompts[i].size() * 4);
    const std::vector<int>& pg = i < pages.size() ? pages[i] : std::vector<int>();
    put<uint32_t>((uint32_t)pg.size());
    append((const char*)pg.data(), pg.size() * 4);
    put<int32_t>(i < starts.size() ? starts[i] : 0);
    const LoopSampling s = i < samp.size() ? samp[i] : LoopSampling();
    put<float>(s.temperature);
    put<int32_t>(s.top_k);
    put<float>(s.top_p);
    put<int64_t>(s.seed);
  }
}

void MirrorSender::stop() {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  target_ = -1;
  put<char>('S');
  flush();
}

// Every follower gets a frame whenever any has records (possibly empty), so frame numbers
// stay the same on every follower.
uint32_t MirrorSender::flush() {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  target_ = -1;
  bool any = false;
  for (auto& b : bufs_) any |= !b.empty();
  if (!any) return 0;
  for (size_t f = 0; f < fds_.size(); ++f) {
    const uint32_t n = (uint32_t)bufs_[f].size();
    std::string frame(reinterpret_cast<const char*>(&n), 4);
    frame += bufs_[f];
    bufs_[f].clear();
    write_all(fds_[f], frame.data(), frame.size());
    bytes_ += (long)frame.size();
  }
  frames_++;
  return (uint32_t)frames_.load();
}

std::vector<int> MirrorSender::take_tokens(int f, uint32_t seq) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  std::vector<int> out;
  if (f < 0 || (size_t)f >= toks_.size()) return out;
  auto it = toks_[f].find(seq);
  if (it == toks_[f].end()) return out;
  out = std::move(it->second);
  toks_[f].erase(it);
  return out;
}

uint32_t MirrorSender::await(uint32_t seq, double timeout_s) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  if (acked_.size() != fds_.size()) acked_.assign(fds_.size(), 0);
  if (toks_.size() != fds_.size()) toks_.resize(fds_.size());
  uint32_t bits = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t f = 0; f < fds_.size(); ++f) {
    while (acked_[f] < seq) {
      const double left =
          timeout_s - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      pollfd pf{fds_[f], POLLIN, 0};
      const int r = left > 0 ? poll(&pf, 1, (int)(left * 1000) + 1) : 0;
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0)
        throw std::runtime_error("group follower " + std::to_string(f + 1) +
                                 " did not report frame " + std::to_string(seq));
      uint32_t rep[3];
      if (!read_exact(fds_[f], (char*)rep, sizeof rep))
        throw std::runtime_error("group follower " + std::to_string(f + 1) + " is gone");
      if (rep[2]) {  // the frame's tokens (dp groups)
        std::vector<int> t(rep[2]);
        if (!read_exact(fds_[f], (char*)t.data(), (size_t)rep[2] * 4))
          throw std::runtime_error("group follower " + std::to_string(f + 1) + " is gone");
        toks_[f][rep[0]] = std::move(t);
      }
      acked_[f] = rep[0];
      bits |= rep[1];
    }
  }
  if (bits) follower_faults_++;
  return bits;
}

// ------------------------------------------------------------------ follower
EngineMirror::EngineMirror(int fd, int device) : fd_(fd), device_(device) {
  const char* e = std::getenv("P2P_MIRROR_INJECT_FAULT");
  inject_at_ = e ? std::atol(e) : 0;
  const char* ec = std::getenv("P2P_MIRROR_INJECT_COLL");
  inject_coll_at_ = ec ? std::atol(ec) : 0;
}

EngineMirror::~EngineMirror() {
  {
    std::lock_guard<std::mutex> lk(rmu_);
    rstop_ = true;
  }
  rcv_.notify_all();
  if (rth_.joinable()) rth_.join();
}

void EngineMirror::shutdown() {
  {
    std::lock_guard<std::mutex> lk(rmu_);
    rstop_ = true;
  }
  rcv_.notify_all();
  if (rth_.joinable()) rth_.join();
  const HipApi& h = hip_api();
  if (!h.ok) return;
  for (int i = 0; i < kRep; ++i) {
    if (rep_ev_[i]) h.eventDestroy(rep_ev_[i]);
    rep_ev_[i] = nullptr;
  }
  if (rep_words_) h.hostFree(rep_words_);
  rep_words_ = nullptr;
  if (rep_toks_) h.hostFree(rep_toks_);
  rep_toks_ = nullptr;
  for (int i = 0; i < 2; ++i) {
    if (stage_[i]) h.hostFree(stage_[i]);
    if (stage_ev_[i]) h.eventDestroy(stage_ev_[i]);
    stage_[i] = stage_ev_[i] = nullptr;
    stage_n_[i] = 0;
  }
  if (stream_) h.streamDestroy(stream_);
  stream_ = nullptr;
}

void EngineMirror::add_decode_graph(const DecodeGraphDesc& d) {
  Graph g;
  g.kind = 'D';
  g.a = d.B;
  g.b = d.ctx;
  g.greedy = d.greedy;
  g.exec = d.exec;
  g.exec_k = d.exec_k;
  g.fields[kFMeta] = d.meta;
  g.fields[kFStep] = d.step;
  g.fields[kFKeys] = d.keys;
  g.fields[kFTemp] = d.temp;
  g.fields[kFTopk] = d.topk;
  g.fields[kFTopp] = d.topp;
  g.fields[kFSeeds] = d.seeds;
  g.err = d.err;
  g.hist = d.hist;
  g.max_steps = d.max_steps;
  std::lock_guard<std::mutex> lk(gmu_);
  graphs_[std::make_tuple('D', g.a, g.b, g.greedy)] = g;
}

void EngineMirror::add_prefill_graph(const PrefillGraphDesc& d) {
  Graph g;
  g.kind = 'P';
  g.a = d.rows;
  g.b = d.n_seq;
  g.greedy = d.greedy;
  g.exec = d.exec;
  g.fields[kFMeta] = d.meta;
  g.fields[kFTemp] = d.temp;
  g.fields[kFTopk] = d.topk;
  g.fields[kFTopp] = d.topp;
  g.fields[kFSeeds] = d.seeds;
  g.err = d.err;
  g.first = d.first;
  std::lock_guard<std::mutex> lk(gmu_);
  graphs_[std::make_tuple('P', g.a, g.b, g.greedy)] = g;
}

EngineMirror::Graph* EngineMirror::find(char kind, int a, int b, bool greedy) {
  std::lock_guard<std::mutex> lk(gmu_);
  auto it = graphs_.find(std::make_tuple(kind, a, b, greedy));
  if (it == graphs_.end())
    throw std::runtime_error(std::string("mirror: no ") + (kind == 'D' ? "decode" : "prefill") +
                             " graph (" + std::to_string(a) + ", " + std::to_string(b) + ", " +
                             (greedy ? "greedy" : "sampled") + ") on this rank");
  return &it->second;
}

void* EngineMirror::staging(size_t n) {
  const HipApi& h = hip_api();
  const int i = cur_;
  if (stage_ev_[i]) hip_check(h.eventSynchronize(stage_ev_[i]), "mirror staging reuse");
  if (stage_n_[i] < n) {
    if (stage_[i]) h.hostFree(stage_[i]);
    stage_[i] = nullptr;
    const size_t sz = std::max(n, (size_t)1 << 16);
    hip_check(h.hostMalloc(&stage_[i], sz, 0), "mirror staging");
    stage_n_[i] = sz;
  }
  return stage_[i];
}

std::map<std::string, double> EngineMirror::metrics() {
  std::map<std::string, double> m;
  m["mirror_frames"] = n_frames_;
  m["mirror_launches"] = n_launches_;
  m["mirror_provides"] = n_provides_;
  m["mirror_eager"] = n_eager_;
  m["mirror_fault_reports"] = n_faults_;
  m["mirror_host_failures"] = n_host_fail_;
  std::lock_guard<std::mutex> lk(gmu_);
  m["mirror_graphs"] = (double)graphs_.size();
  return m;
}

uint32_t EngineMirror::apply(const std::string& frame, std::vector<int32_t*>* launched,
                             FrameOut* out) {
  const HipApi& h = hip_api();
  // h2d payloads of this frame go through one pinned staging buffer (copied up front)
  char* st = (char*)staging(frame.size());
  memcpy(st, frame.data(), frame.size());
  Reader r{frame};
  bool used_stage = false;
  uint32_t host_bits = 0;
  try {
    while (r.i < frame.size()) {
      const char op = r.get<char>();
      if (op == 'S') {
        throw std::string("");  // stop: handled by run()
      }
      if (op == 'F') {  // the leader failed a step: every fault word of this rank back to 0
        std::lock_guard<std::mutex> lk(gmu_);
        for (auto& kv : graphs_)
          if (kv.second.err) hip_check(h.memsetAsync(kv.second.err, 0, 4, stream_), "mirror fault reset");
        if (aux_err_) hip_check(h.memsetAsync(aux_err_, 0, 4, stream_), "mirror split fault reset");
        continue;
      }
      if (op == 'E') {
        const uint32_t n = r.get<uint32_t>();
        const int32_t pad = r.get<int32_t>();
        const bool want = r.get<uint8_t>() != 0;
        std::vector<std::vector<int>> prompts, pages;
        std::vector<int> starts;
        std::vector<LoopSampling> samp;
        for (uint32_t i = 0; i < n; ++i) {
          prompts.push_back(r.ints());
          pages.push_back(r.ints());
          starts.push_back(r.get<int32_t>());
          LoopSampling s;
          s.temperature = r.get<float>();
          s.top_k = r.get<int32_t>();
          s.top_p = r.get<float>();
          s.seed = r.get<int64_t>();
          samp.push_back(s);
        }
        if (!eager_) throw std::runtime_error("mirror: no eager prefill callback");
        hip_check(h.streamSynchronize(stream_), "mirror sync");  // the model code runs on its stream
        std::vector<int> first = eager_(prompts, pages, starts, samp, pad);
        if (want) out->host.insert(out->host.end(), first.begin(), first.end());
        n_eager_++;
        continue;
      }
      const char kind = r.get<char>();
      const int a = r.get<int32_t>(), b = r.get<int32_t>();
      const bool greedy = r.get<uint8_t>() != 0;
      if (op == 'V') {
        if (!provider_) throw std::runtime_error("mirror: no graph provider");
        hip_check(h.streamSynchronize(stream_), "mirror sync");
        provider_(kind == 'D' ? "decode" : "prefill", a, b, greedy);
        n_provides_++;
        (void)find(kind, a, b, greedy);  // the provider must have registered it
        continue;
      }
      Graph* g = find(kind, a, b, greedy);
      if (op == 'T') {  // this rank's tokens go back with the frame's status (dp groups)
        const uint8_t src = r.get<uint8_t>();
        const uint32_t s0 = r.get<uint32_t>(), k = r.get<uint32_t>(), rows = r.get<uint32_t>();
        if (src == 0) {
          if (!g->hist || (int)(s0 + k) > g->max_steps || (int)rows > g->a)
            throw std::runtime_error("mirror: bad decode token record");
          out->copies.push_back(TokCopy{g->hist + s0, (size_t)g->max_steps, rows, k});
        } else {
          if (!g->first || (int)rows > g->b) throw std::runtime_error("mirror: bad prefill token record");
          out->copies.push_back(TokCopy{g->first, 1, rows, 1});
        }
        continue;
      }
      if (op == 'H') {
        const uint8_t f = r.get<uint8_t>();
        const uint32_t n = r.get<uint32_t>();
        const size_t off = r.i;
        (void)r.bytes(n);
        if (f > kFSeeds || !g->fields[f]) throw std::runtime_error("mirror: bad h2d field");
        hip_check(h.memcpyAsync(g->fields[f], st + off, n, kH2D, stream_), "mirror h2d");
        used_stage = true;
      } else if (op == 'M') {
        const uint8_t f = r.get<uint8_t>();
        const uint32_t n = r.get<uint32_t>();
        if (f > kFSeeds || !g->fields[f]) throw std::runtime_error("mirror: bad memset field");
        hip_check(h.memsetAsync(g->fields[f], 0, n, stream_), "mirror memset");
      } else if (op == 'L') {
        const uint8_t which = r.get<uint8_t>();
        const uint32_t count = r.get<uint32_t>();
        void* ex = which ? g->exec_k : g->exec;
        if (!ex) throw std::runtime_error("mirror: graph has no such exec");
        for (uint32_t i = 0; i < count; ++i) hip_check(h.graphLaunch(ex, stream_), "mirror launch");
        n_launches_ += count;
        if (g->err && std::find(launched->begin(), launched->end(), g->err) == launched->end())
          launched->push_back(g->err);
      } else {
        throw std::runtime_error(std::string("mirror: unknown op ") + op);
      }
    }
  } catch (const std::exception& e) {
    // a callback that raised, an unknown graph, a bad record: this frame fails (reported to
    // the leader, which fails its step); the mirror keeps serving the next frames.  (A
    // broken stream or HIP error shows up again on the next frame's own calls.)
    host_bits = 2;
    n_host_fail_++;
    fprintf(stderr, "[mirror] frame failed on this rank: %s\n", e.what());
  }
  if (used_stage) {
    if (!stage_ev_[cur_]) hip_check(h.eventCreateWithFlags(&stage_ev_[cur_], 2), "mirror event");
    hip_check(h.eventRecord(stage_ev_[cur_], stream_), "mirror event");
    cur_ ^= 1;
  }
  return host_bits;
}

// Queue the frame's status: its launched graphs' fault words and the split-K word are
// copied to a pinned slot behind the frame's work; reporter() answers once that landed.
void EngineMirror::report(uint32_t seq, const std::vector<int32_t*>& launched, uint32_t host_bits,
                          const FrameOut& out) {
  const HipApi& h = hip_api();
  std::unique_lock<std::mutex> lk(rmu_);
  const int slot = rep_next_;
  rcv_.wait(lk, [&] { return !rep_busy_[slot] || rstop_; });
  if (rstop_) return;
  rep_next_ = (rep_next_ + 1) % kRep;
  rep_busy_[slot] = true;
  lk.unlock();
  if (!rep_words_) {
    hip_check(h.hostMalloc((void**)&rep_words_, (size_t)kRep * kRepWords * 4, 0), "mirror status");
    memset(rep_words_, 0, (size_t)kRep * kRepWords * 4);
  }
  if (!rep_ev_[slot]) hip_check(h.eventCreateWithFlags(&rep_ev_[slot], 2), "mirror status event");
  int32_t* w = rep_words_ + (size_t)slot * kRepWords;
  int nw = 0;
  for (int32_t* e : launched) {
    if (nw >= kRepWords - 2) break;
    hip_check(h.memcpyAsync(w + nw++, e, 4, kD2H, stream_), "mirror status D2H");
  }
  if (aux_err_) hip_check(h.memcpyAsync(w + nw++, aux_err_, 4, kD2H, stream_), "mirror status D2H");
  int coll = -1;
  if (coll_err_) {
    coll = nw;
    hip_check(h.memcpyAsync(w + nw++, coll_err_, 4, kD2H, stream_), "mirror status D2H");
  }
  // the frame's tokens: host ones first (eager prefill), then the device rows, packed
  int nt = 0;
  if (!out.host.empty() || !out.copies.empty()) {
    if (!rep_toks_) hip_check(h.hostMalloc((void**)&rep_toks_, (size_t)kRep * kRepToks * 4, 0), "mirror tokens");
    int32_t* t = rep_toks_ + (size_t)slot * kRepToks;
    for (int v : out.host) {
      if (nt >= kRepToks) throw std::runtime_error("mirror: frame tokens exceed the report slot");
      t[nt++] = v;
    }
    for (const TokCopy& c : out.copies) {
      if (nt + (size_t)c.rows * c.k > (size_t)kRepToks)
        throw std::runtime_error("mirror: frame tokens exceed the report slot");
      if (c.rows)
        hip_check(h.memcpy2DAsync(t + nt, (size_t)c.k * 4, c.src, c.pitch * 4, (size_t)c.k * 4, c.rows,
                                  kD2H, stream_),
                  "mirror tokens D2H");
      nt += (int)(c.rows * c.k);
    }
  }
  hip_check(h.eventRecord(rep_ev_[slot], stream_), "mirror status event");
  lk.lock();
  rq_.push_back(Report{seq, host_bits, slot, nw, nt, coll});
  lk.unlock();
  rcv_.notify_all();
}

void EngineMirror::reporter() {
  const HipApi& h = hip_api();
  (void)h.setDevice(device_);
  while (true) {
    Report rp;
    {
      std::unique_lock<std::mutex> lk(rmu_);
      rcv_.wait(lk, [&] { return rstop_ || !rq_.empty(); });
      if (rq_.empty()) return;  // stopping, nothing left to answer
      rp = rq_.front();
      rq_.pop_front();
    }
    uint32_t bits = rp.host_bits;
    if (h.eventSynchronize(rep_ev_[rp.slot]) != 0) bits |= 2;
    for (int i = 0; i < rp.nwords; ++i)
      if (rep_words_[(size_t)rp.slot * kRepWords + i] != 0) bits |= i == rp.coll ? 4 : 1;
    if (bits & 1) n_faults_++;
    std::string msg(12 + (size_t)rp.ntok * 4, '\0');
    const uint32_t head[3] = {rp.seq, bits, (uint32_t)rp.ntok};
    memcpy(&msg[0], head, 12);
    if (rp.ntok) memcpy(&msg[12], rep_toks_ + (size_t)rp.slot * kRepToks, (size_t)rp.ntok * 4);
    {
      std::lock_guard<std::mutex> lk(rmu_);  // the slot (and its tokens) is free after the copy
      rep_busy_[rp.slot] = false;
    }
    rcv_.notify_all();
    try {
      write_all(fd_, msg.data(), msg.size());
    } catch (const std::exception&) {  // the leader is gone: nothing to tell
    }
  }
}

std::string EngineMirror::run() {
  const HipApi& h = hip_api();
  try {
    if (!h.ok) throw std::runtime_error("mirror: " + h.error);
    hip_check(h.setDevice(device_), "hipSetDevice");
    if (!stream_) hip_check(h.streamCreateWithFlags(&stream_, 1), "hipStreamCreate");
    {
      std::lock_guard<std::mutex> lk(rmu_);
      rstop_ = false;
    }
    if (!rth_.joinable()) rth_ = std::thread([this] { reporter(); });
    std::string frame;
    uint32_t seq = 0;
    std::vector<int32_t*> launched;
    while (true) {
      uint32_t n = 0;
      if (!read_exact(fd_, (char*)&n, 4)) throw std::runtime_error("group channel closed (leader gone)");
      frame.resize(n);
      if (n && !read_exact(fd_, &frame[0], n)) throw std::runtime_error("group channel closed");
      n_frames_++;
      ++seq;
      launched.clear();
      FrameOut fout;
      uint32_t host_bits;
      try {
        host_bits = apply(frame, &launched, &fout);
      } catch (const std::string&) {  // stop
        hip_check(h.streamSynchronize(stream_), "mirror drain");
        return "";
      }
      if (!launched.empty()) {
        ++launch_frames_;
        if (launch_frames_ == inject_at_ && aux_err_)
          hip_check(h.memsetAsync(aux_err_, 1, 4, stream_), "mirror fault injection");
        if (launch_frames_ == inject_coll_at_ && coll_err_)
          hip_check(h.memsetAsync(coll_err_, 1, 4, stream_), "mirror collective fault injection");
      }
      report(seq, launched, host_bits, fout);
    }
  } catch (const std::exception& e) {
    return e.what();
  }
}

}  // namespace p2p
