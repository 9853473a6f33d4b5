#include "runtime/engine_loop.h"
#include "runtime/loop_remote.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

#include "runtime/hip_dyn.h"
#include "runtime/loop_capi.h"
#include "runtime/mirror.h"

namespace p2p {

namespace {

// pinned staging slots
enum Slot : int {
  kDecodeMeta = 0,
  kPrefillMeta = 1,
  kHist0 = 2,  // kHist0, kHist0 + 1: double-buffered decode history
  kFirst = 4,
  kErr0 = 5,  // kErr0, kErr0 + 1: fault word per decode buffer; kErr0 + 2 prefill
  kSampF = 8,
  kSampI = 9,
  kSampP = 10,
  kSampS = 11,
  kAux0 = 12,  // kAux0, kAux0 + 1: split-K fault word per decode buffer; kAux0 + 2 prefill
  kColl0 = 15,  // the same three for the IPC collectives' timeout word (set_coll_fault)
  kSlots = 18,
};

}  // namespace

EngineLoop::EngineLoop(const LoopConfig& cfg)
    : cfg_(cfg),
      sched_(cfg.num_pages, cfg.page_size, cfg.max_batch, cfg.max_prefill_tokens, cfg.max_ctx) {
  sched_.set_defer_free(true);
  pinned_.assign(kSlots, {nullptr, 0});
}

// The thread only: HIP resources are released by shutdown() (a destructor running at
// interpreter exit may find the HIP runtime already torn down).
EngineLoop::~EngineLoop() {
  if (server_) server_->stop();
  stop();
}

void EngineLoop::serve(const std::string& name) {
  if (server_) throw std::runtime_error("loop already serving");
  server_.reset(new LoopServer(this, name));
  server_->start();
}

void EngineLoop::shutdown() {
  if (server_) server_->stop();  // no new requests; open ones are cancelled
  stop();
  const HipApi& h = hip_api();
  if (!h.ok) return;
  for (auto& p : pinned_)
    if (p.first) h.hostFree(p.first);
  pinned_.assign(kSlots, {nullptr, 0});
  for (void* e : events_)
    if (e) h.eventDestroy(e);
  events_.clear();
  for (void* e : staged_ev_)
    if (e) h.eventDestroy(e);
  staged_ev_.clear();
  if (stream_) h.streamDestroy(stream_);
  stream_ = nullptr;
}

int64_t EngineLoop::now_ns() const {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int EngineLoop::bucket(int x, const std::vector<int>& b) {
  for (int v : b)
    if (x <= v) return v;
  return -1;
}

// A staging slot is rewritten by the host for the next chunk while earlier work may still
// be queued on the stream ahead of the copy that reads it (a pipelined decode chunk, a
// prefill chunk behind a running decode): the leader would then run a chunk on the NEXT
// chunk's metadata or sampling parameters while its followers -- whose frames carry their
// own copy of the bytes -- run the right ones, and the group's ranks drift apart (a sampled
// reply of a TP=8 group differed from the Python loop's on some runs).  So a slot whose copies
// have not run yet is waited for before it is handed out again.
void* EngineLoop::pinned(int slot, size_t bytes) {
  auto& p = pinned_[slot];
  const HipApi& h = hip_api();
  if ((int)staged_ev_.size() > slot && staged_ev_[slot])
    hip_check(h.eventSynchronize(staged_ev_[slot]), "staging slot reuse");
  if (p.second < bytes) {
    if (p.first) h.hostFree(p.first);
    size_t n = std::max(bytes, (size_t)4096);
    hip_check(h.hostMalloc(&p.first, n, 0), "hipHostMalloc");
    p.second = n;
  }
  return p.first;
}

void EngineLoop::staged(int slot) {
  const HipApi& h = hip_api();
  if ((int)staged_ev_.size() < kSlots) staged_ev_.resize(kSlots, nullptr);
  if (!staged_ev_[slot])
    hip_check(h.eventCreateWithFlags(&staged_ev_[slot], 2 /* hipEventDisableTiming */), "hipEventCreate");
  hip_check(h.eventRecord(staged_ev_[slot], stream_), "hipEventRecord");
}

std::vector<std::vector<int64_t>> EngineLoop::split_by_home(const std::vector<int64_t>& ids,
                                                             bool assign) {
  const int W = std::max(1, cfg_.dp_world);
  std::vector<std::vector<int64_t>> parts(W);
  std::lock_guard<std::mutex> lk(mu_);
  if (assign) {
    // a new sequence goes to the rank holding the fewest live ones (ties rotate), as
    // engine/cluster.py LockstepEngine._parts does for the Python loop
    std::vector<int> live(W, 0);
    for (int64_t id : sched_.running()) {
      if (std::find(ids.begin(), ids.end(), id) != ids.end()) continue;
      auto it = reqs_.find(id);
      if (it != reqs_.end()) live[it->second.home]++;
    }
    for (int64_t id : ids) {
      int h = 0;
      for (int r = 1; r < W; ++r) {
        const int a = (r - home_rr_ + W) % W, b = (h - home_rr_ + W) % W;
        if (live[r] < live[h] || (live[r] == live[h] && a < b)) h = r;
      }
      home_rr_ = (h + 1) % W;
      live[h]++;
      reqs_[id].home = h;
    }
  }
  for (int64_t id : ids) {
    auto it = reqs_.find(id);
    parts[it != reqs_.end() ? it->second.home : 0].push_back(id);
  }
  return parts;
}

// A decode graph's batch state for rows `ids` (DecodeState layout: ids | pos | ctx | slots |
// block tables; rows past them are dummies on the null page at position 0) and, for sampled
// graphs, its sampler slots.  Caller holds no lock.
void EngineLoop::decode_meta(const DecodeGraphDesc* g, const std::vector<int64_t>& ids, int32_t* m,
                             float* tf, int32_t* tk, float* tp, int64_t* sd) {
  const int B = g->B, P = g->max_pages;
  std::memset(m, 0, (size_t)B * (4 + P) * 4);
  int32_t *idv = m, *pos = m + B, *ctx = m + 2 * B, *slots = m + 3 * B, *bt = m + 4 * B;
  std::vector<LoopSampling> samp;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t b = 0; b < ids.size(); ++b) {
      const SchedRequest& r = sched_.get(ids[b]);
      for (size_t i = 0; i < r.pages.size() && (int)i < P; ++i) bt[b * P + i] = r.pages[i];
      idv[b] = r.tokens.empty() ? 0 : r.tokens.back();
      pos[b] = r.pos;
      samp.push_back(reqs_[ids[b]].samp);
    }
  }
  for (int b = 0; b < B; ++b) {
    ctx[b] = pos[b] + 1;
    slots[b] = bt[b * P + pos[b] / 64] * 64 + pos[b] % 64;
  }
  if (!tf) return;
  for (int b = 0; b < B; ++b) {
    const LoopSampling d = b < (int)samp.size() ? samp[b] : LoopSampling();
    tf[b] = b < (int)samp.size() ? d.temperature : 0.f;
    tk[b] = d.top_k;
    tp[b] = d.top_p;
    sd[b] = b < (int)samp.size() ? d.seed : 0;
  }
}

// ------------------------------------------------------------------ registration
void EngineLoop::add_decode_graph(const DecodeGraphDesc& d) {
  std::lock_guard<std::mutex> lk(gmu_);
  dgraphs_[std::make_tuple(d.B, d.ctx, d.greedy)] = std::make_unique<DecodeGraphDesc>(d);
}

void EngineLoop::add_prefill_graph(const PrefillGraphDesc& d) {
  std::lock_guard<std::mutex> lk(gmu_);
  pgraphs_[std::make_tuple(d.rows, d.n_seq, d.greedy)] = std::make_unique<PrefillGraphDesc>(d);
}

void EngineLoop::set_provider(GraphProvider p) { provider_ = std::move(p); }

void EngineLoop::set_mirror(const std::vector<int>& fds) {
  mirror_ = fds.empty() ? nullptr : std::make_unique<MirrorSender>(fds);
}

void EngineLoop::mirror_provide(const std::string& kind, int a, int b, bool greedy) {
  if (!mirror_) return;
  mirror_->provide(kind == "decode" ? 'D' : 'P', a, b, greedy);
  mirror_->flush();
}
void EngineLoop::set_eager_prefill(EagerPrefill f) { eager_ = std::move(f); }

const DecodeGraphDesc* EngineLoop::decode_graph(int B, int ctx, bool greedy) {
  const auto key = std::make_tuple(B, ctx, greedy);
  {
    std::lock_guard<std::mutex> lk(gmu_);
    auto it = dgraphs_.find(key);
    if (it != dgraphs_.end()) return it->second.get();
  }
  if (!provider_) throw std::runtime_error("no decode graph for this batch / context bucket");
  drain();  // the provider captures on the GPU: nothing of ours may be in flight
  const int64_t t0 = now_ns();
  provider_("decode", B, ctx, greedy);
  capture_ns_ += now_ns() - t0;
  n_captures_++;
  std::lock_guard<std::mutex> lk(gmu_);
  auto it = dgraphs_.find(key);
  if (it == dgraphs_.end()) throw std::runtime_error("graph provider registered no decode graph");
  return it->second.get();
}

const PrefillGraphDesc* EngineLoop::find_prefill_graph(int rows, int nseq, bool greedy) {
  // the smallest registered graph of this row bucket holding >= nseq sequences (a graph's
  // sequence bucket is the engine's, which a server with a smaller batch may round up)
  std::lock_guard<std::mutex> lk(gmu_);
  const PrefillGraphDesc* best = nullptr;
  for (const auto& kv : pgraphs_) {
    const PrefillGraphDesc* g = kv.second.get();
    if (g->rows == rows && g->greedy == greedy && g->n_seq >= nseq && (!best || g->n_seq < best->n_seq))
      best = g;
  }
  return best;
}

const PrefillGraphDesc* EngineLoop::prefill_graph(int rows, int nseq, bool greedy) {
  const auto key = std::make_tuple(rows, nseq, greedy);
  if (const PrefillGraphDesc* g = find_prefill_graph(rows, nseq, greedy)) return g;
  if (!provider_) return nullptr;
  // capturing costs a few forwards and a drained pipeline: a shape seen once (a rare mix of
  // riders and new prompts) runs eagerly, one that recurs is captured
  if (++puses_[key] < cfg_.prefill_graph_after) return nullptr;
  drain();
  const int64_t t0 = now_ns();
  provider_("prefill", rows, nseq, greedy);
  capture_ns_ += now_ns() - t0;
  n_captures_++;
  return find_prefill_graph(rows, nseq, greedy);
}

// ------------------------------------------------------------------ lifecycle
void EngineLoop::start() {
  std::lock_guard<std::mutex> lk(mu_);
  if (started_) return;
  const HipApi& h = hip_api();
  if (!h.ok) throw std::runtime_error("native engine loop: " + h.error);
  started_ = true;
  th_ = std::thread([this] { run(); });
}

void EngineLoop::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  done_cv_.notify_all();
  if (th_.joinable()) th_.join();
  if (mirror_ && !mirror_stopped_) {  // the followers' mirrors return from run()
    mirror_stopped_ = true;
    try {
      mirror_->stop();
    } catch (...) {
    }
  }
}

int64_t EngineLoop::submit(const std::vector<int>& prompt, int max_new, bool stop_on_eos,
                           const LoopSampling& s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!dead_.empty()) throw std::runtime_error("engine replica is down: " + dead_);
  // decode graphs are picked with slack for chunks that run past a reply's end (pick() in
  // decode): a request whose prompt + max_new + slack exceeds the largest context bucket is
  // refused here, alone, instead of failing every running request later
  if (!cfg_.ctx_buckets.empty() &&
      (int64_t)prompt.size() + max_new + 2 * cfg_.decode_chunk + 2 > cfg_.ctx_buckets.back())
    throw std::invalid_argument("prompt + max_new exceeds the largest context bucket (" +
                                std::to_string(cfg_.ctx_buckets.back()) + " tokens)");
  const int64_t id = sched_.add((int)prompt.size(), max_new, stop_on_eos, cfg_.eos);
  Req& r = reqs_[id];
  r.prompt = prompt;
  r.samp = s;
  r.t_submit = now_ns();
  cv_.notify_all();
  return id;
}

void EngineLoop::cancel(int64_t id) {
  std::lock_guard<std::mutex> lk(mu_);
  cancels_.insert(id);
  cv_.notify_all();
}

bool EngineLoop::wait(int64_t id, double timeout_s, LoopResult* out) {
  std::unique_lock<std::mutex> lk(mu_);
  auto it = reqs_.find(id);
  if (it == reqs_.end()) throw std::runtime_error("unknown request " + std::to_string(id));
  auto ready = [&] { return it->second.done || stop_ || !dead_.empty(); };
  if (timeout_s < 0)
    done_cv_.wait(lk, ready);
  else
    done_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready);
  const Req& r = it->second;
  const SchedRequest& s = sched_.get(id);
  out->tokens = s.tokens;
  out->done = r.done;
  out->error = r.error;
  if (!r.done && (!dead_.empty() || stop_)) {  // nobody will finish it: report why now
    out->done = true;
    out->error = "engine replica is down: " + (dead_.empty() ? std::string("loop stopped") : dead_);
  }
  out->done_reason = s.finish_reason.empty() ? (r.done ? "stop" : "") : s.finish_reason;
  out->prompt_eval_count = s.prompt_len;
  const int64_t t_first = r.t_first ? r.t_first : now_ns();
  const int64_t t_end = r.t_done ? r.t_done : now_ns();
  out->prompt_eval_ns = t_first - (r.t_admit ? r.t_admit : r.t_submit);
  out->eval_ns = t_end - t_first;
  out->total_ns = t_end - r.t_submit;
  out->ttft_ns = t_first - r.t_submit;
  return r.done;
}

std::vector<int> EngineLoop::wait_tokens(int64_t id, size_t have, double timeout_s, bool* done) {
  std::unique_lock<std::mutex> lk(mu_);
  auto it = reqs_.find(id);
  if (it == reqs_.end()) throw std::runtime_error("unknown request " + std::to_string(id));
  auto ready = [&] {
    return it->second.done || stop_ || !dead_.empty() || sched_.get(id).tokens.size() > have;
  };
  done_cv_.wait_for(lk, std::chrono::duration<double>(std::max(0.0, timeout_s)), ready);
  const auto& toks = sched_.get(id).tokens;
  *done = it->second.done || !dead_.empty() || stop_;  // a dead loop finishes nothing more
  if (toks.size() <= have) return {};
  return std::vector<int>(toks.begin() + have, toks.end());
}

void EngineLoop::release(int64_t id) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = reqs_.find(id);
  if (it == reqs_.end()) return;
  if (it->second.done) {
    sched_.release(id);
    reqs_.erase(it);
  } else {
    it->second.released = true;  // dropped when it finishes
    cancels_.insert(id);
    cv_.notify_all();
  }
}

void EngineLoop::stall(double seconds) {
  std::lock_guard<std::mutex> lk(mu_);
  stall_until_ = now_ns() + (int64_t)(seconds * 1e9);
  cv_.notify_all();
}

std::string EngineLoop::dead() {
  std::lock_guard<std::mutex> lk(mu_);
  return dead_;
}

std::map<std::string, double> EngineLoop::metrics() {
  std::lock_guard<std::mutex> lk(mu_);
  std::map<std::string, double> m;
  m["requests"] = n_requests_;
  m["tokens"] = n_tokens_;
  m["prefill_calls"] = n_prefill_calls_;
  m["prefill_tokens"] = n_prefill_tokens_;
  m["eager_prefill_calls"] = n_eager_prefill_;
  m["decode_calls"] = n_decode_calls_;
  m["decode_steps"] = n_decode_steps_;
  m["k_graph_launches"] = n_k_graph_launches_;  // whole k_steps-step decode graph replays
  m["speculated_chunks"] = n_speculated_;
  m["state_loads"] = n_loads_;
  m["errors"] = n_errors_;
  m["busy_s"] = busy_ns_ * 1e-9;
  m["prefill_s"] = prefill_ns_ * 1e-9;
  m["decode_s"] = decode_ns_ * 1e-9;
  m["capture_s"] = capture_ns_ * 1e-9;  // inside the graph provider (captures)
  m["captures"] = n_captures_;
  m["eager_prefill_s"] = eager_ns_ * 1e-9;
  m["prefill_wait_s"] = prefill_wait_ns_ * 1e-9;  // draining decode work before a prefill
  m["prefill_waits"] = n_prefill_waits_;  // prefills that found decode work in flight
  m["admit_wait_hits"] = n_admit_hits_;   // the admit wait saw the expected arrivals
  m["admit_wait_misses"] = n_admit_misses_;
  m["running"] = sched_.n_running();
  m["waiting"] = sched_.n_waiting();
  m["free_kv_pages"] = sched_.free_pages();
  m["native_loop"] = 1;
  m["dp_world"] = cfg_.dp_world;
  if (mirror_) {
    m["mirror_frames"] = mirror_->frames();
    m["mirror_bytes"] = mirror_->bytes();
    m["mirror_follower_faults"] = mirror_->follower_faults();
  }
  return m;
}

// ------------------------------------------------------------------ the loop
void EngineLoop::run() {
  const HipApi& h = hip_api();
  try {
    hip_check(h.setDevice(cfg_.device), "hipSetDevice");
    hip_check(h.streamCreateWithFlags(&stream_, 1 /* hipStreamNonBlocking */), "hipStreamCreate");
    for (int i = 0; i < 2; ++i) {
      void* e = nullptr;
      hip_check(h.eventCreateWithFlags(&e, 2 /* hipEventDisableTiming */), "hipEventCreate");
      events_.push_back(e);
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(mu_);
    dead_ = e.what();
    done_cv_.notify_all();
    return;
  }
  while (true) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      while (!stop_ && flight_.empty() && cancels_.empty() && sched_.n_running() == 0 &&
             sched_.n_waiting() == 0)
        cv_.wait_for(lk, std::chrono::milliseconds(500));
      while (!stop_ && now_ns() < stall_until_)
        cv_.wait_for(lk, std::chrono::nanoseconds(std::min<int64_t>(stall_until_ - now_ns(),
                                                                     50000000)));
      if (stop_) break;
    }
    const int64_t t0 = now_ns();
    try {
      step();
    } catch (const std::exception& e) {
      fail_all(e.what());
    }
    busy_ns_ += now_ns() - t0;
  }
  try {
    drain();
  } catch (...) {
  }
}

void EngineLoop::fail_all(const std::string& why) {
  try {
    drain();
  } catch (...) {
    flight_.clear();
  }
  loaded_ = nullptr;
  std::lock_guard<std::mutex> lk(mu_);
  n_errors_++;
  for (auto& kv : reqs_) {
    if (kv.second.done) continue;
    kv.second.error = why;
    sched_.cancel(kv.first);
  }
  sched_.flush_deferred();
  const int64_t t = now_ns();
  for (int64_t id : sched_.take_finished()) {
    auto it = reqs_.find(id);
    if (it == reqs_.end()) continue;
    it->second.done = true;
    it->second.t_done = t;
    if (it->second.released) {
      sched_.release(id);
      reqs_.erase(it);
    }
  }
  done_cv_.notify_all();
}

void EngineLoop::step() {
  std::vector<int64_t> admitted;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int64_t id : cancels_) sched_.cancel(id);
    cancels_.clear();
    SchedPlan plan = sched_.schedule();
    admitted = plan.prefill;
    const int64_t t = now_ns();
    for (int64_t id : admitted) reqs_[id].t_admit = t;
  }
  if (!admitted.empty()) run_prefill(admitted);
  std::vector<int64_t> running;
  bool waiting;
  {
    std::lock_guard<std::mutex> lk(mu_);
    running = sched_.running();
    waiting = sched_.n_waiting() > 0;
  }
  if (!admitted.empty() && cfg_.prefill_first && waiting) running.clear();
  if (!running.empty()) {
    decode(running, waiting);
  } else if (!flight_.empty()) {
    drain();
  }
  // retire
  int done = 0;
  {
    std::lock_guard<std::mutex> lk(mu_);
    // pages of requests that ended without a decode chunk after them (a 1-token reply, a
    // cancel, a reply that ended in its prefill) wait in the deferred list for the next
    // collect(); with nothing in flight nothing can still write them: free them now (else
    // an idle loop holds them until the next request decodes)
    if (flight_.empty()) sched_.flush_deferred();
    const int64_t t = now_ns();
    for (int64_t id : sched_.take_finished()) {
      auto it = reqs_.find(id);
      if (it == reqs_.end()) continue;
      ++done;
      Req& r = it->second;
      r.done = true;
      r.t_done = t;
      if (!r.t_first) r.t_first = t;
      n_requests_++;
      n_tokens_ += (long)sched_.get(id).tokens.size();
      if (r.released) {
        sched_.release(id);
        reqs_.erase(it);
      }
    }
    if (done) done_cv_.notify_all();
  }
  if (done && cfg_.admit_wait_us > 0) {
    // replies just went out: their peers usually send the next request within a fraction
    // of a millisecond -- admit it at THIS step boundary (bounded wait; only while a batch
    // slot is free, so a full batch never waits)
    std::unique_lock<std::mutex> lk(mu_);
    const int free = cfg_.max_batch - sched_.n_running() - sched_.n_waiting();
    if (free > 0) {
      const int want = std::min(done, free);
      const bool hit = cv_.wait_for(lk, std::chrono::microseconds((int64_t)cfg_.admit_wait_us),
                                    [&] { return stop_ || sched_.n_waiting() >= want; });
      (hit ? n_admit_hits_ : n_admit_misses_)++;
    }
  }
}

// ------------------------------------------------------------------ prefill
void EngineLoop::run_prefill(const std::vector<int64_t>& admitted) {
  const HipApi& h = hip_api();
  const int64_t tw = now_ns();
  if (!flight_.empty()) n_prefill_waits_++;
  drain();  // riders' last tokens must be current; nothing may write KV concurrently
  loaded_ = nullptr;  // the decode state no longer matches (new rows; riders advance)
  const int64_t t0 = now_ns();
  prefill_wait_ns_ += t0 - tw;
  struct Seq {
    int64_t id;
    const std::vector<int>* prompt;  // admitted: the prompt
    int pos = 0, tok = 0;            // rider: one row
    std::vector<int> pages;
    LoopSampling samp;
  };
  std::vector<Seq> seqs;
  std::vector<int64_t> riders;
  int n_rows = 0, max_pages_needed = 0;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int64_t id : admitted) {
      Seq s;
      s.id = id;
      s.prompt = &reqs_[id].prompt;
      s.pages = sched_.get(id).pages;
      s.samp = reqs_[id].samp;
      n_rows += (int)s.prompt->size();
      max_pages_needed = std::max(max_pages_needed, (int)((s.prompt->size() + 63) / 64));
      seqs.push_back(std::move(s));
    }
    if (cfg_.mixed && cfg_.dp_world <= 1) {
      // running sequences fill the chunk's last 64-row tile, never start another one
      // riders_all: every running sequence rides (bounded by the chunk budget) -- under high
      // concurrency a prompt admitted alone would otherwise stall the sequences that do not
      // fit the last tile for a whole step; else only the last 64-row tile's free rows
      int room = cfg_.riders_all ? cfg_.max_prefill_tokens - n_rows
                                 : (n_rows + 63) / 64 * 64 - n_rows;
      for (int64_t id : sched_.running()) {
        if (room <= 0 || (int)seqs.size() >= cfg_.max_batch) break;
        if (std::find(admitted.begin(), admitted.end(), id) != admitted.end()) continue;
        const SchedRequest& r = sched_.get(id);
        if (r.state != RUNNING || r.tokens.empty()) continue;
        // a rider past the prefill graphs' block-table width would send the whole chunk
        // down the eager path: it decodes in the next step instead
        if (r.pos / 64 + 1 > cfg_.prefill_max_pages) continue;
        Seq s;
        s.id = id;
        s.prompt = nullptr;
        s.pos = r.pos;
        s.tok = r.tokens.back();
        s.pages = r.pages;
        s.samp = reqs_[id].samp;
        max_pages_needed = std::max(max_pages_needed, r.pos / 64 + 1);
        seqs.push_back(std::move(s));
        riders.push_back(id);
        --room;
        ++n_rows;
      }
    }
  }
  const int nseq = (int)seqs.size();
  bool greedy = true;
  for (auto& s : seqs) greedy &= s.samp.greedy();
  const int rb = bucket(n_rows, cfg_.row_buckets);
  const int sb = std::min(bucket(nseq, cfg_.batch_buckets), cfg_.max_batch);
  const PrefillGraphDesc* g = nullptr;
  const bool dp = cfg_.dp_world > 1;
  if (!dp && rb > 0 && sb >= nseq && max_pages_needed <= cfg_.prefill_max_pages)
    g = prefill_graph(rb, sb, greedy);
  std::vector<int> first(nseq, 0);
  if (dp) {
    // EP a2a group: every rank prefills its own share of the new sequences, padded to the
    // largest share's rows (the exchange needs equal row counts), through the eager path;
    // the followers' first tokens come back with their frame's status
    riders.clear();
    std::vector<int64_t> ids;
    for (auto& s : seqs)
      if (s.prompt) ids.push_back(s.id);
    const std::vector<std::vector<int64_t>> parts = split_by_home(ids, true);
    std::map<int64_t, const Seq*> by_id;
    for (auto& s : seqs) by_id[s.id] = &s;
    int pad = 1;
    for (auto& part : parts) {
      int rows = 0;
      for (int64_t id : part) rows += (int)by_id[id]->prompt->size();
      pad = std::max(pad, rows);
    }
    auto share = [&](const std::vector<int64_t>& part, std::vector<std::vector<int>>* prompts,
                     std::vector<std::vector<int>>* pages, std::vector<int>* starts,
                     std::vector<LoopSampling>* samp) {
      for (int64_t id : part) {
        const Seq* q = by_id[id];
        prompts->push_back(*q->prompt);
        pages->push_back(q->pages);
        starts->push_back(0);
        samp->push_back(q->samp);
      }
    };
    const int64_t te = now_ns();
    uint32_t mseq = 0;
    if (mirror_) {
      for (size_t f = 1; f < parts.size(); ++f) {
        std::vector<std::vector<int>> pr, pg;
        std::vector<int> st;
        std::vector<LoopSampling> sp;
        share(parts[f], &pr, &pg, &st, &sp);
        mirror_->set_target((int)f - 1);
        mirror_->eager(pr, pg, st, sp, pad, true);
      }
      mseq = mirror_->flush();
    }
    std::vector<std::vector<int>> pr, pg;
    std::vector<int> st;
    std::vector<LoopSampling> sp;
    share(parts[0], &pr, &pg, &st, &sp);
    const std::vector<int> mine = eager_(pr, pg, st, sp, pad);
    eager_ns_ += now_ns() - te;
    n_eager_prefill_++;
    follower_check(mseq, "eager prefill");
    std::map<int64_t, int> tok;
    for (size_t i = 0; i < parts[0].size() && i < mine.size(); ++i) tok[parts[0][i]] = mine[i];
    for (size_t f = 1; f < parts.size(); ++f) {
      const std::vector<int> t = mirror_ ? mirror_->take_tokens((int)f - 1, mseq) : std::vector<int>();
      if (t.size() < parts[f].size())
        throw std::runtime_error("group follower " + std::to_string(f) + " sent " +
                                 std::to_string(t.size()) + " first tokens for " +
                                 std::to_string(parts[f].size()) + " sequences");
      for (size_t i = 0; i < parts[f].size(); ++i) tok[parts[f][i]] = t[i];
    }
    int b = 0;
    for (auto& s : seqs) {
      if (!s.prompt) break;
      first[b++] = tok[s.id];
    }
  } else if (!g) {
    // beyond every captured shape (a long prompt): Python's chunked eager prefill, without
    // riders (they decode in the next step instead)
    if (!eager_) throw std::runtime_error("prompt exceeds the captured prefill shapes");
    std::vector<std::vector<int>> prompts, pages;
    std::vector<int> starts;
    std::vector<LoopSampling> samp;
    for (auto& s : seqs) {
      if (!s.prompt) continue;
      prompts.push_back(*s.prompt);
      pages.push_back(s.pages);
      starts.push_back(0);
      samp.push_back(s.samp);
    }
    riders.clear();
    const int64_t te = now_ns();
    uint32_t mseq = 0;
    if (mirror_) {  // the followers run the same eager prefill (its collectives pair up)
      mirror_->eager(prompts, pages, starts, samp);
      mseq = mirror_->flush();
    }
    first = eager_(prompts, pages, starts, samp, 0);
    eager_ns_ += now_ns() - te;
    n_eager_prefill_++;
    follower_check(mseq, "eager prefill");
  } else {
    // chunk metadata (PrefillGraph.host_meta, engine/graph.py)
    int32_t* m = (int32_t*)pinned(kPrefillMeta, g->meta_len * 4);
    std::memset(m, 0, g->meta_len * 4);
    const int P = g->max_pages, R = g->rows, S = g->n_seq;
    int32_t* bt = m + g->off_bt;
    int32_t* seq = m + g->off_seq;
    int32_t* pos = m + g->off_pos;
    int32_t* ids = m + g->off_ids;
    int32_t* slots = m + g->off_slots;
    int32_t* ctx = m + g->off_ctx;
    int32_t* out = m + g->off_out;
    int32_t* spos = m + g->off_spos;
    int32_t* tiles = m + g->off_tiles;
    int r = 0;
    for (int b = 0; b < nseq; ++b) {
      const Seq& s = seqs[b];
      for (size_t i = 0; i < s.pages.size() && (int)i < P; ++i) bt[b * P + i] = s.pages[i];
      if (s.prompt) {
        for (size_t i = 0; i < s.prompt->size(); ++i, ++r) {
          seq[r] = b;
          pos[r] = (int)i;
          ids[r] = (*s.prompt)[i];
        }
      } else {
        seq[r] = b;
        pos[r] = s.pos;
        ids[r] = s.tok;
        ++r;
      }
      out[b] = r - 1;
      spos[b] = pos[r - 1];
    }
    const int n = r;
    for (int i = n; i < R; ++i) {  // dummy rows: sequence S (the null page), no KV write,
      seq[i] = S;                    // positions wrapped inside its block-table row
      pos[i] = (i - n) % (P * 64);
    }
    for (int i = 0; i < R; ++i) {
      const int p = pos[i];
      slots[i] = i < n ? bt[seq[i] * P + p / 64] * 64 + p % 64 : -1;
      ctx[i] = p + 1;
    }
    int nt = 0;
    for (int i = 0; i < R;) {  // runs of consecutive positions of one sequence, cut at qtile
      int e = i + 1;
      while (e < R && e - i < g->qtile && seq[e] == seq[i] && pos[e] == pos[e - 1] + 1) ++e;
      if (nt >= g->max_tiles) throw std::runtime_error("prefill tiles exceed the graph's bound");
      tiles[4 * nt] = i;
      tiles[4 * nt + 1] = e - i;
      tiles[4 * nt + 2] = seq[i];
      tiles[4 * nt + 3] = pos[i];
      ++nt;
      i = e;
    }
    hip_check(h.memcpyAsync(g->meta, m, g->meta_len * 4, kH2D, stream_), "prefill meta H2D");
    staged(kPrefillMeta);
    if (!g->greedy) {
      float* tf = (float*)pinned(kSampF, S * 4);
      int32_t* tk = (int32_t*)pinned(kSampI, S * 4);
      float* tp = (float*)pinned(kSampP, S * 4);
      int64_t* sd = (int64_t*)pinned(kSampS, S * 8);
      for (int b = 0; b < S; ++b) {
        const LoopSampling d = b < nseq ? seqs[b].samp : LoopSampling();
        tf[b] = d.temperature;
        tk[b] = d.top_k;
        tp[b] = d.top_p;
        sd[b] = d.seed;
      }
      hip_check(h.memcpyAsync(g->temp, tf, S * 4, kH2D, stream_), "samp H2D");
      hip_check(h.memcpyAsync(g->topk, tk, S * 4, kH2D, stream_), "samp H2D");
      hip_check(h.memcpyAsync(g->topp, tp, S * 4, kH2D, stream_), "samp H2D");
      hip_check(h.memcpyAsync(g->seeds, sd, S * 8, kH2D, stream_), "samp H2D");
      for (int sl : {(int)kSampF, (int)kSampI, (int)kSampP, (int)kSampS}) staged(sl);
    }
    uint32_t pf_seq = 0;
    if (mirror_) {
      const char K = 'P';
      mirror_->h2d(K, g->rows, g->n_seq, g->greedy, kFMeta, m, g->meta_len * 4);
      if (!g->greedy) {
        mirror_->h2d(K, g->rows, g->n_seq, g->greedy, kFTemp, pinned_[kSampF].first, S * 4);
        mirror_->h2d(K, g->rows, g->n_seq, g->greedy, kFTopk, pinned_[kSampI].first, S * 4);
        mirror_->h2d(K, g->rows, g->n_seq, g->greedy, kFTopp, pinned_[kSampP].first, S * 4);
        mirror_->h2d(K, g->rows, g->n_seq, g->greedy, kFSeeds, pinned_[kSampS].first, S * 8);
      }
      mirror_->launch(K, g->rows, g->n_seq, g->greedy, 0, 1);
      pf_seq = mirror_->flush();
    }
    hip_check(h.graphLaunch(g->exec, stream_), "prefill graph launch");
    int32_t* f = (int32_t*)pinned(kFirst, S * 4);
    hip_check(h.memcpyAsync(f, g->first, nseq * 4, kD2H, stream_), "first tokens D2H");
    int32_t* ew = (int32_t*)pinned(kErr0 + 2, 4);
    if (g->err) hip_check(h.memcpyAsync(ew, g->err, 4, kD2H, stream_), "fault word D2H");
    int32_t* ea = (int32_t*)pinned(kAux0 + 2, 4);
    if (aux_err_) hip_check(h.memcpyAsync(ea, aux_err_, 4, kD2H, stream_), "split fault D2H");
    int32_t* ec = (int32_t*)pinned(kColl0 + 2, 4);
    if (coll_err_) hip_check(h.memcpyAsync(ec, coll_err_, 4, kD2H, stream_), "collective fault D2H");
    hip_check(h.streamSynchronize(stream_), "prefill sync");
    if (coll_err_ && *ec != 0) on_coll_fault("prefill");
    if (g->err && *ew != 0) on_fault(g->err, "prefill");
    if (aux_err_ && *ea != 0) on_fault(aux_err_, "prefill (split-K)");
    follower_check(pf_seq, "prefill");
    for (int b = 0; b < nseq; ++b) first[b] = f[b];
  }
  const int64_t t1 = now_ns();
  {
    std::lock_guard<std::mutex> lk(mu_);
    int b = 0;
    for (auto& s : seqs) {
      if (!s.prompt) break;
      auto it = reqs_.find(s.id);
      if (it != reqs_.end()) it->second.t_first = t1;
      sched_.on_first_token(s.id, first[b]);
      n_prefill_tokens_ += (long)s.prompt->size();
      ++b;
    }
    if (!riders.empty()) {
      std::vector<std::vector<int>> toks;
      for (size_t i = 0; i < riders.size(); ++i) toks.push_back({first[b + i]});
      sched_.on_decode_tokens(riders, toks);
      n_decode_steps_++;
    }
    n_prefill_calls_++;
    prefill_ns_ += t1 - t0;
  }
  done_cv_.notify_all();
}

// ------------------------------------------------------------------ decode
void EngineLoop::launch_chunk(const DecodeGraphDesc* g, const std::vector<int64_t>& ids,
                              bool load, int k) {
  const HipApi& h = hip_api();
  const bool dp = cfg_.dp_world > 1;
  std::vector<std::vector<int64_t>> parts;
  if (dp) parts = split_by_home(ids, false);
  const std::vector<int64_t>& mine = dp ? parts[0] : ids;
  if (load) {
    const int B = g->B, P = g->max_pages;
    const size_t n = (size_t)B * (4 + P);
    int32_t* m = (int32_t*)pinned(kDecodeMeta, n * 4);
    float* tf = nullptr;
    int32_t* tk = nullptr;
    float* tp = nullptr;
    int64_t* sd = nullptr;
    if (!g->greedy) {
      tf = (float*)pinned(kSampF, B * 4);
      tk = (int32_t*)pinned(kSampI, B * 4);
      tp = (float*)pinned(kSampP, B * 4);
      sd = (int64_t*)pinned(kSampS, B * 8);
    }
    decode_meta(g, mine, m, tf, tk, tp, sd);
    hip_check(h.memcpyAsync(g->meta, m, n * 4, kH2D, stream_), "decode meta H2D");
    staged(kDecodeMeta);
    hip_check(h.memsetAsync(g->step, 0, 4, stream_), "step reset");
    if (g->keys && g->keys_bytes)
      hip_check(h.memsetAsync(g->keys, 0, g->keys_bytes, stream_), "keys reset");
    if (!g->greedy) {
      hip_check(h.memcpyAsync(g->temp, tf, B * 4, kH2D, stream_), "samp H2D");
      hip_check(h.memcpyAsync(g->topk, tk, B * 4, kH2D, stream_), "samp H2D");
      hip_check(h.memcpyAsync(g->topp, tp, B * 4, kH2D, stream_), "samp H2D");
      hip_check(h.memcpyAsync(g->seeds, sd, B * 8, kH2D, stream_), "samp H2D");
      for (int sl : {(int)kSampF, (int)kSampI, (int)kSampP, (int)kSampS}) staged(sl);
    }
    if (mirror_) {
      const char K = 'D';
      if (!dp) {
        mirror_->h2d(K, g->B, g->ctx, g->greedy, kFMeta, m, n * 4);
        if (!g->greedy) {
          mirror_->h2d(K, g->B, g->ctx, g->greedy, kFTemp, tf, B * 4);
          mirror_->h2d(K, g->B, g->ctx, g->greedy, kFTopk, tk, B * 4);
          mirror_->h2d(K, g->B, g->ctx, g->greedy, kFTopp, tp, B * 4);
          mirror_->h2d(K, g->B, g->ctx, g->greedy, kFSeeds, sd, B * 8);
        }
      } else {  // every follower its own share's state (EP a2a: different sequences per rank)
        std::vector<int32_t> fm(n);
        std::vector<float> ftf(B), ftp(B);
        std::vector<int32_t> ftk(B);
        std::vector<int64_t> fsd(B);
        for (size_t f = 1; f < parts.size(); ++f) {
          decode_meta(g, parts[f], fm.data(), g->greedy ? nullptr : ftf.data(), ftk.data(),
                      ftp.data(), fsd.data());
          mirror_->set_target((int)f - 1);
          mirror_->h2d(K, g->B, g->ctx, g->greedy, kFMeta, fm.data(), n * 4);
          if (!g->greedy) {
            mirror_->h2d(K, g->B, g->ctx, g->greedy, kFTemp, ftf.data(), B * 4);
            mirror_->h2d(K, g->B, g->ctx, g->greedy, kFTopk, ftk.data(), B * 4);
            mirror_->h2d(K, g->B, g->ctx, g->greedy, kFTopp, ftp.data(), B * 4);
            mirror_->h2d(K, g->B, g->ctx, g->greedy, kFSeeds, fsd.data(), B * 8);
          }
        }
        mirror_->set_target(-1);
      }
      mirror_->memset0(K, g->B, g->ctx, g->greedy, kFStep, 4);
      if (g->keys && g->keys_bytes) mirror_->memset0(K, g->B, g->ctx, g->greedy, kFKeys, g->keys_bytes);
    }
    loaded_ = g;
    loaded_ids_ = ids;
    loaded_steps_ = 0;
    n_loads_++;
  }
  // k steps: whole k_steps-step graphs first (each one-step launch leaves host work that
  // the next launch of the prompt-chunk graph pays: ~8 us per launch, bench/graph_switch_probe.py)
  const int nk = (g->exec_k && g->k_steps > 1) ? k / g->k_steps : 0;
  const int n1 = k - nk * g->k_steps;
  uint32_t mseq = 0;
  if (mirror_) {  // the followers replay the same graphs (their collectives pair with ours)
    if (nk) mirror_->launch('D', g->B, g->ctx, g->greedy, 1, (uint32_t)nk);
    if (n1) mirror_->launch('D', g->B, g->ctx, g->greedy, 0, (uint32_t)n1);
    if (dp)  // each follower sends its share's k new tokens back with this frame's status
      for (size_t f = 1; f < parts.size(); ++f) {
        mirror_->set_target((int)f - 1);
        mirror_->tokens('D', g->B, g->ctx, g->greedy, 0, (uint32_t)loaded_steps_, (uint32_t)k,
                        (uint32_t)parts[f].size());
      }
    mseq = mirror_->flush();
  }
  for (int i = 0; i < nk; ++i) {
    hip_check(h.graphLaunch(g->exec_k, stream_), "decode graph launch");
    n_k_graph_launches_++;
  }
  for (int i = 0; i < n1; ++i) hip_check(h.graphLaunch(g->exec, stream_), "decode graph launch");
  Chunk c;
  c.g = g;
  c.ids = mine;
  if (dp) c.parts.assign(parts.begin() + 1, parts.end());
  c.s0 = loaded_steps_;
  c.k = k;
  c.buf = hist_buf_;
  c.mseq = mseq;
  hist_buf_ ^= 1;
  // this chunk's k columns of every row: [B, k] packed
  const size_t hb = (size_t)g->B * k * 4;
  void* dst = pinned(kHist0 + c.buf, hb);
  hip_check(h.memcpy2DAsync(dst, (size_t)k * 4, g->hist + c.s0, (size_t)g->max_steps * 4,
                            (size_t)k * 4, g->B, kD2H, stream_),
            "hist D2H");
  if (g->err)
    hip_check(h.memcpyAsync(pinned(kErr0 + c.buf, 4), g->err, 4, kD2H, stream_), "fault D2H");
  if (aux_err_)
    hip_check(h.memcpyAsync(pinned(kAux0 + c.buf, 4), aux_err_, 4, kD2H, stream_), "split fault D2H");
  if (coll_err_)
    hip_check(h.memcpyAsync(pinned(kColl0 + c.buf, 4), coll_err_, 4, kD2H, stream_), "collective fault D2H");
  c.ev = events_[c.buf];
  hip_check(h.eventRecord(c.ev, stream_), "hipEventRecord");
  loaded_steps_ += k;
  flight_.push_back(std::move(c));
  n_decode_calls_++;
}

void EngineLoop::collect() {
  const HipApi& h = hip_api();
  Chunk c = std::move(flight_.front());
  flight_.pop_front();
  hip_check(h.eventSynchronize(c.ev), "decode chunk sync");
  if (coll_err_ && *(int32_t*)pinned_[kColl0 + c.buf].first != 0) {
    flight_.clear();
    on_coll_fault("decode");
  }
  if (c.g->err && *(int32_t*)pinned_[kErr0 + c.buf].first != 0) {
    flight_.clear();  // chunks behind a faulted one ran on its invalid state
    on_fault(c.g->err, "decode");
  }
  if (aux_err_ && *(int32_t*)pinned_[kAux0 + c.buf].first != 0) {
    flight_.clear();
    on_fault(aux_err_, "decode (split-K)");
  }
  if (mirror_ && c.mseq) {
    const uint32_t bits = mirror_->await(c.mseq);
    if (bits) {
      flight_.clear();
      if (bits & 4) on_coll_fault("decode (on a follower rank)");
      on_fault(nullptr, "decode (on a follower rank)");
    }
  }
  faults_in_row_ = 0;  // a clean decode chunk: whatever faulted before was transient
  const int32_t* hist = (const int32_t*)pinned_[kHist0 + c.buf].first;
  std::vector<std::vector<int>> toks(c.ids.size());
  for (size_t b = 0; b < c.ids.size(); ++b) {
    const int32_t* row = hist + (size_t)b * c.k;
    toks[b].assign(row, row + c.k);
  }
  std::vector<int64_t> ids = c.ids;
  for (size_t f = 0; f < c.parts.size(); ++f) {  // dp groups: the followers' shares
    const std::vector<int> t = mirror_->take_tokens((int)f, c.mseq);
    if (t.size() < c.parts[f].size() * (size_t)c.k) {
      flight_.clear();
      throw std::runtime_error("group follower " + std::to_string(f + 1) + " sent " +
                               std::to_string(t.size()) + " tokens for " +
                               std::to_string(c.parts[f].size()) + " x " + std::to_string(c.k));
    }
    for (size_t b = 0; b < c.parts[f].size(); ++b) {
      ids.push_back(c.parts[f][b]);
      toks.emplace_back(t.begin() + b * c.k, t.begin() + (b + 1) * c.k);
    }
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    sched_.on_decode_tokens(ids, toks);
    n_decode_steps_ += c.k;
    if (flight_.empty()) sched_.flush_deferred();  // nothing in flight can touch them now
  }
  done_cv_.notify_all();
}

// A kernel's fault word was set (a bounded spin gave up: a split-K slice or a hand-off
// that never arrived).  The word is cleared -- the Python path does the same in
// check_faults -- so one transient timeout fails only the requests in this step;
// kMaxFaultsInRow faulted steps in a row mark the replica dead, and the router stops
// sending it traffic.
// Group followers report their own fault words per frame (mirror.h status back channel):
// a fault on any rank fails the step here like a local one.
void EngineLoop::follower_check(uint32_t seq, const char* where) {
  if (!mirror_ || !seq) return;
  const uint32_t bits = mirror_->await(seq);
  if (bits & 4) on_coll_fault((std::string(where) + " (on a follower rank)").c_str());
  if (bits) on_fault(nullptr, (std::string(where) + (bits & 2 ? " (failed on a follower rank)"
                                                               : " (on a follower rank)")).c_str());
}

void EngineLoop::on_fault(int32_t* err, const char* where) {
  const HipApi& h = hip_api();
  if (err) (void)h.memsetAsync(err, 0, 4, stream_);
  (void)h.streamSynchronize(stream_);
  if (mirror_) {
    // every rank's words back to 0 ('F'), and the followers' reports of the frames before it
    // (chunks in flight behind the faulted one: still faulted) consumed here, so the next
    // step starts clean
    try {
      mirror_->faults();
      const uint32_t fs = mirror_->flush();
      if (fs) (void)mirror_->await(fs);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu_);
      dead_ = std::string("group follower lost after a fault: ") + e.what();
    }
  }
  loaded_ = nullptr;
  const std::string why = std::string("kernel fault word set during ") + where +
                          " (results invalid)";
  if (++faults_in_row_ >= kMaxFaultsInRow) {
    std::lock_guard<std::mutex> lk(mu_);
    dead_ = why + ", " + std::to_string(faults_in_row_) + " steps in a row";
  }
  throw std::runtime_error(why);
}

// An IPC collective gave up waiting for a peer (parallel/custom_ar.py CollectiveTimeout):
// the group's epochs are out of step and later calls skip their waits, so every number from
// here on is wrong.  Unlike a split-K fault this is not transient: the replica is dead (the
// Python loop raises the same from LlamaModel.check_faults).
void EngineLoop::on_coll_fault(const char* where) {
  const HipApi& h = hip_api();
  (void)h.streamSynchronize(stream_);
  loaded_ = nullptr;
  const std::string why = std::string("collective timeout during ") + where +
                          ": a peer rank never arrived (the TP / EP group is broken)";
  {
    std::lock_guard<std::mutex> lk(mu_);
    dead_ = why;
  }
  throw std::runtime_error(why);
}

void EngineLoop::drain() {
  while (!flight_.empty()) collect();
}

void EngineLoop::decode(const std::vector<int64_t>& running_in, bool waiting) {
  const int64_t t0 = now_ns();
  std::vector<int64_t> running = running_in;
  // chunk length: long chunks amortise the host round trip; a waiting request shortens it
  // (it is admitted at the next chunk boundary)
  int k = waiting ? 2 : ((int)running.size() < cfg_.max_batch ? std::max(2, cfg_.decode_chunk / 2)
                                                              : cfg_.decode_chunk);
  // steps until the first length stop among ids (minus what is already in flight): a chunk
  // ends there, so that reply goes out and its slot is refilled without waiting for more
  auto steps_left = [&](const std::vector<int64_t>& ids, int inflight) {
    int left = 1 << 30;
    std::lock_guard<std::mutex> lk(mu_);
    for (int64_t id : ids) {
      const SchedRequest& r = sched_.get(id);
      left = std::min(left, r.max_new - (int)r.tokens.size());
    }
    return left - inflight;
  };
  auto pick = [&](const std::vector<int64_t>& ids) {
    int need = 1;
    bool greedy = true;
    std::lock_guard<std::mutex> lk(mu_);
    for (int64_t id : ids) {
      const SchedRequest& r = sched_.get(id);
      // slack: a chunk may run past a request's end while the host reads the previous one
      need = std::max(need, r.prompt_len + r.max_new + 2 * cfg_.decode_chunk + 2);
      greedy &= reqs_[id].samp.greedy();
    }
    int rows = (int)ids.size();
    if (cfg_.dp_world > 1) {  // every rank runs the largest share's batch bucket
      std::vector<int> per(cfg_.dp_world, 0);
      rows = 0;
      for (int64_t id : ids) rows = std::max(rows, ++per[reqs_[id].home]);
    }
    const int B = bucket(rows, cfg_.batch_buckets);
    const int C = bucket(need, cfg_.ctx_buckets);
    if (B < 0 || C < 0) throw std::runtime_error("decode batch / context exceeds the buckets");
    return std::make_tuple(B, C, greedy);
  };
  auto [B, C, greedy] = pick(running);
  const DecodeGraphDesc* g = decode_graph(B, C, greedy);
  // speculating a chunk behind the running one doubles what a newly arriving request waits
  // for before its prefill: only while no batch slot is free (nobody could be admitted)
  const bool spec = cfg_.pipeline && !waiting &&
                    (cfg_.pipeline_free_slots || (int)running.size() >= cfg_.max_batch);
  int inflight = 0;
  for (const Chunk& c : flight_) inflight += c.k;
  const int spec_k = spec && !flight_.empty() ? std::min(k, steps_left(running, inflight)) : 0;
  if (spec_k > 0 && flight_.back().g == g && flight_.back().ids == running &&
      loaded_ == g && loaded_steps_ + spec_k <= g->max_steps) {
    // the running set is unchanged as far as the host knows (and no length stop falls inside
    // the chunk in flight): enqueue the next chunk on the device-resident state, then read
    // the previous one while it runs
    launch_chunk(g, running, false, spec_k);
    n_speculated_++;
    collect();
    decode_ns_ += now_ns() - t0;
    return;
  }
  drain();
  {
    std::lock_guard<std::mutex> lk(mu_);
    // a request just finished: its reply goes out at this step's retire and its peer's next
    // request (or one already waiting for the slot) would otherwise wait a whole chunk
    // before its prefill.  Return to the step boundary instead (the next step decodes if
    // nobody came).
    if (sched_.n_finished() > 0) {
      decode_ns_ += now_ns() - t0;
      return;
    }
    running = sched_.running();
  }
  if (running.empty()) return;
  k = std::max(1, std::min(k, steps_left(running, 0)));
  std::tie(B, C, greedy) = pick(running);
  g = decode_graph(B, C, greedy);
  const bool load = !(loaded_ == g && loaded_ids_ == running && loaded_steps_ + k <= g->max_steps);
  launch_chunk(g, running, load, k);
  if (!cfg_.pipeline) collect();
  decode_ns_ += now_ns() - t0;
}

}  // namespace p2p

// ------------------------------------------------------------------ plain-C table
// (runtime/loop_capi.h): the engine C ABI library drives the loop through these, so a
// request from the node daemon never enters Python.  Exceptions stay on this side.
namespace {

using p2p::EngineLoop;

void copy_err(const std::exception& e, char* err, int errlen) {
  if (err && errlen > 0) {
    strncpy(err, e.what(), (size_t)errlen - 1);
    err[errlen - 1] = 0;
  }
}

int64_t c_submit(void* loop, const int32_t* ids, int n, int max_new, int stop_on_eos, float temp,
                 int top_k, float top_p, int64_t seed, char* err, int errlen) {
  try {
    p2p::LoopSampling s;
    s.temperature = temp;
    s.top_k = top_k;
    s.top_p = top_p;
    s.seed = seed;
    return ((EngineLoop*)loop)->submit(std::vector<int>(ids, ids + n), max_new, stop_on_eos != 0, s);
  } catch (const std::exception& e) {
    copy_err(e, err, errlen);
    return -1;
  }
}

int c_wait(void* loop, int64_t id, double timeout_s, P2PLoopResult* out) {
  memset(out, 0, sizeof(*out));
  p2p::LoopResult r;
  try {
    ((EngineLoop*)loop)->wait(id, timeout_s, &r);
  } catch (const std::exception& e) {
    r.error = e.what();
  }
  out->n_tokens = (int)r.tokens.size();
  out->tokens = (int32_t*)malloc(sizeof(int32_t) * std::max<size_t>(1, r.tokens.size()));
  for (size_t i = 0; i < r.tokens.size(); ++i) out->tokens[i] = r.tokens[i];
  out->done = r.done ? 1 : 0;
  out->prompt_eval_count = r.prompt_eval_count;
  out->prompt_eval_ns = r.prompt_eval_ns;
  out->eval_ns = r.eval_ns;
  out->total_ns = r.total_ns;
  out->ttft_ns = r.ttft_ns;
  strncpy(out->done_reason, r.done_reason.c_str(), sizeof(out->done_reason) - 1);
  out->error = r.error.empty() ? nullptr : strdup(r.error.c_str());
  return 0;
}

int c_wait_tokens(void* loop, int64_t id, size_t have, double timeout_s, int32_t** toks, int* n,
                  int* done) {
  bool d = false;
  std::vector<int> t;
  try {
    t = ((EngineLoop*)loop)->wait_tokens(id, have, timeout_s, &d);
  } catch (const std::exception&) {
    d = true;  // unknown request / loop gone: the caller's final wait() reports why
  }
  *toks = (int32_t*)malloc(sizeof(int32_t) * std::max<size_t>(1, t.size()));
  for (size_t i = 0; i < t.size(); ++i) (*toks)[i] = t[i];
  *n = (int)t.size();
  *done = d ? 1 : 0;
  return 0;
}

void c_cancel(void* loop, int64_t id) { ((EngineLoop*)loop)->cancel(id); }
void c_release(void* loop, int64_t id) { ((EngineLoop*)loop)->release(id); }

int c_dead(void* loop, char* buf, int len) {
  const std::string d = ((EngineLoop*)loop)->dead();
  if (buf && len > 0) {
    strncpy(buf, d.c_str(), (size_t)len - 1);
    buf[len - 1] = 0;
  }
  return (int)d.size();
}

void c_free(void* p) { free(p); }

const P2PLoopApi g_loop_api = {P2P_LOOP_API_VERSION, c_submit, c_wait, c_wait_tokens, c_cancel,
                               c_release, c_dead, c_free};

}  // namespace

extern "C" __attribute__((visibility("default"))) const P2PLoopApi* p2p_loop_api(void) {
  return &g_loop_api;
}
