// Continuous-batching request scheduler + paged-KV block allocator (native
// runtime of the suggest-reply engine; the reference has one blocking Ollama
// call per click, `web/streamlit_app.py:163-165`).
//
// Policy: every request reserves the KV pages for prompt + max_new_tokens at
// admission (no preemption / recompute is ever needed), waiting requests are
// admitted FCFS while a batch slot, pages and the per-step prefill token budget
// allow, and prefill is scheduled before decode (minimises TTFT; decode resumes
// on the next step with the new rows merged into the running batch).
#pragma once
#include <stdint.h>

#include <deque>
#include <string>
#include <map>
#include <mutex>
#include <vector>

namespace p2p {

class BlockAllocator {
 public:
  BlockAllocator(int num_pages, int reserved = 1);  // pages [0, reserved) are never handed out
  std::vector<int> alloc(int n);                      // throws std::runtime_error if short
  void free(const std::vector<int>& pages);
  bool can_alloc(int n) const { return (int)free_.size() >= n; }
  int free_count() const { return (int)free_.size(); }
  int num_pages() const { return num_pages_; }

 private:
  int num_pages_;
  int reserved_;
  std::vector<int> free_;
  std::vector<uint8_t> used_;
};

enum ReqState : int { WAITING = 0, RUNNING = 1, FINISHED = 2, CANCELLED = 3 };

struct SchedRequest {
  int64_t id = 0;
  int prompt_len = 0;
  int max_new = 0;
  bool stop_on_eos = true;
  std::vector<int> eos;
  int state = WAITING;
  std::vector<int> pages;
  std::vector<int> tokens;  // generated tokens
  int pos = 0;              // position of the last token fed (next decode input)
  std::string finish_reason;
};

struct SchedPlan {
  std::vector<int64_t> prefill;  // admitted this step (run prefill, then on_first_token)
  std::vector<int64_t> decode;   // running requests for the decode step(s)
};

class Scheduler {
 public:
  Scheduler(int num_pages, int page_size, int max_batch, int max_prefill_tokens, int max_ctx);
  int64_t add(int prompt_len, int max_new, bool stop_on_eos, const std::vector<int>& eos);
  bool cancel(int64_t id);
  SchedPlan schedule();
  void on_first_token(int64_t id, int token);
  // toks[i] are the tokens produced for ids[i] by consecutive decode steps.
  void on_decode_tokens(const std::vector<int64_t>& ids, const std::vector<std::vector<int>>& toks);
  std::vector<int64_t> take_finished();
  size_t n_finished() const { return finished_.size(); }  // not yet taken
  const SchedRequest& get(int64_t id) const;
  void release(int64_t id);  // forget a finished request (frees nothing else)
  int n_waiting() const { return (int)waiting_.size(); }
  int n_running() const { return (int)running_.size(); }
  const std::vector<int64_t>& running() const { return running_; }
  int free_pages() const { return alloc_.free_count(); }
  int page_size() const { return page_size_; }
  // Deferred page release: a finished request's pages are held back until
  // flush_deferred() -- the native loop keeps a decode chunk in flight while it reads
  // the previous one, and that chunk may still write KV for a request that just hit EOS.
  void set_defer_free(bool on) { defer_free_ = on; }
  void flush_deferred();
  int n_deferred_pages() const { return (int)deferred_.size(); }

 private:
  void finish(SchedRequest& r, const char* reason);
  BlockAllocator alloc_;
  int page_size_, max_batch_, max_prefill_tokens_, max_ctx_;
  int64_t next_id_ = 1;
  std::map<int64_t, SchedRequest> reqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
  std::vector<int64_t> finished_;
  bool defer_free_ = false;
  std::vector<int> deferred_;
};

}  // namespace p2p
