#include "scheduler.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace p2p {

BlockAllocator::BlockAllocator(int num_pages, int reserved)
    : num_pages_(num_pages), reserved_(reserved), used_(num_pages, 0) {
  if (num_pages <= reserved) throw std::runtime_error("BlockAllocator: not enough pages");
  for (int p = num_pages - 1; p >= reserved; --p) free_.push_back(p);
  for (int p = 0; p < reserved; ++p) used_[p] = 1;
}

std::vector<int> BlockAllocator::alloc(int n) {
  if (n < 0 || n > (int)free_.size())
    throw std::runtime_error("KV cache exhausted: want " + std::to_string(n) + " pages, " +
                             std::to_string(free_.size()) + " free");
  std::vector<int> out(free_.end() - n, free_.end());
  std::reverse(out.begin(), out.end());
  free_.resize(free_.size() - n);
  for (int p : out) used_[p] = 1;
  return out;
}

void BlockAllocator::free(const std::vector<int>& pages) {
  for (int p : pages) {
    if (p < reserved_ || p >= num_pages_ || !used_[p])
      throw std::runtime_error("BlockAllocator: double free / bad page " + std::to_string(p));
    used_[p] = 0;
    free_.push_back(p);
  }
}

Scheduler::Scheduler(int num_pages, int page_size, int max_batch, int max_prefill_tokens,
                     int max_ctx)
    : alloc_(num_pages, 1), page_size_(page_size), max_batch_(max_batch),
      max_prefill_tokens_(max_prefill_tokens), max_ctx_(max_ctx) {}

int64_t Scheduler::add(int prompt_len, int max_new, bool stop_on_eos, const std::vector<int>& eos) {
  if (prompt_len <= 0) throw std::runtime_error("empty prompt");
  if (max_new <= 0) throw std::runtime_error("max_new_tokens must be > 0");
  if (prompt_len + max_new > max_ctx_)
    throw std::runtime_error("prompt + max_new_tokens exceeds the context limit " +
                             std::to_string(max_ctx_));
  int need = (prompt_len + max_new + page_size_ - 1) / page_size_;
  if (need > alloc_.num_pages() - 1) throw std::runtime_error("request larger than the KV cache");
  SchedRequest r;
  r.id = next_id_++;
  r.prompt_len = prompt_len;
  r.max_new = max_new;
  r.stop_on_eos = stop_on_eos;
  r.eos = eos;
  reqs_[r.id] = r;
  waiting_.push_back(r.id);
  return r.id;
}

bool Scheduler::cancel(int64_t id) {
  auto it = reqs_.find(id);
  if (it == reqs_.end()) return false;
  SchedRequest& r = it->second;
  if (r.state == WAITING) {
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
    r.state = CANCELLED;
    r.finish_reason = "cancelled";
    finished_.push_back(id);
    return true;
  }
  if (r.state == RUNNING) {
    finish(r, "cancelled");
    r.state = CANCELLED;
    return true;
  }
  return false;
}

SchedPlan Scheduler::schedule() {
  SchedPlan p;
  int budget = max_prefill_tokens_;
  while (!waiting_.empty() && (int)running_.size() + (int)p.prefill.size() < max_batch_) {
    SchedRequest& r = reqs_[waiting_.front()];
    int need = (r.prompt_len + r.max_new + page_size_ - 1) / page_size_;
    if (!alloc_.can_alloc(need)) break;
    if (!p.prefill.empty() && r.prompt_len > budget) break;  // first one always fits (chunked)
    r.pages = alloc_.alloc(need);
    budget -= r.prompt_len;
    p.prefill.push_back(r.id);
    waiting_.pop_front();
  }
  for (int64_t id : p.prefill) {
    reqs_[id].state = RUNNING;
  }
  p.decode = running_;
  for (int64_t id : p.prefill) running_.push_back(id);
  return p;
}

void Scheduler::finish(SchedRequest& r, const char* reason) {
  if (r.state != RUNNING) return;
  r.state = FINISHED;
  r.finish_reason = reason;
  if (defer_free_)
    deferred_.insert(deferred_.end(), r.pages.begin(), r.pages.end());
  else
    alloc_.free(r.pages);
  r.pages.clear();
  running_.erase(std::remove(running_.begin(), running_.end(), r.id), running_.end());
  finished_.push_back(r.id);
}

static bool is_eos(const SchedRequest& r, int t) {
  return r.stop_on_eos && std::find(r.eos.begin(), r.eos.end(), t) != r.eos.end();
}

void Scheduler::on_first_token(int64_t id, int token) {
  SchedRequest& r = reqs_.at(id);
  if (r.state != RUNNING) return;
  r.pos = r.prompt_len;  // the first generated token is fed at position prompt_len
  if (is_eos(r, token)) {
    finish(r, "stop");
    return;
  }
  r.tokens.push_back(token);
  if ((int)r.tokens.size() >= r.max_new) finish(r, "length");
}

void Scheduler::on_decode_tokens(const std::vector<int64_t>& ids,
                                 const std::vector<std::vector<int>>& toks) {
  for (size_t i = 0; i < ids.size(); ++i) {
    auto it = reqs_.find(ids[i]);
    if (it == reqs_.end()) continue;
    SchedRequest& r = it->second;
    for (int t : toks[i]) {
      if (r.state != RUNNING) break;
      r.pos += 1;
      if (is_eos(r, t)) {
        finish(r, "stop");
        break;
      }
      r.tokens.push_back(t);
      if ((int)r.tokens.size() >= r.max_new) finish(r, "length");
    }
  }
}

void Scheduler::flush_deferred() {
  if (deferred_.empty()) return;
  alloc_.free(deferred_);
  deferred_.clear();
}

std::vector<int64_t> Scheduler::take_finished() {
  std::vector<int64_t> out;
  out.swap(finished_);
  return out;
}

const SchedRequest& Scheduler::get(int64_t id) const {
  auto it = reqs_.find(id);
  if (it == reqs_.end()) throw std::runtime_error("unknown request " + std::to_string(id));
  return it->second;
}

void Scheduler::release(int64_t id) {
  auto it = reqs_.find(id);
  if (it != reqs_.end() && (it->second.state == FINISHED || it->second.state == CANCELLED))
    reqs_.erase(it);
}

}  // namespace p2p
