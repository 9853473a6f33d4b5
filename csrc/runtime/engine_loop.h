// Native engine step loop: continuous batching driven from a C++ thread that replays the
// engine's captured hipGraphs ("engine step loop (separate C++ thread)").
//
// Python builds the model once (weights, KV cache, autotuned GEMM launch codes) and
// captures the graphs -- decode steps per (batch bucket, context bucket, greedy|sampled)
// and prefill chunks per (row bucket, sequence bucket) -- then registers each graph's
// hipGraphExec handle and the device addresses of its input/output buffers here.  From
// then on a request never enters Python on the hot path:
//
//   submit()  -> Scheduler (admission, KV pages)            [HTTP threads]
//   loop      -> prefill: chunk metadata built in pinned host memory, one H2D copy, one
//                hipGraphLaunch, first tokens D2H                [engine thread]
//             -> decode: per chunk, the batch state is loaded only when the running set
//                changed; k graph replays; the NEXT chunk is enqueued before the host reads
//                this one's tokens (finish detection lags one chunk; pages of a request
//                that ended are released only after the chunk still in flight drained)
//   wait()    <- tokens, Ollama timing fields                    [HTTP threads]
//
// Shapes no registered graph covers ask the provider callback (Python, once per shape)
// to capture and register one; prompts longer than the largest prefill bucket go to the
// eager-prefill callback (Python's chunked prefill).
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "runtime/scheduler.h"

namespace p2p {

class MirrorSender;  // runtime/mirror.h
class LoopServer;    // runtime/loop_remote.h

struct LoopSampling {
  float temperature = 0.f;  // <= 0: greedy
  int top_k = 40;
  float top_p = 0.9f;
  int64_t seed = 0;
  bool greedy() const { return temperature <= 0.f; }
};

// DecodeState (engine/graph.py) of one captured decode graph.
struct DecodeGraphDesc {
  int B = 0, max_pages = 0, ctx = 0;
  bool greedy = true;
  void* exec = nullptr;         // hipGraphExec_t of one decode step (advances its own state)
  int32_t* meta = nullptr;      // [B * (4 + max_pages)]: ids | pos | ctx | slots | block tables
  int32_t* hist = nullptr;      // [B, max_steps] tokens by step
  int max_steps = 0;
  int32_t* step = nullptr;      // [1] step counter (zeroed at load)
  void* keys = nullptr;         // greedy argmax keys (zeroed at load)
  size_t keys_bytes = 0;
  float* temp = nullptr;        // sampler slots [B] (sampled graphs)
  int32_t* topk = nullptr;
  float* topp = nullptr;
  int64_t* seeds = nullptr;
  int32_t* err = nullptr;       // the graph workspace's fault word (nonzero = invalid results)
  void* exec_k = nullptr;       // optional: k_steps decode steps in one graph (greedy)
  int k_steps = 0;
};

// PrefillGraph (engine/graph.py) of one captured prefill chunk.
struct PrefillGraphDesc {
  int rows = 0, n_seq = 0, max_pages = 0, qtile = 16, max_tiles = 0;
  bool greedy = true;
  void* exec = nullptr;
  int32_t* meta = nullptr;
  size_t meta_len = 0;  // int32 elements
  // int32 offsets into meta
  size_t off_bt = 0, off_seq = 0, off_pos = 0, off_ids = 0, off_slots = 0, off_ctx = 0,
         off_out = 0, off_spos = 0, off_tiles = 0;
  int32_t* first = nullptr;  // [n_seq] first tokens
  float* temp = nullptr;     // sampler slots [n_seq] (sampled graphs)
  int32_t* topk = nullptr;
  float* topp = nullptr;
  int64_t* seeds = nullptr;
  int32_t* err = nullptr;    // the graph workspace's fault word
};

struct LoopConfig {
  int num_pages = 0, page_size = 64, max_batch = 16, max_prefill_tokens = 1024, max_ctx = 4096;
  std::vector<int> eos;
  int decode_chunk = 8;
  double admit_wait_us = 500.0;
  bool prefill_first = true;
  bool mixed = true;     // running sequences ride in a prefill chunk as one row each
  bool riders_all = false;  // all of them (budget permitting), not just the last tile's room
  bool pipeline = true;  // enqueue decode chunk i+1 before reading chunk i
  int device = 0;
  std::vector<int> batch_buckets{1, 2, 4, 8, 16, 32, 64};
  std::vector<int> ctx_buckets{256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536, 131072};
  std::vector<int> row_buckets{16, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768, 1024};
  int prefill_max_pages = 64;  // block-table width of the prefill graphs (their context bucket / 64)
  bool pipeline_free_slots = false;  // speculate decode chunks even while a batch slot is free
  int prefill_graph_after = 2;  // a chunk shape is captured on its n-th use (eager before)
  // EP all-to-all groups (DP attention): the group's dp_world ranks hold DIFFERENT sequences.
  // Each sequence gets a home rank at admission (fewest live sequences); every prefill / decode
  // call runs each rank's share through the same shapes (prefill padded to the largest share,
  // decode at the largest share's batch bucket), followers' frames carry their own metadata,
  // and their tokens come back on the status channel (runtime/mirror.h 'T', 'E').  Prefill is
  // the eager callback (the a2a prefill's exact-count exchange is not a graph).  1 = off.
  int dp_world = 1;
};

struct LoopResult {
  std::vector<int> tokens;
  std::string done_reason;
  std::string error;
  int prompt_eval_count = 0;
  int64_t prompt_eval_ns = 0, eval_ns = 0, total_ns = 0, ttft_ns = 0;
  bool done = false;
};

class EngineLoop {
 public:
  // kind "decode": (B bucket, ctx bucket, -); "prefill": (row bucket, seq bucket, -)
  using GraphProvider = std::function<void(const std::string& kind, int a, int b, bool greedy)>;
  // pad_rows > 0 (dp_world > 1): run exactly that many rows (the rest dummies), as every rank
  // of an EP a2a group must
  using EagerPrefill = std::function<std::vector<int>(
      const std::vector<std::vector<int>>& prompts, const std::vector<std::vector<int>>& pages,
      const std::vector<int>& starts, const std::vector<LoopSampling>& sampling, int pad_rows)>;

  explicit EngineLoop(const LoopConfig& cfg);
  ~EngineLoop();
  EngineLoop(const EngineLoop&) = delete;
  EngineLoop& operator=(const EngineLoop&) = delete;

  void add_decode_graph(const DecodeGraphDesc& d);
  void add_prefill_graph(const PrefillGraphDesc& d);
  void set_provider(GraphProvider p);
  void set_eager_prefill(EagerPrefill f);
  // TP / EP group leader: every device operation of the loop (metadata copies, counter
  // resets, graph replays, eager prefills) is also sent to the followers' EngineMirror over
  // these channel fds (owned by the caller), one frame per step (runtime/mirror.h)
  void set_mirror(const std::vector<int>& fds);
  // A second device fault word checked with every graph's own: the kernels' split-K word
  // (p2p_split_fault_word_ptr), which the graphs' split-K GEMMs set when a slice gives up.
  void set_aux_fault(uintptr_t word) { aux_err_ = reinterpret_cast<int32_t*>(word); }
  // the IPC collectives' timeout word (CustomAllReduce.err[0]): nonzero = the group is broken
  void set_coll_fault(uintptr_t word) { coll_err_ = reinterpret_cast<int32_t*>(word); }
  // a graph provider about to capture (kind, a, b, greedy): the followers capture it too
  void mirror_provide(const std::string& kind, int a, int b, bool greedy);
  // serve requests from other processes on the abstract unix socket @name (the node of a
  // multi-GPU cluster routes to this replica natively: runtime/loop_remote.h)
  void serve(const std::string& name);
  void start();
  void stop();
  void shutdown();  // stop + release the loop's HIP resources (stream, events, pinned memory)

  int64_t submit(const std::vector<int>& prompt, int max_new, bool stop_on_eos,
                 const LoopSampling& s);
  void cancel(int64_t id);
  // Blocks until the request finished (true) or timeout_s passed (false; < 0 = no limit).
  bool wait(int64_t id, double timeout_s, LoopResult* out);
  // Streaming: tokens past the first `have` (blocks until some arrive, the request ends,
  // or timeout).  *done is set when the request is over (finished, cancelled or failed).
  std::vector<int> wait_tokens(int64_t id, size_t have, double timeout_s, bool* done);
  void release(int64_t id);  // forget a finished request
  void stall(double seconds);  // fault injection: no step for `seconds`
  std::map<std::string, double> metrics();
  std::string dead();

 private:
  struct Req {
    std::vector<int> prompt;
    LoopSampling samp;
    int64_t t_submit = 0, t_admit = 0, t_first = 0, t_done = 0;
    bool done = false;
    bool released = false;  // the caller gave up on it: drop it when it finishes
    std::string error;
    int home = 0;           // dp_world > 1: the rank that holds this sequence
  };
  struct Chunk {  // a decode chunk in flight
    const DecodeGraphDesc* g = nullptr;
    std::vector<int64_t> ids;
    int s0 = 0, k = 0;  // hist columns [s0, s0 + k)
    int buf = 0;        // pinned hist buffer index
    void* ev = nullptr;
    uint32_t mseq = 0;  // the group frame that launched it (follower status, mirror.h)
    std::vector<std::vector<int64_t>> parts;  // dp_world > 1: follower f + 1's rows (ids)
  };

  void run();
  void step();
  void run_prefill(const std::vector<int64_t>& admitted);
  void decode(const std::vector<int64_t>& running, bool waiting);
  void launch_chunk(const DecodeGraphDesc* g, const std::vector<int64_t>& ids, bool load, int k);
  void collect();  // read the oldest chunk in flight
  void drain();    // read every chunk in flight
  void fail_all(const std::string& why);
  // dp_world > 1: the ids by home rank (index = rank), homes given to ids that have none
  std::vector<std::vector<int64_t>> split_by_home(const std::vector<int64_t>& ids, bool assign);
  // one rank's decode metadata (DecodeState layout) and sampler slots for `ids`
  void decode_meta(const DecodeGraphDesc* g, const std::vector<int64_t>& ids, int32_t* m,
                   float* tf, int32_t* tk, float* tp, int64_t* sd);
  [[noreturn]] void on_fault(int32_t* err, const char* where);
  [[noreturn]] void on_coll_fault(const char* where);
  void follower_check(uint32_t seq, const char* where);
  const DecodeGraphDesc* decode_graph(int B, int ctx, bool greedy);
  const PrefillGraphDesc* find_prefill_graph(int rows, int nseq, bool greedy);
  const PrefillGraphDesc* prefill_graph(int rows, int nseq, bool greedy);
  static int bucket(int x, const std::vector<int>& b);
  void* pinned(int slot, size_t bytes);
  // after the H2D copies from a staging slot are enqueued: the slot is not rewritten (or
  // freed) until they have run -- see pinned()
  void staged(int slot);
  int64_t now_ns() const;

  LoopConfig cfg_;
  Scheduler sched_;
  std::mutex mu_;
  std::condition_variable cv_;       // loop wake-up
  std::condition_variable done_cv_;  // waiters
  std::map<int64_t, Req> reqs_;
  std::set<int64_t> cancels_;
  bool stop_ = false;
  bool started_ = false;
  int64_t stall_until_ = 0;
  std::string dead_;
  std::thread th_;

  // graphs (registered from Python; keyed by bucket)
  std::mutex gmu_;
  std::map<std::tuple<int, int, bool>, std::unique_ptr<DecodeGraphDesc>> dgraphs_;
  std::map<std::tuple<int, int, bool>, std::unique_ptr<PrefillGraphDesc>> pgraphs_;
  std::map<std::tuple<int, int, bool>, int> puses_;  // uses of not-yet-captured chunk shapes
  GraphProvider provider_;
  EagerPrefill eager_;
  std::unique_ptr<MirrorSender> mirror_;
  std::unique_ptr<LoopServer> server_;
  bool mirror_stopped_ = false;

  // device-side state of the loop thread
  void* stream_ = nullptr;
  std::vector<std::pair<void*, size_t>> pinned_;  // host staging buffers by slot
  std::vector<void*> staged_ev_;                   // per slot: recorded after its last H2D
  std::vector<void*> events_;                     // one per hist buffer
  std::deque<Chunk> flight_;                      // decode chunks enqueued, not yet read (<= 2)
  const DecodeGraphDesc* loaded_ = nullptr;       // graph whose state holds loaded_ids_
  std::vector<int64_t> loaded_ids_;
  int loaded_steps_ = 0;                          // replays since the last load
  int hist_buf_ = 0;
  int home_rr_ = 0;  // dp_world > 1: rotating tie-break of home assignment
  static constexpr int kMaxFaultsInRow = 3;
  int faults_in_row_ = 0;  // consecutive steps that ended with a kernel fault word set
  int32_t* aux_err_ = nullptr;  // set_aux_fault
  int32_t* coll_err_ = nullptr;  // set_coll_fault

  // metrics
  std::atomic<long> n_requests_{0}, n_tokens_{0}, n_prefill_calls_{0}, n_decode_calls_{0},
      n_decode_steps_{0}, n_k_graph_launches_{0}, n_prefill_tokens_{0}, n_speculated_{0}, n_loads_{0}, n_errors_{0},
      n_eager_prefill_{0};
  std::atomic<int64_t> busy_ns_{0}, prefill_ns_{0}, decode_ns_{0}, capture_ns_{0}, eager_ns_{0},
      prefill_wait_ns_{0}, n_captures_{0}, n_prefill_waits_{0}, n_admit_hits_{0},
      n_admit_misses_{0};
};

}  // namespace p2p
