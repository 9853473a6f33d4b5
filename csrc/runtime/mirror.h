// Native serving loop for TP / EP groups: the leader's EngineLoop drives its followers.
//
// Every rank of a group captured the same graphs (same shapes, same collectives), so a
// group step is the same sequence of device operations on every rank: copy the step's
// metadata into a graph's input buffers, reset its counters, replay it.  The leader's loop
// (engine_loop.cc) records each of those operations as it performs them -- a few hundred
// bytes per prefill chunk or decode chunk -- and sends them, one frame per step, over the
// group's host channel (the socketpair that connects the leader and each follower process);
// a follower's EngineMirror thread applies them in order on its own stream to its own
// graphs, so the collectives inside the graphs line up without any Python in the loop on
// either side.  Operations that need the model code -- capturing a graph for a new shape,
// the eager prefill of a prompt longer than every captured chunk -- travel the same
// channel, in order, and call back into the follower's Python (graph provider / eager
// prefill), exactly as the leader's loop calls its own.
//
// Replaces the Python LockstepEngine broadcast of round 4 (engine/cluster.py) on the hot
// path: no pickled plan per call, no host sync per decode chunk on the followers, and the
// multi-step decode graphs (captured collectively, through the same provider calls) serve
// groups too.  (The reference has no parallelism; this serves BASELINE configs 3 and 5,
// the same click as `web/streamlit_app.py:161-173`.)
//
// Frame: u32 length (little endian) + payload; payload = a sequence of records
//   'H' h2d      kind a b greedy field n data[n]   (copy into the graph's field buffer)
//   'M' memset0  kind a b greedy field n            (zero n bytes of a field)
//   'L' launch   kind a b greedy which count        (which 0: one-step exec, 1: exec_k)
//   'F' faults                                      (zero every graph's fault word)
//   'V' provide  kind a b greedy                    (capture + register this shape)
//   'E' eager    n_seq pad_rows want {prompt, pages, start, sampling} x n_seq
//   'T' tokens   kind a b greedy src s0 k rows    (dp groups: send back hist[rows][s0 .. s0+k)
//                                                  of a decode graph, src 0, or the first
//                                                  tokens of a prefill graph, src 1)
//   'S' stop
// kind: 'D' decode graph (B, ctx bucket), 'P' prefill graph (rows, seq bucket).
//
// EP all-to-all groups (DP attention, LoopConfig::dp_world): the ranks hold different
// sequences, so a frame is per follower -- the shared records (launches, counter resets,
// captures) go to every follower, the metadata / sampling / eager-prefill records of a
// follower's own share only to it (MirrorSender::set_target) -- and the status answer of a
// frame carries that follower's tokens ('T' records, an 'E' record with want = 1).
//
// Status back channel (a kernel fault is local to the rank that saw it): for
// every frame a follower answers on the same socket, once the device work the frame
// enqueued has completed, with {u32 frame seq, u32 bits}: bit 0 = a fault word of a graph
// the frame launched, or the follower device's split-K word, was set; bit 1 = a host-side
// failure applying the frame (a provider / eager-prefill callback raised, an unknown
// graph) -- the rest of that frame is skipped and the mirror stays alive.  The leader
// reads the answers of every frame up to a step's before it hands that step's tokens out
// (MirrorSender::await), so a fault on any rank fails the step on the leader too; its
// fault record ('F') clears every graph word and the split-K word on the followers.
// Answer: {u32 seq, u32 bits, u32 ntok, i32 tok[ntok]} (ntok = 0 unless the frame asked).
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "runtime/engine_loop.h"

namespace p2p {

enum MirrorField : uint8_t {
  kFMeta = 0,
  kFStep = 1,
  kFKeys = 2,
  kFTemp = 3,
  kFTopk = 4,
  kFTopp = 5,
  kFSeeds = 6,
};

class MirrorSender {
 public:
  explicit MirrorSender(std::vector<int> fds) : fds_(std::move(fds)), bufs_(fds_.size()) {}
  // records from here on go to follower f only (0-based; -1: every follower, the default)
  void set_target(int f) { target_ = f; }
  void tokens(char kind, int a, int b, bool greedy, uint8_t src, uint32_t s0, uint32_t k,
              uint32_t rows);
  void h2d(char kind, int a, int b, bool greedy, uint8_t field, const void* src, size_t n);
  void memset0(char kind, int a, int b, bool greedy, uint8_t field, size_t n);
  void launch(char kind, int a, int b, bool greedy, uint8_t which, uint32_t count);
  void faults();
  void provide(char kind, int a, int b, bool greedy);
  void eager(const std::vector<std::vector<int>>& prompts,
             const std::vector<std::vector<int>>& pages, const std::vector<int>& starts,
             const std::vector<LoopSampling>& samp, int pad_rows = 0, bool want = false);
  void stop();
  // one frame to every follower; returns its sequence number (1, 2, ...; 0 if nothing was
  // pending); throws if a channel is broken
  uint32_t flush();
  // the OR of every follower's status bits over the frames up to `seq` (blocks until each
  // follower answered them; throws if a follower is gone or silent past timeout_s)
  uint32_t await(uint32_t seq, double timeout_s = 120.0);
  // the tokens follower f sent back with frame seq (after await(seq); empty if none)
  std::vector<int> take_tokens(int f, uint32_t seq);
  long frames() const { return frames_; }
  long bytes() const { return bytes_; }
  long follower_faults() const { return follower_faults_; }

 private:
  void head(char op, char kind, int a, int b, bool greedy);
  template <class T>
  void put(T v) {
    append(reinterpret_cast<const char*>(&v), sizeof(T));
  }
  void append(const char* p, size_t n) {
    if (target_ >= 0) {
      bufs_[target_].append(p, n);
    } else {
      for (auto& b : bufs_) b.append(p, n);
    }
  }
  std::vector<int> fds_;
  std::vector<uint32_t> acked_;  // per follower: the last frame it answered
  std::vector<std::string> bufs_;  // per follower: its pending frame
  int target_ = -1;
  std::vector<std::map<uint32_t, std::vector<int>>> toks_;  // per follower: frame -> tokens
  std::recursive_mutex mu_;
  std::atomic<long> frames_{0}, bytes_{0}, follower_faults_{0};
};

class EngineMirror {
 public:
  // P2P_MIRROR_INJECT_FAULT=N (tests): after the N-th frame that launches graphs, this rank
  // sets its split-K fault word, as a slice that gave up on this rank only would;
  // P2P_MIRROR_INJECT_COLL=N: the same for its IPC collectives' timeout word
  EngineMirror(int fd, int device);
  ~EngineMirror();
  EngineMirror(const EngineMirror&) = delete;
  EngineMirror& operator=(const EngineMirror&) = delete;

  void add_decode_graph(const DecodeGraphDesc& d);
  void add_prefill_graph(const PrefillGraphDesc& d);
  void set_provider(EngineLoop::GraphProvider p) { provider_ = std::move(p); }
  void set_eager_prefill(EngineLoop::EagerPrefill f) { eager_ = std::move(f); }
  // this device's split-K fault word (p2p_split_fault_word_ptr): reported and cleared like
  // the graphs' own words
  void set_aux_fault(uintptr_t word) { aux_err_ = reinterpret_cast<int32_t*>(word); }
  // the IPC collectives' timeout word: reported with every frame as status bit 4 and never
  // reset by 'F' (a collective timeout breaks the group: the leader marks the replica dead)
  void set_coll_fault(uintptr_t word) { coll_err_ = reinterpret_cast<int32_t*>(word); }
  // Applies frames until the leader's stop ("" returned) or a failure (its description:
  // a closed channel, an unknown graph, a HIP error).  Blocking; call without the GIL.
  std::string run();
  std::map<std::string, double> metrics();
  void shutdown();  // release the stream and staging buffers

 private:
  struct Graph {
    char kind;
    int a, b;
    bool greedy;
    void* exec = nullptr;
    void* exec_k = nullptr;
    void* fields[7] = {};
    int32_t* err = nullptr;
    int32_t* hist = nullptr;   // decode: [B][max_steps] tokens by step
    int max_steps = 0;
    int32_t* first = nullptr;  // prefill: [n_seq] first tokens
  };
  // what a frame sends back besides its status bits: device token rows to copy (after the
  // frame's work) and tokens the host already has (an eager prefill's first tokens)
  struct TokCopy {
    const int32_t* src;
    size_t pitch;  // int32 elements between rows
    uint32_t rows, k;
  };
  struct FrameOut {
    std::vector<TokCopy> copies;
    std::vector<int> host;
  };
  Graph* find(char kind, int a, int b, bool greedy);
  // applies one frame; returns the host failure bit (the frame's remaining records skipped)
  uint32_t apply(const std::string& frame, std::vector<int32_t*>* launched, FrameOut* out);
  void* staging(size_t n);
  void report(uint32_t seq, const std::vector<int32_t*>& launched, uint32_t host_bits,
              const FrameOut& out);
  void reporter();

  int fd_, device_;
  void* stream_ = nullptr;
  std::mutex gmu_;
  std::map<std::tuple<char, int, int, bool>, Graph> graphs_;
  EngineLoop::GraphProvider provider_;
  EngineLoop::EagerPrefill eager_;
  // double-buffered pinned staging of the frames' h2d payloads: buffer i is reused only
  // once the operations of the frame that last used it completed (its event)
  void* stage_[2] = {nullptr, nullptr};
  size_t stage_n_[2] = {0, 0};
  void* stage_ev_[2] = {nullptr, nullptr};
  int cur_ = 0;
  int32_t* aux_err_ = nullptr;
  int32_t* coll_err_ = nullptr;
  long inject_at_ = 0, inject_coll_at_ = 0, launch_frames_ = 0;
  // status reports: a ring of pinned word slots + events, drained in order by reporter()
  static constexpr int kRep = 32, kRepWords = 16, kRepToks = 8192;
  struct Report {
    uint32_t seq, host_bits;
    int slot, nwords, ntok;
    int coll = -1;  // index of the collectives' timeout word among the words (-1: none)
  };
  int32_t* rep_words_ = nullptr;  // [kRep][kRepWords] pinned
  int32_t* rep_toks_ = nullptr;   // [kRep][kRepToks] pinned: the frame's tokens
  void* rep_ev_[kRep] = {};
  bool rep_busy_[kRep] = {};
  int rep_next_ = 0;
  std::deque<Report> rq_;
  std::mutex rmu_;
  std::condition_variable rcv_;
  bool rstop_ = false;
  std::thread rth_;
  std::atomic<long> n_frames_{0}, n_launches_{0}, n_provides_{0}, n_eager_{0}, n_faults_{0},
      n_host_fail_{0};
};

}  // namespace p2p
