// Self-test of the native engine step loop (csrc/runtime/engine_loop.cc) on the host: the
// HIP entry points are the host-only stand-in (hip_api_use_host_fake: copies are memcpy, a
// "graph exec" is a host function the loop launches) and the model is simulated -- every
// captured graph reads the loop's metadata from the same buffers a real graph would, and
// the next token is a fixed function of (token, position), so every reply is known.
// Concurrent submitters (with cancellations, streaming waits and a stall) drive the loop
// thread; the program exits 0 after checking every reply and the page accounting.  Built
// with the daemons, and with ASan+UBSan / TSan into bin/asan, bin/tsan
// (tests/test_sanitizers.py runs those: the loop's locking under a race detector).
#include <array>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <random>
#include <thread>
#include <utility>
#include <vector>

#include <sys/socket.h>
#include <unistd.h>

#include "runtime/engine_loop.h"
#include "runtime/hip_dyn.h"
#include "runtime/loop_remote.h"
#include "runtime/mirror.h"

using namespace p2p;

namespace {

constexpr int V = 1000, EOS = 999, PAGE = 64, PREFILL_PAGES = 4;

int nxt(int tok, int pos) { return (tok * 31 + pos * 7 + 3) % V; }

std::vector<int> expected(const std::vector<int>& prompt, int max_new, bool stop_on_eos) {
  std::vector<int> out;
  int tok = prompt.back(), pos = (int)prompt.size() - 1;
  while ((int)out.size() < max_new) {
    tok = nxt(tok, pos++);
    if (stop_on_eos && tok == EOS) break;
    out.push_back(tok);
  }
  return out;
}

// graph execs are plain host functions: a fixed table of trampolines into std::function slots
constexpr int kSlots = 256;
std::function<int()> g_slot[kSlots];
std::atomic<int> g_next{0};
std::atomic<int> g_bad{0};
// fault injection on a follower rank (run_group_faults): the next follower decode replay
// sets its graph's fault word; the next follower eager prefill raises
std::atomic<int> g_follower_fault{0}, g_follower_eager_fail{0};
// a collective timeout (run_coll_fault): the next decode replay sets the collective word
std::atomic<int> g_coll_trigger{0}, g_fcoll_trigger{0};
int32_t g_coll_word = 0, g_fcoll_word = 0;  // the leader's / a follower's collective word

template <int I>
int tramp() { return g_slot[I](); }
template <int... I>
constexpr std::array<int (*)(), sizeof...(I)> make_table(std::integer_sequence<int, I...>) {
  return {&tramp<I>...};
}
const auto g_table = make_table(std::make_integer_sequence<int, kSlots>{});

void* exec_of(std::function<int()> f) {
  const int i = g_next++;
  if (i >= kSlots) {
    std::fprintf(stderr, "selftest: out of graph slots\n");
    std::exit(3);
  }
  g_slot[i] = std::move(f);
  return reinterpret_cast<void*>(g_table[i]);
}

uint64_t mix(uint64_t h, uint64_t v) { return (h ^ v) * 0x100000001B3ull; }

struct DecodeGraph {
  std::vector<int32_t> meta, hist, step{0}, errw{0};
  std::vector<int64_t> keys{0};
  DecodeGraphDesc d;
  uint64_t trace = 1469598103934665603ull;  // FNV over (step, meta) at every replay
  long launches = 0;
  DecodeGraph(int B, int ctx, bool follower = false)
      : meta((size_t)B * (4 + ctx / PAGE)), hist((size_t)B * ctx) {
    if (follower) d.err = errw.data();
    d.B = B;
    d.max_pages = ctx / PAGE;
    d.ctx = ctx;
    d.greedy = true;
    d.meta = meta.data();
    d.hist = hist.data();
    d.max_steps = ctx;
    d.step = step.data();
    d.keys = keys.data();
    d.keys_bytes = sizeof(int64_t);
    auto one = [this, follower] {
      const int B = d.B, S = d.max_steps, s = step[0];
      launches++;
      if (follower && g_follower_fault.exchange(0)) errw[0] = 1;
      if (!follower && g_coll_trigger.exchange(0)) g_coll_word = 1;
      if (follower && g_fcoll_trigger.exchange(0)) g_fcoll_word = 1;
      trace = mix(trace, (uint64_t)s);
      for (int32_t v : meta) trace = mix(trace, (uint64_t)(uint32_t)v);
      if (s >= S) {
        g_bad++;
        return 1;
      }
      int32_t *ids = meta.data(), *pos = ids + B, *cx = pos + B;
      for (int b = 0; b < B; ++b) {
        const int t = nxt(ids[b], pos[b]);
        hist[(size_t)b * S + s] = t;
        ids[b] = t;
        pos[b] += 1;
        cx[b] = pos[b] + 1;
      }
      step[0] = s + 1;
      return 0;
    };
    d.exec = exec_of(one);
    d.k_steps = 4;  // a whole 4-step graph (the loop launches those first)
    d.exec_k = exec_of([one] {
      int rc = 0;
      for (int i = 0; i < 4; ++i) rc |= one();
      return rc;
    });
  }
};

struct PrefillGraph {
  std::vector<int32_t> meta, first;
  PrefillGraphDesc d;
  uint64_t trace = 1469598103934665603ull;
  long launches = 0;
  PrefillGraph(int R, int S) : first(S) {
    const int P = PREFILL_PAGES, qtile = 16;
    const int max_tiles = (R + qtile - 1) / qtile + S + 1 + R / (P * PAGE) + 1;
    size_t o = 0;
    auto take = [&](size_t n) { const size_t at = o; o += n; return at; };
    d.off_bt = take((size_t)(S + 1) * P);
    d.off_seq = take(R);
    d.off_pos = take(R);
    d.off_ids = take(R);
    d.off_slots = take(R);
    d.off_ctx = take(R);
    d.off_out = take(S);
    d.off_spos = take(S);
    d.off_tiles = take((size_t)4 * max_tiles);
    meta.assign(o, 0);
    d.rows = R;
    d.n_seq = S;
    d.max_pages = P;
    d.qtile = qtile;
    d.max_tiles = max_tiles;
    d.greedy = true;
    d.meta = meta.data();
    d.meta_len = meta.size();
    d.first = first.data();
    d.exec = exec_of([this] {
      const int R = d.rows, S = d.n_seq;
      launches++;
      for (int32_t v : meta) trace = mix(trace, (uint64_t)(uint32_t)v);
      const int32_t* seq = meta.data() + d.off_seq;
      const int32_t* pos = meta.data() + d.off_pos;
      const int32_t* ids = meta.data() + d.off_ids;
      const int32_t* cx = meta.data() + d.off_ctx;
      const int32_t* out = meta.data() + d.off_out;
      for (int i = 0; i < R; ++i)
        if (cx[i] != pos[i] + 1 || seq[i] < 0 || seq[i] > S) {
          g_bad++;
          return 1;
        }
      for (int s = 0; s < S; ++s) first[s] = nxt(ids[out[s]], pos[out[s]]);
      return 0;
    });
  }
};

int run(bool pipeline, bool riders_all) {
  LoopConfig c;
  c.num_pages = 512;
  c.max_batch = 8;
  c.max_prefill_tokens = 256;
  c.max_ctx = 2048;
  c.eos = {EOS};
  c.decode_chunk = 4;
  c.admit_wait_us = 200.0;
  c.pipeline = pipeline;
  c.pipeline_free_slots = true;
  c.riders_all = riders_all;
  c.row_buckets = {16, 32, 48, 64, 96, 128, 192, 256};
  c.prefill_max_pages = PREFILL_PAGES;
  c.prefill_graph_after = 1;
  EngineLoop loop(c);
  std::vector<std::unique_ptr<DecodeGraph>> dg;
  std::vector<std::unique_ptr<PrefillGraph>> pg;
  loop.set_provider([&](const std::string& kind, int a, int b, bool) {
    if (kind == "decode") {
      dg.emplace_back(new DecodeGraph(a, b));
      loop.add_decode_graph(dg.back()->d);
    } else {
      pg.emplace_back(new PrefillGraph(a, b));
      loop.add_prefill_graph(pg.back()->d);
    }
  });
  loop.set_eager_prefill([](const std::vector<std::vector<int>>& prompts,
                            const std::vector<std::vector<int>>&, const std::vector<int>&,
                            const std::vector<LoopSampling>&, int) {
    std::vector<int> f;
    for (const auto& p : prompts) f.push_back(nxt(p.back(), (int)p.size() - 1));
    return f;
  });
  loop.start();
  const int free0 = (int)loop.metrics()["free_kv_pages"];
  std::atomic<int> failures{0}, checked{0};
  auto peer = [&](int k) {
    std::mt19937 rng(1000 + k);
    for (int n = 0; n < 12; ++n) {
      const int L = std::vector<int>{1, 5, 17, 44, 63, 64, 65, 120, 200, 300}[rng() % 10];
      std::vector<int> prompt(L);
      for (int& t : prompt) t = (int)(rng() % (V - 1));
      const int max_new = 1 + (int)(rng() % 40);
      const bool eos = rng() % 2;
      const int mode = (int)(rng() % 6);  // 0: cancel, 1: stream, else wait
      const int64_t id = loop.submit(prompt, max_new, eos, LoopSampling());
      if (mode == 0) {
        loop.cancel(id);
        LoopResult r;
        loop.wait(id, 30.0, &r);
        loop.release(id);
        if (!r.done || !r.error.empty()) failures++;
        continue;
      }
      std::vector<int> got;
      if (mode == 1) {
        bool done = false;
        while (!done) {
          auto more = loop.wait_tokens(id, got.size(), 5.0, &done);
          got.insert(got.end(), more.begin(), more.end());
        }
      } else {
        LoopResult r;
        if (!loop.wait(id, 30.0, &r) || !r.error.empty()) failures++;
        got = r.tokens;
      }
      loop.release(id);
      if (got != expected(prompt, max_new, eos)) {
        std::fprintf(stderr, "selftest: reply mismatch (L=%d n=%d eos=%d mode=%d)\n", L,
                     max_new, (int)eos, mode);
        failures++;
      }
      checked++;
    }
  };
  std::vector<std::thread> ths;
  for (int k = 0; k < 6; ++k) ths.emplace_back(peer, k);
  std::thread staller([&] {  // fault injection while the peers run
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    loop.stall(0.05);
  });
  for (auto& t : ths) t.join();
  staller.join();
  int free1 = -1;
  for (int i = 0; i < 500; ++i) {
    auto m = loop.metrics();
    free1 = (int)m["free_kv_pages"];
    if (free1 == free0 && m["running"] == 0 && m["waiting"] == 0) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  loop.shutdown();
  if (free1 != free0) {
    std::fprintf(stderr, "selftest: KV pages leaked (%d -> %d)\n", free0, free1);
    failures++;
  }
  std::printf("pipeline=%d riders_all=%d checked=%d failures=%d bad_graph_calls=%d\n",
              (int)pipeline, (int)riders_all, checked.load(), failures.load(), g_bad.load());
  return failures.load() == 0 && g_bad.load() == 0 && checked.load() > 20 ? 0 : 1;
}

// A TP group of 1 leader + 2 followers (runtime/mirror.h): the leader's loop serves mixed
// traffic while two EngineMirror threads apply its frames to graphs of their own, over
// socketpairs.  Every follower graph must have been replayed exactly as often as the
// leader's, with the same metadata at every replay (trace), and each follower must have
// captured every shape and run every eager prefill the leader did.
int run_group() {
  constexpr int NF = 2;
  LoopConfig c;
  c.num_pages = 512;
  c.max_batch = 8;
  c.max_prefill_tokens = 256;
  c.max_ctx = 2048;
  c.eos = {EOS};
  c.decode_chunk = 8;
  c.admit_wait_us = 200.0;
  c.row_buckets = {16, 32, 48, 64, 96, 128, 192, 256};
  c.prefill_max_pages = PREFILL_PAGES;
  c.prefill_graph_after = 1;
  EngineLoop loop(c);
  int sv[NF][2];
  std::vector<int> fds;
  for (int f = 0; f < NF; ++f) {
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv[f]) != 0) return 1;
    fds.push_back(sv[f][0]);
  }
  loop.set_mirror(fds);
  using DMap = std::map<std::tuple<int, int>, std::unique_ptr<DecodeGraph>>;
  using PMap = std::map<std::tuple<int, int>, std::unique_ptr<PrefillGraph>>;
  DMap ld;
  PMap lp;
  std::atomic<int> leader_eager{0};
  loop.set_provider([&](const std::string& kind, int a, int b, bool greedy) {
    loop.mirror_provide(kind, a, b, greedy);  // as NativeEngineServer._provide does
    if (kind == "decode") {
      ld[{a, b}].reset(new DecodeGraph(a, b));
      loop.add_decode_graph(ld[{a, b}]->d);
    } else {
      lp[{a, b}].reset(new PrefillGraph(a, b));
      loop.add_prefill_graph(lp[{a, b}]->d);
    }
  });
  auto eager = [](const std::vector<std::vector<int>>& prompts, const std::vector<std::vector<int>>&,
                  const std::vector<int>&, const std::vector<LoopSampling>&, int) {
    std::vector<int> f;
    for (const auto& p : prompts) f.push_back(nxt(p.back(), (int)p.size() - 1));
    return f;
  };
  loop.set_eager_prefill([&](const std::vector<std::vector<int>>& p, const std::vector<std::vector<int>>& pg,
                             const std::vector<int>& st, const std::vector<LoopSampling>& sm, int) {
    leader_eager++;
    return eager(p, pg, st, sm, 0);
  });
  struct Follower {
    std::unique_ptr<EngineMirror> m;
    DMap d;
    PMap p;
    std::atomic<int> eager{0};
    std::string result = "?";
    std::thread th;
  };
  Follower fol[NF];
  for (int f = 0; f < NF; ++f) {
    Follower& F = fol[f];
    F.m.reset(new EngineMirror(sv[f][1], 0));
    EngineMirror* M = F.m.get();
    F.m->set_provider([&F, M](const std::string& kind, int a, int b, bool) {
      if (kind == "decode") {
        F.d[{a, b}].reset(new DecodeGraph(a, b));
        M->add_decode_graph(F.d[{a, b}]->d);
      } else {
        F.p[{a, b}].reset(new PrefillGraph(a, b));
        M->add_prefill_graph(F.p[{a, b}]->d);
      }
    });
    F.m->set_eager_prefill([&F, eager](const std::vector<std::vector<int>>& p,
                                       const std::vector<std::vector<int>>& pg,
                                       const std::vector<int>& st, const std::vector<LoopSampling>& sm, int) {
      F.eager++;
      return eager(p, pg, st, sm, 0);
    });
    F.th = std::thread([&F] { F.result = F.m->run(); });
  }
  loop.start();
  std::atomic<int> failures{0}, checked{0};
  auto peer = [&](int k) {
    std::mt19937 rng(77 + k);
    for (int n = 0; n < 10; ++n) {
      const int L = std::vector<int>{3, 17, 44, 64, 120, 300}[rng() % 6];
      std::vector<int> prompt(L);
      for (int& t : prompt) t = (int)(rng() % (V - 1));
      const int max_new = 1 + (int)(rng() % 40);
      const int64_t id = loop.submit(prompt, max_new, false, LoopSampling());
      LoopResult r;
      if (!loop.wait(id, 30.0, &r) || !r.error.empty()) failures++;
      loop.release(id);
      if (r.tokens != expected(prompt, max_new, false)) failures++;
      checked++;
    }
  };
  std::vector<std::thread> ths;
  for (int k = 0; k < 8; ++k) ths.emplace_back(peer, k);
  for (auto& t : ths) t.join();
  auto lm = loop.metrics();
  loop.shutdown();  // sends the stop frame
  for (int f = 0; f < NF; ++f) {
    fol[f].th.join();
    fol[f].m->shutdown();
    close(sv[f][0]);
    close(sv[f][1]);
    if (!fol[f].result.empty()) {
      std::fprintf(stderr, "selftest: follower %d ended with '%s'\n", f, fol[f].result.c_str());
      failures++;
    }
    if (fol[f].d.size() != ld.size() || fol[f].p.size() != lp.size() ||
        fol[f].eager.load() != leader_eager.load()) {
      std::fprintf(stderr, "selftest: follower %d captured %zu/%zu graphs, %d/%d eager\n", f,
                   fol[f].d.size() + fol[f].p.size(), ld.size() + lp.size(), fol[f].eager.load(),
                   leader_eager.load());
      failures++;
    }
    for (auto& kv : ld) {
      auto it = fol[f].d.find(kv.first);
      if (it == fol[f].d.end() || it->second->trace != kv.second->trace ||
          it->second->launches != kv.second->launches) {
        std::fprintf(stderr, "selftest: follower %d decode graph replays differ\n", f);
        failures++;
      }
    }
    for (auto& kv : lp) {
      auto it = fol[f].p.find(kv.first);
      if (it == fol[f].p.end() || it->second->trace != kv.second->trace ||
          it->second->launches != kv.second->launches) {
        std::fprintf(stderr, "selftest: follower %d prefill graph replays differ\n", f);
        failures++;
      }
    }
  }
  long k_launch = (long)lm["k_graph_launches"];
  std::printf("group: checked=%d failures=%d frames=%ld k_graph_launches=%ld eager=%d graphs=%zu\n",
              checked.load(), failures.load(), (long)lm["mirror_frames"], k_launch,
              leader_eager.load(), ld.size() + lp.size());
  return failures.load() == 0 && g_bad.load() == 0 && checked.load() == 80 && k_launch > 0 &&
                 leader_eager.load() > 0
             ? 0
             : 1;
}

// An EP all-to-all group (LoopConfig::dp_world = 3: leader + 2 followers, DP attention): each
// sequence lives on one rank, every rank runs its own share through the same shapes (its own
// metadata in its own frame), the followers send their tokens back with their frames' status,
// and every reply must be exactly right -- which it is only if every share's tokens reached
// the leader's scheduler in the right rows.  The eager prefill of every rank gets the same
// padded row count, the largest share's.
int run_group_dp() {
  constexpr int NF = 2;
  LoopConfig c;
  c.num_pages = 512;
  c.max_batch = 8;
  c.max_prefill_tokens = 256;
  c.max_ctx = 2048;
  c.eos = {EOS};
  c.decode_chunk = 8;
  c.admit_wait_us = 200.0;
  c.mixed = false;
  c.dp_world = NF + 1;
  c.row_buckets = {16, 32, 48, 64, 96, 128, 192, 256};
  c.prefill_max_pages = PREFILL_PAGES;
  EngineLoop loop(c);
  int sv[NF][2];
  std::vector<int> fds;
  for (int f = 0; f < NF; ++f) {
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv[f]) != 0) return 1;
    fds.push_back(sv[f][0]);
  }
  loop.set_mirror(fds);
  using DMap = std::map<std::tuple<int, int>, std::unique_ptr<DecodeGraph>>;
  DMap ld;
  std::atomic<int> leader_eager{0}, bad_pad{0};
  loop.set_provider([&](const std::string& kind, int a, int b, bool greedy) {
    loop.mirror_provide(kind, a, b, greedy);
    if (kind == "decode") {
      ld[{a, b}].reset(new DecodeGraph(a, b));
      loop.add_decode_graph(ld[{a, b}]->d);
    } else {
      bad_pad++;  // dp groups prefill eagerly: no prefill graph may be asked for
    }
  });
  auto eager = [&bad_pad](const std::vector<std::vector<int>>& prompts, const std::vector<std::vector<int>>&,
                          const std::vector<int>&, const std::vector<LoopSampling>&, int pad) {
    std::vector<int> f;
    int rows = 0;
    for (const auto& p : prompts) {
      f.push_back(nxt(p.back(), (int)p.size() - 1));
      rows += (int)p.size();
    }
    if (pad < rows || pad < 1) bad_pad++;
    return f;
  };
  loop.set_eager_prefill([&](const std::vector<std::vector<int>>& p, const std::vector<std::vector<int>>& pg,
                             const std::vector<int>& st, const std::vector<LoopSampling>& sm, int pad) {
    leader_eager++;
    return eager(p, pg, st, sm, pad);
  });
  struct Follower {
    std::unique_ptr<EngineMirror> m;
    DMap d;
    std::atomic<int> eager{0};
    std::string result = "?";
    std::thread th;
  };
  Follower fol[NF];
  for (int f = 0; f < NF; ++f) {
    Follower& F = fol[f];
    F.m.reset(new EngineMirror(sv[f][1], 0));
    EngineMirror* M = F.m.get();
    F.m->set_provider([&F, M](const std::string& kind, int a, int b, bool) {
      if (kind == "decode") {
        F.d[{a, b}].reset(new DecodeGraph(a, b));
        M->add_decode_graph(F.d[{a, b}]->d);
      }
    });
    F.m->set_eager_prefill([&F, eager](const std::vector<std::vector<int>>& p,
                                       const std::vector<std::vector<int>>& pg,
                                       const std::vector<int>& st, const std::vector<LoopSampling>& sm, int pad) {
      F.eager++;
      return eager(p, pg, st, sm, pad);
    });
    F.th = std::thread([&F] { F.result = F.m->run(); });
  }
  loop.start();
  std::atomic<int> failures{0}, checked{0};
  auto peer = [&](int k) {
    std::mt19937 rng(301 + k);
    for (int n = 0; n < 8; ++n) {
      const int L = std::vector<int>{3, 17, 44, 64, 120, 200}[rng() % 6];
      std::vector<int> prompt(L);
      for (int& t : prompt) t = (int)(rng() % (V - 1));
      const int max_new = 1 + (int)(rng() % 40);
      const int64_t id = loop.submit(prompt, max_new, false, LoopSampling());
      LoopResult r;
      if (!loop.wait(id, 30.0, &r) || !r.error.empty()) {
        std::fprintf(stderr, "selftest dp: request failed: %s\n", r.error.c_str());
        failures++;
      }
      loop.release(id);
      if (r.tokens != expected(prompt, max_new, false)) {
        std::fprintf(stderr, "selftest dp: reply mismatch (L=%d n=%d)\n", L, max_new);
        failures++;
      }
      checked++;
    }
  };
  std::vector<std::thread> ths;
  for (int k = 0; k < 8; ++k) ths.emplace_back(peer, k);
  for (auto& t : ths) t.join();
  auto lm = loop.metrics();
  loop.shutdown();
  long fol_launches = 0;
  for (int f = 0; f < NF; ++f) {
    fol[f].th.join();
    fol[f].m->shutdown();
    close(sv[f][0]);
    close(sv[f][1]);
    if (!fol[f].result.empty()) {
      std::fprintf(stderr, "selftest dp: follower %d ended with '%s'\n", f, fol[f].result.c_str());
      failures++;
    }
    if (fol[f].eager.load() != leader_eager.load()) failures++;
    for (auto& kv : fol[f].d) fol_launches += kv.second->launches;
  }
  std::printf("group dp: checked=%d failures=%d eager=%d follower_launches=%ld bad=%d frames=%ld\n",
              checked.load(), failures.load(), leader_eager.load(), fol_launches, bad_pad.load(),
              (long)lm["mirror_frames"]);
  return failures.load() == 0 && bad_pad.load() == 0 && g_bad.load() == 0 && checked.load() == 64 &&
                 fol_launches > 0
             ? 0
             : 1;
}

// Faults on a follower rank: a follower whose graph fault word is set, or whose
// eager-prefill callback raises, answers that frame with its status bits; the leader must
// fail exactly that step (the request gets the reason), clear every rank's words, and go
// on serving -- the follower stays alive.
int run_group_faults() {
  LoopConfig c;
  c.num_pages = 256;
  c.max_batch = 4;
  c.max_prefill_tokens = 256;
  c.max_ctx = 2048;
  c.eos = {EOS};
  c.decode_chunk = 4;
  c.row_buckets = {16, 32, 48, 64};
  c.prefill_max_pages = PREFILL_PAGES;
  c.prefill_graph_after = 1;
  EngineLoop loop(c);
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
  loop.set_mirror({sv[0]});
  std::map<std::tuple<int, int>, std::unique_ptr<DecodeGraph>> ld, fd_;
  std::map<std::tuple<int, int>, std::unique_ptr<PrefillGraph>> lp, fp;
  loop.set_provider([&](const std::string& kind, int a, int b, bool greedy) {
    loop.mirror_provide(kind, a, b, greedy);
    if (kind == "decode") {
      ld[{a, b}].reset(new DecodeGraph(a, b));
      loop.add_decode_graph(ld[{a, b}]->d);
    } else {
      lp[{a, b}].reset(new PrefillGraph(a, b));
      loop.add_prefill_graph(lp[{a, b}]->d);
    }
  });
  auto eager = [](const std::vector<std::vector<int>>& prompts, const std::vector<std::vector<int>>&,
                  const std::vector<int>&, const std::vector<LoopSampling>&, int) {
    std::vector<int> f;
    for (const auto& p : prompts) f.push_back(nxt(p.back(), (int)p.size() - 1));
    return f;
  };
  loop.set_eager_prefill(eager);
  EngineMirror m(sv[1], 0);
  m.set_provider([&](const std::string& kind, int a, int b, bool) {
    if (kind == "decode") {
      fd_[{a, b}].reset(new DecodeGraph(a, b, true));
      m.add_decode_graph(fd_[{a, b}]->d);
    } else {
      fp[{a, b}].reset(new PrefillGraph(a, b));
      m.add_prefill_graph(fp[{a, b}]->d);
    }
  });
  m.set_eager_prefill([&](const std::vector<std::vector<int>>& p, const std::vector<std::vector<int>>& pg,
                          const std::vector<int>& st, const std::vector<LoopSampling>& sm, int) {
    if (g_follower_eager_fail.exchange(0)) throw std::runtime_error("injected eager failure");
    return eager(p, pg, st, sm, 0);
  });
  m.set_coll_fault(reinterpret_cast<uintptr_t>(&g_fcoll_word));
  std::string fres = "?";
  std::thread fth([&] { fres = m.run(); });
  loop.start();
  int failures = 0;
  auto ask = [&](int L, std::string* err) {
    std::vector<int> prompt(L);
    for (int i = 0; i < L; ++i) prompt[i] = (i * 13 + 5) % (V - 1);
    const int64_t id = loop.submit(prompt, 12, false, LoopSampling());
    LoopResult r;
    loop.wait(id, 30.0, &r);
    loop.release(id);
    *err = r.error;
    return r.error.empty() && r.tokens == expected(prompt, 12, false);
  };
  std::string e;
  if (!ask(20, &e)) failures++, std::fprintf(stderr, "faults: clean request failed: %s\n", e.c_str());
  g_follower_fault = 1;
  if (ask(20, &e) || e.find("follower") == std::string::npos)
    failures++, std::fprintf(stderr, "faults: follower fault not reported (err '%s')\n", e.c_str());
  if (!ask(20, &e)) failures++, std::fprintf(stderr, "faults: request after the fault failed: %s\n", e.c_str());
  g_follower_eager_fail = 1;
  if (ask(300, &e) || e.find("failed on a follower") == std::string::npos)
    failures++, std::fprintf(stderr, "faults: follower eager failure not reported (err '%s')\n", e.c_str());
  if (!ask(300, &e)) failures++, std::fprintf(stderr, "faults: eager request after the failure failed: %s\n", e.c_str());
  for (auto& kv : fd_)
    if (kv.second->errw[0] != 0) failures++, std::fprintf(stderr, "faults: follower word not cleared\n");
  // last: a collective timeout on the follower (status bit 4) fails the step and kills the replica
  g_fcoll_trigger = 1;
  if (ask(20, &e) || e.find("collective timeout") == std::string::npos)
    failures++, std::fprintf(stderr, "faults: follower collective timeout not reported (err '%s')\n", e.c_str());
  if (loop.dead().find("collective timeout") == std::string::npos)
    failures++, std::fprintf(stderr, "faults: replica not dead after a follower collective timeout\n");
  g_fcoll_word = 0;
  auto lm = loop.metrics();
  auto mm = m.metrics();
  loop.shutdown();
  fth.join();
  m.shutdown();
  close(sv[0]);
  close(sv[1]);
  if (!fres.empty()) failures++, std::fprintf(stderr, "faults: follower ended with '%s'\n", fres.c_str());
  std::printf("group faults: failures=%d follower_faults=%ld fault_reports=%ld host_failures=%ld dead='%s'\n",
              failures, (long)lm["mirror_follower_faults"], (long)mm["mirror_fault_reports"],
              (long)mm["mirror_host_failures"], loop.dead().c_str());
  return failures == 0 && lm["mirror_follower_faults"] >= 2 && mm["mirror_host_failures"] == 1 ? 0 : 1;
}

// The cross-process request path (runtime/loop_remote.h) in one process: two loops serve
// on abstract unix sockets, a RemoteLoops table routes concurrent submitters (blocking
// waits, streaming waits, cancellations) to them; every reply must be exact, both replicas
// must be used, and a replica whose socket is gone must be skipped, not fail requests.
int run_remote() {
  LoopConfig c;
  c.num_pages = 256;
  c.max_batch = 4;
  c.max_prefill_tokens = 256;
  c.max_ctx = 2048;
  c.eos = {EOS};
  c.decode_chunk = 4;
  c.row_buckets = {16, 32, 48, 64, 96, 128, 192, 256};
  c.prefill_max_pages = PREFILL_PAGES;
  c.prefill_graph_after = 1;
  std::vector<std::unique_ptr<EngineLoop>> loops;
  std::vector<std::unique_ptr<DecodeGraph>> dg;
  std::vector<std::unique_ptr<PrefillGraph>> pg;
  std::mutex gm;
  std::vector<std::string> names;
  for (int r = 0; r < 2; ++r) {
    loops.emplace_back(new EngineLoop(c));
    EngineLoop* L = loops.back().get();
    L->set_provider([&gm, &dg, &pg, L](const std::string& kind, int a, int b, bool) {
      std::lock_guard<std::mutex> lk(gm);
      if (kind == "decode") {
        dg.emplace_back(new DecodeGraph(a, b));
        L->add_decode_graph(dg.back()->d);
      } else {
        pg.emplace_back(new PrefillGraph(a, b));
        L->add_prefill_graph(pg.back()->d);
      }
    });
    L->set_eager_prefill([](const std::vector<std::vector<int>>& prompts, const std::vector<std::vector<int>>&,
                            const std::vector<int>&, const std::vector<LoopSampling>&, int) {
      std::vector<int> f;
      for (const auto& p : prompts) f.push_back(nxt(p.back(), (int)p.size() - 1));
      return f;
    });
    names.push_back("p2p-selftest-" + std::to_string(getpid()) + "-" + std::to_string(r));
    L->serve(names.back());
    L->start();
  }
  names.push_back("p2p-selftest-nobody-" + std::to_string(getpid()));  // no server there
  const P2PLoopApi* api = remote_loop_api();
  void* rl = remote_loops_create(names);
  std::atomic<int> failures{0}, checked{0};
  auto peer = [&](int k) {
    std::mt19937 rng(300 + k);
    for (int n = 0; n < 8; ++n) {
      const int Lp = std::vector<int>{3, 17, 44, 64, 120, 300}[rng() % 6];
      std::vector<int32_t> prompt(Lp);
      for (auto& t : prompt) t = (int32_t)(rng() % (V - 1));
      const int max_new = 1 + (int)(rng() % 30);
      char err[256] = {0};
      const int64_t h = api->submit(rl, prompt.data(), Lp, max_new, 0, 0.f, 40, 0.9f, 0, err, sizeof err);
      if (h < 0) {
        std::fprintf(stderr, "remote: submit refused: %s\n", err);
        failures++;
        continue;
      }
      const std::vector<int> want = expected(std::vector<int>(prompt.begin(), prompt.end()), max_new, false);
      if (n % 3 == 2) {  // cancelled right away: released without waiting
        api->cancel(rl, h);
        api->release(rl, h);
        continue;
      }
      std::vector<int> streamed;
      if (n % 2) {  // streaming waits
        int done = 0;
        while (!done) {
          int32_t* t = nullptr;
          int m = 0;
          api->wait_tokens(rl, h, streamed.size(), 0.05, &t, &m, &done);
          streamed.insert(streamed.end(), t, t + m);
          api->free_mem(t);
        }
      }
      P2PLoopResult r;
      api->wait(rl, h, 30.0, &r);
      std::vector<int> got(r.tokens, r.tokens + r.n_tokens);
      if (r.error || !r.done || got != want || (n % 2 && streamed != want)) {
        std::fprintf(stderr, "remote: reply mismatch (err %s)\n", r.error ? r.error : "-");
        failures++;
      }
      api->free_mem(r.tokens);
      api->free_mem(r.error);
      api->release(rl, h);
      checked++;
    }
  };
  std::vector<std::thread> ths;
  for (int k = 0; k < 6; ++k) ths.emplace_back(peer, k);
  for (auto& t : ths) t.join();
  const std::vector<long> routed = remote_loops_routed(rl);
  char dead[256];
  const int dl = api->dead(rl, dead, sizeof dead);
  for (auto& L : loops) L->shutdown();
  // every loop gone: submissions now fail with a reason instead of hanging
  std::vector<int32_t> p{1, 2, 3};
  char err[256] = {0};
  const int64_t h = api->submit(rl, p.data(), 3, 4, 0, 0.f, 40, 0.9f, 0, err, sizeof err);
  remote_loops_destroy(rl);
  std::printf("remote: checked=%d failures=%d routed=%ld/%ld/%ld dead_len=%d after_shutdown=%lld '%s'\n",
              checked.load(), failures.load(), routed[0], routed[1], routed[2], dl, (long long)h, err);
  return failures.load() == 0 && checked.load() >= 30 && routed[0] > 0 && routed[1] > 0 &&
                 routed[2] == 0 && dl == 0 && h < 0
             ? 0
             : 1;
}

}  // namespace

// A collective timeout (the IPC kernels' error word, EngineLoop::set_coll_fault) is not a
// transient fault: the request in flight fails with the reason and the replica is dead.
int run_coll_fault() {
  LoopConfig c;
  c.num_pages = 256;
  c.max_batch = 4;
  c.max_prefill_tokens = 256;
  c.max_ctx = 2048;
  c.eos = {EOS};
  c.decode_chunk = 4;
  c.row_buckets = {16, 32, 48, 64, 96, 128, 192, 256};
  c.prefill_max_pages = PREFILL_PAGES;
  c.prefill_graph_after = 1;
  EngineLoop loop(c);
  std::vector<std::unique_ptr<DecodeGraph>> dg;
  std::vector<std::unique_ptr<PrefillGraph>> pg;
  loop.set_provider([&](const std::string& kind, int a, int b, bool) {
    if (kind == "decode") {
      dg.emplace_back(new DecodeGraph(a, b));
      loop.add_decode_graph(dg.back()->d);
    } else {
      pg.emplace_back(new PrefillGraph(a, b));
      loop.add_prefill_graph(pg.back()->d);
    }
  });
  loop.set_coll_fault(reinterpret_cast<uintptr_t>(&g_coll_word));
  loop.start();
  int failures = 0;
  LoopResult r;
  int64_t id = loop.submit({1, 2, 3, 4, 5}, 12, false, LoopSampling());
  if (!loop.wait(id, 30.0, &r) || !r.error.empty()) failures++;  // clean
  loop.release(id);
  g_coll_trigger = 1;
  id = loop.submit({6, 7, 8}, 12, false, LoopSampling());
  loop.wait(id, 30.0, &r);
  loop.release(id);
  if (r.error.find("collective timeout") == std::string::npos) {
    failures++;
    std::fprintf(stderr, "coll fault: request error '%s'\n", r.error.c_str());
  }
  const std::string dead = loop.dead();
  if (dead.find("collective timeout") == std::string::npos) {
    failures++;
    std::fprintf(stderr, "coll fault: replica not dead ('%s')\n", dead.c_str());
  }
  loop.shutdown();
  g_coll_word = 0;
  std::printf("coll fault: failures=%d dead='%s'\n", failures, dead.c_str());
  return failures == 0 ? 0 : 1;
}

int main() {
  hip_api_use_host_fake();
  int rc = 0;
  rc |= run(true, false);
  rc |= run(false, true);
  rc |= run(true, true);
  rc |= run_group();
  rc |= run_group_faults();
  rc |= run_group_dp();
  rc |= run_coll_fault();
  rc |= run_remote();
  if (rc == 0) std::printf("LOOP_SELFTEST_OK\n");
  return rc;
}
