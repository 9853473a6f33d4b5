// Native request path across processes: the node process serves requests on engine loops
// that live in OTHER processes -- the leader process of every replica group of a
// multi-GPU node (ENGINE_GPUS / ENGINE_TP / ENGINE_EP > 1, engine/cluster.py) -- with no
// Python on either side.
//
//   node process                                   replica leader process
//   engine C ABI (engine_capi.cc)                  EngineLoop (engine_loop.cc)
//     RemoteLoops: a P2PLoopApi table  --unix-->     LoopServer: one thread per request
//     (route to the least-loaded live replica,       connection: submit, stream the
//      one connection per request)                   tokens as they decode, final result
//
// The client side is a loop_capi.h table (P2PLoopApi), so the C ABI's native generate /
// stream code serves a cluster exactly as it serves its own in-process loop.  The leader's
// loop drives its TP / EP followers itself (mirror.h), so one socket per replica is all the
// node needs.  Sockets are Linux abstract-namespace unix sockets ("@p2p-loop-...": nothing
// on the file system to clean up).
//
// Wire (both directions): u32 length (little endian) + payload, payload[0] = op.
//   client -> server  'S' submit: i32 n, i32 ids[n], i32 max_new, u8 stop_on_eos,
//                         f32 temperature, i32 top_k, f32 top_p, i64 seed
//                     'C' cancel (or just close the connection)
//   server -> client  'A' accepted: i64 id (>= 0), or -1 + u32 len + reason
//                     'T' tokens: u32 n + i32[n] (new tokens, in order)
//                     'R' result: u8 done, i32 prompt_eval_count, i64 prompt_eval_ns,
//                         eval_ns, total_ns, ttft_ns, u32 len + done_reason,
//                         u32 len + error, u32 n + i32 tokens[n]
#pragma once
#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime/loop_capi.h"

namespace p2p {

class EngineLoop;

class LoopServer {
 public:
  // serves `loop` on the abstract unix socket `name` (without the leading '@')
  LoopServer(EngineLoop* loop, const std::string& name);
  ~LoopServer();
  LoopServer(const LoopServer&) = delete;
  LoopServer& operator=(const LoopServer&) = delete;
  void start();  // throws if the socket cannot be bound
  void stop();   // closes the listener; request threads end at their next poll
  long served() const { return served_; }

 private:
  void accept_loop();
  void serve(int fd);
  EngineLoop* loop_;
  std::string name_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::atomic<int> active_{0};
  std::atomic<long> served_{0};
  std::thread th_;
};

// Client: a P2PLoopApi over the replicas' sockets.  `loop` pointers passed to the table's
// functions are RemoteLoops objects (remote_loops_create).
const P2PLoopApi* remote_loop_api();
void* remote_loops_create(const std::vector<std::string>& names);
void remote_loops_destroy(void* rl);
// per replica: requests routed to it so far (metrics)
std::vector<long> remote_loops_routed(void* rl);

}  // namespace p2p
