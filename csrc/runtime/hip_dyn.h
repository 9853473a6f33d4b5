// The few HIP runtime entry points the native engine loop needs, resolved at run time
// from the HIP runtime ALREADY loaded into the process (the one PyTorch brought, which
// also owns the captured hipGraphExec handles the loop replays).  Resolving instead of
// linking keeps the chat daemons free of a HIP dependency: only a process that built an
// engine ever touches these.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace p2p {

struct HipApi {
  bool ok = false;
  std::string error;
  int (*graphLaunch)(void* exec, void* stream) = nullptr;
  int (*memcpyAsync)(void* dst, const void* src, size_t n, int kind, void* stream) = nullptr;
  int (*memsetAsync)(void* dst, int value, size_t n, void* stream) = nullptr;
  int (*memcpy2DAsync)(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                       size_t height, int kind, void* stream) = nullptr;
  int (*streamCreateWithFlags)(void** stream, unsigned flags) = nullptr;
  int (*streamDestroy)(void* stream) = nullptr;
  int (*streamSynchronize)(void* stream) = nullptr;
  int (*hostMalloc)(void** p, size_t n, unsigned flags) = nullptr;
  int (*hostFree)(void* p) = nullptr;
  int (*setDevice)(int dev) = nullptr;
  int (*eventCreateWithFlags)(void** ev, unsigned flags) = nullptr;
  int (*eventRecord)(void* ev, void* stream) = nullptr;
  int (*eventSynchronize)(void* ev) = nullptr;
  int (*eventQuery)(void* ev) = nullptr;
  int (*eventDestroy)(void* ev) = nullptr;
  const char* (*getErrorString)(int err) = nullptr;
};

enum : int { kH2D = 1, kD2H = 2 };  // hipMemcpyKind
enum : int { kHipNotReady = 600 };  // hipErrorNotReady

// Resolve once (thread-safe); .ok false with .error set if no HIP runtime is loadable.
const HipApi& hip_api();

// Throws std::runtime_error("<what>: <hip error string>") when rc != 0.
void hip_check(int rc, const char* what);

// Tests without a GPU: replace the resolved API with a host-only stand-in (copies are
// memcpy, streams and events are no-ops, pinned memory is malloc, and a "graph exec" is a
// host function pointer `int (*)(void)` that hipGraphLaunch calls).  Lets the CPU tier run
// the native engine loop against a simulated model.
void hip_api_use_host_fake();

}  // namespace p2p
