#include "runtime/hip_dyn.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace p2p {

namespace {

template <class F>
bool sym(void* h, const char* name, F* out, std::string* err) {
  void* p = dlsym(h, name);
  if (!p) {
    *err = std::string("HIP runtime lacks ") + name;
    return false;
  }
  *out = reinterpret_cast<F>(p);
  return true;
}

HipApi load() {
  HipApi a;
  // the runtime PyTorch already loaded (same soname), else whatever the loader finds
  void* h = nullptr;
  for (const char* n : {"libamdhip64.so.7", "libamdhip64.so.6", "libamdhip64.so"}) {
    h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    if (h) break;
  }
  if (!h) h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    a.error = std::string("cannot load the HIP runtime: ") + dlerror();
    return a;
  }
  std::string& e = a.error;
  a.ok = sym(h, "hipGraphLaunch", &a.graphLaunch, &e) &&
         sym(h, "hipMemcpyAsync", &a.memcpyAsync, &e) &&
         sym(h, "hipMemsetAsync", &a.memsetAsync, &e) &&
         sym(h, "hipMemcpy2DAsync", &a.memcpy2DAsync, &e) &&
         sym(h, "hipStreamCreateWithFlags", &a.streamCreateWithFlags, &e) &&
         sym(h, "hipStreamDestroy", &a.streamDestroy, &e) &&
         sym(h, "hipStreamSynchronize", &a.streamSynchronize, &e) &&
         sym(h, "hipHostMalloc", &a.hostMalloc, &e) && sym(h, "hipHostFree", &a.hostFree, &e) &&
         sym(h, "hipSetDevice", &a.setDevice, &e) &&
         sym(h, "hipEventCreateWithFlags", &a.eventCreateWithFlags, &e) &&
         sym(h, "hipEventRecord", &a.eventRecord, &e) &&
         sym(h, "hipEventSynchronize", &a.eventSynchronize, &e) &&
         sym(h, "hipEventQuery", &a.eventQuery, &e) &&
         sym(h, "hipEventDestroy", &a.eventDestroy, &e) &&
         sym(h, "hipGetErrorString", &a.getErrorString, &e);
  return a;
}

HipApi& api_storage() {
  static HipApi api;
  return api;
}

std::once_flag g_once;

// ---- host-only stand-in (hip_api_use_host_fake) ----
int f_graph_launch(void* exec, void*) { return reinterpret_cast<int (*)()>(exec)(); }
int f_memcpy(void* d, const void* s, size_t n, int, void*) {
  std::memcpy(d, s, n);
  return 0;
}
int f_memset(void* d, int v, size_t n, void*) {
  std::memset(d, v, n);
  return 0;
}
int f_memcpy2d(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, int, void*) {
  for (size_t r = 0; r < h; ++r)
    std::memcpy(static_cast<char*>(d) + r * dp, static_cast<const char*>(s) + r * sp, w);
  return 0;
}
int f_stream_create(void** s, unsigned) {
  *s = reinterpret_cast<void*>(1);
  return 0;
}
int f_ok1(void*) { return 0; }
int f_host_malloc(void** p, size_t n, unsigned) {
  *p = std::malloc(n);
  return *p ? 0 : 2;
}
int f_host_free(void* p) {
  std::free(p);
  return 0;
}
int f_set_device(int) { return 0; }
int f_event_create(void** e, unsigned) {
  *e = reinterpret_cast<void*>(1);
  return 0;
}
int f_event_record(void*, void*) { return 0; }
const char* f_err(int) { return "host fake HIP error"; }

}  // namespace

const HipApi& hip_api() {
  std::call_once(g_once, [] { api_storage() = load(); });
  return api_storage();
}

void hip_api_use_host_fake() {
  std::call_once(g_once, [] {});
  HipApi& a = api_storage();
  a = HipApi();
  a.ok = true;
  a.graphLaunch = f_graph_launch;
  a.memcpyAsync = f_memcpy;
  a.memsetAsync = f_memset;
  a.memcpy2DAsync = f_memcpy2d;
  a.streamCreateWithFlags = f_stream_create;
  a.streamDestroy = f_ok1;
  a.streamSynchronize = f_ok1;
  a.hostMalloc = f_host_malloc;
  a.hostFree = f_host_free;
  a.setDevice = f_set_device;
  a.eventCreateWithFlags = f_event_create;
  a.eventRecord = f_event_record;
  a.eventSynchronize = f_ok1;
  a.eventQuery = f_ok1;
  a.eventDestroy = f_ok1;
  a.getErrorString = f_err;
}

void hip_check(int rc, const char* what) {
  if (rc == 0) return;
  const HipApi& a = hip_api();
  std::string msg = what;
  msg += ": ";
  msg += (a.getErrorString ? a.getErrorString(rc) : "hip error") + std::string(" (") +
         std::to_string(rc) + ")";
  throw std::runtime_error(msg);
}

}  // namespace p2p
