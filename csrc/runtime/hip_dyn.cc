#include "runtime/hip_dyn.h"

#include <dlfcn.h>

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

}  // namespace

const HipApi& hip_api() {
  static std::once_flag once;
  static HipApi api;
  std::call_once(once, [] { api = load(); });
  return api;
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
