// Chat node daemon (`go/cmd/node/main.go`), env-configured like the reference:
// MYNAMEIS, HTTP_ADDR, DIRECTORY_URL, BOOTSTRAP_ADDRS; opt-in extras RELAY_ADDRS,
// KEY_TYPE, IDENTITY_FILE, INBOX_FILE, ENGINE_URL, REGISTER_INTERVAL, STRICT_SENDER,
// SECURITY, NAT_PMP, UPNP, DIAL_PREFER.
// The LLM engine: ENGINE=inproc loads the engine C ABI (libp2p_engine.so,
// csrc/engine/engine_capi.h) into this process -- the node links the engine
// instead of calling Ollama over HTTP; otherwise /api/generate forwards to
// ENGINE_URL (or the node runs inside `python -m p2p_llm_chat_go_amd.net.node`).
#include <dlfcn.h>
#include <limits.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <thread>

#include "engine/engine_capi.h"
#include "net/chat.h"

using namespace p2p;

namespace {

struct EngineApi {
  void* h = nullptr;
  p2p_engine* eng = nullptr;
  decltype(&p2p_engine_create) create = nullptr;
  decltype(&p2p_engine_generate) generate = nullptr;
  decltype(&p2p_engine_generate_stream) generate_stream = nullptr;
  decltype(&p2p_engine_free) free_str = nullptr;
  decltype(&p2p_engine_error) error = nullptr;
  decltype(&p2p_engine_destroy) destroy = nullptr;
};

std::string default_engine_lib() {
  char buf[PATH_MAX];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "libp2p_engine.so";
  std::string exe(buf, (size_t)n);
  std::string dir = exe.substr(0, exe.rfind('/'));  // bin/ (or bin/asan/)
  for (std::string d = dir; !d.empty(); d = d.substr(0, d.rfind('/'))) {
    const std::string cand = d + "/p2p_llm_chat_go_amd/_lib/libp2p_engine.so";
    if (access(cand.c_str(), R_OK) == 0) return cand;
    if (d.find('/') == std::string::npos) break;
  }
  return "libp2p_engine.so";
}

bool load_engine(EngineApi* a) {
  const char* p = getenv("P2P_ENGINE_LIB");
  const std::string path = (p && *p) ? p : default_engine_lib();
  a->h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!a->h) {
    logf("engine: cannot load %s: %s", path.c_str(), dlerror());
    return false;
  }
#define SYM(f, n) a->f = (decltype(a->f))dlsym(a->h, n)
  SYM(create, "p2p_engine_create");
  SYM(generate, "p2p_engine_generate");
  SYM(generate_stream, "p2p_engine_generate_stream");
  SYM(free_str, "p2p_engine_free");
  SYM(error, "p2p_engine_error");
  SYM(destroy, "p2p_engine_destroy");
#undef SYM
  if (!a->create || !a->generate || !a->generate_stream || !a->free_str || !a->destroy) {
    logf("engine: %s lacks the engine C ABI", path.c_str());
    return false;
  }
  a->eng = a->create(getenv("ENGINE_MODEL"), getenv("ENGINE_DEVICE"));
  if (!a->eng) {
    logf("engine: create failed: %s", a->error ? a->error() : "?");
    return false;
  }
  logf("engine: in-process (%s)", path.c_str());
  return true;
}

void install_engine(Node& node, EngineApi* a) {
  node.set_generate_hook([a](const Json& req) -> Json {
    char* out = a->generate(a->eng, req.dump().c_str());
    if (!out) throw std::runtime_error(std::string("engine: ") + (a->error ? a->error() : "?"));
    Json j = Json::parse(out);
    a->free_str(out);
    return j;
  });
  node.set_generate_stream_hook(
      [a](const Json& req, const std::function<bool(const Json&)>& emit) -> Json {
        auto cb = [](const char* chunk, void* ctx) -> int {
          auto* e = (const std::function<bool(const Json&)>*)ctx;
          try {
            return (*e)(Json::parse(chunk)) ? 1 : 0;
          } catch (...) {
            return 0;
          }
        };
        char* out = a->generate_stream(a->eng, req.dump().c_str(), cb, (void*)&emit);
        if (!out) throw std::runtime_error(std::string("engine: ") + (a->error ? a->error() : "?"));
        Json j = Json::parse(out);
        a->free_str(out);
        return j;
      });
}

}  // namespace

int main() {
  signal(SIGPIPE, SIG_IGN);
  // SIGTERM / SIGINT are taken by a waiter thread (blocked here, before any thread
  // exists, so every thread inherits the mask) for an orderly stop: NAT mappings
  // deleted, sessions closed, HTTP drained.
  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGTERM);
  sigaddset(&set, SIGINT);
  pthread_sigmask(SIG_BLOCK, &set, nullptr);
  Node node(NodeConfig::from_env());
  EngineApi eng;
  const char* mode = getenv("ENGINE");
  if (mode && std::string(mode) == "inproc") {
    if (!load_engine(&eng)) return 1;
    install_engine(node, &eng);
  }
  try {
    node.start();
  } catch (const std::exception& e) {
    logf("directory register failed:%s", e.what());  // log.Fatal in the reference
    return 1;
  }
  std::thread([&node, set] {
    int sig = 0;
    sigwait(&set, &sig);
    node.stop();
  }).detach();
  node.wait();
  node.stop();  // blocks until a signal-driven stop() in flight has finished
  if (eng.eng) eng.destroy(eng.eng);
  return 0;
}
