// Chat node daemon (`go/cmd/node/main.go`), env-configured like the reference:
// MYNAMEIS, HTTP_ADDR, DIRECTORY_URL, BOOTSTRAP_ADDRS; opt-in extras RELAY_ADDRS,
// KEY_TYPE, IDENTITY_FILE, INBOX_FILE, ENGINE_URL, REGISTER_INTERVAL, STRICT_SENDER.
// The LLM engine is attached when the node runs inside the Python process
// (python -m p2p_llm_chat_go_amd.net.node); this binary forwards to ENGINE_URL.
#include <pthread.h>
#include <signal.h>

#include <thread>

#include "net/chat.h"

using namespace p2p;

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
  return 0;
}
