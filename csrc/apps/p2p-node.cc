// Chat node daemon (`go/cmd/node/main.go`), env-configured like the reference:
// MYNAMEIS, HTTP_ADDR, DIRECTORY_URL, BOOTSTRAP_ADDRS; opt-in extras RELAY_ADDRS,
// KEY_TYPE, IDENTITY_FILE, INBOX_FILE, ENGINE_URL, REGISTER_INTERVAL, STRICT_SENDER.
// The LLM engine is attached when the node runs inside the Python process
// (python -m p2p_llm_chat_go_amd.net.node); this binary forwards to ENGINE_URL.
#include <signal.h>

#include "net/chat.h"

using namespace p2p;

int main() {
  signal(SIGPIPE, SIG_IGN);
  Node node(NodeConfig::from_env());
  try {
    node.start();
  } catch (const std::exception& e) {
    logf("directory register failed:%s", e.what());  // log.Fatal in the reference
    return 1;
  }
  node.wait();
  return 0;
}
