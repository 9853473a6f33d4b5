// Circuit-relay-v2 hop daemon (`go/cmd/relay/main.go`): prints its multiaddrs
// and serves reservations / circuits forever.
// Env: RELAY_LISTEN (default /ip4/0.0.0.0/tcp/0), KEY_TYPE (rsa|ed25519, default ed25519),
//      IDENTITY_FILE (opt-in persistent identity).
#include <signal.h>
#include <stdio.h>
#include <unistd.h>

#include <fstream>
#include <iterator>
#include <thread>

#include "net/relay.h"

using namespace p2p;

int main() {
  signal(SIGPIPE, SIG_IGN);
  std::string kt = env_or("KEY_TYPE", "ed25519");
  std::string idf = env_or("IDENTITY_FILE", "");
  PrivateKey key;
  std::ifstream f(idf, std::ios::binary);
  if (!idf.empty() && f) {
    Bytes b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    key = PrivateKey::unmarshal(b);
  } else {
    key = PrivateKey::generate(kt == "rsa" ? KeyType::RSA : KeyType::Ed25519, 2048);
    if (!idf.empty()) {
      std::ofstream o(idf, std::ios::binary);
      Bytes b = key.marshal();
      o.write((const char*)b.data(), (std::streamsize)b.size());
    }
  }
  auto h = std::make_shared<Host>(key, "p2p-llm-chat-amd-relay/0.1.0");
  try {
    h->listen(Multiaddr::parse(env_or("RELAY_LISTEN", "/ip4/0.0.0.0/tcp/0")));
  } catch (const std::exception& e) {
    logf("%s", e.what());
    return 1;
  }
  RelayService svc(h);
  printf("🚏 Relay started. Addrs:\n");
  for (auto& a : h->addrs()) printf("  %s/p2p/%s\n", a.str().c_str(), h->id().to_base58().c_str());
  fflush(stdout);
  while (true) std::this_thread::sleep_for(std::chrono::hours(24));
}
