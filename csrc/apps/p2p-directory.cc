// Directory daemon: username -> {peer_id, addrs} (`go/cmd/directory/main.go`).
// Env: ADDR (default 127.0.0.1:8080); DIRECTORY_TTL seconds (0 = no expiry, like the reference).
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>

#include "net/chat.h"

using namespace p2p;

int main() {
  signal(SIGPIPE, SIG_IGN);
  std::string addr = env_or("ADDR", "127.0.0.1:8080");
  DirectoryService dir(atoi(env_or("DIRECTORY_TTL", "0").c_str()));
  HttpServer srv("GIN");
  dir.install(srv);
  try {
    srv.start(addr);
  } catch (const std::exception& e) {
    logf("%s", e.what());
    return 1;
  }
  logf("📒 Directory on %s", addr.c_str());
  srv.serve_forever();
  return 0;
}
