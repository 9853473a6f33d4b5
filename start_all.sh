#!/bin/bash
# Launch the local demo: Directory + two chat nodes (Najy :8081, Cannan :8082),
# each with its in-process suggest-reply engine and browser UI (http://127.0.0.1:8081/).
# Mirrors the reference launcher's topology (Directory on :8080, two nodes); the
# Ollama + Streamlit processes are replaced by the engine inside each node.
# Env: ENGINE_MODEL (default llama3.1-8b on GPU / tiny-llama on CPU), ENGINE=0 disables it.
#      WITH_RELAY=1 also starts a circuit-relay-v2 hop and routes node 2 through it.
set -e
cd "$(dirname "$0")"
python -m p2p_llm_chat_go_amd._build >/dev/null
pids=()
cleanup() { kill "${pids[@]}" 2>/dev/null || true; }
trap cleanup EXIT INT TERM

echo "Starting Directory server..."
ADDR=127.0.0.1:8080 ./bin/p2p-directory & pids+=($!)
sleep 0.5
RELAY=""
if [ "${WITH_RELAY:-0}" = "1" ]; then
  echo "Starting relay..."
  RELAY_LISTEN=/ip4/127.0.0.1/tcp/4001 ./bin/p2p-relay > /tmp/p2p-relay.out & pids+=($!)
  sleep 0.5
  RELAY=$(grep -m1 "/p2p/" /tmp/p2p-relay.out | tr -d ' ')
fi

echo "Starting Node 1 (Najy)..."
MYNAMEIS=Najy HTTP_ADDR=127.0.0.1:8081 DIRECTORY_URL=http://127.0.0.1:8080 \
  python -m p2p_llm_chat_go_amd.net.node & pids+=($!)

echo "Starting Node 2 (Cannan)..."
MYNAMEIS=Cannan HTTP_ADDR=127.0.0.1:8082 DIRECTORY_URL=http://127.0.0.1:8080 RELAY_ADDRS="$RELAY" \
  ENGINE_DEVICE=${NODE2_DEVICE:-} python -m p2p_llm_chat_go_amd.net.node & pids+=($!)

echo "All services started! UIs: http://127.0.0.1:8081/  http://127.0.0.1:8082/"
wait
