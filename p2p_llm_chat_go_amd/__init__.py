"""MI355X-native P2P LLM chat node (capabilities of NajyFannoun/P2P-LLM-Chat-Go).

Layers (see SURVEY.md §1 for the reference's layer map):
  net/       chat plane: native C++ libp2p subset (TCP + Noise XX + yamux +
             multistream-select), /p2p-llm-chat/1.0.0, Directory, circuit relay v2,
             node HTTP API (POST /send, GET /inbox, GET /me, /suggest, /api/generate)
  engine/    in-process suggest-reply engine (paged KV, hipGraph decode,
             continuous batching) replacing the reference's Ollama hop
  models/    Llama-3.1 (8B/70B) and Mixtral-8x7B configs, weights, forward, oracle
  ops/       hand-written gfx950 HIP kernels (MFMA skinny GEMM, paged attention, ...)
  parallel/  tensor / expert / data parallelism over RCCL (xGMI)
  utils/     env config, timing, roctx
"""
__version__ = "0.1.0"
