"""Long-context suggest-reply at llama3.1-8B (1 GPU): TTFT of a P-token prompt (chunked
prefill, MFMA flash attention) and decode ms/token at that context (hipGraph, split-K
paged attention).  Synthetic token ids, random-init weights.
Run on the GPU: python bench/long_ctx_bench.py [P ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402


def main():
    Ps = [int(p) for p in sys.argv[1:]] or [1024, 8192, 32768]
    n = 32
    eng = Engine(LLAMA31_8B, device="cuda", max_batch=1, max_prefill_tokens=4096)
    eng.warmup((1,), ctx=256)
    for P in Ps:
        prompt = [(i * 7919) % 120000 + 100 for i in range(P)]
        pages = [eng.kv.allocator.alloc((P + n + 63) // 64)]
        eng.prefill([prompt], pages).cpu()  # warm (workspace, graphs of this bucket)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        first = eng.prefill([prompt], pages).cpu().tolist()
        ttft = time.perf_counter() - t0
        g = eng.decode_graph(1, P + n + 1)
        g.state.load(first, [P], pages)
        g.replay(2)
        torch.cuda.synchronize()
        g.state.load(first, [P], pages)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay(n)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        eng.kv.allocator.free(pages[0])
        print(json.dumps({"model": "llama3.1-8b", "prompt_tokens": P, "ttft_ms": round(ttft * 1e3, 2),
                          "prefill_tokens_per_s": round(P / ttft, 1),
                          "decode_ms_per_token": round(dt * 1e3, 3),
                          "decode_tokens_per_s": round(1 / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
