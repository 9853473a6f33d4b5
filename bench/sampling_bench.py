"""Sampled vs greedy decode at llama3.1-8B (1 GPU): ops.sample kernel time per row
count, and tokens/s of 64-token continuations through the decode graph with
Ollama's default sampler (temperature 0.8, top_k 40, top_p 0.9) vs greedy.
Run on the GPU: python bench/sampling_bench.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.sampling import SamplingParams  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402
from kernel_bench import graph_time  # noqa: E402


def main():
    V = LLAMA31_8B.vocab
    for B in (1, 8, 32):
        lg = torch.randn(B, V, device="cuda") * 3
        temp = torch.full((B,), 0.8, device="cuda")
        topk = torch.full((B,), 40, device="cuda", dtype=torch.int32)
        topp = torch.full((B,), 0.9, device="cuda")
        seeds = torch.arange(B, device="cuda", dtype=torch.int64)
        pos = torch.arange(B, device="cuda", dtype=torch.int32)
        out = torch.empty(B, device="cuda", dtype=torch.int32)
        t = graph_time(lambda i: ops.sample(lg, temp, topk, topp, seeds, pos, out=out), n_inner=20)
        print(json.dumps({"kernel": "sample", "rows": B, "vocab": V, "us": round(t, 2)}), flush=True)
    eng = Engine(LLAMA31_8B, device="cuda", kv_pages=64, max_batch=1)
    prompt = list(range(1000, 1036))
    n = 64
    for name, params in (("greedy", None),
                         ("sampled_t0.8_k40_p0.9", [SamplingParams(temperature=0.8, seed=1)])):
        pages = [eng.kv.allocator.alloc(2)]
        first = eng.prefill([prompt], pages, sampling=params).cpu().tolist()
        g = eng.decode_graph(1, len(prompt) + n + 1, greedy=params is None)
        best = 1e9
        for _ in range(4):
            g.state.load(first, [len(prompt)], pages)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if params is None:
                g.replay(n)
            else:
                g.step_sampled(params, n)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        eng.kv.allocator.free(pages[0])
        print(json.dumps({"decode": name, "tokens": n, "ms_per_token": round(best * 1e3 / n, 4),
                          "tokens_per_s": round(n / best, 1)}), flush=True)


if __name__ == "__main__":
    main()
