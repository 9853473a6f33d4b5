"""Decode micro-benchmarks: skinny GEMV time vs N at K=4096 (do 16-row groups that do
not divide evenly over the 256 CUs cost a whole extra round?), and paged attention vs
context at batch 1 (graph-replayed, rotating weight copies beyond the Infinity Cache)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from kernel_bench import copies, graph_time  # noqa: E402


def main():
    K = 4096
    x = torch.randn(1, K, device="cuda").to(torch.bfloat16)
    for N in (2048, 3072, 4096, 5120, 6144, 7168, 8192, 12288, 16384):
        W = copies(N, K)
        out = torch.zeros(1, N, device="cuda", dtype=torch.bfloat16)
        best = None
        for waves in (1, 2, 4, 8):
            for u in (4, 8):
                code = waves | (u << 8)
                t = graph_time(lambda i: ops.skinny_gemm(W[i % len(W)], x, ops.EPI_STORE,
                                                         out=out, waves=code))
                if best is None or t < best[0]:
                    best = (t, waves, u)
        t, waves, u = best
        print(json.dumps({"gemv_N": N, "K": K, "groups": N // 16, "us": round(t, 2),
                          "waves": waves, "U": u,
                          "TBps": round(N * K * 2 / (t * 1e-6) / 1e12, 3)}), flush=True)
        del W
    # attention at batch 1, 32 q / 8 kv heads
    from p2p_llm_chat_go_amd.engine.kv_cache import KVCache
    from p2p_llm_chat_go_amd.models.config import LLAMA31_8B

    cfg = LLAMA31_8B.replace(n_layers=1)
    kv = KVCache(cfg, 600, "cuda")
    kv.k.normal_()
    kv.v.normal_()
    kc, vc = kv.layer(0)
    for ctx in (64, 128, 256, 512, 1024, 4096):
        pages = (ctx + 63) // 64
        bt = torch.arange(1, pages + 1, dtype=torch.int32, device="cuda")[None]
        q = torch.randn(1, 32 * 128, device="cuda").to(torch.bfloat16)
        cl = torch.tensor([ctx], dtype=torch.int32, device="cuda")
        ws = ops.attn_workspace(1, 32, ctx, "cuda")
        out = torch.empty_like(q)
        t = graph_time(lambda i: ops.paged_attention(q, kc, vc, bt, None, cl, 32, 8, ctx, out=out,
                                                     workspace=ws))
        print(json.dumps({"attn_ctx": ctx, "us": round(t, 2)}), flush=True)


if __name__ == "__main__":
    main()
