"""Decode attention + o_proj at llama3.1-8B shapes: separate kernels vs the fused
one-launch kernels -- the hand-off kernel (ops.attn_oproj) and the head-split kernel
(ops.attn_oproj_heads) -- graph-replayed over 32 cold weight copies."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402


def main():
    from p2p_llm_chat_go_amd.ops import _lib
    L = _lib.experimental()
    Hq, Hkv, H = 32, 8, 4096
    for R, ctx_len in ((1, 50), (1, 100), (1, 250), (2, 100), (4, 100), (8, 100), (16, 200)):
        P = 1 + R * 4
        kc = torch.randn(P, Hkv, 64, 128, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = (torch.arange(R * 4, device="cuda", dtype=torch.int32) + 1).view(R, 4)
        rb = torch.arange(R, device="cuda", dtype=torch.int32)
        ctx = torch.full((R,), ctx_len, device="cuda", dtype=torch.int32)
        q = torch.randn(R, Hq * 128, device="cuda").to(torch.bfloat16)
        h = torch.randn(R, H, device="cuda").to(torch.bfloat16)
        attn = torch.zeros_like(q)
        Wo = [torch.randn(H // 16, Hq * 128 // 32, 64, 8, device="cuda").to(torch.bfloat16)
              for _ in range(32)]
        sync = torch.zeros(2, dtype=torch.int32, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        ws = ops.attn_workspace(R, Hq, 256, "cuda")
        slab, tickets = ops.attn_oproj_heads_workspace(R, Hkv, H, "cuda")

        def sep(i):
            ops.paged_attention(q, kc, vc, bt, rb, ctx, Hq, Hkv, 256, out=attn, workspace=ws)
            ops.skinny_gemm(Wo[i % 32], attn, ops.EPI_RESID, out=h)

        def fused(i):
            ops.attn_oproj(q, kc, vc, bt, rb, ctx, Hq, Hkv, 256, Wo[i % 32], h, attn, sync, err)
        def heads(i):
            ops.attn_oproj_heads(q, kc, vc, bt, rb, ctx, Hq, Hkv, 256, Wo[i % 32], h, slab,
                                 tickets)
        ts = graph_time(sep, n_inner=32)
        tf = graph_time(fused, n_inner=32)
        th = {}
        for flags, name in ((1, "heads_us"), (0, "heads_wfirst_us"), (3, "heads_nofanin_us")):
            L.p2p_attn_oproj_heads_tune(flags)
            th[name] = round(graph_time(heads, n_inner=32), 2)
        L.p2p_attn_oproj_heads_tune(1)
        torch.cuda.synchronize()
        print(json.dumps(dict({"R": R, "ctx": ctx_len, "separate_us": round(ts, 2),
                               "fused_handoff_us": round(tf, 2)}, **th,
                              err=int(err.item()))), flush=True)


if __name__ == "__main__":
    main()
