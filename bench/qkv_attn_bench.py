#!/usr/bin/env python3
"""Decode qkv+RoPE+KV write followed by attention: the two-kernel path (skinny GEMM +
paged attention) vs the one-launch kernel (ops.qkv_attn) and its probes, at llama3.1-8B
(TP=1) and 70B TP=8 rank shapes, graph-replayed over 32 cold weight copies.  One JSON
line per (shape, variant)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B, rope_table  # noqa: E402
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402


def run(name, Hq, Hkv, K, M, ctx_len, L=32, hidden=None):
    hidden = hidden or K
    dev = "cuda"
    N = (Hq + 2 * Hkv) * 128
    wts = [torch.randn(N // 16, K // 32, 64, 8, device=dev).mul_(0.02).to(torch.bfloat16)
           for _ in range(L)]
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    P = 1 + 4 * M
    kc = torch.randn(P, Hkv, 64, 128, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = (torch.arange(4 * M, device=dev, dtype=torch.int32) + 1).view(M, 4)
    ctx = torch.full((M,), ctx_len, device=dev, dtype=torch.int32)
    pos = ctx - 1
    slots = (bt[torch.arange(M), (pos // 64).long()] * 64 + pos % 64).to(torch.int32)
    cs = rope_table(LLAMA31_8B, max_pos=512, device=dev)
    q = torch.zeros(M, Hq * 128, device=dev, dtype=torch.bfloat16)
    out = torch.zeros_like(q)
    ws = ops.qkv_attn_workspace(M, Hq, Hkv, dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    Lb = _lib.lib()

    def two(i):
        ops.qkv_rope_gemm(wts[i % L], x, pos, slots, cs, Hq, Hkv, q, kc, vc)
        ops.paged_attention(q, kc, vc, bt, None, ctx, Hq, Hkv, 256, out=out)

    def qkv_only(i):
        ops.qkv_rope_gemm(wts[i % L], x, pos, slots, cs, Hq, Hkv, q, kc, vc)

    def fused(i, waves=None):
        ops.qkv_attn(wts[i % L], x, pos, slots, cs, Hq, Hkv, kc, vc, bt, ctx, out, ws, err,
                     waves=waves)

    No = hidden  # o_proj output width: the model's hidden size
    wos = [torch.randn(No // 16, Hq * 128 // 32, 64, 8, device=dev).mul_(0.02).to(torch.bfloat16)
           for _ in range(L)]
    h = torch.zeros(M, No, device=dev, dtype=torch.bfloat16)

    # the unfused o_proj at its best skinny launch code (what the engine's autotuner picks)
    best_o = min(((graph_time(lambda i, c=c: ops.skinny_gemm(wos[i % L], out, ops.EPI_RESID,
                                                               out=h, waves=c), n_inner=L), c)
                  for c in [w | (u << 8) for w in (1, 2, 4, 8) for u in (4, 8)]))
    res_o = {"o_proj_alone": best_o[0]}

    def fused_then_oproj(i):
        ops.qkv_attn(wts[i % L], x, pos, slots, cs, Hq, Hkv, kc, vc, bt, ctx, out, ws, err)
        ops.skinny_gemm(wos[i % L], out, ops.EPI_RESID, out=h, waves=best_o[1])

    def fused_oproj(i, waves=None):
        ops.qkv_attn(wts[i % L], x, pos, slots, cs, Hq, Hkv, kc, vc, bt, ctx, None, ws, err,
                     waves=waves, oproj=(wos[i % L], h))

    res = dict(res_o)
    res["qkv_attn+o_proj_2launch"] = graph_time(fused_then_oproj, n_inner=L)
    for wv in (4, 8):
        if ops.qkv_attn_oproj_ok(wos[0], Hq, Hkv, wv, rows=M, hidden=K):
            res["qkv_attn_oproj_w%d" % wv] = graph_time(lambda i: fused_oproj(i, wv), n_inner=L)
    for wv in (4, 8):
        res["fused_w%d" % wv] = graph_time(lambda i: fused(i, wv), n_inner=L)
        # k-split producers (launch code bits 8..15: slices per column group)
        for ks in (1, 2, 3, 4, 6, 8):
            if (K // 32) // ks < 16:
                continue
            if ks > 1:
                res["fused_w%d_ks%d" % (wv, ks)] = graph_time(lambda i: fused(i, wv | (ks << 8)),
                                                              n_inner=L)
            if ctx_len <= 128 and ks <= 4:  # consumers with 2 key waves (contexts <= 128)
                res["fused_w%d_ks%d_kw2" % (wv, ks)] = graph_time(
                    lambda i: fused(i, wv | (ks << 8) | (2 << 16)), n_inner=L)
    res["two_kernels"] = graph_time(two, n_inner=L)
    res["qkv_only"] = graph_time(qkv_only, n_inner=L)
    for mode, label in ((0, "fused"), (1, "fused_producers_only"), (2, "fused_handoff_only"),
                        (6, "fused_kv_wait_handoff_only")):
        Lb.p2p_qkv_attn_probe(mode)
        res[label] = graph_time(fused, n_inner=L)
        if ctx_len <= 128:  # the engine's launch for <= 128 keys: 2 key waves (w4, whole groups)
            res[label + "_kw2"] = graph_time(lambda i: fused(i, 4 | (2 << 16)), n_inner=L)
    Lb.p2p_qkv_attn_probe(0)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    print(json.dumps({"shape": name, "M": M, "ctx": ctx_len,
                      **{k: round(v, 2) for k, v in res.items()}, "unit": "us per layer"}),
          flush=True)


if __name__ == "__main__":
    run("llama3.1-8B TP=1", 32, 8, 4096, 1, 108)
    run("llama3.1-8B TP=1", 32, 8, 4096, 8, 108)
    run("llama3.1-70B TP=8 rank", 8, 1, 8192, 1, 108)
