"""Per-kernel decode microbenchmarks at llama3.1-8B shapes (graph-replayed, so
launch overhead is the in-graph boundary, as in the real decode step).

Each kernel is captured N times into one hipGraph over rotating weight copies
(> 256 MiB in total, so the Infinity Cache cannot serve re-reads) and the
replay is timed with events.  Prints one JSON line per kernel: us / call and
achieved HBM TB/s for the weight stream.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B, rope_table  # noqa: E402


def graph_time(fn, n_inner=40, n_rep=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n_inner):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(n_rep):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000 / n_inner)
    return best


def copies(n, k, nbytes_target=300 << 20, lead=()):
    per = n * k * 2
    c = max(1, min(16, nbytes_target // per + 1))
    return [torch.randn(*lead, n // 16, k // 32, 64, 8, device="cuda").to(torch.bfloat16)
            for _ in range(c)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--prefill", type=int, nargs="*", default=[512, 2048])
    ap.add_argument("--attn-prefill", type=int, nargs="*", default=[64, 512, 2048, 8192])
    a = ap.parse_args()
    cfg = LLAMA31_8B
    H, F, V = cfg.hidden, cfg.ffn, cfg.vocab
    nq, nkv = cfg.n_heads, cfg.n_kv_heads
    cs = rope_table(cfg, 4096, "cuda")
    P = 64
    kc = torch.randn(P, nkv, 64, 128, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    prefill_attn_bench(a.attn_prefill)
    prefill_bench(a.prefill)
    for M in a.M:
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        xf = torch.randn(M, F, device="cuda").to(torch.bfloat16)
        h = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        q = torch.zeros(M, nq * 128, device="cuda", dtype=torch.bfloat16)
        act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
        pos = torch.full((M,), 100, device="cuda", dtype=torch.int32)
        slots = torch.arange(M, device="cuda", dtype=torch.int32) + 64
        keys = ops.new_argmax_keys(M, "cuda")
        res = []
        Wq = copies((nq + 2 * nkv) * 128, H)
        t = graph_time(lambda i: ops.qkv_rope_gemm(Wq[i % len(Wq)], x, pos, slots, cs, nq, nkv, q,
                                                   kc, vc, waves=a.waves))
        res.append(("qkv_rope", t, (nq + 2 * nkv) * 128 * H * 2))
        Wo = copies(H, nq * 128)
        t = graph_time(lambda i: ops.skinny_gemm(Wo[i % len(Wo)], q, ops.EPI_RESID, out=h,
                                                 waves=a.waves))
        res.append(("o_proj_resid", t, H * nq * 128 * 2))
        t = graph_time(lambda i: ops.skinny_gemm(Wo[0], q, ops.EPI_RESID, out=h, waves=a.waves))
        res.append(("o_proj_resid_l3hot", t, H * nq * 128 * 2))
        t = graph_time(lambda i: ops.qkv_rope_gemm(Wq[0], x, pos, slots, cs, nq, nkv, q, kc, vc,
                                                   waves=a.waves))
        res.append(("qkv_rope_l3hot", t, (nq + 2 * nkv) * 128 * H * 2))
        Wgu = copies(2 * F, H)
        t = graph_time(lambda i: ops.skinny_gemm(Wgu[i % len(Wgu)], x, ops.EPI_SILU, norm=True,
                                                 out=act, waves=a.waves))
        res.append(("gate_up_silu", t, 2 * F * H * 2))
        Wd = copies(H, F)
        t = graph_time(lambda i: ops.skinny_gemm(Wd[i % len(Wd)], xf, ops.EPI_RESID, out=h,
                                                 waves=a.waves))
        res.append(("down_resid", t, H * F * 2))
        Wl = copies(V, H)
        t = graph_time(lambda i: ops.lm_head_argmax(Wl[i % len(Wl)], x, keys, waves=a.waves),
                       n_inner=10)
        res.append(("lm_head_argmax", t, V * H * 2))
        bt = torch.arange(1, 1 + M * 4, device="cuda", dtype=torch.int32).view(M, 4) % P
        rb = torch.arange(M, device="cuda", dtype=torch.int32)
        for ctx_len in (100, 1000):
            ctx = torch.full((M,), ctx_len, device="cuda", dtype=torch.int32)
            bt2 = (torch.arange(M * 16, device="cuda", dtype=torch.int32).view(M, 16) % (P - 1)) + 1
            ws = ops.attn_workspace(M, nq, ctx_len, "cuda")
            out = torch.zeros(M, nq * 128, device="cuda", dtype=torch.bfloat16)
            t = graph_time(lambda i: ops.paged_attention(q, kc, vc, bt2, rb, ctx, nq, nkv, ctx_len,
                                                         out=out, workspace=ws))
            res.append(("attention_ctx%d" % ctx_len, t, M * ctx_len * nkv * 128 * 2 * 2))
        del bt
        total = 0
        for name, t, nbytes in res:
            print(json.dumps({"M": M, "kernel": name, "us": round(t, 2),
                              "TBps": round(nbytes / (t * 1e-6) / 1e12, 3)}), flush=True)
        d = {n: t for n, t, _ in res}
        layer = (d["qkv_rope"] + d["o_proj_resid"] + d["gate_up_silu"] + d["down_resid"]
                 + d["attention_ctx100"])
        print(json.dumps({"M": M, "layer_us_ctx100": round(layer, 2),
                          "est_step_ms": round((32 * layer + d["lm_head_argmax"]) / 1000, 3)}),
              flush=True)


def prefill_attn_bench(Ts):
    """Causal prefill attention, one sequence of T tokens (8B heads): MFMA flash
    kernel vs the per-row paged kernel.  TFLOP/s counts the causal half."""
    cfg = LLAMA31_8B
    nq, nkv = cfg.n_heads, cfg.n_kv_heads
    for T in Ts:
        npg = (T + 63) // 64
        kc = torch.randn(npg + 1, nkv, 64, 128, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(1, npg + 1, device="cuda", dtype=torch.int32)[None]
        q = torch.randn(T, nq * 128, device="cuda").to(torch.bfloat16)
        out = torch.empty_like(q)
        pos = list(range(T))
        from p2p_llm_chat_go_amd.ops import attention as A

        res = []
        for v2 in (True, False):
            A.FLASH_V2 = v2
            qt = ops.flash_tile(nq, nkv)
            tiles = ops.prefill_tiles([0] * T, pos, qt).to("cuda")
            res.append(("flash_prefill_v2" if v2 else "flash_prefill_v1",
                        graph_time(lambda i: ops.flash_prefill(q, kc, vc, bt, tiles, nq, nkv,
                                                               out=out, qtile=qt), n_inner=10)))
        A.FLASH_V2 = True
        rb = torch.zeros(T, device="cuda", dtype=torch.int32)
        ctx = torch.arange(1, T + 1, device="cuda", dtype=torch.int32)
        ws = ops.attn_workspace(T, nq, T, "cuda")
        flops = 2 * 2 * nq * 128 * T * (T + 1) / 2
        if T <= 8192:
            res.append(("per_row_paged", graph_time(
                lambda i: ops.paged_attention(q, kc, vc, bt, rb, ctx, nq, nkv, T, out=out,
                                              workspace=ws), n_inner=10)))
        for name, t in res:
            print(json.dumps({"prefill_attn_T": T, "kernel": name, "us": round(t, 1),
                              "TFLOPs": round(flops / (t * 1e-6) / 1e12, 1)}), flush=True)


def prefill_bench(Ms):
    """Tiled MFMA GEMMs at prefill M (compute-bound): TFLOP/s per projection."""
    cfg = LLAMA31_8B
    H, F = cfg.hidden, cfg.ffn
    for M in Ms:
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        xf = torch.randn(M, F, device="cuda").to(torch.bfloat16)
        h = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
        o = torch.zeros(M, 6144, device="cuda", dtype=torch.bfloat16)
        for name, N, K, fn in [
            ("qkv", 6144, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_STORE, norm=True, out=o)),
            ("gate_up", 2 * F, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_SILU, norm=True, out=act)),
            ("down", H, F, lambda W: ops.skinny_gemm(W, xf, ops.EPI_RESID, out=h))]:
            W = copies(N, K, nbytes_target=0)
            t = graph_time(lambda i: fn(W[0]), n_inner=10)
            torch_t = graph_time(lambda i: torch.matmul(x if K == H else xf,
                                                        torch.empty(K, N, device="cuda",
                                                                    dtype=torch.bfloat16)),
                                 n_inner=10) if False else None
            print(json.dumps({"prefill_M": M, "gemm": name, "us": round(t, 1),
                              "TFLOPs": round(2 * M * N * K / (t * 1e-6) / 1e12, 1)}), flush=True)
        Wb = torch.randn(H, 2 * F, device="cuda").to(torch.bfloat16)
        t = graph_time(lambda i: torch.matmul(x, Wb), n_inner=10)
        print(json.dumps({"prefill_M": M, "gemm": "hipblaslt_gate_up_reference", "us": round(t, 1),
                          "TFLOPs": round(2 * M * 2 * F * H / (t * 1e-6) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
