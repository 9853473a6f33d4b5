"""How much of a projection's time is the HBM stream: each llama3.1-8B projection at its
pinned launch code, graph-replayed over 32 layers' weights (cold in the Infinity Cache,
as in the model) vs the SAME layer's weights 32 times (resident in the 256 MB Infinity
Cache after the first launch).  A big cold/warm gap says a prefetch of the next
projection's weights (during a kernel's tail) has something to win; no gap says the
kernel is bound by something other than the memory-side stream.

Run on the GPU: python bench/mall_probe.py [M ...]   (one JSON line per (M, projection))"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _graph_time, describe, load_table  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402


def main():
    Ms = [int(m) for m in sys.argv[1:]] or [1, 48]
    eng = Engine(LLAMA31_8B, device="cuda", kv_pages=64, max_batch=1)
    m = eng.model
    layers = m.w.layers
    H, nq, nkv = LLAMA31_8B.hidden, m.nq, m.nkv
    kc, vc = m.kv.layer(0)
    codes = load_table("llama3.1-8b")
    for M in Ms:
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        h = torch.zeros(M, H, device="cuda", dtype=torch.bfloat16)
        q = torch.randn(M, nq * 128, device="cuda").to(torch.bfloat16)
        pos = torch.zeros(M, device="cuda", dtype=torch.int32)
        slots = torch.arange(M, device="cuda", dtype=torch.int32) % 64
        F = layers[0].gate_up.shape[0] * 16 // 2
        act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
        xf = torch.randn(M, F, device="cuda").to(torch.bfloat16)
        jobs = [("qkv_rope", [lw.qkv for lw in layers],
                 lambda wt, c: ops.qkv_rope_gemm(wt, x, pos, slots, m.rope, nq, nkv, q, kc, vc,
                                                 waves=c)),
                ("o_proj", [lw.o for lw in layers],
                 lambda wt, c: ops.skinny_gemm(wt, q, ops.EPI_RESID, out=h, waves=c)),
                ("gate_up", [lw.gate_up for lw in layers],
                 lambda wt, c: ops.skinny_gemm(wt, x, ops.EPI_SILU, norm=True, out=act, waves=c)),
                ("down", [lw.down for lw in layers],
                 lambda wt, c: ops.skinny_gemm(wt, xf, ops.EPI_RESID, out=h, waves=c))]
        for name, wts, fn in jobs:
            N, K = G.tiled_shape(wts[0])
            code = codes.get("%s:N%d:K%d:M%d" % (name, N, K, M))
            if code is None:
                continue
            cold = _graph_time(lambda: [fn(wt, code) for wt in wts], reps=5) * 1000 / len(wts)
            warm = _graph_time(lambda: [fn(wts[0], code) for _ in wts], reps=5) * 1000 / len(wts)
            mb = N * K * 2 / 1e6
            print(json.dumps({"M": M, "gemm": name, "code": describe(code), "MB": round(mb, 1),
                              "cold_us": round(cold, 2), "warm_us": round(warm, 2),
                              "cold_TBps": round(mb / cold, 2),
                              "warm_TBps": round(mb / warm, 2)}), flush=True)
    assert ops.tiled_split_fault() == 0


if __name__ == "__main__":
    main()
