"""Batch-1 decode GEMVs (llama3.1-8B) at every skinny launch code, 32 layers' weights
(cold), graph-replayed: the spread between codes and the fixed cost per launch beyond the
weight stream (us - MB / 7.0 TB/s, the rate the 1 GB LM head streams at).

Run on the GPU: python bench/gemv_codes_probe.py   (one JSON line per projection)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _configs, _graph_time, describe  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402


def main():
    eng = Engine(LLAMA31_8B, device="cuda", kv_pages=64, max_batch=1)
    m = eng.model
    layers = m.w.layers
    H, nq, nkv = LLAMA31_8B.hidden, m.nq, m.nkv
    kc, vc = m.kv.layer(0)
    M = 1
    x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    h = torch.zeros(M, H, device="cuda", dtype=torch.bfloat16)
    q = torch.randn(M, nq * 128, device="cuda").to(torch.bfloat16)
    pos = torch.zeros(M, device="cuda", dtype=torch.int32)
    slots = torch.zeros(M, device="cuda", dtype=torch.int32)
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
    # a dependent chain of tiny kernels (8 KB fills): the launch-to-launch cost alone
    t = _graph_time(lambda: [h.fill_(0.5) for _ in range(128)], reps=5) * 1000 / 128
    print(json.dumps({"tiny_kernel_us_per_launch": round(t, 2)}), flush=True)
    for name, wts, fn in jobs:
        N, K = G.tiled_shape(wts[0])
        mb = N * K * 2 / 1e6
        row = {"gemm": name, "MB": round(mb, 1), "stream_us_at_7TBps": round(mb / 7.0, 2)}
        for code in _configs(K, M):
            try:
                t = _graph_time(lambda: [fn(wt, code) for wt in wts], reps=5) * 1000 / len(wts)
            except RuntimeError as e:  # a code this epilogue does not launch
                row[describe(code)] = str(e)[:40]
                continue
            row[describe(code)] = round(t, 2)
        print(json.dumps(row), flush=True)
    assert ops.tiled_split_fault() == 0


if __name__ == "__main__":
    main()
