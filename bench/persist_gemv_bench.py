"""Persistent GEMV (ops.gemm.PERSIST_FLAG) vs the tuned skinny launch on the 8B decode
projections (32 layers' weights, graph-replayed, M = 1 and 8): one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _graph_time  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402


def main():
    dev = "cuda"
    L = 32
    shapes = [("gate_up", 28672, 4096, ops.EPI_SILU, 1025), ("down", 4096, 14336, ops.EPI_RESID, 2056),
              ("o_proj", 4096, 4096, ops.EPI_RESID, 1032)]
    for name, N, K, epi, skinny in shapes:
        wts = [torch.randn(N // 16, K // 32, 64, 8, device=dev).to(torch.bfloat16) * 0.02 for _ in range(L)]
        for M in (1, 8):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = torch.zeros(M, N // 2 if epi == ops.EPI_SILU else N, device=dev, dtype=torch.bfloat16)
            norm = epi == ops.EPI_SILU
            res = {"shape": name, "M": M, "N": N, "K": K}
            for label, code in (("skinny", skinny), ("persist_x1", G.PERSIST_FLAG),
                                ("persist_x2", G.PERSIST_FLAG | (2 << 8))):
                t = _graph_time(lambda: [ops.skinny_gemm(w, x, epi, norm=norm, out=out, waves=code)
                                         for w in wts])
                res[label + "_us"] = round(t * 1000 / L, 2)
            print(json.dumps(res), flush=True)
        del wts


if __name__ == "__main__":
    main()
