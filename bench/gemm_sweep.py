"""Sweep the skinny-GEMM pipeline depth (U) and split-K waves at llama3.1-8B decode
shapes (M=1 and M=8); prints us / TB/s per configuration (graph-replayed, cold weights)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402
from kernel_bench import copies, graph_time  # noqa: E402


def main():
    L = _lib.lib()
    H, F, QKV = 4096, 14336, 6144
    shapes = [("qkv", QKV, H, ops.EPI_STORE, True), ("o", H, H, ops.EPI_RESID, False),
              ("gate_up", 2 * F, H, ops.EPI_SILU, True), ("down", H, F, ops.EPI_RESID, False)]
    for M in (1, 8):
        for name, N, K, epi, norm in shapes:
            W = copies(N, K)
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.zeros(M, N // 2 if epi == ops.EPI_SILU else N, device="cuda",
                              dtype=torch.bfloat16)
            for u in (4, 8):
                L.p2p_skinny_gemm_tune(u, 0)
                for waves in (1, 2, 4, 8):
                    if (K // 32) // waves < 8:
                        continue
                    t = graph_time(lambda i: ops.skinny_gemm(W[i % len(W)], x, epi, norm=norm,
                                                             out=out, waves=waves))
                    print(json.dumps({"M": M, "gemm": name, "U": u, "waves": waves,
                                      "us": round(t, 2),
                                      "TBps": round(N * K * 2 / (t * 1e-6) / 1e12, 3)}), flush=True)
            del W


if __name__ == "__main__":
    main()
