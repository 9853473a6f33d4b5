"""Cost of the fused RMSNorm statistics in the prefill GEMM main loop: the same qkv-shaped
projection (EPI_STORE) with norm=True (sums of squares of the A fragments accumulated
in the k loop, rstd applied in the epilogue) vs norm=False.  One JSON line per M."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops.gemm import set_tiled_min_m  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402

H = 4096
set_tiled_min_m(1)
for N in (6144, 28672):
    W = (torch.randn(N // 16, H // 32, 64, 8, device="cuda") * 0.02).to(torch.bfloat16)
    for M in (288, 2048, 8192):
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        o = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        t = {nm: graph_time(lambda i: ops.skinny_gemm(W, x, ops.EPI_STORE, norm=nm, out=o), n_inner=10)
             for nm in (True, False)}
        print(json.dumps({"M": M, "N": N, "K": H, "us_norm": round(t[True], 1),
                          "us_plain": round(t[False], 1),
                          "norm_cost_pct": round(100 * (t[True] / t[False] - 1), 1)}), flush=True)
    del W
