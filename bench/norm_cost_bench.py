"""Cost of the fused RMSNorm statistics in the prefill GEMM: the same projection
(EPI_STORE) with norm=True computed in the k loop (sums of squares of the A fragments,
pre_rstd=0), with norm=True from the row_rstd kernel (pre_rstd=1, the default), and with
norm=False.  One JSON line per (N, M)."""
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
L = __import__("p2p_llm_chat_go_amd.ops._lib", fromlist=["lib"]).lib()
set_tiled_min_m(1)
for N in (6144, 28672):
    W = (torch.randn(N // 16, H // 32, 64, 8, device="cuda") * 0.02).to(torch.bfloat16)
    for M in (288, 2048, 8192):
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        o = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        t = {}
        for key, nm, pre in (("inloop", True, 0), ("pre", True, 1), ("plain", False, 1)):
            L.p2p_prefill_pre_rstd(pre)
            t[key] = graph_time(lambda i: ops.skinny_gemm(W, x, ops.EPI_STORE, norm=nm, out=o),
                                n_inner=10)
        L.p2p_prefill_pre_rstd(1)
        print(json.dumps({"M": M, "N": N, "K": H, "us_norm_inloop": round(t["inloop"], 1),
                          "us_norm_pre": round(t["pre"], 1), "us_plain": round(t["plain"], 1),
                          "speedup_pre": round(t["inloop"] / t["pre"], 3)}), flush=True)
    del W
