"""PMC target: the prefill GEMM at two operating points, each launched 5 times with
the tile forced -- gate_up at 288 rows on the one-m-tile 320x128 tile (mid-M) and at
8192 rows on the phased 256x256 tile (large M) -- so rocprofv3 --pmc rows can be
compared per k-step (scripts/gemm_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops.gemm import set_tiled_min_m, tiled_config  # noqa: E402

H, F = 4096, 14336
W = (torch.randn(2 * F // 16, H // 32, 64, 8, device="cuda") * 0.02).to(torch.bfloat16)
set_tiled_min_m(1)
for M, cfg in ((288, (2, 6, 1)), (8192, (2, 1, 1))):
    x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
    tiled_config(*cfg)
    for _ in range(5):
        ops.skinny_gemm(W, x, ops.EPI_SILU, norm=True, out=act)
    torch.cuda.synchronize()
print("ok")
