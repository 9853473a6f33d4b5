"""PMC target: the 44-row qkv projection (llama3.1-8B shape, RMSNorm + RoPE + KV-write
epilogue) on the wide kernel (split-K, 5 slices) and on the skinny kernel (w4/U4/NG2),
5 launches each, so rocprofv3 --pmc rows compare the two mid-M designs
(scripts/midm_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B, rope_table  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402

M, K, Hq, Hkv = 44, 4096, 32, 8
N = (Hq + 2 * Hkv) * 128
W = (torch.randn(N // 16, K // 32, 64, 8, device="cuda") * 0.02).to(torch.bfloat16)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
cs = rope_table(LLAMA31_8B, max_pos=256).to("cuda")
pos = torch.arange(M, device="cuda", dtype=torch.int32)
slots = torch.arange(M, device="cuda", dtype=torch.int32)
q = torch.zeros(M, Hq * 128, device="cuda", dtype=torch.bfloat16)
kc = torch.zeros(4, Hkv, 64, 128, device="cuda", dtype=torch.bfloat16)
vc = torch.zeros_like(kc)
for code in (G.WIDE_FLAG | (5 << 8), 4 | (4 << 8) | (2 << 16)):
    for _ in range(5):
        ops.qkv_rope_gemm(W, x, pos, slots, cs, Hq, Hkv, q, kc, vc, waves=code)
    torch.cuda.synchronize()
print("ok")
