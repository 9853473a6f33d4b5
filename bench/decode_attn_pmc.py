"""Decode paged attention at batch 1, ctx 100 (llama3.1-8B heads), a few launches, for a
rocprofv3 --pmc pass."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402


def main():
    ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    kc = torch.randn(64, 8, 64, 128, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    pages = (ctx + 63) // 64
    bt = torch.arange(1, pages + 1, dtype=torch.int32, device="cuda")[None]
    q = torch.randn(1, 32 * 128, device="cuda").to(torch.bfloat16)
    cl = torch.tensor([ctx], dtype=torch.int32, device="cuda")
    ws = ops.attn_workspace(1, 32, ctx, "cuda")
    out = torch.empty_like(q)
    for _ in range(5):
        ops.paged_attention(q, kc, vc, bt, None, cl, 32, 8, ctx, out=out, workspace=ws)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
