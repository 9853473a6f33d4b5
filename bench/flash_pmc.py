"""Runs the flash-prefill v2 kernel a few times at T=8192 (llama3.1-8B heads) for a
rocprofv3 --pmc pass (counters of the attention kernel alone)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402


def main():
    T, Hq, Hkv = 8192, 32, 8
    pages = T // 64
    kc = torch.randn(pages + 1, Hkv, 64, 128, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(T, Hq * 128, device="cuda").to(torch.bfloat16)
    bt = torch.arange(1, pages + 1, dtype=torch.int32, device="cuda")[None]
    qt = ops.flash_tile(Hq, Hkv, T)
    tiles_h = ops.prefill_tiles([0] * T, list(range(T)), qt)
    tiles = tiles_h.cuda()
    out = torch.empty_like(q)
    for _ in range(3):
        ops.flash_prefill(q, kc, vc, bt, tiles, Hq, Hkv, out=out, tiles_host=tiles_h, qtile=qt)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
