"""Decode attention at llama3.1-8B heads (32 q / 8 kv), contexts <= 256: the 4-wave MFMA
kernel vs the 16-wave kernel (paged_attention.hip), graph-replayed, per launch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402


def main():
    from p2p_llm_chat_go_amd.engine.kv_cache import KVCache
    from p2p_llm_chat_go_amd.models.config import LLAMA31_8B

    L = _lib.lib()
    cfg = LLAMA31_8B.replace(n_layers=1)
    kv = KVCache(cfg, 600, "cuda")
    kv.k.normal_()
    kv.v.normal_()
    kc, vc = kv.layer(0)
    for B in (1, 8):
        for ctx in (44, 108, 200, 256):
            bt = torch.arange(1, 4 * B + 1, dtype=torch.int32, device="cuda").view(B, 4)
            q = torch.randn(B, 32 * 128, device="cuda").to(torch.bfloat16)
            cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
            out = torch.empty_like(q)
            res = {}
            for on, name in ((0, "wave16_us"), (1, "mfma_us")):
                L.p2p_paged_attention_mfma(on)
                res[name] = round(graph_time(
                    lambda i: ops.paged_attention(q, kc, vc, bt, None, cl, 32, 8, 256, out=out)), 2)
            L.p2p_paged_attention_mfma(1)
            print(json.dumps(dict(B=B, ctx=ctx, **res)), flush=True)


if __name__ == "__main__":
    main()
