"""Re-time every launch candidate of the 8B prompt-sized projections (33-64 rows) on this
box, twice, next to the pinned table's pick: checks that a pinned near-tie pick does not
lose on another box (the table is shared by every box)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _configs, _graph_time, describe, load_table  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402


def main():
    dev = "cuda"
    L = 8
    table = load_table("llama3.1-8b")
    for name, N, K, epi in (("gate_up", 28672, 4096, G.EPI_SILU), ("o_proj", 4096, 4096, G.EPI_RESID),
                            ("down", 4096, 14336, G.EPI_RESID)):
        wts = [(torch.randn(N // 16, K // 32, 64, 8, device=dev) * 0.02).to(torch.bfloat16) for _ in range(L)]
        for M in (44, 64):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = torch.zeros(M, N // 2 if epi == G.EPI_SILU else N, device=dev, dtype=torch.bfloat16)
            norm = epi == G.EPI_SILU
            codes = _configs(K, M, G.tiled_ok(N, K, epi), midm=True, wide=G.wide_ok(N, K, epi))
            res = {}
            for rep in range(2):
                for c in codes:
                    t = _graph_time(lambda: [ops.skinny_gemm(w, x, epi, norm=norm, out=out, waves=c)
                                             for w in wts]) * 1000 / L
                    res.setdefault(describe(c), []).append(round(t, 2))
            mb = 48 if M <= 48 else 64
            pinned = table.get("%s:N%d:K%d:M%d" % (name, N, K, mb))
            best = sorted(res.items(), key=lambda kv: min(kv[1]))[:4]
            print(json.dumps({"shape": name, "M": M, "pinned": describe(int(pinned)) if pinned else None,
                              "pinned_us": res.get(describe(int(pinned))) if pinned else None,
                              "best4": best}), flush=True)
        del wts


if __name__ == "__main__":
    main()
