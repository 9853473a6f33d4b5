"""Does the skinny GEMM's activation access pattern bound it at prompt-sized M?  Per
llama3.1-8B projection shape: the best skinny launch on row-major X against the same
launches on a fragment-major copy of X (ops.gemm.pack_frag, launch-code bit AFRAG_FLAG:
every A-fragment load 1 KiB contiguous instead of 16 half lines), plus the pack kernel
itself.  32 distinct cold weights per shape, graph-replayed.

python bench/afrag_probe.py [M ...]   (one JSON line per (M, projection))"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _configs, _graph_time, describe  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402

SHAPES = (("qkv", 6144, 4096, G.EPI_STORE, True), ("o_proj", 4096, 4096, G.EPI_RESID, False),
          ("gate_up", 28672, 4096, G.EPI_SILU, True), ("down", 4096, 14336, G.EPI_RESID, False))


def main():
    Ms = [int(m) for m in sys.argv[1:]] or [8, 44, 64]
    for name, N, K, epi, norm in SHAPES:
        wts = [ops.tile_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
               for _ in range(32)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            xp = G.pack_frag(x)
            n_out = N // 2 if epi == G.EPI_SILU else N
            out = torch.zeros(M, n_out, device="cuda", dtype=torch.bfloat16)
            row = {"M": M, "gemm": name, "N": N, "K": K}
            for tag, xin, flag in (("rowmajor", x, 0), ("afrag", xp[:M], G.AFRAG_FLAG)):
                best = None
                for code in _configs(K, M, False, midm=False):
                    t = _graph_time(lambda: [ops.skinny_gemm(w, xin, epi, norm=norm, out=out,
                                                             waves=code | flag, x_packed=bool(flag))
                                             for w in wts]) * 1000 / 32
                    if best is None or t < best[0]:
                        best = (t, describe(code))
                row[tag] = "%s %.2fus" % (best[1], best[0])
            t = _graph_time(lambda: [G.pack_frag(x, out=xp) for _ in range(32)]) * 1000 / 32
            row["pack_us"] = round(t, 2)
            # numerics: the fragment-major launch equals the row-major one
            a = torch.zeros(M, n_out, device="cuda", dtype=torch.bfloat16)
            b = torch.zeros(M, n_out, device="cuda", dtype=torch.bfloat16)
            ops.skinny_gemm(wts[0], x, epi, norm=norm, out=a, waves=4)
            ops.skinny_gemm(wts[0], xp[:M], epi, norm=norm, out=b, waves=4 | G.AFRAG_FLAG,
                            x_packed=True)
            row["max_diff"] = float((a.float() - b.float()).abs().max())
            print(json.dumps(row), flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
