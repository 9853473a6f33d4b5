"""Mid-M (prefill chunks of <= 64 rows) projections on the split-K tiled kernel: serial
split-K reduction (the last arriving slice reduces the tile) vs parallel (every slice
finishes 8/splitk of the tile's waves, write-through slabs, no release fence), at
llama3.1-8B shapes with rotating weight copies (cold L3), graph-timed."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops.gemm import set_tiled_min_m, tiled_config, tiled_split_parallel  # noqa: E402
from kernel_bench import copies, graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="*", default=[44, 64])
    a = ap.parse_args()
    H, F = 4096, 14336
    set_tiled_min_m(1)
    for M in a.M:
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        xf = torch.randn(M, F, device="cuda").to(torch.bfloat16)
        h = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
        o = torch.zeros(M, 6144, device="cuda", dtype=torch.bfloat16)
        for name, N, K, fn in [
                ("qkv", 6144, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_STORE, norm=True, out=o)),
                ("o_proj", H, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_RESID, out=h)),
                ("gate_up", 2 * F, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_SILU, norm=True, out=act)),
                ("down", H, F, lambda W: ops.skinny_gemm(W, xf, ops.EPI_RESID, out=h))]:
            Ws = copies(N, K, nbytes_target=600 << 20)
            c = len(Ws)
            res = {"M": M, "gemm": name, "MB": round(N * K * 2 / 1e6, 1)}
            for tile in (4, 5):
                for sk in (1, 2, 4, 8):
                    for par in (0, 1):
                        if sk == 1 and par:
                            continue
                        tiled_config(2, tile, sk)
                        tiled_split_parallel(par)
                        try:
                            t = graph_time(lambda i: fn(Ws[i % c]), n_inner=20)
                        except Exception as e:  # shape does not tile
                            t = float("nan")
                            print(json.dumps({"skip": name, "tile": tile, "err": str(e)[:80]}))
                        res["t%d_s%d%s" % (tile, sk, "p" if par else "")] = round(t, 2)
            best = min((v, k) for k, v in res.items() if k.startswith("t") and v == v)
            res["best"] = best[1]
            print(json.dumps(res), flush=True)
            del Ws
    tiled_config(2, 0, 0)
    tiled_split_parallel(1)
    set_tiled_min_m(65)
    assert ops.tiled_split_fault() == 0


if __name__ == "__main__":
    main()
