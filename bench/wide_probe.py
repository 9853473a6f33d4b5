"""Fixed-cost probe of the mid-M GEMM families: time vs K at a fixed N (qkv-like N=6144),
so the intercept (launch + prologue + reduction + epilogue) separates from the per-k
streaming slope.  32 distinct cold weights per point, graph-replayed.

python bench/wide_probe.py [M ...]   (one JSON line per (M, K))"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _configs, _graph_time, describe  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402


def main():
    Ms = [int(m) for m in sys.argv[1:]] or [8, 44]
    N = int(os.environ.get("PROBE_N", "6144"))
    for K in (256, 512, 1024, 2048, 4096):
        wts = [ops.tile_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
               for _ in range(32)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row = {"M": M, "K": K, "N": N, "MB": round(N * K * 2 / 1e6, 2)}
            best = None
            for code in _configs(K, M, False, midm=False):
                t = _graph_time(lambda: [ops.skinny_gemm(w, x, ops.EPI_STORE, out=out, waves=code)
                                         for w in wts]) * 1000 / 32
                if best is None or t < best[0]:
                    best = (t, describe(code))
            row["skinny"] = "%s %.2fus" % (best[1], best[0])
            for s in (1, 2, 4, 8):
                if (K // 256) < s:
                    continue
                code = G.WIDE_FLAG | (s << 8)
                t = _graph_time(lambda: [ops.skinny_gemm(w, x, ops.EPI_STORE, out=out, waves=code)
                                         for w in wts]) * 1000 / 32
                row["wide_s%d" % s] = round(t, 2)
            print(json.dumps(row), flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
