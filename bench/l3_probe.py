"""Infinity-Cache probe for batch-1 decode GEMVs: the same GEMV with its weights cold
(rotating copies past the 256 MiB L3) vs resident, the prefetch kernel's own rate, and
a GEMV whose NEXT weights are prefetched on a parallel graph branch (does the branch
overlap, and does the consumer then run at L3 speed?)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from kernel_bench import copies, graph_time  # noqa: E402

SHAPES = {"o_proj": (4096, 4096, 8 | (8 << 8)), "qkv": (6144, 4096, 4 | (4 << 8)),
          "down": (4096, 14336, 4 | (8 << 8)), "gate_up": (28672, 4096, 1 | (4 << 8))}


def main():
    side = torch.cuda.Stream()
    for name, (N, K, code) in SHAPES.items():
        W = copies(N, K, nbytes_target=600 << 20)
        x = torch.randn(1, K, device="cuda").to(torch.bfloat16)
        out = torch.zeros(1, N, device="cuda", dtype=torch.bfloat16)
        c = len(W)
        gemv = lambda w: ops.skinny_gemm(w, x, ops.EPI_STORE, out=out, waves=code)  # noqa: E731
        cold = graph_time(lambda i: gemv(W[i % c]))
        hot = graph_time(lambda i: gemv(W[0]))
        res = {"gemv": name, "N": N, "K": K, "MB": round(N * K * 2 / 1e6, 1), "copies": c,
               "cold_us": round(cold, 2), "hot_us": round(hot, 2)}
        for grid in (256, 512, 1024):
            res["prefetch_g%d_us" % grid] = round(graph_time(
                lambda i: ops.l3_prefetch(W[i % c], grid=grid)), 2)

        def branch(i, grid=512):
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                ops.l3_prefetch(W[(i + 1) % c], grid=grid)
            gemv(W[i % c])
            cur.wait_stream(side)

        def serial(i):  # prefetch next, then consume (no overlap possible)
            gemv(W[i % c])
            ops.l3_prefetch(W[(i + 1) % c], grid=512)

        res["branch_us"] = round(graph_time(branch), 2)
        res["serial_us"] = round(graph_time(serial), 2)
        print(json.dumps(res), flush=True)
        del W


if __name__ == "__main__":
    main()
