"""Is the batch-1 gate_up GEMV tail-bound?  SwiGLU pairs give 896 blocks (3.5 per CU on
256 CUs: half the CUs stream a quarter more); storing gate and up as separate fp32
columns gives 1792 blocks (7 per CU).  Rotating weight copies (cold L3), graph-timed."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from kernel_bench import copies, graph_time  # noqa: E402


def main():
    H, F = 4096, 14336
    W = copies(2 * F, H, nbytes_target=600 << 20)
    c = len(W)
    x = torch.randn(1, H, device="cuda").to(torch.bfloat16)
    act = torch.zeros(1, F, device="cuda", dtype=torch.bfloat16)
    g32 = torch.zeros(1, 2 * F, device="cuda", dtype=torch.float32)
    for w in (1, 2, 4):
        for u in (4, 8):
            code = w | (u << 8)
            t1 = graph_time(lambda i: ops.skinny_gemm(W[i % c], x, ops.EPI_SILU, norm=True, out=act,
                                                      waves=code))
            t2 = graph_time(lambda i: ops.skinny_gemm(W[i % c], x, ops.EPI_F32, norm=True, out=g32,
                                                      waves=code))
            print(json.dumps({"waves": w, "U": u, "silu_pairs_us": round(t1, 2),
                              "f32_split_us": round(t2, 2)}), flush=True)
    K2 = 6144
    Wq = copies(K2, H, nbytes_target=600 << 20)
    cq = len(Wq)
    o = torch.zeros(1, K2, device="cuda", dtype=torch.bfloat16)
    for w in (1, 2, 4, 8):
        t = graph_time(lambda i: ops.skinny_gemm(Wq[i % cq], x, ops.EPI_STORE, norm=True, out=o,
                                                 waves=w | (4 << 8)))
        print(json.dumps({"qkv_like_N": K2, "waves": w, "us": round(t, 2)}), flush=True)


if __name__ == "__main__":
    main()
