"""Alternating A/B of two prefill GEMM tile configurations on one projection (cold weights:
4 copies, > 900 MB, rotate through the 256 MB Infinity Cache), after a warm-up of both, so
clock ramp and launch order do not favour either.  llama3.1-8B shapes.

Run on the GPU: python bench/tile_ab.py M gemm "v,t,s" "v,t,s" [rounds]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _graph_time  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402
from p2p_llm_chat_go_amd.ops.gemm import tiled_config  # noqa: E402


def main():
    M, gemm = int(sys.argv[1]), sys.argv[2]
    cfgs = [tuple(int(v) for v in a.split(",")) for a in sys.argv[3:5]]
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    H, F = LLAMA31_8B.hidden, LLAMA31_8B.ffn
    shapes = {"gate_up": (2 * F, H, ops.EPI_SILU, True), "qkv": (6144, H, ops.EPI_STORE, True),
              "o_proj": (H, H, ops.EPI_RESID, False), "down": (H, F, ops.EPI_RESID, False)}
    N, K, epi, norm = shapes[gemm]
    ws = [ops.tile_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
          for _ in range(4)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.zeros(M, N // 2 if epi == ops.EPI_SILU else N, device="cuda",
                      dtype=torch.bfloat16)

    def run():
        for w in ws:
            ops.skinny_gemm(w, x, epi, norm=norm, out=out)

    def timed(c):
        tiled_config(*c)
        try:
            return _graph_time(run, reps=5) * 1000 / len(ws)
        finally:
            tiled_config(2, 0, 0)

    for c in cfgs:  # warm-up
        timed(c)
    res = {str(c): [] for c in cfgs}
    for _ in range(rounds):
        for c in cfgs:
            res[str(c)].append(round(timed(c), 1))
    print(json.dumps({"M": M, "gemm": gemm, "us": res}), flush=True)
    assert ops.tiled_split_fault() == 0


if __name__ == "__main__":
    main()
