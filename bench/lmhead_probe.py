"""The batch-1 LM head (llama3.1-8B: 128256 x 4096 bf16, 1.05 GB) against the weight
stream: every skinny launch code with the greedy argmax epilogue (the decode graph's
head), the same codes with the fp32-logits epilogue (sampled requests), and gate_up's
SwiGLU GEMV over 4.5 layers' worth of the same bytes as the stream reference.

Run on the GPU: python bench/lmhead_probe.py   (one JSON line per code)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.autotune import _configs, _graph_time, describe  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402


def main():
    eng = Engine(LLAMA31_8B, device="cuda", kv_pages=64, max_batch=1)
    m = eng.model
    w = m.w
    H = LLAMA31_8B.hidden
    x = torch.randn(1, H, device="cuda").to(torch.bfloat16)
    N, K = G.tiled_shape(w.lm_head)
    keys = ops.new_argmax_keys(1, "cuda")
    logits = torch.empty(1, N, device="cuda", dtype=torch.float32)
    mb = N * K * 2 / 1e6
    F = w.layers[0].gate_up.shape[0] * 16 // 2
    act = torch.zeros(1, F, device="cuda", dtype=torch.bfloat16)
    gu = [lw.gate_up for lw in w.layers[:9]]
    gu_mb = 9 * G.tiled_shape(gu[0])[0] * K * 2 / 1e6
    t = _graph_time(lambda: [ops.skinny_gemm(wt, x, ops.EPI_SILU, norm=True, out=act,
                                             waves=1 | (4 << 8)) for wt in gu], reps=5) * 1000
    print(json.dumps({"ref": "gate_up w1/U4 x9 layers", "MB": round(gu_mb, 1),
                      "us_per_MB_x1000": round(t / gu_mb * 1000, 2),
                      "us_at_lm_head_bytes": round(t / gu_mb * mb, 1),
                      "TBps": round(gu_mb / t, 2)}), flush=True)
    for code in _configs(K, 1):
        ta = _graph_time(lambda: [ops.lm_head_argmax(w.lm_head, x, keys, waves=code)
                                  for _ in range(4)], reps=5) * 1000 / 4
        keys.zero_()
        tf = _graph_time(lambda: [ops.skinny_gemm(w.lm_head, x, ops.EPI_F32, norm=True,
                                                  out=logits, waves=code)
                                  for _ in range(4)], reps=5) * 1000 / 4
        print(json.dumps({"code": describe(code), "MB": round(mb, 1), "argmax_us": round(ta, 1),
                          "f32_us": round(tf, 1), "argmax_TBps": round(mb / ta, 2),
                          "f32_TBps": round(mb / tf, 2)}), flush=True)
    assert ops.tiled_split_fault() == 0


if __name__ == "__main__":
    main()
