"""Wide mid-M GEMM (csrc/kernels/wide_gemm.hip) against the other mid-M families at
llama3.1-8B shapes: per projection, the best skinny / midm / tiled launch and the wide
kernel at each K-slice count, all 32 layers' weights (cold, graph-replayed).

Run on the GPU: python bench/wide_bench.py [M ...]   (one JSON line per (M, projection))"""
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


def family(code):
    if code & G.TILED_FLAG:
        return "tiled"
    if code & G.MIDM_FLAG:
        return "midm"
    return "skinny"


def main():
    Ms = [int(m) for m in sys.argv[1:]] or [8, 44, 64]
    splits = [int(s) for s in os.environ.get("WIDE_SPLITS", "0,1,2,3,4,5,6,8,12,16").split(",")]
    others = os.environ.get("WIDE_OTHERS", "1") == "1"
    eng = Engine(LLAMA31_8B, device="cuda", kv_pages=64, max_batch=1)
    m = eng.model
    layers = m.w.layers
    H, nq, nkv = LLAMA31_8B.hidden, m.nq, m.nkv
    kc, vc = m.kv.layer(0)
    for M in Ms:
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        h = torch.zeros(M, H, device="cuda", dtype=torch.bfloat16)
        q = torch.randn(M, nq * 128, device="cuda").to(torch.bfloat16)
        pos = torch.zeros(M, device="cuda", dtype=torch.int32)
        slots = torch.arange(M, device="cuda", dtype=torch.int32) % 64
        F = layers[0].gate_up.shape[0] * 16 // 2
        act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
        xf = torch.randn(M, F, device="cuda").to(torch.bfloat16)
        jobs = [("qkv_rope", [lw.qkv for lw in layers], G.EPI_QKV_ROPE,
                 lambda wt, c: ops.qkv_rope_gemm(wt, x, pos, slots, m.rope, nq, nkv, q, kc, vc,
                                                 waves=c)),
                ("o_proj", [lw.o for lw in layers], G.EPI_RESID,
                 lambda wt, c: ops.skinny_gemm(wt, q, ops.EPI_RESID, out=h, waves=c)),
                ("gate_up", [lw.gate_up for lw in layers], G.EPI_SILU,
                 lambda wt, c: ops.skinny_gemm(wt, x, ops.EPI_SILU, norm=True, out=act, waves=c)),
                ("down", [lw.down for lw in layers], G.EPI_RESID,
                 lambda wt, c: ops.skinny_gemm(wt, xf, ops.EPI_RESID, out=h, waves=c))]
        for name, wts, epi, fn in jobs:
            N, K = G.tiled_shape(wts[0])
            row = {"M": M, "gemm": name, "MB": round(N * K * 2 / 1e6, 1)}
            if others:
                best = {}
                for code in _configs(K, M, G.tiled_ok(N, K, epi) and M > 16, midm=True):
                    t = _graph_time(lambda: [fn(wt, code) for wt in wts]) * 1000 / len(wts)
                    f = family(code)
                    if f not in best or t < best[f][0]:
                        best[f] = (t, describe(code))
                row.update({f: "%s %.1fus" % (d, t) for f, (t, d) in sorted(best.items())})
            from p2p_llm_chat_go_amd.ops import _lib
            for res in (1, 0) if os.environ.get("WIDE_AB_RES", "0") == "1" else (1,):
                _lib.lib().p2p_wide_resident(res)
                for nw in [int(v) for v in os.environ.get("WIDE_NWS", "8,16").split(",")]:
                    for s in splits:
                        code = G.WIDE_FLAG | (s << 8) | (G.WIDE16 if nw == 16 else 0)
                        t = _graph_time(lambda: [fn(wt, code) for wt in wts]) * 1000 / len(wts)
                        row["wide%s%s_s%s" % ("16" if nw == 16 else "", "" if res else "ring",
                                             s if s else "auto")] = round(t, 2)
            _lib.lib().p2p_wide_resident(1)
            assert ops.tiled_split_fault() == 0
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
