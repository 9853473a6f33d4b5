"""Prefill GEMM comparison at llama3.1-8B shapes: register-staged v1 vs the
8-wave LDS-DMA v2 kernel (each tile) vs hipBLASLt (torch.matmul, plain GEMM
without the fused epilogue).  One JSON line per (M, projection, variant)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops.gemm import set_tiled_min_m, tiled_config  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="*", default=[36, 64, 288, 512, 2048, 8192])
    ap.add_argument("--deep", action="store_true",
                    help="A/B the deep LDS pipeline: each variant with shallow stages (deep=0) "
                         "and with the default rule (deep=1)")
    ap.add_argument("--deep-modes", type=int, nargs="*", default=[0, 1])
    ap.add_argument("--only", nargs="*", default=None, help="variant names to run")
    ap.add_argument("--no-hipblaslt", action="store_true")
    ap.add_argument("--gemms", nargs="*", default=None, help="projection names to run")
    ap.add_argument("--cold", action="store_true",
                    help="rotate over enough weight copies (> 600 MB) that no launch finds its "
                         "weights in the 256 MB Infinity Cache, as in a model's layer sequence")
    a = ap.parse_args()
    H, F = LLAMA31_8B.hidden, LLAMA31_8B.ffn
    variants = [("v2_auto", (2, 0, 0)), ("v2_256x256_phased", (2, 1, 1)),
                ("v2_256x256_2stage", (2, 1, 1, 0)),
                ("v2_128x256", (2, 2, 1)), ("v2_128x128", (2, 3, 1)),
                ("v2_128x128_s2", (2, 3, 2)), ("v2_128x128_s4", (2, 3, 4)),
                ("v2_320x128", (2, 6, 1)), ("v2_320x128_s2", (2, 6, 2)), ("v2_192x128", (2, 7, 1)),
                ("v2_192x128_s2", (2, 7, 2)), ("v2_192x256", (2, 8, 1)), ("v2_192x256_s2", (2, 8, 2)), ("v2_192x256_auto", (2, 8, 0)), ("v2_256x256_s3", (2, 1, 3, 0)),
                ("v2_256x256_s5", (2, 1, 5, 0)), ("v2_128x256_s2", (2, 2, 2)),
                ("v2_128x256_s3", (2, 2, 3)), ("v2_128x128_s2", (2, 3, 2))]
    L = __import__("p2p_llm_chat_go_amd.ops._lib", fromlist=["lib"]).lib()
    for M in a.M:
        x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        xf = torch.randn(M, F, device="cuda").to(torch.bfloat16)
        h = torch.randn(M, H, device="cuda").to(torch.bfloat16)
        act = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
        o = torch.zeros(M, 6144, device="cuda", dtype=torch.bfloat16)
        for name, N, K, fn in [
            ("qkv", 6144, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_STORE, norm=True, out=o)),
            ("gate_up", 2 * F, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_SILU, norm=True, out=act)),
            ("down", H, F, lambda W: ops.skinny_gemm(W, xf, ops.EPI_RESID, out=h)),
            ("o_proj", H, H, lambda W: ops.skinny_gemm(W, x, ops.EPI_RESID, out=h))]:
            if a.gemms and name not in a.gemms:
                continue
            W = (torch.randn(N // 16, K // 32, 64, 8, device="cuda") * 0.02).to(torch.bfloat16)
            ncp = min(12, 600 * 2**20 // (N * K * 2) + 2) if a.cold else 1
            Ws = [W] + [W.clone() for _ in range(ncp - 1)]
            flops = 2 * M * N * K
            vs = variants
            if M <= 64:  # decode-style skinny kernel vs the split-K tiled kernel
                vs = [("skinny", None), ("v2_auto", (2, 0, 0)), ("v2_64x128", (2, 4, 1)),
                      ("v2_64x128_s2", (2, 4, 2)), ("v2_64x128_s4", (2, 4, 4)),
                      ("v2_64x128_s8", (2, 4, 8)), ("v2_64x256", (2, 5, 1)),
                      ("v2_64x256_s2", (2, 5, 2)), ("v2_128x128_s4", (2, 3, 4))]
            if a.deep:
                vs = [(v + "_deep%d" % d, c, d) for v, c in vs if c is not None
                      for d in a.deep_modes]
            else:
                vs = [(v, c, 1) for v, c in vs]
            if a.only:
                vs = [v for v in vs if v[0].rsplit("_deep", 1)[0] in a.only]
            if name == "gate_up" and 64 < M <= 384:
                vs = [("tall", "tall", 1)] + vs
            for vname, cfg, deep in vs:
                ops.gemm.TALL_SILU = cfg == "tall"
                if cfg == "tall":
                    t = graph_time(lambda i: fn(Ws[i % ncp]), n_inner=10)
                    print(json.dumps({"M": M, "gemm": name, "variant": vname, "us": round(t, 1),
                                      "TFLOPs": round(flops / (t * 1e-6) / 1e12, 1),
                                      "TBps": round(N * K * 2 / (t * 1e-6) / 1e12, 2)}), flush=True)
                    continue
                set_tiled_min_m(65 if cfg is None else 1)
                L.p2p_prefill_deep(deep)
                if cfg is not None:
                    tiled_config(*cfg[:3])
                    L.p2p_prefill_phased(cfg[3] if len(cfg) > 3 else 1)
                t = graph_time(lambda i: fn(Ws[i % ncp]), n_inner=10)
                print(json.dumps({"M": M, "gemm": name, "variant": vname, "us": round(t, 1),
                                  "TFLOPs": round(flops / (t * 1e-6) / 1e12, 1),
                                  "TBps": round(N * K * 2 / (t * 1e-6) / 1e12, 2)}), flush=True)
            set_tiled_min_m(65)
            tiled_config(2, 0, 0)
            L.p2p_prefill_deep(1)
            if a.no_hipblaslt:
                del W, Ws
                continue
            Wbs = [torch.randn(K, N, device="cuda").to(torch.bfloat16) for _ in range(ncp)]
            xin = x if K == H else xf
            t = graph_time(lambda i: torch.matmul(xin, Wbs[i % ncp]), n_inner=10)
            print(json.dumps({"M": M, "gemm": name, "variant": "hipblaslt", "us": round(t, 1),
                              "TFLOPs": round(flops / (t * 1e-6) / 1e12, 1)}), flush=True)
            del W, Ws, Wbs


if __name__ == "__main__":
    main()
