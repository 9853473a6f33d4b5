"""Micro-benchmark: per-kernel cost of tiny launches, eager vs hipGraph replay."""
import json
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402


def timed(fn, n):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n  # us


def main():
    dev = torch.device("cuda")
    B = 1
    ids = torch.zeros(B, dtype=torch.int32, device=dev)
    pos = torch.zeros(B, dtype=torch.int32, device=dev)
    ctx = torch.ones(B, dtype=torch.int32, device=dev)
    slots = torch.zeros(B, dtype=torch.int32, device=dev)
    bt = torch.zeros(B, 4096, dtype=torch.int32, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)

    def tiny():
        ops.advance(ids, pos, ctx, slots, bt, None, step)

    out = {}
    for _ in range(100):
        tiny()
    out["eager_tiny_us"] = timed(tiny, 2000)
    N = 200
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tiny()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(N):
            tiny()
    pos.zero_()
    out["graph_tiny_per_kernel_us"] = timed(g.replay, 20) / N
    # a graph of 200 skinny GEMMs (4096x4096, M=1): per-kernel time vs byte time
    W = torch.randn(4096 // 16, 4096 // 32, 64, 8, device=dev).to(torch.bfloat16)
    Ws = [W.clone() for _ in range(8)]
    x = torch.randn(1, 4096, device=dev).to(torch.bfloat16)
    y = torch.zeros(1, 4096, device=dev, dtype=torch.bfloat16)

    def gemms():
        for i in range(N):
            ops.skinny_gemm(Ws[i % 8], x, ops.EPI_STORE, out=y)
    gemms()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        gemms()
    t = timed(g2.replay, 10) / N
    out["graph_gemv_4096x4096_us"] = t
    out["graph_gemv_4096x4096_TBps"] = 4096 * 4096 * 2 / (t * 1e-6) / 1e12
    W2 = torch.randn(28672 // 16, 4096 // 32, 64, 8, device=dev).to(torch.bfloat16)
    a2 = torch.zeros(1, 14336, device=dev, dtype=torch.bfloat16)
    t2 = timed(lambda: ops.skinny_gemm(W2, x, ops.EPI_SILU, norm=True, out=a2), 200)
    out["eager_gateup_us"] = t2
    out["eager_gateup_TBps"] = 28672 * 4096 * 2 / (t2 * 1e-6) / 1e12
    print(json.dumps(out))


if __name__ == "__main__":
    main()
