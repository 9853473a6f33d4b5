"""PMC target (scripts/gpu_run.sh STEPS=pmc): the four llama3.1-8B projections of one layer at
the suggest-reply prompt size (48-row bucket, 44 rows) on the wide mid-M kernel (auto split,
the autotuner's family at 48 rows), the same weights at batch 1 on the skinny GEMV (the decode
pick), and the pure weight stream of the same bytes (csrc/experimental/stream_probe.hip, 256 x
512 threads, 8 loads in flight) -- eager launches, 8 rotating weight copies per projection (cold
in the Infinity Cache), so rocprofv3 --pmc rows compare the three per projection.

Kernel-name key: wide_gemm_kernel = 48-row prompt, skinny_gemm_kernel = batch 1,
stream_vgpr_kernel = the stream floor."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.models.config import LLAMA31_8B, rope_table  # noqa: E402
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402
from p2p_llm_chat_go_amd.ops import gemm as G  # noqa: E402

M = int(os.environ.get("PMC_M", "44"))
H, F, nq, nkv = 4096, 14336, 32, 8
dev = torch.device("cuda")


def wts(n, k):
    return [(torch.randn(n // 16, k // 32, 64, 8, device=dev) * 0.02).to(torch.bfloat16) for _ in range(8)]


def main():
    L = _lib.experimental()
    sp = L.p2p_stream_probe
    sp.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1, device=dev)
    cs = rope_table(LLAMA31_8B, max_pos=256).to(dev)
    kc = torch.zeros(4, nkv, 64, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    for rows, code, tag in ((M, G.WIDE_FLAG, "wide"), (1, 0, "skinny")):
        x = torch.randn(rows, H, device=dev).to(torch.bfloat16)
        xf = torch.randn(rows, F, device=dev).to(torch.bfloat16)
        q = torch.zeros(rows, nq * 128, device=dev, dtype=torch.bfloat16)
        h = torch.zeros(rows, H, device=dev, dtype=torch.bfloat16)
        act = torch.zeros(rows, F, device=dev, dtype=torch.bfloat16)
        pos = torch.arange(rows, device=dev, dtype=torch.int32)
        slots = torch.arange(rows, device=dev, dtype=torch.int32)
        for name, n, k in (("qkv", (nq + 2 * nkv) * 128, H), ("o_proj", H, H), ("gate_up", 2 * F, H), ("down", H, F)):
            ws = wts(n, k)
            for i in range(16):
                wt = ws[i % 8]
                if name == "qkv":
                    ops.qkv_rope_gemm(wt, x, pos, slots, cs, nq, nkv, q, kc, vc, waves=code)
                elif name == "o_proj":
                    ops.skinny_gemm(wt, q, ops.EPI_RESID, out=h, waves=code)
                elif name == "gate_up":
                    ops.skinny_gemm(wt, x, ops.EPI_SILU, norm=True, out=act, waves=code)
                else:
                    ops.skinny_gemm(wt, xf, ops.EPI_RESID, out=h, waves=code)
            if tag == "wide":  # the stream floor of the same bytes, once per projection size
                kib = n * k * 2 // 1024
                for i in range(16):
                    _lib.check(sp(0, 8, 256, 512, ws[i % 8].data_ptr(), kib // 2048, sink.data_ptr(),
                                  _lib.stream_ptr(dev)), "stream_probe")
            torch.cuda.synchronize()
            del ws
    assert ops.tiled_split_fault() == 0
    print("ok")


if __name__ == "__main__":
    main()
