"""Weight-stream probe (csrc/experimental/stream_probe.hip): the time a once-read weight
matrix of each llama3.1-8B projection size takes to stream through a grid of a given shape
(blocks x waves per block x loads in flight per wave), with no math -- the floor of a
prompt-sized GEMM on that grid.  32 rotating copies per size (one per layer, like the
model: cold in the Infinity Cache), graph-replayed, us per launch including the dependent
boundary.

Run on the GPU: python bench/stream_probe.py   (one JSON line per (size, config))"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402

# llama3.1-8B projections: KiB per matrix = N * K * 2 / 1024
SIZES = {"qkv": 6144 * 4096 * 2 // 1024, "o_proj": 4096 * 4096 * 2 // 1024,
         "down": 4096 * 14336 * 2 // 1024, "gate_up": 28672 * 4096 * 2 // 1024}


def configs(kib):
    """(blocks, threads) x U with blocks * waves * steps == kib exactly."""
    out = []
    for blocks, threads in ((240, 512), (256, 512), (384, 256), (512, 512), (768, 256),
                            (1024, 256), (1536, 64), (512, 256), (256, 1024), (128, 512)):
        waves = blocks * threads // 64
        if kib % waves:
            continue
        steps = kib // waves
        for u in (4, 8, 16):
            if steps >= u:
                out.append((blocks, threads, steps, u))
    return out


def main():
    L = _lib.experimental()
    fn = L.p2p_stream_probe
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda")
    out = torch.zeros(1, device=dev)
    only = sys.argv[1:] or list(SIZES)
    modes = [int(m) for m in os.environ.get("STREAM_MODES", "0,1").split(",")]
    for name in only:
        kib = SIZES[name]
        bufs = [torch.randn(kib * 512, device=dev).to(torch.bfloat16) for _ in range(32)]
        for blocks, threads, steps, u in configs(kib):
            for mode in modes:
                if mode == 1 and (threads // 64) * u > 160:
                    continue

                def f(i):
                    _lib.check(fn(mode, u, blocks, threads, bufs[i % 32].data_ptr(), steps,
                                  out.data_ptr(), _lib.stream_ptr(dev)), "stream_probe")
                t = graph_time(f, n_inner=32)
                print(json.dumps({"gemm": name, "MB": round(kib * 1024 / 1e6, 1), "mode": ("vgpr", "ldsdma")[mode],
                                  "blocks": blocks, "threads": threads, "steps": steps, "U": u,
                                  "us": round(t, 2), "TBps": round(kib * 1024 / t / 1e6, 2)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
