"""Per-launch cost of a dependent kernel boundary vs workgroup shape and an in-kernel
chain of dependent loads (graph-replayed, 32 launches per graph).  Context: the batch-1
decode attention launch (8 x 1024 threads, ~75 KB LDS) costs ~6.4 us of which its waves
live ~1.65 us."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import graph_time  # noqa: E402


def main():
    L = _lib.experimental()  # csrc/experimental (built with --only experimental)
    fn = L.p2p_launch_probe
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p]
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda")
    n = 1 << 24  # 64 MB of random pointers: chains start at a different place per launch
    chain = torch.randperm(n, device=dev).to(torch.int32)
    out = torch.zeros(1, device=dev)
    st = _lib.stream_ptr(dev)
    for blocks, threads, lds in ((8, 1024, 76 * 1024), (8, 1024, 0), (8, 256, 0), (8, 512, 40 * 1024),
                                 (32, 256, 0), (256, 256, 0), (256, 512, 96 * 1024), (1024, 256, 0)):
        for depth in (0, 1, 2, 3):
            def f(i):
                _lib.check(fn(blocks, threads, lds, chain.data_ptr(), depth, (i * 7919) % n,
                              out.data_ptr(), _lib.stream_ptr(dev)), "launch_probe")
            t = graph_time(f, n_inner=32)
            print(json.dumps({"blocks": blocks, "threads": threads, "lds_kb": lds // 1024,
                              "dep_loads": depth, "us_per_launch": round(t, 2)}), flush=True)
    del st


if __name__ == "__main__":
    main()
