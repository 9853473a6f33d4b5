"""Feasibility probe for a persistent batch-1 decode layer (csrc/experimental/persist_probe.hip):
the 8B layer's weight bytes (qkv 50.3 MB, attention stand-in, o_proj 33.5, gate_up 234.9,
down 117.4) streamed as 5 launches per layer (graph) vs ONE launch for all 32 layers with
grid barriers, with and without an LDS-DMA prefetch of each workgroup's next-phase slice
before the barrier.  Pure data movement; prints us per layer."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402


def main():
    L = _lib.experimental()  # csrc/experimental (built with --only experimental)
    fn = L.p2p_persist_probe
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_void_p]
    fn.restype = ctypes.c_int
    sizes = [50_331_648, 0, 33_554_432, 234_881_024, 117_440_512]
    bufs = [torch.empty(max(s, 16) // 2, dtype=torch.bfloat16, device="cuda").normal_() for s in sizes]
    ptrs = (ctypes.c_void_p * 5)(*[b.data_ptr() for b in bufs])
    nbytes = (ctypes.c_longlong * 5)(*sizes)
    bar = torch.zeros(16, dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    layers = 32
    attn_iters = int(os.environ.get("ATTN_ITERS", "300"))
    s = torch.cuda.current_stream().cuda_stream

    def run(mode, grid, pf):
        return fn(mode, ptrs, nbytes, layers, grid, pf, attn_iters, bar.data_ptr(), err.data_ptr(),
                  sink.data_ptr(), s)

    def timeit(mode, grid, pf, graph):
        assert run(mode, grid, pf) == 0
        torch.cuda.synchronize()
        if graph:
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                with torch.cuda.graph(g, stream=st):
                    fn(mode, ptrs, nbytes, layers, grid, pf, attn_iters, bar.data_ptr(),
                       err.data_ptr(), sink.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if graph:
                g.replay()
            else:
                run(mode, grid, pf)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1000 / layers)
        return round(best, 2)

    res = {"cus": cus, "layer_MB": round(sum(sizes) / 1e6, 1),
           "ideal_us_at_6.4TBps": round(sum(sizes) / 6.4e12 * 1e6, 1)}
    # attention stand-in alone (8 workgroups of busy work)
    res["launches_per_phase_us"] = timeit(0, cus, 0, True)
    res["launches_per_phase_grid2x_us"] = timeit(0, 2 * cus, 0, True)
    for pf in (0, 32 << 10, 64 << 10, 128 << 10):
        res["persistent_pf%dK_us" % (pf >> 10)] = timeit(1, cus, pf, False)
    res["barrier_timeouts"] = int(err.item())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
