"""Where the wide mid-M GEMM spends a prompt-sized launch (round-5 TTFT work).

Runs the stamped probe build of ``csrc/kernels/wide_gemm.hip`` (``csrc/experimental/
wide_stamp.hip``, per-block ``wall_clock64`` stamps at the phase boundaries) on the four
8B projections at a 48-row prompt chunk, cold weights (a fresh copy per launch, more
bytes than the Infinity Cache holds), and prints per-phase quantiles over the blocks:

  skew   entry - first block's entry          (dispatch spread)
  first  first chunk landed - entry           (HBM latency + activation DMA)
  stream main loop done - first chunk         (the weight stream)
  drain  slabs written through - loop done    (split-K only)
  meet   every slice arrived - slabs drained  (split-K only: arrival skew + ticket)
  epi    stores done - slices met             (reduction loads + epilogue)
  end    last block's end - first entry       (the kernel's span on the GPU)

python -m p2p_llm_chat_go_amd._build --only experimental && python bench/wide_stamp_probe.py
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

TICK_US = 0.01  # wall_clock64: 100 MHz

SHAPES = {  # name: (N, K, epi, norm)
    "qkv": (6144, 4096, ops.EPI_STORE, True),
    "o_proj": (4096, 4096, ops.EPI_RESID, False),
    "gate_up": (28672, 4096, ops.EPI_SILU, True),
    "down": (4096, 14336, ops.EPI_RESID, False),
}


def q(v, p):
    v = sorted(v)
    return v[min(len(v) - 1, int(p * (len(v) - 1) + 0.5))]


def main():
    M = int(os.environ.get("PROBE_M", "48"))
    splits = [int(s) for s in os.environ.get("PROBE_SPLITS", "0").split(",")]
    names = sys.argv[1:] or list(SHAPES)
    L = _lib.experimental()
    L.p2p_wide_stamp_dispatch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p]
    L.p2p_wide_stamp_dispatch.restype = ctypes.c_int
    L.p2p_wide_stamp_set.argtypes = [ctypes.c_void_p]
    ea = ctypes.create_string_buffer(2048)  # zeroed EpiArgs (no RoPE / MoE / FP8)
    stamps = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    assert L.p2p_wide_stamp_set(stamps.data_ptr()) == 0
    st = torch.cuda.current_stream().cuda_stream
    for name in names:
        N, K, epi, norm = SHAPES[name]
        # PROBE_HOT=1: one copy, replayed back to back (weights served from the Infinity
        # Cache where they fit): the ceiling a run-ahead L3 warm-up could reach
        hot = os.environ.get("PROBE_HOT", "0") == "1"
        copies = 1 if hot else max(2, int(320e6 // (N * K * 2)) + 1)
        wts = [ops.tile_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
               for _ in range(copies)]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        n_out = N // 2 if epi == ops.EPI_SILU else N
        out = torch.randn(M, n_out, device="cuda").to(torch.bfloat16)
        for req in splits:
            rows = []
            ev = []
            for it in range(3 * max(copies, 4)):
                stamps.zero_()
                w = wts[it % copies]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                # PROBE_NW=16: the 16-wave form (dispatch code bit 8)
                code = req | (256 if os.environ.get("PROBE_NW", "8") == "16" else 0)
                err = L.p2p_wide_stamp_dispatch(w.data_ptr(), x.data_ptr(), K, M, K, N, epi, int(norm),
                                                out.data_ptr(), n_out, 1e-5, ctypes.addressof(ea), code, st)
                e1.record()
                assert err == 0, err
                torch.cuda.synchronize()
                if it < max(copies, 4):
                    continue  # warm-up round
                ev.append(e0.elapsed_time(e1) * 1000)
                s = stamps.view(-1, 8).cpu()
                s = s[s[:, 0] != 0]
                rows.append(s)
            nb = rows[0].shape[0]
            ph = {k: [] for k in ("skew", "first", "stream", "drain", "meet", "epi", "end")}
            by_xcd = {k: [[] for _ in range(8)] for k in ("first", "arrive")}
            by_split = [[] for _ in range(16)]
            for s in rows:
                t0 = int(s[:, 0].min())
                for b, r in enumerate(s.tolist()):  # blockIdx b runs on XCD b % 8
                    by_xcd["first"][b % 8].append((r[1] - r[0]) * TICK_US)
                    by_xcd["arrive"][b % 8].append((r[2] - t0) * TICK_US)
                    by_split[int(r[7]) % 16].append((r[2] - t0) * TICK_US)
                ends = [int(v) for v in s[:, 5] if v != 0]
                ph["end"].append((max(ends) - t0) * TICK_US if ends else 0.0)
                for r in s.tolist():
                    ph["skew"].append((r[0] - t0) * TICK_US)
                    ph["first"].append((r[1] - r[0]) * TICK_US)
                    ph["stream"].append((r[2] - r[1]) * TICK_US)
                    if r[3]:  # split-K (r5 granule seam: 3 = granules stored, 4 = polls done;
                        # blocks whose wave 0 finishes no unit stamp neither 4 nor 5)
                        ph["drain"].append((r[3] - r[2]) * TICK_US)
                        if r[4]:
                            ph["meet"].append((r[4] - r[3]) * TICK_US)
                        if r[4] and r[5]:
                            ph["epi"].append((r[5] - r[4]) * TICK_US)
                    elif r[5]:
                        ph["epi"].append((r[5] - r[2]) * TICK_US)
            out_row = {"gemm": name, "hot": hot, "nw": int(os.environ.get("PROBE_NW", "8")), "M": M,
                       "N": N, "K": K, "req_split": req, "blocks": nb,
                       "splitk": int(rows[0][:, 7].max()) + 1,
                       "event_us_p50": round(q(ev, 0.5), 2)}
            for k, v in ph.items():
                if v:
                    out_row[k] = [round(q(v, p), 2) for p in (0.1, 0.5, 0.9, 1.0)]
            for k, v in by_xcd.items():  # per-XCD median / max (straggler placement)
                out_row[k + "_by_xcd"] = [[round(q(x, 0.5), 2), round(q(x, 1.0), 2)] for x in v if x]
            out_row["arrive_by_split"] = [[round(q(x, 0.5), 2), round(q(x, 1.0), 2)] for x in by_split if x]
            print(json.dumps(out_row), flush=True)
        del wts
        torch.cuda.empty_cache()
    L.p2p_wide_stamp_set(None)


if __name__ == "__main__":
    main()
