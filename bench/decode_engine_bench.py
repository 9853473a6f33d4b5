"""Persistent decode engine vs the per-layer launches: one decode step of llama3.1-8B (all
32 layers, random-init bf16, context 108) captured in a hipGraph each way and replayed;
--trace adds the engine's per-phase wall-clock stamps (csrc/experimental/decode_engine.hip TR):
per layer, the median / max over workgroups of each phase's duration.

  python bench/decode_engine_bench.py [--rows 1] [--ctx 108] [--iters 200] [--trace]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.models.config import get_config  # noqa: E402
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

PHASES = ["Q sweep", "Q qkv", "A attn", "O sweep", "O proj", "U sweep", "U gate_up", "D sweep",
          "D down"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--ctx", type=int, default=108)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--tp8-shard", action="store_true",
                    help="a TP=1 model with the per-rank shapes of llama3.1-70B at TP=8 (8 q + 1 "
                         "kv heads, 3584 ffn columns, 16032-column vocab shard, 80 layers): the "
                         "persistent engine vs the launches at the shard's shapes, collectives "
                         "excluded on both sides (VERDICT r4 next-round item 2)")
    ap.add_argument("--ffn", type=int, default=0, help="override the ffn width (shape probes)")
    a = ap.parse_args()
    cfg = get_config(a.model)
    if a.tp8_shard:
        cfg = get_config("llama3.1-70b")
        cfg = cfg.replace(name="llama3.1-70b-tp8-shard", n_heads=cfg.n_heads // 8, n_kv_heads=1,
                          ffn=cfg.ffn // 8, vocab=cfg.vocab // 8)
    if a.ffn:
        cfg = cfg.replace(ffn=a.ffn)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    eng = Engine(cfg, device="cuda", seed=3, kv_pages=64, max_batch=8)
    m = eng.model
    R, dev = a.rows, "cuda"
    pages = [eng.kv.allocator.alloc(4) for _ in range(R)]
    ids = torch.full((R,), 1000, dtype=torch.int32, device=dev)
    pos = torch.full((R,), a.ctx - 1, dtype=torch.int32, device=dev)
    slots = torch.tensor([p[(a.ctx - 1) // 64] * 64 + (a.ctx - 1) % 64 for p in pages],
                         dtype=torch.int32, device=dev)
    bt = torch.tensor(pages, dtype=torch.int32, device=dev)
    ctx = torch.full((R,), a.ctx, dtype=torch.int32, device=dev)
    ws = m.new_workspace(R, 256)
    out = {"model": cfg.name, "layers": cfg.n_layers, "rows": R, "ctx": a.ctx}
    for mode in (False, True):
        m.decode_engine = mode
        for _ in range(3):
            m.forward(ws, ids, pos, slots, bt, None, ctx, R, 256, greedy=True)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m.forward(ws, ids, pos, slots, bt, None, ctx, R, 256, greedy=True)
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.iters * 1e6
        m.check_faults(ws)
        out["engine_us" if mode else "layers_us"] = round(us, 1)
    out["engine_ran"] = m._de is not None
    if a.trace and m._de is not None:
        L = _lib.experimental()  # the engine lives in the experimental library
        nb = L.p2p_decode_engine_grid(cfg.hidden, m.nq, m.nkv)
        tr = torch.zeros(nb * cfg.n_layers * 10, dtype=torch.int64, device=dev)
        L.p2p_decode_engine_trace(tr.data_ptr())
        m.decode_engine = True
        m.forward(ws, ids, pos, slots, bt, None, ctx, R, 256, greedy=True)
        torch.cuda.synchronize()
        L.p2p_decode_engine_trace(None)
        t = tr.view(nb, cfg.n_layers, 10).double().cpu() * 0.01  # 100 MHz ticks -> us
        d = t[:, :, 1:] - t[:, :, :-1]  # [nb, L, 9]
        mid = d[:, 1:-1]  # inner layers
        out["phase_us_median"] = {p: round(float(mid[:, :, i].median()), 2) for i, p in enumerate(PHASES)}
        out["phase_us_max"] = {p: round(float(mid[:, :, i].max(0).values.mean()), 2)
                               for i, p in enumerate(PHASES)}
        lay = t[:, 2:, 0] - t[:, 1:-1, 0]
        out["layer_us_median"] = round(float(lay.median()), 2)
        out["layer_us_max"] = round(float(lay.max(0).values.mean()), 2)
        # attention workgroups only
        n_att = R * m.nkv
        out["attn_us"] = round(float(d[nb - n_att:, 1:-1, 2].mean()), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
