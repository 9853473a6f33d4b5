"""TTFT anatomy for one suggest-reply prompt: wall time of Engine.prefill (host
prep + all layers + LM head + first-token sync) vs GPU time, for profiling
under rocprofv3 (`--kernel-trace --stats`) to get the per-kernel split."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.tokenizer import SAMPLE_MESSAGES, get_tokenizer, suggest_prompt  # noqa: E402
from p2p_llm_chat_go_amd.models.config import get_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--peers", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--message", type=int, default=0, help="SAMPLE_MESSAGES index (bench.py: 4)")
    ap.add_argument("--pages", type=int, default=1, help="KV pages per sequence (bench.py: 2)")
    ap.add_argument("--generate", action="store_true",
                    help="also report Engine.generate's own TTFT (64 new tokens)")
    a = ap.parse_args()
    cfg = get_config(a.model)
    tok = get_tokenizer(cfg)
    eng = Engine(cfg, device="cuda", kv_pages=256, max_batch=max(8, a.peers))
    eng.warmup((a.peers,), ctx=128)
    prompts = [tok.chat_ids(suggest_prompt(SAMPLE_MESSAGES[(a.message + i) % len(SAMPLE_MESSAGES)]))
               for i in range(a.peers)]
    pages = [eng.kv.allocator.alloc(a.pages) for _ in prompts]
    for _ in range(3):
        eng.prefill(prompts, pages).cpu()
    torch.cuda.synchronize()
    walls, gpus, enq = [], [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.iters):
        t0 = time.perf_counter()
        e0.record()
        first = eng.prefill(prompts, pages)
        e1.record()
        enq.append((time.perf_counter() - t0) * 1e3)  # host: every launch enqueued
        first.cpu()
        walls.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        gpus.append(e0.elapsed_time(e1))
    walls.sort()
    gpus.sort()
    enq.sort()
    gen = {}
    if a.generate:
        # the prefill again, each time right after a 63-step decode-graph replay (as inside
        # Engine.generate): does alternating graphs cost host or GPU time?
        assert all(a.pages * 64 >= len(p) + 64 for p in prompts), "--generate needs --pages 2"
        g = eng.decode_graph(len(prompts), len(prompts[0]) + 64)
        aw, ag, ae = [], [], []
        for _ in range(a.iters):
            g.state.load([1] * len(prompts), [len(p) for p in prompts], pages)
            g.replay(63)
            g.state.hist[:1, :1].cpu()
            t0 = time.perf_counter()
            e0.record()
            first = eng.prefill(prompts, pages)
            e1.record()
            ae.append((time.perf_counter() - t0) * 1e3)
            first.cpu()
            aw.append((time.perf_counter() - t0) * 1e3)
            torch.cuda.synchronize()
            ag.append(e0.elapsed_time(e1))
        for v in (aw, ag, ae):
            v.sort()
        gen = {"after_decode_wall_ms_p50": round(aw[len(aw) // 2], 3),
               "after_decode_gpu_ms_p50": round(ag[len(ag) // 2], 3),
               "after_decode_enqueue_ms_p50": round(ae[len(ae) // 2], 3)}
        for p in pages:
            eng.kv.allocator.free(p)
        for _ in range(3):
            eng.generate(prompts, 64, stop_on_eos=False)
        tt = sorted(r.ttft_ns / 1e6 for _ in range(a.iters)
                    for r in eng.generate(prompts, 64, stop_on_eos=False))
        gen["generate_ttft_ms_p50"] = round(tt[len(tt) // 2], 3)
    print(json.dumps({"model": cfg.name, "peers": a.peers, "prompt_tokens": len(prompts[0]),
                      "prefill_wall_ms_p50": round(walls[len(walls) // 2], 3),
                      "prefill_gpu_event_ms_p50": round(gpus[len(gpus) // 2], 3),
                      # host time to enqueue the whole prefill (launch-bound when close
                      # to the wall time: the GPU then waits on the host)
                      "prefill_host_enqueue_ms_p50": round(enq[len(enq) // 2], 3),
                      "prefill_graph": bool(getattr(eng, "prefill_graphs_enabled", False)),
                      **gen,
                      "tuning": {"%s@M%d" % k: "%s %.1fus" % v for k, v in eng.tuning.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
