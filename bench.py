#!/usr/bin/env python3
"""Headline benchmark: suggest-reply tokens/s + p50 TTFT (BASELINE.json).

One *step* = one complete suggest-reply per peer: the reference co-pilot
prompt (`web/streamlit_app.py:93`) for a synthetic incoming chat message,
wrapped in the llama3.1 chat template (~50 tokens), prefilled, then
``--new-tokens`` greedy tokens decoded (EOS ignored so every step does the same
work).  Model: llama3.1-8B, bf16, random-init weights (no checkpoints on the
box), TP=1 -- one engine replica per GPU (``dp{N}``, weak scaling: each GPU
serves ``--peers`` concurrent peers, batched decode).

``value`` = generated tokens/s summed over all GPUs, measured over K steps
bracketed by barrier + synchronize on every rank, MAX elapsed over ranks.
TTFT p50 is over every request of the timed steps.  tokens/s counts the
whole reply (prefill time included), so it is the user-visible rate.

Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.tokenizer import (SAMPLE_MESSAGES, get_tokenizer,  # noqa: E402
                                                  suggest_prompt)
from p2p_llm_chat_go_amd.models.config import get_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--peers", type=int, default=1, help="concurrent peers per GPU (batched decode)")
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree (ranks per engine replica, RCCL over xGMI)")
    ap.add_argument("--weights", choices=("bf16", "fp8"), default="bf16",
                    help="weight storage of the dense projections (fp8: weight-only e4m3, "
                         "bf16 compute; opt-in -- the headline number is bf16)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = get_config(a.model)
    tok = get_tokenizer(cfg)
    tp = max(1, a.tp)
    assert world % tp == 0, "world size must be a multiple of --tp"
    replica, tp_rank = rank // tp, rank % tp
    comm = None
    if tp > 1:
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        groups = [dist.new_group(list(range(g * tp, (g + 1) * tp))) for g in range(world // tp)]
        comm = TPComm(groups[replica])
    prompts = []
    for p in range(a.peers):
        msg = SAMPLE_MESSAGES[(replica * a.peers + p) % len(SAMPLE_MESSAGES)]
        prompts.append(tok.chat_ids(suggest_prompt(msg)))
    need_pages = sum((len(p) + a.new_tokens + 63) // 64 for p in prompts) + 8
    eng = Engine(cfg, device=dev, seed=1234 + replica, kv_pages=max(need_pages, 64),
                 max_prefill_tokens=1024, max_batch=max(a.peers, 1), use_graph=not a.no_graph,
                 comm=comm, tp_rank=tp_rank, tp_size=tp, weight_dtype=a.weights)
    eng.warmup((a.peers,), ctx=max(len(p) for p in prompts) + a.new_tokens)

    for _ in range(a.warmup):
        eng.generate(prompts, a.new_tokens, stop_on_eos=False)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    ttfts, toks = [], 0
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = eng.generate(prompts, a.new_tokens, stop_on_eos=False)
        for r in res:
            ttfts.append(r.ttft_ns / 1e6)
            if tp_rank == 0:  # a TP group produces each token once
                toks += r.eval_count
    barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed, float(toks)], dtype=torch.float64, device=dev)
    all_ttft = ttfts
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(mx[1:2], op=dist.ReduceOp.SUM)
        t = mx
        gathered = [None] * world
        dist.all_gather_object(gathered, ttfts)
        all_ttft = [x for g in gathered for x in g]
    elapsed, total_toks = float(t[0]), float(t[1])
    if rank == 0:
        value = total_toks / elapsed
        prompt_len = len(prompts[0])
        out = {
            "metric": "suggest-reply tokens/sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic chat prompts (reference co-pilot template, llama3.1 chat format); "
                    "random-init weights",
            "config": {"model": cfg.name, "global_batch": world * a.peers,
                       "seq_len": prompt_len + a.new_tokens, "prompt_tokens": prompt_len,
                       "new_tokens": a.new_tokens,
                       "parallelism": ("dp%d" % (world // tp)) + ("-tp%d" % tp if tp > 1 else ""),
                       "tp": tp,
                       "peers_per_gpu": a.peers, "hipgraph_decode": not a.no_graph,
                       "weights": a.weights},
            "ttft_p50_ms": round(statistics.median(all_ttft), 3),
            "ttft_p99_ms": round(sorted(all_ttft)[min(len(all_ttft) - 1,
                                                      int(0.99 * len(all_ttft)))], 3),
            "per_gpu_tokens_per_sec": round(value / world, 2),
            "gemm_autotune": {"%s@M%d" % k: "%s %.1fus" % v
                              for k, v in getattr(eng, "tuning", {}).items()},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
