#!/usr/bin/env python3
"""Headline benchmark: suggest-reply tokens/s + p50 TTFT (BASELINE.json).

One *step* = one complete suggest-reply per peer: the reference co-pilot
prompt (`web/streamlit_app.py:93`) for a synthetic incoming chat message,
wrapped in the llama3.1 chat template, prefilled, then ``--new-tokens`` greedy
tokens decoded (EOS ignored so every step does the same work).  The default
message is the median-length one of the sample set (44 prompt tokens, inside
SURVEY §2A.1's 40-60-token workload).  Model: llama3.1-8B, bf16, random-init
weights (no checkpoints on the box).

Parallel layouts (one process per GPU, RCCL over xGMI between them):
  * default ``dp{N}``: one engine replica per GPU, each serving ``--peers``
    concurrent peers (batched decode) -- weak scaling (BASELINE configs 2, 4).
  * ``--tp T``: replicas of T ranks, Megatron-sharded (``--model llama3.1-70b
    --tp 8`` is BASELINE config 3).
  * ``--ep E`` (MoE models): experts sharded over E ranks (config 5).

``value`` = generated tokens/s summed over all replicas, measured over K steps
bracketed by barrier + synchronize on every rank, MAX elapsed over ranks.
TTFT p50 is over every request of the timed steps.  tokens/s counts the whole
reply (prefill time included), so it is the user-visible rate.

Launch: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (spawns the N
rank processes itself, before any GPU call), or under
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
bench.py --gpus N`` (the driver's form).  ``--device cpu`` runs the same
multi-rank path over gloo on the CPU (tests, tiny models).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# median-length first (44 tokens with the synthetic tokenizer), then the rest
MESSAGE_ORDER = (4, 1, 2, 3, 5, 6, 7, 0)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--peers", type=int, default=1, help="concurrent peers per replica (batched decode)")
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree (ranks per engine replica, RCCL over xGMI)")
    ap.add_argument("--ep", type=int, default=1,
                    help="expert-parallel degree for MoE models (ranks per replica)")
    ap.add_argument("--ep-mode", choices=("allreduce", "a2a"), default="allreduce")
    ap.add_argument("--weights", choices=("bf16", "fp8"), default="bf16",
                    help="weight storage of the dense projections (fp8: weight-only e4m3, "
                         "bf16 compute; opt-in -- the headline number is bf16)")
    ap.add_argument("--message", type=int, default=None,
                    help="index into SAMPLE_MESSAGES for peer 0 (default: the median-length one)")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu: gloo + the CPU engine (plumbing tests with tiny models)")
    ap.add_argument("--layers", type=int, default=None,
                    help="override n_layers (tests only; a reduced model is not a valid bench)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(a, argv) -> int:
    """Parent of a ``--gpus N`` run without torchrun: start N rank processes (fresh
    interpreters; this process never touches the GPU) and return the worst exit code."""
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   P2P_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = []
    for p in procs:
        rcs.append(p.wait())
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch(a, argv))
    run(a)


def run(a):
    import torch
    import torch.distributed as dist

    from p2p_llm_chat_go_amd.engine import Engine
    from p2p_llm_chat_go_amd.engine.tokenizer import SAMPLE_MESSAGES, get_tokenizer, suggest_prompt
    from p2p_llm_chat_go_amd.models.config import get_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit("bench: --gpus %d but the launcher started %d ranks" % (a.gpus, world))
    cuda = a.device == "cuda"
    backend = None
    if cuda:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // world))  # no oversubscription
    if world > 1:
        backend = "nccl" if cuda else "gloo"
        if cuda:
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != a.gpus:
            raise SystemExit("bench: process group has %d ranks, expected %d"
                             % (dist.get_world_size(), a.gpus))

    cfg = get_config(a.model)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    tok = get_tokenizer(cfg)
    tp, ep = max(1, a.tp), max(1, a.ep)
    if ep > 1 and not cfg.is_moe:
        raise SystemExit("bench: --ep needs an MoE model")
    group_size = tp * ep
    if world % group_size:
        raise SystemExit("bench: world size %d is not a multiple of tp*ep=%d" % (world, group_size))
    replica, sub_rank = rank // group_size, rank % group_size
    comm = None
    if group_size > 1:
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        groups = [dist.new_group(list(range(g * group_size, (g + 1) * group_size)))
                  for g in range(world // group_size)]
        comm = TPComm(groups[replica])
    first_msg = MESSAGE_ORDER[0] if a.message is None else a.message
    order = [first_msg] + [i for i in MESSAGE_ORDER if i != first_msg]
    prompts = []
    for p in range(a.peers):
        msg = SAMPLE_MESSAGES[order[(replica * a.peers + p) % len(order)]]
        prompts.append(tok.chat_ids(suggest_prompt(msg)))
    need_pages = sum((len(p) + a.new_tokens + 63) // 64 for p in prompts) + 8
    kw = dict(tp_rank=sub_rank, tp_size=tp) if tp > 1 else {}
    if ep > 1:
        kw = dict(ep_rank=sub_rank, ep_size=ep, ep_mode=a.ep_mode)
    eng = Engine(cfg, device=dev, seed=1234 + replica, kv_pages=max(need_pages, 64),
                 max_prefill_tokens=1024, max_batch=max(a.peers, 1),
                 use_graph=cuda and not a.no_graph, comm=comm, weight_dtype=a.weights, **kw)
    if cuda:
        eng.warmup((a.peers,), ctx=max(len(p) for p in prompts) + a.new_tokens)

    for _ in range(a.warmup):
        eng.generate(prompts, a.new_tokens, stop_on_eos=False)

    def barrier():
        if world > 1:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize(dev)

    ttfts, toks = [], 0
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = eng.generate(prompts, a.new_tokens, stop_on_eos=False)
        for r in res:
            ttfts.append(r.ttft_ns / 1e6)
            if sub_rank == 0:  # a TP/EP group produces each token once
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
    graphs = list(getattr(eng, "_graphs", {}).values())
    captured = bool(graphs) and all(g.graph is not None for g in graphs)
    if rank == 0:
        value = total_toks / elapsed
        prompt_len = len(prompts[0])
        par = "dp%d" % (world // group_size)
        if tp > 1:
            par += "-tp%d" % tp
        if ep > 1:
            par += "-ep%d" % ep
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
            # weight-only fp8 runs are labelled as such (bf16 activations / MFMA inputs,
            # e4m3 weights): never readable as the bf16 headline
            "dtype": "bf16" if a.weights == "bf16" else "fp8-weights/bf16-compute",
            "data": "synthetic chat prompts (reference co-pilot template, llama3.1 chat format, "
                    "median-length sample message); random-init weights",
            "config": {"model": cfg.name, "global_batch": (world // group_size) * a.peers,
                       "seq_len": prompt_len + a.new_tokens, "prompt_tokens": prompt_len,
                       "new_tokens": a.new_tokens, "parallelism": par, "tp": tp, "ep": ep,
                       "peers_per_replica": a.peers, "hipgraph_decode": cuda and not a.no_graph,
                       "weights": a.weights, "n_layers": cfg.n_layers},
            "ttft_p50_ms": round(statistics.median(all_ttft), 3),
            "ttft_p99_ms": round(sorted(all_ttft)[min(len(all_ttft) - 1,
                                                      int(0.99 * len(all_ttft)))], 3),
            "per_gpu_tokens_per_sec": round(value / world, 2),
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "backend": backend,
            "decode_graph_captured": captured,
            "gemm_autotune": {"%s@M%d" % k: "%s %.1fus" % v
                              for k, v in getattr(eng, "tuning", {}).items()},
        }
        print(json.dumps(out), flush=True)
    if comm is not None and hasattr(comm, "close"):
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
