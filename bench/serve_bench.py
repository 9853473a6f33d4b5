#!/usr/bin/env python3
"""Continuous-batching serving benchmark (BASELINE config 4: concurrent peers ->
batched decode), in-process through EngineServer + the native scheduler.

``--peers`` clients each issue ``--requests`` suggest-reply requests back to back
(closed loop: a peer sends its next request when the previous reply arrives),
so the engine sees requests join and leave the running batch at arbitrary
steps.  Prints one JSON line: aggregate generated tokens/s, TTFT p50/p99
(submit -> first token, queueing included), mean batch occupancy.
``--gpus N [--tp T | --ep E]``: the node's multi-GPU path instead (engine.cluster:
N / (T*E) replicas of one process per GPU, least-loaded routing of the peers'
Ollama JSON requests), i.e. exactly what a node with ENGINE_GPUS/ENGINE_TP serves.
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.sampling import SamplingParams  # noqa: E402
from p2p_llm_chat_go_amd.engine.server import EngineServer  # noqa: E402
from p2p_llm_chat_go_amd.engine.tokenizer import SAMPLE_MESSAGES, get_tokenizer, suggest_prompt  # noqa: E402
from p2p_llm_chat_go_amd.models.config import get_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--requests", type=int, default=4, help="requests per peer (timed)")
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--jitter", type=int, default=16,
                    help="reply lengths vary in [new-tokens - jitter, new-tokens]")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--max-prefill", type=int, default=1024,
                    help="prefill rows per engine step (a burst of prompts beyond it waits a step)")
    ap.add_argument("--mixed", type=int, default=1,
                    help="1: running sequences ride in prefill steps (mixed batches)")
    ap.add_argument("--gpus", type=int, default=1, help="serve through engine.cluster on N GPUs")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--virtual", type=int, default=0,
                    help="1: every rank of the group on ONE GPU (virtual ranks; compares the "
                         "serving loops, not multi-GPU speed)")
    ap.add_argument("--kv-pages", type=int, default=0, help="KV pages per rank (0: from free memory)")
    ap.add_argument("--ep", type=int, default=1)
    ap.add_argument("--ep-mode", choices=("allreduce", "a2a"), default="allreduce",
                    help="EP groups: replicated attention + all-reduce, or DP attention + "
                         "expert all-to-all")
    ap.add_argument("--warm-rounds", type=int, default=1,
                    help="untimed rounds of the timed pattern first (every peer's requests in "
                         "sequence): graphs for the shapes the mix hits -- a prompt-chunk shape "
                         "is captured on its 2nd use")
    ap.add_argument("--loop", choices=("native", "python"), default="native",
                    help="native: the C++ step loop replaying captured graphs "
                         "(engine.native_loop); python: engine.server's loop")
    a = ap.parse_args()
    if a.gpus > 1 or a.tp > 1 or a.ep > 1:
        return cluster_main(a)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(a.device, local) if a.device == "cuda" else torch.device(a.device)
    cfg = get_config(a.model)
    tok = get_tokenizer(cfg)
    eng = Engine(cfg, device=dev, seed=7, max_batch=max(a.peers, 1),
                 max_prefill_tokens=a.max_prefill)
    eng.warmup(tuple(sorted({1, 2, 4, 8, a.peers} - {0})), ctx=256)
    chunk = int(os.environ.get("ENGINE_DECODE_CHUNK", "8"))
    if a.loop == "native":
        from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer

        srv = NativeEngineServer(eng, tok, max_batch=a.peers, decode_chunk=chunk)

        def stats():
            return srv.metrics()
    else:
        srv = EngineServer(eng, tok, max_batch=a.peers, decode_chunk=chunk, mixed=bool(a.mixed))

        def stats():
            return dict(srv.stats)
    prompts = [tok.chat_ids(suggest_prompt(SAMPLE_MESSAGES[i % len(SAMPLE_MESSAGES)]))
               for i in range(a.peers)]

    def params(i):
        n = a.new_tokens - (i * 7919) % (a.jitter + 1)
        return SamplingParams(max_tokens=max(1, n), stop_on_eos=False)

    results, lock = [], threading.Lock()

    def peer(p, keep=True):
        for r in range(a.requests):
            out = srv.generate(prompts[p], params(p * 31 + r))
            if keep:
                with lock:
                    results.append(out)

    # warm pass (graphs for every batch bucket the burst hits), then untimed rounds of the
    # timed pattern (the steady-state prompt-chunk shapes: one new prompt + riders)
    ths = [threading.Thread(target=srv.generate, args=(prompts[p], params(p), 600))
           for p in range(a.peers)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    for _ in range(a.warm_rounds):
        ths = [threading.Thread(target=peer, args=(p, False)) for p in range(a.peers)]
        [t.start() for t in ths]
        [t.join() for t in ths]

    occ0 = stats()
    t0 = time.perf_counter()
    ths = [threading.Thread(target=peer, args=(p,)) for p in range(a.peers)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    el = time.perf_counter() - t0
    occ1 = stats()
    srv.close()
    toks = sum(r["eval_count"] for r in results)
    ttft = sorted(r["ttft_ns"] / 1e6 for r in results)
    queue = sorted((r["ttft_ns"] - r["prompt_eval_duration"]) / 1e6 for r in results)
    steps = occ1["decode_steps"] - occ0["decode_steps"]
    print(json.dumps({
        "metric": "suggest-reply tokens/sec (continuous batching)", "value": round(toks / el, 2),
        "unit": "tokens/s", "model": cfg.name, "peers": a.peers, "requests": len(results),
        "new_tokens": a.new_tokens, "elapsed_s": round(el, 3),
        "ttft_p50_ms": round(statistics.median(ttft), 3),
        "ttft_p99_ms": round(ttft[min(len(ttft) - 1, int(0.99 * len(ttft)))], 3),
        "queue_p50_ms": round(statistics.median(queue), 3),
        "queue_p99_ms": round(queue[min(len(queue) - 1, int(0.99 * len(queue)))], 3),
        "decode_chunk": srv.decode_chunk, "loop": a.loop, "warm_rounds": a.warm_rounds,
        "mean_batch": round(toks / max(steps, 1), 2), "mixed": bool(a.mixed), "dtype": "bf16",
        "engine_time_s": {k: round(occ1[k] - occ0[k], 4) for k in
                          ("busy_s", "prefill_s", "decode_s", "prefill_calls", "decode_calls",
                           "capture_s", "captures", "eager_prefill_s", "eager_prefill_calls",
                           "prefill_wait_s", "prefill_waits", "admit_wait_hits",
                           "admit_wait_misses") if k in occ1},
        "data": "synthetic chat prompts, random-init weights"}), flush=True)


def cluster_main(a):
    """Peers -> Ollama JSON -> ClusterServer router -> replica leaders (no GPU in this
    process)."""
    from p2p_llm_chat_go_amd.engine.cluster import ClusterServer

    # the replica leaders' loop (read by engine.cluster when the rank processes start)
    os.environ["ENGINE_NATIVE_LOOP"] = "1" if a.loop == "native" else "0"
    cs = ClusterServer(a.model, gpus=a.gpus, tp=a.tp, ep=a.ep,
                       device="cpu" if a.device == "cpu" else "cuda",
                       max_batch=max(8, a.peers), max_tokens=a.new_tokens,
                       virtual_ranks=bool(a.virtual), kv_pages=a.kv_pages or None,
                       ep_mode=a.ep_mode)

    def req(p, r):
        n = a.new_tokens - ((p * 31 + r) * 7919) % (a.jitter + 1)
        msg = SAMPLE_MESSAGES[p % len(SAMPLE_MESSAGES)]
        return json.dumps({"model": "llama3.1", "prompt": suggest_prompt(msg), "stream": False,
                           "options": {"temperature": 0, "num_predict": max(1, n),
                                       "ignore_eos": True}})

    try:
        ths = [threading.Thread(target=lambda p=p: cs.handle_json(req(p, -1)))
               for p in range(a.peers)]  # warm pass
        [t.start() for t in ths]
        [t.join() for t in ths]
        results, lock = [], threading.Lock()

        def peer(p):
            for r in range(a.requests):
                out = json.loads(cs.handle_json(req(p, r)))
                with lock:
                    results.append(out)

        t0 = time.perf_counter()
        ths = [threading.Thread(target=peer, args=(p,)) for p in range(a.peers)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        el = time.perf_counter() - t0
        m = cs.metrics()
    finally:
        cs.close()
    toks = sum(r["eval_count"] for r in results)
    ttft = sorted((r["total_duration"] - r["eval_duration"]) / 1e6 for r in results)
    print(json.dumps({
        "metric": "suggest-reply tokens/sec (continuous batching, multi-GPU node)",
        "value": round(toks / el, 2), "unit": "tokens/s", "model": a.model, "gpus": a.gpus,
        "tp": a.tp, "ep": a.ep, "ep_mode": a.ep_mode, "replicas": m.get("replicas"),
        "peers": a.peers,
        "requests": len(results), "new_tokens": a.new_tokens, "elapsed_s": round(el, 3),
        "ttft_p50_ms": round(statistics.median(ttft), 3),
        "ttft_p99_ms": round(ttft[min(len(ttft) - 1, int(0.99 * len(ttft)))], 3),
        "routed": [r.get("routed") for r in m.get("per_replica", [])], "dtype": "bf16",
        "loop": "native" if all(r.get("native_loop") for r in m.get("per_replica", [])) else "python",
        "mirror_frames": sum(r.get("mirror_frames", 0) for r in m.get("per_replica", [])),
        "k_graph_launches": sum(r.get("k_graph_launches", 0) for r in m.get("per_replica", [])),
        "virtual_ranks": bool(a.virtual),
        "data": "synthetic chat prompts, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
