"""Per-rank proxy of a TP=8 engine on ONE MI355X (BASELINE config 3).

Builds the rank-0 shard of the full model at ``tp_size=8`` (70B: 80 layers, 8 query
heads + 1 KV head per rank, 3584 ffn columns, a 16032-column vocab shard, the full
embedding table) and runs the real suggest-reply loop on it: prefill of the
44-token chat prompt, then hipGraph decode.  The TP collectives are the one-shot IPC
kernels of ``parallel/custom_ar.py`` at world 1 (``TPComm.car_at_world1``): every
row-parallel sum and the greedy argmax-key MAX launch exactly as on 8 GPUs, but the
peers are this rank itself, so the numbers are a **projected per-rank floor with the
xGMI latency excluded** (the pushes go to local HBM and no flag wait is ever
satisfied late).  The gap to a real 8-GPU run is therefore 160 all-reduce
latencies per token (2 per layer) plus the argmax MAX.

Prints one JSON line: decode ms/token (graph replay, GPU events), the suggest-reply
tokens/s of one replica (prefill + 63 decode steps per reply, as bench.py), TTFT p50,
the rank's weight bytes and the weight-stream rate the decode step reaches.  Run it
under ``rocprofv3 --kernel-trace --stats`` for the per-kernel table.

The reference has no TP: the call served is `web/streamlit_app.py:91-95`.
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.engine import Engine  # noqa: E402
from p2p_llm_chat_go_amd.engine.tokenizer import SAMPLE_MESSAGES, get_tokenizer, suggest_prompt  # noqa: E402
from p2p_llm_chat_go_amd.models.config import get_config  # noqa: E402
from p2p_llm_chat_go_amd.parallel.comm import TPComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0, help="which shard to build")
    ap.add_argument("--peers", type=int, default=1)
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=None, help="tests only (not a valid proxy)")
    a = ap.parse_args()

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    cfg = get_config(a.model)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    tok = get_tokenizer(cfg)
    comm = TPComm()
    comm.car_at_world1 = True
    prompts = [tok.chat_ids(suggest_prompt(SAMPLE_MESSAGES[(4 + i) % len(SAMPLE_MESSAGES)]))
               for i in range(a.peers)]
    need_pages = sum((len(p) + a.new_tokens + 63) // 64 for p in prompts) + 8
    eng = Engine(cfg, device="cuda", seed=1234, kv_pages=max(64, need_pages),
                 max_batch=max(1, a.peers), comm=comm, tp_rank=a.rank, tp_size=a.tp)
    assert comm.car is not None, "one-shot kernels not set up"
    eng.warmup((a.peers,), ctx=max(len(p) for p in prompts) + a.new_tokens)
    for _ in range(a.warmup):
        eng.generate(prompts, a.new_tokens, stop_on_eos=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ttfts, toks = [], 0
    for _ in range(a.steps):
        for r in eng.generate(prompts, a.new_tokens, stop_on_eos=False):
            ttfts.append(r.ttft_ns / 1e6)
            toks += r.eval_count
    torch.cuda.synchronize()
    el = time.perf_counter() - t0

    # decode step alone: k graph replays between GPU events
    g = eng.decode_graph(a.peers, max(len(p) for p in prompts) + a.new_tokens)
    pages = [eng.kv.allocator.alloc(2) for _ in prompts]
    g.state.load([1] * len(prompts), [len(p) for p in prompts], pages)
    k = min(32, a.new_tokens)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay(4)
    torch.cuda.synchronize()
    g.state.load([1] * len(prompts), [len(p) for p in prompts], pages)
    e0.record()
    g.replay(k)
    e1.record()
    torch.cuda.synchronize()
    dec_ms = e0.elapsed_time(e1) / k
    eng.check_comm()
    wbytes = eng.weights.nbytes()
    # bytes one decode step streams: everything but the embedding table (one row is read)
    stream = wbytes - eng.weights.embed.numel() * 2
    print(json.dumps({
        "what": "projected per-rank floor, xGMI latency excluded",
        "model": cfg.name, "n_layers": cfg.n_layers, "tp": a.tp, "rank": a.rank,
        "peers": a.peers, "prompt_tokens": len(prompts[0]), "new_tokens": a.new_tokens,
        "decode_ms_per_token": round(dec_ms, 4),
        "decode_tokens_per_sec_per_replica": round(a.peers * 1000.0 / dec_ms, 2),
        "suggest_reply_tokens_per_sec": round(toks / el, 2),
        "ttft_p50_ms": round(statistics.median(ttfts), 3),
        "rank_weight_gb": round(wbytes / 1e9, 3),
        "decode_weight_stream_tb_s": round(stream / (dec_ms * 1e-3) / 1e12, 3),
        "collectives": "one-shot IPC kernels at world 1 (custom_allreduce.hip)",
        "gemm_autotune": {"%s@M%d" % kk: "%s %.1fus" % v for kk, v in eng.tuning.items()},
    }), flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
