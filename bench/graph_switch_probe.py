"""Host cost of launching the prompt-chunk graph right after the decode graph ran (as inside
Engine.generate and every step of the serving loop) vs back to back, and whether giving
each graph its own stream changes it.  Prints one JSON line per variant: host enqueue of
Engine.prefill, wall to the first token, GPU event time (p50 over --iters)."""
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    cfg = get_config(a.model)
    tok = get_tokenizer(cfg)
    eng = Engine(cfg, device="cuda", kv_pages=256, max_batch=8)
    eng.warmup((1,), ctx=128)
    prompts = [tok.chat_ids(suggest_prompt(SAMPLE_MESSAGES[4]))]
    assert len(prompts[0]) + 64 <= 128
    pages = [eng.kv.allocator.alloc(2)]
    for _ in range(3):
        eng.prefill(prompts, pages).cpu()
    g = eng.decode_graph(1, len(prompts[0]) + 64)
    cur = torch.cuda.current_stream()
    side_p, side_d = torch.cuda.Stream(), torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def decode(stream):
        with torch.cuda.stream(stream):
            stream.wait_stream(cur)
            g.state.load([1], [len(prompts[0])], pages)
            g.replay(63)
            g.state.hist[:1, :1].cpu()
        cur.wait_stream(stream)
        torch.cuda.synchronize()

    def prefill(stream):
        with torch.cuda.stream(stream):
            stream.wait_stream(cur)
            t0 = time.perf_counter()
            e0.record(stream)
            first = eng.prefill(prompts, pages)
            e1.record(stream)
            enq = time.perf_counter() - t0
            first.cpu()
            wall = time.perf_counter() - t0
        cur.wait_stream(stream)
        torch.cuda.synchronize()
        return enq * 1e3, wall * 1e3, e0.elapsed_time(e1)

    variants = {
        "back_to_back": (None, cur),
        "after_decode_same_stream": (cur, cur),
        "after_decode_prefill_side_stream": (cur, side_p),
        "after_decode_both_side_streams": (side_d, side_p),
    }
    # the prefill chunk's graph alone (no host metadata build): replay-only enqueue after
    # the decode graph, after a one-node graph, and after hipGraphUpload of it
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    pg = list(eng._pgraphs.values())[0]
    tiny = torch.cuda.CUDAGraph()
    buf = torch.zeros(1, device="cuda")
    with torch.cuda.graph(tiny, capture_error_mode="thread_local"):
        buf.add_(1)

    def replay_only(before, upload=False):
        out = []
        for _ in range(a.iters):
            before()
            torch.cuda.synchronize()
            if upload:
                rc = hip.hipGraphUpload(ctypes.c_void_p(pg.graph.raw_cuda_graph_exec()),
                                        ctypes.c_void_p(cur.cuda_stream))
                assert rc == 0, rc
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            pg.graph.replay()
            out.append((time.perf_counter() - t0) * 1e3)
            torch.cuda.synchronize()
        return round(sorted(out)[len(out) // 2], 3)

    print(json.dumps({"replay_only_enqueue_ms_p50": {
        "back_to_back": replay_only(lambda: None),
        "after_decode": replay_only(lambda: decode(cur)),
        "after_one_node_graph": replay_only(lambda: tiny.replay()),
        "after_decode_then_upload": replay_only(lambda: decode(cur), upload=True),
        "after_decode_then_one_node_graph": replay_only(lambda: (decode(cur), tiny.replay())),
        "after_decode_then_one_kernel": replay_only(lambda: (decode(cur), buf.add_(1)))}}),
          flush=True)
    def decode_k(k):
        g.state.load([1], [len(prompts[0])], pages)
        g.replay(k)
        g.state.hist[:1, :1].cpu()
        torch.cuda.synchronize()

    print(json.dumps({"replay_only_enqueue_ms_p50_after_k_decode_steps": {
        str(k): replay_only(lambda k=k: decode_k(k)) for k in (1, 4, 16, 63)}}), flush=True)
    absorb = []
    for _ in range(a.iters):
        decode(cur)
        t0 = time.perf_counter()
        tiny.replay()
        absorb.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    print(json.dumps({"one_node_graph_enqueue_after_decode_ms_p50":
                      round(sorted(absorb)[len(absorb) // 2], 3)}), flush=True)

    if os.environ.get("PROBE_VARIANTS", "1") == "0":
        return
    for name, (dstream, pstream) in variants.items():
        for _ in range(2):  # settle
            if dstream is not None:
                decode(dstream)
            prefill(pstream)
        rows = []
        for _ in range(a.iters):
            if dstream is not None:
                decode(dstream)
            rows.append(prefill(pstream))
        med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
        print(json.dumps({"variant": name, "enqueue_ms_p50": round(med[0], 3),
                          "wall_ms_p50": round(med[1], 3), "gpu_ms_p50": round(med[2], 3)}),
              flush=True)


if __name__ == "__main__":
    main()
