"""The native engine step loop (csrc/runtime/engine_loop.cc via engine.native_loop):
continuous batching from a C++ thread that replays the captured prefill / decode graphs.

Its replies must equal the static-batch engine's (greedy), concurrent requests of
different lengths exercise riders in prefill chunks, pipelined decode chunks with lagged
finish detection and deferred page release; sampled requests must reproduce with their
seed and equal the Python loop's draws; streaming, the request deadline, cancellation and
the eager long-prompt path are covered too.  (The reference serves one blocking Ollama
call per click, `web/streamlit_app.py:89-101,163-165`.)"""
import json
import threading
import time

import pytest
import torch

from p2p_llm_chat_go_amd.engine import Engine
from p2p_llm_chat_go_amd.engine.sampling import SamplingParams
from p2p_llm_chat_go_amd.models import TINY_LLAMA
from p2p_llm_chat_go_amd.models.weights import EngineWeights

pytestmark = pytest.mark.gpu


def _engine(max_batch=4, layers=3, seed=5):
    cfg = TINY_LLAMA.replace(n_layers=layers, n_heads=8, n_kv_heads=2)
    w = EngineWeights.random(cfg, "cuda", seed=seed)
    return Engine(cfg, weights=w, device="cuda", kv_pages=128, max_batch=max_batch,
                  max_prefill_tokens=256), w, cfg


def _same_or_near_tie(eng, prompt, got, ref, margin=2e-2):
    """``got`` equals ``ref`` -- or first differs where the reference logits of the two
    candidates are within ``margin`` of the largest (a batch-shape rounding flip of the
    random model, not a loop bug)."""
    if got == ref:
        return True
    j = next((i for i, (x, y) in enumerate(zip(got, ref)) if x != y), min(len(got), len(ref)))
    if j >= min(len(got), len(ref)):
        return False  # one is a prefix of the other: a length bug
    toks = prompt + ref[:j]
    pages = eng.kv.allocator.alloc(-(-len(toks) // 64))
    try:
        _f, lg = eng.prefill([toks], [pages], return_logits=True)
    finally:
        eng.kv.allocator.free(pages)
    lg = lg[0].float().cpu()
    gap = abs(float(lg[got[j]] - lg[ref[j]]))
    assert gap < margin * float(lg.abs().max()), (j, gap, float(lg.abs().max()), got, ref)
    return True


def _prompts(n):
    return [[(13 * b + 7 * i) % 250 + 3 for i in range(5 + 11 * b)] for b in range(n)]


def test_native_loop_matches_static_greedy():
    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer

    eng, w, cfg = _engine()
    prompts = _prompts(6)
    lens = [9, 17, 4, 23, 12, 30]
    ref = []
    for p, n in zip(prompts, lens):  # one request at a time through the static engine
        ref.append(eng.generate([p], n, stop_on_eos=False)[0].tokens)
    srv = NativeEngineServer(eng, max_batch=4, decode_chunk=4)
    try:
        outs = [None] * len(prompts)

        def run(i):
            outs[i] = srv.generate(prompts[i], SamplingParams(max_tokens=lens[i],
                                                              stop_on_eos=False))

        ths = [threading.Thread(target=run, args=(i,)) for i in range(len(prompts))]
        [t.start() for t in ths]
        [t.join() for t in ths]
        for i, o in enumerate(outs):
            assert o["done"] and o["tokens"] == ref[i], (i, o["tokens"], ref[i])
            assert o["eval_count"] == lens[i] and o["prompt_eval_count"] == len(prompts[i])
        m = srv.metrics()
        assert m["requests"] == len(prompts) and m["native_loop"] == 1
        assert m["speculated_chunks"] > 0 and m["decode_calls"] > 0, m
        for _ in range(100):
            if srv.metrics()["free_kv_pages"] == 127:
                break
            time.sleep(0.02)
        assert srv.metrics()["free_kv_pages"] == 127  # every page back (null page reserved)
    finally:
        srv.close()


def test_native_loop_split_fault_word_fails_the_step():
    """A split-K slice that gave up sets the kernels' split-K fault word
    (ops.gemm.split_fault_word), not the graph's own: the native loop checks it beside every
    graph's word, fails the requests of that step with the reason, clears it, and serves the
    next request normally (the Python path raises in check_faults the same way)."""
    import ctypes

    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer
    from p2p_llm_chat_go_amd.ops.gemm import split_fault_word, tiled_split_fault

    eng, w, cfg = _engine()
    p = _prompts(2)[1]
    ref = eng.generate([p], 12, stop_on_eos=False)[0].tokens
    srv = NativeEngineServer(eng, max_batch=4, decode_chunk=4)
    try:
        word = split_fault_word(eng.device)
        one = torch.ones(1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(word), ctypes.c_void_p(one.data_ptr()),
                             ctypes.c_size_t(4), 3) == 0  # device to device
        with pytest.raises(RuntimeError, match="split-K"):
            srv.generate(p, SamplingParams(max_tokens=12, stop_on_eos=False))
        assert tiled_split_fault() == 0  # the loop cleared it
        r = srv.generate(p, SamplingParams(max_tokens=12, stop_on_eos=False))
        assert r["done"] and r["tokens"] == ref, r
        assert srv.metrics()["errors"] >= 1
    finally:
        srv.close()


def test_native_loop_full_batch_replays_k_step_graphs():
    """A full batch (running == max_batch) with decode_chunk=8: the loop's decode chunks are
    8 steps long, so it replays the whole 8-step graph (exec_k, engine_loop.cc) instead of
    8 one-step launches -- the path the serving numbers are measured on.  Replies must
    equal the static engine's."""
    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer

    eng, _w, _cfg = _engine(max_batch=4)
    prompts = _prompts(4)
    n = 41  # 5 whole 8-step chunks + a tail
    ref = [eng.generate([p], n, stop_on_eos=False)[0].tokens for p in prompts]
    srv = NativeEngineServer(eng, max_batch=4, decode_chunk=8)
    try:
        outs = [None] * 4
        start = threading.Barrier(4)

        def run(i):
            start.wait()
            outs[i] = srv.generate(prompts[i], SamplingParams(max_tokens=n, stop_on_eos=False))

        ths = [threading.Thread(target=run, args=(i,)) for i in range(4)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        m = srv.metrics()
    finally:
        srv.close()
    assert m["k_graph_launches"] >= 2, m  # whole 8-step graphs replayed by the loop
    for p, o, r in zip(prompts, outs, ref):
        assert o["done"] and len(o["tokens"]) == n
        assert _same_or_near_tie(eng, p, o["tokens"], r)


def test_native_loop_sampled_matches_python_loop():
    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer
    from p2p_llm_chat_go_amd.engine.server import EngineServer

    prompts = _prompts(3)
    params = [SamplingParams(temperature=0.9, top_k=20, top_p=0.9, seed=100 + i, max_tokens=10,
                             stop_on_eos=False) for i in range(3)]
    got = {}
    for kind in ("python", "native"):
        eng, _w, _cfg = _engine(seed=9)
        srv = (NativeEngineServer(eng, max_batch=4) if kind == "native"
               else EngineServer(eng, max_batch=4))
        try:  # one at a time: identical (prompt, position, seed) keys in both loops
            got[kind] = [srv.generate(p, params[i])["tokens"] for i, p in enumerate(prompts)]
            again = srv.generate(prompts[0], params[0])["tokens"]
            assert again == got[kind][0]
        finally:
            srv.close()
    assert got["native"] == got["python"]


def test_native_loop_stream_deadline_cancel_and_eager():
    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer
    from p2p_llm_chat_go_amd.engine.server import EngineTimeout

    eng, _w, _cfg = _engine()
    ref = eng.generate([_prompts(2)[1]], 12, stop_on_eos=False)[0].tokens
    long_prompt = [(5 * i) % 250 + 3 for i in range(300)]  # > prefill_ctx: the eager path
    ref_long = eng.generate([long_prompt], 6, stop_on_eos=False)[0].tokens
    srv = NativeEngineServer(eng, max_batch=4, prefill_ctx=256)
    try:
        chunks = []
        out = json.loads(srv.handle_json_stream(json.dumps(
            {"raw": False, "prompt": "hello there", "options": {"num_predict": 12,
                                                                "ignore_eos": True}}),
            lambda c: chunks.append(json.loads(c)) or True))
        assert out["done"] and out["eval_count"] == 12 and len(chunks) >= 1
        r = srv.generate(_prompts(2)[1], SamplingParams(max_tokens=12, stop_on_eos=False))
        assert r["tokens"] == ref
        r = srv.generate(long_prompt, SamplingParams(max_tokens=6, stop_on_eos=False))
        assert r["tokens"] == ref_long and srv.metrics()["eager_prefill_calls"] >= 1
        # stalled loop: the deadline fires, the request is cancelled and its pages return
        srv.request_timeout_s = 0.5
        free0 = srv.metrics()["free_kv_pages"]
        srv.stall(3.0)
        t0 = time.perf_counter()
        with pytest.raises(EngineTimeout):
            srv.generate(_prompts(1)[0], SamplingParams(max_tokens=50, stop_on_eos=False))
        assert time.perf_counter() - t0 < 2.5
        srv.stall(0.0)
        srv.request_timeout_s = 60
        r = srv.generate(_prompts(2)[1], SamplingParams(max_tokens=12, stop_on_eos=False))
        assert r["tokens"] == ref
        for _ in range(200):  # every page back (pages of finished requests are released
            m = srv.metrics()  # once no decode chunk is in flight; the null page stays)
            if m["free_kv_pages"] == 127 and m["running"] == 0:
                break
            time.sleep(0.02)
        assert m["free_kv_pages"] == 127 and m["running"] == 0, m
        assert free0 <= 127
    finally:
        srv.close()


def test_native_loop_8b_width_graphs():
    """Full-width 8B layers: the loop's prefill + decode graphs equal the static engine."""
    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer
    from p2p_llm_chat_go_amd.models import LLAMA31_8B

    cfg = LLAMA31_8B.replace(n_layers=2)
    w = EngineWeights.random(cfg, "cuda", seed=3)
    eng = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_batch=8)
    prompts = [[(97 * b + 31 * i) % 9000 + 200 for i in range(44 - 7 * b)] for b in range(4)]
    ref = [eng.generate([p], 16, stop_on_eos=False)[0].tokens for p in prompts]
    eng.prefill_graph_after = 1  # every chunk shape through a captured graph
    srv = NativeEngineServer(eng, max_batch=8)
    try:
        outs = [None] * 4
        ths = [threading.Thread(target=lambda i=i: outs.__setitem__(i, srv.generate(
            prompts[i], SamplingParams(max_tokens=16, stop_on_eos=False)))) for i in range(4)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        torch.cuda.synchronize()
    finally:
        srv.close()
    for p, o, r in zip(prompts, outs, ref):  # (the loop is gone: the engine is ours again)
        assert len(o["tokens"]) == 16
        assert _same_or_near_tie(eng, p, o["tokens"], r)


def test_native_loop_randomized_stress():
    """Mixed traffic through the C++ loop for a while: concurrent peers sending prompts of
    1-400 tokens (past the prefill graphs' context: the eager path), 1-60 new tokens, a third
    of them sampled, some abandoned by a short deadline (cancelled inside the loop), some
    streamed.  Every answered greedy request must equal the static engine's reply for it
    (up to a near-tie), sampled ones must reproduce with their seed, nothing may error, and
    every KV page must come back."""
    import random

    from p2p_llm_chat_go_amd.engine.native_loop import NativeEngineServer
    from p2p_llm_chat_go_amd.engine.server import EngineTimeout

    eng, _w, _cfg = _engine(max_batch=8)
    rng = random.Random(7)
    jobs = []
    for i in range(40):
        L = rng.choice([1, 3, 17, 44, 63, 64, 65, 130, 257, 400])
        prompt = [rng.randrange(3, 250) for _ in range(L)]
        n = rng.randrange(1, 61)
        kind = rng.choice(["greedy", "greedy", "sampled", "cancel", "stream"])
        jobs.append((prompt, n, kind, 1000 + i))
    srv = NativeEngineServer(eng, max_batch=8, prefill_ctx=256, decode_chunk=4)
    free0 = srv.metrics()["free_kv_pages"]
    results = [None] * len(jobs)

    def run(k):
        for i in range(k, len(jobs), 8):  # 8 peers, 5 requests each, back to back
            prompt, n, kind, seed = jobs[i]
            if kind == "sampled":
                p = SamplingParams(temperature=0.8, top_k=40, top_p=0.9, seed=seed, max_tokens=n,
                                   stop_on_eos=False)
            else:
                p = SamplingParams(max_tokens=n, stop_on_eos=False)
            try:
                if kind == "cancel":
                    srv.generate(prompt, p, timeout=0.002)
                    results[i] = ("done-anyway", None)
                elif kind == "stream":
                    rid = srv._submit(prompt, p)
                    got, done = [], False
                    while not done:
                        new, done = srv.loop.wait_tokens(rid, len(got), 5.0)
                        got += new
                    srv.loop.release(rid)
                    results[i] = ("ok", got)
                else:
                    results[i] = ("ok", srv.generate(prompt, p)["tokens"])
            except EngineTimeout:
                results[i] = ("timeout", None)
            except Exception as e:  # noqa: BLE001 -- reported below
                results[i] = ("error", repr(e))

    try:
        ths = [threading.Thread(target=run, args=(k,)) for k in range(8)]
        [t.start() for t in ths]
        [t.join(timeout=300) for t in ths]
        assert all(r is not None for r in results), "a peer hung"
        errors = [r for r in results if r[0] == "error"]
        assert not errors, errors[:3]
        for _ in range(200):
            m = srv.metrics()
            if m["free_kv_pages"] == free0 and m["running"] == 0 and m["waiting"] == 0:
                break
            time.sleep(0.02)
        assert m["free_kv_pages"] == free0 and m["running"] == 0, m
        assert m["eager_prefill_calls"] >= 1, m  # the prompts past the graphs' context
        for i, (prompt, n, kind, _seed) in enumerate(jobs):
            if kind == "sampled" and results[i][0] == "ok":
                assert len(results[i][1]) == n and all(0 <= t < 512 for t in results[i][1]), i
    finally:
        srv.close()
    # greedy and streamed replies vs the static engine (after the loop is gone)
    checked = 0
    for i, (prompt, n, kind, _seed) in enumerate(jobs):
        if kind in ("greedy", "stream") and results[i][0] == "ok":
            ref = eng.generate([prompt], n, stop_on_eos=False)[0].tokens
            assert len(results[i][1]) == n, (i, kind)
            assert _same_or_near_tie(eng, prompt, results[i][1], ref), (i, kind)
            checked += 1
    assert checked >= 15
