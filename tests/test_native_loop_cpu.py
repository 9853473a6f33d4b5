"""The native engine loop (csrc/runtime/engine_loop.cc) on the CPU tier.

``_native.loop_use_host_fake_hip()`` swaps the loop's HIP entry points for a host-only
stand-in (copies are memcpy, a "graph exec" is a host function the loop "launches"), so
its scheduling can be checked without a GPU against a simulated model: every captured
graph is a Python callback that reads the loop's metadata from the same buffers a real
graph would, and the next token is a fixed function of (token, position) -- so the
expected reply of every request is known.  Covered: continuous batching of concurrent
requests (riders in prefill chunks, pipelined decode chunks with lagged finish
detection, deferred page release), EOS / length stops, the eager long-prompt path,
sampled rows (per-row seeds reach the graph), streaming, cancellation, the deadline with a
stalled loop, and the prefill metadata itself (slots, positions, tiles)."""
import ctypes
import random
import threading
import time

import numpy as np
import pytest

from p2p_llm_chat_go_amd.native import available, load

# the host fake replaces the process's HIP entry points for the loop: never next to a GPU
# run of the real loop in the same process
pytestmark = [pytest.mark.skipif(not available(), reason="native module not built"),
              pytest.mark.skipif(__import__("torch").cuda.is_available(),
                                 reason="CPU-tier test (host-fake HIP)")]

V, EOS, PAGE = 1000, 999, 64
CB = ctypes.CFUNCTYPE(ctypes.c_int)


def nxt(tok, pos, seed=0):
    return (int(tok) * 31 + int(pos) * 7 + 3 + int(seed)) % V


def expected(prompt, max_new, stop_on_eos=True, seed=0):
    out, tok, pos = [], prompt[-1], len(prompt) - 1
    while len(out) < max_new:
        tok = nxt(tok, pos, seed)
        pos += 1
        if stop_on_eos and tok == EOS:
            break
        out.append(tok)
    return out


class FakeModel:
    """Host 'graphs' for the loop: decode steps and prefill chunks over numpy buffers."""

    def __init__(self, prefill_pages, k_steps=0):
        self.P = prefill_pages
        self.keep = []
        self.errors = []
        self.loop = None
        self.k_steps = k_steps  # > 1: decode graphs also offer a k-step exec (exec_k)
        self.k_runs = 0         # exec_k launches seen
        self.fault_steps = set()  # decode step numbers (over all graphs) that set the fault word
        self.n_steps = 0

    def _exec(self, fn):
        def run():
            try:
                fn()
                return 0
            except Exception as e:  # noqa: BLE001 -- surfaced by the test
                self.errors.append(repr(e))
                return 1
        cb = CB(run)
        self.keep.append(cb)
        return ctypes.cast(cb, ctypes.c_void_p).value

    def decode(self, B, ctx, greedy):
        P, S = ctx // PAGE, ctx
        meta = np.zeros(B * (4 + P), np.int32)
        hist = np.zeros(B * S, np.int32)
        step = np.zeros(1, np.int32)
        keys = np.zeros(B * 32, np.int64)
        temp = np.zeros(B, np.float32)
        topk = np.zeros(B, np.int32)
        topp = np.zeros(B, np.float32)
        seeds = np.zeros(B, np.int64)
        err = np.zeros(1, np.int32)

        def run():
            ids, pos, cx = meta[:B], meta[B:2 * B], meta[2 * B:3 * B]
            s = int(step[0])
            assert s < S, "decode ran past its history"
            for b in range(B):
                t = nxt(ids[b], pos[b], 0 if greedy or temp[b] <= 0 else seeds[b])
                hist[b * S + s] = t
                ids[b] = t
                pos[b] += 1
                cx[b] = pos[b] + 1
            step[0] = s + 1
            self.n_steps += 1
            if self.n_steps in self.fault_steps:
                err[0] = 1  # as a kernel whose bounded spin gave up

        def run_k():
            self.k_runs += 1
            for _ in range(self.k_steps):
                run()
        self.keep += [meta, hist, step, keys, temp, topk, topp, seeds, err]
        d = {"B": B, "max_pages": P, "ctx": ctx, "greedy": greedy, "exec": self._exec(run),
             "meta": meta.ctypes.data, "hist": hist.ctypes.data, "max_steps": S,
             "step": step.ctypes.data, "keys": keys.ctypes.data, "keys_bytes": keys.nbytes,
             "err": err.ctypes.data}
        if greedy and self.k_steps > 1:
            d.update(exec_k=self._exec(run_k), k_steps=self.k_steps)
        if not greedy:
            d.update(temp=temp.ctypes.data, topk=topk.ctypes.data, topp=topp.ctypes.data,
                     seeds=seeds.ctypes.data)
        return d

    def prefill(self, rows, nseq, greedy, qtile=16):
        R, S, P = rows, nseq, self.P
        max_tiles = -(-R // qtile) + S + 1 + R // (P * PAGE) + 1  # as PrefillGraph
        sizes = [("bt", (S + 1) * P), ("seq", R), ("pos", R), ("ids", R), ("slots", R),
                 ("ctx", R), ("out", S), ("spos", S), ("tiles", 4 * max_tiles)]
        off, o = {}, 0
        for k, n in sizes:
            off[k] = o
            o += n
        meta = np.zeros(o, np.int32)
        first = np.zeros(S, np.int32)
        temp = np.zeros(S, np.float32)
        topk = np.zeros(S, np.int32)
        topp = np.zeros(S, np.float32)
        seeds = np.zeros(S, np.int64)

        def v(k, n):
            return meta[off[k]:off[k] + n]

        def run():
            bt = v("bt", (S + 1) * P).reshape(S + 1, P)
            seq, pos, ids = v("seq", R), v("pos", R), v("ids", R)
            slots, cx, out, spos = v("slots", R), v("ctx", R), v("out", S), v("spos", S)
            tiles = v("tiles", 4 * max_tiles).reshape(max_tiles, 4)
            for i in range(R):  # the loop's metadata, as the real kernels read it
                if seq[i] == S:
                    assert slots[i] == -1
                else:
                    assert slots[i] == bt[seq[i], pos[i] // PAGE] * PAGE + pos[i] % PAGE
                assert cx[i] == pos[i] + 1
            covered = np.zeros(R, bool)
            for r0, n, sq, p0 in tiles:
                if n == 0:
                    continue
                assert 0 < n <= qtile
                assert (seq[r0:r0 + n] == sq).all() and (pos[r0:r0 + n] == p0 + np.arange(n)).all()
                covered[r0:r0 + n] = True
            assert covered.all()
            for s in range(S):
                r = out[s]
                assert spos[s] == pos[r]
                sd = 0 if greedy or temp[s] <= 0 else seeds[s]
                first[s] = nxt(ids[r], pos[r], sd)
        self.keep += [meta, first, temp, topk, topp, seeds]
        d = {"rows": R, "n_seq": S, "max_pages": P, "qtile": qtile, "max_tiles": max_tiles,
             "greedy": greedy, "exec": self._exec(run), "meta": meta.ctypes.data,
             "meta_len": meta.size, "first": first.ctypes.data}
        for k in off:
            d["off_" + k] = off[k]
        if not greedy:
            d.update(temp=temp.ctypes.data, topk=topk.ctypes.data, topp=topp.ctypes.data,
                     seeds=seeds.ctypes.data)
        return d

    def provide(self, kind, a, b, greedy):
        if kind == "decode":
            self.loop.add_decode_graph(self.decode(a, b, greedy))
        else:
            self.loop.add_prefill_graph(self.prefill(a, b, greedy))

    def eager(self, prompts, pages, starts, samp):
        return [nxt(p[-1], len(p) - 1, 0 if t <= 0 else s) for p, (t, _k, _p, s) in zip(prompts, samp)]


def make_loop(pipeline=True, max_batch=8, chunk=4, free_slots=True, riders_all=False, k_steps=0):
    N = load()
    N.loop_use_host_fake_hip()
    model = FakeModel(prefill_pages=4, k_steps=k_steps)
    loop = N.EngineLoop({"num_pages": 256, "max_batch": max_batch, "max_prefill_tokens": 256,
                         "max_ctx": 2048, "eos": [EOS], "decode_chunk": chunk,
                         "admit_wait_us": 200.0, "pipeline": pipeline,
                         "pipeline_free_slots": free_slots, "riders_all": riders_all,
                         "row_buckets": [16, 32, 48, 64, 96, 128, 192, 256],
                         "prefill_max_pages": 4})
    model.loop = loop
    loop.set_provider(model.provide)
    loop.set_eager_prefill(model.eager)
    loop.start()
    return loop, model


def _wait_idle(loop, pages=255):
    for _ in range(300):
        m = loop.metrics()
        if m["running"] == 0 and m["waiting"] == 0 and m["free_kv_pages"] == pages:
            return m
        time.sleep(0.01)
    return loop.metrics()


@pytest.mark.parametrize("pipeline,riders_all", [(True, False), (False, False), (True, True)])
def test_loop_concurrent_requests_match_model(pipeline, riders_all):
    loop, model = make_loop(pipeline=pipeline, riders_all=riders_all)
    rng = random.Random(3)
    reqs = []
    for i in range(24):
        L = rng.choice([1, 5, 17, 44, 63, 64, 65, 120, 200]) if i else 300  # 300: eager path
        prompt = [rng.randrange(V - 1) for _ in range(L)]
        reqs.append((prompt, rng.randrange(1, 40), rng.random() < 0.8))
    outs = [None] * len(reqs)

    def run(i):
        p, n, eos = reqs[i]
        time.sleep(rng.random() * 0.02)
        rid = loop.submit(p, n, eos)
        outs[i] = loop.wait(rid, 30.0)
        loop.release(rid)

    try:
        ths = [threading.Thread(target=run, args=(i,)) for i in range(len(reqs))]
        [t.start() for t in ths]
        [t.join() for t in ths]
        assert not model.errors, model.errors[:3]
        for (p, n, eos), o in zip(reqs, outs):
            assert o["done"] and not o["error"], o
            assert o["tokens"] == expected(p, n, eos), (len(p), n, eos)
            assert o["done_reason"] in ("stop", "length")
        m = _wait_idle(loop)
        assert m["free_kv_pages"] == 255 and m["running"] == 0, m  # every page came back
        assert m["requests"] == len(reqs) and m["eager_prefill_calls"] >= 1
        if pipeline:
            assert m["speculated_chunks"] > 0, m
        else:
            assert m["speculated_chunks"] == 0, m
    finally:
        loop.shutdown()


def test_loop_sampled_rows_stream_and_cancel():
    loop, model = make_loop()
    try:
        prompt = [7, 8, 9, 10]
        # sampled rows: the per-row seed reaches the prefill and decode graphs
        rid = loop.submit(prompt, 12, False, 0.8, 40, 0.9, 5)
        r = loop.wait(rid, 10.0)
        loop.release(rid)
        assert r["tokens"] == expected(prompt, 12, False, seed=5)
        # greedy and sampled in one batch
        a = loop.submit(prompt, 9, False)
        b = loop.submit(prompt, 9, False, 0.7, 40, 0.9, 11)
        ra, rb = loop.wait(a, 10.0), loop.wait(b, 10.0)
        assert ra["tokens"] == expected(prompt, 9, False)
        assert rb["tokens"] == expected(prompt, 9, False, seed=11)
        loop.release(a)
        loop.release(b)
        # streaming: tokens arrive in order, then done
        rid = loop.submit([3, 4], 30, False)
        got, done = [], False
        while not done:
            new, done = loop.wait_tokens(rid, len(got), 1.0)
            got += new
        assert got == expected([3, 4], 30, False)
        loop.release(rid)
        # cancellation: a long request stops early and its pages come back
        rid = loop.submit([1, 2, 3], 1500, False)
        loop.wait_tokens(rid, 0, 5.0)  # running
        loop.stall(1.0)  # (the simulated model is fast: hold the loop while cancelling)
        loop.cancel(rid)
        loop.stall(0.0)
        r = loop.wait(rid, 10.0)
        assert r["done"] and r["done_reason"] == "cancelled" and len(r["tokens"]) < 1500
        loop.release(rid)
        m = _wait_idle(loop)
        assert m["free_kv_pages"] == 255, m
        assert not model.errors, model.errors[:3]
    finally:
        loop.shutdown()


def test_loop_deadline_with_stall():
    loop, model = make_loop()
    try:
        loop.stall(2.0)
        t0 = time.perf_counter()
        rid = loop.submit([5, 6], 10, False)
        r = loop.wait(rid, 0.3)
        assert not r["done"] and time.perf_counter() - t0 < 1.5
        loop.release(rid)  # the caller gave up: cancelled, dropped when it ends
        loop.stall(0.0)
        rid = loop.submit([5, 6], 10, False)
        r = loop.wait(rid, 10.0)
        assert r["done"] and r["tokens"] == expected([5, 6], 10, False)
        loop.release(rid)
        m = _wait_idle(loop)
        assert m["free_kv_pages"] == 255 and m["running"] == 0, m
    finally:
        loop.shutdown()


@pytest.mark.parametrize("max_batch,n,spec", [(4, 4, True), (8, 2, False)])
def test_loop_speculates_only_with_full_batch(max_batch, n, spec):
    """Default policy: a decode chunk is speculated behind the running one only while every
    batch slot is taken -- otherwise a request arriving would wait for two chunks."""
    loop, model = make_loop(max_batch=max_batch, free_slots=False)
    try:
        prompts = [[11 + i, 12, 13] for i in range(n)]
        loop.stall(0.5)  # all of them admitted in one step
        ids = [loop.submit(p, 60, False) for p in prompts]
        loop.stall(0.0)
        for p, rid in zip(prompts, ids):
            r = loop.wait(rid, 10.0)
            assert r["tokens"] == expected(p, 60, False)
            loop.release(rid)
        m = _wait_idle(loop)
        assert (m["speculated_chunks"] > 0) == spec, m
        assert not model.errors, model.errors[:3]
    finally:
        loop.shutdown()


def test_loop_full_batch_replays_k_step_graphs():
    """with every batch slot taken and decode_chunk = 8 the loop launches
    whole 8-step graphs (exec_k); replies still equal the model's."""
    loop, model = make_loop(max_batch=4, chunk=8, free_slots=False, k_steps=8)
    try:
        prompts = [[21 + i, 22, 23] for i in range(4)]
        loop.stall(0.5)  # all admitted in one step: a full batch
        ids = [loop.submit(p, 70, False) for p in prompts]
        loop.stall(0.0)
        for p, rid in zip(prompts, ids):
            r = loop.wait(rid, 10.0)
            assert r["done"] and not r["error"], r
            assert r["tokens"] == expected(p, 70, False)
            loop.release(rid)
        assert model.k_runs > 0
        assert not model.errors, model.errors[:3]
    finally:
        loop.shutdown()


def test_loop_fault_word_is_cleared_and_repeated_faults_mark_dead():
    """a fault word set by one decode step fails the requests of that
    step only -- the loop clears the word and serves the next request -- while faults in
    kMaxFaultsInRow (3) consecutive steps mark the replica dead (the router's signal)."""
    loop, model = make_loop(pipeline=False)
    try:
        model.fault_steps = {3}
        rid = loop.submit([5, 6, 7], 10, False)
        r = loop.wait(rid, 10.0)
        loop.release(rid)
        assert r["done"] and "fault word" in r["error"], r
        rid = loop.submit([5, 6, 7], 10, False)  # the word was cleared: this one is served
        r = loop.wait(rid, 10.0)
        loop.release(rid)
        assert r["done"] and not r["error"] and r["tokens"] == expected([5, 6, 7], 10, False), r
        assert loop.dead() == ""
        n = model.n_steps
        model.fault_steps = set(range(n + 1, n + 100))  # every step faults from now on
        for _ in range(3):
            rid = loop.submit([8, 9], 10, False)
            r = loop.wait(rid, 10.0)
            loop.release(rid)
            assert r["done"] and r["error"], r
        assert "fault word" in loop.dead()
        with pytest.raises(RuntimeError, match="replica is down"):
            loop.submit([1, 2], 4, False)
    finally:
        loop.shutdown()


def test_loop_refuses_request_past_largest_context_bucket():
    """prompt + max_new + decode slack beyond the largest context bucket
    is refused at submit, alone, instead of failing the running batch later."""
    N = load()
    N.loop_use_host_fake_hip()
    model = FakeModel(prefill_pages=4)
    loop = N.EngineLoop({"num_pages": 256, "max_batch": 4, "max_prefill_tokens": 256,
                         "max_ctx": 2048, "eos": [EOS], "decode_chunk": 4,
                         "ctx_buckets": [256, 512, 1024, 2048],
                         "row_buckets": [16, 32, 64, 128, 256], "prefill_max_pages": 4})
    model.loop = loop
    loop.set_provider(model.provide)
    loop.set_eager_prefill(model.eager)
    loop.start()
    try:
        with pytest.raises(ValueError, match="largest context bucket"):
            loop.submit([1] * 100, 2048 - 100, False)
        rid = loop.submit([1, 2, 3], 20, False)  # the loop still serves
        r = loop.wait(rid, 10.0)
        loop.release(rid)
        assert r["done"] and r["tokens"] == expected([1, 2, 3], 20, False)
    finally:
        loop.shutdown()


def test_loop_dead_wait_tokens_reports_down():
    """once the loop is stopped, wait_tokens reports done (no busy spin to
    the deadline) and wait() carries the reason."""
    loop, model = make_loop()
    loop.stall(5.0)
    rid = loop.submit([5, 6], 10, False)
    loop.stop()
    t0 = time.perf_counter()
    new, done = loop.wait_tokens(rid, 0, 5.0)
    assert done and time.perf_counter() - t0 < 1.0
    r = loop.wait(rid, 1.0)
    assert r["done"] and "replica is down" in r["error"], r
    loop.shutdown()
