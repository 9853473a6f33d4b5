"""Continuous-batching server + in-process node/engine integration (CPU tiny-llama).

This is BASELINE config 1: 2 libp2p nodes on loopback + Directory, CPU greedy
tiny-llama behind the node's Ollama-compatible /api/generate and /suggest.
"""
import json
import threading
import time

import pytest

from netutil import free_port, http, wait_http
from p2p_llm_chat_go_amd.engine import Engine
from p2p_llm_chat_go_amd.engine.sampling import SamplingParams
from p2p_llm_chat_go_amd.models import TINY_LLAMA
from p2p_llm_chat_go_amd.models.weights import EngineWeights
from p2p_llm_chat_go_amd.native import available, load

pytestmark = pytest.mark.skipif(not available(), reason="native module not built")


def make_server(max_batch=4, chunk=3, eos=None):
    from p2p_llm_chat_go_amd.engine.server import EngineServer

    cfg = TINY_LLAMA if eos is None else TINY_LLAMA.replace(eos_ids=eos)
    w = EngineWeights.random(cfg, "cpu", seed=7)
    eng = Engine(cfg, weights=w, device="cpu", kv_pages=128, max_batch=max_batch,
                 max_prefill_tokens=64)
    return EngineServer(eng, decode_chunk=chunk), w, cfg


def test_scheduler_native_policy():
    N = load()
    s = N.Scheduler(num_pages=9, page_size=64, max_batch=2, max_prefill_tokens=100, max_ctx=1024)
    a = s.add(50, 20)          # 2 pages
    b = s.add(100, 100)        # 4 pages
    c = s.add(10, 10)          # 1 page, but batch is full
    p = s.schedule()
    assert list(p.prefill) == [a] and list(p.decode) == []  # b exceeds the prefill budget
    p = s.schedule()
    assert list(p.prefill) == [b] and list(p.decode) == [a]
    assert s.free_pages == 8 - 6 and s.n_waiting == 1
    s.on_first_token(a, 5)
    s.on_decode_tokens([a], [[6] * 19])
    assert s.get(a).state == 2 and s.get(a).finish_reason == "length"
    assert len(s.get(a).tokens) == 20 and s.take_finished() == [a]
    p = s.schedule()
    assert list(p.prefill) == [c]  # slot freed
    s.on_first_token(c, 9)
    s.on_decode_tokens([c], [[1, 2, 3]])
    s.on_decode_tokens([c], [[2]])  # eos id 2 not set -> keeps going
    assert s.get(c).pos == 10 + 4
    with pytest.raises(Exception):
        s.add(1000, 100)  # exceeds max_ctx
    al = N.BlockAllocator(4)
    x = al.alloc(3)
    assert sorted(x) == [1, 2, 3] and al.free_pages == 0
    with pytest.raises(Exception):
        al.alloc(1)
    al.free(x)
    with pytest.raises(Exception):
        al.free([1])  # double free


def test_server_matches_static_batch_and_concurrency():
    srv, w, cfg = make_server(max_batch=3, chunk=2)
    try:
        prompts = [[1, 2, 3, 4], list(range(5, 40)), [9], [7, 7, 7, 7, 7, 7], [3] * 70]
        lens = [5, 9, 1, 12, 4]
        futs = []
        for p, n in zip(prompts, lens):
            futs.append(srv.submit(p, SamplingParams(max_tokens=n, stop_on_eos=False)))
        res = [f.result(120) for f in futs]
        ref_eng = Engine(cfg, weights=w, device="cpu", kv_pages=64, max_batch=8)
        for p, n, r in zip(prompts, lens, res):
            ref = ref_eng.generate([p], n, stop_on_eos=False)[0].tokens
            assert r["tokens"] == ref and r["eval_count"] == n and r["done_reason"] == "length"
            assert r["prompt_eval_count"] == len(p) and r["ttft_ns"] > 0
        m = srv.metrics()
        assert m["requests"] == 5 and m["free_kv_pages"] == 127 and m["running"] == 0
    finally:
        srv.close()


def test_server_eos_and_ollama_json():
    srv, _, _ = make_server(eos=tuple(range(512)))  # every token is EOS
    try:
        out = json.loads(srv.handle_json(json.dumps({"model": "llama3.1", "prompt": "hi",
                                                     "stream": False})))
        assert out["done"] is True and out["done_reason"] == "stop" and out["eval_count"] == 0
        for k in ("total_duration", "load_duration", "prompt_eval_count", "prompt_eval_duration",
                  "eval_duration", "created_at", "response", "model"):
            assert k in out
    finally:
        srv.close()


def test_server_sampling_and_chat():
    srv, _, _ = make_server()
    try:
        req = {"model": "m", "prompt": "hello", "stream": False,
               "options": {"temperature": 0.8, "top_k": 40, "top_p": 0.9, "num_predict": 6}}
        out = json.loads(srv.handle_json(json.dumps(req)))
        assert out["eval_count"] == 6 or out["done_reason"] == "stop"
        chat = json.loads(srv.handle_json(json.dumps(
            {"endpoint": "chat", "messages": [{"role": "user", "content": "hey"}],
             "options": {"num_predict": 3}})))
        assert chat["message"]["role"] == "assistant"
        assert json.loads(srv.handle_json('{"endpoint": "metrics"}'))["requests"] == 2
    finally:
        srv.close()


def test_chat_keeps_roles():
    """/api/chat renders every message with its role (system and assistant turns are
    part of the prompt, Ollama's llama3.1 / [INST] templates), not one joined user turn."""
    from p2p_llm_chat_go_amd.engine.tokenizer import SyntheticTokenizer

    srv, _, cfg = make_server()
    try:
        def chat(msgs):
            return json.loads(srv.handle_json(json.dumps(
                {"endpoint": "chat", "messages": msgs, "options": {"num_predict": 2}})))

        user = [{"role": "user", "content": "hey there"}]
        base = chat(user)["prompt_eval_count"]
        sys_ = chat([{"role": "system", "content": "answer in French"}] + user)
        multi = chat(user + [{"role": "assistant", "content": "hello"},
                             {"role": "user", "content": "how are you"}])
        assert sys_["prompt_eval_count"] > base and multi["prompt_eval_count"] > base
    finally:
        srv.close()
    tok = SyntheticTokenizer()  # llama3 template: header per message, open assistant header
    ids = tok.chat_messages_ids([{"role": "system", "content": "s"}, {"role": "user", "content": "u"}])
    assert ids[0] == 128000 and ids.count(128006) == 3 and ids.count(128009) == 2
    assert tok.chat_messages_ids([{"role": "user", "content": "x y"}]) == tok.chat_ids("x y")


def test_nodes_with_inprocess_engine():
    """Two native nodes in this process, node B with the engine as its LLM hook."""
    N = load()
    N.set_log_quiet(True)
    d = N.Directory()
    dport = d.start("127.0.0.1:0")
    durl = "http://127.0.0.1:%d" % dport
    srv, _, _ = make_server()
    nodes = []
    try:
        for name in ("A", "B"):
            n = N.Node({"username": name, "http_addr": "127.0.0.1:%d" % free_port(),
                        "directory_url": durl, "key_type": "ed25519", "access_log": False,
                        "listen": ["/ip4/127.0.0.1/tcp/0"]})
            if name == "B":
                n.set_generate_hook(srv.handle_json)
                n.set_generate_stream_hook(srv.handle_json_stream)
            n.start()
            nodes.append(n)
        a = "http://127.0.0.1:%d" % nodes[0].http_port
        b = "http://127.0.0.1:%d" % nodes[1].http_port
        wait_http(b + "/me")
        st, body, _ = http("POST", a + "/send", {"to_username": "B", "content": "Hey! How's it going?"})
        assert st == 200
        for _ in range(100):
            inbox = json.loads(http("GET", b + "/inbox")[1])
            if inbox:
                break
            time.sleep(0.05)
        mid = inbox[0]["id"]
        # the reference UI's exact call, pointed at the node (OLLAMA_URL = node)
        st, body, _ = http("POST", b + "/api/generate", {
            "model": "llama3.1", "stream": False,
            "prompt": "You are a helpful assistant. Draft a concise, friendly reply to the "
                      "following message:\n\nHey! How's it going?\n\nReply:"}, timeout=60)
        g = json.loads(body)
        assert st == 200 and g["done"] and "response" in g and g["eval_count"] > 0
        # streaming NDJSON (Ollama default): token-by-token chunks, then the stats object;
        # the concatenated stream equals the non-streamed greedy reply
        req = {"prompt": "x", "options": {"num_predict": 12}}
        st, body, hdr = http("POST", b + "/api/generate", req, timeout=60)
        lines = [json.loads(x) for x in body.strip().split("\n")]
        assert st == 200 and hdr["Content-Type"].startswith("application/x-ndjson")
        assert lines[-1]["done"] is True and lines[-1]["eval_count"] > 0
        assert len(lines) >= 3 and all(x["done"] is False for x in lines[:-1])
        streamed = "".join(x["response"] for x in lines[:-1])
        full = json.loads(http("POST", b + "/api/generate", dict(req, stream=False),
                               timeout=60)[1])["response"]
        assert streamed == full
        st, body, _ = http("POST", b + "/api/chat", {"messages": [{"role": "user", "content": "x"}],
                                                     "options": {"num_predict": 6}}, timeout=60)
        chunks = [json.loads(x) for x in body.strip().split("\n")]
        assert chunks[-1]["done"] is True and chunks[0]["message"]["role"] == "assistant"
        # one-click suggest + send back to the original sender
        st, body, _ = http("POST", b + "/suggest", {"id": mid, "send": True,
                                                    "options": {"num_predict": 5}}, timeout=60)
        s = json.loads(body)
        assert st == 200 and s["sent"] is True and "suggestion" in s
        for _ in range(100):
            back = json.loads(http("GET", a + "/inbox")[1])
            if back:
                break
            time.sleep(0.05)
        assert back[0]["from_user"] == "B" and back[0]["content"] == s["suggestion"]
        assert http("POST", b + "/suggest", {"id": "missing"})[0] == 404
        metrics = http("GET", b + "/metrics")[1]
        assert "p2p_messages_received_total 1" in metrics and "p2p_engine_requests" in metrics
        # concurrent peers -> batched decode
        outs = [None] * 4

        def ask(i):
            outs[i] = http("POST", b + "/api/generate", {"prompt": "q%d" % i, "stream": False,
                                                         "options": {"num_predict": 4}}, timeout=60)
        ts = [threading.Thread(target=ask, args=(i,)) for i in range(4)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert all(o[0] == 200 for o in outs)
    finally:
        for n in nodes:
            n.stop()
        srv.close()
        d.stop()


@pytest.mark.gpu
def test_server_gpu_graphs_batched():
    """Continuous batching on the GPU with hipGraph decode: results equal the static path."""
    from p2p_llm_chat_go_amd.engine.server import EngineServer

    cfg = TINY_LLAMA.replace(n_layers=3)
    w = EngineWeights.random(cfg, "cuda", seed=11)
    eng = Engine(cfg, weights=w, device="cuda", kv_pages=128, max_batch=8)
    srv = EngineServer(eng, decode_chunk=4)
    try:
        prompts = [[1, 2, 3], list(range(5, 90)), [9] * 7, [4, 4], [8] * 130]
        lens = [6, 17, 9, 3, 11]
        futs = [srv.submit(p, SamplingParams(max_tokens=n, stop_on_eos=False))
                for p, n in zip(prompts, lens)]
        res = [f.result(300) for f in futs]
        ref = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_batch=8)
        for p, n, r in zip(prompts, lens, res):
            assert r["tokens"] == ref.generate([p], n, stop_on_eos=False)[0].tokens
    finally:
        srv.close()


def test_server_cancel_and_stream_disconnect():
    """A cancelled request (or a streaming client that goes away) stops early and
    frees its KV pages."""
    srv, _, _ = make_server()
    try:
        free0 = srv.sched.free_pages
        p = SamplingParams(max_tokens=400, stop_on_eos=False)
        fut = srv.submit([1, 2, 3], p)
        srv.cancel(fut)
        r = fut.result(60)
        assert r["done_reason"] == "cancelled" and r["eval_count"] < 400
        # streaming consumer that refuses the first chunk
        calls = []

        def emit(chunk):
            calls.append(chunk)
            return False
        out = json.loads(srv.handle_json_stream(json.dumps(
            {"prompt": "x", "options": {"num_predict": 400}}), emit))
        assert out["done"] is True and out["done_reason"] == "cancelled"
        assert len(calls) == 1 and out["eval_count"] < 400
        for _ in range(100):
            if srv.sched.free_pages == free0:
                break
            time.sleep(0.02)
        assert srv.sched.free_pages == free0
    finally:
        srv.close()


def test_sampling_reference_semantics():
    """ops.sample's reference (the GPU kernel's oracle): top-k then top-p keep set,
    greedy rows, reproducible draws per (seed, position), and draws that follow the
    kept distribution."""
    import torch

    from p2p_llm_chat_go_amd import ops
    from p2p_llm_chat_go_amd.ops import sampling as S

    torch.manual_seed(0)
    lg = torch.randn(3, 500) * 2
    ids, p = S.keep_set(lg[0], 0.7, 5, 1.0)
    assert len(ids) == 5 and torch.equal(ids, lg[0].topk(5).indices)
    assert abs(float(p.sum()) - 1) < 1e-6 and bool((p[:-1] >= p[1:]).all())
    ids2, _ = S.keep_set(lg[0], 0.7, 40, 0.5)
    q = torch.softmax(lg[0].topk(40).values / 0.7, -1)
    n_keep = int(((q.cumsum(-1) - q) <= 0.5).sum())
    assert len(ids2) == n_keep and 1 <= n_keep < 40
    args = (torch.tensor([0.0, 0.8, 0.8]), torch.tensor([40, 40, 40], dtype=torch.int32),
            torch.tensor([0.9, 0.9, 0.9]), torch.tensor([1, 2, 2]))
    a = ops.sample(lg, *args, torch.tensor([7, 7, 7], dtype=torch.int32))
    b = ops.sample(lg, *args, torch.tensor([7, 7, 7], dtype=torch.int32))
    assert torch.equal(a, b) and int(a[0]) == int(lg[0].argmax())
    # empirical frequencies over positions (fresh draws) match the kept distribution
    row = torch.tensor([[4.0, 3.5, 3.0, 0.0, -1.0] + [-9.0] * 20])
    ids, p = S.keep_set(row[0], 1.0, 3, 1.0)
    cnt = torch.zeros(3)
    n = 3000
    for t in range(n):
        tok = int(ops.sample(row, torch.tensor([1.0]), torch.tensor([3], dtype=torch.int32),
                             torch.tensor([1.0]), torch.tensor([11]),
                             torch.tensor([t], dtype=torch.int32))[0])
        assert tok in (0, 1, 2)
        cnt[tok] += 1
    assert (cnt / n - p[torch.argsort(ids)]).abs().max() < 0.03


def test_server_sampled_requests_reproducible_with_seed():
    """/api/generate with options.seed: the same seed replays the same reply (draws are
    keyed by (seed, position, token)); the first token is sampled too."""
    srv, _, _ = make_server()
    try:
        def gen(seed):
            req = {"model": "m", "prompt": "hello there", "stream": False,
                   "options": {"temperature": 1.5, "top_k": 50, "top_p": 0.95,
                               "num_predict": 8, "seed": seed}}
            return json.loads(srv.handle_json(json.dumps(req)))["response"]

        a, b = gen(123), gen(123)
        assert a == b
        outs = {gen(s) for s in range(6)}
        assert len(outs) > 1  # different seeds draw different replies
    finally:
        srv.close()


def test_stalled_engine_times_out_with_503(monkeypatch):
    """SURVEY §5 fault injection "stall engine": with the engine loop stalled, the
    co-pilot call fails within ENGINE_TIMEOUT (the reference UI's 60 s bound,
    `web/streamlit_app.py:95`) -- /suggest answers 503 "LLM unavailable: ..." as the UI's
    `(LLM unavailable: ...)` -- the request is cancelled, its KV pages come back, and the
    engine serves again once the stall ends."""
    from p2p_llm_chat_go_amd.engine.server import EngineTimeout

    monkeypatch.setenv("ENGINE_TIMEOUT", "1.0")
    srv, _, _ = make_server()
    N = load()
    N.set_log_quiet(True)
    d = N.Directory()
    durl = "http://127.0.0.1:%d" % d.start("127.0.0.1:0")
    node = N.Node({"username": "B", "http_addr": "127.0.0.1:%d" % free_port(),
                   "directory_url": durl, "key_type": "ed25519", "access_log": False,
                   "listen": ["/ip4/127.0.0.1/tcp/0"]})
    node.set_generate_hook(srv.handle_json)
    node.set_generate_stream_hook(srv.handle_json_stream)
    try:
        node.start()
        b = "http://127.0.0.1:%d" % node.http_port
        wait_http(b + "/me")
        free0 = srv.sched.free_pages
        srv.stall(30.0)
        t0 = time.perf_counter()
        st, body, _ = http("POST", b + "/suggest", {"message": "Hey! How's it going?",
                                                    "options": {"num_predict": 4}}, timeout=30)
        dt = time.perf_counter() - t0
        assert st == 503 and json.loads(body)["error"].startswith("LLM unavailable: ")
        assert "within 1s" in json.loads(body)["error"]
        assert 0.9 < dt < 5.0, dt
        # the streaming path has the same deadline
        t0 = time.perf_counter()
        with pytest.raises(EngineTimeout):
            srv.handle_json_stream(json.dumps({"prompt": "x", "options": {"num_predict": 4}}),
                                   lambda c: True)
        assert time.perf_counter() - t0 < 5.0
        srv.stall(0.0)  # the GPU "recovers": cancelled requests drain, serving resumes
        st, body, _ = http("POST", b + "/suggest", {"message": "again",
                                                    "options": {"num_predict": 4}}, timeout=30)
        assert st == 200 and "suggestion" in json.loads(body)
        for _ in range(200):
            if srv.sched.free_pages == free0 and srv.sched.n_running == 0:
                break
            time.sleep(0.02)
        assert srv.sched.free_pages == free0 and srv.sched.n_running == 0
    finally:
        node.stop()
        srv.close()
        d.stop()
