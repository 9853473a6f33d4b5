"""TP groups on the native serving loop (runtime/mirror.h): the leader's C++ EngineLoop
serves the requests and its followers' EngineMirror threads replay its device operations
-- prefill chunks and (multi-step) decode graphs with their IPC collectives -- with no
Python on the hot path of any rank.  Ranks are virtual (every rank process on the one GPU
of the test box, IPC collectives between the processes), the group is a real
ClusterServer replica.

Replies must equal the same group's Python lockstep loop (ENGINE_NATIVE_LOOP=0: the
round-4 path, pickled plans over the pipes) -- greedy and seeded sampling, riders and
concurrent requests -- and the leader's metrics must show the mirror at work.  (The
reference serves one click per Ollama call, `web/streamlit_app.py:161-173`; BASELINE
configs 3 and 5 serve it from TP / EP groups.)"""
import json
import os
import threading

import pytest

from p2p_llm_chat_go_amd.engine.cluster import ClusterServer

pytestmark = pytest.mark.gpu

MSGS = ["Did you see the game last night? That last-minute goal was unbelievable!",
        "Hey! How's it going?", "Are we still on for lunch tomorrow at noon?",
        "Quick question: do you know where the spare keys for the storage room are?"]


def _req(i, sampled=False, n=24):
    opts = {"num_predict": n, "ignore_eos": True}
    if sampled:
        opts.update(temperature=0.8, top_k=40, top_p=0.9, seed=100 + i)
    return json.dumps({"model": "llama3.1", "prompt": MSGS[i % len(MSGS)], "stream": False,
                       "options": opts})


def _serve(world, native, reqs):
    env = {"ENGINE_NATIVE_LOOP": "1" if native else "0", "P2P_CAR_TIMEOUT_MS": "30000",
           "P2P_QA_TIMEOUT_MS": "30000",
           # the fused all-reduce epilogue at every width: its launch keeps to the ranks'
           # share of the one device (tests/test_world8_gpu.py explains the residency limit)
           "P2P_TP_FUSED_AR": os.environ.get("P2P_TP_FUSED_AR", "1")}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        cs = ClusterServer("tiny-llama-gqa", gpus=world, tp=world, device="cuda", sd_seed=3,
                           max_batch=2, warmup=False, virtual_ranks=True, start_timeout=600,
                           kv_pages=256)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        seq = [json.loads(cs.handle_json(r)) for r in reqs]  # one at a time
        conc = [None] * len(reqs)

        def run(i):
            conc[i] = json.loads(cs.handle_json(reqs[i]))

        ths = [threading.Thread(target=run, args=(i,)) for i in range(len(reqs))]
        [t.start() for t in ths]
        [t.join(timeout=300) for t in ths]
        # a full batch (max_batch = 2) of long replies with nobody waiting: 8-step chunks
        full = [None] * 2
        ths = [threading.Thread(target=lambda i=i: full.__setitem__(
            i, json.loads(cs.handle_json(_req(i, n=96))))) for i in range(2)]
        [t.start() for t in ths]
        [t.join(timeout=300) for t in ths]
        assert all(f is not None and f["eval_count"] == 96 for f in full)
        m = cs.metrics()
    finally:
        cs.close()
    return seq, conc, m


@pytest.mark.parametrize("world", [2, 4, 8])
def test_group_native_loop_matches_python_lockstep(world):
    reqs = [_req(0), _req(1), _req(2, sampled=True), _req(3, n=40)]
    seq_n, conc_n, m = _serve(world, True, reqs)
    rep = m["per_replica"][0]
    assert rep.get("native_loop") == 1 and rep.get("mirror_frames", 0) > 0, rep
    show = {k: rep.get(k) for k in ("k_step_graphs", "k_graph_launches", "decode_calls",
                                     "decode_steps", "captures", "prefill_calls",
                                     "eager_prefill_calls", "mirror_frames")}
    assert rep.get("k_step_graphs", 0) > 0, show  # captured collectively on every rank
    assert rep.get("k_graph_launches", 0) > 0, show  # and replayed as whole k-step graphs
    seq_p, _conc_p, mp = _serve(world, False, reqs)
    assert "mirror_frames" not in mp["per_replica"][0]
    for i, (a, b) in enumerate(zip(seq_n, seq_p)):
        assert a["eval_count"] == b["eval_count"]
        if i == 2:
            # the sampled request: the same seed and positions draw the same uniforms, but
            # the two loops run the prompt chunk in different forms (captured graph with IPC
            # collectives vs eager), and a sampled draw turns a last-bit logit difference
            # into a different token whenever its uniform lands on a CDF boundary (round 5:
            # 2 of 7 TP=8 runs, after a shared first line); its first token must agree
            assert a["response"].split()[:1] == b["response"].split()[:1], (a, b)
            continue
        assert a["response"] == b["response"], (i, a["response"], b["response"])
    # concurrent (batched decode, riders in prompt chunks): every reply complete (the
    # batch shapes differ from the sequential run's, so bf16 rounding may flip near-ties)
    for a, b in zip(conc_n, seq_p):
        assert a is not None and a["done"] and a["eval_count"] == b["eval_count"]


def test_group_follower_fault_fails_the_step():
    """a kernel fault is local to the rank that saw it.  A follower whose split-K
    fault word is set (P2P_MIRROR_INJECT_FAULT: after its 3rd launching frame, inside the
    first request) reports it on the group channel's status back channel (runtime/mirror.h);
    the leader fails exactly that request with the reason, every rank's words are cleared,
    and the next request's reply equals a clean group's."""
    os.environ["P2P_MIRROR_INJECT_FAULT"] = "3"
    try:
        cs = ClusterServer("tiny-llama-gqa", gpus=2, tp=2, device="cuda", sd_seed=3, max_batch=2,
                           warmup=False, virtual_ranks=True, start_timeout=600, kv_pages=256)
    finally:
        os.environ.pop("P2P_MIRROR_INJECT_FAULT", None)
    try:
        with pytest.raises(RuntimeError, match="follower rank"):
            cs.handle_json(_req(0))
        after = json.loads(cs.handle_json(_req(0)))
        m = cs.metrics()["per_replica"][0]
    finally:
        cs.close()
    assert m.get("mirror_follower_faults", 0) >= 1, m
    clean, _conc, _m = _serve(2, True, [_req(0)])
    assert after["response"] == clean[0]["response"] and after["eval_count"] == 24
