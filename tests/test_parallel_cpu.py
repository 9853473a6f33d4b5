"""Tensor-parallel correctness on CPU: gloo, world_size 2 (and 4), Megatron
sharding of qkv / o / gate_up / down / vocab-parallel LM head against the
unsharded engine (SURVEY §4.2 distributed tier (a))."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from p2p_llm_chat_go_amd.models import TINY_LLAMA

TP_CFG = TINY_LLAMA.replace(name="tiny-tp", n_heads=4, n_kv_heads=4, ffn=512, n_layers=2)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, moe, a2a=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from p2p_llm_chat_go_amd.engine import Engine
        from p2p_llm_chat_go_amd.models.reference import random_state_dict
        from p2p_llm_chat_go_amd.models.weights import EngineWeights
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        cfg = TP_CFG
        if moe:
            from p2p_llm_chat_go_amd.models import TINY_MIXTRAL
            cfg = TINY_MIXTRAL.replace(n_heads=4, n_kv_heads=4)
        sd = random_state_dict(cfg, seed=3)
        prompts = [[1, 2, 3, 4, 5], list(range(10, 50))]
        if a2a:  # DP attention: every rank serves its own peers (equal lengths: lockstep)
            prompts = [[1 + rank, 2, 3 + 2 * rank, 4, 5], list(range(10 + rank, 50 + rank))]
        full = Engine(cfg, weights=EngineWeights.from_state_dict(sd, cfg, "cpu"), device="cpu",
                      kv_pages=32)
        ref = [r.tokens for r in full.generate(prompts, 6, stop_on_eos=False)]
        kw = dict(tp_rank=rank, tp_size=world)
        if moe:
            kw = dict(ep_rank=rank, ep_size=world)
        w = EngineWeights.from_state_dict(sd, cfg, "cpu", **kw)
        eng = Engine(cfg, weights=w, device="cpu", kv_pages=32, comm=TPComm(),
                     tp_rank=w.tp_rank, tp_size=w.tp_size,
                     ep_mode="a2a" if a2a else "allreduce")
        got = [r.tokens for r in eng.generate(prompts, 6, stop_on_eos=False)]
        if not moe and got == ref:
            # Ollama sampler under TP: every rank gathers the vocab shards and draws the
            # same token (keyed by seed, position, token) as the unsharded engine
            ref, got = _sampled(full, prompts), _sampled(eng, prompts)
        q.put((rank, got == ref, got, ref))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, False, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def _sampled(eng, prompts, n=5):
    from p2p_llm_chat_go_amd.engine.sampling import SamplingParams

    params = [SamplingParams(temperature=1.2, top_k=20, top_p=0.95, seed=11 + b)
              for b in range(len(prompts))]
    pages = [eng.kv.allocator.alloc(2) for _ in prompts]
    first = eng.prefill(prompts, pages, sampling=params).tolist()
    g = eng.decode_graph(len(prompts), 128, greedy=False)
    g.state.load(first, [len(p) for p in prompts], pages)
    g.step_sampled(params, n)
    out = [[first[b]] + g.state.hist[b, :n].tolist() for b in range(len(prompts))]
    for p in pages:
        eng.kv.allocator.free(p)
    return out


def _run(world, moe=False, a2a=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, moe, a2a)) for r in range(world)]
    [p.start() for p in ps]
    res = [q.get(timeout=300) for _ in range(world)]
    [p.join(timeout=60) for p in ps]
    for rank, ok, got, ref in res:
        assert ok, (rank, got, ref)


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_matches_single(world):
    _run(world)


def test_expert_parallel_matches_single():
    _run(2, moe=True)


@pytest.mark.parametrize("world", [2, 4])
def test_expert_parallel_all_to_all_dp_attention(world):
    """EP with token dispatch/return by all-to-all (DP attention, distinct prompts per rank)."""
    _run(world, moe=True, a2a=True)


def test_u64_max_allreduce_ordering():
    from p2p_llm_chat_go_amd.parallel import comm

    # unsigned order must survive the signed all-reduce: keys with the top bit set are larger
    k = torch.tensor([[0x7FFFFFFF_00000001, -0x7FFFFFFF_00000000]], dtype=torch.int64)
    flipped = k ^ comm._SIGN
    assert int(flipped.max()) == int(flipped[0, 1])  # the "negative" int64 is the larger u64
