"""Tensor-parallel correctness on CPU: gloo, world_size 2, 4 and 8, Megatron
sharding of qkv / o / gate_up / down / vocab-parallel LM head against the
unsharded engine (SURVEY §4.2 distributed tier (a)).  The TP model has the
8B/70B head structure (32 q / 8 kv heads: one kv head per rank at world 8) and
the EP model 8 experts (one per rank at world 8, Mixtral EP=8)."""
import datetime
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from p2p_llm_chat_go_amd.models.config import TINY_LLAMA_GQA, TINY_MIXTRAL_8E

TP_CFG = TINY_LLAMA_GQA


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, moe, a2a=False, exact=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if exact:  # every EP exchange takes the exact-count form (variable-split all-to-all)
        os.environ["P2P_A2A_STATIC_MAX_BYTES"] = "0"
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from p2p_llm_chat_go_amd.engine import Engine
        from p2p_llm_chat_go_amd.models.reference import random_state_dict
        from p2p_llm_chat_go_amd.models.weights import EngineWeights
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        cfg = TP_CFG
        if moe:
            cfg = TINY_MIXTRAL_8E
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


def _run(world, moe=False, a2a=False, exact=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, moe, a2a, exact))
          for r in range(world)]
    [p.start() for p in ps]
    res = [q.get(timeout=300) for _ in range(world)]
    [p.join(timeout=60) for p in ps]
    for rank, ok, got, ref in res:
        assert ok, (rank, got, ref)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tensor_parallel_matches_single(world):
    _run(world)


@pytest.mark.parametrize("world", [2, 8])
def test_expert_parallel_matches_single(world):
    _run(world, moe=True)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_expert_parallel_all_to_all_dp_attention(world):
    """EP with token dispatch/return by all-to-all (DP attention, distinct prompts per rank),
    static per-destination capacity."""
    _run(world, moe=True, a2a=True)


@pytest.mark.parametrize("world", [2, 8])
def test_expert_parallel_all_to_all_exact_counts(world):
    """The exact-count exchange (counts all-to-all, then variable splits: only routed rows
    travel) gives the same tokens."""
    _run(world, moe=True, a2a=True, exact=True)


def test_u64_max_allreduce_ordering():
    from p2p_llm_chat_go_amd.parallel import comm

    # unsigned order must survive the signed all-reduce: keys with the top bit set are larger
    k = torch.tensor([[0x7FFFFFFF_00000001, -0x7FFFFFFF_00000000]], dtype=torch.int64)
    flipped = k ^ comm._SIGN
    assert int(flipped.max()) == int(flipped[0, 1])  # the "negative" int64 is the larger u64


def _put_exit(q, item, code=0):
    # os._exit skips the queue's feeder-thread flush: drain it first, or the result can be
    # lost on a loaded machine and the parent waits for nothing
    q.put(item)
    q.close()
    q.join_thread()
    os._exit(code)


def _dying_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    try:
        # a bounded collective timeout: a survivor blocked on a dead peer's socket still raises
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        from p2p_llm_chat_go_amd.engine import Engine
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        comm = TPComm()
        eng = Engine(TP_CFG, device="cpu", kv_pages=32, comm=comm, tp_rank=rank, tp_size=world)
        prompts = [[1, 2, 3, 4, 5]]
        eng.generate(prompts, 4, stop_on_eos=False)
    except Exception as e:  # rendezvous lost (e.g. the port was taken meanwhile): retry
        _put_exit(q, (rank, None, "setup: %s" % e))
    if rank == 1:  # die mid-decode: after a few collectives of the next reply
        calls = [0]
        orig = comm.allreduce_add_

        def dying(h, p):
            calls[0] += 1
            if calls[0] == 12:
                os._exit(3)
            return orig(h, p)

        comm.allreduce_add_ = dying
    import time
    t0 = time.time()
    try:
        eng.generate(prompts, 16, stop_on_eos=False)
        item = (rank, False, "tokens returned with a dead peer")
    except Exception as e:
        item = (rank, True, "%s after %.1fs" % (type(e).__name__, time.time() - t0))
    _put_exit(q, item)


def test_tp_peer_death_raises_cpu():
    """A TP rank dying mid-decode makes the survivor raise (no silent tokens)."""
    ctx = mp.get_context("spawn")
    for attempt in range(3):  # a fresh port per attempt if the rendezvous itself failed
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_dying_worker, args=(r, 2, port, q)) for r in range(2)]
        [p.start() for p in ps]
        rank, ok, info = q.get(timeout=600)  # spawned ranks import torch: slow under pytest -n
        [p.join(timeout=90) for p in ps]
        [p.terminate() for p in ps if p.is_alive()]
        if ok is not None:
            break
    assert rank == 0 and ok, info
    assert ps[1].exitcode == 3


def _max_int_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    from p2p_llm_chat_go_amd.parallel.comm import TPComm

    comm = TPComm()
    # rank 1 alone saw a split-K fault (bit 2): every rank must see it (check_faults then
    # raises on all of them together)
    got = comm.max_int(2 if rank == 1 else 0)
    dist.destroy_process_group()
    _put_exit(q, (rank, got))


def test_fault_bits_shared_across_group():
    import multiprocessing as mp
    import socket

    ctx = mp.get_context("spawn")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    q = ctx.Queue()
    ps = [ctx.Process(target=_max_int_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    assert res == [(0, 2), (1, 2)]


def _local_timeout_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    import types

    from p2p_llm_chat_go_amd.models.llama import LlamaModel
    from p2p_llm_chat_go_amd.parallel.comm import TPComm
    from p2p_llm_chat_go_amd.parallel.custom_ar import CollectiveTimeout

    class Comm(TPComm):
        def check(self):  # rank 1's one-shot spin timed out; rank 0's did not
            if rank == 1:
                raise CollectiveTimeout("local spin timeout")

    fake = types.SimpleNamespace(device=torch.device("cpu"), comm=Comm())
    try:
        LlamaModel.check_faults(fake, None)
        got = "no raise"
    except CollectiveTimeout as e:
        got = "raised: " + str(e)[:20]
    dist.destroy_process_group()
    _put_exit(q, (rank, got))


def test_local_collective_timeout_raises_on_every_rank():
    """a rank whose own one-shot wait timed out shares it (fault bit 4) through
    the group MAX before raising, so its peers raise CollectiveTimeout at the same point
    instead of blocking in the MAX collective until the process-group timeout."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_local_timeout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(30)
    assert res[0][1].startswith("raised: a one-shot") and res[1][1] == "raised: local spin timeout"


def _peer_worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), P2P_CUSTOM_AR=mode)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    from p2p_llm_chat_go_amd.parallel import custom_ar
    from p2p_llm_chat_go_amd.parallel.comm import TPComm

    def no_path_1_2(a, b):  # mocked hipDeviceCanAccessPeer: devices 1 and 2 see no peer path
        return {a, b} != {1, 2}

    fails = custom_ar.peer_access_failures(None, torch.device("cuda", rank), can_access=no_path_1_2)
    # TPComm.setup on "GPU" rank devices with the same mock: raise (default) or fall back
    real = custom_ar.peer_access_failures
    custom_ar.peer_access_failures = lambda g, d: real(g, d, can_access=no_path_1_2)
    comm = TPComm()
    try:
        comm.setup(torch.device("cuda", rank))
        outcome = ("fallback", comm.car is None, len(comm.peer_failures))
    except custom_ar.PeerAccessError as e:
        outcome = ("raised", str(e))
    dist.destroy_process_group()
    _put_exit(q, (rank, sorted(fails), outcome))


@pytest.mark.parametrize("mode", ["1", "auto"])
def test_peer_access_preflight_names_pair(mode):
    """before mapping IPC buffers every rank checks peer access to every
    other device of the group; the failing pairs are gathered so all ranks agree, the error
    names them and points at P2P_CUSTOM_AR=0, and P2P_CUSTOM_AR=auto falls back to RCCL."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _port()
    q = ctx.Queue()
    world = 4
    ps = [ctx.Process(target=_peer_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    want = [(1, 1, 2, 2), (2, 2, 1, 1)]
    for rank, fails, outcome in res:
        assert [f[:4] for f in fails] == want, fails  # every rank sees the same pairs
        if mode == "1":
            assert outcome[0] == "raised"
            assert "rank 1 (device 1) -> rank 2 (device 2)" in outcome[1]
            assert "P2P_CUSTOM_AR=0" in outcome[1]
        else:
            assert outcome == ("fallback", True, 2)
