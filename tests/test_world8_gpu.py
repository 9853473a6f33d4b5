"""World-8 tensor / expert parallelism at REAL model widths on the one MI355X of the
test box (VERDICT r2 "next round" item 1; SURVEY §4.2 distributed tier (b)).

Eight rank processes share the device ("virtual ranks"): host-side setup runs over
gloo, the decode step's collectives are the one-shot IPC kernels
(``csrc/kernels/custom_allreduce.hip``) between the eight processes, and decode runs
as captured hipGraphs -- the exact launch structure of an 8-GPU node, with one KV head
per rank (8B / 70B at TP=8), 16032-column vocab shards, and 8 IPC peers per
collective.  What one device cannot show is xGMI bandwidth/latency; what it does show
is that the protocol, the sharding and the graphs are right at world 8.

* dense: llama3.1-8B full width (2 layers), TP=8.  The vocab-sharded prefill logits,
  gathered, match a TP=1 engine on the same checkpoint within bf16 tolerance, and every
  greedy token the TP=8 graph emits is an argmax (to bf16 tolerance) of the TP=1
  model's logits at that position.
* MoE: Mixtral-8x7B full width (2 layers), EP=8 (one expert per rank), in the
  ``allreduce`` mode (replicated attention, partial expert sums all-reduced) and the
  ``a2a`` mode (DP attention, token dispatch/combine all-to-all on the IPC kernels,
  decode graph-captured).

The reference has no parallelism; the call these engines serve is
`web/streamlit_app.py:91-95` (BASELINE configs 3 and 5).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 8


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _prompts(rank, per_rank):
    # two chat-length prompts (44 and 23 tokens); a2a: different tokens per rank, same lengths
    off = 17 * rank if per_rank else 0
    return [[(101 + 37 * i + off) % 30000 + 5 for i in range(44)],
            [(7 + 211 * i + off) % 30000 + 5 for i in range(23)]]


def _check_logits(got, ref, what):
    """got/ref fp32 [B, V]: bf16-level agreement (relative to the logit spread)."""
    err = (got - ref).abs().max().item()
    spread = ref.std().item()
    assert err <= 0.08 * spread + 0.02, "%s: max |diff| %.4f vs logit std %.4f" % (what, err, spread)


def _worker(rank, world, port, q, kind, mode, env):
    # 8 processes time-share one device: a rank's kernel can wait on a peer whose queue is
    # not scheduled yet, so the spin bounds (all-reduce, fused qkv+attention hand-off) are
    # generous here (5 s on real GPUs)
    # (the wide GEMM's K slices also meet inside one launch: capped to one slice, as the
    # cluster does for virtual ranks, engine/cluster.py)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), P2P_CAR_TIMEOUT_MS="30000",
                      P2P_QA_TIMEOUT_MS="30000", P2P_WIDE_SPLIT_CAP="1", **env)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    WORLD = world
    try:
        from p2p_llm_chat_go_amd.engine import Engine
        from p2p_llm_chat_go_amd.models.config import LLAMA31_8B, MIXTRAL_8X7B
        from p2p_llm_chat_go_amd.models.reference import random_state_dict
        from p2p_llm_chat_go_amd.models.weights import EngineWeights
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        torch.cuda.set_device(0)
        moe = kind == "moe"
        cfg = (MIXTRAL_8X7B if moe else LLAMA31_8B).replace(n_layers=2)
        # same checkpoint in every process (device generator, one device)
        sd = random_state_dict(cfg, seed=11, device="cuda", on_device=True)
        kw = dict(ep_rank=rank, ep_size=WORLD) if moe else dict(tp_rank=rank, tp_size=WORLD)
        w = EngineWeights.from_state_dict(sd, cfg, "cuda", **kw)
        full_w = EngineWeights.from_state_dict(sd, cfg, "cuda") if rank == 0 else None
        del sd
        torch.cuda.empty_cache()
        # every mode decodes through captured graphs; a2a's decode exchanges run on the IPC
        # kernels (parallel.ep_a2a), its prefill (exact counts) over gloo
        graphs = True
        eng = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_batch=2, comm=TPComm(),
                     tp_rank=w.tp_rank, tp_size=w.tp_size, use_graph=graphs,
                     ep_mode=mode if moe else "allreduce")
        prompts = _prompts(rank, per_rank=(mode == "a2a"))
        n_new = 8
        torch.cuda.synchronize()
        dist.barrier()  # every rank built (rank 0 also holds the TP=1 weights) before decoding
        res = eng.generate(prompts, n_new, stop_on_eos=False)
        toks = [r.tokens for r in res]
        gs = list(eng._graphs.values())
        assert not graphs or (gs and all(g.graph is not None for g in gs)), \
            "decode graph not captured at world %d" % WORLD
        toks2 = [r.tokens for r in eng.generate(prompts, n_new, stop_on_eos=False)]  # replays
        assert toks2 == toks, ("graph replay changed the tokens", toks, toks2)
        # prefill logits (TP: the rank's vocab shard; EP: full vocab on every rank)
        pages = [eng.kv.allocator.alloc(2) for _ in prompts]
        _, lg = eng.prefill(prompts, pages, return_logits=True)
        for p in pages:
            eng.kv.allocator.free(p)
        eng.check_comm()
        lg = lg.float().cpu()
        if not moe:
            parts = [torch.empty_like(lg) for _ in range(WORLD)]
            dist.all_gather(parts, lg)
            lg = torch.cat(parts, 1)
        msg = "ok"
        if rank == 0:
            ref_eng = Engine(cfg, weights=full_w, device="cuda", kv_pages=64, max_batch=8,
                             use_graph=False)
            pages = [ref_eng.kv.allocator.alloc(2) for _ in prompts]
            _, ref = ref_eng.prefill(prompts, pages, return_logits=True)
            for p in pages:
                ref_eng.kv.allocator.free(p)
            _check_logits(lg, ref.float().cpu(), "%s/%s prefill logits" % (kind, mode))
            # every generated token is a (bf16-tolerance) argmax of the TP=1 model there
            for b, p in enumerate(prompts):
                seqs = [p + toks[b][:j] for j in range(n_new)]
                pg = [ref_eng.kv.allocator.alloc(2) for _ in seqs]
                _, ref_l = ref_eng.prefill(seqs, pg, return_logits=True)
                for x in pg:
                    ref_eng.kv.allocator.free(x)
                ref_l = ref_l.float().cpu()
                for j in range(n_new):
                    row = ref_l[j]
                    gap = (row.max() - row[toks[b][j]]).item()
                    assert gap <= 0.05 * row.std().item() + 0.02, (
                        "%s/%s seq %d step %d: token %d is %.4f below the TP=1 max"
                        % (kind, mode, b, j, toks[b][j], gap))
            msg = "tokens %s" % toks
        q.put((rank, True, msg))
    except Exception:
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        try:
            eng.model.comm.close()
        except Exception:
            pass
        dist.destroy_process_group()


# TP=4 and TP=8 run the fused all-reduce epilogue (ops.skinny_gemm_ar).  Its workgroups wait
# in place for the same column group of every peer, so every rank's grid must be resident at
# once and every rank PROCESS scheduled at once: true on a node with a GPU per rank, not by
# default for virtual ranks sharing one device (profiles/r6_fused_ar.md):
#  * residency: round 5's TP=4 case deadlocked until the spin bound (4 ranks x 256 workgroups
#    x 8 waves > the device's wave slots).  Since round 6 each rank's fused launch holds at most
#    half of its 1/n share of the device's block slots (CustomAllReduce.coresident ->
#    p2p_far_set_coresident) and walks the column groups in a grid-stride loop;
#  * co-scheduling: with a 9th process holding a GPU context on the device (the pytest
#    process itself, once any in-process GPU test has run), the TP=8 case stalled until the
#    spin bound on every run; with the 8 rank processes alone it passes.  So the TP=8 fused
#    case runs only when this process has not initialised HIP (its own pytest process).
# The unfused pair keeps a case of its own.
@pytest.mark.parametrize("kind,mode,world,env", [
    ("dense", "tp", 8, {}),
    ("dense", "tp", 4, {}),
    ("dense", "tp", 8, {"P2P_TP_FUSED_AR": "0"}),
    ("moe", "allreduce", 8, {}), ("moe", "a2a", 8, {})])
def test_world8_virtual_ranks_full_width(kind, mode, world, env):
    if (world >= 8 and kind == "dense" and env.get("P2P_TP_FUSED_AR", "1") == "1"
            and torch.cuda.is_initialized()):
        pytest.skip("this pytest process holds a GPU context: 9 processes on one device are "
                    "not co-scheduled, which the fused epilogue's in-place waits need "
                    "(run this case in a pytest process of its own)")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, kind, mode, env))
          for r in range(world)]
    [p.start() for p in ps]
    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=240))
    finally:
        [p.join(timeout=30) for p in ps]
        [p.terminate() for p in ps if p.is_alive()]
    for rank, ok, info in sorted(res):
        if not ok:
            print("rank %d failed:\n%s" % (rank, info))
    for rank, ok, info in sorted(res):
        assert ok, (rank, info)
    print([info for rank, _, info in res if rank == 0][0])
