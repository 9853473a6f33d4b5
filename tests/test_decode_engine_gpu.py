"""The persistent decode engine (csrc/kernels/decode_engine.hip, ops.decode_engine): every
layer of a decode step in one launch must give what the per-layer launches give -- the
final residual, the logits, this token's K/V in the paged cache -- for 1-4 rows at
contexts 1-256 (page boundaries, the 4-page limit), over repeated launches (the launch
epoch advances, tags never collide) and inside captured decode graphs (engine.generate).
The reference for both is the skinny-kernel path, itself checked against fp32 PyTorch in
test_kernels_gpu.py; here the tolerance covers the split-K summation order only."""
import pytest
import torch

from p2p_llm_chat_go_amd.engine import Engine
from p2p_llm_chat_go_amd.models import LLAMA31_8B
from p2p_llm_chat_go_amd.models.weights import EngineWeights

pytestmark = pytest.mark.gpu


def _shard_cfg(layers):
    """llama3.1-70B's per-rank shapes at TP=8 as a TP=1 model (bench/decode_engine_bench.py
    --tp8-shard): 8 q heads + 1 kv head, 3584 ffn columns (28 k-steps per wave in down, not
    a multiple of the 8-step batch), o_proj K = 1024 (8 k-steps per wave, under the
    16-fragment prefetch credit), 160 qkv half groups for 256 workgroups."""
    from p2p_llm_chat_go_amd.models.config import get_config

    c = get_config("llama3.1-70b")
    return c.replace(name="llama3.1-70b-tp8-shard", n_heads=c.n_heads // 8, n_kv_heads=1,
                     ffn=c.ffn // 8, vocab=c.vocab // 8, n_layers=layers)


def _setup(ctxs, layers=3, seed=5, shard=False):
    cfg = _shard_cfg(layers) if shard else LLAMA31_8B.replace(n_layers=layers)
    w = EngineWeights.random(cfg, "cuda", seed=seed)
    eng = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_batch=8)
    pages = [eng.kv.allocator.alloc(4) for _ in ctxs]
    V = min(30000, cfg.vocab - 200)
    prompts = [[(31 * b + 7 * i) % V + 100 for i in range(c)] for b, c in enumerate(ctxs)]
    pre = [(p[:-1], pg) for p, pg in zip(prompts, pages) if len(p) > 1]
    if pre:
        eng.prefill([x[0] for x in pre], [x[1] for x in pre])
    return eng, cfg, pages, prompts


def _rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-6))


@pytest.mark.parametrize("ctxs,shard", [([1], False), ([108], False), ([64, 200], False),
                                        ([5, 65, 128, 256], False), ([256, 1, 77], False),
                                        ([108], True), ([5, 200], True)])
def test_decode_engine_matches_layer_launches(ctxs, shard):
    """shard: the 70B TP=8 rank shapes (the engine had refused them)."""
    from p2p_llm_chat_go_amd.ops.decode_engine import decode_engine_ok

    eng, cfg, pages, prompts = _setup(ctxs, shard=shard)
    m = eng.model
    R = len(ctxs)
    assert decode_engine_ok(m, R, 256)
    ws = m.new_workspace(R, 256)
    dev = "cuda"
    ids = torch.tensor([p[-1] for p in prompts], dtype=torch.int32, device=dev)
    pos = torch.tensor([c - 1 for c in ctxs], dtype=torch.int32, device=dev)
    slots = torch.tensor([pages[b][(c - 1) // 64] * 64 + (c - 1) % 64 for b, c in enumerate(ctxs)],
                         dtype=torch.int32, device=dev)
    bt = torch.tensor(pages, dtype=torch.int32, device=dev)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=dev)
    out = {}
    for mode in (False, True, True):  # the engine twice: the launch epoch advances
        m.decode_engine = mode
        logits = m.forward(ws, ids, pos, slots, bt, None, ctx, R, 256).float().clone()
        torch.cuda.synchronize()
        m.check_faults(ws)
        kv = []
        for i in range(cfg.n_layers):
            kc, vc = eng.kv.layer(i)
            for b, c in enumerate(ctxs):
                pg, off = pages[b][(c - 1) // 64], (c - 1) % 64
                kv += [kc[pg, :, off].float().clone(), vc[pg, :, off].float().clone()]
        out.setdefault(mode, []).append((ws.h[:R].float().clone(), logits, kv))
    assert m._de is not None
    h0, l0, kv0 = out[False][0]
    for h1, l1, kv1 in out[True]:
        assert _rel(h1, h0) < 1e-2, _rel(h1, h0)
        assert _rel(l1, l0) < 1e-2, _rel(l1, l0)
        for a, b in zip(kv1, kv0):
            assert _rel(a, b) < 1e-2
    assert int(m._de.epoch[0].item()) == 2 and int(m._de.epoch[1].item()) == 0


@pytest.mark.parametrize("lens", [[44], [5, 37, 12], [130, 9, 60, 1]])
def test_decode_engine_generate_graphs(lens):
    """Captured decode graphs (engine.generate): greedy tokens equal the per-layer launches'
    (up to a near-tie of the random model, whose margin is checked)."""
    cfg = LLAMA31_8B.replace(n_layers=2)
    w = EngineWeights.random(cfg, "cuda", seed=9)
    prompts = [[(37 * b + 11 * i) % 5000 + 100 for i in range(L)] for b, L in enumerate(lens)]
    res = {}
    for mode in (False, True):
        eng = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_batch=4)
        eng.model.decode_engine = mode
        res[mode] = ([r.tokens for r in eng.generate(prompts, 24, stop_on_eos=False)], eng)
        assert (eng.model._de is not None) == mode
    (g0, e0), (g1, _e1) = res[False], res[True]
    for p, a, b in zip(prompts, g1, g0):
        if a == b:
            continue
        j = next(i for i, (x, y) in enumerate(zip(a, b)) if x != y)
        toks = p + b[:j]
        pg = e0.kv.allocator.alloc(-(-len(toks) // 64))
        _f, lg = e0.prefill([toks], [pg], return_logits=True)
        e0.kv.allocator.free(pg)
        lg = lg[0].float().cpu()
        assert abs(float(lg[a[j]] - lg[b[j]])) < 2e-2 * float(lg.abs().max()), (j, a, b)
