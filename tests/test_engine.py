"""End-to-end engine numerics: tiny-llama (CPU plumbing config) and GPU paths.

Greedy comparisons are teacher-forced: the engine's logits for the reference's
token stream must match the fp32 oracle within bf16 tolerance, and the engine's
argmax must equal the oracle's wherever the oracle's top-2 margin is not a
near-tie (random-init models have many near-ties).
"""
import numpy as np
import pytest
import torch

from p2p_llm_chat_go_amd import ops
from p2p_llm_chat_go_amd.engine import Engine
from p2p_llm_chat_go_amd.models import TINY_LLAMA
from p2p_llm_chat_go_amd.models.reference import (random_state_dict, reference_forward,
                                                  reference_greedy)
from p2p_llm_chat_go_amd.models.weights import EngineWeights


def _check_prefill_logits(eng, sd, cfg, prompts):
    """Engine prefill logits of the last prompt token vs oracle."""
    from p2p_llm_chat_go_amd.engine.kv_cache import pages_for

    pages = [eng.kv.allocator.alloc(pages_for(len(p) + 1)) for p in prompts]
    try:
        _first, logits = eng.prefill(prompts, pages, return_logits=True)
        logits = logits.float().cpu()
    finally:
        for p in pages:
            eng.kv.allocator.free(p)
    for b, p in enumerate(prompts):
        ref = reference_forward(sd, cfg, torch.tensor(p))[-1]
        rel = (logits[b] - ref).norm() / ref.norm()
        assert rel < 3e-2, rel


def _greedy_ok(sd, cfg, prompt, got, margin=2e-2):
    toks = list(prompt)
    for t in got:
        ref = reference_forward(sd, cfg, torch.tensor(toks))[-1]
        top = ref.topk(2)
        if int(top.indices[0]) != t:
            gap = float(top.values[0] - ref[t])
            assert gap < margin * float(ref.abs().max()), (t, top, gap)
        toks.append(t)


@pytest.mark.parametrize("chunk", [16, 1024])
def test_tiny_engine_cpu(chunk):
    cfg = TINY_LLAMA
    sd = random_state_dict(cfg, seed=1)
    w = EngineWeights.from_state_dict(sd, cfg, "cpu")
    eng = Engine(cfg, weights=w, device="cpu", kv_pages=64, max_prefill_tokens=chunk, max_batch=4)
    prompts = [[1, 5, 9, 33, 100, 7], list(range(3, 40)), [4]]
    _check_prefill_logits(eng, sd, cfg, prompts)
    res = eng.generate(prompts, max_new_tokens=6, stop_on_eos=False)
    for p, r in zip(prompts, res):
        assert len(r.tokens) == 6
        _greedy_ok(sd, cfg, p, r.tokens)
    assert res[0].tokens == reference_greedy(sd, cfg, prompts[0], 6)


def test_engine_stop_on_eos_cpu():
    cfg = TINY_LLAMA.replace(eos_ids=tuple(range(0, 512)))  # every token is EOS
    sd = random_state_dict(cfg, seed=2)
    eng = Engine(cfg, weights=EngineWeights.from_state_dict(sd, cfg, "cpu"), device="cpu",
                 kv_pages=16)
    r = eng.generate([[3, 4, 5]], max_new_tokens=10)[0]
    assert r.tokens == [] and r.done_reason == "stop"


@pytest.mark.gpu
@pytest.mark.parametrize("use_graph", [False, True])
def test_tiny_engine_gpu(use_graph):
    cfg = TINY_LLAMA
    sd = random_state_dict(cfg, seed=1)
    w = EngineWeights.from_state_dict(sd, cfg, "cuda")
    eng = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_prefill_tokens=16, max_batch=4,
                 use_graph=use_graph)
    prompts = [[1, 5, 9, 33, 100, 7], list(range(3, 40)), [4]]
    _check_prefill_logits(eng, sd, cfg, prompts)
    res = eng.generate(prompts, max_new_tokens=8, stop_on_eos=False)
    for p, r in zip(prompts, res):
        assert len(r.tokens) == 8
        _greedy_ok(sd, cfg, p, r.tokens)


@pytest.mark.gpu
def test_graph_equals_eager_gpu():
    cfg = TINY_LLAMA.replace(n_layers=3)
    w = EngineWeights.random(cfg, "cuda", seed=3)
    prompts = [[1, 2, 3, 4, 5], [9] * 70]
    outs = []
    for g in (False, True):
        eng = Engine(cfg, weights=w, device="cuda", kv_pages=32, max_batch=2, use_graph=g)
        outs.append([r.tokens for r in eng.generate(prompts, 20, stop_on_eos=False)])
    assert outs[0] == outs[1]


@pytest.mark.gpu
def test_llama8b_two_layers_gpu():
    from p2p_llm_chat_go_amd.models import LLAMA31_8B

    cfg = LLAMA31_8B.replace(n_layers=2)
    sd = random_state_dict(cfg, seed=4)
    w = EngineWeights.from_state_dict(sd, cfg, "cuda")
    eng = Engine(cfg, weights=w, device="cuda", kv_pages=16, max_batch=2)
    prompts = [list(range(100, 150))]
    _check_prefill_logits(eng, sd, cfg, prompts)
    r = eng.generate(prompts, 4, stop_on_eos=False)[0]
    _greedy_ok(sd, cfg, prompts[0], r.tokens)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_tiny_mixtral(dev):
    from p2p_llm_chat_go_amd.models import TINY_MIXTRAL

    cfg = TINY_MIXTRAL
    sd = random_state_dict(cfg, seed=5)
    w = EngineWeights.from_state_dict(sd, cfg, dev)
    eng = Engine(cfg, weights=w, device=dev, kv_pages=64, max_prefill_tokens=100, max_batch=4)
    prompts = [[1, 5, 9, 33, 100, 7], list(range(3, 90)), [4]]
    _check_prefill_logits(eng, sd, cfg, prompts)
    res = eng.generate(prompts, max_new_tokens=6, stop_on_eos=False)
    for p, r in zip(prompts, res):
        _greedy_ok(sd, cfg, p, r.tokens)


@pytest.mark.gpu
def test_sampled_decode_graph_gpu():
    """Sampled decode steps are one graph replay each (forward + ops.sample + advance):
    temperature 0 rows reproduce the greedy graph exactly; a fixed seed reproduces a
    sampled continuation, graph == eager."""
    from p2p_llm_chat_go_amd.engine.sampling import SamplingParams

    cfg = TINY_LLAMA.replace(n_layers=2)
    w = EngineWeights.random(cfg, "cuda", seed=9)
    prompts = [[1, 2, 3, 4, 5], [7] * 40]

    def run(greedy, params, use_graph=True, n=12):
        eng = Engine(cfg, weights=w, device="cuda", kv_pages=32, max_batch=2,
                     use_graph=use_graph)
        pages = [eng.kv.allocator.alloc(2) for _ in prompts]
        first = eng.prefill(prompts, pages).cpu().tolist()
        g = eng.decode_graph(2, 128, greedy=greedy)
        g.state.load(first, [len(p) for p in prompts], pages)
        if greedy:
            g.replay(n)
        else:
            g.step_sampled(params, n)
        return g.state.hist[:2, :n].cpu().tolist()

    ref = run(True, None)
    assert run(False, [SamplingParams(temperature=0.0)] * 2) == ref
    hot = [SamplingParams(temperature=1.3, top_k=64, top_p=0.95, seed=s) for s in (5, 6)]
    a = run(False, hot)
    assert a == run(False, hot) == run(False, hot, use_graph=False)
    assert a != ref


def test_fp8_quantize_roundtrip_cpu():
    from p2p_llm_chat_go_amd import ops

    torch.manual_seed(0)
    W = (torch.randn(256, 512) * 0.03).to(torch.bfloat16)
    q = ops.quantize_fp8(ops.tile_weight(W))
    assert q.data.dtype == torch.uint8 and q.data.shape == (16, 16, 64, 8)
    assert q.scale.shape == (256,)
    Wd = ops.untile_weight(q.dequantize()).float()
    # e4m3: 3 mantissa bits -> relative error <= 2^-4 per element (normal range)
    err = (Wd - W.float()).abs() / W.float().abs().amax(1, keepdim=True)
    assert err.max() < 0.07
    assert ((Wd - W.float()).norm() / W.float().norm()) < 0.04


def test_fp8_pair_layout_cpu():
    """Lane l's 16 bytes at pair p = its fragment of k-step 2p, then of k-step 2p+1."""
    from p2p_llm_chat_go_amd import ops

    t = torch.randint(0, 256, (3, 6, 64, 8), dtype=torch.uint8)
    p = ops.gemm.pair_f8(t)
    assert p.shape == t.shape
    flat = p.reshape(3, 3, 64, 16)
    for g, pp, lane in [(0, 0, 0), (1, 2, 17), (2, 1, 63)]:
        assert torch.equal(flat[g, pp, lane, :8], t[g, 2 * pp, lane])
        assert torch.equal(flat[g, pp, lane, 8:], t[g, 2 * pp + 1, lane])
    assert torch.equal(ops.gemm.unpair_f8(p), t)
    with pytest.raises(AssertionError):
        ops.quantize_fp8(ops.tile_weight(torch.randn(16, 96).to(torch.bfloat16)))


def test_fp8_engine_cpu_matches_dequantized_weights():
    w8 = EngineWeights.random(TINY_LLAMA, "cpu", seed=5)
    e8 = Engine(TINY_LLAMA, weights=w8, device="cpu", kv_pages=64, max_batch=4,
                weight_dtype="fp8")
    wd = EngineWeights.random(TINY_LLAMA, "cpu", seed=5)
    for lw, l8 in zip(wd.layers, e8.weights.layers):
        for n in ("qkv", "o", "gate_up", "down"):
            setattr(lw, n, getattr(l8, n).dequantize())
    if isinstance(e8.weights.lm_head, ops.Fp8Weight):  # fp8 mode quantizes the LM head too
        wd.lm_head = e8.weights.lm_head.dequantize()
    ed = Engine(TINY_LLAMA, weights=wd, device="cpu", kv_pages=64, max_batch=4)
    prompts = [[1, 5, 9, 200, 31], [7, 7, 3]]
    a = e8.generate(prompts, max_new_tokens=6)
    b = ed.generate(prompts, max_new_tokens=6)
    assert [r.tokens for r in a] == [r.tokens for r in b]
    assert e8.weights.nbytes() < 0.75 * EngineWeights.random(TINY_LLAMA, "cpu", seed=5).nbytes()
    with pytest.raises(ValueError):
        Engine(TINY_LLAMA, device="cpu", kv_pages=8, weight_dtype="int3")


@pytest.mark.parametrize("name", ["tiny-llama-gqa", "tiny-mixtral"])
def test_lazy_safetensors_reads_shard_slices(tmp_path, name):
    """A TP rank built from a LazySafetensors checkpoint reads only its slice of every
    sharded tensor (get_slice) and gets the same weights as slicing the full tensors."""
    from safetensors.torch import save_file

    from p2p_llm_chat_go_amd.models.config import get_config
    from p2p_llm_chat_go_amd.models.reference import random_state_dict
    from p2p_llm_chat_go_amd.models.weights import EngineWeights, LazySafetensors

    cfg = get_config(name)
    sd = random_state_dict(cfg, seed=3)
    half = sorted(sd)[:len(sd) // 2]
    save_file({k: sd[k].contiguous() for k in half}, str(tmp_path / "a.safetensors"))
    save_file({k: sd[k].contiguous() for k in sd if k not in half}, str(tmp_path / "b.safetensors"))
    lazy = LazySafetensors(str(tmp_path))
    reads = []
    orig = lazy.get_rows_cols

    def spy(n, rows=None, cols=None):
        t = orig(n, rows, cols)
        reads.append((n, tuple(t.shape), tuple(sd[n].shape)))
        return t
    lazy.get_rows_cols = spy
    tp = 2 if cfg.n_kv_heads % 2 == 0 else 1
    for r in range(tp):
        a = EngineWeights.from_state_dict(sd, cfg, "cpu", tp_rank=r, tp_size=tp)
        b = EngineWeights.from_state_dict(lazy, cfg, "cpu", tp_rank=r, tp_size=tp)
        assert torch.equal(a.lm_head, b.lm_head) and torch.equal(a.embed, b.embed)
        for la, lb in zip(a.layers, b.layers):
            for f in ("qkv", "o", "gate_up", "down", "router", "w13", "w2"):
                x, y = getattr(la, f), getattr(lb, f)
                assert (x is None and y is None) or torch.equal(x, y), f
    if tp > 1:  # projections came off the disk as shards, not whole tensors
        q = [x for x in reads if x[0].endswith("q_proj.weight")]
        assert q and all(got[0] * tp == full[0] for _n, got, full in q)
        o = [x for x in reads if x[0].endswith("o_proj.weight")]
        assert o and all(got[1] * tp == full[1] for _n, got, full in o)


@pytest.mark.parametrize("rows,n_seq,pages,real", [(384, 8, 4, []), (1024, 8, 4, []),
                                                     (384, 8, 4, [(0, 40), (1, 250)]),
                                                     (64, 2, 1, [(0, 5)])])
def test_prefill_graph_host_meta(rows, n_seq, pages, real):
    """PrefillGraph.host_meta on the host: dummy rows (slot -1, the null-page sequence) keep
    positions inside their block-table row even when the row bucket holds more rows than
    the context bucket has positions (the capture-time image has no real rows at all), and
    the query tiles cover every row, never straddle sequences and fit the bound."""
    import types

    from p2p_llm_chat_go_amd.engine.graph import PAGE, PrefillGraph

    g = PrefillGraph(types.SimpleNamespace(device="cpu", nq=32, nkv=8), None, rows, n_seq,
                     pages, pages * PAGE)
    rws, bts, outs = [], [], []
    for s, L in real:
        bts.append([3 + s * pages + i for i in range(-(-L // PAGE))])
        rws += [(s, i, 7) for i in range(L)]
        outs.append(len(rws) - 1)
    host = g.host_meta(rws, bts, outs).numpy()
    v = {k: host[a:a + n] for k, (a, n) in g.offsets.items()}
    n = len(rws)
    assert (v["pos"] < pages * PAGE).all() and (v["pos"] >= 0).all()
    assert (v["slots"][n:] == -1).all() and (v["seq"][n:] == n_seq).all()
    for r, (s, i, _t) in enumerate(rws):
        assert v["slots"][r] == bts[s][i // PAGE] * PAGE + i % PAGE
    assert (v["ctx"] == v["pos"] + 1).all()
    covered = np.zeros(rows, int)
    for r0, k, sq, p0 in v["tiles"].reshape(-1, 4):
        if k:
            assert (v["seq"][r0:r0 + k] == sq).all()
            assert (v["pos"][r0:r0 + k] == p0 + np.arange(k)).all()
            covered[r0:r0 + k] += 1
    assert (covered == 1).all()


def test_prefill_graph_host_meta_long_allocation():
    """a caller passes the sequence's whole page allocation (prompt +
    max_new tokens), which can be wider than the chunk's context bucket; host_meta keeps the
    first max_pages pages (the only ones the chunk reads) instead of asserting."""
    import types

    from p2p_llm_chat_go_amd.engine.graph import PAGE, PrefillGraph

    pages = 4  # a 256-token context bucket
    g = PrefillGraph(types.SimpleNamespace(device="cpu", nq=32, nkv=8), None, 256, 1, pages,
                     pages * PAGE)
    alloc = [11, 12, 13, 14, 15, 16]  # 200-token prompt + 128 new tokens: 6 pages
    rws = [(0, i, 5) for i in range(200)]
    host = g.host_meta(rws, [alloc], [199]).numpy()
    v = {k: host[a:a + n] for k, (a, n) in g.offsets.items()}
    assert list(v["bt"][:pages]) == alloc[:pages]
    assert v["slots"][199] == alloc[199 // PAGE] * PAGE + 199 % PAGE
    with pytest.raises(AssertionError):  # a row past the context bucket is a caller bug
        g.host_meta([(0, 300, 5)], [alloc], [0])


@pytest.mark.gpu
@pytest.mark.parametrize("lens", [[44], [5, 37, 12], [60, 3], [130], [44] * 7])
def test_prefill_graph_equals_eager_gpu(lens):
    """A graph-captured prefill chunk (engine.graph.PrefillGraph: padded row bucket,
    padding tiles, dummy rows on the null page) gives the eager prefill's first tokens,
    logits and KV cache contents, and decoding continues identically."""
    from p2p_llm_chat_go_amd.models import LLAMA31_8B

    cfg = LLAMA31_8B.replace(n_layers=2)
    w = EngineWeights.random(cfg, "cuda", seed=11)
    prompts = [[(37 * b + 11 * i) % 5000 + 100 for i in range(L)] for b, L in enumerate(lens)]
    out = {}
    for graph in (False, True):
        eng = Engine(cfg, weights=w, device="cuda", kv_pages=64, max_batch=8)
        assert eng.prefill_graphs_enabled
        eng.prefill_graphs_enabled = graph
        eng.prefill_graph_after = 1  # capture on first use
        pages = [eng.kv.allocator.alloc(3) for _ in prompts]
        first = eng.prefill(prompts, pages).cpu()
        assert bool(eng._pgraphs) == graph
        kv = []
        for i in range(cfg.n_layers):
            kc, vc = eng.kv.layer(i)
            for b, p in enumerate(prompts):
                pos = torch.arange(len(p))
                pg = torch.tensor(pages[b])[pos // 64].cuda()
                kv.append(kc[pg, :, (pos % 64).cuda()].float().cpu())
                kv.append(vc[pg, :, (pos % 64).cuda()].float().cpu())
        if graph:  # the sampled-request graph's logits vs the eager return_logits path
            rows = [(b, i, t) for b, p in enumerate(prompts) for i, t in enumerate(p)]
            last = [sum(lens[:b + 1]) - 1 for b in range(len(lens))]
            g = eng.prefill_graph(len(rows), len(prompts), max(lens), greedy=False)
            g.load(g.host_meta(rows, pages, last))
            g.replay()
            logits = g.ws.logits[:len(prompts)].float().cpu()
        else:
            _f, logits = eng.prefill(prompts, pages, return_logits=True)
            logits = logits.float().cpu()
        for p in pages:
            eng.kv.allocator.free(p)
        gen = [r.tokens for r in eng.generate(prompts, 12, stop_on_eos=False)]
        out[graph] = (first, kv, logits, gen, eng)
    (f0, kv0, l0, g0, eager), (f1, kv1, l1, g1, _) = out[False], out[True]
    assert torch.equal(f0, f1)
    for a, b in zip(kv0, kv1):
        assert (a - b).abs().max() <= 1e-2 * max(1.0, float(a.abs().max()))
    assert ((l0 - l1).norm() / l0.norm()) < 1e-2
    # decoding continues identically -- up to a near-tie of the random model, which the
    # padded chunk's different GEMM shape may round the other way: check its margin
    for p, a, b in zip(prompts, g0, g1):
        if a == b:
            continue
        j = next(i for i, (x, y) in enumerate(zip(a, b)) if x != y)
        toks = p + a[:j]
        pages = eager.kv.allocator.alloc(-(-len(toks) // 64))
        _f, lg = eager.prefill([toks], [pages], return_logits=True)
        eager.kv.allocator.free(pages)
        lg = lg[0].float().cpu()
        assert abs(float(lg[a[j]] - lg[b[j]])) < 2e-2 * float(lg.abs().max()), (j, a, b)
