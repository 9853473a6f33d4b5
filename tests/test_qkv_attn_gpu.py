"""Decode qkv + RoPE + KV write + attention in one launch (ops.qkv_attn,
csrc/kernels/qkv_attn.hip) against the two-kernel path (skinny qkv+RoPE GEMM, then the
paged-attention kernel) and against the fp32 PyTorch reference of the same math: GQA
ratios 1/2/4/8, 1..16 rows with ragged contexts up to 256 keys, repeated calls on the
same hand-off buffers (tags advance), and hipGraph replay."""
import math

import pytest
import torch

from p2p_llm_chat_go_amd import ops
from p2p_llm_chat_go_amd.models.config import TINY_LLAMA, rope_table
from p2p_llm_chat_go_amd.ops.attention import paged_attention_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(M, Hq, Hkv, K, seed, max_keys=256):
    g = torch.Generator().manual_seed(seed)
    N = (Hq + 2 * Hkv) * 128
    w = torch.randn(N, K, generator=g) * 0.05
    wt = ops.tile_weight(w.to(torch.bfloat16)).to(DEV)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    ctx = torch.randint(1, max_keys + 1, (M,), generator=g, dtype=torch.int32)
    ctx[0] = max_keys
    if M > 1:
        ctx[1] = 1
    P = 1 + 4 * M
    kc = (torch.randn(P, Hkv, 64, 128, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    vc = torch.randn(P, Hkv, 64, 128, generator=g).to(torch.bfloat16).to(DEV)
    bt = (torch.randperm(P - 1, generator=g)[:4 * M] + 1).view(M, 4).to(torch.int32)
    pos = (ctx - 1).to(torch.int32)
    slots = (bt[torch.arange(M), (pos // 64).long()] * 64 + pos % 64).to(torch.int32)
    cs = rope_table(TINY_LLAMA.replace(rope_theta=5e5), max_pos=512, device=DEV)
    return dict(wt=wt, x=x, ctx=ctx.to(DEV), kc=kc, vc=vc, bt=bt.to(DEV), pos=pos.to(DEV),
                slots=slots.to(DEV), cs=cs)


def _two_kernel(d, Hq, Hkv, kc, vc):
    M = d["x"].shape[0]
    q = torch.zeros(M, Hq * 128, dtype=torch.bfloat16, device=DEV)
    ops.qkv_rope_gemm(d["wt"], d["x"], d["pos"], d["slots"], d["cs"], Hq, Hkv, q, kc, vc)
    out = ops.paged_attention(q, kc, vc, d["bt"], None, d["ctx"], Hq, Hkv, 256)
    return q, out


@pytest.mark.parametrize("ks,kw", [(1, 4), (2, 4), (3, 4), (6, 4), (1, 2), (2, 2)])
@pytest.mark.parametrize("M,Hq,Hkv,K", [(1, 32, 8, 4096), (3, 32, 8, 1024), (16, 32, 8, 1024),
                                        (1, 8, 1, 8192), (5, 8, 1, 1024), (2, 4, 4, 512),
                                        (4, 16, 8, 512)])
def test_qkv_attn_matches_two_kernels(M, Hq, Hkv, K, ks, kw):
    """ks > 1: k-split producers (fp32 partials, the consumer sums them in slice order and
    applies rstd, RoPE and the KV write itself); kw = 2: consumers with two key waves for
    contexts <= 128 keys."""
    if (K // 32) // ks < 4:
        pytest.skip("fewer than 4 k-steps per slice")
    d = _setup(M, Hq, Hkv, K, seed=M * 100 + Hq + K, max_keys=64 * kw)
    kc1, vc1 = d["kc"].clone(), d["vc"].clone()
    q_ref, ref = _two_kernel(d, Hq, Hkv, kc1, vc1)
    # fp32 reference of the attention on the two-kernel path's q and cache
    ref32 = paged_attention_ref(q_ref.cpu(), kc1.cpu(), vc1.cpu(), d["bt"].cpu(), None,
                                d["ctx"].cpu(), Hq, Hkv, 1 / math.sqrt(128),
                                torch.empty(M, Hq * 128, dtype=torch.float32))
    ws = ops.qkv_attn_workspace(M, Hq, Hkv, DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    for rep in range(3):  # the hand-off tags advance call by call on the same buffers
        kc2, vc2 = d["kc"].clone(), d["vc"].clone()
        out = torch.full((M, Hq * 128), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.qkv_attn(d["wt"], d["x"], d["pos"], d["slots"], d["cs"], Hq, Hkv, kc2, vc2, d["bt"],
                     d["ctx"], out, ws, err, waves=(ks << 8) | ((kw if kw == 2 else 0) << 16))
        torch.cuda.synchronize()
        assert int(err.item()) == 0, "hand-off timed out"
        assert not out.isnan().any()
        # the current token's k / v reach the cache as the skinny epilogue writes them (the
        # fp32 sums may round differently in the last bf16 bit: a handful of 1-ulp flips;
        # k-split sums slice partials in another order: up to 1/16 of the row's values)
        for name, a_, b_ in (("k", kc2, kc1), ("v", vc2, vc1)):
            assert torch.allclose(a_.float(), b_.float(), rtol=1e-2, atol=1e-3), (rep, name)
            assert int((a_ != b_).sum()) <= (8 if ks == 1 else M * Hkv * 16), (
                rep, name, int((a_ != b_).sum()))
        rel = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        assert rel < 2e-2, (rep, rel)
        rel32 = ((out.cpu().float() - ref32).abs().max() / ref32.abs().max()).item()
        assert rel32 < 2e-2, (rep, rel32)


def test_qkv_attn_graph_replay():
    M, Hq, Hkv, K = 2, 32, 8, 1024
    d = _setup(M, Hq, Hkv, K, seed=7)
    kc1, vc1 = d["kc"].clone(), d["vc"].clone()
    _q, ref = _two_kernel(d, Hq, Hkv, kc1, vc1)
    ws = ops.qkv_attn_workspace(M, Hq, Hkv, DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    kc2, vc2 = d["kc"].clone(), d["vc"].clone()
    out = torch.zeros(M, Hq * 128, dtype=torch.bfloat16, device=DEV)

    def body():
        ops.qkv_attn(d["wt"], d["x"], d["pos"], d["slots"], d["cs"], Hq, Hkv, kc2, vc2, d["bt"],
                     d["ctx"], out, ws, err)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            body()
            body()
    torch.cuda.synchronize()
    for _ in range(4):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        rel = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        assert rel < 2e-2, rel


@pytest.mark.parametrize("M,Hq,Hkv,K,No", [(1, 32, 8, 4096, 4096), (3, 32, 8, 1024, 512),
                                           (16, 32, 8, 1024, 256), (9, 32, 8, 4096, 4096),
                                           (5, 8, 2, 1024, 1024), (2, 4, 4, 512, 256)])
def test_qkv_attn_oproj_matches_unfused(M, Hq, Hkv, K, No):
    """o_proj (+ residual) inside the qkv+attention launch == qkv_attn followed by the
    o_proj GEMM (skinny, EPI_RESID), and == the fp32 reference of attention @ Wo^T + h;
    repeated calls and graph replays advance the granule epoch on the same buffers."""
    d = _setup(M, Hq, Hkv, K, seed=M * 31 + Hq + No)
    g = torch.Generator().manual_seed(M + No)
    wo32 = torch.randn(No, Hq * 128, generator=g) * 0.03
    wo = ops.tile_weight(wo32.to(torch.bfloat16)).to(DEV)
    assert ops.qkv_attn_oproj_ok(wo, Hq, Hkv, rows=M, hidden=K)
    # a 70B TP=8 rank's o_proj (512 column groups) has more groups than producers (80)
    assert not ops.qkv_attn_oproj_ok(torch.empty(512, 32, 64, 8, dtype=torch.bfloat16), 8, 1)
    h0 = torch.randn(M, No, generator=g).to(torch.bfloat16).to(DEV)
    ws = ops.qkv_attn_workspace(M, Hq, Hkv, DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    # unfused reference on the same kernels
    kc1, vc1 = d["kc"].clone(), d["vc"].clone()
    attn = torch.zeros(M, Hq * 128, dtype=torch.bfloat16, device=DEV)
    ops.qkv_attn(d["wt"], d["x"], d["pos"], d["slots"], d["cs"], Hq, Hkv, kc1, vc1, d["bt"],
                 d["ctx"], attn, ws, err)
    h_ref = h0.clone()
    ops.skinny_gemm(wo, attn, ops.EPI_RESID, out=h_ref)
    ref32 = h0.float().cpu() + attn.float().cpu() @ wo32.to(torch.bfloat16).float().t()
    torch.cuda.synchronize()
    for rep in range(3):
        kc2, vc2 = d["kc"].clone(), d["vc"].clone()
        h = h0.clone()
        ops.qkv_attn(d["wt"], d["x"], d["pos"], d["slots"], d["cs"], Hq, Hkv, kc2, vc2, d["bt"],
                     d["ctx"], None, ws, err, oproj=(wo, h))
        torch.cuda.synchronize()
        assert int(err.item()) == 0, "granule sweep timed out"
        for a_, b_ in ((kc2, kc1), (vc2, vc1)):
            assert int((a_ != b_).sum()) <= 8
        rel = ((h.float() - h_ref.float()).abs().max() / h_ref.float().abs().max()).item()
        assert rel < 1e-2, (rep, rel)
        rel32 = ((h.float().cpu() - ref32).abs().max() / ref32.abs().max()).item()
        assert rel32 < 2e-2, (rep, rel32)
    # graph capture + replays (the epoch advances inside the graph)
    hg = h0.clone()
    kc3, vc3 = d["kc"].clone(), d["vc"].clone()

    def body():
        hg.copy_(h0)
        ops.qkv_attn(d["wt"], d["x"], d["pos"], d["slots"], d["cs"], Hq, Hkv, kc3, vc3, d["bt"],
                     d["ctx"], None, ws, err, oproj=(wo, hg))

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            body()
            body()
    torch.cuda.synchronize()
    for _ in range(3):
        gr.replay()
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        rel = ((hg.float() - h_ref.float()).abs().max() / h_ref.float().abs().max()).item()
        assert rel < 1e-2, rel
