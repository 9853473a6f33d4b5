"""Debug: per-row / per-column errors of ops.attn_oproj_heads vs the two-kernel path."""
import math
import sys

import torch

sys.path.insert(0, ".")
from p2p_llm_chat_go_amd import ops  # noqa: E402
from p2p_llm_chat_go_amd.ops import attention as A  # noqa: E402

DEV = "cuda"
for R, Hkv, G, ctxs in [(3, 2, 2, [1, 17, 256]), (2, 8, 4, [100, 100]), (3, 8, 4, [50, 60, 70]),
                        (3, 2, 2, [100, 100, 100]), (2, 2, 2, [1, 17])]:
    torch.manual_seed(0)
    Hq = Hkv * G
    K = Hq * 128
    N = 256 if K < 4096 else 4096
    npg = 4
    P = 1 + R * npg
    k = torch.randn(P, Hkv, 64, 128).to(torch.bfloat16)
    v = torch.randn(P, Hkv, 64, 128).to(torch.bfloat16)
    bt = (torch.randperm(P - 1)[:R * npg] + 1).view(R, npg).to(torch.int32)
    q = torch.randn(R, Hq * 128).to(torch.bfloat16)
    ctx = torch.tensor(ctxs, dtype=torch.int32)
    Wo = (torch.randn(N, K) * 0.02).to(torch.bfloat16)
    h0 = torch.randn(R, N).to(torch.bfloat16)
    d = {n: t.to(DEV) for n, t in dict(q=q, k=k, v=v, bt=bt, ctx=ctx).items()}
    wt = ops.tile_weight(Wo).to(DEV)
    attn = torch.zeros(R, Hq * 128, dtype=torch.bfloat16, device=DEV)
    ops.paged_attention(d["q"], d["k"], d["v"], d["bt"], None, d["ctx"], Hq, Hkv, 256, out=attn)
    href = h0.to(DEV)
    ops.skinny_gemm(wt, attn, ops.EPI_RESID, out=href)
    slab, tickets = ops.attn_oproj_heads_workspace(R, Hkv, N, DEV)
    h = h0.to(DEV)
    a2 = torch.zeros_like(attn)
    ops.attn_oproj_heads(d["q"], d["k"], d["v"], d["bt"], None, d["ctx"], Hq, Hkv, 256, wt, h,
                         slab, tickets, attn=a2)
    torch.cuda.synchronize()
    err = (h.float() - href.float()).abs()
    print("R", R, "Hkv", Hkv, "G", G, "attn maxdiff", [round(x,4) for x in (a2.float() - attn.float()).abs().max(1).values.tolist()],
          "h maxdiff per row", [round(x, 4) for x in err.max(1).values.tolist()])
    bad = (err > 0.05).nonzero()
    if len(bad):
        cols = bad[:, 1].unique()
        print("  bad cols", cols.numel(), "first", cols[:20].tolist())
        # which partial slab rows look wrong: compare each head partial to reference
        sl = slab.view(Hkv, R, N)
        for g in range(Hkv):
            ref_p = attn[:, g * G * 128:(g + 1) * G * 128].float() @ Wo[:, g * G * 128:(g + 1) * G * 128].float().t().to(DEV)
            print("  head", g, "partial maxdiff per row",
                  [round(x, 4) for x in (sl[g] - ref_p).abs().max(1).values.tolist()])
    if len(bad):
        Wd = Wo.float().to(DEV)
        af = attn.float()
        for g in range(Hkv):
            for r in range(R):
                tgt = sl[g][r]
                best = []
                for g2 in range(Hkv):
                    for r2 in range(R):
                        cand = af[r2, g2 * G * 128:(g2 + 1) * G * 128] @ Wd[:, g * G * 128:(g + 1) * G * 128].t()
                        best.append(((tgt - cand).abs().max().item(), g2, r2))
                # sums of rows
                cand = af[:, g * G * 128:(g + 1) * G * 128].sum(0) @ Wd[:, g * G * 128:(g + 1) * G * 128].t()
                best.append(((tgt - cand).abs().max().item(), "sum", "rows"))
                best.sort(key=lambda x: x[0])
                print("  slab[g=%d][r=%d] best match" % (g, r), best[:2])
        break
