"""Mixtral sparse-MoE FFN on the engine kernels (replaces the dense SwiGLU MLP).

Per layer, for R rows (chunks of <= 64 rows on the skinny grouped kernel; above 64 rows
all rows at once on the LDS-tiled grouped kernel, ``moe_forward_tiled``):
    ids, w = top_k(softmax(rstd(h) h Wr'))   moe_router_route (+ per-expert slot lists)
    act[s] = silu(g) * u of expert(s)        grouped_gemm SILU | NORM
    o[s]   = w[s] * act[s] @ W2_e            grouped_gemm STORE (row-scaled)
    h     += sum_k o[r*K + k]                moe_combine (EP/TP: partial + all-reduce)
Expert parallelism, two modes:
* ``allreduce`` (default; TP or replicated attention): rank r owns experts
  [r*E/ep, (r+1)*E/ep); every rank routes all rows (h is replicated), computes
  its experts' contributions, and the partial sums are all-reduced.
* ``a2a`` (DP attention + EP, ``moe_forward_a2a``): every rank serves its own
  sequences; each (token, expert) pair is dispatched to the expert's owner with
  one all-to-all, the owner runs its grouped GEMMs on everything it received,
  and a second all-to-all returns the weighted outputs (SURVEY §2C EP row,
  BASELINE config 5 "expert all-to-all over xGMI").  Slots per destination are
  a static capacity (rows x top_k), so ranks must step in lockstep with equal
  row counts (bench / lockstep serving) and the path is hipGraph-capturable.
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..ops import moe as moe_ops

CHUNK = 64
# rows above which a layer routes all rows at once onto the tiled grouped kernel
# (P2P_MOE_TILED_MIN=100000 keeps the 64-row skinny chunks, for A/B measurements)
TILED_MIN = int(os.environ.get("P2P_MOE_TILED_MIN", str(CHUNK + 1)))


class MoeWorkspace:
    def __init__(self, cfg, rows, device, e_local, f_local):
        K = cfg.top_k
        dev = torch.device(device)
        self.logits = torch.zeros(rows, 16, device=dev, dtype=torch.float32)
        self.topk_ids = torch.zeros(rows * K, device=dev, dtype=torch.int32)
        self.topk_w = torch.zeros(rows * K, device=dev, dtype=torch.float32)
        self.cnt = torch.zeros(e_local, device=dev, dtype=torch.int32)
        self.rows = torch.zeros(e_local, rows, device=dev, dtype=torch.int32)
        self.act = torch.zeros(rows * K, f_local, device=dev, dtype=torch.bfloat16)
        self.o = torch.zeros(rows * K, cfg.hidden, device=dev, dtype=torch.bfloat16)


def router_tiled(lw):
    """Router [E, H] padded to 16 rows and tiled (cached on the layer)."""
    rt = getattr(lw, "_router_t", None)
    if rt is None:
        E, H = lw.router.shape
        pad = torch.zeros(16, H, dtype=lw.router.dtype, device=lw.router.device)
        pad[:E] = lw.router
        rt = ops.tile_weight(pad)
        lw._router_t = rt
    return rt


def moe_forward(model, lw, ws, R):
    cfg = model.cfg
    w = model.w
    if w.ep_size > 1 and getattr(model, "ep_mode", "allreduce") == "a2a":
        return moe_forward_a2a(model, lw, ws, R)
    if R >= TILED_MIN:
        return moe_forward_tiled(model, lw, ws, R)
    e_local = cfg.n_experts // w.ep_size
    e_lo = w.ep_rank * e_local
    if ws.moe is None:
        ws.moe = MoeWorkspace(cfg, CHUNK, model.device, e_local, lw.w13.shape[1] * 16 // 2)
    m = ws.moe
    K = cfg.top_k
    distributed = w.ep_size > 1 or w.tp_size > 1
    for r0 in range(0, R, CHUNK):
        rc = min(CHUNK, R - r0)
        h = ws.h[r0:r0 + rc]
        # router GEMM + softmax/top-k + per-expert slot lists in one kernel
        moe_ops.moe_router_route(h, lw.router, cfg.n_experts, K, e_lo, e_local, m.topk_ids,
                                 m.topk_w, m.cnt, m.rows, eps=cfg.eps)
        moe_ops.grouped_gemm(lw.w13, m.cnt, m.rows, h, K, rc, ops.EPI_SILU, m.act, norm=True,
                             eps=cfg.eps)
        moe_ops.grouped_gemm(lw.w2, m.cnt, m.rows, m.act, 1, rc, ops.EPI_STORE, m.o,
                             row_w=m.topk_w)
        if not distributed:
            moe_ops.moe_combine(m.o, m.topk_ids, rc, K, e_lo, e_local, h, accumulate=True)
        else:
            part = ws.partial[r0:r0 + rc]
            moe_ops.moe_combine(m.o, m.topk_ids, rc, K, e_lo, e_local, part, accumulate=False)
            model.comm.allreduce_add_(h, part)


def moe_forward_tiled(model, lw, ws, R):
    """Prefill / large batches (R > 64 rows): route all R rows at once, then each expert's
    gate_up and down run as ONE grouped launch of the LDS-tiled MFMA kernel over its own
    rows (``ops.moe.grouped_gemm`` with max_rows > 64), so every selected expert's weights
    stream once per 128-row tile of its rows -- not once per 64-row chunk of the prompt."""
    cfg, w = model.cfg, model.w
    E, K = cfg.n_experts, cfg.top_k
    e_local = E // w.ep_size
    e_lo = w.ep_rank * e_local
    m = getattr(ws, "moe_big", None)
    if m is None:
        m = ws.moe_big = MoeWorkspace(cfg, ws.max_rows, model.device, e_local,
                                      lw.w13.shape[1] * 16 // 2)
    h = ws.h[:R]
    rt = router_tiled(lw)
    for r0 in range(0, R, CHUNK):
        rc = min(CHUNK, R - r0)
        ops.skinny_gemm(rt, h[r0:r0 + rc], ops.EPI_F32, norm=True, out=m.logits[r0:r0 + rc],
                        eps=cfg.eps)
    moe_ops.moe_route(m.logits[:R], E, K, e_lo, e_local, m.topk_ids, m.topk_w, m.cnt, m.rows)
    moe_ops.grouped_gemm(lw.w13, m.cnt, m.rows, h, K, R, ops.EPI_SILU, m.act, norm=True,
                         eps=cfg.eps)
    moe_ops.grouped_gemm(lw.w2, m.cnt, m.rows, m.act, 1, R, ops.EPI_STORE, m.o, row_w=m.topk_w)
    if not (w.ep_size > 1 or w.tp_size > 1):
        moe_ops.moe_combine(m.o, m.topk_ids, R, K, e_lo, e_local, h, accumulate=True)
    else:
        part = ws.partial[:R]
        moe_ops.moe_combine(m.o, m.topk_ids, R, K, e_lo, e_local, part, accumulate=False)
        model.comm.allreduce_add_(h, part)


def moe_forward_a2a(model, lw, ws, R):
    """DP-attention + EP MoE layer for this rank's R rows (see module doc)."""
    cfg, w, comm = model.cfg, model.w, model.comm
    E, K, H = cfg.n_experts, cfg.top_k, cfg.hidden
    W = w.ep_size
    El = E // W
    C = R * K  # static per-destination capacity
    dev = model.device
    h = ws.h[:R]
    logits = torch.empty(R, 16, device=dev, dtype=torch.float32)
    for r0 in range(0, R, CHUNK):
        rc = min(CHUNK, R - r0)
        ops.skinny_gemm(router_tiled(lw), h[r0:r0 + rc], ops.EPI_F32, norm=True,
                        out=logits[r0:r0 + rc], eps=cfg.eps)
    p = torch.softmax(logits[:, :E], dim=-1)
    tw, tid = p.topk(K, dim=-1)
    tw = tw / tw.sum(-1, keepdim=True)
    flat = tid.reshape(-1)                                     # [R*K] expert ids
    dest = torch.div(flat, El, rounding_mode="floor")
    onehot = torch.nn.functional.one_hot(dest, W)
    pos = (onehot.cumsum(0) - 1).gather(1, dest[:, None]).squeeze(1)
    slot = dest * C + pos                                      # unique send slot per pair
    send_x = torch.zeros(W * C, H, device=dev, dtype=torch.bfloat16)
    send_x.index_copy_(0, slot, h.repeat_interleave(K, dim=0))
    meta = torch.full((W * C, 2), -1, device=dev, dtype=torch.int32)
    meta[:, 1] = 0
    meta.index_copy_(0, slot, torch.stack([(flat % El).to(torch.int32),
                                           tw.reshape(-1).float().view(torch.int32)], 1))
    recv_x = torch.empty_like(send_x)
    recv_meta = torch.empty_like(meta)
    comm.all_to_all_(recv_x, send_x)
    comm.all_to_all_(recv_meta, meta)
    lexp = recv_meta[:, 0]
    row_w = recv_meta[:, 1].contiguous().view(torch.float32)
    # per-local-expert slot lists (invalid slots sort last)
    key = torch.where(lexp < 0, torch.full_like(lexp, El), lexp).long()
    order = torch.argsort(key, stable=True).to(torch.int32)
    counts = torch.bincount(key, minlength=El + 1)[:El]
    offs = counts.cumsum(0) - counts
    n = W * C
    idx = (offs[:, None] + torch.arange(n, device=dev)[None]).clamp(max=n - 1)
    rows = order[idx].contiguous()                             # [El, n]
    Fs = lw.w13.shape[1] * 16 // 2
    act = torch.empty(n, Fs, device=dev, dtype=torch.bfloat16)
    o = torch.zeros(n, H, device=dev, dtype=torch.bfloat16)
    # one grouped launch per projection over every received row (tiled kernel above 64)
    cnt = counts.to(torch.int32)
    moe_ops.grouped_gemm(lw.w13, cnt, rows, recv_x, 1, n, ops.EPI_SILU, act, norm=True,
                         eps=cfg.eps)
    moe_ops.grouped_gemm(lw.w2, cnt, rows, act, 1, n, ops.EPI_STORE, o, row_w=row_w)
    back = torch.empty_like(o)
    comm.all_to_all_(back, o)
    contrib = back.index_select(0, slot).float().view(R, K, H).sum(1)
    h.copy_((h.float() + contrib).to(h.dtype))
