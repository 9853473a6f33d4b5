"""Mixtral sparse-MoE FFN on the engine kernels (replaces the dense SwiGLU MLP).

Per layer, for R rows (chunks of <= 64 rows, the grouped kernel's M tile):
    logits = rstd(h) * h @ Wrouter'          skinny_gemm (router padded to 16 rows)
    ids, w = top_k(softmax(logits))          moe_route  (+ per-expert slot lists)
    act[s] = silu(g) * u of expert(s)        grouped_gemm SILU | NORM
    o[s]   = w[s] * act[s] @ W2_e            grouped_gemm STORE (row-scaled)
    h     += sum_k o[r*K + k]                moe_combine (EP/TP: partial + all-reduce)
Expert parallelism: rank r owns experts [r*E/ep, (r+1)*E/ep); every rank routes
all rows, computes its experts' contributions, and the partial sums are
all-reduced (decode-size messages; see parallel/comm.py).
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import moe as moe_ops

CHUNK = 64


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
        logits = m.logits[:rc]
        ops.skinny_gemm(router_tiled(lw), h, ops.EPI_F32, norm=True, out=logits, eps=cfg.eps)
        moe_ops.moe_route(logits, cfg.n_experts, K, e_lo, e_local, m.topk_ids, m.topk_w, m.cnt,
                          m.rows)
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
