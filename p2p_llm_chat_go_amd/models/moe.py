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
  BASELINE config 5 "expert all-to-all over xGMI").  Dispatch, grouping and combine
  are kernels; decode uses a static per-destination capacity (rows x top_k, no host
  sync, hipGraph-capturable), prefill exchanges exact counts and moves only the
  routed rows.  Ranks step in lockstep with equal row counts (bench / lockstep serving).
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
# rows up to which the fused single-block router+route kernel is used (decode batches);
# above, per-row logits workgroups + moe_route (the single block serialised a 43-row
# prompt chunk: 69 us per layer)
ROUTER_FUSED_MAX = 8


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
        if rc <= ROUTER_FUSED_MAX:
            # router GEMM + softmax/top-k + per-expert slot lists in one (single-block) kernel
            moe_ops.moe_router_route(h, lw.router, cfg.n_experts, K, e_lo, e_local, m.topk_ids,
                                     m.topk_w, m.cnt, m.rows, eps=cfg.eps)
        else:  # prefill chunks: logits one workgroup per row, then the routing kernel
            moe_ops.moe_router_logits(h, lw.router, cfg.n_experts, m.logits, eps=cfg.eps)
            moe_ops.moe_route(m.logits[:rc], cfg.n_experts, K, e_lo, e_local, m.topk_ids,
                              m.topk_w, m.cnt, m.rows)
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


class _Grow:
    """Grow-only device buffers of the EP all-to-all path, one flat allocation per name,
    handed out as [rows, cols] views.  A grown buffer's predecessor is kept alive: a
    decode graph captured earlier (another batch bucket) still addresses it."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}
        self.retired = []

    def get(self, name, rows, cols=None, dtype=torch.bfloat16):
        need = max(rows, 1) * (cols or 1)
        t = self.bufs.get(name)
        if t is None or t.numel() < need or t.dtype != dtype:
            if t is not None:
                self.retired.append(t)
            t = torch.empty(need, device=self.device, dtype=dtype)
            self.bufs[name] = t
        if cols is None:
            return t[:rows]
        return t[:rows * cols].view(rows, cols)


# static per-destination capacity (graph-capturable, padded) while the padded send stays
# below this many bytes; larger calls (prefill) exchange exact counts first
A2A_STATIC_MAX_BYTES = int(os.environ.get("P2P_A2A_STATIC_MAX_BYTES", str(4 << 20)))


def moe_forward_a2a(model, lw, ws, R):
    """DP-attention + EP MoE layer for this rank's R rows (see module doc).

    Kernels (``moe.hip``): routing (``moe_route``), dispatch (``a2a_dispatch``: slot ->
    owner rank, row packing), slot grouping on the owner (``a2a_group``), the grouped
    expert GEMMs, and the combine (``a2a_combine``).  Two exchange forms:
      * static capacity C = R*K rows per destination -- no host sync, hipGraph-capturable
        (decode), W*C rows on the wire, mostly padding;
      * exact counts (padded send above ``A2A_STATIC_MAX_BYTES``, not while capturing):
        rows per destination go to the host, one tiny all-to-all of counts, then the
        variable-split all-to-all moves only the R*K routed rows (prefill)."""
    cfg, w, comm = model.cfg, model.w, model.comm
    E, K, H = cfg.n_experts, cfg.top_k, cfg.hidden
    W = w.ep_size
    El = E // W
    dev = model.device
    h = ws.h[:R]
    buf = getattr(ws, "a2a", None)
    if buf is None:
        buf = ws.a2a = _Grow(dev)
    n_slots = R * K
    # routing: logits (RMSNorm folded) -> top-k ids / renormalised weights
    logits = buf.get("logits", R, 16, torch.float32)
    for r0 in range(0, R, CHUNK):
        rc = min(CHUNK, R - r0)
        ops.skinny_gemm(router_tiled(lw), h[r0:r0 + rc], ops.EPI_F32, norm=True,
                        out=logits[r0:r0 + rc], eps=cfg.eps)
    topk_ids = buf.get("topk_ids", n_slots, None, torch.int32)
    topk_w = buf.get("topk_w", n_slots, None, torch.float32)
    dummy_rows = buf.get("route_rows", 1, R, torch.int32)
    dummy_cnt = buf.get("route_cnt", 1, None, torch.int32)
    moe_ops.moe_route(logits, E, K, 0, 0, topk_ids, topk_w, dummy_cnt, dummy_rows)
    ipc = getattr(comm, "ep_ipc", None)
    if ipc is not None and dev.type == "cuda" and ipc.fits(n_slots):
        return _a2a_ipc(model, lw, buf, ipc, h, topk_ids, topk_w, R)
    capturing = dev.type == "cuda" and torch.cuda.is_current_stream_capturing()
    exact = (not capturing) and W * n_slots * H * 2 > A2A_STATIC_MAX_BYTES
    C = 0 if exact else n_slots
    n_send = n_slots if exact else W * C
    send_x = buf.get("send_x", n_send, H)
    send_meta = buf.get("send_meta", n_send, 2, torch.int32)
    send_map = buf.get("send_map", n_slots, None, torch.int32)
    slot_pos = buf.get("slot_pos", n_slots, None, torch.int32)
    dest_cnt = buf.get("dest_cnt", W, None, torch.int32)
    moe_ops.a2a_dispatch(h, topk_ids, topk_w, K, El, W, C, send_x, send_meta, send_map, dest_cnt,
                         slot_pos)
    if exact:
        in_splits = [int(x) for x in dest_cnt.cpu().tolist()]
        recv_cnt = buf.get("recv_cnt", W, None, torch.int32)
        comm.all_to_all_(recv_cnt, dest_cnt)
        out_splits = [int(x) for x in recv_cnt.cpu().tolist()]
        n = sum(out_splits)
        recv_x = buf.get("recv_x", n, H)
        recv_meta = buf.get("recv_meta", n, 2, torch.int32)
        comm.all_to_all_v_(recv_x, send_x, out_splits, in_splits)
        comm.all_to_all_v_(recv_meta, send_meta, out_splits, in_splits)
    else:
        n = n_send
        recv_x = buf.get("recv_x", n, H)
        recv_meta = buf.get("recv_meta", n, 2, torch.int32)
        comm.all_to_all_(recv_x, send_x)
        comm.all_to_all_(recv_meta, send_meta)
    Fs = lw.w13.shape[1] * 16 // 2
    o = buf.get("o", max(n, 1), H)
    if n > 0:
        cnt = buf.get("cnt", El, None, torch.int32)
        rows = buf.get("rows", El, n, torch.int32)
        moe_ops.a2a_group(recv_meta, n, El, cnt, rows)
        row_w = recv_meta[:, 1].contiguous().view(torch.float32)
        act = buf.get("act", n, Fs)
        # one grouped launch per projection over every received row (tiled kernel above 64)
        moe_ops.grouped_gemm(lw.w13, cnt, rows, recv_x, 1, n, ops.EPI_SILU, act, norm=True,
                             eps=cfg.eps)
        moe_ops.grouped_gemm(lw.w2, cnt, rows, act, 1, n, ops.EPI_STORE, o[:n], row_w=row_w)
    back = buf.get("back", n_send, H)
    if exact:
        comm.all_to_all_v_(back, o[:n], in_splits, out_splits)
    else:
        comm.all_to_all_(back, o[:n])
    moe_ops.a2a_combine(back, send_map, R, K, h)


def _a2a_ipc(model, lw, buf, ipc, h, topk_ids, topk_w, R):
    """Decode-size exchanges of ``moe_forward_a2a`` on the IPC kernels
    (``parallel.ep_a2a``): no host sync, no RCCL call, only routed rows on the wire --
    the whole layer is captured in the decode hipGraph.  Same numbers as the RCCL path
    (rows land in another order inside a destination; every row is computed on its own
    and the combine sums a token's K returns in k order)."""
    cfg = model.cfg
    K, H = cfg.top_k, cfg.hidden
    W = model.w.ep_size
    El = cfg.n_experts // W
    C = R * K
    nb = ipc.blocks_per_pair(C, W)
    send_map = buf.get("ipc_send_map", C, None, torch.int32)
    ipc.dispatch(h, topk_ids, topk_w, K, El, send_map, R, nb)
    n = W * C
    recv_x = buf.get("recv_x", n, H)
    recv_meta = buf.get("recv_meta", n, 2, torch.int32)
    recv_w = buf.get("ipc_recv_w", n, None, torch.float32)
    recv_cnt = buf.get("ipc_recv_cnt", W, None, torch.int32)
    ipc.recv(C, recv_x, recv_meta, recv_w, recv_cnt, nb)
    cnt = buf.get("cnt", El, None, torch.int32)
    rows = buf.get("rows", El, n, torch.int32)
    moe_ops.a2a_group(recv_meta, n, El, cnt, rows)
    Fs = lw.w13.shape[1] * 16 // 2
    act = buf.get("act", n, Fs)
    o = buf.get("o", n, H)
    moe_ops.grouped_gemm(lw.w13, cnt, rows, recv_x, 1, n, ops.EPI_SILU, act, norm=True,
                         eps=cfg.eps)
    moe_ops.grouped_gemm(lw.w2, cnt, rows, act, 1, n, ops.EPI_STORE, o, row_w=recv_w)
    ipc.give_back(C, o, recv_cnt, nb)
    ipc.combine(send_map, R, K, h, nb)
