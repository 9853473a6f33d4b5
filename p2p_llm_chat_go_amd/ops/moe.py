"""Sparse-MoE ops (Mixtral): routing, grouped expert GEMMs, combine.

The expert GEMMs are the grouped mode of the skinny MFMA kernel
(``csrc/kernels/skinny_gemm.hip``): one launch covers all local experts
(grid.y), each expert reads its weights only if at least one row was routed to
it -- at decode batch 1 Mixtral streams 2 of its 8 experts per layer.
Slots: a token r routed to its k-th expert is slot r*top_k + k.
"""
from __future__ import annotations

import torch

from . import _lib
from .gemm import EPI_SILU, EPI_STORE, _ref, tiled_shape


def moe_route(logits, E, K, e_lo, e_local, topk_ids, topk_w, cnt, rows):
    """logits [R, >=E] fp32 -> topk ids/weights [R*K], cnt [e_local], rows [e_local, R]."""
    R = logits.shape[0]
    if logits.device.type != "cuda":
        p = torch.softmax(logits[:, :E].float(), -1)
        w, ids = p.topk(K, dim=-1)
        w = w / w.sum(-1, keepdim=True)
        topk_ids[:R * K] = ids.reshape(-1).to(torch.int32)
        topk_w[:R * K] = w.reshape(-1)
        cnt.zero_()
        for s, e in enumerate(ids.reshape(-1).tolist()):
            le = e - e_lo
            if 0 <= le < e_local:
                rows[le, int(cnt[le])] = s
                cnt[le] += 1
        return
    L = _lib.lib()
    _lib.check(L.p2p_moe_route(logits.data_ptr(), logits.stride(0), R, E, K, e_lo, e_local,
                               topk_ids.data_ptr(), topk_w.data_ptr(), cnt.data_ptr(),
                               rows.data_ptr(), rows.stride(0), _lib.stream_ptr(logits.device)),
               "moe_route")


def moe_router_route(h, wr, E, K, e_lo, e_local, topk_ids, topk_w, cnt, rows, eps=1e-5):
    """Fused router (rstd(h) * h @ Wr^T, RMSNorm gain folded into wr) + moe_route for
    R <= 64 rows: topk ids/weights [R*K], cnt [e_local], rows [e_local, >=R]."""
    R, H = h.shape
    if h.device.type != "cuda":
        hf = h.float()
        logits = (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)) @ wr.float().t()
        return moe_route(logits, E, K, e_lo, e_local, topk_ids, topk_w, cnt, rows)
    if h.dtype != torch.bfloat16 or wr.dtype != torch.bfloat16 or not wr.is_contiguous():
        raise TypeError("moe_router_route: h and wr must be bf16 (wr contiguous)")
    L = _lib.lib()
    _lib.check(L.p2p_moe_router_route(h.data_ptr(), h.stride(0), R, H, wr.data_ptr(), float(eps),
                                      E, K, e_lo, e_local, topk_ids.data_ptr(), topk_w.data_ptr(),
                                      cnt.data_ptr(), rows.data_ptr(), rows.stride(0),
                                      _lib.stream_ptr(h.device)), "moe_router_route")
    return topk_ids, topk_w


def moe_router_logits(h, wr, E, logits, eps=1e-5):
    """logits[:R, :E] = rstd(h) * h @ wr^T (gain folded into wr), one workgroup per row."""
    R, H = h.shape
    if h.device.type != "cuda":
        hf = h.float()
        logits[:R, :E] = (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)) @ wr.float().t()
        return logits
    L = _lib.lib()
    _lib.check(L.p2p_moe_router_logits(h.data_ptr(), h.stride(0), R, H, wr.data_ptr(), E, float(eps),
                                       logits.data_ptr(), logits.stride(0),
                                       _lib.stream_ptr(h.device)), "moe_router_logits")
    return logits


def grouped_gemm(wt, cnt, rows, x, x_div, max_rows, epi, out, norm=False, row_w=None, eps=1e-5):
    """Per local expert e: out[slot] = epi(x[slot // x_div] @ W_e^T) for its routed slots.

    wt: [E_local, N/16, K/32, 64, 8] tiled expert weights.
    """
    E = wt.shape[0]
    N, K = tiled_shape(wt[0])
    if x.device.type != "cuda":
        for e in range(E):
            c = int(cnt[e])
            if c == 0:
                continue
            slots = rows[e, :c].long()
            xs = x[slots // x_div]
            n_out = N // 2 if epi == EPI_SILU else N
            o = torch.empty(c, n_out, dtype=torch.bfloat16)
            _ref(wt[e], xs, epi, norm, o, eps)
            if row_w is not None:
                o = (o.float() * row_w[slots][:, None]).to(torch.bfloat16)
            out[slots] = o
        return out
    L = _lib.lib()
    w_stride = wt[0].numel() // 8  # in bf16x8 units
    _lib.check(L.p2p_grouped_gemm(wt.data_ptr(), w_stride, E, cnt.data_ptr(), rows.data_ptr(),
                                  rows.stride(0), x_div, _lib.ptr(row_w), x.data_ptr(), x.stride(0),
                                  max_rows, K, N, epi, int(norm), out.data_ptr(), out.stride(0),
                                  float(eps), 0, _lib.stream_ptr(x.device)), "grouped_gemm")
    return out


def moe_combine(o, topk_ids, R, K, e_lo, e_local, out, accumulate=True):
    """accumulate: out[r] += sum_k o[r*K+k] (local experts only); else out[r] = the sum."""
    H = out.shape[1]
    if o.device.type != "cpu":
        L = _lib.lib()
        _lib.check(L.p2p_moe_combine(o.data_ptr(), o.stride(0), topk_ids.data_ptr(), R, K, e_lo,
                                     e_local, H, out.data_ptr(), out.stride(0), int(accumulate),
                                     _lib.stream_ptr(o.device)), "moe_combine")
        return out
    ids = topk_ids[:R * K].view(R, K).long() - e_lo
    mask = ((ids >= 0) & (ids < e_local)).float()
    s = (o[:R * K].float().view(R, K, H) * mask[..., None]).sum(1)
    if accumulate:
        out[:R] = (out[:R].float() + s).to(out.dtype)
    else:
        out[:R] = s.to(out.dtype)
    return out


# ------------------------------------------------------------ expert-parallel all-to-all
def a2a_dispatch(h, topk_ids, topk_w, K, El, W, C, send_x, send_meta, send_map, dest_cnt,
                 slot_pos):
    """Pack every (token, k) slot's row of h for its expert's owner rank (dest = id // El).

    C > 0: static capacity, dest d's rows at [d*C, d*C + count) (padding rows carry expert
    id -1 in send_meta); C == 0: packed by destination.  Writes send_x [rows, H], send_meta
    [rows, 2] int32 (local expert id, weight bits), send_map [R*K] (the send row of each
    slot) and dest_cnt [W] (rows per destination)."""
    R, H = h.shape
    n = R * K
    if h.device.type != "cuda":
        ids = topk_ids[:n].long()
        dest = ids // El
        onehot = torch.nn.functional.one_hot(dest, W)
        pos = (onehot.cumsum(0) - 1).gather(1, dest[:, None]).squeeze(1)
        cnt = onehot.sum(0)
        off = dest * C if C > 0 else (cnt.cumsum(0) - cnt)[dest]
        row = off + pos
        if C > 0:
            send_meta[:W * C].fill_(-1)
        send_x[row] = h.repeat_interleave(K, dim=0)
        send_meta[row, 0] = (ids % El).to(torch.int32)
        send_meta[row, 1] = topk_w[:n].float().view(torch.int32)
        send_map[:n] = row.to(torch.int32)
        dest_cnt[:W] = cnt.to(dest_cnt.dtype)
        return
    L = _lib.lib()
    _lib.check(L.p2p_moe_a2a_dispatch(h.data_ptr(), h.stride(0), R, H, topk_ids.data_ptr(),
                                      topk_w.data_ptr(), K, El, W, C, dest_cnt.data_ptr(),
                                      slot_pos.data_ptr(), send_x.data_ptr(), send_meta.data_ptr(),
                                      send_map.data_ptr(), _lib.stream_ptr(h.device)),
               "moe_a2a_dispatch")


def a2a_group(meta, n, El, cnt, rows):
    """Received rows [n] -> per-local-expert slot lists cnt [El], rows [El, >= n]."""
    if meta.device.type != "cuda":
        le = meta[:n, 0].long()
        cnt.zero_()
        for r, e in enumerate(le.tolist()):
            if 0 <= e < El:
                rows[e, int(cnt[e])] = r
                cnt[e] += 1
        return
    L = _lib.lib()
    _lib.check(L.p2p_moe_a2a_group(meta.data_ptr(), n, El, cnt.data_ptr(), rows.data_ptr(),
                                   rows.stride(0), _lib.stream_ptr(meta.device)), "moe_a2a_group")


def a2a_combine(back, send_map, R, K, h):
    """h[r] += sum_k back[send_map[r*K + k]] (fp32 sum in k order, one bf16 rounding)."""
    H = h.shape[1]
    if h.device.type != "cuda":
        contrib = back.index_select(0, send_map[:R * K].long()).float().view(R, K, H).sum(1)
        h[:R] = (h[:R].float() + contrib).to(h.dtype)
        return h
    L = _lib.lib()
    _lib.check(L.p2p_moe_a2a_combine(back.data_ptr(), H, send_map.data_ptr(), R, K, h.data_ptr(),
                                     h.stride(0), _lib.stream_ptr(h.device)), "moe_a2a_combine")
    return h
