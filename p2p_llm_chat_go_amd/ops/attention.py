"""Paged-KV attention (decode + per-token causal prefill) and RoPE/KV-cache write.

KV cache layout: ``[num_pages, n_kv_heads, PAGE=64, head_dim=128]`` bf16 for K
and for V (see ``engine/kv_cache.py``).  A *query row* is one token with its
sequence's block-table row and a context length (number of keys it attends,
positions ``0 .. ctx-1``), so decode (ctx = pos+1 of the new token) and causal
prefill (one row per prompt token) share one kernel.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib

PAGE = 64
HEAD_DIM = 128
CHUNK = 256


def attn_workspace(rows: int, n_heads: int, max_ctx: int, device) -> tuple:
    n_chunks = max(1, (max_ctx + CHUNK - 1) // CHUNK)
    if n_chunks == 1:
        return None, None
    part_o = torch.empty(rows * n_heads * n_chunks * HEAD_DIM, device=device, dtype=torch.float32)
    part_ml = torch.empty(rows * n_heads * n_chunks * 2, device=device, dtype=torch.float32)
    return part_o, part_ml


def _gather_kv(cache, bt_row, ctx, h):
    pos = torch.arange(ctx, device=cache.device)
    pages = bt_row[pos // PAGE].long()
    return cache[pages, h, pos % PAGE].float()  # [ctx, D]


def paged_attention_ref(q, k_cache, v_cache, block_tables, row_bt, ctx_lens, n_heads, n_kv,
                        scale, out):
    R = q.shape[0]
    G = n_heads // n_kv
    qv = q.view(R, n_heads, HEAD_DIM).float()
    res = torch.empty(R, n_heads, HEAD_DIM, dtype=torch.float32, device=q.device)
    for r in range(R):
        ctx = int(ctx_lens[r])
        bt_row = block_tables[int(row_bt[r]) if row_bt is not None else r]
        for h in range(n_kv):
            K = _gather_kv(k_cache, bt_row, ctx, h)
            V = _gather_kv(v_cache, bt_row, ctx, h)
            qh = qv[r, h * G:(h + 1) * G]  # [G, D]
            s = (qh @ K.t()) * scale
            p = torch.softmax(s, dim=-1)
            res[r, h * G:(h + 1) * G] = p @ V
    out.view(R, n_heads, HEAD_DIM).copy_(res.to(out.dtype))
    return out


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                    block_tables: torch.Tensor, row_bt: torch.Tensor, ctx_lens: torch.Tensor,
                    n_heads: int, n_kv: int, max_ctx: int, out: torch.Tensor | None = None,
                    workspace: tuple | None = None, scale: float | None = None) -> torch.Tensor:
    """q: [R, n_heads*128] bf16 -> out [R, n_heads*128] bf16.  row_bt None: row r reads
    block-table row r (decode batches)."""
    R = q.shape[0]
    if scale is None:
        scale = 1.0 / math.sqrt(HEAD_DIM)
    if out is None:
        out = torch.empty(R, n_heads * HEAD_DIM, device=q.device, dtype=q.dtype)
    if q.device.type != "cuda":
        return paged_attention_ref(q, k_cache, v_cache, block_tables, row_bt, ctx_lens, n_heads,
                                   n_kv, scale, out)
    if workspace is None:
        workspace = attn_workspace(R, n_heads, max_ctx, q.device)
    po, pml = workspace
    L = _lib.lib()
    _lib.check(L.p2p_paged_attention(q.data_ptr(), q.stride(0), k_cache.data_ptr(),
                                     v_cache.data_ptr(), block_tables.data_ptr(),
                                     block_tables.stride(0), _lib.ptr(row_bt), ctx_lens.data_ptr(),
                                     R, n_heads, n_kv, HEAD_DIM, float(scale), int(max_ctx),
                                     out.data_ptr(), out.stride(0), _lib.ptr(po), _lib.ptr(pml),
                                     _lib.stream_ptr(q.device)), "paged_attention")
    return out


FUSED_MAX_ROWS = 16
FUSED_MAX_CTX = 256

# decode qkv + RoPE + KV write + attention in one launch (csrc/kernels/qkv_attn.hip)
QKV_ATTN_MAX_ROWS = 16
QKV_ATTN_MAX_CTX = 256


def qkv_attn_ok(R: int, n_heads: int, n_kv: int, max_ctx: int) -> bool:
    return (1 <= R <= QKV_ATTN_MAX_ROWS and max_ctx <= QKV_ATTN_MAX_CTX and n_kv > 0
            and n_heads % n_kv == 0 and n_heads // n_kv in (1, 2, 4, 8))


QKV_ATTN_MAX_KSPLIT = 8


def qkv_attn_workspace(rows: int, n_heads: int, n_kv: int, device) -> tuple:
    """(granules u64 [rows][n_kv][G + 2][64], tag counters u32 [rows][n_kv],
    attention-output granules u64 [rows][n_heads * 64] + launch epoch u32 [2] for the
    fused o_proj role), zeroed."""
    G = n_heads // n_kv
    # (k-split producers publish one fp32 partial per dim and slice: up to 8 slices)
    gran = torch.zeros(rows * n_kv * (G + 2) * 128 * QKV_ATTN_MAX_KSPLIT, dtype=torch.int64,
                       device=device)
    cnt = torch.zeros(rows * n_kv, dtype=torch.int32, device=device)
    gran2 = torch.zeros(rows * n_heads * 64, dtype=torch.int64, device=device)
    epoch = torch.zeros(2, dtype=torch.int32, device=device)
    return gran, cnt, gran2, epoch


# o_proj in the qkv+attention launch: the weights of a wave's k-range sit in registers
QKV_ATTN_OPROJ_MAX_KSTEPS = 32


_OPROJ_FITS: dict = {}


def qkv_attn_oproj_ok(wo, n_heads: int, n_kv: int, waves: int | None = None, rows: int = 1,
                      hidden: int | None = None) -> bool:
    """Can ops.qkv_attn run this o_proj (bf16, fragment-major) in its own launch for
    ``rows`` batch rows?  Each 16-column group of o_proj is taken by one of the
    (n_heads + 2 n_kv) * 8 producer workgroups after its qkv slice (so o_proj may not have
    more groups than that), and the producers that wait for the attention need the whole
    grid resident at once (checked against the device's occupancy, GPU only)."""
    if not isinstance(wo, torch.Tensor) or wo.dtype != torch.bfloat16:
        return False
    K = n_heads * HEAD_DIM
    w = QKV_ATTN_WAVES if waves is None else int(waves)
    if not (wo.shape[1] * 32 == K and -(-(K // 32) // (w or 4)) <= QKV_ATTN_OPROJ_MAX_KSTEPS
            and wo.shape[0] <= (n_heads + 2 * n_kv) * (HEAD_DIM // 16)):
        return False
    if wo.device.type != "cuda":
        return True
    key = (rows, hidden or wo.shape[0] * 16, n_heads, n_kv, w)
    ok = _OPROJ_FITS.get(key)
    if ok is None:
        ok = bool(_lib.lib().p2p_qkv_attn_oproj_fits(rows, key[1], n_heads, n_kv, w))
        _OPROJ_FITS[key] = ok
    return ok


QKV_ATTN_WAVES = int(os.environ.get("P2P_QA_WAVES", "0"))  # 0: heuristic (4 or 8)


def qkv_attn(wt, x, pos, slots, cos_sin, n_heads, n_kv, k_cache, v_cache, block_tables,
             ctx_lens, out, workspace, err, eps=1e-5, scale=None, waves=None, oproj=None):
    """Decode step's qkv projection (RMSNorm folded, rope_row_perm rows) + RoPE + paged-KV
    write + attention in one launch (csrc/kernels/qkv_attn.hip): out[r] = attention of
    row r's q over its ctx_lens[r] keys (this step's token last), block-table row r.
    Same numbers as qkv_rope_gemm followed by paged_attention (up to summation order).

    oproj=(wo, h): the o_proj projection runs in the same launch (its workgroups hold their
    weight slice in registers from the start and sweep the attention output as tagged
    granules): h += attention @ wo^T, and ``out`` is not written."""
    from .gemm import tiled_shape

    R = x.shape[0]
    N, K = tiled_shape(wt)
    assert N == (n_heads + 2 * n_kv) * HEAD_DIM and x.stride(1) == 1
    if scale is None:
        scale = 1.0 / math.sqrt(HEAD_DIM)
    gran, cnt = workspace[0], workspace[1]
    assert gran.numel() >= R * n_kv * (n_heads // n_kv + 2) * 64 and cnt.numel() >= R * n_kv
    L = _lib.lib()
    if oproj is not None:
        wo, h = oproj
        No, Ko = tiled_shape(wo)
        gran2, epoch = workspace[2], workspace[3]
        assert Ko == n_heads * HEAD_DIM and h.shape[1] == No and h.stride(1) == 1
        assert gran2.numel() >= R * n_heads * 64 and h.shape[0] >= R
        _lib.check(L.p2p_qkv_attn_oproj(
            wt.data_ptr(), x.data_ptr(), x.stride(0), R, K, n_heads, n_kv, pos.data_ptr(),
            slots.data_ptr(), cos_sin.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
            block_tables.data_ptr(), block_tables.stride(0), ctx_lens.data_ptr(), float(scale),
            float(eps), gran.data_ptr(), cnt.data_ptr(), err.data_ptr(),
            QKV_ATTN_WAVES if waves is None else int(waves), wo.data_ptr(), No, h.data_ptr(),
            h.stride(0), gran2.data_ptr(), epoch.data_ptr(), _lib.stream_ptr(x.device)),
            "qkv_attn_oproj")
        return h
    _lib.check(L.p2p_qkv_attn(
        wt.data_ptr(), x.data_ptr(), x.stride(0), R, K, n_heads, n_kv, pos.data_ptr(),
        slots.data_ptr(), cos_sin.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
        block_tables.data_ptr(), block_tables.stride(0), ctx_lens.data_ptr(), float(scale),
        out.data_ptr(), out.stride(0), float(eps), gran.data_ptr(), cnt.data_ptr(),
        err.data_ptr(), QKV_ATTN_WAVES if waves is None else int(waves),
        _lib.stream_ptr(x.device)), "qkv_attn")
    return out


def attn_oproj_ok(R: int, n_heads: int, n_kv: int, max_ctx: int, N: int) -> bool:
    """Shapes the fused attention + o_proj kernel handles (else run the two ops)."""
    G = n_heads // n_kv
    S = n_heads * HEAD_DIM // 32
    return (R <= FUSED_MAX_ROWS and max_ctx <= FUSED_MAX_CTX and G in (1, 2, 4) and S % 16 == 0
            and S // 16 in (1, 2, 4, 8, 16) and N % 16 == 0)


def attn_oproj(q, k_cache, v_cache, block_tables, row_bt, ctx_lens, n_heads, n_kv, max_ctx, wo,
               h, attn, sync, err, scale=None):
    """h += attention(q) @ Wo^T in ONE launch (decode, R <= 16 rows, ctx <= 256):
    the o_proj blocks stream their weights while the attention blocks run.
    attn: [R, n_heads*128] scratch; sync: int32 [2] zeros; err: int32 [1]."""
    from .gemm import EPI_RESID, skinny_gemm, tiled_shape

    R = q.shape[0]
    if scale is None:
        scale = 1.0 / math.sqrt(HEAD_DIM)
    N, K = tiled_shape(wo)
    if q.device.type != "cuda":
        paged_attention(q, k_cache, v_cache, block_tables, row_bt, ctx_lens, n_heads, n_kv,
                        max_ctx, out=attn, scale=scale)
        return skinny_gemm(wo, attn, EPI_RESID, out=h)
    L = _lib.experimental()
    _lib.check(L.p2p_attn_oproj(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                block_tables.data_ptr(), block_tables.stride(0), row_bt.data_ptr(),
                                ctx_lens.data_ptr(), R, n_heads, n_kv, HEAD_DIM, float(scale),
                                int(max_ctx), attn.data_ptr(), attn.stride(0), wo.data_ptr(), N,
                                h.data_ptr(), h.stride(0), sync.data_ptr(), err.data_ptr(),
                                _lib.stream_ptr(q.device)), "attn_oproj")
    return h


HEADS_MAX_ROWS = 16  # kernel limit (one MFMA M-tile); the engine's default is lower
HEADS_COLS = 128     # output columns per workgroup


def attn_oproj_heads_ok(R: int, n_heads: int, n_kv: int, max_ctx: int, N: int) -> bool:
    """Shapes the head-split fused attention + o_proj kernel handles."""
    return (R <= HEADS_MAX_ROWS and max_ctx <= FUSED_MAX_CTX and n_heads % n_kv == 0
            and n_heads // n_kv in (1, 2, 4) and N % HEADS_COLS == 0)


def attn_oproj_heads_workspace(R: int, n_kv: int, N: int, device) -> tuple:
    """(fp32 partial slab [n_kv * R * N], u32 tickets [N / 128] zeroed once)."""
    slab = torch.zeros(n_kv * R * N, device=device, dtype=torch.float32)
    tickets = torch.zeros(N // HEADS_COLS, device=device, dtype=torch.int32)
    return slab, tickets


def attn_oproj_heads(q, k_cache, v_cache, block_tables, row_bt, ctx_lens, n_heads, n_kv, max_ctx,
                     wo, h, slab, tickets, attn=None, scale=None):
    """h += attention(q) @ Wo^T in ONE launch without a cross-workgroup hand-off
    (decode, R <= 16 rows, ctx <= 256): workgroup (column block, kv head) streams its
    o_proj slice while it computes that head's attention, stores a partial o_proj, and
    the last head of each column block sums the partials + residual
    (csrc/kernels/attn_oproj_heads.hip).  row_bt None = identity; attn (optional):
    [R, n_heads*128] copy of the attention output."""
    from .gemm import EPI_RESID, skinny_gemm, tiled_shape

    R = q.shape[0]
    if scale is None:
        scale = 1.0 / math.sqrt(HEAD_DIM)
    N, K = tiled_shape(wo)
    if q.device.type != "cuda":
        a = attn if attn is not None else torch.empty(R, n_heads * HEAD_DIM, dtype=q.dtype)
        paged_attention(q, k_cache, v_cache, block_tables, row_bt, ctx_lens, n_heads, n_kv,
                        max_ctx, out=a, scale=scale)
        return skinny_gemm(wo, a, EPI_RESID, out=h)
    if slab.numel() < n_kv * R * N or tickets.numel() < N // HEADS_COLS:
        raise ValueError("attn_oproj_heads: workspace too small")
    L = _lib.experimental()
    _lib.check(L.p2p_attn_oproj_heads(
        q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
        block_tables.stride(0), _lib.ptr(row_bt), ctx_lens.data_ptr(), R, n_heads, n_kv, HEAD_DIM,
        float(scale), int(max_ctx), wo.data_ptr(), N, h.data_ptr(), h.stride(0), slab.data_ptr(),
        tickets.data_ptr(), _lib.ptr(attn), attn.stride(0) if attn is not None else 0,
        _lib.stream_ptr(q.device)), "attn_oproj_heads")
    return h


QTILE = 16
# v2 flash prefill (256 query rows per workgroup, 32x32x16 MFMA); P2P_FLASH_V2=0 selects v1
FLASH_V2 = os.environ.get("P2P_FLASH_V2", "1") != "0"


# v2 pays from about this many (query tile, kv head) workgroups; below it the 16-token
# v1 tiles spread a short prompt over more CUs (profiles/r2_flash_prefill_v2.jsonl:
# T=512 v1 27 us vs v2 40 us; T=2048 v2 138 us vs v1 236 us)
FLASH_V2_MIN_BLOCKS = 128  # v1 wins up to T=512 at 8 KV heads, v2 from ~1K (profiles/r2_flash_prefill_v2_conflict_free.jsonl)


def flash_tile(n_heads: int, n_kv: int, rows: int | None = None) -> int:
    """Tokens per query tile for a prefill chunk of ``rows`` tokens: v2 (256 / (Hq/Hkv))
    when it yields enough workgroups, else v1 (16)."""
    G = n_heads // n_kv
    if FLASH_V2 and G in (1, 2, 4, 8):
        t = 256 // G
        if rows is None or -(-rows // t) * n_kv >= FLASH_V2_MIN_BLOCKS:
            return t
    return QTILE


def prefill_tiles(seq, pos, tile: int = QTILE) -> torch.Tensor:
    """Split flat prefill rows into query tiles for :func:`flash_prefill`.

    ``seq``/``pos`` are host int sequences (one entry per row, rows of one
    sequence consecutive with consecutive positions).  Returns int32 [n, 4] =
    (first row, n tokens, sequence, first position).
    """
    seq = [int(s) for s in seq]
    pos = [int(p) for p in pos]
    out = []
    r, R = 0, len(seq)
    while r < R:
        e = r + 1
        while e < R and e - r < tile and seq[e] == seq[r] and pos[e] == pos[e - 1] + 1:
            e += 1
        out.append((r, e - r, seq[r], pos[r]))
        r = e
    return torch.tensor(out, dtype=torch.int32).view(-1, 4)


def flash_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                  block_tables: torch.Tensor, tiles: torch.Tensor, n_heads: int, n_kv: int,
                  out: torch.Tensor | None = None, scale: float | None = None,
                  tiles_host: torch.Tensor | None = None, *, qtile: int) -> torch.Tensor:
    """Causal prefill attention on MFMA for query tiles (see ``prefill_tiles``).

    Equivalent to :func:`paged_attention` with one row per prompt token
    (ctx = pos + 1), but reads each K/V page once per query tile x G heads.  The
    tiles must come from ``prefill_tiles(seq, pos, qtile)`` with the SAME ``qtile``
    (from ``flash_tile``): > 16 runs the v2 kernel.  ``qtile`` is required -- the tile
    width the tiles were cut with decides which kernel may read them.
    """
    if qtile is None or qtile < 1:
        raise ValueError("flash_prefill: qtile (the prefill_tiles width) is required")
    if tiles_host is not None and tiles_host.numel() and int(tiles_host[:, 1].max()) > qtile:
        raise ValueError("flash_prefill: tiles are wider than qtile=%d" % qtile)
    R = q.shape[0]
    if scale is None:
        scale = 1.0 / math.sqrt(HEAD_DIM)
    if out is None:
        out = torch.empty(R, n_heads * HEAD_DIM, device=q.device, dtype=q.dtype)
    if q.device.type != "cuda":
        th = (tiles_host if tiles_host is not None else tiles).cpu()
        row_bt = torch.empty(R, dtype=torch.int32)
        ctx = torch.empty(R, dtype=torch.int32)
        for r0, n, s, p0 in th.tolist():
            row_bt[r0:r0 + n] = s
            ctx[r0:r0 + n] = torch.arange(p0 + 1, p0 + n + 1, dtype=torch.int32)
        return paged_attention_ref(q, k_cache, v_cache, block_tables, row_bt, ctx, n_heads, n_kv,
                                   scale, out)
    L = _lib.lib()
    fn = L.p2p_flash_prefill2 if qtile > QTILE else L.p2p_flash_prefill
    _lib.check(fn(q.data_ptr(), q.stride(0), k_cache.data_ptr(),
                                   v_cache.data_ptr(), block_tables.data_ptr(),
                                   block_tables.stride(0), tiles.data_ptr(), tiles.shape[0],
                                   n_heads, n_kv, HEAD_DIM, float(scale), out.data_ptr(),
                                   out.stride(0), _lib.stream_ptr(q.device)), "flash_prefill")
    return out


def rope_cache_ref(qkv, pos, slots, cos_sin, n_heads, n_kv, q_out, k_cache, v_cache):
    T = qkv.shape[0]
    D = HEAD_DIM
    x = qkv.view(T, n_heads + 2 * n_kv, D).float()
    cs = cos_sin[pos.long()]  # [T, 64, 2]
    c, s = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    qk = x[:, :n_heads + n_kv]
    x1, x2 = qk[..., :D // 2], qk[..., D // 2:]
    rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    q_out.view(T, n_heads, D).copy_(rot[:, :n_heads].to(q_out.dtype))
    for t in range(T):
        slot = int(slots[t])
        if slot < 0:
            continue
        page, off = slot // PAGE, slot % PAGE
        k_cache[page, :, off] = rot[t, n_heads:].to(k_cache.dtype)
        v_cache[page, :, off] = x[t, n_heads + n_kv:].to(v_cache.dtype)
    return q_out


def rope_cache(qkv: torch.Tensor, pos: torch.Tensor, slots: torch.Tensor, cos_sin: torch.Tensor,
               n_heads: int, n_kv: int, q_out: torch.Tensor, k_cache: torch.Tensor,
               v_cache: torch.Tensor) -> torch.Tensor:
    """Rotate q/k (HF rotate_half, llama3-scaled table), write k/v to the paged cache."""
    T = qkv.shape[0]
    if qkv.device.type != "cuda":
        return rope_cache_ref(qkv, pos, slots, cos_sin, n_heads, n_kv, q_out, k_cache, v_cache)
    L = _lib.lib()
    _lib.check(L.p2p_rope_cache(qkv.data_ptr(), qkv.stride(0), pos.data_ptr(), slots.data_ptr(),
                                cos_sin.data_ptr(), T, n_heads, n_kv, HEAD_DIM, q_out.data_ptr(),
                                q_out.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                _lib.stream_ptr(qkv.device)), "rope_cache")
    return q_out
