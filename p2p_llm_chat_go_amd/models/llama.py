"""Llama / Mixtral decoder forward on the engine's kernels.

One ``forward`` serves prefill and decode: its input is a flat list of *query
rows* (tokens) with per-row position, KV slot, sequence (block-table row) and
context length.  Per layer (TP=1, dense):

    q,k,v = rope(rstd(h) * h @ Wqkv');   skinny_gemm  NORM | QKV_ROPE
            k,v -> KV pages               (RoPE + cache write in the epilogue)
    a     = paged_attention(q, pages)    paged_attention (GQA-packed)
    h    += a @ Wo                       skinny_gemm  RESID
    act   = silu(g) * u, [g|u] = rstd(h) * h @ Wgu'   skinny_gemm NORM | SILU
    h    += act @ Wdown                  skinny_gemm  RESID

i.e. 5 launches per layer, every RMSNorm / RoPE / KV write / residual add /
SwiGLU fused into a GEMM; the LM head fuses greedy argmax (64-bit atomicMax
keys) so no logits round trip on the greedy path.  With TP>1 the row-parallel outputs
(o_proj, down) are summed across ranks in the GEMM epilogue itself at decode sizes
(``ops.skinny_gemm_ar``, one launch); larger chunks go to a scratch buffer and
``comm.allreduce_add_(h, partial)`` sums them into the residual.
MoE layers (Mixtral) route through ``models.moe``.

Every buffer lives in a preallocated ``Workspace`` so the decode step can be
captured in a hipGraph (``engine.graph``).
"""
from __future__ import annotations

import os

import torch

from .. import ops
from .config import ModelConfig, rope_table
from .weights import EngineWeights


class Workspace:
    def __init__(self, cfg: ModelConfig, max_rows: int, max_ctx: int, device, tp_size: int = 1,
                 max_out_rows: int | None = None):
        dev = torch.device(device)
        self.max_rows = max_rows
        self.max_ctx = max_ctx
        nq = cfg.n_heads // tp_size
        nkv = cfg.n_kv_heads // tp_size
        D = cfg.head_dim
        bf = torch.bfloat16
        self.h = torch.zeros(max_rows, cfg.hidden, device=dev, dtype=bf)
        self.qkv = torch.zeros(max_rows, (nq + 2 * nkv) * D, device=dev, dtype=bf)
        self.q = torch.zeros(max_rows, nq * D, device=dev, dtype=bf)
        self.attn = torch.zeros(max_rows, nq * D, device=dev, dtype=bf)
        self.act = torch.zeros(max_rows, cfg.ffn // tp_size, device=dev, dtype=bf)
        self.partial = torch.zeros(max_rows, cfg.hidden, device=dev, dtype=bf) if tp_size > 1 or cfg.is_moe else None
        mo = max_out_rows or max_rows
        self.last = torch.zeros(mo, cfg.hidden, device=dev, dtype=bf)
        self.logits = torch.zeros(mo, cfg.vocab // tp_size, device=dev, dtype=torch.float32)
        self.ids_out = torch.zeros(mo, device=dev, dtype=torch.int32)
        self.keys = ops.new_argmax_keys(mo, dev)
        self.attn_ws = ops.attn_workspace(max_rows, nq, max_ctx, dev)
        self.moe = None  # lazily sized by models.moe
        # fused attention + o_proj hand-off counters (re-armed by the kernel) + fault flag
        self.sync = torch.zeros(2, device=dev, dtype=torch.int32)
        # head-split attention + o_proj (ops.attn_oproj_heads): fp32 partial slab + tickets
        self.heads_slab = self.heads_tickets = None
        if (dev.type == "cuda" and tp_size == 1 and cfg.hidden % ops.attention.HEADS_COLS == 0
                and os.environ.get("P2P_FUSED_ATTN_OPROJ", "0") == "heads"):  # experimental lib
            rows = min(max_rows, ops.attention.HEADS_MAX_ROWS)
            self.heads_slab, self.heads_tickets = ops.attn_oproj_heads_workspace(
                rows, nkv, cfg.hidden, dev)
        self.row_ids = torch.arange(max_rows, device=dev, dtype=torch.int32)  # identity row_bt
        # decode qkv + attention in one launch (ops.qkv_attn): granules + tag counters
        self.qa = None
        if dev.type == "cuda" and max_rows <= ops.attention.QKV_ATTN_MAX_ROWS and \
                ops.qkv_attn_ok(max_rows, nq, nkv, max_ctx):
            self.qa = ops.qkv_attn_workspace(max_rows, nq, nkv, dev)
        self.err = torch.zeros(1, device=dev, dtype=torch.int32)


class LlamaModel:
    def __init__(self, weights: EngineWeights, kv, comm=None):
        self.w = weights
        self.cfg = weights.cfg
        self.kv = kv
        self.comm = comm
        self.tp = weights.tp_size
        self.device = weights.device
        self.nq = self.cfg.n_heads // self.tp
        self.nkv = self.cfg.n_kv_heads // self.tp
        max_pos = min(self.cfg.max_pos, 1 << 17)
        self.rope = rope_table(self.cfg, max_pos=max_pos, device=self.device)
        # decode: attention and o_proj in one launch (ops.attn_oproj).  Opt-in: measured on
        # MI355X it is 16.5 us vs 14.0 us for the two kernels at 8B / batch 1
        # (profiles/r1_fused_attn_oproj_vs_separate.jsonl), so the two-kernel path stays default.
        # "heads": the head-split fused kernel (ops.attn_oproj_heads) -- every workgroup
        # computes one kv head's attention while its o_proj slice streams in, no hand-off,
        # the last head of each column block sums the partials -- for decode batches of
        # <= P2P_HEADS_MAX_ROWS rows at contexts <= 256.  Also measured slower (16.9 vs
        # 14.5 us at batch 1, profiles/r2_attn_oproj_heads_negative.jsonl: the 8-way fan-in
        # tail ~4 us); "1": the hand-off kernel above; "0" (default): two kernels.  Both fused
        # kernels live in the opt-in experimental library (csrc/experimental).
        mode = os.environ.get("P2P_FUSED_ATTN_OPROJ", "0")
        self.fuse_attn_oproj = mode == "1"
        self.fuse_heads = mode == "heads"
        # decode (rows <= 16, contexts <= 256): qkv projection + RoPE + KV write + attention
        # as ONE launch (ops.qkv_attn): the attention's block-table -> K/V load chain runs
        # behind the qkv weight stream.  P2P_QKV_ATTN=0: the two kernels.
        self.fuse_qkv_attn = os.environ.get("P2P_QKV_ATTN", "1") == "1"
        # ... and, at TP = 1, the o_proj projection + residual in that same launch (the
        # producer workgroups take an o_proj column group after their qkv slice, weights in
        # registers, the attention output swept from tagged granules).  Opt-in
        # (P2P_QKV_ATTN_OPROJ=1): measured SLOWER than the separate o_proj launch at 8B --
        # 24.1 vs 21.5 us per layer at batch 1, 33.0 vs 25.1 at 8 rows
        # (profiles/r4_qkv_attn_oproj_negative.jsonl): the o_proj stream starts only when
        # a producer's qkv slice is done, so it does not hide behind the attention
        self.fuse_qkv_attn_oproj = os.environ.get("P2P_QKV_ATTN_OPROJ", "0") == "1"
        self.heads_max_rows = int(os.environ.get("P2P_HEADS_MAX_ROWS", "4"))
        # decode steps of <= 4 rows at contexts <= 256 (TP = 1, dense, bf16 weights): every
        # layer in ONE persistent launch (ops.decode_engine; hand-offs between workgroups
        # instead of kernel boundaries).  Opt-in (P2P_DECODE_ENGINE=1): measured SLOWER at
        # 8B -- 88-99 vs ~81 us per layer (profiles/r4_decode_engine_negative.jsonl): its
        # weight streams beat the separate kernels, but a chip-wide hand-off costs 3.5-5 us
        # under streaming load against ~1.5 us per kernel boundary
        self.decode_engine = os.environ.get("P2P_DECODE_ENGINE", "0") == "1"
        self._de = None
        self._de_ok = {}
        # TP prefill: row-parallel GEMMs of >= this many rows overlap their all-reduce
        # (chunked, separate communication stream); decode-size sums use the one-shot AR
        self.overlap_min_rows = int(os.environ.get("P2P_TP_OVERLAP_MIN_ROWS", "256"))
        self.overlap_chunks = int(os.environ.get("P2P_TP_OVERLAP_CHUNKS", "4"))
        # TP row-parallel projections of <= 64 rows (decode, short prompt chunks) on the
        # skinny kernel sum across ranks in their own epilogue (ops.skinny_gemm_ar): 5
        # launches per layer instead of 7.  P2P_TP_FUSED_AR=0: partial store + one-shot kernel
        self.fused_ar = os.environ.get("P2P_TP_FUSED_AR", "1") == "1"
        self._comm_stream = None
        # TP sampling reference path: gather the full logits row instead of per-shard top-128
        # candidates (same draw; tests compare the two on the same sharded numerics)
        self.sample_full_gather = False

    def new_workspace(self, max_rows, max_ctx, max_out_rows=None) -> Workspace:
        return Workspace(self.cfg, max_rows, max_ctx, self.device, self.tp, max_out_rows)

    # ----------------------------------------------------------------- layers
    def _row_parallel(self, wt, x, h, ws, R):
        """h += x @ W (row-parallel across TP ranks)."""
        if self.tp == 1:
            ops.skinny_gemm(wt, x, ops.EPI_RESID, out=h)
            return
        car = getattr(self.comm, "car", None)
        if (self.fused_ar and car is not None and h.device.type == "cuda"
                and ops.skinny_ar_ok(wt, R) and car.fused_ok(R, h.shape[1], h.stride(0))):
            # decode-size sums: the all-reduce + residual run in the GEMM's own epilogue
            ops.skinny_gemm_ar(wt, x, h, car)
            return
        part = ws.partial[:R]
        if R >= self.overlap_min_rows and h.device.type == "cuda":
            return self._row_parallel_overlapped(wt, x, h, part, R)
        ops.skinny_gemm(wt, x, ops.EPI_STORE, out=part)
        self.comm.allreduce_add_(h, part)

    def _row_parallel_overlapped(self, wt, x, h, part, R):
        """Prefill-size row-parallel sum with the all-reduce overlapped with the GEMM:
        the rows are cut into chunks; chunk i's all-reduce (RCCL over xGMI) + residual
        add run on a communication stream while the compute stream runs chunk i+1's
        GEMM (BASELINE north star: "RCCL all-reduce over xGMI overlapped with GEMMs")."""
        cur = torch.cuda.current_stream(h.device)
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(h.device)
        cs = self._comm_stream
        n = max(1, min(self.overlap_chunks, R // 64))
        step = -(-R // n)
        step = -(-step // 16) * 16  # whole 16-row MFMA tiles per chunk
        for a in range(0, R, step):
            b = min(R, a + step)
            ops.skinny_gemm(wt, x[a:b], ops.EPI_STORE, out=part[a:b])
            ev = torch.cuda.Event()
            ev.record(cur)
            with torch.cuda.stream(cs):
                cs.wait_event(ev)
                self.comm.allreduce_add_(h[a:b], part[a:b])
        cur.wait_stream(cs)
        return h

    def _mlp(self, lw, ws, R):
        h = ws.h[:R]
        if self.cfg.is_moe:
            from . import moe

            moe.moe_forward(self, lw, ws, R)
            return
        act = ws.act[:R]
        ops.skinny_gemm(lw.gate_up, h, ops.EPI_SILU, norm=True, out=act, eps=self.cfg.eps)
        self._row_parallel(lw.down, act, h, ws, R)

    def forward(self, ws: Workspace, ids, pos, slots, block_tables, row_bt, ctx_lens, R: int,
                max_ctx: int, out_rows=None, n_out: int | None = None, greedy: bool = False,
                tiles=None, tiles_host=None, qtile=None):
        """Run all layers on R query rows.

        out_rows: int32 [n_out] indices of rows whose logits are needed (prefill:
        the last token of each sequence); None = all R rows (decode).
        Returns fp32 logits of the selected rows, or with greedy=True the int64
        argmax keys (ws.keys, see ops.lm_head_argmax).
        tiles: int32 [n, 4] prefill query tiles (ops.prefill_tiles) -> causal
        attention runs on the MFMA flash-prefill kernel instead of per row.
        row_bt: block-table row of each query row; None = row r uses row r (decode).
        """
        cfg = self.cfg
        h = ws.h[:R]
        ops.gather_rows(self.w.embed, ids[:R], out=h)
        if (self.decode_engine and tiles is None and row_bt is None and out_rows is None
                and self._decode_engine_ok(R, max_ctx)):
            self._de.run(h, pos[:R], slots[:R], self.rope, block_tables, ctx_lens[:R], ws.err)
            return self._head(ws, h, R, out_rows, n_out, greedy)
        q, attn = ws.q[:R], ws.attn[:R]
        fused = (self.fuse_attn_oproj and tiles is None and self.tp == 1
                 and self.device.type == "cuda" and isinstance(self.w.layers[0].o, torch.Tensor)
                 and ops.attn_oproj_ok(R, self.nq, self.nkv, max_ctx, cfg.hidden))
        heads = (not fused and self.fuse_heads and tiles is None and ws.heads_slab is not None
                 and R <= self.heads_max_rows and isinstance(self.w.layers[0].o, torch.Tensor)
                 and ops.attn_oproj_heads_ok(R, self.nq, self.nkv, max_ctx, cfg.hidden))
        qa = (self.fuse_qkv_attn and not fused and not heads and tiles is None
              and row_bt is None and ws.qa is not None and isinstance(self.w.layers[0].qkv, torch.Tensor)
              and ops.qkv_attn_ok(R, self.nq, self.nkv, max_ctx))
        qa_o = (qa and self.fuse_qkv_attn_oproj and self.tp == 1
                and ops.qkv_attn_oproj_ok(self.w.layers[0].o, self.nq, self.nkv, rows=R,
                                          hidden=cfg.hidden))
        # contexts bounded by 128 keys (the 128-key decode graphs): 2 key waves per consumer
        qa_waves = None
        if qa and max_ctx <= 128 and not (ops.attention.QKV_ATTN_WAVES >> 16) & 0xff:
            qa_waves = ops.attention.QKV_ATTN_WAVES | (2 << 16)
        for i, lw in enumerate(self.w.layers):
            kc, vc = self.kv.layer(i)
            if qa:
                ops.qkv_attn(lw.qkv, h, pos[:R], slots[:R], self.rope, self.nq, self.nkv, kc, vc,
                             block_tables, ctx_lens[:R], attn, ws.qa, ws.err, eps=cfg.eps,
                             oproj=(lw.o, h) if qa_o else None, waves=qa_waves)
                if not qa_o:
                    self._row_parallel(lw.o, attn, h, ws, R)
                self._mlp(lw, ws, R)
                continue
            ops.qkv_rope_gemm(lw.qkv, h, pos[:R], slots[:R], self.rope, self.nq, self.nkv, q, kc,
                              vc, eps=cfg.eps)
            if heads:
                ops.attn_oproj_heads(q, kc, vc, block_tables,
                                     row_bt[:R] if row_bt is not None else None, ctx_lens[:R],
                                     self.nq, self.nkv, max_ctx, lw.o, h, ws.heads_slab,
                                     ws.heads_tickets)
            elif fused:
                rb = row_bt[:R] if row_bt is not None else ws.row_ids[:R]
                ops.attn_oproj(q, kc, vc, block_tables, rb, ctx_lens[:R], self.nq,
                               self.nkv, max_ctx, lw.o, h, attn, ws.sync, ws.err)
            else:
                if tiles is not None:
                    ops.flash_prefill(q, kc, vc, block_tables, tiles, self.nq, self.nkv, out=attn,
                                      tiles_host=tiles_host, qtile=qtile)
                else:
                    ops.paged_attention(q, kc, vc, block_tables,
                                        row_bt[:R] if row_bt is not None else None, ctx_lens[:R],
                                        self.nq, self.nkv, max_ctx, out=attn,
                                        workspace=ws.attn_ws)
                self._row_parallel(lw.o, attn, h, ws, R)
            self._mlp(lw, ws, R)
        return self._head(ws, h, R, out_rows, n_out, greedy)

    def _decode_engine_ok(self, R: int, max_ctx: int) -> bool:
        from ..ops.decode_engine import DecodeEngine, decode_engine_ok

        key = (R, max_ctx)
        ok = self._de_ok.get(key)
        if ok is None:
            ok = self._de_ok[key] = decode_engine_ok(self, R, max_ctx)
        if ok and self._de is None:
            self._de = DecodeEngine(self)
        return ok

    def _head(self, ws: Workspace, h, R: int, out_rows, n_out, greedy: bool):
        cfg = self.cfg
        if n_out == 0:
            return None
        if out_rows is None:
            x = h
            n = R
        else:
            n = n_out if n_out is not None else out_rows.shape[0]
            x = ops.gather_rows(h, out_rows[:n], out=ws.last[:n])
        if greedy:
            off = self.w.tp_rank * (cfg.vocab // self.tp)
            return ops.lm_head_argmax(self.w.lm_head, x, ws.keys, col_offset=off, eps=cfg.eps)
        logits = ws.logits[:n]
        ops.skinny_gemm(self.w.lm_head, x, ops.EPI_F32, norm=True, out=logits, eps=cfg.eps)
        return logits

    def check_faults(self, ws: Workspace):
        """Raise if a bounded wait timed out -- a fused kernel's cross-workgroup hand-off, a
        split-K GEMM slice, or a one-shot TP collective whose peer never arrived (the tokens
        would be wrong).  Call where the host syncs anyway (every rank of a TP/EP group at
        the same point).  A kernel fault is local to the rank that saw it, so a group first
        takes the MAX of the ranks' fault bits and every rank raises together (a follower
        raising alone would split the group and surface later as a collective timeout).
        A rank's own one-shot timeout (comm.check) is fault bit 4: it too is shared
        before raising, so the peers raise CollectiveTimeout with it instead of blocking
        in the MAX collective until the process-group timeout."""
        fault = 0
        if self.device.type == "cuda":
            if int(ws.err.item()) != 0:
                ws.err.zero_()
                fault |= 1
            if ops.tiled_split_fault():
                fault |= 2
        local_timeout = None
        if self.comm is not None and hasattr(self.comm, "check"):
            try:
                self.comm.check()
            except Exception as e:  # noqa: BLE001 -- raised below, after the group agrees
                local_timeout = e
                fault |= 4
        if self.comm is not None and getattr(self.comm, "world", 1) > 1 and \
                hasattr(self.comm, "max_int"):
            # every rank takes part in the MAX before anyone raises, so a rank whose own
            # one-shot wait timed out does not leave its peers blocked in this collective
            fault = self.comm.max_int(fault)
        if fault & 4:
            from ..parallel.custom_ar import CollectiveTimeout

            # name every wait that timed out in the group: a stuck in-launch hand-off or
            # split-K slice on one rank starves the others' collectives
            also = "".join(s for bit, s in ((1, "; an in-launch hand-off also timed out"),
                                            (2, "; a split-K slice wait also timed out"))
                           if fault & bit)
            if local_timeout is not None:
                raise CollectiveTimeout(str(local_timeout) + also) from local_timeout
            raise CollectiveTimeout("a one-shot collective timed out on a peer rank of the "
                                    "group (the TP group is broken)" + also)
        if fault & 1:
            raise RuntimeError("fused in-launch hand-off (qkv -> attention, attention -> "
                               "o_proj) timed out on a rank of the group (results invalid)")
        if fault & 2:
            raise RuntimeError("split-K GEMM slice wait timed out on a rank of the group "
                               "(results invalid)")

    def finalize_greedy(self, ws: Workspace, n: int, out=None):
        """keys -> token ids (TP: all-reduce MAX of the keys across vocab shards first)."""
        out = ws.ids_out[:n] if out is None else out
        if self.tp > 1:
            self.comm.allreduce_max_u64_(ws.keys[:n])
        return ops.argmax_finalize(ws.keys[:n], out)

    def sample_greedy(self, ws: Workspace, logits, out=None):
        n = logits.shape[0]
        out = ws.ids_out[:n] if out is None else out
        if self.tp == 1:
            return ops.argmax(logits, out=out)
        return self.comm.vocab_parallel_argmax(logits, out, self.cfg.vocab // self.tp)
