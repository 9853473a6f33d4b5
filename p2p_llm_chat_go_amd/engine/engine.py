"""In-process suggest-reply engine (replaces the reference's Ollama HTTP hop).

The reference's only LLM call is ``POST {OLLAMA_URL}/api/generate`` with
``stream: false`` (`web/streamlit_app.py:89-101`); Ollama answers with the
text plus ``prompt_eval_count/_duration`` and ``eval_count/_duration``.  This
engine produces the same record in-process:

  prefill   : all prompt tokens of the batch as one flat row list (chunked at
              ``max_prefill_tokens``), causal paged attention, LM head on the last
              row of each sequence only, greedy argmax -> first token (TTFT).
  decode    : hipGraph replay of the whole step (engine.graph), state advanced
              on the device; EOS is checked every ``check_every`` steps.

Continuous batching across peers lives in ``engine.scheduler``; this class is
the execution backend it drives (``prefill`` / ``decode_graph``).
"""
from __future__ import annotations

import dataclasses
import os
import time

import torch

from ..models.config import ModelConfig
from ..models.llama import LlamaModel
from ..models.weights import EngineWeights
from .. import ops
from ..utils.trace import span
from ..ops import PAGE
from .graph import PREFILL_ROW_BUCKETS, DecodeGraph, DecodeState, PrefillGraph
from .kv_cache import KVCache, pages_for

BATCH_BUCKETS = (1, 2, 4, 8, 16, 32, 64)
CTX_BUCKETS = (256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536, 131072)
# decode graphs also come in a 128-key bucket: a suggest-reply (a chat message + 64 new
# tokens) fits it, and its qkv+attention launch then runs 2-key-wave consumers (half the
# LDS, csrc/kernels/qkv_attn.hip launch-code bits 16..23): bench.py 364.4-365.3 ->
# 367.0-367.1 tok/s, alternating runs on one box (round 5)
DECODE_CTX_BUCKETS = (128,) + CTX_BUCKETS


def bucket(x, buckets):
    for b in buckets:
        if x <= b:
            return b
    raise ValueError("%d exceeds the largest bucket %d" % (x, buckets[-1]))


@dataclasses.dataclass
class GenResult:
    tokens: list
    prompt_eval_count: int
    prompt_eval_duration_ns: int
    eval_count: int
    eval_duration_ns: int
    total_duration_ns: int
    ttft_ns: int
    done_reason: str = "length"


class Engine:
    def __init__(self, cfg: ModelConfig, weights: EngineWeights | None = None, device="cuda",
                 seed: int = 0, kv_pages: int | None = None, max_prefill_tokens: int = 1024,
                 max_batch: int = 64, use_graph: bool = True, comm=None, tp_rank: int = 0,
                 tp_size: int = 1, kv_fraction: float = 0.85, ep_rank: int = 0,
                 ep_size: int = 1, ep_mode: str = "allreduce", weight_dtype: str | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        own = weights is None
        if own:
            weights = EngineWeights.random(cfg, self.device, seed=seed, tp_rank=tp_rank,
                                           tp_size=tp_size, ep_rank=ep_rank, ep_size=ep_size)
        # weight_dtype "fp8": weight-only e4m3 dense projections (EngineWeights.quantize_fp8)
        self.weight_dtype = weight_dtype or os.environ.get("ENGINE_WEIGHTS", "bf16")
        if self.weight_dtype == "fp8":
            # a caller's store stays bf16 (it may back a reference engine); ours is swapped
            weights = (weights if own else weights.shallow_copy()).quantize_fp8()
            if self.device.type == "cuda":
                # the bf16 originals and the quantizer's fp32 temporaries stay reserved in
                # torch's caching allocator; release them before sizing the KV pool
                torch.cuda.empty_cache()
        elif self.weight_dtype != "bf16":
            raise ValueError("weight_dtype must be bf16 or fp8, got %r" % self.weight_dtype)
        self.weights = weights
        if kv_pages is None:
            self.kv = KVCache.from_free_memory(cfg, self.device, fraction=kv_fraction,
                                               tp_size=tp_size)
        else:
            self.kv = KVCache(cfg, kv_pages, self.device, tp_size)
        if comm is not None and hasattr(comm, "setup"):
            comm.setup(self.device)
            if (cfg.is_moe and max(ep_size, weights.ep_size) > 1 and ep_mode == "a2a"
                    and self.device.type == "cuda" and hasattr(comm, "setup_ep_ipc")):
                # decode-size expert exchanges on the IPC kernels: up to the largest decode
                # bucket's rows x top_k slots per call (larger calls: RCCL exact counts)
                comm.setup_ep_ipc(cfg.top_k * bucket(max(1, min(max_batch, BATCH_BUCKETS[-1])),
                                                     BATCH_BUCKETS), cfg.hidden)
        self.model = LlamaModel(weights, self.kv, comm)
        # MoE expert parallelism: "allreduce" (replicated h) or "a2a" (DP attention,
        # tokens dispatched to expert owners; ranks must step in lockstep)
        self.model.ep_mode = ep_mode
        self.max_prefill_tokens = max_prefill_tokens
        # prefill chunks with at least this many rows use the MFMA flash kernel
        # (0 = always the per-row paged kernel)
        self.flash_prefill_min = int(os.environ.get("P2P_FLASH_PREFILL_MIN", "1"))
        self.max_batch = max_batch
        self.use_graph = use_graph
        self._prefill_ws = {}
        self._graphs = {}
        # graph-captured prefill chunks (engine.graph.PrefillGraph): dense TP=1 engines on
        # the GPU; P2P_PREFILL_GRAPH=0 keeps every prefill eager
        # TP groups: chunks whose every collective runs on the one-shot IPC kernels (the
        # row-parallel sums fit the IPC buffer: rows x hidden x 2 bytes), so the graph holds
        # no host-side collective; longer chunks stay eager.  Every rank decides alike (same
        # calls, same use counts), so the group's graphs pair up.
        car = getattr(comm, "car", None)
        self.prefill_graph_max_rows = PREFILL_ROW_BUCKETS[-1]
        if tp_size > 1:
            self.prefill_graph_max_rows = (car.max_bytes // (2 * cfg.hidden)) if car is not None else 0
        self.prefill_graphs_enabled = (
            use_graph and self.device.type == "cuda" and not cfg.is_moe
            and (tp_size == 1 or self.prefill_graph_max_rows >= PREFILL_ROW_BUCKETS[0])
            and os.environ.get("P2P_PREFILL_GRAPH", "1") != "0")
        self._pgraphs = {}
        # a chunk shape is captured once it has been seen this many times (eager before):
        # capturing costs ~3 forwards, so a shape seen once (a rare rider / batch mix) is
        # not worth it.  P2P_PREFILL_GRAPH_AFTER
        self.prefill_graph_after = int(os.environ.get("P2P_PREFILL_GRAPH_AFTER", "2"))
        self._pgraph_uses = {}

    # -------------------------------------------------------------- helpers
    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def prefill_workspace(self, max_ctx):
        key = bucket(max_ctx, CTX_BUCKETS)
        ws = self._prefill_ws.get(key)
        if ws is None:
            ws = self.model.new_workspace(self.max_prefill_tokens, key, max_out_rows=self.max_batch)
            self._prefill_ws[key] = ws
        return ws

    def decode_graph(self, B: int, ctx: int, greedy: bool = True) -> DecodeGraph:
        key = (bucket(B, BATCH_BUCKETS), bucket(ctx, DECODE_CTX_BUCKETS), greedy)
        g = self._graphs.get(key)
        if g is None:
            st = DecodeState(self.model, key[0], key[1] // PAGE, key[1], key[1])
            g = DecodeGraph(st, self.use_graph, greedy=greedy).capture()
            self._graphs[key] = g
        return g

    def prefill_graph_key(self, rows: int, n_seq: int, max_ctx: int, greedy: bool = True):
        return (bucket(rows, PREFILL_ROW_BUCKETS), min(bucket(n_seq, BATCH_BUCKETS), self.max_batch),
                bucket(max_ctx, CTX_BUCKETS), greedy)

    def prefill_graph_wanted(self, key) -> bool:
        """Count a use of this chunk shape; True once it is (or should now be) captured."""
        if key in self._pgraphs:
            return True
        n = self._pgraph_uses.get(key, 0) + 1
        self._pgraph_uses[key] = n
        return n >= self.prefill_graph_after

    def prefill_graph(self, rows: int, n_seq: int, max_ctx: int, greedy: bool = True) -> PrefillGraph:
        """The captured prefill of a chunk of <= ``rows`` rows from <= ``n_seq`` sequences
        (bucketed), contexts <= ``max_ctx``; captured on first call."""
        key = self.prefill_graph_key(rows, n_seq, max_ctx, greedy)
        rb, sb, cb, _ = key
        g = self._pgraphs.get(key)
        if g is None:
            g = PrefillGraph(self.model, self.prefill_workspace(cb), rb, sb, cb // PAGE, cb,
                             greedy=greedy).capture()
            self._pgraphs[key] = g
        return g

    def _graph_prefill_ok(self, n_rows: int, B: int, max_ctx: int, n_dummy: int,
                          return_logits: bool) -> bool:
        return (self.prefill_graphs_enabled and not return_logits and not n_dummy
                and n_rows <= min(self.max_prefill_tokens, self.prefill_graph_max_rows)
                and B <= self.max_batch and max_ctx <= CTX_BUCKETS[-1])

    def autotune(self, batch_sizes=(1,), verbose=False):
        """Pick the fastest GEMM launch configs for this model (before graph capture)."""
        from .autotune import autotune_model

        if self.device.type == "cuda" and os.environ.get("P2P_AUTOTUNE", "1") != "0":
            self.tuning = autotune_model(self.model, batch_sizes, verbose=verbose)
            self._share_tuning()
        return getattr(self, "tuning", {})

    def _share_tuning(self):
        """TP/EP: every rank adopts the group leader's launch codes.  The ranks must agree
        on which kernel runs a row-parallel projection (the fused all-reduce epilogue
        exists on the skinny kernel only), and a group steps at its slowest rank anyway."""
        comm = self.model.comm
        if comm is None or getattr(comm, "world", 1) <= 1:
            return
        import torch.distributed as dist

        from ..ops import gemm as G

        src = 0 if comm.group is None else dist.get_global_rank(comm.group, 0)
        box = [dict(G._TUNE), self.tuning]
        dist.broadcast_object_list(box, src=src, group=comm.group)
        G._TUNE.clear()
        G._TUNE.update(box[0])
        self.tuning = box[1]

    def warmup(self, batch_sizes=(1,), ctx=256, autotune=True):
        if autotune and not getattr(self, "tuning", None):
            # decode buckets + the prefill tile (prompt chunks run at M <= 64 rows per call)
            # decode buckets + prompt chunks of 33-48 rows (chat-length prompts) and 49-64
            self.autotune(tuple(bucket(b, BATCH_BUCKETS) for b in batch_sizes) + (48, 64))
        for b in batch_sizes:
            self.decode_graph(b, ctx)

    def check_comm(self):
        """Raise if a TP/EP collective timed out (a peer rank is dead or hung)."""
        comm = self.model.comm
        if comm is not None and hasattr(comm, "check"):
            comm.check()

    # -------------------------------------------------------------- prefill
    def prefill(self, prompts: list, block_tables: list, return_logits: bool = False,
                sampling: list | None = None, starts: list | None = None,
                pad_rows: int | None = None, graph: bool = True):
        """Run all prompts (flat rows, chunked at max_prefill_tokens); ``graph=False``
        keeps it off the captured-chunk path (the native loop owns that policy).

        Returns int32 first tokens [B] on the device (and, with return_logits,
        the fp32 last-position logits [B, V_local] of every sequence).
        sampling: one SamplingParams per prompt; non-greedy ones draw their first
        token with ops.sample (else every first token is the fused greedy argmax).
        starts: per sequence, the first position to run (the KV of earlier positions is
        already in its pages).  A running sequence rides along as one row (start =
        its last position): the server mixes decode rows into a prefill this way.
        pad_rows: run exactly this many rows (>= the real ones), the rest dummy rows of an
        extra sequence on the KV null page -- EP all-to-all ranks serving different
        sequences (DP attention) must run the same chunks with equal row counts.
        """
        sampled = sampling is not None and not all(p.greedy for p in sampling)
        dev = self.device
        B = len(prompts)
        rows = []  # (seq, pos, token)
        for b, p in enumerate(prompts):
            s0 = starts[b] if starts else 0
            rows += [(b, i, p[i]) for i in range(s0, len(p))]
        n_dummy = 0
        if pad_rows is not None:
            n_dummy = pad_rows - len(rows)
            assert n_dummy >= 0, (pad_rows, len(rows))
            rows += [(B, i, 0) for i in range(n_dummy)]  # sequence B: the null page
        max_ctx = max([len(p) for p in prompts] + [n_dummy, 1])
        if (graph and self._graph_prefill_ok(len(rows), B, max_ctx, n_dummy, return_logits) and
                self.prefill_graph_wanted(self.prefill_graph_key(len(rows), B, max_ctx,
                                                                 not sampled))):
            return self._prefill_graphed(prompts, block_tables, rows, max_ctx, sampling, sampled)
        ws = self.prefill_workspace(max_ctx)
        max_pages = bucket(max_ctx, CTX_BUCKETS) // PAGE
        bt = torch.zeros(B + (1 if n_dummy else 0),
                         max([max_pages] + [len(b) for b in block_tables]), dtype=torch.int32)
        for b, pages in enumerate(block_tables):
            bt[b, :len(pages)] = torch.tensor(pages, dtype=torch.int32)
        first = torch.zeros(B, dtype=torch.int32, device=dev)
        all_logits = None
        if return_logits:
            all_logits = torch.zeros(B, ws.logits.shape[1], dtype=torch.float32, device=dev)
        C = self.max_prefill_tokens
        for c0 in range(0, len(rows), C):
            chunk = rows[c0:c0 + C]
            R = len(chunk)
            seq = torch.tensor([r[0] for r in chunk], dtype=torch.int32)
            pos = torch.tensor([r[1] for r in chunk], dtype=torch.int32)
            ids = torch.tensor([r[2] for r in chunk], dtype=torch.int32)
            slots = bt[seq.long(), (pos // PAGE).long()] * PAGE + pos % PAGE
            if n_dummy:
                slots[seq == B] = -1  # dummy rows write no KV
            # rows that end a sequence inside this chunk need logits
            outs, out_seq = [], []
            for j, (b, i, _t) in enumerate(chunk):
                if b < B and i == len(prompts[b]) - 1:
                    outs.append(j)
                    out_seq.append(b)
            greedy = all_logits is None and not sampled
            tiles_h = qtile = None
            if self.flash_prefill_min and R >= self.flash_prefill_min:
                qtile = ops.flash_tile(self.model.nq, self.model.nkv, R)
                tiles_h = ops.prefill_tiles(seq.tolist(), pos.tolist(), qtile)
            # every host-built input of the chunk (block tables, row metadata, output rows,
            # flash tiles, result scatter) in ONE host->device copy: each separate copy of
            # a pageable tensor is a synchronous staging round trip before the first kernel
            parts = [bt.reshape(-1), seq, pos, ids, slots, pos + 1,
                     torch.tensor(outs or [0], dtype=torch.int32),
                     torch.tensor(out_seq or [0], dtype=torch.int32)]
            if tiles_h is not None:
                parts.append(tiles_h.reshape(-1))
            dev_all = torch.cat(parts).to(dev, non_blocking=True)
            o = bt.numel()
            bt_d = dev_all[:o].view(bt.shape)
            seq_d, pos_d, ids_d, slots_d, ctx_d = (dev_all[o + k * R:o + (k + 1) * R] for k in range(5))
            o += 5 * R
            n_o = max(1, len(outs))
            out_rows = dev_all[o:o + n_o]
            sel = dev_all[o + n_o:o + 2 * n_o].long()
            o += 2 * n_o
            tiles = None if tiles_h is None else dev_all[o:o + tiles_h.numel()].view(tiles_h.shape)
            res = self.model.forward(ws, ids_d, pos_d, slots_d, bt_d, seq_d, ctx_d, R,
                                     max_ctx, out_rows=out_rows, n_out=len(outs), greedy=greedy,
                                     tiles=tiles, tiles_host=tiles_h, qtile=qtile)
            if not outs:
                continue
            if greedy:
                toks = self.model.finalize_greedy(ws, len(outs))
            elif sampled:
                from .sampling import sample, sample_tp

                params = [sampling[b] for b in out_seq]
                spos = [len(prompts[b]) - 1 for b in out_seq]
                if self.model.tp == 1:
                    toks = sample(res, params, spos)
                elif getattr(self.model, "sample_full_gather", False):  # reference path (tests)
                    toks = sample(self.model.comm.all_gather_cols(res), params, spos)
                else:
                    toks = sample_tp(self.model, res, params, spos)
            else:
                toks = self.model.sample_greedy(ws, res)
            first.index_copy_(0, sel, toks)
            if all_logits is not None:
                all_logits.index_copy_(0, sel, res)
        return (first, all_logits) if return_logits else first

    def _prefill_graphed(self, prompts, block_tables, rows, max_ctx, sampling, sampled):
        """One chunk through its captured graph: one metadata copy + one graph launch."""
        B = len(prompts)
        g = self.prefill_graph(len(rows), B, max_ctx, greedy=not sampled)
        last = [0] * B
        for j, r in enumerate(rows):  # rows are grouped by sequence, in order
            last[r[0]] = j
        g.load(g.host_meta(rows, block_tables, last))
        if sampled:
            g.samp._key = None  # the native loop may have written these slots directly
            g.samp.load(list(sampling))
        g.replay()
        return g.first[:B]

    # --------------------------------------------------------------- decode
    def decode_steps(self, last_ids: list, pos: list, block_tables: list, ctx: int, k: int,
                     params: list | None = None, batch_bucket: int | None = None,
                     greedy: bool | None = None) -> list:
        """k decode steps for running sequences (continuous batching): row b continues
        from token ``last_ids[b]`` at position ``pos[b]`` in its pages; ``params`` =
        per-row SamplingParams (None / all greedy: the fused-argmax graph).  Returns the
        k new tokens of every row (host lists).  Every TP/EP rank makes the same call
        (engine.cluster broadcasts it), so the graphs' collectives line up.
        batch_bucket: run the graph of this many rows (>= len(last_ids); DP-attention EP
        ranks with different batches must replay the same bucket).
        greedy: the graph kind when the caller decides it for the whole group (DP-attention
        shares: one rank's all-greedy share still replays the sampled graph when another
        rank's share samples -- a graph kind captured on one rank only would run its capture
        warmup's collectives alone)."""
        if greedy is None:
            greedy = params is None or all(p.greedy for p in params)
        elif not greedy and params is None:
            params = []
        g = self.decode_graph(max(len(last_ids), batch_bucket or 1), ctx, greedy=greedy)
        st = g.state
        st.load(last_ids, pos, block_tables)
        if greedy:
            g.replay(k)
        else:
            g.step_sampled(params, k)
        hist = st.hist[:len(last_ids), :k].cpu().tolist()
        self.model.check_faults(st.ws)
        return hist

    # ------------------------------------------------------------- generate
    def generate(self, prompts: list, max_new_tokens: int = 64, stop_on_eos: bool = True,
                 check_every: int = 8) -> list:
        """Greedy suggest-reply for a static batch of prompts (token id lists)."""
        t0 = time.perf_counter_ns()
        B = len(prompts)
        assert 0 < B <= self.max_batch
        need = [len(p) + max_new_tokens for p in prompts]
        pages = [self.kv.allocator.alloc(pages_for(n)) for n in need]
        try:
            with span("prefill", batch=B, tokens=sum(len(p) for p in prompts)):
                first = self.prefill(prompts, pages)
                first_h = first.cpu()  # sync: first token is on the host -> TTFT
            self.check_comm()
            t1 = time.perf_counter_ns()
            out = [[int(first_h[b])] for b in range(B)]
            done = [stop_on_eos and out[b][0] in self.cfg.eos_ids for b in range(B)]
            n_dec = max_new_tokens - 1
            steps_run = 0
            if n_dec > 0 and not all(done):
                g = self.decode_graph(B, max(need))
                st = g.state
                st.load([o[0] for o in out], [len(p) for p in prompts], pages)
                while steps_run < n_dec:
                    k = n_dec - steps_run if not stop_on_eos else min(check_every,
                                                                      n_dec - steps_run)
                    with span("decode", batch=B, steps=k):
                        g.replay(k)
                    steps_run += k
                    if stop_on_eos:
                        h = st.hist[:B, :steps_run].cpu()
                        for b in range(B):
                            if not done[b] and any(int(t) in self.cfg.eos_ids for t in h[b]):
                                done[b] = True
                        if all(done):
                            break
                hist = st.hist[:B, :steps_run].cpu()
                self.model.check_faults(st.ws)
                for b in range(B):
                    out[b] += [int(t) for t in hist[b]]
            else:
                self._sync()
            t2 = time.perf_counter_ns()
        finally:
            for p in pages:
                self.kv.allocator.free(p)
        res = []
        for b in range(B):
            toks = out[b][:max_new_tokens]
            reason = "length"
            if stop_on_eos:
                for j, t in enumerate(toks):
                    if t in self.cfg.eos_ids:
                        toks = toks[:j]
                        reason = "stop"
                        break
            res.append(GenResult(tokens=toks, prompt_eval_count=len(prompts[b]),
                                 prompt_eval_duration_ns=t1 - t0, eval_count=len(toks),
                                 eval_duration_ns=t2 - t1, total_duration_ns=t2 - t0,
                                 ttft_ns=t1 - t0, done_reason=reason))
        return res
