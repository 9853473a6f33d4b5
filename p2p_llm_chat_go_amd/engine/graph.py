"""hipGraph-captured decode steps (one graph per batch-size / context bucket).

A decode step is ~200 kernel launches for Llama-3.1-8B (6 per layer + head);
eager launch overhead (~3-4 us each on the host) would exceed the GPU time.
The whole step -- embedding gather, 32 layers, LM head, greedy argmax, and the
device-side state advance (positions, KV slots, output history) -- is
captured once per bucket with ``torch.cuda.graph`` (hipGraph underneath) and
replayed.  Because the step advances its own state on the device, N tokens
are N back-to-back replays with no host synchronisation in between.

Graphs are captured on dummy state that points every row at the KV null page
(page 0); real sequences are loaded into the same static buffers before
replay.  Padding rows of a bucket stay on the null page.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import ops
from ..ops import PAGE


class DecodeState:
    def __init__(self, model, B: int, max_pages: int, max_steps: int, max_ctx: int):
        dev = model.device
        i32 = torch.int32
        self.model = model
        self.B = B
        self.max_pages = max_pages
        self.max_steps = max_steps
        self.max_ctx = max_ctx
        # ids | pos | ctx | slots | block tables: views of ONE device buffer, so `load`
        # refreshes a batch's whole state with one host->device copy
        self.meta = torch.zeros(B * (4 + max_pages), device=dev, dtype=i32)
        self.ids, self.pos, self.ctx, self.slots = (self.meta[k * B:(k + 1) * B] for k in range(4))
        self.bt = self.meta[4 * B:].view(B, max_pages)
        self.ctx.fill_(1)
        self.row_bt = torch.arange(B, device=dev, dtype=i32)
        self.hist = torch.zeros(B, max_steps, device=dev, dtype=i32)
        self.step = torch.zeros(1, device=dev, dtype=i32)
        self.ws = model.new_workspace(B, max_ctx)
        from .sampling import SamplerSlots

        self.samp = SamplerSlots(B, dev)  # sampled graphs read these (ops.sample)
        if model.tp > 1:  # vocab-parallel sampling: per-shard top-128 candidates, gathered
            W = model.tp
            self.cand_v = torch.empty(B, 128, device=dev, dtype=torch.float32)
            self.cand_id = torch.empty(B, 128, device=dev, dtype=torch.int32)
            self.cand_all_v = torch.empty(W * B, 128, device=dev, dtype=torch.float32)
            self.cand_all_id = torch.empty(W * B, 128, device=dev, dtype=torch.int32)

    def reset_dummy(self):
        self.ids.zero_()
        self.pos.zero_()
        self.ctx.fill_(1)
        self.slots.zero_()
        self.bt.zero_()
        self.step.zero_()
        self.ws.keys.zero_()

    def load(self, ids, pos, block_tables):
        """ids/pos: int lists (n <= B); block_tables: list of page lists."""
        n = len(ids)
        B = self.B
        assert n <= B
        self.step.zero_()
        self.ws.keys.zero_()
        host = torch.zeros(B * (4 + self.max_pages), dtype=torch.int32)
        bt = host[4 * B:].view(B, self.max_pages)
        for b, pages in enumerate(block_tables):
            bt[b, :len(pages)] = torch.tensor(pages, dtype=torch.int32)
        p = host[B:2 * B]
        p[:n] = torch.tensor(pos, dtype=torch.int32)
        host[:n] = torch.tensor(ids, dtype=torch.int32)
        host[2 * B:3 * B] = p + 1
        host[3 * B:4 * B] = bt.gather(1, (p // PAGE).long()[:, None])[:, 0] * PAGE + p % PAGE
        self.meta.copy_(host, non_blocking=True)  # rows >= n: dummies (page 0, position 0)

    def body_logits(self):
        """Forward only (sampling mode): logits of every row in ws.logits."""
        self.model.forward(self.ws, self.ids, self.pos, self.slots, self.bt, None,
                           self.ctx, self.B, self.max_ctx)

    def advance(self):
        ops.advance(self.ids, self.pos, self.ctx, self.slots, self.bt, self.hist, self.step)

    def body_sampled(self):
        """Forward + on-device sampling (ops.sample, per-row params in self.samp) +
        advance: a sampled decode step as one graph replay."""
        self.body_logits()
        logits = self.ws.logits[:self.B]
        m = self.model
        sp = self.samp
        if m.tp > 1 and getattr(m, "sample_full_gather", False):  # reference path (tests)
            full = m.comm.all_gather_cols(logits)
            ops.sample(full, sp.temp, sp.topk, sp.topp, sp.seeds, self.pos, out=self.ids)
        elif m.tp > 1:
            # vocab-parallel LM head: each rank keeps its shard's top-128 (value, id) pairs,
            # one all-gather of B x world x 128 candidates (not B x V logits), and every rank
            # draws the same token as the unsharded sampler (the draw is capped at top-128)
            ops.topk_candidates(logits, m.w.tp_rank * (m.cfg.vocab // m.tp), self.cand_v,
                                self.cand_id)
            m.comm.all_gather_rows_into(self.cand_all_v, self.cand_v)
            m.comm.all_gather_rows_into(self.cand_all_id, self.cand_id)
            ops.sample_candidates(self.cand_all_v, self.cand_all_id, m.tp, sp.temp, sp.topk,
                                  sp.topp, sp.seeds, self.pos, out=self.ids)
        else:
            ops.sample(logits, sp.temp, sp.topk, sp.topp, sp.seeds, self.pos, out=self.ids)
        self.advance()

    def body(self):
        m = self.model
        keys = m.forward(self.ws, self.ids, self.pos, self.slots, self.bt, None, self.ctx,
                         self.B, self.max_ctx, greedy=True)
        if m.tp > 1:
            m.comm.allreduce_max_u64_(keys[:self.B])
        # keys -> ids (+ reset) folded into the state advance: no extra launch
        ops.advance(self.ids, self.pos, self.ctx, self.slots, self.bt, self.hist, self.step,
                    keys=keys[:self.B])


class DecodeGraph:
    """greedy=True: the whole step incl. argmax + advance is one graph replay.
    greedy=False: the graph computes logits; sampling + advance run after it."""

    def __init__(self, state: DecodeState, use_graph: bool = True, greedy: bool = True):
        self.state = state
        self.graph = None
        self.greedy = greedy
        self.use_graph = use_graph and state.model.device.type == "cuda"
        # multi-step graph (see _capture_steps).  A TP / EP group captures it collectively:
        # every rank captures the same K steps for the same shapes (the Python lockstep
        # replays the same n on every rank; the native group loop mirrors the leader's
        # provider calls), and the IPC collectives keep their epochs on the device, so K
        # recorded steps replay like K launches (P2P_GROUP_GRAPH_STEPS overrides for groups)
        comm = getattr(state.model, "comm", None)
        solo = getattr(comm, "world", 1) <= 1
        k = os.environ.get("P2P_DECODE_GRAPH_STEPS", "8")
        self.k_steps = int(k if solo else os.environ.get("P2P_GROUP_GRAPH_STEPS", k))
        self.graph_k = None

    def _body(self):
        if self.greedy:
            self.state.body()
        else:
            self.state.body_sampled()

    def capture(self, warmup: int = 2):
        st = self.state
        if not self.use_graph:
            return self
        st.reset_dummy()
        s = torch.cuda.Stream(st.model.device)
        s.wait_stream(torch.cuda.current_stream(st.model.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream(st.model.device).wait_stream(s)
        torch.cuda.synchronize(st.model.device)
        st.reset_dummy()
        g = torch.cuda.CUDAGraph()
        try:
            # thread_local: HIP calls other threads make meanwhile (a serving loop's host
            # copies, a collective's helper threads) are not this capture's business
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._body()
        except Exception as e:  # e.g. a collective backend that cannot be captured
            import os
            import traceback
            import warnings

            comm = st.model.comm
            if (getattr(comm, "world", 1) > 1 and st.model.device.type == "cuda"
                    and os.environ.get("P2P_ALLOW_EAGER", "0") != "1"):
                # a TP / EP group must not silently lose its graphs (eager group decode is
                # several times slower); P2P_ALLOW_EAGER=1 accepts it
                raise RuntimeError("group decode graph capture failed: %s (set "
                                   "P2P_ALLOW_EAGER=1 to run the step eagerly)\n%s"
                                   % (e, traceback.format_exc())) from e
            warnings.warn("decode graph capture failed (%s); running the step eagerly\n%s"
                          % (e, traceback.format_exc()))
            torch.cuda.synchronize(st.model.device)
            st.reset_dummy()
            self.graph = None
            return self
        torch.cuda.synchronize(st.model.device)
        st.reset_dummy()
        self.graph = g
        return self

    def _capture_steps(self):
        """The greedy step captured K times in ONE graph (P2P_DECODE_GRAPH_STEPS, default 8;
        single-device engines).  Measured (bench/graph_switch_probe.py,
        profiles/r4_graph_switch_probe.jsonl): every launch of the one-step graph leaves
        ~8 us of host work that the NEXT launch of a different graph (the prompt chunk)
        pays, 0.5 ms after a 63-step reply -- on the next request's TTFT.  K steps per
        launch cut the launches K-fold.  Capture only records (nothing runs), so the
        loaded batch state is untouched."""
        st = self.state
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for _ in range(self.k_steps):
                    self._body()
        except Exception:  # noqa: BLE001 -- keep the one-step graph
            torch.cuda.synchronize(st.model.device)
            self.graph_k = False
            return
        self.graph_k = g

    def replay(self, n: int = 1):
        assert self.greedy
        if self.graph is None:
            for _ in range(n):
                self.state.body()
            return
        K = self.k_steps
        if n >= K > 1 and self.graph_k is not False:
            if self.graph_k is None:
                self._capture_steps()
            if self.graph_k:
                while n >= K:
                    self.graph_k.replay()
                    n -= K
        for _ in range(n):
            self.graph.replay()

    def describe(self) -> dict:
        """Addresses and layout for the native loop (runtime/engine_loop.h DecodeGraphDesc)."""
        st = self.state
        d = {"B": st.B, "max_pages": st.max_pages, "ctx": st.max_ctx, "greedy": self.greedy,
             "exec": self.graph.raw_cuda_graph_exec(), "meta": st.meta.data_ptr(),
             "hist": st.hist.data_ptr(), "max_steps": st.max_steps, "step": st.step.data_ptr(),
             "keys": st.ws.keys.data_ptr(), "keys_bytes": st.ws.keys.numel() * 8,
             "err": st.ws.err.data_ptr()}
        if self.graph_k:
            d.update(exec_k=self.graph_k.raw_cuda_graph_exec(), k_steps=self.k_steps)
        if not self.greedy:
            sp = st.samp
            d.update(temp=sp.temp.data_ptr(), topk=sp.topk.data_ptr(), topp=sp.topp.data_ptr(),
                     seeds=sp.seeds.data_ptr())
        return d

    def step_sampled(self, params: list, n: int = 1):
        """n decode steps with per-row SamplingParams (temperature <= 0 rows stay greedy):
        the parameters are loaded into device slots (only when they change), then each
        step is one replay -- forward, ops.sample and advance are all in the graph."""
        assert not self.greedy
        self.state.samp.load(params)
        for _ in range(n):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.state.body_sampled()


# rows of a captured prefill (a chunk of <= max_prefill_tokens rows is padded up to the
# next bucket with dummy rows on the KV null page)
PREFILL_ROW_BUCKETS = (16, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768, 1024)


class PrefillGraph:
    """A whole prefill chunk -- embedding gather, every layer (fused-epilogue GEMMs, flash
    prefill attention on paged KV), last-row gather, LM head and the greedy argmax (or the
    fp32 logits for sampled requests) -- captured as ONE hipGraph per (row bucket, sequence
    bucket, context bucket).

    Eager prefill issues ~170 launches from Python per chunk; on a slow host that, not the
    GPU, sets the time to first token.  Replaying a graph costs one host->device copy of the
    chunk's metadata (``load``) plus one ``hipGraphLaunch``.

    Every launch parameter is static per bucket; what varies per chunk lives in one device
    int32 buffer (``meta``): block tables (``n_seq`` + 1 rows; the last one is the dummy
    sequence on the null page), per-row sequence / position / token / KV slot / context,
    the output rows, and the flash-attention query tiles (padded to ``max_tiles`` with
    zero-length tiles, which the kernel skips).  Dummy rows carry slot -1 (no KV write)."""

    def __init__(self, model, ws, rows: int, n_seq: int, max_pages: int, max_ctx: int,
                 greedy: bool = True):
        dev = model.device
        self.model, self.ws = model, ws
        self.rows, self.n_seq, self.max_pages, self.max_ctx = rows, n_seq, max_pages, max_ctx
        self.n_out = n_seq
        self.greedy = greedy
        self.qtile = ops.flash_tile(model.nq, model.nkv, rows)
        # tiles never straddle sequences: <= rows / qtile + one partial tile per sequence
        # (the dummy sequence included) + one per wrap of the dummy rows' positions
        self.max_tiles = -(-rows // self.qtile) + n_seq + 1 + rows // (max_pages * PAGE) + 1
        R, S = rows, n_seq
        sizes = [("bt", (S + 1) * max_pages), ("seq", R), ("pos", R), ("ids", R), ("slots", R),
                 ("ctx", R), ("out", S), ("spos", S), ("tiles", 4 * self.max_tiles)]
        self.offsets = {}
        o = 0
        for name, n in sizes:
            self.offsets[name] = (o, n)
            o += n
        self.meta = torch.zeros(o, device=dev, dtype=torch.int32)
        v = {name: self.meta[a:a + n] for name, (a, n) in self.offsets.items()}
        self.bt = v["bt"].view(S + 1, max_pages)
        self.seq, self.pos, self.ids, self.slots, self.ctx = (v[k] for k in ("seq", "pos", "ids",
                                                                               "slots", "ctx"))
        self.out_rows = v["out"]
        self.spos = v["spos"]  # position each output row's token is drawn for (sampling)
        self.tiles = v["tiles"].view(self.max_tiles, 4)
        self.first = torch.zeros(S, device=dev, dtype=torch.int32)
        self.samp = None
        if not greedy:  # per-sequence sampling parameters, read by the captured ops.sample
            from .sampling import SamplerSlots

            self.samp = SamplerSlots(S, dev)
            if model.tp > 1:  # vocab-parallel draw: top-128 per shard, one all-gather
                W = model.tp
                self.cand_v = torch.empty(S, 128, device=dev, dtype=torch.float32)
                self.cand_id = torch.empty(S, 128, device=dev, dtype=torch.int32)
                self.cand_all_v = torch.empty(W * S, 128, device=dev, dtype=torch.float32)
                self.cand_all_id = torch.empty(W * S, 128, device=dev, dtype=torch.int32)
        self.graph = None

    # ------------------------------------------------------------------ host side
    def host_meta(self, rows: list, block_tables: list, out_rows: list) -> torch.Tensor:
        """The ``meta`` image of one chunk: rows = [(seq, pos, token)] (sequences
        consecutive, in order), block_tables[s] = page list of sequence s, out_rows = the
        row of each sequence whose logits are needed (its last).  numpy throughout: this
        runs on the TTFT path, once per prefill."""
        R, S, P = self.rows, self.n_seq, self.max_pages
        n = len(rows)
        assert n <= R and len(block_tables) <= S and len(out_rows) <= S, (n, len(block_tables))
        host = np.zeros(self.meta.numel(), dtype=np.int32)
        v = {name: host[a:a + k] for name, (a, k) in self.offsets.items()}
        bt = v["bt"].reshape(S + 1, P)
        for s, pages in enumerate(block_tables):
            # callers pass a sequence's whole allocation (prompt + max_new pages); the chunk
            # reads only the pages of its context bucket, so the rest is cut off here (the
            # native loop does the same, runtime/engine_loop.cc)
            pages = pages[:P]
            bt[s, :len(pages)] = pages
        seq, pos = v["seq"], v["pos"]
        if n:
            a = np.asarray(rows, dtype=np.int32).reshape(n, 3)
            seq[:n], pos[:n], v["ids"][:n] = a[:, 0], a[:, 1], a[:, 2]
            assert int(a[:, 1].max()) < P * PAGE, (int(a[:, 1].max()), P)
        seq[n:] = S  # dummy rows: sequence S (the null page), positions 0.. wrapped inside
        pos[n:] = np.arange(R - n, dtype=np.int32) % (P * PAGE)  # its block-table row
        slots = bt[seq, pos // PAGE] * PAGE + pos % PAGE
        slots[n:] = -1  # dummy rows write no KV
        v["slots"][:] = slots
        v["ctx"][:] = pos + 1
        v["out"][:len(out_rows)] = out_rows
        v["spos"][:] = pos[v["out"]]
        # query tiles: runs of consecutive positions of one sequence, cut at qtile rows
        # (ops.prefill_tiles); the rest stay n = 0 padding tiles
        brk = np.flatnonzero((seq[1:] != seq[:-1]) | (pos[1:] != pos[:-1] + 1)) + 1
        bounds = np.concatenate(([0], brk, [R]))
        tl = []
        q = self.qtile
        for r0, r1 in zip(bounds[:-1].tolist(), bounds[1:].tolist()):
            for t0 in range(r0, r1, q):
                tl.append((t0, min(q, r1 - t0), int(seq[t0]), int(pos[t0])))
        assert len(tl) <= self.max_tiles, (len(tl), self.max_tiles)
        v["tiles"][:4 * len(tl)] = np.asarray(tl, dtype=np.int32).reshape(-1)
        return torch.from_numpy(host)

    def load(self, host: torch.Tensor):
        self.meta.copy_(host, non_blocking=True)

    # ------------------------------------------------------------------ device side
    def body(self):
        m, ws = self.model, self.ws
        res = m.forward(ws, self.ids, self.pos, self.slots, self.bt, self.seq, self.ctx,
                        self.rows, self.max_ctx, out_rows=self.out_rows, n_out=self.n_out,
                        greedy=self.greedy, tiles=self.tiles, qtile=self.qtile)
        if self.greedy:
            m.finalize_greedy(ws, self.n_out, out=self.first)
        elif m.tp > 1:  # the shard's logits: the same draw as the decode graph's (DecodeState)
            sp, lg = self.samp, ws.logits[:self.n_out]
            ops.topk_candidates(lg, m.w.tp_rank * (m.cfg.vocab // m.tp), self.cand_v, self.cand_id)
            m.comm.all_gather_rows_into(self.cand_all_v, self.cand_v)
            m.comm.all_gather_rows_into(self.cand_all_id, self.cand_id)
            ops.sample_candidates(self.cand_all_v, self.cand_all_id, m.tp, sp.temp, sp.topk,
                                  sp.topp, sp.seeds, self.spos, out=self.first)
        else:
            sp = self.samp
            ops.sample(ws.logits[:self.n_out], sp.temp, sp.topk, sp.topp, sp.seeds, self.spos,
                       out=self.first)
        return res

    def capture(self, warmup: int = 2):
        dev = self.model.device
        # a valid dummy chunk (every row on the null page) for the warmup runs and capture
        self.load(self.host_meta([], [], []))
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):  # sizes lazily-grown workspaces before capture
                self.body()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.body()
        torch.cuda.synchronize(dev)
        self.graph = g
        return self

    def replay(self):
        """Runs the loaded chunk: the first token of every sequence lands in
        ``self.first[:n]`` (greedy argmax, or drawn with the parameters loaded into
        ``self.samp``); the sampled graph also leaves the fp32 logits of the output rows in
        ``self.ws.logits[:n]``.  Both are overwritten by the next replay."""
        self.graph.replay()

    def describe(self) -> dict:
        """Addresses and layout for the native loop (runtime/engine_loop.h PrefillGraphDesc)."""
        d = {"rows": self.rows, "n_seq": self.n_seq, "max_pages": self.max_pages,
             "qtile": self.qtile, "max_tiles": self.max_tiles, "greedy": self.greedy,
             "exec": self.graph.raw_cuda_graph_exec(), "meta": self.meta.data_ptr(),
             "meta_len": self.meta.numel(), "first": self.first.data_ptr(),
             "err": self.ws.err.data_ptr()}
        for name, (a, _n) in self.offsets.items():
            d["off_" + name] = a
        if self.samp is not None:
            d.update(temp=self.samp.temp.data_ptr(), topk=self.samp.topk.data_ptr(),
                     topp=self.samp.topp.data_ptr(), seeds=self.samp.seeds.data_ptr())
        return d
