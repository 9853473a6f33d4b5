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
            with torch.cuda.graph(g):
                self._body()
        except Exception as e:  # e.g. a collective backend that cannot be captured
            import os
            import warnings

            if st.model.tp > 1 and os.environ.get("P2P_ALLOW_EAGER", "0") != "1":
                # a TP group must not silently lose its graphs (eager TP decode is several
                # times slower); P2P_ALLOW_EAGER=1 accepts it
                raise RuntimeError("TP decode graph capture failed: %s (set P2P_ALLOW_EAGER=1 to "
                                   "run the step eagerly)" % e) from e
            warnings.warn("decode graph capture failed (%s); running the step eagerly" % e)
            torch.cuda.synchronize(st.model.device)
            st.reset_dummy()
            self.graph = None
            return self
        torch.cuda.synchronize(st.model.device)
        st.reset_dummy()
        self.graph = g
        return self

    def replay(self, n: int = 1):
        assert self.greedy
        for _ in range(n):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.state.body()

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
