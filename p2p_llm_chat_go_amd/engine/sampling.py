"""Token sampling: greedy (fused into the LM head kernel, see ops.lm_head_argmax)
and Ollama-style temperature / top-k / top-p sampling for requests that ask for
it (``options`` of ``/api/generate``; Ollama's defaults are temperature 0.8,
top_k 40, top_p 0.9).

The stochastic path is ``ops.sample`` (csrc/kernels/sampling.hip), captured in
the decode graph right after the LM head: top-k first (k <= 128, radix select,
so the full-vocab softmax is never materialised), then top-p over the k
survivors, then an exponential-race draw (argmax of p / Exp(1)), equivalent to
multinomial sampling.  The random stream is keyed by (request seed, position,
token id), so replays draw fresh numbers with no host state and a given seed
reproduces a reply.  Rows with temperature <= 0 are greedy.
"""
from __future__ import annotations

import dataclasses
import random

import torch


@dataclasses.dataclass
class SamplingParams:
    temperature: float = 0.0   # 0 = greedy (engine default: deterministic)
    top_k: int = 40
    top_p: float = 0.9
    seed: int | None = None
    max_tokens: int = 128
    stop_on_eos: bool = True

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0

    def resolved_seed(self) -> int:
        """The request's random-stream key: ``seed`` if given, else drawn once per request."""
        if self.seed is None:
            self.seed = random.getrandbits(62)
        return int(self.seed) & ((1 << 63) - 1)

    @classmethod
    def from_ollama(cls, options: dict | None, default_max: int = 128) -> "SamplingParams":
        o = options or {}
        n = int(o.get("num_predict", default_max))
        if n < 0:
            n = default_max
        # ignore_eos (llama.cpp server option; benchmarks): decode exactly num_predict tokens
        return cls(temperature=float(o.get("temperature", 0.0)), top_k=int(o.get("top_k", 40)),
                   top_p=float(o.get("top_p", 0.9)), seed=o.get("seed"), max_tokens=max(1, n),
                   stop_on_eos=not bool(o.get("ignore_eos", False)))


class SamplerSlots:
    """Per-row sampling parameters of a decode batch as device tensors, read by the
    graph-captured ``ops.sample`` launch (so a sampled decode step replays like a
    greedy one).  ``load`` copies only when the batch's parameters change."""

    def __init__(self, B: int, device):
        self.B = B
        self.temp = torch.zeros(B, device=device, dtype=torch.float32)
        self.topk = torch.full((B,), 40, device=device, dtype=torch.int32)
        self.topp = torch.full((B,), 0.9, device=device, dtype=torch.float32)
        self.seeds = torch.zeros(B, device=device, dtype=torch.int64)
        self._key = None

    def load(self, params: list):
        params = list(params[:self.B]) + [SamplingParams()] * (self.B - len(params))
        key = tuple((p.temperature, p.top_k, p.top_p, p.resolved_seed()) for p in params)
        if key == self._key:
            return
        self.temp.copy_(torch.tensor([k[0] for k in key], dtype=torch.float32))
        self.topk.copy_(torch.tensor([k[1] for k in key], dtype=torch.int32))
        self.topp.copy_(torch.tensor([k[2] for k in key], dtype=torch.float32))
        self.seeds.copy_(torch.tensor([k[3] for k in key], dtype=torch.int64))
        self._key = key


def sample(logits: torch.Tensor, params: list, pos) -> torch.Tensor:
    """logits [B, V] fp32 -> int32 token ids [B] (one SamplingParams per row; pos =
    the position each row's token is drawn for).  Runs ops.sample (the GPU kernel,
    or its PyTorch reference on CPU tensors)."""
    from .. import ops

    B = logits.shape[0]
    params = list(params[:B]) + [SamplingParams()] * (B - len(params))
    dev = logits.device
    temp = torch.tensor([p.temperature for p in params], dtype=torch.float32).to(dev)
    topk = torch.tensor([p.top_k for p in params], dtype=torch.int32).to(dev)
    topp = torch.tensor([p.top_p for p in params], dtype=torch.float32).to(dev)
    seeds = torch.tensor([p.resolved_seed() for p in params], dtype=torch.int64).to(dev)
    pos = torch.as_tensor(pos, dtype=torch.int32).to(dev)
    return ops.sample(logits, temp, topk, topp, seeds, pos)


def sample_tp(model, logits: torch.Tensor, params: list, pos) -> torch.Tensor:
    """Vocab-parallel ``sample`` (TP prefill): per-shard top-128 candidates, one all-gather,
    then the same draw on every rank (see DecodeState.body_sampled)."""
    from .. import ops

    B = logits.shape[0]
    params = list(params[:B]) + [SamplingParams()] * (B - len(params))
    dev = logits.device
    W = model.tp
    temp = torch.tensor([p.temperature for p in params], dtype=torch.float32).to(dev)
    topk = torch.tensor([p.top_k for p in params], dtype=torch.int32).to(dev)
    topp = torch.tensor([p.top_p for p in params], dtype=torch.float32).to(dev)
    seeds = torch.tensor([p.resolved_seed() for p in params], dtype=torch.int64).to(dev)
    posd = torch.tensor(list(pos), dtype=torch.int32).to(dev)
    cv = torch.empty(B, 128, device=dev, dtype=torch.float32)
    ci = torch.empty(B, 128, device=dev, dtype=torch.int32)
    ops.topk_candidates(logits, model.w.tp_rank * (model.cfg.vocab // W), cv, ci)
    av = torch.empty(W * B, 128, device=dev, dtype=torch.float32)
    ai = torch.empty(W * B, 128, device=dev, dtype=torch.int32)
    model.comm.all_gather_rows_into(av, cv)
    model.comm.all_gather_rows_into(ai, ci)
    out = torch.empty(B, dtype=torch.int32, device=dev)
    return ops.sample_candidates(av, ai, W, temp, topk, topp, seeds, posd, out)
