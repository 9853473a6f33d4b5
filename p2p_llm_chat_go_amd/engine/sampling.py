"""Token sampling: greedy (fused into the LM head kernel, see ops.lm_head_argmax)
and Ollama-style temperature / top-k / top-p sampling for requests that ask for
it (``options`` of ``/api/generate``; Ollama's defaults are temperature 0.8,
top_k 40, top_p 0.9).

The stochastic path runs on the logits of a graph-captured forward: top-k is
taken first (k <= 128, so the full-vocab softmax is never materialised), then
top-p over the k survivors, then an exponential-race draw (argmax of
p / Exp(1)), which is equivalent to multinomial sampling and needs one random
tensor per step.  Rows with temperature <= 0 are greedy.
"""
from __future__ import annotations

import dataclasses

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

    @classmethod
    def from_ollama(cls, options: dict | None, default_max: int = 128) -> "SamplingParams":
        o = options or {}
        n = int(o.get("num_predict", default_max))
        if n < 0:
            n = default_max
        return cls(temperature=float(o.get("temperature", 0.0)), top_k=int(o.get("top_k", 40)),
                   top_p=float(o.get("top_p", 0.9)), seed=o.get("seed"), max_tokens=max(1, n))


def sample(logits: torch.Tensor, params: list, generator: torch.Generator | None = None):
    """logits [B, V] fp32 -> int32 token ids [B] (one SamplingParams per row)."""
    B = logits.shape[0]
    out = logits.argmax(-1).to(torch.int32)
    rows = [i for i, p in enumerate(params[:B]) if not p.greedy]
    if not rows:
        return out
    idx = torch.tensor(rows, device=logits.device)
    lg = logits.index_select(0, idx)
    temps = torch.tensor([params[i].temperature for i in rows], device=logits.device)
    ks = [max(1, min(int(params[i].top_k) if params[i].top_k > 0 else 128, 128)) for i in rows]
    kmax = max(ks)
    vals, ids = lg.topk(kmax, dim=-1)
    kmask = torch.arange(kmax, device=logits.device)[None, :] >= torch.tensor(
        ks, device=logits.device)[:, None]
    vals = vals / temps[:, None]
    vals = vals.masked_fill(kmask, float("-inf"))
    probs = torch.softmax(vals, dim=-1)
    tps = torch.tensor([params[i].top_p for i in rows], device=logits.device)
    cum = probs.cumsum(-1)
    drop = (cum - probs) > tps[:, None]  # keep the smallest prefix with mass >= top_p
    probs = probs.masked_fill(drop, 0.0)
    probs = probs / probs.sum(-1, keepdim=True)
    e = torch.empty_like(probs).exponential_(1.0, generator=generator)
    choice = (probs / e).argmax(-1)
    out[idx] = ids.gather(1, choice[:, None])[:, 0].to(torch.int32)
    return out
