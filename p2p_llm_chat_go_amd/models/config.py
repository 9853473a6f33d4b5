"""Model configurations (public Llama-3.1 / Mixtral shapes) and the RoPE table.

The reference never names a model beyond Ollama's ``llama3.1`` tag
(`web/streamlit_app.py:28`); BASELINE.json names the configs this engine must
serve: llama3.1-8B, llama3.1-70B and Mixtral-8x7B, plus a tiny-llama for the
CPU plumbing config.  Shapes are the published HF configs.
"""
from __future__ import annotations

import dataclasses
import math

import torch


@dataclasses.dataclass(frozen=True)
class ModelConfig:
    name: str
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn: int
    vocab: int
    head_dim: int = 128
    rope_theta: float = 500000.0
    # llama3 rope scaling (factor, low_freq_factor, high_freq_factor, original_max_pos); None = plain
    rope_llama3: tuple | None = (8.0, 1.0, 4.0, 8192)
    eps: float = 1e-5
    max_pos: int = 131072
    n_experts: int = 0  # >0: Mixtral-style sparse MoE FFN
    top_k: int = 0
    tie_embeddings: bool = False
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128008, 128009)

    @property
    def is_moe(self) -> bool:
        return self.n_experts > 0

    @property
    def qkv_dim(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    def n_params(self) -> int:
        H, F, L, V = self.hidden, self.ffn, self.n_layers, self.vocab
        attn = H * self.qkv_dim + self.q_dim * H
        mlp = 3 * H * F * (self.n_experts if self.is_moe else 1) + (H * self.n_experts)
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    def weight_bytes(self) -> int:
        return 2 * self.n_params()

    def kv_bytes_per_token(self) -> int:
        return 2 * self.n_layers * self.n_kv_heads * self.head_dim * 2

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


LLAMA31_8B = ModelConfig("llama3.1-8b", hidden=4096, n_layers=32, n_heads=32, n_kv_heads=8,
                         ffn=14336, vocab=128256)
LLAMA31_70B = ModelConfig("llama3.1-70b", hidden=8192, n_layers=80, n_heads=64, n_kv_heads=8,
                          ffn=28672, vocab=128256)
MIXTRAL_8X7B = ModelConfig("mixtral-8x7b", hidden=4096, n_layers=32, n_heads=32, n_kv_heads=8,
                           ffn=14336, vocab=32000, rope_theta=1e6, rope_llama3=None,
                           max_pos=32768, n_experts=8, top_k=2, bos_id=1, eos_ids=(2,))
# CPU plumbing config (BASELINE.json config 1).  head_dim stays 128 (the kernels'
# tile), everything else is shrunk.
TINY_LLAMA = ModelConfig("tiny-llama", hidden=256, n_layers=2, n_heads=2, n_kv_heads=1, ffn=512,
                         vocab=512, max_pos=4096, rope_theta=10000.0, rope_llama3=None,
                         bos_id=1, eos_ids=(2,))
TINY_MIXTRAL = ModelConfig("tiny-mixtral", hidden=256, n_layers=2, n_heads=2, n_kv_heads=1,
                           ffn=256, vocab=512, max_pos=4096, rope_theta=1e6, rope_llama3=None,
                           n_experts=4, top_k=2, bos_id=1, eos_ids=(2,))

# CPU config with the 8B/70B head structure at 8 ranks (8 kv heads -> one per TP rank,
# 4 query heads per kv head) and 8 experts (Mixtral EP=8: one expert per rank).
TINY_LLAMA_GQA = ModelConfig("tiny-llama-gqa", hidden=256, n_layers=2, n_heads=32, n_kv_heads=8,
                             ffn=1024, vocab=1024, max_pos=4096, rope_theta=10000.0,
                             rope_llama3=None, bos_id=1, eos_ids=(2,))
TINY_MIXTRAL_8E = ModelConfig("tiny-mixtral-8e", hidden=256, n_layers=2, n_heads=8, n_kv_heads=8,
                              ffn=256, vocab=512, max_pos=4096, rope_theta=1e6, rope_llama3=None,
                              n_experts=8, top_k=2, bos_id=1, eos_ids=(2,))

PRESETS = {c.name: c for c in (LLAMA31_8B, LLAMA31_70B, MIXTRAL_8X7B, TINY_LLAMA, TINY_MIXTRAL,
                               TINY_LLAMA_GQA, TINY_MIXTRAL_8E)}
ALIASES = {"llama3.1": "llama3.1-8b", "llama3.1:8b": "llama3.1-8b", "llama3.1:70b": "llama3.1-70b",
           "mixtral": "mixtral-8x7b", "mixtral:8x7b": "mixtral-8x7b", "tiny": "tiny-llama"}


def get_config(name: str) -> ModelConfig:
    key = ALIASES.get(name, name)
    if key not in PRESETS:
        raise KeyError("unknown model %r (known: %s)" % (name, ", ".join(sorted(PRESETS))))
    return PRESETS[key]


def rope_inv_freq(cfg: ModelConfig) -> torch.Tensor:
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    if cfg.rope_llama3 is None:
        return inv
    factor, low, high, old_ctx = cfg.rope_llama3
    low_wl = old_ctx / low
    high_wl = old_ctx / high
    wl = 2 * math.pi / inv
    inv_l = torch.where(wl > low_wl, inv / factor, inv)
    smooth = (old_ctx / wl - low) / (high - low)
    smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
    medium = (wl >= high_wl) & (wl <= low_wl)
    return torch.where(medium, smoothed, inv_l)


def rope_table(cfg: ModelConfig, max_pos: int | None = None, device="cpu") -> torch.Tensor:
    """float32 [max_pos, head_dim/2, 2] = (cos, sin) of pos * inv_freq."""
    n = max_pos or cfg.max_pos
    inv = rope_inv_freq(cfg)
    ang = torch.arange(n, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float().to(device).contiguous()
