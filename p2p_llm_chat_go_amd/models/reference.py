"""Plain-PyTorch fp32 oracle for the HF Llama / Mixtral decoder (numerics tests).

Operates on an HF-named, natural-layout state dict (``nn.Linear`` [out, in]
weights), exactly what a ``safetensors`` checkpoint of Llama-3.1 / Mixtral
holds, so the same dict feeds the oracle and ``models.weights.load``.
"""
from __future__ import annotations

import torch

from .config import ModelConfig, rope_table


def random_state_dict(cfg: ModelConfig, seed: int = 0, std: float = 0.02,
                      dtype=torch.bfloat16, device="cpu", on_device: bool = False) -> dict:
    """HF-named random checkpoint.  on_device=True draws with a generator on ``device``
    (full-width models in multi-process GPU tests: every process of one device gets the
    same tensors without a multi-GiB CPU draw); False draws on the CPU (the default, so
    CPU and GPU tests see identical weights for a seed)."""
    gdev = torch.device(device) if on_device else torch.device("cpu")
    g = torch.Generator(device=gdev).manual_seed(seed)

    def rnd(*shape, s=std):
        return (torch.randn(*shape, generator=g, device=gdev) * s).to(dtype).to(device)

    def gain(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g, device=gdev)).to(dtype).to(device)

    H, D = cfg.hidden, cfg.head_dim
    sd = {"model.embed_tokens.weight": rnd(cfg.vocab, H, s=1.0), "model.norm.weight": gain(H)}
    if not cfg.tie_embeddings:
        sd["lm_head.weight"] = rnd(cfg.vocab, H)
    for i in range(cfg.n_layers):
        p = "model.layers.%d." % i
        sd[p + "input_layernorm.weight"] = gain(H)
        sd[p + "post_attention_layernorm.weight"] = gain(H)
        sd[p + "self_attn.q_proj.weight"] = rnd(cfg.n_heads * D, H)
        sd[p + "self_attn.k_proj.weight"] = rnd(cfg.n_kv_heads * D, H)
        sd[p + "self_attn.v_proj.weight"] = rnd(cfg.n_kv_heads * D, H)
        sd[p + "self_attn.o_proj.weight"] = rnd(H, cfg.n_heads * D)
        if cfg.is_moe:
            sd[p + "block_sparse_moe.gate.weight"] = rnd(cfg.n_experts, H, s=0.5)
            for e in range(cfg.n_experts):
                q = p + "block_sparse_moe.experts.%d." % e
                sd[q + "w1.weight"] = rnd(cfg.ffn, H)
                sd[q + "w3.weight"] = rnd(cfg.ffn, H)
                sd[q + "w2.weight"] = rnd(H, cfg.ffn)
        else:
            sd[p + "mlp.gate_proj.weight"] = rnd(cfg.ffn, H)
            sd[p + "mlp.up_proj.weight"] = rnd(cfg.ffn, H)
            sd[p + "mlp.down_proj.weight"] = rnd(H, cfg.ffn)
    return sd


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _rope(x, cos, sin):
    D = x.shape[-1]
    x1, x2 = x[..., :D // 2], x[..., D // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def moe_ref(x, sd, p, cfg):
    """Mixtral sparse MoE: softmax router, top-k, renormalised weights."""
    logits = x @ sd[p + "block_sparse_moe.gate.weight"].float().t()
    probs = torch.softmax(logits, dim=-1)
    w, idx = probs.topk(cfg.top_k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    out = torch.zeros_like(x)
    for e in range(cfg.n_experts):
        q = p + "block_sparse_moe.experts.%d." % e
        sel = (idx == e)
        rows = sel.any(-1).nonzero()[:, 0]
        if rows.numel() == 0:
            continue
        we = (w * sel).sum(-1)[rows]
        xe = x[rows]
        h = torch.nn.functional.silu(xe @ sd[q + "w1.weight"].float().t()) * (
            xe @ sd[q + "w3.weight"].float().t())
        out[rows] += we[:, None] * (h @ sd[q + "w2.weight"].float().t())
    return out


@torch.no_grad()
def reference_forward(sd: dict, cfg: ModelConfig, tokens: torch.Tensor) -> torch.Tensor:
    """Full causal forward of ONE sequence: tokens [T] -> fp32 logits [T, V]."""
    T = tokens.shape[0]
    H, D, nh, nkv = cfg.hidden, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
    G = nh // nkv
    dev = sd["model.embed_tokens.weight"].device  # runs where the checkpoint lives
    tokens = tokens.to(dev)
    cs = rope_table(cfg, max_pos=T, device=dev)
    cos, sin = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    x = sd["model.embed_tokens.weight"].float()[tokens.long()]
    mask = torch.full((T, T), float("-inf"), device=dev).triu(1)
    for i in range(cfg.n_layers):
        p = "model.layers.%d." % i
        h = _rms(x, sd[p + "input_layernorm.weight"], cfg.eps)
        q = (h @ sd[p + "self_attn.q_proj.weight"].float().t()).view(T, nh, D)
        k = (h @ sd[p + "self_attn.k_proj.weight"].float().t()).view(T, nkv, D)
        v = (h @ sd[p + "self_attn.v_proj.weight"].float().t()).view(T, nkv, D)
        q, k = _rope(q, cos, sin), _rope(k, cos, sin)
        k = k.repeat_interleave(G, dim=1)
        v = v.repeat_interleave(G, dim=1)
        s = torch.einsum("thd,shd->hts", q, k) / (D ** 0.5) + mask
        a = torch.einsum("hts,shd->thd", torch.softmax(s, -1), v).reshape(T, nh * D)
        x = x + a @ sd[p + "self_attn.o_proj.weight"].float().t()
        h = _rms(x, sd[p + "post_attention_layernorm.weight"], cfg.eps)
        if cfg.is_moe:
            x = x + moe_ref(h, sd, p, cfg)
        else:
            g = h @ sd[p + "mlp.gate_proj.weight"].float().t()
            u = h @ sd[p + "mlp.up_proj.weight"].float().t()
            x = x + (torch.nn.functional.silu(g) * u) @ sd[p + "mlp.down_proj.weight"].float().t()
    x = _rms(x, sd["model.norm.weight"], cfg.eps)
    head = sd["model.embed_tokens.weight"] if cfg.tie_embeddings else sd["lm_head.weight"]
    return x @ head.float().t()


@torch.no_grad()
def reference_greedy(sd, cfg, prompt: list, n_new: int) -> list:
    toks = list(prompt)
    for _ in range(n_new):
        logits = reference_forward(sd, cfg, torch.tensor(toks))
        toks.append(int(logits[-1].argmax()))
    return toks[len(prompt):]
