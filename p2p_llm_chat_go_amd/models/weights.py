"""Engine weight store: HF checkpoint / random init -> folded, sharded, MFMA-tiled.

Load-time transforms (all one-off, none on the hot path):
  * RMSNorm gains are folded into the projection that consumes the normed
    activations (input_layernorm -> qkv, post_attention_layernorm -> gate_up /
    router / experts, model.norm -> lm_head); the kernels then only apply
    rstd (``ops.gemm``).
  * q|k|v rows are concatenated into one qkv projection; gate|up into one
    gate_up projection (SwiGLU epilogue pairs row g with row g + F).
  * Tensor-parallel sharding (Megatron): qkv / gate_up / lm_head split by
    output rows (heads, ffn columns, vocab), o_proj / down split by input
    columns; the row-parallel outputs are summed by ``parallel.comm``.
  * qkv rows are permuted per head (``ops.rope_row_perm``) so RoPE and the KV
    cache write run in the projection's epilogue.
  * Every projection is re-laid out fragment-major (``ops.tile_weight``).

Random init (BASELINE: no checkpoints on the box) draws N(0, std) directly in
the tiled layout -- statistically identical to tiling a random natural
matrix, without the transient copy (a 70B model is ~140 GB).
"""
from __future__ import annotations

import dataclasses
import glob
import json
import os

import torch

from .. import ops
from .config import ModelConfig


@dataclasses.dataclass
class LayerWeights:
    qkv: torch.Tensor          # tiled [(nq+2nkv)/tp * D, H]
    o: torch.Tensor            # tiled [H, nq/tp * D]
    gate_up: torch.Tensor | None = None   # tiled [2F/tp, H]
    down: torch.Tensor | None = None      # tiled [H, F/tp]
    # MoE
    router: torch.Tensor | None = None    # natural [E, H] bf16 (norm folded), replicated
    w13: torch.Tensor | None = None       # tiled per local expert [E_local, 2F/16, H/32, 64, 8]
    w2: torch.Tensor | None = None        # tiled per local expert [E_local, H/16, F/32, 64, 8]


@dataclasses.dataclass
class EngineWeights:
    cfg: ModelConfig
    embed: torch.Tensor        # [V, H] bf16 (full table, replicated)
    lm_head: torch.Tensor      # tiled [V/tp, H] (final norm folded)
    layers: list
    tp_rank: int = 0
    tp_size: int = 1
    ep_rank: int = 0
    ep_size: int = 1

    @property
    def device(self):
        return self.embed.device

    def nbytes(self) -> int:
        def nb(t):
            if isinstance(t, ops.Fp8Weight):
                return t.data.numel() + 4 * t.scale.numel()
            return t.numel() * t.element_size()

        n = nb(self.embed) + nb(self.lm_head)
        for lw in self.layers:
            for f in dataclasses.fields(lw):
                t = getattr(lw, f.name)
                if t is not None:
                    n += nb(t)
        return n

    def shallow_copy(self) -> "EngineWeights":
        """New weight store sharing every tensor, with its own layer objects (so swapping a
        projection -- e.g. quantize_fp8 -- does not touch the caller's store)."""
        return dataclasses.replace(self, layers=[dataclasses.replace(lw) for lw in self.layers])

    def quantize_fp8(self, names=("qkv", "o", "gate_up", "down"), lm_head=True) -> "EngineWeights":
        """Weight-only FP8 (e4m3, per-output-channel scale) for the dense projections and
        the LM head, in place: the decode weight stream -- the roofline of batch-1 decode --
        halves (the 8B LM head alone is 1 GiB of bf16 per token).  The embedding, router
        and MoE experts stay bf16.  Opt-in (ENGINE_WEIGHTS=fp8 / bench.py --weights fp8);
        the headline numbers are bf16."""
        for lw in self.layers:
            for name in names:
                t = getattr(lw, name)
                if isinstance(t, torch.Tensor):
                    setattr(lw, name, ops.quantize_fp8(t))
        if lm_head and isinstance(self.lm_head, torch.Tensor) and \
                ops.tiled_shape(self.lm_head)[1] % 64 == 0:
            self.lm_head = ops.quantize_fp8(self.lm_head)
        return self

    # ------------------------------------------------------------------ build
    @classmethod
    def from_state_dict(cls, sd: dict, cfg: ModelConfig, device="cpu", tp_rank=0, tp_size=1,
                        ep_rank=0, ep_size=1) -> "EngineWeights":
        D, nh, nkv, F = cfg.head_dim, cfg.n_heads, cfg.n_kv_heads, cfg.ffn
        assert nh % tp_size == 0 and nkv % tp_size == 0, "heads must divide tp"
        qs, ks = nh // tp_size * D, nkv // tp_size * D
        dev = torch.device(device)

        sliced = hasattr(sd, "get_rows_cols")

        def get(name, rows=None, cols=None):
            """The [rows, cols] slice of a tensor on the target device.  A LazySafetensors
            store reads only that slice from disk (safetensors get_slice), so a TP rank
            moves only its own shard of each sharded tensor."""
            if sliced:
                return sd.get_rows_cols(name, rows, cols).to(dev)
            t = sd[name]
            if rows is not None:
                t = t[rows[0]:rows[1]]
            if cols is not None:
                t = t[:, cols[0]:cols[1]]
            return t.to(dev)

        def tile(w):
            return ops.tile_weight(w.to(torch.bfloat16).contiguous())

        layers = []
        for i in range(cfg.n_layers):
            p = "model.layers.%d." % i
            g_in = get(p + "input_layernorm.weight")
            g_post = get(p + "post_attention_layernorm.weight")
            q = get(p + "self_attn.q_proj.weight", rows=(tp_rank * qs, (tp_rank + 1) * qs))
            k = get(p + "self_attn.k_proj.weight", rows=(tp_rank * ks, (tp_rank + 1) * ks))
            v = get(p + "self_attn.v_proj.weight", rows=(tp_rank * ks, (tp_rank + 1) * ks))
            qkv = ops.fold_norm(torch.cat([q, k, v], 0), g_in)
            # fused qkv+RoPE epilogue row order (ops.rope_row_perm)
            qkv = qkv[ops.rope_row_perm(qkv.shape[0] // D, D).to(qkv.device)]
            o = get(p + "self_attn.o_proj.weight", cols=(tp_rank * qs, (tp_rank + 1) * qs))
            lw = LayerWeights(qkv=tile(qkv), o=tile(o))
            if cfg.is_moe:
                E = cfg.n_experts
                assert E % ep_size == 0
                el = E // ep_size
                lw.router = ops.fold_norm(get(p + "block_sparse_moe.gate.weight"), g_post).to(
                    torch.bfloat16).contiguous()
                w13, w2 = [], []
                Fs = F // tp_size
                for e in range(ep_rank * el, (ep_rank + 1) * el):
                    q_ = p + "block_sparse_moe.experts.%d." % e
                    w1 = get(q_ + "w1.weight", rows=(tp_rank * Fs, (tp_rank + 1) * Fs))
                    w3 = get(q_ + "w3.weight", rows=(tp_rank * Fs, (tp_rank + 1) * Fs))
                    w13.append(tile(ops.fold_norm(torch.cat([w1, w3], 0), g_post)))
                    w2.append(tile(get(q_ + "w2.weight", cols=(tp_rank * Fs, (tp_rank + 1) * Fs))))
                lw.w13 = torch.stack(w13).contiguous()
                lw.w2 = torch.stack(w2).contiguous()
            else:
                Fs = F // tp_size
                gate = get(p + "mlp.gate_proj.weight", rows=(tp_rank * Fs, (tp_rank + 1) * Fs))
                up = get(p + "mlp.up_proj.weight", rows=(tp_rank * Fs, (tp_rank + 1) * Fs))
                lw.gate_up = tile(ops.fold_norm(torch.cat([gate, up], 0), g_post))
                lw.down = tile(get(p + "mlp.down_proj.weight", cols=(tp_rank * Fs, (tp_rank + 1) * Fs)))
            layers.append(lw)
        embed = get("model.embed_tokens.weight").to(torch.bfloat16).contiguous()
        Vs = cfg.vocab // tp_size
        vrows = (tp_rank * Vs, (tp_rank + 1) * Vs)
        head = embed[vrows[0]:vrows[1]] if cfg.tie_embeddings else get("lm_head.weight", rows=vrows)
        head = ops.fold_norm(head, get("model.norm.weight"))
        return cls(cfg, embed, tile(head), layers, tp_rank, tp_size, ep_rank, ep_size)

    @classmethod
    def random(cls, cfg: ModelConfig, device="cuda", seed=0, std=0.02, tp_rank=0, tp_size=1,
               ep_rank=0, ep_size=1) -> "EngineWeights":
        """Random-init weights generated directly in the tiled layout (see module doc)."""
        dev = torch.device(device)
        # shared (replicated) weights depend on the TP shard only, so every EP rank
        # holds the same attention / router / embeddings; experts use their own stream
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed * 1000003 + tp_rank * 7919)
        egen = torch.Generator(device=dev)
        egen.manual_seed(seed * 1000003 + tp_rank * 7919 + (ep_rank + 1) * 104729)
        H, D, F = cfg.hidden, cfg.head_dim, cfg.ffn

        def rnd_tiled(n, k, s=std, lead=(), g=gen):
            t = torch.empty(*lead, n // 16, k // 32, 64, 8, device=dev, dtype=torch.bfloat16)
            t.normal_(0.0, s, generator=g)
            return t

        qkv_rows = (cfg.n_heads + 2 * cfg.n_kv_heads) // tp_size * D
        q_cols = cfg.n_heads // tp_size * D
        Fs = F // tp_size
        layers = []
        for _ in range(cfg.n_layers):
            lw = LayerWeights(qkv=rnd_tiled(qkv_rows, H), o=rnd_tiled(H, q_cols))
            if cfg.is_moe:
                el = cfg.n_experts // ep_size
                lw.router = torch.empty(cfg.n_experts, H, device=dev, dtype=torch.bfloat16).normal_(
                    0.0, 0.5, generator=gen)
                lw.w13 = rnd_tiled(2 * Fs, H, lead=(el,), g=egen)
                lw.w2 = rnd_tiled(H, Fs, lead=(el,), g=egen)
            else:
                lw.gate_up = rnd_tiled(2 * Fs, H)
                lw.down = rnd_tiled(H, Fs)
            layers.append(lw)
        embed = torch.empty(cfg.vocab, H, device=dev, dtype=torch.bfloat16).normal_(0.0, 1.0,
                                                                                    generator=gen)
        head = rnd_tiled(cfg.vocab // tp_size, H)
        return cls(cfg, embed, head, layers, tp_rank, tp_size, ep_rank, ep_size)


class LazySafetensors:
    """Read-on-access view of an HF checkpoint directory's ``*.safetensors`` shards (no
    pickle).  ``EngineWeights.from_state_dict`` asks for one tensor slice at a time
    (``get_rows_cols``), and only that slice is read from disk (safetensors ``get_slice``):
    a TP rank reads and holds only its own shard of every sharded tensor (a 70B checkpoint
    is ~140 GB; eight ranks each reading it whole would be ~1.1 TB of I/O).  Replicated
    tensors (norm gains, the embedding table, the MoE router) are read whole."""

    def __init__(self, path: str):
        from safetensors import safe_open

        self.path = path
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            raise FileNotFoundError("no .safetensors files under %s" % path)
        self._where = {}
        self._handles = {}
        for f in files:
            h = safe_open(f, framework="pt", device="cpu")
            self._handles[f] = h
            for k in h.keys():
                self._where[k] = f

    def __contains__(self, name):
        return name in self._where

    def keys(self):
        return self._where.keys()

    def __getitem__(self, name):
        return self._handles[self._where[name]].get_tensor(name)

    def get_rows_cols(self, name, rows=None, cols=None):
        """tensor[rows[0]:rows[1], cols[0]:cols[1]] read from disk as that slice only."""
        if rows is None and cols is None:
            return self[name]
        sl = self._handles[self._where[name]].get_slice(name)
        r = slice(*rows) if rows is not None else slice(None)
        c = slice(*cols) if cols is not None else slice(None)
        return sl[r, c] if len(sl.get_shape()) > 1 else sl[r]


def load_safetensors_dir(path: str, device="cpu") -> dict:
    """Read every ``*.safetensors`` shard of an HF checkpoint directory (no pickle)."""
    from safetensors.torch import load_file

    sd = {}
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError("no .safetensors files under %s" % path)
    for f in files:
        sd.update(load_file(f, device=str(device)))
    return sd


def config_from_hf(path: str, base: ModelConfig | None = None) -> ModelConfig:
    """Build a ModelConfig from an HF ``config.json`` (Llama / Mixtral)."""
    with open(os.path.join(path, "config.json")) as f:
        c = json.load(f)
    # transformers < 5: rope_theta + rope_scaling; >= 5: rope_parameters (theta inside)
    rs = c.get("rope_scaling") or c.get("rope_parameters") or None
    theta = c.get("rope_theta", (rs or {}).get("rope_theta", 10000.0))
    llama3 = None
    if rs and rs.get("rope_type", rs.get("type")) == "llama3":
        llama3 = (float(rs["factor"]), float(rs["low_freq_factor"]), float(rs["high_freq_factor"]),
                  int(rs["original_max_position_embeddings"]))
    eos = c.get("eos_token_id", 2)
    eos = tuple(eos) if isinstance(eos, list) else (eos,)
    return ModelConfig(
        name=c.get("_name_or_path", os.path.basename(path.rstrip("/"))) or "hf",
        hidden=c["hidden_size"], n_layers=c["num_hidden_layers"],
        n_heads=c["num_attention_heads"], n_kv_heads=c.get("num_key_value_heads",
                                                           c["num_attention_heads"]),
        ffn=c["intermediate_size"], vocab=c["vocab_size"],
        head_dim=c.get("head_dim", c["hidden_size"] // c["num_attention_heads"]),
        rope_theta=float(theta), rope_llama3=llama3,
        eps=float(c.get("rms_norm_eps", 1e-5)), max_pos=int(c.get("max_position_embeddings", 8192)),
        n_experts=int(c.get("num_local_experts", 0)), top_k=int(c.get("num_experts_per_tok", 0)),
        tie_embeddings=bool(c.get("tie_word_embeddings", False)),
        bos_id=int(c.get("bos_token_id", 1)), eos_ids=eos)
