"""Persistent decode engine: every layer of a dense TP=1 decode step (<= 4 rows, contexts
<= 256 keys) in ONE launch of one workgroup per CU (csrc/experimental/decode_engine.hip, libp2p_experimental.so).

The separate-launch decode layer (qkv+attention, o_proj, gate_up, down) pays a dependent
kernel boundary between every pair of weight streams; here the four streams are phases of
one grid with tagged-granule hand-offs between workgroups, and every wave issues the next
projection's first weight loads before it waits for that projection's input.  Replaces the
per-layer launches of ``LlamaModel.forward`` for decode batches it can run
(``P2P_DECODE_ENGINE=0`` keeps the separate launches).  The math is the skinny-kernel
path's: RMSNorm statistics of the bf16 residual, RoPE, bf16 rounding of every stored
activation and residual -- only the summation order of the split-K partials differs.
"""
from __future__ import annotations

import torch

from . import _lib

MAX_ROWS = 4
MAX_CTX = 256


class DecodeEngine:
    """Device-side state of one model's engine launches: the per-layer weight / KV cache
    pointer tables, the granule workspace and the launch epoch (zeroed once; the kernel
    keeps them consistent across launches and graph replays)."""

    def __init__(self, model):
        w, kv = model.w, model.kv
        cfg = model.cfg
        dev = model.device
        self.L = cfg.n_layers
        self.H, self.I = cfg.hidden, cfg.ffn
        self.Hq, self.Hkv = model.nq, model.nkv
        self.eps = cfg.eps
        self.scale = cfg.head_dim ** -0.5
        ptrs = []
        for lw in w.layers:
            ptrs += [lw.qkv.data_ptr(), lw.o.data_ptr(), lw.gate_up.data_ptr(), lw.down.data_ptr()]
        self.wptr = torch.tensor(ptrs, dtype=torch.int64, device=dev)
        kvp = []
        for i in range(self.L):
            kc, vc = kv.layer(i)
            kvp += [kc.data_ptr(), vc.data_ptr()]
        self.kvptr = torch.tensor(kvp, dtype=torch.int64, device=dev)
        L = _lib.experimental()
        nbytes = L.p2p_decode_engine_ws_bytes(MAX_ROWS, self.H, self.I, self.Hq, self.Hkv)
        self.ws = torch.zeros((nbytes + 7) // 8, dtype=torch.int64, device=dev)
        self.epoch = torch.zeros(2, dtype=torch.int32, device=dev)
        self._keep = (w, kv)  # the pointer tables reference these tensors

    def run(self, h, pos, slots, rope, block_tables, ctx_lens, err):
        """h [R, H] bf16: embedding rows in, final residual out (before the final norm)."""
        R = h.shape[0]
        assert R <= MAX_ROWS and h.stride(1) == 1 and h.dtype == torch.bfloat16
        L = _lib.experimental()
        _lib.check(L.p2p_decode_engine(
            self.wptr.data_ptr(), self.kvptr.data_ptr(), self.L, R, self.H, self.I, self.Hq,
            self.Hkv, float(self.eps), float(self.scale), h.data_ptr(), h.stride(0),
            pos.data_ptr(), slots.data_ptr(), rope.data_ptr(), block_tables.data_ptr(),
            block_tables.stride(0), ctx_lens.data_ptr(), self.ws.data_ptr(),
            self.epoch.data_ptr(), err.data_ptr(), _lib.stream_ptr(h.device)), "decode_engine")
        return h


def decode_engine_ok(model, R: int, max_ctx: int) -> bool:
    """Can the engine run this decode step (shape, dtype, residency of the whole grid)?"""
    cfg = model.cfg
    if (model.device.type != "cuda" or model.tp != 1 or cfg.is_moe or R < 1 or R > MAX_ROWS
            or max_ctx > MAX_CTX or cfg.head_dim != 128):
        return False
    lw = model.w.layers[0]
    if not all(isinstance(t, torch.Tensor) and t.dtype == torch.bfloat16
               for t in (lw.qkv, lw.o, lw.gate_up, lw.down)):
        return False  # weight-only fp8 keeps the separate launches
    L = _lib.experimental()
    return bool(L.p2p_decode_engine_ok(R, cfg.hidden, cfg.ffn, model.nq, model.nkv, max_ctx))
