"""Row gather (embedding), greedy argmax and the graph-resident decode advance."""
from __future__ import annotations

import torch

from . import _lib
from .attention import PAGE


def gather_rows(src: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None):
    T = idx.shape[0]
    H = src.shape[1]
    if out is None:
        out = torch.empty(T, H, device=src.device, dtype=src.dtype)
    if src.device.type != "cuda":
        out.copy_(src[idx.long()])
        return out
    L = _lib.lib()
    assert src.stride(1) == 1 and src.stride(0) == H
    _lib.check(L.p2p_gather_rows(src.data_ptr(), idx.data_ptr(), T, H, src.shape[0],
                                 out.data_ptr(), out.stride(0), _lib.stream_ptr(src.device)),
               "gather_rows")
    return out


_SINKS = {}


def l3_prefetch(t: torch.Tensor, nbytes: int | None = None, grid: int = 0):
    """Pull t's bytes (its first nbytes) into the Infinity Cache with a discarded
    streaming read (l3_prefetch.hip); no effect on values.  CPU tensors: no-op."""
    if t.device.type != "cuda":
        return
    n = t.numel() * t.element_size() if nbytes is None else int(nbytes)
    sink = _SINKS.get(t.device)
    if sink is None:
        sink = _SINKS[t.device] = torch.zeros(256 * 4, dtype=torch.int32, device=t.device)
    L = _lib.experimental()
    _lib.check(L.p2p_l3_prefetch(t.data_ptr(), n, grid, sink.data_ptr(),
                                 _lib.stream_ptr(t.device)), "l3_prefetch")


def argmax(logits: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    M, V = logits.shape
    if out is None:
        out = torch.empty(M, device=logits.device, dtype=torch.int32)
    if logits.device.type != "cuda":
        out.copy_(logits.argmax(-1).to(torch.int32))
        return out
    L = _lib.lib()
    _lib.check(L.p2p_argmax(logits.data_ptr(), M, V, logits.stride(0), out.data_ptr(),
                            _lib.stream_ptr(logits.device)), "argmax")
    return out


def advance(ids, pos, ctx, slots, block_tables, hist, step, keys=None):
    """Decode-state advance (all int32, device-resident): see elementwise.hip.

    keys: optional int64 greedy keys from ops.lm_head_argmax -> converted into ids
    (and reset) before the advance.
    """
    B = ids.shape[0]
    if ids.device.type != "cuda":
        if keys is not None:
            from .gemm import reduce_keys_ref

            ids.copy_(reduce_keys_ref(keys, B))
        st = int(step[0])
        if hist is not None:
            hist[:, st] = ids
        pos += 1
        ctx.copy_(pos + 1)
        pages = block_tables.gather(1, (pos // PAGE).long()[:, None])[:, 0]
        slots.copy_(pages * PAGE + pos % PAGE)
        step += 1
        return
    L = _lib.lib()
    _lib.check(L.p2p_advance(ids.data_ptr(), _lib.ptr(keys), pos.data_ptr(), ctx.data_ptr(),
                             slots.data_ptr(),
                             block_tables.data_ptr(), block_tables.stride(0),
                             _lib.ptr(hist), 0 if hist is None else hist.stride(0),
                             step.data_ptr(), B, _lib.stream_ptr(ids.device)), "advance")
