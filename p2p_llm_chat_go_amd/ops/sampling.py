"""Stochastic token sampling (temperature -> top-k -> top-p -> draw) on the GPU.

``sample`` runs ``sampling.hip`` (one workgroup per row, radix-select top-k,
graph-capturable: every per-row parameter is a device tensor and the random
stream is a counter-based hash of (seed, position, token id)).  CPU tensors run
``sample_ref``, the same algorithm in PyTorch with the same hash, which is the
numerics oracle of the kernel test.
"""
from __future__ import annotations

import torch

from . import _lib

KMAX = 128
_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def uniform01(seed: int, pos: int, tok: int) -> float:
    """The kernel's uniform in (0, 1) for a draw at (seed, pos, token)."""
    h = _mix64((seed & _M64) ^ _mix64(((pos & 0xFFFFFFFF) << 32) | (tok & 0xFFFFFFFF)))
    return ((h >> 40) + 0.5) / 16777216.0


def _order(x: torch.Tensor, ids: torch.Tensor | None):
    """Indices of x in (descending value, ascending id) order."""
    if ids is None:
        return torch.sort(-x, stable=True).indices  # positions are the ids
    by_id = torch.sort(ids, stable=True).indices
    return by_id[torch.sort(-x[by_id], stable=True).indices]


def keep_set(logits_row: torch.Tensor, temperature: float, top_k: int, top_p: float,
             ids: torch.Tensor | None = None):
    """(token ids, renormalised probabilities) the draw picks from, in descending order.
    ids: the token id of each entry (vocab-parallel candidates); None = the position."""
    V = logits_row.shape[0]
    k = top_k if 0 < top_k <= KMAX else KMAX
    k = min(k, V)
    x = logits_row.float()
    sel = _order(x, ids)[:k]
    vals = x[sel]
    ids = sel if ids is None else ids[sel].long()
    p = torch.softmax(vals / temperature, -1)
    cum = p.cumsum(-1)
    keep = (cum - p) <= top_p
    pk = p[keep]
    return ids[keep], pk / pk.sum()


def sample_ref(logits, temp, topk, topp, seeds, pos, out, cand_ids=None):
    for r in range(logits.shape[0]):
        T = float(temp[r])
        cid = None if cand_ids is None else cand_ids[r]
        if not T > 0:
            out[r] = int(_order(logits[r].float(), cid)[0]) if cid is None else int(
                cid[_order(logits[r].float(), cid)[0]])
            continue
        ids, p = keep_set(logits[r], T, int(topk[r]), float(topp[r]), cid)
        s, ps = int(seeds[r]) & _M64, int(pos[r])
        score = [float(p[i]) / -torch.log(torch.tensor(uniform01(s, ps, int(ids[i])))).item()
                 for i in range(len(ids))]
        out[r] = int(ids[max(range(len(ids)), key=lambda i: score[i])])
    return out


def sample(logits: torch.Tensor, temp: torch.Tensor, topk: torch.Tensor, topp: torch.Tensor,
           seeds: torch.Tensor, pos: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """logits fp32 [B, V] -> int32 ids [B].  temp/topp fp32 [B], topk int32 [B],
    seeds int64 [B], pos int32 [B] (the position being decoded: a fresh draw per step)."""
    B, V = logits.shape
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    if logits.device.type != "cuda":
        return sample_ref(logits, temp, topk, topp, seeds, pos, out)
    assert logits.dtype == torch.float32 and logits.stride(1) == 1
    assert temp.dtype == torch.float32 and topp.dtype == torch.float32
    assert topk.dtype == torch.int32 and pos.dtype == torch.int32 and seeds.dtype == torch.int64
    L = _lib.lib()
    _lib.check(L.p2p_sample(logits.data_ptr(), logits.stride(0), B, V, temp.data_ptr(),
                            topk.data_ptr(), topp.data_ptr(), seeds.data_ptr(), pos.data_ptr(),
                            out.data_ptr(), _lib.stream_ptr(logits.device)), "sample")
    return out


def topk_candidates(logits: torch.Tensor, id_off: int, cand_v: torch.Tensor,
                    cand_id: torch.Tensor):
    """Vocab-parallel sampling, step 1: this shard's top-128 (value, global id) per row,
    sorted (descending value, ascending id; padded with -inf / INT32_MAX) into
    cand_v fp32 / cand_id int32 [B, 128]."""
    B, V = logits.shape
    if logits.device.type != "cuda":
        for r in range(B):
            x = logits[r].float()
            sel = _order(x, None)[:KMAX]
            n = sel.shape[0]
            cand_v[r].fill_(float("-inf"))
            cand_id[r].fill_(0x7FFFFFFF)
            cand_v[r, :n] = x[sel]
            cand_id[r, :n] = (sel + id_off).to(torch.int32)
        return cand_v, cand_id
    assert logits.dtype == torch.float32 and logits.stride(1) == 1
    L = _lib.lib()
    _lib.check(L.p2p_topk_candidates(logits.data_ptr(), logits.stride(0), B, V, int(id_off),
                                     cand_v.data_ptr(), cand_id.data_ptr(),
                                     _lib.stream_ptr(logits.device)), "topk_candidates")
    return cand_v, cand_id


def sample_candidates(cand_v: torch.Tensor, cand_id: torch.Tensor, world: int, temp, topk, topp,
                      seeds, pos, out: torch.Tensor) -> torch.Tensor:
    """Step 2: the draw over the gathered candidates ([world * B, 128], rank-major) --
    the same token as ``sample`` over the full vocabulary row."""
    B = cand_v.shape[0] // world
    if cand_v.device.type != "cuda":
        v = cand_v.view(world, B, KMAX).permute(1, 0, 2).reshape(B, world * KMAX)
        i = cand_id.view(world, B, KMAX).permute(1, 0, 2).reshape(B, world * KMAX)
        return sample_ref(v, temp, topk, topp, seeds, pos, out, cand_ids=i)
    L = _lib.lib()
    _lib.check(L.p2p_sample_candidates(cand_v.data_ptr(), cand_id.data_ptr(), world, B,
                                       temp.data_ptr(), topk.data_ptr(), topp.data_ptr(),
                                       seeds.data_ptr(), pos.data_ptr(), out.data_ptr(),
                                       _lib.stream_ptr(cand_v.device)), "sample_candidates")
    return out
