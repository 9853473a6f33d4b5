"""Paged KV cache sized from free HBM.

Layout (one tensor for K, one for V, all layers):
    [n_layers, num_pages, n_kv_heads_local, PAGE=64, head_dim=128] bf16
One page of one kv head is a contiguous 16 KiB tile (what a decode-attention
wave streams).  Page 0 is reserved as the *null page*: padding rows of a
graph batch bucket write and read there, so bucketed graphs never touch a
live sequence.

On a 288 GB MI355X, llama3.1-8B leaves ~270 GB for KV = ~2.1 M tokens at
128 KiB/token; the default fraction below keeps headroom for workspaces.
"""
from __future__ import annotations

import torch

from ..models.config import ModelConfig
from ..ops import HEAD_DIM, PAGE


class PageAllocator:
    """Free-list page allocator (page 0 reserved).  The C++ runtime has the same
    allocator for the scheduler (``_native.BlockAllocator``); this Python one is
    used when the native module is not built (CPU tests)."""

    def __init__(self, num_pages: int):
        if num_pages < 2:
            raise ValueError("need at least 2 pages (page 0 is the null page)")
        self.num_pages = num_pages
        self._free = list(range(num_pages - 1, 0, -1))

    @property
    def free_pages(self) -> int:
        return len(self._free)

    def alloc(self, n: int) -> list:
        if n > len(self._free):
            raise MemoryError("KV cache exhausted: want %d pages, %d free" % (n, len(self._free)))
        out = [self._free.pop() for _ in range(n)]
        return out

    def free(self, pages):
        for p in pages:
            if p <= 0 or p >= self.num_pages:
                raise ValueError("bad page %d" % p)
        self._free.extend(pages)


def pages_for(tokens: int) -> int:
    return (tokens + PAGE - 1) // PAGE


class KVCache:
    def __init__(self, cfg: ModelConfig, num_pages: int, device, tp_size: int = 1,
                 dtype=torch.bfloat16):
        assert cfg.head_dim == HEAD_DIM
        self.cfg = cfg
        self.num_pages = num_pages
        self.n_kv_local = cfg.n_kv_heads // tp_size
        shape = (cfg.n_layers, num_pages, self.n_kv_local, PAGE, HEAD_DIM)
        self.k = torch.zeros(shape, device=device, dtype=dtype)
        self.v = torch.zeros(shape, device=device, dtype=dtype)
        self.allocator = PageAllocator(num_pages)

    @staticmethod
    def bytes_per_page(cfg: ModelConfig, tp_size: int = 1) -> int:
        return 2 * cfg.n_layers * (cfg.n_kv_heads // tp_size) * PAGE * HEAD_DIM * 2

    @classmethod
    def from_free_memory(cls, cfg: ModelConfig, device, fraction: float = 0.85, tp_size: int = 1,
                         max_pages: int | None = None, reserve_bytes: int = 4 << 30):
        dev = torch.device(device)
        if dev.type == "cuda":
            free, _total = torch.cuda.mem_get_info(dev)
            budget = max(0, int((free - reserve_bytes) * fraction))
        else:
            budget = 256 << 20
        n = max(2, budget // cls.bytes_per_page(cfg, tp_size))
        if max_pages:
            n = min(n, max_pages)
        return cls(cfg, int(n), dev, tp_size)

    def layer(self, i: int):
        return self.k[i], self.v[i]
