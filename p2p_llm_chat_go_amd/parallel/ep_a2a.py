"""Expert-parallel all-to-all on IPC one-shot kernels (``csrc/kernels/ep_a2a.hip``).

The DP-attention + EP MoE layer (``models.moe.moe_forward_a2a``) exchanges tokens twice
per layer: dispatch (each routed (token, expert) row to the expert's owner) and combine
(the weighted expert outputs back).  At decode sizes both are latency-bound, and RCCL's
static-capacity ``all_to_all_single`` pads every (source, destination) pair to R·K rows
(8x padding on the wire at EP = 8) and is a host-driven collective that the decode graph
never captured.  Here each exchange is a pair of kernels on the compute stream, so the
whole MoE layer -- routing, dispatch, expert GEMMs, return, combine -- is captured in the
decode hipGraph:

    dispatch : this rank's routed rows -> owners' receive regions (xGMI stores), one
               {seq, count} flag per (source, block); only routed rows travel
    recv     : wait for every source's flags, copy its rows into a local [W, C, H] buffer
               (unused capacity marked padding), per-row expert id and routing weight
    return   : expert outputs -> each source's return region, one flag per block
    combine  : wait for the owners of this row's K slots, h += the K rows (k order)

Buffers come from the group's ``CustomAllReduce`` IPC machinery (uncached, hipIpc
exported, peers mapped); a timeout sets the same error word ``comm.check()`` raises on.
``cmax`` bounds the slots (R·K) of one call; larger calls (prefill chunks) keep the
RCCL exact-count path.
"""
from __future__ import annotations

import os

import torch

from ..ops import _lib


class IpcAllToAll:
    def __init__(self, car, cmax: int, hidden: int):
        self.car = car
        self.rank, self.world = car.rank, car.world
        self.cmax, self.H = int(cmax), int(hidden)
        self.L = car.L
        nbytes = self.L.p2p_ep_buffer_bytes(self.cmax, self.H)
        with torch.cuda.device(car.device):
            self._bases = car._map(nbytes)  # collective over the group (handle exchange)
            self.state = torch.zeros(2, dtype=torch.int32, device=car.device)
        tmo = int(os.environ.get("P2P_CAR_TIMEOUT_MS", "0"))
        if tmo > 0:
            _lib.check(self.L.p2p_ep_set_timeout_ms(tmo), "ep_set_timeout_ms")

    @staticmethod
    def blocks_per_pair(n_slots: int, world: int) -> int:
        per = n_slots / max(1, world)  # rows one (source, destination) pair carries on average
        return 1 if per <= 8 else (2 if per <= 32 else 4)

    def fits(self, n_slots: int) -> bool:
        return 0 < n_slots <= self.cmax

    def dispatch(self, h, topk_ids, topk_w, K: int, El: int, send_map, R: int, nb: int):
        _lib.check(self.L.p2p_ep_dispatch(
            self._bases, self.rank, self.world, self.cmax, self.H, h.data_ptr(), h.stride(0), R,
            K, El, topk_ids.data_ptr(), topk_w.data_ptr(), send_map.data_ptr(),
            self.state.data_ptr(), nb, _lib.stream_ptr(h.device)), "ep_dispatch")

    def recv(self, C: int, recv_x, recv_meta, recv_w, recv_cnt, nb: int):
        _lib.check(self.L.p2p_ep_recv(
            self._bases, self.rank, self.world, self.cmax, self.H, C, recv_x.data_ptr(),
            recv_meta.data_ptr(), recv_w.data_ptr(), recv_cnt.data_ptr(), self.state.data_ptr(),
            self.car.err.data_ptr(), nb, _lib.stream_ptr(recv_x.device)), "ep_recv")

    def give_back(self, C: int, o, recv_cnt, nb: int):
        _lib.check(self.L.p2p_ep_return(
            self._bases, self.rank, self.world, self.cmax, self.H, C, o.data_ptr(),
            recv_cnt.data_ptr(), self.state.data_ptr(), nb, _lib.stream_ptr(o.device)),
            "ep_return")

    def combine(self, send_map, R: int, K: int, h, nb: int):
        _lib.check(self.L.p2p_ep_combine(
            self._bases, self.rank, self.world, self.cmax, self.H, R, K, send_map.data_ptr(),
            h.data_ptr(), h.stride(0), self.state.data_ptr(), self.car.err.data_ptr(), nb,
            _lib.stream_ptr(h.device)), "ep_combine")
