"""One-shot all-reduce over IPC-mapped peer buffers (kernel K12, xGMI).

Decode-size tensor-parallel messages (B x hidden bf16: 16 KiB for 70B at
batch 1, 160 of them per token) are latency-bound.  RCCL's ring needs 2(W-1)
dependent hops; here every rank pushes its partial into every peer's buffer
at once (all 7 xGMI links of a rank in parallel), posts a flag, waits for the
peers' flags on its own memory and sums locally -- one hop.  The kernel is an
ordinary launch on the current stream, so it is captured in the decode
hipGraph with the GEMMs around it.  See ``csrc/kernels/custom_allreduce.hip``.

The same buffers carry the two small per-step exchanges of vocab-parallel
sampling: a MAX all-reduce of the greedy argmax keys (u64) and an all-gather
of per-shard top-k candidates.  With those, a TP decode graph holds no RCCL
call at all (one-shot kernels only).

Mid-size sums (prefill chunks below the overlapped-RCCL row threshold, batched decode)
take the two-shot form of the same kernel (``allreduce_add_`` picks it from
``two_shot_min`` bytes at 4+ ranks): reduce-scatter to shard owners, then all-gather of
the reduced shards -- 2(W-1)/W of the message per rank over xGMI instead of W-1, in two
hops instead of one, with a bit-identical result.

Handles are exchanged with ``dist.all_gather_object`` over the TP group (any
backend).  Messages above ``max_bytes`` fall back to the caller's RCCL path.
Timeouts are loud: ``check()`` raises once a peer failed to arrive within the
spin bound (``LlamaModel.check_faults`` calls it wherever the host syncs).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from ..ops import _lib


class CollectiveTimeout(RuntimeError):
    """A one-shot collective gave up waiting for a peer rank (dead or hung)."""


class PeerAccessError(RuntimeError):
    """Two ranks of a TP / EP group cannot map each other's memory (no xGMI / PCIe peer
    path, or ranks on different hosts): the IPC kernels cannot run in this group."""


_HINT = ("set P2P_CUSTOM_AR=0 to run every collective on RCCL, or P2P_CUSTOM_AR=auto to "
         "fall back to RCCL automatically when the peer check fails")


def peer_access_failures(group=None, device=None, can_access=None) -> list:
    """Collective preflight of the IPC kernels: every rank reports
    (host, device ordinal, PCI bus id); each rank checks ``hipDeviceCanAccessPeer`` from its
    device to every peer on another device of its host, and the failures of all ranks are
    gathered, so the whole group sees the same list (every rank must make the same
    IPC-or-RCCL choice: the kernels' tags count calls).  Ranks sharing one device (virtual
    ranks) need no peer path.  Returns ``[(rank, dev, peer_rank, peer_dev, why), ...]``."""
    import socket

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    try:
        bus = torch.cuda.get_device_properties(idx).pci_bus_id
    except Exception:  # noqa: BLE001 -- older torch: no bus id, ordinals only
        bus = None
    me = (socket.gethostname(), idx, bus)
    info = [None] * world
    dist.all_gather_object(info, me, group=group)
    can = can_access or torch.cuda.can_device_access_peer
    mine = []
    for r, (host, pidx, pbus) in enumerate(info):
        if r == rank:
            continue
        if host != me[0]:
            mine.append((rank, idx, r, pidx, "ranks on different hosts (%s, %s)" % (me[0], host)))
        elif pidx == idx or (bus is not None and pbus == bus):
            continue  # the same device: virtual ranks
        elif not can(idx, pidx):
            mine.append((rank, idx, r, pidx, "hipDeviceCanAccessPeer(%d, %d) = 0" % (idx, pidx)))
    every = [None] * world
    dist.all_gather_object(every, mine, group=group)
    return [f for fs in every for f in fs]


def coresident_ranks(group=None, device=None) -> int:
    """How many ranks of ``group`` (this one included) run on this rank's device: same host
    and the same device ordinal or PCI bus id (virtual ranks share one)."""
    import socket

    world = dist.get_world_size(group)
    dev = torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    try:
        bus = torch.cuda.get_device_properties(idx).pci_bus_id
    except Exception:  # noqa: BLE001
        bus = None
    me = (socket.gethostname(), idx, bus)
    info = [None] * world
    dist.all_gather_object(info, me, group=group)
    return sum(1 for h, i, b in info if h == me[0] and (i == idx or (bus is not None and b == bus)))


def describe_failures(fails) -> str:
    return "; ".join("rank %d (device %d) -> rank %d (device %d): %s" % f for f in fails)


# ranks the fused all-reduce epilogue's buffer holds (csrc/kernels/fused_ar.h FAR_MAX_RANKS)
FAR_MAX_RANKS = 8


class CustomAllReduce:
    MAX_RANKS = 8

    def __init__(self, group=None, device=None, max_bytes: int = 1 << 20):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > self.MAX_RANKS:
            raise ValueError("custom all-reduce supports at most 8 ranks")
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.max_bytes = int(max_bytes)
        # two-shot from this many bytes (and 4+ ranks: at 2 ranks both forms move the same
        # bytes and the one-shot has one hop less)
        self.two_shot_min = int(os.environ.get("P2P_CAR_2SHOT_MIN", str(256 << 10)))
        L = self.L = _lib.lib()
        tmo = int(os.environ.get("P2P_CAR_TIMEOUT_MS", "0"))
        if tmo > 0:  # spin bound of every one-shot / fused call (default 5 s)
            self.set_timeout_ms(tmo)
        # partials of the fused row-parallel epilogue (ops.skinny_gemm_ar), as 8-byte tagged
        # granules of two bf16 (4 bytes per element): up to 64 rows of a 16384-wide state
        self.far_max_bytes = int(os.environ.get("P2P_FAR_MAX_BYTES", str(4 << 20)))
        self._opened = []
        self._owned = []
        with torch.cuda.device(self.device):
            self._bases = self._map(L.p2p_car_buffer_bytes(self.max_bytes))
            self._far_bases = self._map(L.p2p_far_buffer_bytes(self.far_max_bytes))
            self.counters = torch.zeros(64, dtype=torch.int32, device=self.device)
            self.far_counters = torch.zeros(1024, dtype=torch.int32, device=self.device)
            # [0]: timeout bits (1 one-shot, 2 fused); [1..3]: the fused epilogue's first
            # timeout (column group + 1, call seq, mask of the sources that never arrived)
            self.err = torch.zeros(4, dtype=torch.int32, device=self.device)
        torch.cuda.synchronize(self.device)
        # ranks of this group on THIS device (virtual ranks: all of them; a node with one GPU
        # per rank: 1): the fused all-reduce launch keeps to its share of the device's block
        # slots, so every rank's grid fits at once (csrc/kernels/skinny_gemm_impl.h EPI_AR)
        self.coresident = coresident_ranks(self.group, self.device)
        L.p2p_far_set_coresident(self.coresident)
        dist.barrier(group=self.group)

    def _map(self, size):
        """Allocate an uncached buffer, exchange IPC handles over the group, map the peers'.
        Returns the world's base pointers (own at [rank])."""
        L = self.L
        buf = ctypes.c_void_p()
        _lib.check(L.p2p_car_alloc(size, ctypes.byref(buf)), "car_alloc")
        self._owned.append(buf)
        hsz = L.p2p_car_handle_size()
        handle = ctypes.create_string_buffer(hsz)
        _lib.check(L.p2p_car_get_handle(buf, handle), "car_get_handle")
        handles = [None] * self.world
        dist.all_gather_object(handles, handle.raw, group=self.group)
        bases = []
        for r, hb in enumerate(handles):
            if r == self.rank:
                bases.append(buf.value)
                continue
            ptr = ctypes.c_void_p()
            err = L.p2p_car_open_handle(ctypes.create_string_buffer(hb, hsz), ctypes.byref(ptr))
            if err != 0:
                raise PeerAccessError(
                    "custom all-reduce: rank %d cannot map rank %d's IPC buffer (hipError %d, "
                    "hipIpcOpenMemHandle); %s" % (self.rank, r, err, _HINT))
            self._opened.append(ptr)
            bases.append(ptr.value)
        return (ctypes.c_void_p * self.world)(*bases)

    def fits(self, t: torch.Tensor) -> bool:
        return (t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
                and t.numel() * 2 <= self.max_bytes)

    def fits_bytes(self, nbytes: int) -> bool:
        return nbytes % 16 == 0 and nbytes <= self.max_bytes

    def allreduce_max_u64_(self, keys: torch.Tensor, blocks: int = 0):
        """keys = elementwise max over ranks (int64 storage, unsigned order), in place."""
        assert keys.dtype == torch.int64 and keys.is_contiguous() and self.fits_bytes(keys.numel() * 8)
        _lib.check(self.L.p2p_car_allreduce_max_u64(self._bases, self.rank, self.world,
                                                    self.max_bytes, keys.data_ptr(),
                                                    keys.data_ptr(), keys.numel(),
                                                    self.counters.data_ptr(), self.err.data_ptr(),
                                                    blocks, _lib.stream_ptr(keys.device)),
                   "car_allreduce_max_u64")
        return keys

    def all_gather_(self, out: torch.Tensor, t: torch.Tensor, blocks: int = 0):
        """out (world x t's bytes, rank-major) = every rank's t."""
        nb = t.numel() * t.element_size()
        assert t.is_contiguous() and out.is_contiguous() and self.fits_bytes(nb)
        assert out.numel() * out.element_size() == self.world * nb
        _lib.check(self.L.p2p_car_all_gather(self._bases, self.rank, self.world, self.max_bytes,
                                             t.data_ptr(), out.data_ptr(), nb,
                                             self.counters.data_ptr(), self.err.data_ptr(),
                                             blocks, _lib.stream_ptr(t.device)), "car_all_gather")
        return out

    @staticmethod
    def set_timeout_ms(ms: int):
        """Spin bound of the one-shot kernels (default 5 s); fault-injection tests lower it."""
        _lib.check(_lib.lib().p2p_car_set_timeout_ms(int(ms)), "car_set_timeout_ms")

    def use_two_shot(self, nbytes: int) -> bool:
        return self.world >= 4 and nbytes >= self.two_shot_min

    def allreduce_add_(self, h: torch.Tensor, partial: torch.Tensor, blocks: int = 0,
                       two_shot: bool | None = None):
        """h += sum over ranks of partial (bf16, same shape, contiguous).  two_shot: None =
        by size (``use_two_shot``); both forms give bit-identical sums."""
        assert self.fits(partial) and h.is_contiguous() and h.numel() == partial.numel()
        if two_shot is None:
            two_shot = self.use_two_shot(partial.numel() * 2)
        fn = self.L.p2p_car_allreduce_add_2shot if two_shot else self.L.p2p_car_allreduce_add
        _lib.check(fn(self._bases, self.rank, self.world, self.max_bytes, partial.data_ptr(),
                      h.data_ptr(), partial.numel(), self.counters.data_ptr(),
                      self.err.data_ptr(), blocks, _lib.stream_ptr(h.device)),
                   "car_allreduce_add" + ("_2shot" if two_shot else ""))
        return h

    def check(self):
        """Raise if any call timed out waiting for a peer (numbers would be wrong)."""
        ev = self.err.cpu().tolist()
        e = ev[0]
        if e != 0:
            where = {1: "one-shot kernel", 2: "fused GEMM epilogue"}.get(e, "one-shot + fused")
            if e & 2:  # where the first fused wait gave up, and each group's call count
                c = self.far_counters[:256].cpu()
                miss = [p for p in range(self.world) if ev[3] >> p & 1]
                where += (" (rank %d, coresident %d: first timeout at column group %d of call %d, "
                          "no granule from ranks %s; call counts over column groups min %d max %d)"
                          % (self.rank, self.coresident, ev[1] - 1, ev[2], miss, int(c.min()),
                             int(c.max())))
            raise CollectiveTimeout("custom all-reduce: a peer never arrived (timeout in the %s); "
                                    "the TP group is broken" % where)

    def fused_ok(self, M: int, N: int, ld: int) -> bool:
        """Can ops.skinny_gemm_ar sum an [M, N] partial (row stride ld) through the fused
        buffer?  (A group wider than the kernel's FAR_MAX_RANKS takes the partial store +
        one-shot path instead.)"""
        return self.world <= FAR_MAX_RANKS and 1 <= M <= 64 and N % 16 == 0 and N // 16 <= 1024 and ld % 8 == 0 and \
            ((M - 1) * ld + N) * 4 <= self.far_max_bytes

    def close(self):
        if not self._owned:
            return
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.L.p2p_car_close_handle(p)
        self._opened = []
        for b in self._owned:
            self.L.p2p_car_free(b)
        self._owned = []
