"""Collectives for tensor / expert parallelism over ``torch.distributed``.

On ROCm the ``nccl`` backend *is* RCCL, which rides xGMI between the GPUs of a
node; on CPU the same code runs over ``gloo`` (used by the multi-process CPU
tests).  One process per GPU; every collective is issued on the current
stream so it is captured into the decode hipGraph together with the kernels.

Decode-size messages are tiny (B x 8192 bf16 = 16 KiB per all-reduce for 70B
at batch 1), i.e. latency-bound: 2 all-reduces per layer plus one 64-bit MAX
all-reduce of the greedy argmax keys per step.  On GPUs those row-parallel
sums go through the one-shot IPC all-reduce kernel (``custom_ar.py``, one
xGMI hop instead of RCCL's 2(W-1)); messages above its buffer (long prefill
chunks) use RCCL.  Greedy sampling never gathers
vocab-parallel logits: each rank reduces its vocab shard to (value, token) keys
in the LM-head epilogue and one MAX all-reduce picks the global argmax.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_SIGN = -(2 ** 63)


class TPComm:
    def __init__(self, group=None, custom_ar: bool | None = None, car_max_bytes: int | None = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        # P2P_CUSTOM_AR: 1 (default) IPC kernels, a failed peer-access preflight raises;
        # auto: the same, but a failed preflight falls back to RCCL; 0: RCCL only
        mode = os.environ.get("P2P_CUSTOM_AR", "1")
        if custom_ar is None:
            custom_ar = mode in ("1", "auto")
        self.want_custom_ar = custom_ar
        self.car_fallback = mode == "auto"
        self.peer_failures = []
        # one-/two-shot kernels cover sums up to this size (70B: every row-parallel sum
        # below the overlapped-RCCL threshold of 256 rows); larger ones use RCCL
        if car_max_bytes is None:
            car_max_bytes = int(os.environ.get("P2P_CAR_MAX_BYTES", str(4 << 20)))
        self.car_max_bytes = car_max_bytes
        self.car = None
        self.ep_ipc = None  # parallel.ep_a2a.IpcAllToAll (EP a2a decode exchanges)
        # world-1 groups normally skip the IPC kernels; the TP rank proxy
        # (bench/tp_rank_proxy.py) keeps them so one rank's launch structure is the real one
        self.car_at_world1 = False

    def setup(self, device):
        """Collective-side allocations for ``device`` (call before graph capture)."""
        device = torch.device(device)
        if (self.want_custom_ar and device.type == "cuda" and self.car is None
                and (self.world > 1 or self.car_at_world1)):
            from .custom_ar import (_HINT, CustomAllReduce, PeerAccessError,
                                    describe_failures, peer_access_failures)

            if self.world > 1:
                self.peer_failures = peer_access_failures(self.group, device)
                if self.peer_failures:
                    msg = ("IPC collectives need peer access between every pair of the group's "
                           "GPUs: " + describe_failures(self.peer_failures))
                    if not self.car_fallback:
                        raise PeerAccessError(msg + "; " + _HINT)
                    import warnings

                    warnings.warn(msg + "; using RCCL for every collective (P2P_CUSTOM_AR=auto)")
                    return self
            self.car = CustomAllReduce(self.group, device, self.car_max_bytes)
        return self

    def setup_ep_ipc(self, cmax: int, hidden: int):
        """IPC all-to-all buffers of the DP-attention + EP MoE layer (call on every rank of
        the group, before graph capture).  P2P_EP_IPC=0 keeps RCCL for every exchange."""
        if (self.car is not None and self.ep_ipc is None
                and os.environ.get("P2P_EP_IPC", "1") != "0"):
            from .ep_a2a import IpcAllToAll

            self.ep_ipc = IpcAllToAll(self.car, cmax, hidden)
        return self.ep_ipc

    def close(self):
        self.ep_ipc = None  # its buffers are the car's (freed below)
        if self.car is not None:
            self.car.close()
            self.car = None

    # row-parallel outputs: h += sum_r partial_r
    def allreduce_add_(self, h: torch.Tensor, partial: torch.Tensor):
        if (self.car is not None and h.device.type == "cuda" and self.car.fits(partial)
                and h.is_contiguous()):
            return self.car.allreduce_add_(h, partial)
        if h.device.type == "cpu" or self.backend != "nccl":
            # gloo (CPU tests, virtual ranks on one GPU): reduce in fp32
            buf = partial.float()
            dist.all_reduce(buf, group=self.group)
            h.copy_((h.float() + buf).to(h.dtype))
            return h
        dist.all_reduce(partial, group=self.group)
        h.add_(partial)
        return h

    def allreduce_(self, t: torch.Tensor):
        dist.all_reduce(t, group=self.group)
        return t

    def allreduce_max_u64_(self, keys: torch.Tensor):
        """MAX all-reduce of unsigned 64-bit argmax keys stored in int64."""
        if (self.car is not None and keys.device.type == "cuda" and keys.is_contiguous()
                and self.car.fits_bytes(keys.numel() * 8) and keys.numel() % 2 == 0):
            return self.car.allreduce_max_u64_(keys)  # one-shot, graph-capturable
        keys.bitwise_xor_(_SIGN)  # unsigned order -> signed order
        dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=self.group)
        keys.bitwise_xor_(_SIGN)
        return keys

    def vocab_parallel_argmax(self, logits: torch.Tensor, out: torch.Tensor, v_local: int):
        v, i = logits.max(-1)
        g = i.to(torch.int64) + self.rank * v_local
        if logits.device.type == "cuda" and self.backend != "nccl":
            # gloo moves host memory only (virtual ranks on one GPU in tests)
            v, g = v.cpu(), g.cpu()
        vals = [torch.empty_like(v) for _ in range(self.world)]
        idxs = [torch.empty_like(g) for _ in range(self.world)]
        dist.all_gather(vals, v, group=self.group)
        dist.all_gather(idxs, g, group=self.group)
        V = torch.stack(vals, 0)
        I = torch.stack(idxs, 0)
        best = V.argmax(0)
        out.copy_(I.gather(0, best[None])[0].to(out.dtype))
        return out

    def all_to_all_(self, out: torch.Tensor, inp: torch.Tensor):
        """Equal-split all-to-all along dim 0 (pure data movement: bf16 pairs travel as
        int32, which every backend moves; gloo has no 16-bit types)."""
        a, b = out, inp
        if out.dtype == torch.bfloat16:
            a, b = out.view(torch.int32), inp.view(torch.int32)
        if out.device.type == "cuda" and self.backend != "nccl":
            # gloo moves host memory only (virtual ranks on one GPU in tests)
            ah = torch.empty_like(a, device="cpu")
            dist.all_to_all_single(ah, b.cpu(), group=self.group)
            a.copy_(ah)
            return out
        dist.all_to_all_single(a, b, group=self.group)
        return out

    def all_to_all_v_(self, out: torch.Tensor, inp: torch.Tensor, out_splits: list,
                      in_splits: list):
        """Variable-split all-to-all along dim 0 (rows per peer given on the host)."""
        a, b = out, inp
        if out.dtype == torch.bfloat16:
            a, b = out.view(torch.int32), inp.view(torch.int32)
        if out.device.type == "cuda" and self.backend != "nccl":
            ah = torch.empty_like(a, device="cpu")
            dist.all_to_all_single(ah, b.cpu(), out_splits, in_splits, group=self.group)
            a.copy_(ah)
            return out
        dist.all_to_all_single(a, b, out_splits, in_splits, group=self.group)
        return out

    def max_int(self, v: int) -> int:
        """MAX of a small int over the group (host value in, host value out): the ranks'
        fault bits (LlamaModel.check_faults)."""
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" \
            else torch.device("cpu")
        t = torch.tensor([int(v)], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def check(self):
        """Raise if a one-shot collective timed out waiting for a peer."""
        if self.car is not None:
            self.car.check()

    def all_gather_rows_into(self, out: torch.Tensor, t: torch.Tensor):
        """out [world * n, ...] = every rank's t [n, ...] (rank-major); one-shot on GPUs."""
        if (self.car is not None and t.device.type == "cuda" and t.is_contiguous()
                and self.car.fits_bytes(t.numel() * t.element_size())):
            return self.car.all_gather_(out, t)
        if t.device.type == "cuda" and self.backend != "nccl":  # gloo: host copies
            parts = [torch.empty_like(t, device="cpu") for _ in range(self.world)]
            dist.all_gather(parts, t.cpu(), group=self.group)
            out.copy_(torch.cat(parts, 0))
            return out
        parts = list(out.view(self.world, *t.shape).unbind(0))
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return out

    def all_gather_cols(self, t: torch.Tensor):
        """[B, n] per rank -> [B, world * n] (rank-major columns: vocab-parallel logits)."""
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, 1)

    def all_gather_rows(self, t: torch.Tensor):
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return torch.cat(parts, 0)


def init_distributed(backend: str | None = None):
    """Init from torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); returns (rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local
