"""One-shot IPC all-reduce (csrc/kernels/custom_allreduce.hip) with two ranks
sharing the test box's single MI355X (virtual ranks, SURVEY §4.2 tier (b)):
each process maps the other's uncached buffer through hipIpc, exactly as
ranks on different GPUs do over xGMI.  Checked against the fp32 sum, across
parity reuse, uneven sizes and hipGraph replay."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(seed, n):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _expect(h, world, n, call):
    acc = h.float()
    for r in range(world):
        acc = acc + _data(1000 * call + r, n).float()
    return acc.to(torch.bfloat16)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = None
    try:
        from p2p_llm_chat_go_amd.parallel.custom_ar import CustomAllReduce

        torch.cuda.set_device(0)
        car = CustomAllReduce(device="cuda:0", max_bytes=1 << 20)
        errs = []
        call = 0
        for n in (8, 4096, 8192, 3 * 8192 + 8, 1 << 19):
            for _ in range(3):  # both parities, repeated
                call += 1
                h0 = _data(7 + call, n)
                h = h0.cuda()
                p = _data(1000 * call + rank, n).cuda()
                dist.barrier()
                car.allreduce_add_(h, p)
                torch.cuda.synchronize()
                ref = _expect(h0, world, n, call)
                e = ((h.cpu().float() - ref.float()).abs().max() /
                     (ref.float().abs().max() + 1e-6)).item()
                errs.append(e)
        # captured in a hipGraph, replayed: the per-block counters advance on the device
        n = 8192
        h = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        p = torch.ones(n, dtype=torch.bfloat16, device="cuda") * (rank + 1)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(4):
                    car.allreduce_add_(h, p)
        torch.cuda.synchronize()
        h.zero_()
        torch.cuda.synchronize()
        dist.barrier()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        want = 12 * sum(r + 1 for r in range(world))
        graph_ok = bool((h.float() == want).all().item())
        car.check()
        q.put((rank, max(errs) < 1e-2 and graph_ok, (max(errs), graph_ok)))
    except Exception:
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        if car is not None:
            dist.barrier()
            car.close()
        dist.destroy_process_group()


def test_custom_allreduce_two_ranks_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = [q.get(timeout=300) for _ in range(world)]
    [p.join(timeout=60) for p in ps]
    for rank, ok, info in res:
        assert ok, (rank, info)
