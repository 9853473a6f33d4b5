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
        # back-to-back calls alternating above / below 32768 vectors (slices of different
        # block counts) with one rank delayed on the GPU: no host sync between calls
        dist.barrier()
        sizes = [1 << 19, 8, 300008, 4096, 1 << 19, 16, 262152, 8, 1 << 19, 4096] * 2
        outs, refs = [], []
        for i, n in enumerate(sizes):
            call += 1
            h0 = _data(7 + call, n)
            h = h0.cuda()
            p = _data(1000 * call + rank, n).cuda()
            if rank == 1 and i % 3 == 0:
                torch.cuda._sleep(2_000_000)  # the slow peer
            car.allreduce_add_(h, p)
            outs.append(h)
            refs.append(_expect(h0, world, n, call))
        torch.cuda.synchronize()
        stress = max(((o.cpu().float() - r.float()).abs().max() / (r.float().abs().max() + 1e-6)).item()
                     for o, r in zip(outs, refs))
        # u64 MAX (unsigned order: keys with the top bit set are the largest) and all-gather
        g = torch.Generator().manual_seed(rank + 5)
        keys = torch.randint(-2 ** 62, 2 ** 62, (64, 32), generator=g, dtype=torch.int64)
        keys[rank, 0] = -5  # 0xFFFF...FB: the unsigned maximum of row `rank`
        allk = [None] * world
        dist.all_gather_object(allk, keys)
        kd = keys.cuda()
        car.allreduce_max_u64_(kd)
        u = torch.stack([k for k in allk]).view(torch.int64) ^ (-(2 ** 63))
        want_k = (u.max(0).values ^ (-(2 ** 63)))
        max_ok = bool((kd.cpu() == want_k).all().item())
        t = (torch.arange(1000, dtype=torch.float32) + 10000 * rank).cuda()
        out = torch.empty(world * 1000, dtype=torch.float32, device="cuda")
        car.all_gather_(out, t)
        torch.cuda.synchronize()
        gat_ok = bool((out.cpu() == torch.cat([torch.arange(1000, dtype=torch.float32) + 10000 * r
                                               for r in range(world)])).all().item())
        car.check()
        q.put((rank, max(errs) < 1e-2 and graph_ok and stress < 1e-2 and max_ok and gat_ok,
               (max(errs), graph_ok, stress, max_ok, gat_ok)))
    except Exception:
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        if car is not None:
            dist.barrier()
            car.close()
        dist.destroy_process_group()


def _dead_peer_worker(rank, world, port, q):
    """Rank 1 stops calling: rank 0's one-shot kernel must give up within the spin bound,
    set the error word, and skip later waits; check() raises."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = None
    try:
        from p2p_llm_chat_go_amd.parallel.custom_ar import CollectiveTimeout, CustomAllReduce

        torch.cuda.set_device(0)
        car = CustomAllReduce(device="cuda:0", max_bytes=1 << 20)
        CustomAllReduce.set_timeout_ms(300)
        h = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")
        p = torch.ones_like(h)
        car.allreduce_add_(h, p)
        torch.cuda.synchronize()
        car.check()
        dist.barrier()
        if rank == 1:  # stop calling; keep the buffer mapped until rank 0 is done
            q.put((rank, True, "peer left"))
            dist.barrier()
            return
        t0 = time.time()
        for _ in range(20):  # one timeout, then every later call returns at once
            car.allreduce_add_(h, p)
        torch.cuda.synchronize()
        dt = time.time() - t0
        try:
            car.check()
            q.put((rank, False, "no error after a dead peer"))
        except CollectiveTimeout:
            q.put((rank, dt < 5.0, "raised after %.2fs" % dt))
        dist.barrier()
    except Exception:
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        if car is not None:
            car.close()
        dist.destroy_process_group()


def test_custom_allreduce_dead_peer_raises():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_dead_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = [q.get(timeout=300) for _ in range(2)]
    [p.join(timeout=60) for p in ps]
    [p.terminate() for p in ps if p.is_alive()]
    for rank, ok, info in res:
        assert ok, (rank, info)


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


def _two_shot_worker(rank, world, port, q):
    """Two-shot sum (reduce-scatter to shard owners + all-gather) against the one-shot
    form (bit-identical) and the fp32 reference: uneven shards, alternating forms and
    sizes with a delayed peer, hipGraph replay."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = None
    try:
        from p2p_llm_chat_go_amd.parallel.custom_ar import CustomAllReduce

        torch.cuda.set_device(0)
        car = CustomAllReduce(device="cuda:0", max_bytes=4 << 20)
        call = 0
        same, errs = True, []
        sizes = [8, 4096 + 8, 8 * world * 3 + 8, 300008, 1 << 20, 2 << 20, 24, 1 << 19] * 2
        outs = []
        for i, n in enumerate(sizes):
            call += 1
            h0 = _data(7 + call, n)
            p = _data(1000 * call + rank, n).cuda()
            h1, h2 = h0.cuda(), h0.cuda()
            if rank == world - 1 and i % 3 == 1:
                torch.cuda._sleep(2_000_000)  # the slow peer
            car.allreduce_add_(h1, p, two_shot=False)
            car.allreduce_add_(h2, p, two_shot=True)
            outs.append((h1, h2, _expect(h0, world, n, call)))
        torch.cuda.synchronize()
        for h1, h2, ref in outs:
            same = same and torch.equal(h1, h2)
            errs.append(((h2.cpu().float() - ref.float()).abs().max() /
                         (ref.float().abs().max() + 1e-6)).item())
        n = 1 << 18
        h = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        p = torch.ones(n, dtype=torch.bfloat16, device="cuda") * (rank + 1)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(4):
                    car.allreduce_add_(h, p, two_shot=True)
        torch.cuda.synchronize()
        h.zero_()
        torch.cuda.synchronize()
        dist.barrier()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        graph_ok = bool((h.float() == 12 * sum(r + 1 for r in range(world))).all().item())
        # timing (virtual ranks share one GPU: relative only, not xGMI numbers)
        tim = {}
        for n in (1 << 17, 1 << 20, 2 << 20):
            hh = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
            pp = torch.ones_like(hh)
            for two in (False, True):
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                car.allreduce_add_(hh, pp, two_shot=two)
                e0.record()
                for _ in range(10):
                    car.allreduce_add_(hh, pp, two_shot=two)
                e1.record()
                torch.cuda.synchronize()
                tim["%s_%dKiB" % ("2shot" if two else "1shot", n * 2 >> 10)] = round(
                    e0.elapsed_time(e1) * 100, 1)
        car.check()
        q.put((rank, same and max(errs) < 1e-2 and graph_ok, (same, max(errs), graph_ok, tim)))
    except Exception:
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        if car is not None:
            dist.barrier()
            car.close()
        dist.destroy_process_group()


def test_custom_allreduce_two_shot_four_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 4
    port = _port()
    ps = [ctx.Process(target=_two_shot_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = [q.get(timeout=300) for _ in range(world)]
    [p.join(timeout=60) for p in ps]
    [p.terminate() for p in ps if p.is_alive()]
    for rank, ok, info in res:
        print("rank", rank, info)
        assert ok, (rank, info)
