"""TP row-parallel projection with the all-reduce fused into the GEMM epilogue
(``ops.skinny_gemm_ar``, ``csrc/kernels/fused_ar.h``) on virtual ranks sharing the one
MI355X: bit-identical to the unfused pair (partial store + one-shot all-reduce) on every
rank, equal to the fp32 sum of the ranks' products, across parity reuse, row counts
1..64, split-K wave counts, interleaving with the one-shot kernel, and hipGraph replay;
at world 2, 4 and 8."""
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


def _worker(rank, world, port, q):
    # virtual ranks time-share one device: a generous spin bound (5 s on real GPUs)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), P2P_CAR_TIMEOUT_MS="30000",
                      P2P_QA_TIMEOUT_MS="30000")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = None
    try:
        from p2p_llm_chat_go_amd import ops
        from p2p_llm_chat_go_amd.parallel.custom_ar import CustomAllReduce

        torch.cuda.set_device(0)
        car = CustomAllReduce(device="cuda:0", max_bytes=1 << 20)
        dev = torch.device("cuda:0")
        same, errs, n = True, [], 0
        first_fault = None
        cases = [(1, 4096, 1024, 0), (1, 8192, 1024, 2 | (8 << 8)), (5, 4096, 512, 1),
                 (16, 4096, 3584, 8 | (4 << 8)), (44, 4096, 1024, 4), (64, 8192, 512, 0),
                 (3, 1024, 4096, 2), (1, 4096, 1024, 0)]
        if world == 8:
            # 8 virtual ranks on ONE device: 8 x 512 spinning workgroups (N = 8192) exceed
            # what the CUs hold at once, so a rank's resident blocks can wait on a peer's
            # blocks that never get a slot (timeout; profiles/r3_fused_ar_world8_coschedule.log).
            # On 8 GPUs each device runs only its own grid and in-order dispatch guarantees
            # progress.  Here: the 8B TP=8 widths (N = 4096, 256 workgroups per rank).
            cases = [c for c in cases if c[1] <= 4096]
        for rep in range(2):
            for M, N, K, code in cases:
                n += 1
                g = torch.Generator(device=dev).manual_seed(100 * n + rank)  # rank's shard
                w = torch.randn(N, K, generator=g, device=dev) * 0.05
                x = torch.randn(M, K, generator=g, device=dev)
                wt = ops.tile_weight(w.to(torch.bfloat16))
                xb = x.to(torch.bfloat16)
                gh = torch.Generator(device=dev).manual_seed(7 * n)  # residual: same on all
                h0 = torch.randn(M, N, generator=gh, device=dev).to(torch.bfloat16)
                h1, h2 = h0.clone(), h0.clone()
                part = ops.skinny_gemm(wt, xb, ops.EPI_STORE, waves=code)
                car.allreduce_add_(h1, part, two_shot=False)
                ops.skinny_gemm_ar(wt, xb, h2, car, waves=code)
                torch.cuda.synchronize()
                if first_fault is None and int(car.err[0].item()):
                    first_fault = (rep, M, N, K, code)
                same = same and torch.equal(h1, h2)
                # fp32 reference: sum over ranks of their bf16 partials
                parts = [torch.empty_like(part.cpu()) for _ in range(world)]
                dist.all_gather(parts, part.cpu())
                ref = h0.cpu().float() + sum(p.float() for p in parts)
                errs.append(((h2.cpu().float() - ref).abs().max() / (ref.abs().max() + 1e-6)).item())
        # hipGraph: fused calls of two widths interleaved with one-shot calls, replayed
        M = 1
        gw = torch.Generator(device=dev).manual_seed(5 + rank)
        na = 8192 if world < 8 else 2048
        wa = ops.tile_weight((torch.randn(na, 1024, generator=gw, device=dev) * 0.05).to(torch.bfloat16))
        wb = ops.tile_weight((torch.randn(4096, 512, generator=gw, device=dev) * 0.05).to(torch.bfloat16))
        xa = torch.ones(M, 1024, device=dev, dtype=torch.bfloat16)
        xb_ = torch.ones(M, 512, device=dev, dtype=torch.bfloat16)
        ha = torch.zeros(M, na, device=dev, dtype=torch.bfloat16)
        hb = torch.zeros(M, 4096, device=dev, dtype=torch.bfloat16)
        hc = torch.zeros(4096, device=dev, dtype=torch.bfloat16)
        pc = torch.ones(4096, device=dev, dtype=torch.bfloat16)

        def body():
            ops.skinny_gemm_ar(wa, xa, ha, car)
            car.allreduce_add_(hc, pc)
            ops.skinny_gemm_ar(wb, xb_, hb, car)

        body()  # eager, then captured
        torch.cuda.synchronize()
        ea, eb = ha.clone(), hb.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                body()
        torch.cuda.synchronize()
        ha.zero_(), hb.zero_(), hc.zero_()
        torch.cuda.synchronize()
        dist.barrier()
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        graph_ok = (torch.allclose(ha.float(), 3 * ea.float(), rtol=2e-2, atol=1e-2)
                    and torch.allclose(hb.float(), 3 * eb.float(), rtol=2e-2, atol=1e-2)
                    and bool((hc.float() == 3 * world).all().item()))
        if first_fault is not None:
            raise RuntimeError("fused all-reduce timed out first at case %r" % (first_fault,))
        car.check()
        q.put((rank, same and max(errs) < 1e-2 and graph_ok, (same, max(errs), graph_ok)))
    except Exception:
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        if car is not None:
            dist.barrier()
            car.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fused_allreduce_epilogue_bit_identical(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=240))
    finally:
        [p.join(timeout=60) for p in ps]
        [p.terminate() for p in ps if p.is_alive()]
    for rank, ok, info in res:
        assert ok, (rank, info)
