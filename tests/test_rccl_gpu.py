"""RCCL (the ``nccl`` backend of torch.distributed on ROCm) under the engine's collective
layer, on the real GPU.  The test pool has one MI355X and RCCL refuses two ranks on one
device, so this runs a one-rank RCCL communicator: every ``TPComm`` entry point that
takes the RCCL branch (row-parallel sum, unsigned-64 MAX of argmax keys, variable-split
all-to-all, row all-gather, vocab-parallel argmax) is executed by RCCL kernels, eagerly
and captured in a hipGraph -- the same calls the 8-GPU TP/EP paths issue (SURVEY §2C
"collective backend").  Multi-rank numerics are covered by gloo at world 2/4/8
(test_parallel_cpu.py) and the one-shot IPC kernels by test_custom_ar_gpu.py."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from p2p_llm_chat_go_amd.parallel.comm import TPComm

        comm = TPComm().setup(dev)
        assert comm.backend == "nccl" and comm.car is None  # world 1: RCCL for everything
        g = torch.Generator().manual_seed(0)
        h0 = torch.randn(4, 4096, generator=g).to(torch.bfloat16).to(dev)
        p = torch.randn(4, 4096, generator=g).to(torch.bfloat16).to(dev)
        h = h0.clone()
        comm.allreduce_add_(h, p.clone())
        torch.cuda.synchronize()
        assert torch.equal(h, h0 + p), "allreduce_add_"
        keys = torch.tensor([(-2 ** 63) + 5, 7, -1, 2 ** 62], dtype=torch.int64, device=dev)
        k0 = keys.clone()
        comm.allreduce_max_u64_(keys)
        assert torch.equal(keys, k0), "allreduce_max_u64_"
        inp = torch.randn(6, 128, generator=g).to(torch.bfloat16).to(dev)
        out = torch.empty_like(inp)
        comm.all_to_all_v_(out, inp, [6], [6])
        assert torch.equal(out, inp), "all_to_all_v_"
        out2 = torch.empty(3, 128, dtype=torch.bfloat16, device=dev)
        comm.all_gather_rows_into(out2, inp[:3].contiguous())
        assert torch.equal(out2, inp[:3]), "all_gather_rows_into"
        logits = torch.randn(2, 1000, generator=g).to(dev)
        ids = torch.empty(2, dtype=torch.int32, device=dev)
        comm.vocab_parallel_argmax(logits, ids, 1000)
        assert torch.equal(ids.long(), logits.argmax(-1)), "vocab_parallel_argmax"
        # the decode path: an RCCL all-reduce captured in a hipGraph and replayed
        hg, pg = h0.clone(), p.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            comm.allreduce_add_(hg, pg)  # warm the communicator outside capture
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
                comm.allreduce_add_(hg, pg)
        torch.cuda.synchronize()
        for _ in range(3):
            hg.copy_(h0)
            graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(hg, h0 + p), "captured allreduce_add_"
        dist.destroy_process_group()
        q.put((True, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((False, "%s: %s" % (type(e).__name__, e)))


def test_rccl_collectives_one_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_worker, args=(_port(), q))
    pr.start()
    ok, info = q.get(timeout=180)
    pr.join(timeout=60)
    if pr.is_alive():
        pr.terminate()
    assert ok, info
