"""The RCCL (``nccl`` backend) code paths of ``parallel.comm.TPComm`` on a real RCCL
communicator: one rank on the box's one GPU (RCCL refuses two ranks on one device, so
world > 1 needs the driver's multi-GPU node; the protocol itself is covered at world 2-8 by
the gloo / IPC tests).  Exercised here under RCCL instead of gloo: the row-parallel sum
(with the one-shot kernel off: the RCCL all-reduce + add), the chunked prefill overlap
(all-reduces on a side stream behind per-chunk events, as ``LlamaModel._row_parallel_
overlapped``), the MAX of argmax keys and of fault bits, the equal- and variable-split
all-to-alls of the MoE exchange (bf16 moved as int32), the gathers, and the all-reduce
captured inside a hipGraph.  Reference behaviour: none (the reference has no collectives);
results are checked against the world-1 identities."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r"""
    import os, sys, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["ROOT"])
    from p2p_llm_chat_go_amd.parallel.comm import TPComm
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    comm = TPComm(custom_ar=False)
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(1)
    # row-parallel sum: h += sum over ranks of partial (world 1: h + partial), RCCL path
    h = torch.randn(37, 4096, generator=g).to(torch.bfloat16).to(dev)
    part = torch.randn(37, 4096, generator=g).to(torch.bfloat16).to(dev)
    ref = (h.float() + part.float()).to(torch.bfloat16)
    comm.allreduce_add_(h, part)
    torch.cuda.synchronize()
    assert torch.equal(h, ref), "allreduce_add_"
    # chunked prefill overlap: the all-reduce of chunk i on a comm stream behind an event
    h = torch.randn(512, 1024, generator=g).to(torch.bfloat16).to(dev)
    part = torch.randn(512, 1024, generator=g).to(torch.bfloat16).to(dev)
    ref = (h.float() + part.float()).to(torch.bfloat16)
    cur, cs = torch.cuda.current_stream(), torch.cuda.Stream()
    for a in range(0, 512, 128):
        ev = torch.cuda.Event()
        ev.record(cur)
        with torch.cuda.stream(cs):
            cs.wait_event(ev)
            comm.allreduce_add_(h[a:a + 128], part[a:a + 128])
    cur.wait_stream(cs)
    torch.cuda.synchronize()
    assert torch.equal(h, ref), "overlapped chunks"
    # MAX of unsigned 64-bit argmax keys and of fault bits
    keys = torch.tensor([-1, 5, 1 << 62, 7], dtype=torch.int64, device=dev)
    assert torch.equal(comm.allreduce_max_u64_(keys.clone()), keys)
    assert comm.max_int(4) == 4
    # MoE exchange: equal and variable splits, bf16 moved as int32
    x = torch.randn(64, 256, generator=g).to(torch.bfloat16).to(dev)
    out = torch.empty_like(x)
    comm.all_to_all_(out, x)
    out2 = torch.empty_like(x)
    comm.all_to_all_v_(out2, x, [64], [64])
    torch.cuda.synchronize()
    assert torch.equal(out, x) and torch.equal(out2, x), "all_to_all"
    # gathers (vocab-parallel logits, rows)
    t = torch.randn(3, 100, generator=g).to(dev)
    assert torch.equal(comm.all_gather_cols(t), t) and torch.equal(comm.all_gather_rows(t), t)
    rows = torch.empty(3, 100, device=dev)
    comm.all_gather_rows_into(rows, t)
    assert torch.equal(rows, t)
    # an RCCL all-reduce captured in a hipGraph and replayed
    buf = torch.ones(1024, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        comm.allreduce_(buf)  # warm the communicator outside capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    # thread_local as the engine captures (engine/graph.py): under the default global mode
    # the process group's watchdog thread, polling the warm-up call's event during the
    # capture, is an illegal call and aborts the process (the likely cause of one abort of
    # this test on the box)
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        comm.allreduce_(buf)
        buf.mul_(2)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(buf, torch.full_like(buf, 8.0)), "graph replay"
    dist.destroy_process_group()
    print("RCCL_WORLD1_OK")
""")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_tpcomm_rccl_paths_world1():
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=240, cwd=ROOT)
    if r.returncode != 0:
        print(r.stdout[-3000:])
        print(r.stderr[-8000:])
    assert r.returncode == 0 and "RCCL_WORLD1_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
