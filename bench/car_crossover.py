#!/usr/bin/env python3
"""One-shot vs two-shot IPC all-reduce (csrc/kernels/custom_allreduce.hip) across message
sizes at world W, on virtual ranks sharing ONE device (W processes, gloo for setup).

What this measures: the kernels' own structure (one push + one wait vs two pushes + two
waits, per-block work, launch shape) with every "xGMI" transfer landing in local HBM.
What it cannot measure: link bandwidth / latency -- on 8 GPUs the one-shot moves (W-1)x
the message per rank over 7 links, the two-shot 2(W-1)/W x.  The crossover it reports is
therefore a lower bound for the real one (the one-shot's extra bytes cost more over
xGMI than in HBM).  Prints one JSON line per size (rank 0)."""
import argparse
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, port, sizes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), P2P_CAR_TIMEOUT_MS="30000")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from p2p_llm_chat_go_amd.parallel.custom_ar import CustomAllReduce

    torch.cuda.set_device(0)
    car = CustomAllReduce(device="cuda:0", max_bytes=4 << 20)
    out = []
    for nbytes in sizes:
        n = nbytes // 2
        h = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        p = torch.ones_like(h)
        row = {"bytes": nbytes, "world": world}
        for two in (False, True):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(20):
                        car.allreduce_add_(h, p, two_shot=two)
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(3):
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1000 / 20)
            row["two_shot_us" if two else "one_shot_us"] = round(best, 2)
        out.append(row)
    car.check()
    q.put((rank, out))
    dist.barrier()
    car.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    sizes = [16 << 10, 64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, a.world, port, sizes, q)) for r in range(a.world)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=600) for _ in range(a.world))
    [p.join(timeout=60) for p in ps]
    for row in res[0]:
        row["slowest_rank_one_shot_us"] = max(res[r][i]["one_shot_us"] for r in res
                                              for i in range(len(res[r])) if res[r][i]["bytes"] == row["bytes"])
        row["slowest_rank_two_shot_us"] = max(res[r][i]["two_shot_us"] for r in res
                                              for i in range(len(res[r])) if res[r][i]["bytes"] == row["bytes"])
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
