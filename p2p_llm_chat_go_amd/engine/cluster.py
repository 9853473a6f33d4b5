"""Multi-GPU serving behind one node: data-parallel replicas of tensor/expert-
parallel engine groups (SURVEY §2C "TP", "EP", "DP / replica serving").

The reference serves one suggestion per click from a single Ollama process
(`web/streamlit_app.py:89-101`, reached from the node API of
`go/cmd/node/main.go:213-283`).  On an 8 x MI355X box this node instead runs

    node process (HTTP, libp2p, router; never touches a GPU)
      |-- replica 0: leader rank (scheduler + EngineServer) --pipes--> follower ranks
      |-- replica 1: ...
      ...

with ``ENGINE_GPUS`` GPUs split into ``ENGINE_GPUS / (ENGINE_TP * ENGINE_EP)``
replicas.  Every rank is its own process pinned to one GPU (one process per
GPU; RCCL over xGMI plus the one-shot IPC collectives inside each group).

* **TP/EP lockstep.**  Only the group leader runs the continuous-batching
  scheduler.  Each engine-level call it makes (a prefill batch, a chunk of k
  decode steps) is first sent to its followers over a host pipe as a small
  plan (prompt ids, block tables, positions, sampling params, k), then executed
  locally; the followers execute the same call, so every rank replays the same
  hipGraphs and their collectives line up.  Results (tokens) are identical on
  every rank -- greedy keys are MAX-reduced, sampled draws are keyed by
  (seed, position, token) -- so the leader uses its own.
* **DP router.**  The node process sends each request to the live replica with
  the fewest outstanding requests (least-loaded) and relays streamed chunks.
* **Failures are loud.**  A rank that dies breaks its group's collectives: the
  leader's next call raises (``CollectiveTimeout`` / transport error), the
  leader reports ``dead`` and exits non-zero, its in-flight requests fail with
  an error reply, and the router stops sending it work.  A follower whose pipe
  closes (leader gone) exits non-zero.

The worker processes are started with the ``spawn`` method before anything
in the node process initialises the GPU (only ``torch.cuda.device_count()`` is
consulted), so no process that touched the GPU ever forks or execs.
"""
from __future__ import annotations

import itertools
import json
import os
import socket
import threading
import time
import traceback
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutureTimeout


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ------------------------------------------------------------------ rank side
class LockstepEngine:
    """The leader's view of its engine group: every call that runs collectives is
    broadcast to the followers first (plan over the host pipes), then run locally.
    Everything else (cfg, kv, limits) is the local engine's.

    ``dp_split`` (EP ``a2a`` mode: DP attention + expert all-to-all): each sequence lives
    on ONE rank (its home, chosen once when the sequence is admitted: the rank with the
    fewest live sequences, ties rotating; kept keyed by the sequence's first KV page), so
    the group serves world x the sequences of a replicated-attention group.  A prefill / decode call is split by home;
    every rank runs its share padded to the group's largest share (equal row counts and
    chunking, as the static-capacity all-to-all needs), followers send their tokens back
    over the pipe, and the leader reassembles them in call order."""

    def __init__(self, engine, follower_conns, dp_split: bool = False):
        self._eng = engine
        self._conns = list(follower_conns)
        self._lock = threading.Lock()
        self.dp_split = dp_split
        self.world = 1 + len(self._conns)
        self._homes = {}   # dp_split: first KV page of a sequence -> its home rank
        self._load = [0] * self.world  # live sequences per rank (as of the last decode call)
        self._rr = 0

    def __getattr__(self, name):
        return getattr(self._eng, name)

    def _bcast(self, msg):
        for c in self._conns:
            c.send(msg)

    @staticmethod
    def _resolve(params):
        # a request without a seed draws one lazily; draw it HERE so every rank samples
        # with the same key (ranks that drew different tokens would corrupt each other's KV)
        for p in params or ():
            if p is not None and not p.greedy:
                p.resolved_seed()

    # ------------------------------------------------------------ dp_split
    def _parts(self, block_tables, fresh=(), decode=False):
        """Split a call's sequences by home rank.  ``fresh``: indices of sequences admitted
        by this call (a prompt from position 0): each gets a home now, on the rank with the
        fewest live sequences (ties rotate).  Deriving the home from the page id instead
        piles sequences onto a few ranks whenever the allocator's page pattern shares a
        factor with the world size.  A decode call carries every running
        sequence, so it refreshes the live counts."""
        fresh = set(fresh)
        homes = [None if b in fresh else self._homes.get(bt[0])
                 for b, bt in enumerate(block_tables)]
        load = [0] * self.world if decode else list(self._load)
        if decode:
            for h in homes:
                if h is not None:
                    load[h] += 1
        W = self.world
        for b, bt in enumerate(block_tables):
            if homes[b] is None:
                h = min(range(W), key=lambda r: (load[r], (r - self._rr) % W))
                self._rr = (h + 1) % W
                homes[b] = h
                load[h] += 1
                self._homes[bt[0]] = h
        self._load = load
        return [[b for b, h in enumerate(homes) if h == r] for r in range(self.world)]

    @staticmethod
    def _sub(xs, idx):
        return None if xs is None else [xs[i] for i in idx]

    def _recv(self, c):
        try:
            msg = c.recv()
        except (EOFError, OSError):
            raise RuntimeError("peer rank is dead (pipe closed)")
        if msg[0] == "dead":
            raise RuntimeError("peer rank is dead: %s" % (msg[1].strip().splitlines()[-1:],))
        return msg[1]

    def _prefill_split(self, prompts, block_tables, return_logits, sampling, starts):
        parts = self._parts(block_tables, fresh=[b for b in range(len(prompts))
                                                 if not starts or starts[b] == 0])
        rows = [sum(len(prompts[b]) - (starts[b] if starts else 0) for b in part)
                for part in parts]
        pad = max(1, max(rows))
        for k, c in enumerate(self._conns, start=1):
            idx = parts[k]
            c.send(("prefill_part", self._sub(prompts, idx), self._sub(block_tables, idx),
                    return_logits, self._sub(sampling, idx), self._sub(starts, idx), pad))
        idx = parts[0]
        mine = self._eng.prefill(self._sub(prompts, idx), self._sub(block_tables, idx),
                                 return_logits=return_logits, sampling=self._sub(sampling, idx),
                                 starts=self._sub(starts, idx), pad_rows=pad)
        results = [mine] + [self._recv(c) for c in self._conns]
        import torch

        dev = self._eng.device
        first = torch.zeros(len(prompts), dtype=torch.int32)
        logits = None
        for part, res in zip(parts, results):
            if return_logits:
                toks, lg = res
                if logits is None:
                    logits = torch.zeros(len(prompts), lg.shape[1], dtype=torch.float32)
                if part:
                    logits[part] = lg.float().cpu()
            else:
                toks = res
            if part:
                first[part] = toks.cpu() if hasattr(toks, "cpu") else torch.tensor(toks)
        first = first.to(dev)
        return (first, logits.to(dev)) if return_logits else first

    def _decode_split(self, last_ids, pos, block_tables, ctx, k, params):
        parts = self._parts(block_tables, decode=True)
        bmax = max(1, max(len(p) for p in parts))
        # one graph kind for the whole group (every rank replays the same graph)
        greedy = params is None or all(p.greedy for p in params)
        for r, c in enumerate(self._conns, start=1):
            idx = parts[r]
            c.send(("decode_part", self._sub(last_ids, idx), self._sub(pos, idx),
                    self._sub(block_tables, idx), ctx, k, self._sub(params, idx), bmax,
                    greedy))
        idx = parts[0]
        mine = self._eng.decode_steps(self._sub(last_ids, idx), self._sub(pos, idx),
                                      self._sub(block_tables, idx), ctx, k,
                                      self._sub(params, idx), batch_bucket=bmax, greedy=greedy)
        results = [mine] + [self._recv(c) for c in self._conns]
        hist = [None] * len(last_ids)
        for part, res in zip(parts, results):
            for b, h in zip(part, res):
                hist[b] = h
        return hist

    # ------------------------------------------------------------ engine calls
    def prefill(self, prompts, block_tables, return_logits=False, sampling=None, starts=None):
        self._resolve(sampling)
        if self.dp_split:
            with self._lock:
                return self._prefill_split(prompts, block_tables, return_logits, sampling,
                                           starts)
        with self._lock:
            self._bcast(("prefill", prompts, block_tables, return_logits, sampling, starts))
            return self._eng.prefill(prompts, block_tables, return_logits=return_logits,
                                     sampling=sampling, starts=starts)

    def decode_steps(self, last_ids, pos, block_tables, ctx, k, params=None):
        self._resolve(params)
        if self.dp_split:
            with self._lock:
                return self._decode_split(last_ids, pos, block_tables, ctx, k, params)
        with self._lock:
            self._bcast(("decode", last_ids, pos, block_tables, ctx, k, params))
            return self._eng.decode_steps(last_ids, pos, block_tables, ctx, k, params)

    def generate(self, prompts, max_new_tokens=64, stop_on_eos=True, check_every=8):
        if self.dp_split:
            return self._generate_split(prompts, max_new_tokens, stop_on_eos, check_every)
        with self._lock:
            self._bcast(("generate", prompts, max_new_tokens, stop_on_eos, check_every))
            return self._eng.generate(prompts, max_new_tokens, stop_on_eos, check_every)

    def _generate_split(self, prompts, max_new_tokens, stop_on_eos, check_every):
        """Static-batch generate over the split calls (bench / tests; the server drives
        prefill / decode_steps itself)."""
        import time

        from .engine import GenResult
        from .kv_cache import pages_for

        eng = self._eng
        t0 = time.perf_counter_ns()
        pages = [eng.kv.allocator.alloc(pages_for(len(p) + max_new_tokens)) for p in prompts]
        try:
            first = self.prefill(prompts, pages).cpu().tolist()
            t1 = time.perf_counter_ns()
            out = [[int(t)] for t in first]
            eos = set(eng.cfg.eos_ids)
            while len(out[0]) < max_new_tokens:
                live = [b for b in range(len(prompts))
                        if not (stop_on_eos and any(t in eos for t in out[b]))]
                if not live:
                    break
                k = min(check_every, max_new_tokens - len(out[0]))
                hist = self.decode_steps([out[b][-1] for b in range(len(prompts))],
                                         [len(prompts[b]) + len(out[b]) - 1
                                          for b in range(len(prompts))],
                                         pages, max(len(p) for p in prompts) + max_new_tokens, k)
                for b in range(len(prompts)):
                    out[b] += [int(t) for t in hist[b]]
            t2 = time.perf_counter_ns()
        finally:
            for p in pages:
                eng.kv.allocator.free(p)
        res = []
        for b, p in enumerate(prompts):
            toks, reason = out[b][:max_new_tokens], "length"
            if stop_on_eos:
                for j, t in enumerate(toks):
                    if t in eng.cfg.eos_ids:
                        toks, reason = toks[:j], "stop"
                        break
            res.append(GenResult(tokens=toks, prompt_eval_count=len(p),
                                 prompt_eval_duration_ns=t1 - t0, eval_count=len(toks),
                                 eval_duration_ns=t2 - t1, total_duration_ns=t2 - t0,
                                 ttft_ns=t1 - t0, done_reason=reason))
        return res

    def stop(self):
        for c in self._conns:
            try:
                c.send(("stop",))
            except (OSError, EOFError):
                pass


def _follower_loop(eng, conn):
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            os._exit(2)  # leader gone: this group is over
        op = msg[0]
        if op == "stop":
            return
        if op == "prefill":
            _, prompts, bts, ret, sampling, starts = msg
            eng.prefill(prompts, bts, return_logits=ret, sampling=sampling, starts=starts)
        elif op == "decode":
            _, ids, pos, bts, ctx, k, params = msg
            eng.decode_steps(ids, pos, bts, ctx, k, params)
        elif op == "generate":
            _, prompts, n, eos, every = msg
            eng.generate(prompts, n, eos, every)
        elif op == "mirror":  # the native group loop: the leader's frames from here on
            from .native_loop import run_follower_mirror

            run_follower_mirror(eng, conn.fileno(), msg[1])
            return
        elif op == "prefill_part":  # dp_split: this rank's share, result back to the leader
            _, prompts, bts, ret, sampling, starts, pad = msg
            res = eng.prefill(prompts, bts, return_logits=ret, sampling=sampling, starts=starts,
                              pad_rows=pad)
            res = (res[0].cpu(), res[1].cpu()) if ret else res.cpu()
            conn.send(("part", res))
        elif op == "decode_part":
            _, ids, pos, bts, ctx, k, params, bmax, greedy = msg
            conn.send(("part", eng.decode_steps(ids, pos, bts, ctx, k, params,
                                                batch_bucket=bmax, greedy=greedy)))
        if eng.device.type == "cuda":
            import torch

            torch.cuda.synchronize(eng.device)


def build_rank_engine(spec: dict, rank: int, device: str):
    """Engine of one rank of a replica group (also used by tests)."""
    from ..engine import Engine
    from ..models.config import get_config
    from ..models.weights import EngineWeights
    from ..parallel.comm import TPComm

    tp, ep = spec.get("tp", 1), spec.get("ep", 1)
    par = dict(tp_rank=rank, tp_size=tp) if tp > 1 else {}
    if ep > 1:
        par = dict(ep_rank=rank, ep_size=ep, ep_mode=spec.get("ep_mode", "allreduce"))
    weights = None
    ckpt = spec.get("checkpoint")
    if ckpt:  # HF checkpoint: every rank reads only its own shard of each tensor
        from ..models.weights import LazySafetensors, config_from_hf

        cfg = config_from_hf(ckpt)
        weights = EngineWeights.from_state_dict(LazySafetensors(ckpt), cfg, device, **{
            k: v for k, v in par.items() if k != "ep_mode"})
    else:
        cfg = get_config(spec["model"])
    if not ckpt and spec.get("sd_seed") is not None:  # sharding-invariant random init (tests)
        from ..models.reference import random_state_dict

        sd = random_state_dict(cfg, seed=int(spec["sd_seed"]))
        weights = EngineWeights.from_state_dict(sd, cfg, device, **{
            k: v for k, v in par.items() if k != "ep_mode"})
    comm = TPComm() if tp * ep > 1 else None
    cuda = device.startswith("cuda")
    return Engine(cfg, weights=weights, device=device, seed=spec.get("seed", 0),
                  kv_pages=spec.get("kv_pages") or (None if cuda else 256),
                  max_batch=spec.get("max_batch", 16), comm=comm,
                  weight_dtype=spec.get("weights"), **par)


def _rank_main(spec, replica, rank, device, port, parent_conn, follower_conns, leader_conn):
    """Entry of one rank process (spawned)."""
    try:
        group = spec.get("tp", 1) * spec.get("ep", 1)
        import torch

        if device.startswith("cuda"):
            torch.cuda.set_device(torch.device(device))
        else:
            torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, spec["world"])))
        if group > 1:
            import datetime

            import torch.distributed as dist

            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            # virtual ranks (tests: a whole group on ONE device) cannot share RCCL's device
            backend = "nccl" if device.startswith("cuda") and not spec.get("virtual") else "gloo"
            if spec.get("virtual") and group > 1:
                # the group's processes share the device's CUs: the wide kernel's K slices meet
                # inside one launch and need each other resident (wide_gemm.hip split_cap)
                os.environ.setdefault("P2P_WIDE_SPLIT_CAP", "1")
            kw = {"device_id": torch.device(device)} if backend == "nccl" else {}
            dist.init_process_group(backend, rank=rank, world_size=group,
                                    timeout=datetime.timedelta(seconds=spec.get("pg_timeout", 600)),
                                    **kw)
        eng = build_rank_engine(spec, rank, device)
        if device.startswith("cuda") and spec.get("warmup", True):
            mb = spec.get("max_batch", 16)
            eng.warmup(tuple(b for b in (1, 2, 4, 8, 16) if b <= mb), ctx=256)
        if rank != 0:
            leader_conn.send(("ready", rank))
            _follower_loop(eng, leader_conn)
            os._exit(0)
        for c in follower_conns:  # every follower built its engine
            msg = c.recv()
            if msg[0] != "ready":
                raise RuntimeError("follower failed: %r" % (msg,))
        _leader_main(spec, replica, eng, parent_conn, follower_conns)
    except BaseException:
        tb = traceback.format_exc()
        try:
            (parent_conn or leader_conn).send(("dead", tb))
        except Exception:
            pass
        print(tb, flush=True)
        os._exit(1)


def _leader_main(spec, replica, eng, parent_conn, follower_conns):
    from .server import EngineServer
    from .tokenizer import get_tokenizer

    from .native_loop import PREFILL_CTX, NativeEngineServer, group_native_ok, make_server

    group = spec.get("tp", 1) * spec.get("ep", 1)
    split = spec.get("ep", 1) > 1 and spec.get("ep_mode", "allreduce") == "a2a"
    front = LockstepEngine(eng, follower_conns, dp_split=split) if group > 1 else eng
    tok = get_tokenizer(eng.cfg, spec.get("tokenizer") or spec.get("checkpoint"))
    kw = dict(model_name=spec.get("model_name", "llama3.1"),
              default_max_tokens=spec.get("max_tokens", 128))
    mirror = group > 1 and group_native_ok(eng, split)
    if group == 1:  # a single-GPU replica runs the native step loop when it can
        server = make_server(eng, tok, **kw)
    elif mirror:
        # TP / EP group on the native loop: the followers switch to their EngineMirror (the
        # channels carry the leader loop's frames from now on, runtime/mirror.h)
        for c in follower_conns:
            c.send(("mirror", PREFILL_CTX))
        # (EP a2a: every rank serves its own sequences, dp_world = the group)
        server = NativeEngineServer(eng, tok, mirror_fds=[c.fileno() for c in follower_conns],
                                    dp_world=group if split else 1, **kw)
    else:  # the Python loop (ENGINE_NATIVE_LOOP=0, CPU engines): the leader broadcasts its calls
        server = EngineServer(front, tok, **kw)
    send_lock = threading.Lock()
    cancelled = set()

    def send(msg):
        with send_lock:
            parent_conn.send(msg)

    def run(kind, rid, text):
        try:
            if kind == "gen":
                out = server.handle_json(text)
            elif kind == "metrics":
                out = json.dumps(dict(server.metrics(), replica=replica, errors=server.errors))
            else:
                def emit(chunk):
                    if rid in cancelled:
                        return False
                    send(("chunk", rid, chunk))
                    return True

                out = server.handle_json_stream(text, emit)
            send(("done", rid, out))
        except BaseException as e:  # noqa: BLE001 -- every failure becomes an error reply
            send(("err", rid, "%s: %s" % (type(e).__name__, e)))
        finally:
            cancelled.discard(rid)

    sock = None
    if hasattr(server, "serve_socket"):
        # the node's engine C ABI reaches this replica's native loop directly over this
        # socket (runtime/loop_remote.h): no pickled pipe, no Python on either side
        try:
            sock = server.serve_socket("p2p-loop-%d-r%d" % (os.getpid(), replica))
        except Exception as e:  # noqa: BLE001 -- the pipe path still serves
            print("replica %d: native socket unavailable: %s" % (replica, e), flush=True)
    send(("ready", replica, sock))

    def watchdog():  # a fatal engine error ends the replica loudly
        while server.dead is None:
            time.sleep(0.1)
        send(("dead", "replica %d: %s" % (replica, server.dead)))
        time.sleep(0.5)
        os._exit(3)

    threading.Thread(target=watchdog, daemon=True).start()
    while True:
        try:
            msg = parent_conn.recv()
        except (EOFError, OSError):
            break
        op = msg[0]
        if op == "stop":
            break
        if op == "cancel":
            cancelled.add(msg[1])
            continue
        threading.Thread(target=run, args=(op, msg[1], msg[2]), daemon=True).start()
    server.close()  # (native group loop: its stop frame ends the followers' mirrors)
    if group > 1 and not mirror:
        front.stop()
    os._exit(0)


# ------------------------------------------------------------------ node side
class _Replica:
    def __init__(self, idx, conn, procs):
        self.idx = idx
        self.conn = conn
        self.procs = procs
        self.socket = None  # the leader loop's native request socket (loop_remote.h)
        self.outstanding = 0
        self.served = 0
        self.alive = True
        self.error = None
        self.lock = threading.Lock()


class ClusterServer:
    """DP router over replica groups; the node's generate hooks (same interface as
    EngineServer: handle_json / handle_json_stream / metrics / close)."""

    def __init__(self, model: str, gpus: int = 1, tp: int = 1, ep: int = 1, device: str = "cuda",
                 max_batch: int = 16, max_tokens: int = 128, model_name: str = "llama3.1",
                 weights: str | None = None, tokenizer: str | None = None, sd_seed=None,
                 kv_pages=None, warmup: bool = True, start_timeout: float = 1800.0,
                 first_gpu: int = 0, checkpoint: str | None = None, ep_mode: str = "allreduce",
                 virtual_ranks: bool = False):
        import multiprocessing as mp

        group = tp * ep
        if gpus % group:
            raise ValueError("ENGINE_GPUS=%d is not a multiple of TP*EP=%d" % (gpus, group))
        self.n_replicas = gpus // group
        self.group = group
        self.model = model
        self.model_name = model_name
        self.max_tokens = max_tokens
        self.tokenizer_path = tokenizer or checkpoint
        self._front_tok = None
        spec = dict(model=model, tp=tp, ep=ep, max_batch=max_batch, max_tokens=max_tokens,
                    model_name=model_name, weights=weights, tokenizer=tokenizer, sd_seed=sd_seed,
                    kv_pages=kv_pages, warmup=warmup, world=gpus, checkpoint=checkpoint or None,
                    ep_mode=ep_mode, virtual=virtual_ranks)
        ctx = mp.get_context("spawn")
        self._replicas = []
        self._rid = itertools.count(1)
        self._waiters = {}  # rid -> (future, emit)
        self._wlock = threading.Lock()
        self._closed = False
        for r in range(self.n_replicas):
            parent_end, leader_end = ctx.Pipe()
            pipes = [ctx.Pipe() for _ in range(group - 1)]
            port = _free_port()
            procs = []
            for k in range(group):
                dev = "cuda:%d" % (first_gpu + r * group + k) if device == "cuda" else "cpu"
                if device == "cuda" and virtual_ranks:  # tests: every rank on one device
                    dev = "cuda:%d" % first_gpu
                if k == 0:
                    args = (spec, r, 0, dev, port, leader_end, [p[0] for p in pipes], None)
                else:
                    args = (spec, r, k, dev, port, None, [], pipes[k - 1][1])
                p = ctx.Process(target=_rank_main, args=args, daemon=True,
                                name="engine-r%d-k%d" % (r, k))
                p.start()
                procs.append(p)
            self._replicas.append(_Replica(r, parent_end, procs))
        deadline = time.time() + start_timeout
        for rep in self._replicas:
            while not rep.conn.poll(1.0):
                if time.time() > deadline or not all(p.is_alive() for p in rep.procs):
                    self.close()
                    raise RuntimeError("engine replica %d failed to start" % rep.idx)
            msg = rep.conn.recv()
            if msg[0] != "ready":
                self.close()
                raise RuntimeError("engine replica %d failed to start:\n%s" % (rep.idx, msg[1]))
            rep.socket = msg[2] if len(msg) > 2 else None
        for rep in self._replicas:
            threading.Thread(target=self._reader, args=(rep,), daemon=True,
                             name="replica-%d-reader" % rep.idx).start()
            threading.Thread(target=self._monitor, args=(rep,), daemon=True,
                             name="replica-%d-monitor" % rep.idx).start()

    def _monitor(self, rep: _Replica):
        """A rank process that exits breaks its group: fail the replica's requests now
        and end its other ranks, instead of waiting for a collective to time out (RCCL
        paths -- prefill sums, all-to-alls -- would hang until the process-group timeout)."""
        from multiprocessing.connection import wait

        live = {p.sentinel: (k, p) for k, p in enumerate(rep.procs)}
        while live and not self._closed:
            ready = wait(list(live), timeout=1.0)
            for s in ready:
                k, p = live.pop(s)
                if self._closed:
                    return
                why = "rank %d exited with code %s" % (k, p.exitcode)
                self._mark_dead(rep, why)
                for q in rep.procs:
                    if q.is_alive():
                        q.terminate()
                return

    # ------------------------------------------------------------ plumbing
    def _reader(self, rep: _Replica):
        while True:
            try:
                msg = rep.conn.recv()
            except (EOFError, OSError):
                msg = ("dead", "replica %d exited" % rep.idx)
            op = msg[0]
            if op == "dead":
                self._mark_dead(rep, msg[1])
                return
            rid = msg[1]
            with self._wlock:
                w = self._waiters.get(rid)
            if w is None:
                continue
            fut, emit = w
            if op == "chunk":
                ok = False
                try:
                    ok = bool(emit(msg[2])) if emit else True
                except Exception:
                    ok = False
                if not ok:
                    self._send(rep, ("cancel", rid))
                continue
            with self._wlock:
                self._waiters.pop(rid, None)
            with rep.lock:
                rep.outstanding -= 1
                rep.served += 1
            if op == "done":
                fut.set_result(msg[2])
            else:
                fut.set_exception(RuntimeError(msg[2]))

    def _mark_dead(self, rep: _Replica, why: str):
        with rep.lock:
            rep.alive = False
            rep.error = why
        with self._wlock:  # fail what this replica still owed
            for rid, (fut, _emit) in list(self._waiters.items()):
                if getattr(fut, "_replica", None) == rep.idx:
                    self._waiters.pop(rid, None)
                    if not fut.done():
                        fut.set_exception(RuntimeError("engine replica %d died: %s"
                                                       % (rep.idx, why.strip().splitlines()[-1]
                                                          if why.strip() else why)))

    def _send(self, rep, msg):
        try:
            with rep.lock:
                rep.conn.send(msg)
        except (OSError, EOFError, ValueError) as e:
            self._mark_dead(rep, "send failed: %s" % e)
            raise

    def _pick(self) -> _Replica:
        live = [r for r in self._replicas if r.alive]
        if not live:
            errs = "; ".join("%d: %s" % (r.idx, (r.error or "").strip().splitlines()[-1:])
                             for r in self._replicas)
            raise RuntimeError("no live engine replica (%s)" % errs)
        return min(live, key=lambda r: (r.outstanding, r.idx))

    def _call(self, kind, text, emit=None, timeout=None):
        """Route one request.  The replica's EngineServer enforces ENGINE_TIMEOUT itself
        (cancel + error reply); this side waits a little longer as a backstop for a
        replica that stopped answering altogether, then cancels and gives up."""
        if timeout is None:
            t = float(os.environ.get("ENGINE_TIMEOUT", "60"))
            timeout = t + 5.0 if t > 0 else None
        rep = self._pick()
        rid = next(self._rid)
        fut = Future()
        fut._replica = rep.idx
        with self._wlock:
            self._waiters[rid] = (fut, emit)
        with rep.lock:
            rep.outstanding += 1
        self._send(rep, (kind, rid, text))
        try:
            return fut.result(timeout)
        except FutureTimeout:
            with self._wlock:
                gone = self._waiters.pop(rid, None) is not None
            if gone:
                with rep.lock:
                    rep.outstanding -= 1
                try:
                    self._send(rep, ("cancel", rid))
                except Exception:  # noqa: BLE001 -- the replica is already marked dead
                    pass
            from .server import EngineTimeout

            raise EngineTimeout("engine replica %d did not answer within %gs" % (rep.idx, timeout)) \
                from None

    # ------------------------------------------------------------- hooks
    def native_front(self) -> dict | None:
        """The engine C ABI's native request path over this cluster (csrc/engine/
        engine_capi.cc + runtime/loop_remote.h): every replica leader's loop socket, and the
        tokenizer's native spec (requests are tokenised here, in the node process, exactly
        as a leader would).  None when a replica has no native loop (EP a2a groups, CPU
        engines): requests then go through handle_json and the replica pipes."""
        if not self._replicas or not all(r.socket for r in self._replicas):
            return None
        import json as _json

        tok = self._tokenizer()
        return {"cluster": [r.socket for r in self._replicas], "model": self.model_name,
                "default_max_tokens": int(self.max_tokens),
                "timeout_s": float(os.environ.get("ENGINE_TIMEOUT", "60")),
                "tokenizer": _json.dumps(tok.native_spec())}

    def _tokenizer(self):
        """The tokenizer a replica leader uses (built once, in this process)."""
        if self._front_tok is None:
            from .tokenizer import get_tokenizer

            if self.tokenizer_path and os.path.isdir(self.tokenizer_path) \
                    and os.path.exists(os.path.join(self.tokenizer_path, "config.json")):
                from ..models.weights import config_from_hf

                cfg = config_from_hf(self.tokenizer_path)
            else:
                from ..models.config import get_config

                cfg = get_config(self.model)
            self._front_tok = get_tokenizer(cfg, self.tokenizer_path)
        return self._front_tok

    def encode_request(self, req_text: str) -> list:
        """Prompt ids of an Ollama request: the C ABI's fallback tokenisation on the
        native_front path (non-ASCII text with the synthetic tokenizer), the same as a
        replica leader's (native_loop.NativeLoopServer.encode_request)."""
        tok = self._tokenizer()
        req = json.loads(req_text)
        if req.get("endpoint") == "chat":
            return tok.chat_messages_ids(req.get("messages") or [])
        if req.get("raw"):
            return tok.encode(req.get("prompt", ""), bos=True)
        return tok.chat_ids(req.get("prompt", ""))

    def decode_ids(self, ids) -> str:
        return self._tokenizer().decode(list(ids))

    def handle_json(self, req_text: str) -> str:
        req = json.loads(req_text)
        if req.get("endpoint") == "metrics":
            return json.dumps(self.metrics())
        return self._call("gen", req_text)

    def handle_json_stream(self, req_text: str, emit) -> str:
        return self._call("stream", req_text, emit=emit)

    def metrics(self) -> dict:
        per = []
        tot = {}
        for rep in self._replicas:
            if not rep.alive:
                per.append({"replica": rep.idx, "alive": False})
                continue
            try:
                rid = next(self._rid)
                fut = Future()
                fut._replica = rep.idx
                with self._wlock:
                    self._waiters[rid] = (fut, None)
                with rep.lock:
                    rep.outstanding += 1
                self._send(rep, ("metrics", rid, ""))
                m = json.loads(fut.result(30))
            except Exception as e:  # noqa: BLE001
                per.append({"replica": rep.idx, "alive": rep.alive, "error": str(e)})
                continue
            m["alive"] = True
            m["routed"] = rep.served
            per.append(m)
            for k, v in m.items():
                if isinstance(v, (int, float)) and not isinstance(v, bool) and k != "replica":
                    tot[k] = tot.get(k, 0) + v
        tot["replicas"] = self.n_replicas
        tot["live_replicas"] = sum(1 for r in self._replicas if r.alive)
        tot["group_size"] = self.group
        tot["per_replica"] = per
        return tot

    def close(self):
        if self._closed:
            return
        self._closed = True
        for rep in self._replicas:
            try:
                rep.conn.send(("stop",))
            except Exception:
                pass
        for rep in self._replicas:
            for p in rep.procs:
                p.join(timeout=30)
                if p.is_alive():
                    p.terminate()


def from_env(device: str | None = None):
    """ClusterServer from the node's ENGINE_* environment (net.node)."""
    gpus = int(os.environ.get("ENGINE_GPUS", "1"))
    tp = int(os.environ.get("ENGINE_TP", "1"))
    ep = int(os.environ.get("ENGINE_EP", "1"))
    dev = device or os.environ.get("ENGINE_DEVICE") or "cuda"
    dev = "cpu" if dev.startswith("cpu") else "cuda"
    model = os.environ.get("ENGINE_MODEL") or ("llama3.1-8b" if dev == "cuda" else "tiny-llama")
    seed = os.environ.get("ENGINE_SD_SEED")
    return ClusterServer(model, gpus=gpus, tp=tp, ep=ep, device=dev,
                         max_batch=int(os.environ.get("ENGINE_MAX_BATCH", "16")),
                         max_tokens=int(os.environ.get("ENGINE_MAX_TOKENS", "128")),
                         model_name=os.environ.get("LLM_MODEL", "llama3.1"),
                         weights=os.environ.get("ENGINE_WEIGHTS") or None,
                         tokenizer=os.environ.get("TOKENIZER_PATH") or None,
                         sd_seed=int(seed) if seed else None,
                         warmup=os.environ.get("ENGINE_WARMUP", "1") != "0",
                         first_gpu=int(os.environ.get("ENGINE_FIRST_GPU", "0")),
                         checkpoint=os.environ.get("ENGINE_CHECKPOINT") or None,
                         ep_mode=os.environ.get("ENGINE_EP_MODE", "allreduce"),
                         kv_pages=int(os.environ["ENGINE_KV_PAGES"]) if os.environ.get("ENGINE_KV_PAGES") else None,
                         # tests: every rank process on the one GPU of the box
                         virtual_ranks=os.environ.get("ENGINE_VIRTUAL_RANKS", "0") == "1")
