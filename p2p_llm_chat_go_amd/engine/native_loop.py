"""The suggest-reply server on the native engine loop (``csrc/runtime/engine_loop.cc``).

Same interface as :class:`engine.server.EngineServer` (the node's generate hooks), but
the continuous-batching step loop runs in a C++ thread: admission, prefill launches,
decode-chunk control, finish detection and KV-page release never enter Python.  Python
only tokenises / formats at the HTTP boundary and, once per new shape, captures a graph
for the loop (``provider``).  The loop replays:

  * prefill chunks: ``engine.graph.PrefillGraph`` (row bucket x sequence bucket, greedy
    argmax or in-graph sampling), with running sequences riding along as one row each;
  * decode steps: ``engine.graph.DecodeGraph`` per (batch bucket, context bucket),
    chunk i+1 enqueued before chunk i is read, the batch state reloaded only when the
    running set changes.

Prompts longer than the largest prefill bucket fall back to Python's chunked prefill
(``eager``).  Used for single-GPU replicas (TP = EP = 1) when the engine runs its graphs
on a GPU (``ENGINE_NATIVE_LOOP``, default on), and for TP / EP groups: the leader's loop
records its device operations and the followers' ``EngineMirror`` threads replay them
(``run_follower_mirror``, ``csrc/runtime/mirror.h``) -- the EP a2a mode (DP attention,
per-rank sequences) included: each rank's share travels in its own frame
(``LoopConfig::dp_world``).
"""
from __future__ import annotations

import json
import os
import time

from ..native import load as load_native
from .engine import BATCH_BUCKETS, CTX_BUCKETS, DECODE_CTX_BUCKETS, Engine
from .graph import PREFILL_ROW_BUCKETS
from .sampling import SamplingParams
from .server import EngineServer, EngineTimeout
from .tokenizer import get_tokenizer

# context bucket (block-table width) of the loop's prefill graphs: prompts up to this many
# tokens prefill through a captured graph; longer ones through the eager chunked path
PREFILL_CTX = int(os.environ.get("ENGINE_PREFILL_GRAPH_CTX", "4096"))


def native_loop_ok(engine: Engine) -> bool:
    return (engine.device.type == "cuda" and engine.use_graph and engine.model.tp == 1
            and engine.prefill_graphs_enabled
            and os.environ.get("ENGINE_NATIVE_LOOP", "1") != "0")


class NativeEngineServer(EngineServer):
    def __init__(self, engine: Engine, tokenizer=None, model_name: str = "llama3.1",
                 max_batch: int | None = None, decode_chunk: int = 8,
                 default_max_tokens: int = 128, max_ctx: int | None = None,
                 prewarm: bool = True, prefill_ctx: int | None = None,
                 mirror_fds: list | None = None, dp_world: int = 1):
        # no Python engine thread: the EngineServer state this class uses is set here
        self.engine = engine
        self.tok = tokenizer or get_tokenizer(engine.cfg)
        self.model_name = model_name
        self.max_batch = max_batch or engine.max_batch
        self.decode_chunk = decode_chunk
        self.default_max_tokens = default_max_tokens
        self.request_timeout_s = float(os.environ.get("ENGINE_TIMEOUT", "60"))
        self.max_ctx = max_ctx or min(engine.cfg.max_pos, CTX_BUCKETS[-1],
                                      engine.kv.num_pages * 64)
        self.errors = 0
        self.prefill_ctx = min(prefill_ctx or PREFILL_CTX, CTX_BUCKETS[-1])
        N = load_native()
        dev = engine.device
        self.loop = N.EngineLoop({
            "num_pages": engine.kv.num_pages, "page_size": 64, "max_batch": self.max_batch,
            "max_prefill_tokens": engine.max_prefill_tokens, "max_ctx": self.max_ctx,
            "eos": [int(e) for e in engine.cfg.eos_ids], "decode_chunk": decode_chunk,
            "admit_wait_us": float(os.environ.get("ENGINE_ADMIT_WAIT_US", "500")),
            "prefill_first": os.environ.get("ENGINE_PREFILL_FIRST", "1") != "0",
            # EP a2a groups (dp_world > 1: DP attention, per-rank sequences) prefill each
            # rank's share eagerly, padded to the largest share; no riders
            "mixed": dp_world <= 1, "dp_world": int(dp_world),
            "pipeline": os.environ.get("ENGINE_PIPELINE", "1") != "0",
            # every running sequence rides in a prompt chunk (ENGINE_RIDERS=tile: only the
            # last 64-row tile's free rows): +4 % at 32 peers, +16 % at 64, same at 8
            # (profiles/r4_serve_native_vs_python.jsonl)
            "riders_all": os.environ.get("ENGINE_RIDERS", "all") == "all",
            "device": dev.index or 0, "batch_buckets": list(BATCH_BUCKETS),
            "ctx_buckets": list(DECODE_CTX_BUCKETS),  # the loop's decode graph buckets
            "row_buckets": [r for r in PREFILL_ROW_BUCKETS
                            if r <= min(engine.max_prefill_tokens, engine.prefill_graph_max_rows)],
            "prefill_max_pages": self.prefill_ctx // 64,
            "prefill_graph_after": engine.prefill_graph_after})
        if mirror_fds:
            # TP / EP group leader (engine.cluster): the followers' EngineMirror threads
            # replay every device operation of this loop (runtime/mirror.h)
            self.loop.set_mirror([int(f) for f in mirror_fds])
        if dev.type == "cuda":
            # the kernels' split-K fault word: a split-K slice that gave up inside a graph
            # fails the step like the graph's own fault word does
            from ..ops.gemm import split_fault_word

            self.loop.set_aux_fault(split_fault_word(dev))
            cw = coll_fault_word(engine)
            if cw:  # an IPC collective that timed out breaks the group: the replica dies
                self.loop.set_coll_fault(cw)
        self.group = 1 + len(mirror_fds or ())
        self.dp_world = int(dp_world)
        self.loop.set_provider(self._provide)
        self.loop.set_eager_prefill(self._eager_prefill)
        self._registered = set()
        self.k_step_graphs = 0  # decode graphs registered with a whole k-step graph
        if prewarm:
            self.prewarm()
        self.loop.start()

    # --------------------------------------------------------------- graphs
    def _provide(self, kind: str, a: int, b: int, greedy: bool):
        """Capture (once) and register the graph the loop asked for (loop thread, GIL)."""
        key = (kind, a, b, greedy)
        if key in self._registered:
            return
        self.loop.mirror_provide(kind, a, b, greedy)  # a group's followers capture it too
        desc = capture_for_loop(self.engine, kind, a, b, greedy, self.prefill_ctx)
        if kind == "decode":
            self.k_step_graphs += 1 if desc.get("exec_k") else 0
            self.loop.add_decode_graph(desc)
        else:
            self.loop.add_prefill_graph(desc)
        self._registered.add(key)

    def prewarm(self, batches=None, rows=None, mode=None):
        """Capture the chat-typical shapes before the first request: decode graphs of every
        batch bucket at the 256-token context, and greedy prompt chunks of every (row
        bucket, sequence bucket) -- a chunk's sequence count is the new prompts plus the
        riders, so under load it is the batch bucket, and a shape first met under load
        would otherwise be captured in the middle of serving (~15-100 ms stalls at the p99:
        profiles/r4_serve_native_vs_python.jsonl).  ENGINE_PREWARM: "full" (default),
        "basic" (one-prompt chunks of <= 128 rows), "off"."""
        mode = mode or os.environ.get("ENGINE_PREWARM", "full")
        if mode == "off":
            return
        for B in batches or [b for b in BATCH_BUCKETS if b <= self.max_batch]:
            self._provide("decode", B, 256, True)
        eng = self.engine
        if self.dp_world > 1:
            return  # prompt chunks run eagerly in EP a2a groups (no prefill graphs)
        if mode == "basic":
            seqs, rows = [1], rows or (16, 32, 48, 64, 96, 128)
        else:
            seqs = sorted({min(b, self.max_batch) for b in BATCH_BUCKETS
                           if b < 2 * self.max_batch})
            rows = rows or PREFILL_ROW_BUCKETS
        for sb in seqs:
            for r in rows:
                if sb <= r <= min(eng.max_prefill_tokens, eng.prefill_graph_max_rows):
                    self._provide("prefill", r, sb, True)

    def _eager_prefill(self, prompts, pages, starts, samp, pad_rows=0):
        params = [SamplingParams(temperature=t, top_k=k, top_p=p, seed=s) for t, k, p, s in samp]
        first = self.engine.prefill(prompts, pages, sampling=params or None,
                                    starts=starts if any(starts) else None, graph=False,
                                    pad_rows=pad_rows or None)
        return [int(x) for x in first.cpu().tolist()]

    # --------------------------------------------------------------- API
    @property
    def dead(self):
        d = self.loop.dead()
        return d or None

    def _submit(self, prompt_ids, params: SamplingParams) -> int:
        return self.loop.submit(list(prompt_ids), int(params.max_tokens), bool(params.stop_on_eos),
                                float(params.temperature), int(params.top_k), float(params.top_p),
                                int(params.resolved_seed()) if not params.greedy else 0)

    def generate(self, prompt_ids, params: SamplingParams, timeout: float | None = None) -> dict:
        t = self.request_timeout_s if timeout is None else float(timeout)
        rid = self._submit(prompt_ids, params)
        r = self.loop.wait(rid, t if t > 0 else -1.0)
        self.loop.release(rid)  # done: forgotten; else cancelled, dropped when it ends
        if r["error"]:
            self.errors += 1
            raise RuntimeError(r["error"])
        if not r["done"]:
            raise EngineTimeout("engine did not answer within %gs (request cancelled)" % t)
        return r

    def native_front(self) -> dict:
        """Everything the engine C ABI (csrc/engine/engine_capi.cc) needs to serve requests
        without entering Python: the loop's plain-C table (runtime/loop_capi.h) and address,
        the tokenizer's native spec, and the server's defaults.  Requests then go
        JSON -> ids -> EngineLoop::submit/wait -> text -> JSON in C++ (tokenisation falls
        back to ``encode_request`` / ``decode_ids`` under the GIL for tokenizers the native
        side does not implement, or non-ASCII text)."""
        N = load_native()
        spec = self.tok.native_spec() if hasattr(self.tok, "native_spec") else {"kind": "hf"}
        return {"api": int(N.loop_api()), "loop": int(self.loop.handle()),
                "model": self.model_name, "default_max_tokens": int(self.default_max_tokens),
                "timeout_s": float(self.request_timeout_s), "tokenizer": json.dumps(spec)}

    def serve_socket(self, name: str) -> str:
        """Serve requests of other processes on the abstract unix socket @name (the node
        of a multi-GPU cluster routes to this replica without Python: runtime/loop_remote.h)."""
        self.loop.serve(name)
        return name

    def encode_request(self, req_text: str) -> list:
        """Prompt ids of an Ollama request (the C ABI's fallback tokenisation)."""
        req = json.loads(req_text)
        if req.get("endpoint") == "chat":
            return self.tok.chat_messages_ids(req.get("messages") or [])
        if req.get("raw"):
            return self.tok.encode(req.get("prompt", ""), bos=True)
        return self.tok.chat_ids(req.get("prompt", ""))

    def decode_ids(self, ids) -> str:
        return self.tok.decode(list(ids))

    def stall(self, seconds: float):
        self.loop.stall(float(seconds))

    def close(self):
        self.loop.shutdown()

    def metrics(self) -> dict:
        m = {k: (int(v) if float(v).is_integer() else v) for k, v in self.loop.metrics().items()}
        m["k_step_graphs"] = self.k_step_graphs
        return m

    def handle_json_stream(self, req_text: str, emit) -> str:
        """Ollama streaming (NDJSON) on the loop: token batches as they are decoded."""
        req = json.loads(req_text)
        params = SamplingParams.from_ollama(req.get("options"), self.default_max_tokens)
        chat = req.get("endpoint") == "chat"
        if chat:
            ids = self.tok.chat_messages_ids(req.get("messages") or [])
        elif req.get("raw"):
            ids = self.tok.encode(req.get("prompt", ""), bos=True)
        else:
            ids = self.tok.chat_ids(req.get("prompt", ""))
        rid = self._submit(ids, params)
        model = req.get("model", self.model_name)
        t_lim = self.request_timeout_s
        deadline = time.perf_counter() + t_lim if t_lim > 0 else None
        toks, text_sent, alive = [], "", True

        def now():
            return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime()) + ".000000Z"

        def flush(final=False):
            nonlocal text_sent, alive
            text = self.tok.decode(toks)
            if not final and text.endswith("\ufffd"):
                return
            delta = text[len(text_sent):] if text.startswith(text_sent) else text
            text_sent = text
            if not delta or not alive:
                return
            chunk = {"model": model, "created_at": now(), "done": False}
            if chat:
                chunk["message"] = {"role": "assistant", "content": delta}
            else:
                chunk["response"] = delta
            alive = bool(emit(json.dumps(chunk)))
            if not alive:  # client went away: stop generating for it
                self.loop.cancel(rid)

        try:
            while True:
                new, done = self.loop.wait_tokens(rid, len(toks), 0.05)
                if new:
                    toks += new
                    flush()
                if done:
                    break
                if deadline is not None and time.perf_counter() > deadline:
                    raise EngineTimeout("engine did not answer within %gs (request cancelled)"
                                        % t_lim)
            r = self.loop.wait(rid, 0.0)
        finally:
            self.loop.release(rid)
        if r["error"]:
            raise RuntimeError(r["error"])
        toks = r["tokens"]
        flush(final=True)
        out = {"model": model, "created_at": now(), "done": True,
               "done_reason": r["done_reason"], "total_duration": r["total_duration"],
               "load_duration": 0, "prompt_eval_count": r["prompt_eval_count"],
               "prompt_eval_duration": r["prompt_eval_duration"], "eval_count": r["eval_count"],
               "eval_duration": r["eval_duration"]}
        if chat:
            out["message"] = {"role": "assistant", "content": ""}
        else:
            out["response"] = ""
            out["context"] = []
        return json.dumps(out)


def capture_for_loop(eng: Engine, kind: str, a: int, b: int, greedy: bool, prefill_ctx: int) -> dict:
    """Capture (or reuse) the graph of one loop shape and describe it for the native loop /
    a follower's mirror: decode (batch bucket a, context bucket b) with its whole k-step
    graph, or a prompt chunk (row bucket a, sequence bucket b).  Every rank of a group runs
    this for the same shapes in the same order (the leader's provider, mirrored), so the
    collectives recorded in the graphs pair up."""
    if kind == "decode":
        g = eng.decode_graph(a, b, greedy=greedy)
        if greedy and g.graph is not None and g.k_steps > 1 and g.graph_k is None:
            g._capture_steps()  # the loop launches whole k-step graphs first
        return g.describe()
    # (the loop asks only for shapes that recur: prefill_graph_after)
    return eng.prefill_graph(a, b, prefill_ctx, greedy=greedy).describe()


def group_native_ok(engine: Engine, dp_split: bool) -> bool:
    """A TP / EP group serves on the native loop (leader) + mirrors (followers) when its
    engines run graphs on GPUs.  The EP a2a mode (DP attention, dp_split: the ranks hold
    different sequences) runs there too since round 6 -- each rank's share in its own frame,
    the followers' tokens back on the status channel (LoopConfig::dp_world); its prompt
    chunks prefill eagerly, so it does not need prefill graphs."""
    return (engine.device.type == "cuda" and engine.use_graph
            and (dp_split or engine.prefill_graphs_enabled)
            and os.environ.get("ENGINE_NATIVE_LOOP", "1") != "0")


def coll_fault_word(engine: Engine) -> int:
    """Device address of the IPC collectives' timeout word (parallel/custom_ar.py
    CustomAllReduce.err[0]; 0 without IPC collectives).  The Python loop raises on it in
    LlamaModel.check_faults; the native loop reads it behind every step."""
    car = getattr(getattr(engine.model, "comm", None), "car", None)
    return int(car.err.data_ptr()) if car is not None else 0


def run_follower_mirror(engine: Engine, fd: int, prefill_ctx: int) -> None:
    """A follower rank's side of the native group loop: apply the leader's frames from the
    channel ``fd`` until its stop.  Graph captures and eager prefills the leader mirrors
    call back here (same code as the leader's provider).  Raises if the mirror failed."""
    N = load_native()
    dev = engine.device
    m = N.EngineMirror(int(fd), dev.index or 0)

    def provide(kind, a, b, greedy):
        desc = capture_for_loop(engine, kind, a, b, greedy, prefill_ctx)
        (m.add_decode_graph if kind == "decode" else m.add_prefill_graph)(desc)

    def eager(prompts, pages, starts, samp, pad_rows=0):
        params = [SamplingParams(temperature=t, top_k=k, top_p=p, seed=s) for t, k, p, s in samp]
        first = engine.prefill(prompts, pages, sampling=params or None,
                               starts=starts if any(starts) else None, graph=False,
                               pad_rows=pad_rows or None)
        return [int(x) for x in first.cpu().tolist()]

    m.set_provider(provide)
    m.set_eager_prefill(eager)
    if dev.type == "cuda":  # reported to the leader with the graphs' own words (mirror.h)
        from ..ops.gemm import split_fault_word

        m.set_aux_fault(split_fault_word(dev))
        cw = coll_fault_word(engine)
        if cw:
            m.set_coll_fault(cw)
    err = m.run()
    import torch

    torch.cuda.synchronize(dev)
    m.shutdown()
    if err:
        raise RuntimeError("group mirror failed: %s" % err)


def make_server(engine: Engine, tokenizer=None, **kw) -> EngineServer:
    """The native-loop server when the engine supports it, else the Python loop."""
    if native_loop_ok(engine):
        return NativeEngineServer(engine, tokenizer, **kw)
    return EngineServer(engine, tokenizer, **kw)
