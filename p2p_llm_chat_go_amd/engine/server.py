"""Continuous-batching suggest-reply server (the in-process Ollama replacement).

HTTP threads of the C++ node call ``handle_json`` (Ollama ``/api/generate`` /
``/api/chat`` request JSON -> response JSON).  Requests are queued in the
native ``Scheduler`` (csrc/runtime/scheduler.cc); one engine thread runs the
loop:

    plan = scheduler.schedule()
    prefill the newly admitted prompts (one flat batch)     -> first tokens (TTFT)
      ... with one decode row per already-running sequence  (mixed batch)
    decode every running sequence for a chunk of k steps     (hipGraph replays)
    retire finished sequences (EOS / num_predict), free their KV pages

so concurrent peers share every weight read of the decode step (the reference
serves one blocking request per click, `web/streamlit_app.py:163-165`).
"""
from __future__ import annotations

import json
import os
import threading
import time
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutureTimeout

import torch

from ..native import load as load_native
from ..utils.trace import span
from .engine import CTX_BUCKETS, Engine
from .sampling import SamplingParams
from .tokenizer import get_tokenizer


class _RiderRow:
    """A running sequence riding in a prefill batch as one row: behaves like a prompt of
    length pos + 1 whose only read position is ``pos`` (O(1), not an O(context) list)."""
    __slots__ = ("pos", "tok")

    def __init__(self, pos: int, tok: int):
        self.pos, self.tok = pos, tok

    def __len__(self):
        return self.pos + 1

    def __getitem__(self, i):
        if i != self.pos:
            raise IndexError("rider rows only expose their last position")
        return self.tok


class EngineTimeout(TimeoutError):
    """A request got no reply within the engine deadline (ENGINE_TIMEOUT); it was
    cancelled.  The node answers /suggest with 503 "LLM unavailable: ..." -- the reference
    UI's 60 s bound on the co-pilot call (`web/streamlit_app.py:95,99-101`)."""


class EngineServer:
    def __init__(self, engine: Engine, tokenizer=None, model_name: str = "llama3.1",
                 max_batch: int | None = None, decode_chunk: int = 8,
                 default_max_tokens: int = 128, max_ctx: int | None = None,
                 mixed: bool = True):
        self.engine = engine
        self.tok = tokenizer or get_tokenizer(engine.cfg)
        self.model_name = model_name
        self.max_batch = max_batch or engine.max_batch
        self.decode_chunk = decode_chunk
        # a prefill step also advances every running sequence by one token (its row rides
        # in the prefill batch): admissions no longer stall the running batch for a step
        self.mixed = mixed
        # every running sequence rides in a prompt chunk ("all", budget permitting) or only
        # the chunk's last 64-row tile's free rows ("tile"): ENGINE_RIDERS (engine/native_loop)
        self.riders_all = os.environ.get("ENGINE_RIDERS", "all") == "all"
        # after a reply finishes, wait up to this long for the next request before the next
        # step (closed-loop peers resubmit at once; a free slot left for a whole decode
        # chunk costs batch occupancy): ENGINE_ADMIT_WAIT_US, default 500 us
        self.admit_wait_s = float(os.environ.get("ENGINE_ADMIT_WAIT_US", "500")) * 1e-6
        # prefill-first: while prompts still wait after a prefill step (a burst larger than
        # one step's prefill budget), run the next prefill before decoding the running set
        # (their next tokens wait one prefill; the burst's last first token does not wait
        # for decode chunks): ENGINE_PREFILL_FIRST, default on
        self.prefill_first = os.environ.get("ENGINE_PREFILL_FIRST", "1") != "0"
        self.default_max_tokens = default_max_tokens
        # per-request deadline (s): the reference UI bounds the co-pilot call at 60 s
        # (`web/streamlit_app.py:95`); past it the request is cancelled (KV pages freed at
        # the next step) and the caller gets EngineTimeout.  ENGINE_TIMEOUT=0: no deadline
        self.request_timeout_s = float(os.environ.get("ENGINE_TIMEOUT", "60"))
        # fault injection (SURVEY §5 "stall engine"): the loop sleeps until this time
        # before its next step (stall(); ENGINE_FAULT_STALL_S stalls the first step)
        self._stall_until = time.perf_counter() + float(os.environ.get("ENGINE_FAULT_STALL_S", "0"))
        self.max_ctx = max_ctx or min(engine.cfg.max_pos, CTX_BUCKETS[-1],
                                      engine.kv.num_pages * 64)
        N = load_native()
        self.sched = N.Scheduler(num_pages=engine.kv.num_pages, page_size=64,
                                 max_batch=self.max_batch,
                                 max_prefill_tokens=engine.max_prefill_tokens, max_ctx=self.max_ctx)
        # the scheduler owns page allocation for served requests
        self._lock = threading.Condition()
        self._reqs = {}      # id -> dict(prompt, params, future, t_submit, t_admit, t_first)
        self._pending = []   # (prompt_ids, params, future, t_submit) waiting to enter the scheduler
        self._cancels = set()  # futures whose requests should stop
        self._stop = False
        self._dead = None
        self.errors = 0
        self.stats = {"requests": 0, "tokens": 0, "prefill_tokens": 0, "decode_steps": 0,
                      "busy_s": 0.0, "prefill_s": 0.0, "decode_s": 0.0, "prefill_calls": 0,
                      "decode_calls": 0}
        self._thread = threading.Thread(target=self._loop, name="engine-loop", daemon=True)
        self._thread.start()

    # --------------------------------------------------------------- API
    @staticmethod
    def fatal(e: BaseException) -> bool:
        """Errors after which this engine cannot serve again: a TP/EP peer rank is dead
        (one-shot collective timeout, or the process group's transport broke)."""
        from ..parallel.custom_ar import CollectiveTimeout

        if isinstance(e, CollectiveTimeout):
            return True
        dbe = getattr(torch.distributed, "DistBackendError", None)
        if dbe is not None and isinstance(e, dbe):
            return True
        msg = str(e)
        return any(s in msg for s in ("Connection closed by peer", "Connection reset by peer",
                                      "Broken pipe", "peer rank is dead"))

    @property
    def dead(self):
        """The fatal error that stopped this server (None while healthy)."""
        return self._dead

    def submit(self, prompt_ids: list, params: SamplingParams, on_tokens=None) -> Future:
        """Queue a request.  on_tokens(list[int]) is called from the engine thread with
        every batch of newly generated tokens (streaming), before the future resolves."""
        fut = Future()
        if self._dead is not None:
            fut.set_exception(RuntimeError("engine replica is down: %s" % self._dead))
            return fut
        with self._lock:
            self._pending.append((list(prompt_ids), params, fut, time.perf_counter_ns(),
                                  on_tokens))
            self._lock.notify()
        return fut

    def cancel(self, fut: Future):
        """Stop a request early (e.g. its streaming client went away); its KV pages are
        freed at the next engine step and the future resolves with done_reason
        "cancelled"."""
        with self._lock:
            self._cancels.add(fut)
            self._lock.notify()

    def generate(self, prompt_ids, params: SamplingParams, timeout: float | None = None) -> dict:
        """Blocking request with the engine deadline (``timeout`` s, default
        ENGINE_TIMEOUT): on expiry the request is cancelled and EngineTimeout raised."""
        t = self.request_timeout_s if timeout is None else float(timeout)
        fut = self.submit(prompt_ids, params)
        try:
            return fut.result(t if t > 0 else None)
        except FutureTimeout:
            self.cancel(fut)
            raise EngineTimeout("engine did not answer within %gs (request cancelled)" % t) \
                from None

    def stall(self, seconds: float):
        """Fault injection: the engine loop takes no step for ``seconds`` (tests of the
        request deadline; a hung GPU looks like this from the HTTP side)."""
        with self._lock:
            self._stall_until = time.perf_counter() + float(seconds)
            self._lock.notify()

    def close(self):
        with self._lock:
            self._stop = True
            self._lock.notify()
        self._thread.join(timeout=10)

    def metrics(self) -> dict:
        s = dict(self.stats)
        s["running"] = self.sched.n_running
        s["waiting"] = self.sched.n_waiting + len(self._pending)
        s["free_kv_pages"] = self.sched.free_pages
        return s

    def handle_json(self, req_text: str) -> str:
        """Ollama-compatible generate/chat handler (installed as the node's hook)."""
        req = json.loads(req_text)
        if req.get("endpoint") == "metrics":
            return json.dumps(self.metrics())
        params = SamplingParams.from_ollama(req.get("options"), self.default_max_tokens)
        if req.get("endpoint") == "chat":
            ids = self.tok.chat_messages_ids(req.get("messages") or [])
        elif req.get("raw"):
            ids = self.tok.encode(req.get("prompt", ""), bos=True)
        else:
            ids = self.tok.chat_ids(req.get("prompt", ""))
        r = self.generate(ids, params)
        text = self.tok.decode(r["tokens"])
        now = time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime()) + ".000000Z"
        out = {"model": req.get("model", self.model_name), "created_at": now, "done": True,
               "done_reason": r["done_reason"], "total_duration": r["total_duration"],
               "load_duration": 0, "prompt_eval_count": r["prompt_eval_count"],
               "prompt_eval_duration": r["prompt_eval_duration"], "eval_count": r["eval_count"],
               "eval_duration": r["eval_duration"]}
        if req.get("endpoint") == "chat":
            out["message"] = {"role": "assistant", "content": text}
        else:
            out["response"] = text
            out["context"] = []
        return json.dumps(out)

    def handle_json_stream(self, req_text: str, emit) -> str:
        """Ollama streaming (NDJSON): emit(chunk_json_text) -> bool per token batch;
        returns the final ``done: true`` object (stats, empty response)."""
        import queue

        req = json.loads(req_text)
        params = SamplingParams.from_ollama(req.get("options"), self.default_max_tokens)
        chat = req.get("endpoint") == "chat"
        if chat:
            ids = self.tok.chat_messages_ids(req.get("messages") or [])
        elif req.get("raw"):
            ids = self.tok.encode(req.get("prompt", ""), bos=True)
        else:
            ids = self.tok.chat_ids(req.get("prompt", ""))
        q = queue.Queue()
        fut = self.submit(ids, params, on_tokens=q.put)
        t_lim = self.request_timeout_s
        deadline = time.perf_counter() + t_lim if t_lim > 0 else None
        model = req.get("model", self.model_name)
        toks, text_sent, alive = [], "", True

        def now():
            return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime()) + ".000000Z"

        def flush(final=False):
            nonlocal text_sent, alive
            text = self.tok.decode(toks)
            if not final and text.endswith("\ufffd"):
                return  # incomplete UTF-8 sequence: wait for the next token
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
            if not alive:  # client disconnected: stop generating for it
                self.cancel(fut)

        while True:
            try:
                toks += q.get(timeout=0.05)
                flush()
            except queue.Empty:
                if fut.done() and q.empty():
                    break
                if deadline is not None and time.perf_counter() > deadline:
                    self.cancel(fut)
                    raise EngineTimeout("engine did not answer within %gs (request "
                                        "cancelled)" % t_lim)
        r = fut.result()
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

    # --------------------------------------------------------------- loop
    def _admit_pending(self):
        with self._lock:
            pend, self._pending = self._pending, []
        for prompt, params, fut, t0, cb in pend:
            try:
                rid = self.sched.add(len(prompt), params.max_tokens, params.stop_on_eos,
                                     list(self.engine.cfg.eos_ids))
            except Exception as e:  # too long / bad request
                fut.set_exception(e)
                continue
            self._reqs[rid] = {"prompt": prompt, "params": params, "future": fut, "t_submit": t0,
                               "cb": cb, "streamed": 0}

    def _stream(self, rids):
        """Hand newly accepted tokens of streaming requests to their callbacks."""
        for rid in rids:
            r = self._reqs.get(rid)
            if r is None or r["cb"] is None:
                continue
            toks = list(self.sched.get(rid).tokens)
            if len(toks) > r["streamed"]:
                new = toks[r["streamed"]:]
                r["streamed"] = len(toks)
                try:
                    r["cb"](new)
                except Exception:  # a broken consumer must not stop the engine
                    r["cb"] = None

    def _loop(self):
        eng = self.engine
        while True:
            with self._lock:
                while (not self._stop and not self._pending and self.sched.n_running == 0
                       and self.sched.n_waiting == 0):
                    self._lock.wait(timeout=0.5)
                if self._stop:
                    break
                while not self._stop and time.perf_counter() < self._stall_until:
                    self._lock.wait(timeout=min(0.05, self._stall_until - time.perf_counter()))
                if self._stop:
                    break
            t_busy = time.perf_counter()
            try:
                self._step(eng)
            except Exception as e:  # fail every in-flight request, keep serving
                for rid, r in list(self._reqs.items()):
                    if not r["future"].done():
                        r["future"].set_exception(e)
                    self.sched.cancel(rid)
                for rid in self.sched.take_finished():
                    self.sched.release(rid)  # scheduler entries + KV pages
                self._reqs.clear()
                self.errors += 1
                if self.fatal(e):  # a TP peer is gone: this replica cannot serve again
                    self._dead = e
                    break
            self.stats["busy_s"] += time.perf_counter() - t_busy
        if self._dead is not None:  # nothing queued may wait forever on a dead replica
            with self._lock:
                pend, self._pending = self._pending, []
            for _p, _params, fut, _t, _cb in pend:
                if not fut.done():
                    fut.set_exception(RuntimeError("engine replica is down: %s" % self._dead))

    def _apply_cancels(self):
        with self._lock:
            cancels, self._cancels = self._cancels, set()
        if not cancels:
            return
        for rid, r in list(self._reqs.items()):
            if r["future"] in cancels:
                self.sched.cancel(rid)

    def _step(self, eng: Engine):
        self._admit_pending()
        self._apply_cancels()
        plan = self.sched.schedule()
        if plan.prefill:
            prompts = [self._reqs[i]["prompt"] for i in plan.prefill]
            pages = [list(self.sched.get(i).pages) for i in plan.prefill]
            ride = [i for i in plan.decode if self.sched.get(i).state == 1] if self.mixed else []
            # riders: every running sequence (within the chunk budget), or only the rows left
            # in the prefill's last 64-row GEMM tile
            n_rows = sum(len(p) for p in prompts)
            room = (eng.max_prefill_tokens - n_rows if self.riders_all
                    else -(-n_rows // 64) * 64 - n_rows)
            ride = ride[:max(0, room)]
            starts = [0] * len(prompts)
            for i in ride:  # running sequences: one decode row each (last token at r.pos)
                r = self.sched.get(i)
                prompts.append(_RiderRow(r.pos, r.tokens[-1]))
                pages.append(list(r.pages))
                starts.append(r.pos)
            ids = list(plan.prefill) + ride
            t0 = time.perf_counter_ns()
            for i in plan.prefill:
                self._reqs[i]["t_admit"] = t0
            with span("server.prefill", batch=len(plan.prefill), decode_rows=len(ride)):
                first = eng.prefill(prompts, pages, sampling=[self._reqs[i]["params"] for i in ids],
                                    starts=starts if ride else None).cpu().tolist()
            eng.check_comm()
            t1 = time.perf_counter_ns()
            self.stats["prefill_s"] += (t1 - t0) * 1e-9
            self.stats["prefill_calls"] += 1
            self.stats["prefill_tokens"] += sum(len(self._reqs[i]["prompt"]) for i in plan.prefill)
            for i, tkn in zip(plan.prefill, first):
                self._reqs[i]["t_first"] = t1
                self.sched.on_first_token(i, int(tkn))
            if ride:
                self.sched.on_decode_tokens(ride, [[int(t)] for t in first[len(plan.prefill):]])
                self.stats["decode_steps"] += 1
            self._stream(ids)
        running = [i for i in list(plan.decode) + list(plan.prefill)
                   if self.sched.get(i).state == 1]
        if plan.prefill and self.prefill_first and self.sched.n_waiting > 0:
            running = []  # the rest of the burst first (see prefill_first)
        if running:
            self._decode(eng, running)
        done = self._retire()
        free = self.max_batch - self.sched.n_running - self.sched.n_waiting
        if done and free > 0 and self.admit_wait_s > 0:
            # replies just went out: their peers (or queued clients) usually send the next
            # requests within a fraction of a millisecond -- admit them at THIS step
            # boundary instead of leaving their batch slots idle for a whole step.  Wait
            # (bounded) until as many requests are pending as replies were sent, capped by
            # the free slots (already-queued requests fill slots first; with no free slot
            # an arrival could not be admitted anyway, so the running batch never waits)
            want = min(done, free)
            deadline = time.perf_counter() + self.admit_wait_s
            with self._lock:
                while len(self._pending) < want and not self._stop:
                    left = deadline - time.perf_counter()
                    if left <= 0:
                        break
                    self._lock.wait(timeout=left)

    def _decode(self, eng: Engine, running: list):
        reqs = [self.sched.get(i) for i in running]
        params = [self._reqs[i]["params"] for i in running]
        ctx = max(r.prompt_len + r.max_new for r in reqs)
        remaining = min(r.max_new - len(r.tokens) for r in reqs)
        waiting = self.sched.n_waiting + len(self._pending)
        # chunk length: long chunks amortise the host round trip; a waiting request or a
        # free batch slot (a request may arrive any moment) shortens it to bound TTFT
        chunk = self.decode_chunk
        if waiting:
            chunk = 2
        elif len(running) < self.max_batch:
            chunk = max(2, self.decode_chunk // 2)
        k = max(1, min(chunk, remaining))
        t0 = time.perf_counter()
        with span("server.decode", batch=len(running), steps=k):
            hist = eng.decode_steps([r.tokens[-1] for r in reqs], [r.pos for r in reqs],
                                    [list(r.pages) for r in reqs], ctx, k, params)
        self.stats["decode_s"] += time.perf_counter() - t0
        self.stats["decode_calls"] += 1
        self.stats["decode_steps"] += k
        self.sched.on_decode_tokens(running, hist)
        self._stream(running)

    def _retire(self) -> int:
        now = time.perf_counter_ns()
        done = 0
        for rid in self.sched.take_finished():
            done += 1
            self._stream([rid])
            r = self._reqs.pop(rid, None)
            sr = self.sched.get(rid)
            if r is not None and not r["future"].done():
                t_first = r.get("t_first", now)
                toks = list(sr.tokens)
                self.stats["requests"] += 1
                self.stats["tokens"] += len(toks)
                r["future"].set_result({
                    "tokens": toks, "done_reason": sr.finish_reason or "stop",
                    "prompt_eval_count": sr.prompt_len,
                    "prompt_eval_duration": t_first - r.get("t_admit", r["t_submit"]),
                    "eval_count": len(toks), "eval_duration": now - t_first,
                    "total_duration": now - r["t_submit"],
                    "ttft_ns": t_first - r["t_submit"]})
            self.sched.release(rid)
        return done
