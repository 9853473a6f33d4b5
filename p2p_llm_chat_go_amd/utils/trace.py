"""Tracing: roctx ranges for rocprofv3 + an in-process span recorder.

SURVEY.md §5 "Tracing / profiling": the reference has none (Ollama's timing
fields are dropped, `web/streamlit_app.py:97-98`).  Two layers here:

* ``span(name)`` pushes/pops a roctx range (``librocprofiler-sdk-roctx``), so
  ``rocprofv3 --marker-trace`` shows the engine phases (prefill chunk, decode
  graph replay, collectives) on the same timeline as the kernels.  Enabled
  with ``P2P_ROCTX=1`` (a ctypes call costs ~1 us, so it is off by default).
* ``Recorder`` keeps host-side spans and exports Chrome-trace JSON
  (``P2P_TRACE=/path/trace.json`` records every span and writes at exit);
  EngineServer also uses it for per-request queue / prefill / decode timing.
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import json
import os
import threading
import time

_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"):
        for d in ("", "/opt/rocm/lib/"):
            try:
                lib = ctypes.CDLL(d + name)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.restype = None
            _roctx = lib
            return _roctx
    return None


class Recorder:
    """Thread-safe span store; ``to_chrome()`` -> Chrome trace event list."""

    def __init__(self, limit: int = 1_000_000):
        self.events = []
        self.limit = limit
        self._lock = threading.Lock()
        self._t0 = time.perf_counter_ns()

    def add(self, name: str, start_ns: int, end_ns: int, **args):
        with self._lock:
            if len(self.events) < self.limit:
                self.events.append((name, start_ns, end_ns, threading.get_ident(), args))

    def to_chrome(self) -> list:
        pid = os.getpid()
        out = []
        with self._lock:
            for name, s, e, tid, args in self.events:
                out.append({"name": name, "ph": "X", "pid": pid, "tid": tid,
                            "ts": (s - self._t0) / 1000.0, "dur": (e - s) / 1000.0,
                            "args": args})
        return out

    def dump(self, path: str):
        with open(path, "w") as f:
            json.dump({"traceEvents": self.to_chrome()}, f)

    def summary(self) -> dict:
        """name -> {count, total_ms, mean_ms}."""
        agg = {}
        with self._lock:
            for name, s, e, _tid, _a in self.events:
                c, t = agg.get(name, (0, 0))
                agg[name] = (c + 1, t + (e - s))
        return {k: {"count": c, "total_ms": t / 1e6, "mean_ms": t / 1e6 / c}
                for k, (c, t) in agg.items()}


_ENABLED_ROCTX = os.environ.get("P2P_ROCTX", "0") == "1"
_TRACE_PATH = os.environ.get("P2P_TRACE")
recorder = Recorder() if _TRACE_PATH else None
if recorder is not None:
    atexit.register(lambda: recorder.dump(_TRACE_PATH))


def enable(roctx: bool = True, record: bool = True):
    """Turn tracing on at runtime (tests / benches)."""
    global _ENABLED_ROCTX, recorder
    _ENABLED_ROCTX = roctx
    if record and recorder is None:
        recorder = Recorder()
    return recorder


def disable():
    global _ENABLED_ROCTX, recorder
    _ENABLED_ROCTX = False
    recorder = None


@contextlib.contextmanager
def span(name: str, **args):
    lib = _load_roctx() if _ENABLED_ROCTX else None
    rec = recorder
    if lib is None and rec is None:
        yield
        return
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
        if rec is not None:
            rec.add(name, t0, time.perf_counter_ns(), **args)


def mark(name: str):
    lib = _load_roctx() if _ENABLED_ROCTX else None
    if lib is not None:
        lib.roctxMarkA(name.encode())
