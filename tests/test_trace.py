"""Tracing spans (utils/trace.py): engine phases are recorded and exported as
Chrome-trace JSON; roctx is loadable on this image (ranges are no-ops without
a profiler attached)."""
import json

from p2p_llm_chat_go_amd.utils import trace


def test_engine_spans_recorded(tmp_path):
    from p2p_llm_chat_go_amd.engine import Engine
    from p2p_llm_chat_go_amd.models import TINY_LLAMA

    rec = trace.enable(roctx=True, record=True)
    try:
        eng = Engine(TINY_LLAMA, device="cpu", kv_pages=16, use_graph=False)
        eng.generate([[1, 2, 3, 4]], 5, stop_on_eos=False)
        summ = rec.summary()
        assert summ["prefill"]["count"] == 1
        assert summ["decode"]["count"] >= 1
        path = tmp_path / "t.json"
        rec.dump(str(path))
        ev = json.load(open(path))["traceEvents"]
        assert {e["name"] for e in ev} >= {"prefill", "decode"}
        assert all(e["ph"] == "X" and e["dur"] >= 0 for e in ev)
    finally:
        trace.disable()


def test_span_disabled_is_noop():
    trace.disable()
    with trace.span("x"):
        pass
    trace.mark("m")
