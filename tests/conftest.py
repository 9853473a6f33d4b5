import ctypes
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    # device_count() does not initialise the HIP runtime (is_available() does): a pytest
    # parent that only spawns rank processes (tests/test_world8_gpu.py) then holds no GPU
    # context of its own, so 8 virtual ranks are the only 8 processes on the device
    if torch.cuda.device_count() > 0:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


ENGINE_LIB = os.path.join(ROOT, "p2p_llm_chat_go_amd", "_lib", "libp2p_engine.so")


@pytest.fixture(scope="module")
def probe():
    """The engine C ABI's tokenizer probe: (native spec, Ollama request, ids) -> its
    {"native", "ids", "text"} (tests of csrc/engine/native_tok.h and bpe_tok.h)."""
    if not os.path.exists(ENGINE_LIB):
        pytest.skip("engine C ABI not built")
    L = ctypes.CDLL(ENGINE_LIB)
    L.p2p_engine_tok_probe.restype = ctypes.c_void_p
    L.p2p_engine_tok_probe.argtypes = [ctypes.c_char_p] * 3
    L.p2p_engine_free.argtypes = [ctypes.c_void_p]

    def run(spec, req, ids=()):
        p = L.p2p_engine_tok_probe(json.dumps(spec).encode(), json.dumps(req).encode(),
                                   json.dumps(list(ids)).encode())
        assert p, "probe failed"
        out = json.loads(ctypes.string_at(p).decode())
        L.p2p_engine_free(p)
        return out
    return run
