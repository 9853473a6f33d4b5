"""Loader for the C++ module ``_lib/_native*.so`` (chat plane + engine runtime).

Build it with ``python -m p2p_llm_chat_go_amd._build --only native`` (or
``__graft_entry__.build()``).  ``load()`` raises with that hint if it is missing.
"""
from __future__ import annotations

import importlib.util
import os
import sys

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    for f in sorted(os.listdir(_LIBDIR)) if os.path.isdir(_LIBDIR) else []:
        if f.startswith("_native") and f.endswith(".so"):
            spec = importlib.util.spec_from_file_location("p2p_llm_chat_go_amd._native",
                                                          os.path.join(_LIBDIR, f))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["p2p_llm_chat_go_amd._native"] = mod
            _mod = mod
            return mod
    raise ImportError("native module not built: run `python -m p2p_llm_chat_go_amd._build`")


def available() -> bool:
    try:
        load()
        return True
    except ImportError:
        return False


def bin_path(name: str) -> str:
    """Path of a built daemon (p2p-node, p2p-directory, p2p-relay)."""
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", name)
