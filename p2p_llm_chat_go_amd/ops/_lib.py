"""ctypes binding of the gfx950 kernel library (``_lib/libp2p_kernels.so``).

The kernels take raw device pointers and the caller's HIP stream, so every
launch lands on ``torch.cuda.current_stream()`` and is captured by
``torch.cuda.graph`` (hipGraph) like any other work on that stream.

torch must be imported first: it brings its own ``libamdhip64.so.7`` and the
kernel library resolves against that already-loaded runtime (same soname),
so there is exactly one HIP runtime in the process.

On a machine with a GPU the library is mandatory: ``lib()`` raises if it is
missing or fails to load (no silent eager fallback).  CPU tensors never reach
this module (ops dispatch CPU tensors to their PyTorch reference path).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib",
                         "libp2p_kernels.so")
_lock = threading.Lock()
_lib = None

c_int = ctypes.c_int
c_float = ctypes.c_float
c_void_p = ctypes.c_void_p

_SIGS = {
    # name: argtypes (all return int hipError_t)
    "p2p_skinny_gemm": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                        c_int, c_float, c_int, c_void_p, c_void_p],
    "p2p_paged_attention": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                            c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_int,
                            c_void_p, c_void_p, c_void_p],
    "p2p_flash_prefill": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                          c_int, c_int, c_int, c_float, c_void_p, c_int, c_void_p],
    "p2p_flash_prefill2": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                           c_int, c_int, c_int, c_float, c_void_p, c_int, c_void_p],
    "p2p_flash_prefill_tile": [c_int, c_int],
    "p2p_tall_silu": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_float,
                      c_void_p],
    "p2p_tall_silu_ok": [c_int, c_int, c_int],
    "p2p_car_alloc": [ctypes.c_size_t, c_void_p],
    "p2p_car_free": [c_void_p],
    "p2p_car_get_handle": [c_void_p, c_void_p],
    "p2p_car_open_handle": [c_void_p, c_void_p],
    "p2p_car_close_handle": [c_void_p],
    "p2p_car_handle_size": [],
    "p2p_car_allreduce_add": [c_void_p, c_int, c_int, ctypes.c_size_t, c_void_p, c_void_p, c_int,
                              c_void_p, c_void_p, c_int, c_void_p],
    "p2p_car_allreduce_add_2shot": [c_void_p, c_int, c_int, ctypes.c_size_t, c_void_p, c_void_p,
                                    c_int, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_car_allreduce_max_u64": [c_void_p, c_int, c_int, ctypes.c_size_t, c_void_p, c_void_p,
                                  c_int, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_car_all_gather": [c_void_p, c_int, c_int, ctypes.c_size_t, c_void_p, c_void_p,
                           ctypes.c_longlong, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_car_set_timeout_ms": [c_int],
    "p2p_qkv_attn": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_float, c_void_p,
                     c_int, c_float, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_qkv_attn_oproj_fits": [c_int, c_int, c_int, c_int, c_int],
    "p2p_qkv_attn_oproj": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                           c_float, c_float, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                           c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "p2p_skinny_gemm_ar": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                           c_void_p, c_int, c_int, ctypes.c_size_t, c_void_p, c_void_p, c_int,
                           c_void_p, c_void_p],
    "p2p_attn_oproj": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                       c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_int, c_void_p,
                       c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "p2p_attn_oproj_heads": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                             c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_int,
                             c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_attn_oproj_heads_tune": [c_int],
    "p2p_paged_attention_mfma": [c_int],
    "p2p_l3_prefetch": [c_void_p, ctypes.c_size_t, c_int, c_void_p, c_void_p],
    "p2p_gather_rows": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p],
    "p2p_pack_frag": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "p2p_rope_cache": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                       c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "p2p_argmax": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "p2p_advance": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                    c_int, c_void_p, c_int, c_void_p],
    "p2p_argmax_finalize": [c_void_p, c_void_p, c_int, c_void_p],
    "p2p_skinny_gemm_argmax": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                               c_float, c_int, c_void_p, c_void_p],
    "p2p_skinny_gemm_qkv_rope": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_float,
                                 c_int, c_void_p, c_void_p],
    "p2p_sample": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                   c_void_p, c_void_p],
    "p2p_topk_candidates": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "p2p_sample_candidates": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p],
    "p2p_tiled_gemm": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                       c_int, c_float, c_void_p],
    "p2p_tiled_gemm_qkv_rope": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_float,
                                c_void_p],
    "p2p_tiled_gemm_argmax": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                              c_float, c_void_p],
    "p2p_grouped_gemm": [c_void_p, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_int, c_int,
                         c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                         c_int, c_float, c_int, c_void_p],
    "p2p_moe_route": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                      c_void_p, c_void_p, c_int, c_void_p],
    "p2p_moe_router_route": [c_void_p, c_int, c_int, c_int, c_void_p, c_float, c_int, c_int, c_int,
                             c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_moe_a2a_dispatch": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                             c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p],
    "p2p_moe_a2a_group": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_moe_a2a_combine": [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p],
    "p2p_moe_router_logits": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_float, c_void_p,
                              c_int, c_void_p],
    "p2p_moe_combine": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                        c_int, c_int, c_void_p],
    "p2p_persist_gemv_ok": [c_int, c_int, c_int, c_int],
    # persistent decode engine (decode_engine.hip)
    "p2p_decode_engine_ok": [c_int, c_int, c_int, c_int, c_int, c_int],
    "p2p_decode_engine_grid": [c_int, c_int, c_int],
    "p2p_decode_engine_trace": [c_void_p],
    "p2p_decode_engine": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                          c_float, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    # expert-parallel all-to-all over IPC peer buffers (ep_a2a.hip)
    "p2p_ep_set_timeout_ms": [c_int],
    "p2p_ep_dispatch": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                        c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_ep_recv": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                    c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "p2p_ep_return": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                      c_int, c_void_p],
    "p2p_ep_combine": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                       c_int, c_void_p, c_void_p, c_int, c_void_p],
}


class KernelError(RuntimeError):
    pass


def check_stamp(path: str, experimental: bool = False) -> None:
    """Refuse a library that no build of the current sources produced: ``_build`` records a
    digest of the sources and headers next to the library (``<lib>.stamp``); a mismatch
    means the binary is stale (an edited kernel that was never rebuilt, or a copy pushed
    from elsewhere).  Skipped where the sources are not present; P2P_ALLOW_STALE_LIB=1
    downgrades the error to a warning."""
    from .. import _build

    srcs, hdrs = _build.kernel_sources(experimental)
    if not srcs:
        return  # installed without csrc/: nothing to compare against
    why = None
    try:
        import json

        with open(path + ".stamp") as f:
            rec = json.load(f)
        if rec.get("sources_sha256") != _build.sources_digest(srcs + hdrs):
            why = "was built from different sources than the tree's csrc/"
    except FileNotFoundError:
        why = "has no build stamp (%s.stamp)" % os.path.basename(path)
    if why is None:
        return
    msg = ("%s %s -- rebuild with `python -m p2p_llm_chat_go_amd._build`" % (path, why))
    if os.environ.get("P2P_ALLOW_STALE_LIB", "0") == "1":
        import warnings

        warnings.warn(msg)
        return
    raise KernelError(msg)


def lib_path() -> str:
    return _LIB_PATH


def lib():
    """Load (once) and return the kernel library; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise KernelError(
                "HIP kernel library missing at %s -- run `python -m p2p_llm_chat_go_amd._build` "
                "(or __graft_entry__.build())" % _LIB_PATH)
        check_stamp(_LIB_PATH)
        L = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name in ("p2p_car_buffer_bytes", "p2p_far_buffer_bytes"):
            fn = getattr(L, name, None)
            if fn is not None:
                fn.argtypes = [ctypes.c_size_t]
                fn.restype = ctypes.c_size_t
        fn = getattr(L, "p2p_ep_buffer_bytes", None)
        if fn is not None:
            fn.argtypes = [c_int, c_int]
            fn.restype = ctypes.c_size_t
        fn = getattr(L, "p2p_tiled_gemm_config", None)
        if fn is not None:
            fn.argtypes = [c_int, c_int, c_int]
            fn.restype = None
        fn = getattr(L, "p2p_tiled_split_parallel", None)
        if fn is not None:
            fn.argtypes = [c_int]
            fn.restype = None
        fn = getattr(L, "p2p_tiled_split_fault", None)
        if fn is not None:
            fn.argtypes = []
            fn.restype = c_int
        for name in ("p2p_prefill_phased", "p2p_prefill_deep", "p2p_prefill_pre_rstd",
                     "p2p_prefill_tile8"):
            fn = getattr(L, name, None)
            if fn is not None:
                fn.argtypes = [c_int]
                fn.restype = None
        fn = getattr(L, "p2p_qkv_attn_probe", None)
        if fn is not None:
            fn.argtypes = [c_int]
            fn.restype = None
        fn = getattr(L, "p2p_skinny_gemm_tune", None)
        if fn is not None:
            fn.argtypes = [c_int, c_int]
            fn.restype = None
        for name, args in _SIGS.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = c_int
        _lib = L
        return _lib


_EXP_PATH = os.path.join(os.path.dirname(_LIB_PATH), "libp2p_experimental.so")
_exp = None

# experimental library (csrc/experimental: measured-negative fusions, hardware probes)
_EXP_SIGS = ("p2p_attn_oproj", "p2p_attn_oproj_heads", "p2p_attn_oproj_heads_tune",
             "p2p_l3_prefetch", "p2p_persist_gemv_ok", "p2p_decode_engine_ok",
             "p2p_decode_engine_grid", "p2p_decode_engine_trace", "p2p_decode_engine",
             "p2p_tall_silu", "p2p_tall_silu_ok")


def experimental():
    """The opt-in library of measured-negative kernels and probes (built by
    ``python -m p2p_llm_chat_go_amd._build --only experimental``); raises if absent."""
    global _exp
    if _exp is not None:
        return _exp
    lib()  # the main library first (same HIP runtime)
    with _lock:
        if _exp is None:
            if not os.path.exists(_EXP_PATH):
                raise KernelError(
                    "experimental kernel library missing at %s -- build it with "
                    "`python -m p2p_llm_chat_go_amd._build --only experimental`" % _EXP_PATH)
            check_stamp(_EXP_PATH, experimental=True)
            L = ctypes.CDLL(_EXP_PATH, mode=ctypes.RTLD_GLOBAL)
            for name in _EXP_SIGS:
                fn = getattr(L, name, None)
                if fn is not None:
                    fn.argtypes = _SIGS[name]
                    fn.restype = c_int
            fn = getattr(L, "p2p_decode_engine_ws_bytes", None)
            if fn is not None:
                fn.argtypes = [c_int, c_int, c_int, c_int, c_int]
                fn.restype = ctypes.c_size_t
            _exp = L
    return _exp


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def check(err: int, name: str):
    if err != 0:
        raise KernelError("%s failed with hipError %d" % (name, err))


def ptr(t):
    return None if t is None else t.data_ptr()
