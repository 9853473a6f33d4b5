"""Hot ops of the engine: hand-written gfx950 HIP kernels behind thin wrappers.

CUDA (HIP) tensors always run the native kernels (the library must be built;
a missing library raises).  CPU tensors run the PyTorch reference of the same
math -- that is the CPU tiny-llama plumbing config and the numerics oracle,
never a fallback for GPU tensors.
"""
from .gemm import (EPI_AR, EPI_F32, EPI_RESID, EPI_SILU, EPI_STORE, Fp8Weight, skinny_ar_ok,
                   skinny_gemm_ar, argmax_finalize, fold_norm,
                   quantize_fp8,
                   lm_head_argmax, new_argmax_keys, qkv_rope_gemm, rope_row_perm, skinny_gemm, tile_weight,
                   tiled_shape, tiled_split_fault, tiled_split_parallel, untile_weight)
from .attention import (PAGE, HEAD_DIM, attn_oproj, attn_oproj_ok, attn_oproj_heads,
                        attn_oproj_heads_ok, attn_oproj_heads_workspace, attn_workspace,
                        flash_prefill, flash_tile, paged_attention, prefill_tiles, rope_cache,
                        qkv_attn, qkv_attn_ok, qkv_attn_oproj_ok, qkv_attn_workspace)
from .elementwise import advance, argmax, gather_rows, l3_prefetch
from .sampling import sample, sample_candidates, topk_candidates
from ._lib import available as kernels_available, lib as kernel_lib, lib_path as kernel_lib_path

__all__ = [
    "EPI_AR", "skinny_ar_ok", "skinny_gemm_ar", "EPI_F32", "EPI_RESID", "EPI_SILU", "EPI_STORE", "fold_norm", "skinny_gemm", "tile_weight",
    "tiled_shape", "untile_weight", "argmax_finalize", "lm_head_argmax", "new_argmax_keys", "qkv_rope_gemm",
    "rope_row_perm", "PAGE", "HEAD_DIM", "attn_workspace", "paged_attention", "flash_prefill", "flash_tile", "prefill_tiles",
    "attn_oproj", "attn_oproj_ok", "attn_oproj_heads", "attn_oproj_heads_ok",
    "attn_oproj_heads_workspace", "tiled_split_fault", "tiled_split_parallel", "l3_prefetch",
    "rope_cache", "qkv_attn", "qkv_attn_ok", "qkv_attn_oproj_ok", "qkv_attn_workspace", "sample", "sample_candidates", "topk_candidates", "advance", "argmax", "gather_rows", "kernels_available", "kernel_lib",
    "kernel_lib_path",
]
