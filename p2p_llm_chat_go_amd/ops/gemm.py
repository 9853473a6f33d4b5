"""Projection GEMMs on the fragment-major weight layout.

Weights are stored once, at load time, in the layout the MFMA B operand wants
(``csrc/kernels/skinny_gemm.hip`` header): a ``[N/16, K/32, 64, 8]`` bf16
tensor where tile ``[g, s]`` is exactly what the 64 lanes of a wave hold for
``v_mfma_f32_16x16x32_bf16``.  The decode weight stream is then one contiguous
1 KiB load per wave per k-step.

GPU tensors run the HIP kernels (mandatory); CPU tensors run the PyTorch
reference of the same math (used by the tiny-llama CPU config and as the
numerics oracle in tests).
"""
from __future__ import annotations

import os

import torch

from . import _lib

EPI_STORE, EPI_RESID, EPI_SILU, EPI_F32 = 0, 1, 2, 3
EPI_QKV_ROPE, EPI_ARGMAX = 4, 5
EPI_AR = 6  # TP row-parallel projection + fused all-reduce + residual (skinny_gemm_ar)
SKINNY_MAX_M = 64

# Autotuned launch codes: (N, K, epi, norm, m_tile[, "fp8"]) -> waves | (U << 8)
# (engine/autotune.py)
_TUNE: dict = {}

FP8_MAX = 448.0  # OCP e4m3 (the gfx950 format; torch.float8_e4m3fn)


class Fp8Weight:
    """Weight-only FP8 projection: e4m3 codes in the fragment-major order of
    ``tile_weight`` with k-steps interleaved in pairs (uint8 ``[N/16, K/32, 64, 8]``, see
    ``pair_f8``: each lane's 16-byte load holds its codes of two consecutive k-steps, so
    a wave still moves 1 KiB per load instruction, as in bf16) and a per-output-channel
    fp32 scale ``[N]``.  The skinny GEMM widens the codes to bf16 in registers and applies
    the scale in its epilogue."""

    def __init__(self, data: torch.Tensor, scale: torch.Tensor):
        self.data = data
        self.scale = scale

    @property
    def shape(self):
        return self.data.shape

    @property
    def device(self):
        return self.data.device

    def numel(self):
        return self.data.numel()

    def to(self, device):
        return Fp8Weight(self.data.to(device), self.scale.to(device))

    def element_size(self):
        return 1

    def dequantize_f32(self) -> torch.Tensor:
        """Exact fp32 [N, K] (natural layout) values the kernel multiplies with."""
        q = untile_weight(unpair_f8(self.data).view(torch.float8_e4m3fn)).float()
        return q * self.scale.float()[:, None].to(q.device)

    def dequantize(self) -> torch.Tensor:
        """bf16 fragment-major weight with (bf16-rounded) same values (CPU reference)."""
        return tile_weight(self.dequantize_f32().to(torch.bfloat16))


def quantize_fp8(wt: torch.Tensor) -> Fp8Weight:
    """bf16 fragment-major weight -> Fp8Weight (per-output-channel absmax scaling)."""
    w = untile_weight(wt).float()
    assert w.shape[1] % 64 == 0, "fp8 weights need K % 64 == 0 (k-step pairs)"
    amax = w.abs().amax(dim=1).clamp_min(1e-12)
    scale = amax / FP8_MAX
    q = (w / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return Fp8Weight(pair_f8(tile_weight(q.view(torch.uint8))), scale.float().contiguous())


def pair_f8(t: torch.Tensor) -> torch.Tensor:
    """Fragment-major 1-byte codes [G, S, 64, 8] -> k-step pairs: [G, S/2, lane, (2, 8)],
    i.e. lane l's 16 bytes at pair p are its fragments of k-steps 2p and 2p+1."""
    G, S = t.shape[0], t.shape[1]
    return t.reshape(G, S // 2, 2, 64, 8).transpose(2, 3).contiguous().reshape(G, S, 64, 8)


def unpair_f8(t: torch.Tensor) -> torch.Tensor:
    G, S = t.shape[0], t.shape[1]
    return t.reshape(G, S // 2, 64, 2, 8).transpose(2, 3).contiguous().reshape(G, S, 64, 8)


def _is_f8(wt) -> bool:
    return isinstance(wt, Fp8Weight)


def _wptr(wt):
    return (wt.data.data_ptr(), wt.scale.data_ptr()) if _is_f8(wt) else (wt.data_ptr(), None)


def m_tile(M: int) -> int:
    """Autotune bucket of M: 16-row MFMA tiles (1..4).  The skinny kernel runs 3 tiles as
    4; the midm / tiled kernels use the exact count, so 33-48 rows tune separately."""
    return min(4, (max(M, 1) + 15) // 16)


def tune_key(wt, M, epi, norm):
    N, K = tiled_shape(wt)
    key = (N, K, int(epi), bool(norm), m_tile(min(M, SKINNY_MAX_M)))
    return key + ("fp8",) if _is_f8(wt) else key


def set_tune(key, code: int):
    _TUNE[key] = int(code)


TILED_MIN_M = SKINNY_MAX_M + 1  # rows from which the tiled kernel is used (bench override)


def set_tiled_min_m(m: int):
    global TILED_MIN_M
    TILED_MIN_M = int(m)


# the tall SwiGLU kernel (csrc/experimental/tall_gemm.hip: every row of a batched prompt chunk
# in one workgroup, weights streamed once) -- correct but SLOWER than the split-K tiled kernel
# at every height measured (384 rows 152 vs 105 us, 128 rows 89 vs 54;
# profiles/r5_tall_silu_negative.jsonl): opt-in P2P_TALL_SILU=1
TALL_SILU = os.environ.get("P2P_TALL_SILU", "0") == "1"


def tall_silu_ok(M: int, K: int, N: int) -> bool:
    return bool(_lib.experimental().p2p_tall_silu_ok(M, K, N))


def wide_ok(N, K, epi) -> bool:
    """Shapes the wide mid-M kernel tiles: 128 output columns per workgroup (SwiGLU: 64
    gate/up pairs), K in 256-wide chunks."""
    if K % 256:
        return False
    return (N // 2) % 64 == 0 if epi == EPI_SILU else N % 128 == 0


def tiled_ok(N, K, epi) -> bool:
    if K % 64:
        return False
    return (N // 2) % 64 == 0 if epi == EPI_SILU else N % 128 == 0


def use_tiled(M, N, K, epi) -> bool:
    """Prefill-sized M goes to the LDS-tiled MFMA kernel (compute-bound), decode to skinny."""
    return M >= TILED_MIN_M and tiled_ok(N, K, epi)


# launch-code bit: run this (shape, M tile) on the tiled LDS-DMA kernel (autotuned for
# 16 < M <= 64, where the split-K tiled kernel can beat the skinny one)
TILED_FLAG = 1 << 24
# launch-code bit: the mid-M LDS-DMA kernel (csrc/kernels/midm_gemm.h: one column group
# per workgroup over the whole K, activations + weights streamed through an LDS ring);
# bf16 dense weights, K % 128 == 0, M <= 64 (autotuned against skinny / tiled)
MIDM_FLAG = 1 << 25
# launch-code bit: the wide mid-M kernel (csrc/kernels/wide_gemm.hip: 8 waves x 16 columns
# per workgroup share the activation chunks in LDS, each wave streams its own weight group
# into VGPRs, split-K over workgroups); bits 8..15 = K slices (0 = heuristic); bf16 dense
# weights, K % 256 == 0, 1 < M <= 64
WIDE_FLAG = 1 << 26
# with WIDE_FLAG: 16 waves per workgroup (two per column group, k-steps split by parity),
# else 8 -- a weight stream needs 16 waves per CU to reach HBM speed (bench/stream_probe.py)
WIDE16 = 1 << 16
# launch-code bit: the skinny kernel's X is fragment-major (pack_frag), not row-major
AFRAG_FLAG = 1 << 27
# the persistent GEMV (csrc/experimental/persist_gemv.hip, libp2p_experimental.so): one 4-wave workgroup per CU (x the
# multiple in bits 8..15) walking balanced 16-column units with the weight stream carried
# across them; M <= 16, bf16 weights, K % 1024 == 0.  Measured 1.3-1.6x slower than the
# skinny launches (profiles/r4_persist_gemv_negative.jsonl): explicit launch codes only
PERSIST_FLAG = 1 << 28


def persist_ok(M: int, K: int, N: int, epi: int) -> bool:
    return bool(_lib.experimental().p2p_persist_gemv_ok(M, K, N, epi))


_PACK_BUF: dict = {}


def _packed(x: torch.Tensor) -> torch.Tensor:
    """x packed fragment-major into a per-device grow-only buffer (a captured graph keeps
    the address: the buffer is sized at autotune time, before any capture)."""
    M, K = x.shape
    n = (M + 15) // 16 * 16 * K
    buf = _PACK_BUF.get(x.device)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 64 * 16384), device=x.device, dtype=torch.bfloat16)
        _PACK_BUF[x.device] = buf
    out = buf[:n].view((M + 15) // 16 * 16, K)
    return pack_frag(x, out=out)[:M]


def pack_frag(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Row-major [M, K] bf16 -> fragment-major copy (16-row m-tiles of K/32 MFMA A fragments,
    padded rows zero) for the skinny GEMM's AFRAG_FLAG launches: every A-fragment load is
    then 1 KiB contiguous.  Returns a [ceil(M/16)*16, K] buffer (fragment order inside)."""
    M, K = x.shape
    rows = (M + 15) // 16 * 16
    if out is None:
        out = torch.empty(rows, K, device=x.device, dtype=torch.bfloat16)
    if x.device.type != "cuda":
        xp = torch.zeros(rows, K, dtype=x.dtype)
        xp[:M] = x
        out.copy_(xp.reshape(rows // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(rows, K))
        return out
    _lib.check(_lib.lib().p2p_pack_frag(x.data_ptr(), x.stride(0), M, K, out.data_ptr(),
                                        _lib.stream_ptr(x.device)), "pack_frag")
    return out


def _want_tiled(wt, M, N, K, epi, norm, waves) -> bool:
    if _is_f8(wt):  # FP8 weights run on the skinny kernel only (M chunks of 64)
        return False
    if use_tiled(M, N, K, epi):
        return True
    if M > SKINNY_MAX_M or not tiled_ok(N, K, epi):
        return False
    return bool(_code(wt, M, epi, norm, waves) & TILED_FLAG)


def tiled_config(version: int = 2, tile: int = 0, splitk: int = 0):
    """Prefill GEMM selection: version 2 = 8-wave LDS-DMA kernel (tile 0 = heuristic,
    1 = 256x256, 2 = 128x256, 3 = 128x128; splitk 0 = heuristic, 1 = off, n = forced),
    version 1 = register-staged 128x128."""
    _lib.lib().p2p_tiled_gemm_config(int(version), int(tile), int(splitk))


def tiled_split_parallel(on: bool = True):
    """Split-K reduction of the tiled kernel: parallel (every K slice finishes a share of
    its tile; default where the grid fits one block per CU) or serial (the last arriving
    slice reduces the whole tile)."""
    _lib.lib().p2p_tiled_split_parallel(int(bool(on)))


def split_fault_word(device=None) -> int:
    """Device address of the kernels' split-K fault word on the current device (one int,
    allocated on first use and never moved; the wide and tiled split-K GEMMs set it when a
    slice gives up waiting).  The native loop checks it with every graph's own fault word."""
    import ctypes

    L = _lib.lib()
    fn = L.p2p_split_fault_word_ptr
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_void_p
    p = fn(_lib.stream_ptr(device))
    if not p:
        raise _lib.KernelError("split-K fault word: allocation failed")
    torch.cuda.synchronize(device)  # its zeroing is done before any loop stream reads it
    return int(p)


def tiled_split_fault() -> int:
    """Nonzero if a parallel split-K slice gave up waiting for its tile (output invalid);
    clears the flag.  Synchronises the device."""
    L = _lib.lib()
    return int(L.p2p_tiled_split_fault()) if hasattr(L, "p2p_tiled_split_fault") else 0


def _code(wt, M, epi, norm, waves):
    if waves:
        return waves
    return _TUNE.get(tune_key(wt, M, epi, norm), 0)


def tile_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] (nn.Linear layout) -> fragment-major [N/16, K/32, 64, 8]."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0, (N, K)
    # W_t[g, s, q, r, j] = W[16 g + r, 32 s + 8 q + j]
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(
        N // 16, K // 32, 64, 8)


def untile_weight(wt: torch.Tensor) -> torch.Tensor:
    G, S = wt.shape[0], wt.shape[1]
    return wt.reshape(G, S, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(G * 16, S * 32)


def tiled_shape(wt: torch.Tensor):
    return wt.shape[0] * 16, wt.shape[1] * 32  # (N, K)


def fold_norm(w: torch.Tensor, gain: torch.Tensor) -> torch.Tensor:
    """Fold an RMSNorm gain into the consuming projection: W' = W * diag(gain)."""
    return (w.float() * gain.float()[None, :]).to(w.dtype)


def _ref(wt, x, epi, norm, out, eps):
    N, K = tiled_shape(wt)
    W = wt.dequantize_f32() if _is_f8(wt) else untile_weight(wt).float()
    xf = x.float()
    acc = xf @ W.t()
    if norm:
        rstd = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
        acc = acc * rstd
    if epi == EPI_STORE:
        out.copy_(acc.to(out.dtype))
    elif epi == EPI_RESID:
        out.copy_((out.float() + acc).to(out.dtype))
    elif epi == EPI_SILU:
        F = N // 2
        g, u = acc[:, :F], acc[:, F:]
        out.copy_((torch.nn.functional.silu(g) * u).to(out.dtype))
    elif epi == EPI_F32:
        out.copy_(acc)
    else:
        raise ValueError(epi)
    return out


def skinny_gemm(wt: torch.Tensor, x: torch.Tensor, epi: int = EPI_STORE, norm: bool = False,
                out: torch.Tensor | None = None, eps: float = 1e-5, waves: int = 0,
                x_packed: bool = False) -> torch.Tensor:
    """out = epi(rstd(x) * x @ W^T) for x [M, K] with M <= 64 (rows > 64 are chunked).
    A launch code with AFRAG_FLAG packs x fragment-major first (pack_frag) unless
    ``x_packed`` says the caller already did (then x is pack_frag's output, rows <= 64)."""
    N, K = tiled_shape(wt)
    M = x.shape[0]
    assert x.shape[1] == K and x.dtype == torch.bfloat16, (x.shape, K, x.dtype)
    n_out = N // 2 if epi == EPI_SILU else N
    if out is None:
        if epi == EPI_RESID:
            raise ValueError("EPI_RESID needs the residual tensor as `out`")
        out = torch.empty(M, n_out, device=x.device,
                          dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    if x.device.type != "cuda":
        return _ref(wt, x, epi, norm, out, eps)
    assert x.stride(1) == 1 and out.stride(1) == 1
    L = _lib.lib()
    s = _lib.stream_ptr(x.device)
    if (epi == EPI_SILU and norm and M > SKINNY_MAX_M and TALL_SILU and not _is_f8(wt)
            and not (waves & TILED_FLAG) and tall_silu_ok(M, K, N)):
        # batched-prompt gate_up: all rows in one workgroup, weights streamed once (tall_gemm.hip)
        _lib.check(_lib.experimental().p2p_tall_silu(wt.data_ptr(), x.data_ptr(), x.stride(0), M, K, N,
                                   out.data_ptr(), out.stride(0), float(eps), s), "tall_silu")
        return out
    if _want_tiled(wt, M, N, K, epi, norm, waves):
        _lib.check(L.p2p_tiled_gemm(wt.data_ptr(), x.data_ptr(), x.stride(0), M, K, N, epi,
                                    int(norm), out.data_ptr(), out.stride(0), float(eps), s),
                   "tiled_gemm")
        return out
    for m0 in range(0, M, SKINNY_MAX_M):
        mc = min(SKINNY_MAX_M, M - m0)
        xs = x[m0:m0 + mc]
        os_ = out[m0:m0 + mc]
        wp, sp = _wptr(wt)
        code = _code(wt, mc, epi, norm, waves)
        if code & PERSIST_FLAG:
            _lib.experimental()  # the persistent GEMV's library (its symbol, found by dlsym)
        if code & AFRAG_FLAG and not x_packed:
            xs = _packed(xs)  # a launch of its own: the autotuner times pack + GEMM together
        _lib.check(L.p2p_skinny_gemm(wp, xs.data_ptr(), x.stride(0), mc, K, N, epi,
                                     int(norm), os_.data_ptr(), out.stride(0), float(eps),
                                     code, sp, s), "skinny_gemm")
    return out


_FAR_MAX_WAVES = int(os.environ.get("P2P_FAR_MAX_WAVES", "0"))


def skinny_ar_ok(wt, M: int) -> bool:
    """Would ``skinny_gemm_ar`` run this projection at M rows on its tuned kernel?  Only the
    skinny kernel has the fused all-reduce epilogue: a shape whose tuned launch is the
    tiled / mid-M kernel (prompt-sized M) keeps the partial store + one-shot kernel."""
    if M > SKINNY_MAX_M:
        return False
    return not (_code(wt, M, EPI_AR, False, 0) & (TILED_FLAG | MIDM_FLAG | WIDE_FLAG | PERSIST_FLAG))


def skinny_gemm_ar(wt, x: torch.Tensor, h: torch.Tensor, car, waves: int = 0) -> torch.Tensor:
    """h += sum over the TP group of x @ W^T, the all-reduce fused into the GEMM epilogue
    (``csrc/kernels/fused_ar.h``): every block pushes its bf16 partial tile to every rank,
    waits for the same tile of the peers and adds the rank-ordered sum to the residual --
    one launch where the unfused path takes two (partial store, one-shot all-reduce), with
    a bit-identical result.  ``car``: the group's ``parallel.custom_ar.CustomAllReduce``.
    Every rank must make the same calls (same N, M) in the same order."""
    N, K = tiled_shape(wt)
    M = x.shape[0]
    assert x.device.type == "cuda" and h.dtype == torch.bfloat16 and h.shape[0] == M
    assert x.stride(1) == 1 and h.stride(1) == 1 and h.shape[1] == N
    assert car.fused_ok(M, N, h.stride(0)), (M, N, h.stride(0))
    code = _code(wt, M, EPI_AR, False, waves)
    if _FAR_MAX_WAVES and not 0 < (code & 0xff) <= _FAR_MAX_WAVES:
        # virtual ranks sharing one device: fewer spinning waves per rank so every rank's
        # grid can be resident at once (tests; a real device runs only its own grid)
        code = (code & ~0xff) | _FAR_MAX_WAVES
    wp, sp = _wptr(wt)
    _lib.check(_lib.lib().p2p_skinny_gemm_ar(
        wp, x.data_ptr(), x.stride(0), M, K, N, h.data_ptr(), h.stride(0), car._far_bases,
        car.rank, car.world, car.far_max_bytes, car.far_counters.data_ptr(), car.err.data_ptr(),
        code, sp, _lib.stream_ptr(x.device)), "skinny_gemm_ar")
    return h


# ------------------------------------------------------------ fused epilogues
def rope_row_perm(n_heads_total: int, head_dim: int = 128) -> torch.Tensor:
    """Row order of the fused qkv+RoPE projection (skinny_gemm.hip, EPI_QKV_ROPE).

    Within every head, 16-row group k holds dims 8k..8k+7 and 64+8k..64+8k+7 so the
    rotate_half partner of a lane is lane ^ 8.  Returns perm with new_row = old[perm].
    """
    half = head_dim // 2
    one = []
    for k in range(head_dim // 16):
        one += [8 * k + r for r in range(8)] + [half + 8 * k + r for r in range(8)]
    one = torch.tensor(one, dtype=torch.long)
    return (torch.arange(n_heads_total)[:, None] * head_dim + one[None, :]).reshape(-1)


def qkv_rope_gemm(wt, x, pos, slots, cos_sin, n_heads, n_kv, q_out, k_cache, v_cache,
                  eps=1e-5, waves=0):
    """q_out, k/v pages <- rope(rstd(x) * x @ Wqkv^T) with Wqkv rows in rope_row_perm order."""
    from .attention import rope_cache_ref

    M = x.shape[0]
    N, K = tiled_shape(wt)
    assert N == (n_heads + 2 * n_kv) * 128
    if x.device.type != "cuda":
        perm = rope_row_perm(n_heads + 2 * n_kv)
        qkv_p = torch.empty(M, N, dtype=torch.bfloat16)
        _ref(wt, x, EPI_STORE, True, qkv_p, eps)
        qkv = torch.empty_like(qkv_p)
        qkv[:, perm] = qkv_p
        return rope_cache_ref(qkv, pos, slots, cos_sin, n_heads, n_kv, q_out, k_cache, v_cache)
    L = _lib.lib()
    s = _lib.stream_ptr(x.device)
    if _want_tiled(wt, M, N, K, EPI_QKV_ROPE, True, waves):
        _lib.check(L.p2p_tiled_gemm_qkv_rope(
            wt.data_ptr(), x.data_ptr(), x.stride(0), M, K, n_heads, n_kv, pos.data_ptr(),
            slots.data_ptr(), cos_sin.data_ptr(), q_out.data_ptr(), q_out.stride(0),
            k_cache.data_ptr(), v_cache.data_ptr(), float(eps), s), "tiled_gemm_qkv_rope")
        return q_out
    for m0 in range(0, M, SKINNY_MAX_M):
        mc = min(SKINNY_MAX_M, M - m0)
        wp, sp = _wptr(wt)
        code = _code(wt, mc, EPI_QKV_ROPE, True, waves)
        xs = x[m0:m0 + mc]
        if code & AFRAG_FLAG:
            xs = _packed(xs)
        _lib.check(L.p2p_skinny_gemm_qkv_rope(
            wp, xs.data_ptr(), x.stride(0), mc, K, n_heads, n_kv,
            pos[m0:].data_ptr(), slots[m0:].data_ptr(), cos_sin.data_ptr(), q_out[m0:].data_ptr(),
            q_out.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), float(eps),
            code, sp, s), "skinny_gemm_qkv_rope")
    return q_out


KEY_SHARDS = 32


def new_argmax_keys(rows: int, device) -> torch.Tensor:
    return torch.zeros(rows, KEY_SHARDS, dtype=torch.int64, device=device)


def lm_head_argmax(wt, x, keys, col_offset: int = 0, eps: float = 1e-5, waves: int = 0):
    """Greedy LM head: keys[m, shard] = max of (ordered logit << 32 | ~token) over the
    vocab columns of that shard's blocks.

    keys (int64 [M, KEY_SHARDS], zeroed) are reduced into token ids (and reset) by
    argmax_finalize / advance.
    """
    M = x.shape[0]
    N, K = tiled_shape(wt)
    if x.device.type != "cuda":
        logits = _ref(wt, x, EPI_F32, True, torch.empty(M, N), eps)
        v, i = logits.max(-1)
        u = v.view(torch.int32).long() & 0xFFFFFFFF
        u = torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
        k = (u << 32) | (0xFFFFFFFF - (i + col_offset))
        # unsigned 64-bit max on int64 storage: compare with the sign bit flipped
        sign = torch.tensor(-(2 ** 63), dtype=torch.int64)
        cur = keys[:M, 0]
        keys[:M, 0] = torch.where((k ^ sign) > (cur ^ sign), k, cur)
        return keys
    L = _lib.lib()
    if _want_tiled(wt, M, N, K, EPI_ARGMAX, True, waves):
        _lib.check(L.p2p_tiled_gemm_argmax(wt.data_ptr(), x.data_ptr(), x.stride(0), M, K, N,
                                           keys.data_ptr(), int(col_offset), float(eps),
                                           _lib.stream_ptr(x.device)), "tiled_gemm_argmax")
        return keys
    wp, sp = _wptr(wt)
    for m0 in range(0, M, SKINNY_MAX_M):  # > 64 rows only reach here with FP8 weights
        mc = min(SKINNY_MAX_M, M - m0)
        _lib.check(L.p2p_skinny_gemm_argmax(wp, x[m0:].data_ptr(), x.stride(0), mc, K, N,
                                            keys[m0:].data_ptr(), int(col_offset), float(eps),
                                            _code(wt, mc, EPI_ARGMAX, True, waves), sp,
                                            _lib.stream_ptr(x.device)), "skinny_gemm_argmax")
    return keys


def reduce_keys_ref(keys, M):
    sign = torch.tensor(-(2 ** 63), dtype=torch.int64)
    k = keys[:M]
    best = ((k ^ sign).max(dim=1).values) ^ sign
    keys[:M] = 0
    return (0xFFFFFFFF - (best & 0xFFFFFFFF)).to(torch.int32)


def argmax_finalize(keys, ids):
    M = ids.shape[0]
    if keys.device.type != "cuda":
        ids.copy_(reduce_keys_ref(keys, M))
        return ids
    L = _lib.lib()
    _lib.check(L.p2p_argmax_finalize(keys.data_ptr(), ids.data_ptr(), M,
                                     _lib.stream_ptr(keys.device)), "argmax_finalize")
    return ids
