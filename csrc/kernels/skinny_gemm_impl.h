// Skinny GEMM kernel template and its launch ladder (MT x WAVES x U), shared by the
// per-epilogue instantiation units skinny_inst_*.hip (compiled in parallel) and the
// dispatcher in skinny_gemm.hip.  See skinny_gemm.hip for the design notes.
#pragma once
#include "gemm_epilogue.h"

#include <type_traits>

namespace {

// F8: weight-only FP8 (OCP e4m3) -- half the bytes of bf16, widened to bf16 in registers
// right before the MFMA; the per-output-channel scale (ea.wscale) is applied to the
// accumulator in the epilogue.  The codes of k-steps 2p and 2p+1 are interleaved per lane
// (ops.gemm.pair_f8), so one 16-byte load per lane (1 KiB per wave, as in bf16) feeds two
// MFMAs: the pipeline runs over "super-steps" of KP = 2 k-steps.  (8-byte loads, one
// k-step each, left the fp8 stream at ~2.5-4.8 TB/s: half the bytes in flight per load.)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <bool F8>
using wraw_t = typename std::conditional<F8, u32x4, bf16x8>::type;

__device__ __forceinline__ bf16x8 widen(const bf16x8& w, int) { return w; }
// 8 e4m3 codes (half h of the pair) -> 8 bf16: four gfx950 v_cvt_scalef32_pk_bf16_fp8
__device__ __forceinline__ bf16x8 widen(const u32x4& p, int h) {
  const unsigned lo = h ? p.z : p.x, hi = h ? p.w : p.y;
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, true);
  bf16x8 r;
  r[0] = a.x; r[1] = a.y; r[2] = b.x; r[3] = b.y;
  r[4] = c.x; r[5] = c.y; r[6] = d.x; r[7] = d.y;
  return r;
}

// One block's work: column group(s) g0 = bid * NG.  (A function of its own so the EPI_AR
// launch can walk several column groups per block, skinny_gemm_kernel below.)
template <int MT, int WAVES, int EPI, bool NORM, int U, bool MOE, int NG, bool F8>
__device__ __forceinline__ void skinny_body(
    const bf16x8* __restrict__ Wt, const bf16* __restrict__ X, int ldx, int M, int K,
    int up_group_offset, void* __restrict__ out, int ldo, float eps, const EpiArgs& ea, int bid) {
  // NG column groups per block share every A (activation) fragment: at MT > 1 the
  // A loads (MT per k-step) and the NORM sum of squares dominate unless reused.
  constexpr int NB = (EPI == EPI_SILU) ? 2 : 1;
  constexpr int NW = NG * NB;  // weight fragments per k-step
  constexpr int KP = F8 ? 2 : 1;  // k-steps per 16-byte weight load
  const int S = (K >> 5) / KP;    // super-steps
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g0 = bid * NG;
  const int s0 = (S * w) / WAVES;
  const int s1 = (S * (w + 1)) / WAVES;
  const int r = lane & 15, q = lane >> 4;
  const int* mrows = nullptr;
  if constexpr (MOE) {
    const int e = blockIdx.y;
    M = min(ea.moe_cnt[e], M);
    if (M <= 0) return;  // expert not selected by any row: its weights are never read
    Wt += (size_t)e * ea.w_stride;
    mrows = ea.moe_rows + (size_t)e * ea.rows_stride;
  }

  using WR = wraw_t<F8>;
  const WR* wq = reinterpret_cast<const WR*>(Wt);
  const WR* wp[NW];
#pragma unroll
  for (int c = 0; c < NG; ++c) {
    wp[c * NB] = wq + (size_t)(g0 + c) * S * 64 + lane;
    if constexpr (NB == 2) wp[c * NB + 1] = wq + (size_t)(g0 + c + up_group_offset) * S * 64 + lane;
  }

  const bf16* xp[MT];
  bool xv[MT];
  // fragment-major X (ea.afrag, p2p_pack_frag): A fragment (mt, s) is 1 KiB contiguous, so
  // an A load is 8 whole cache lines instead of 16 half lines of 16 rows
  const bool af = !MOE && ea.afrag;
  const int xs = af ? 512 : 32;  // elements between consecutive k-steps of one lane
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = mt * 16 + r;
    xv[mt] = af ? mt * 16 < M : row < M;
    int xrow = xv[mt] ? row : 0;
    if constexpr (MOE) xrow = xv[mt] ? mrows[row] / ea.x_div : 0;
    xp[mt] = af ? X + ((size_t)mt * (K >> 5) * 64 + lane) * 8 : X + (size_t)xrow * ldx + 8 * q;
  }

  // EPI_QKV_ROPE: fetch (cos, sin) and the KV slot of this lane's output rows now,
  // so the epilogue's dependent pos -> table loads overlap the weight stream.
  // (NG > 1: the rows' slots/positions only; the table is read in the epilogue.)
  float2 rc[MT][4];
  int rslot[MT][4];
  int rpos[MT][4];
  if constexpr (EPI == EPI_QKV_ROPE) {
    const int kk = g0 & 7;
    const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int m = mt * 16 + q * 4 + j;
        int mm = m;
        if constexpr (MOE) mm = 0;
        const bool ok = m < M && w == 0;
        rslot[mt][j] = ok ? ea.slots[mm] : -1;
        rpos[mt][j] = ok ? ea.pos[mm] : 0;
        if constexpr (NG == 1)
          rc[mt][j] = ok ? ea.cs[(size_t)rpos[mt][j] * 64 + dd] : float2{1.f, 0.f};
      }
  }

  // EPI_RESID at batch 1: the residual values are loaded BEFORE the weight stream (one
  // 2-byte load per lane of wave 0, in flight under the whole stream), so the epilogue never
  // waits a memory round trip after the split-K reduction.  (Only this block ever writes
  // these columns, at its very end, so the early read sees the pre-call residual.)
  constexpr bool kEarlyResid = EPI == EPI_RESID && !MOE && MT == 1;
  float resv[NG][MT][4];
  float2 csv[NG][MT][4];
  auto load_epi_operands = [&]() {
#pragma unroll
    for (int c = 0; c < NG; ++c)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = mt * 16 + q * 4 + j;
          const bool ok = w == 0 && m < M;
          resv[c][mt][j] = 0.f;
          csv[c][mt][j] = float2{1.f, 0.f};
          if constexpr (EPI == EPI_RESID && !MOE)
            if (ok) resv[c][mt][j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + (g0 + c) * 16 + r];
          if constexpr (EPI == EPI_QKV_ROPE && NG > 1) {
            const int kk = (g0 + c) & 7;
            const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
            if (ok) csv[c][mt][j] = ea.cs[(size_t)rpos[mt][j] * 64 + dd];
          }
        }
  };
  if constexpr (kEarlyResid) load_epi_operands();
  // EPI_AR (fused all-reduce epilogue) at batch 1: the same for the residual pair each lane
  // of wave 0 sums into (fused_ar.h epilogue, its first granule i = lane)
  unsigned h_pre = 0;
  if constexpr (EPI == EPI_AR && MT == 1)
    if (w == 0 && lane < 8 * M)
      h_pre = reinterpret_cast<const unsigned*>(out)[((size_t)(lane >> 3) * ldo) / 2 + (size_t)g0 * 8 + (lane & 7)];

  f32x4 acc[NW][MT];
  float ss[MT];
#pragma unroll
  for (int b = 0; b < NW; ++b)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[b][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ss[mt] = 0.f;

  // A fragments of super-step s: ax[h * MT + mt] = rows of m-tile mt at k-step s*KP + h
  auto loadx = [&](int s, bf16x8(&ax)[KP * MT]) {
#pragma unroll
    for (int h = 0; h < KP; ++h)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        ax[h * MT + mt] = xv[mt] ? *reinterpret_cast<const bf16x8*>(xp[mt] + (size_t)(s * KP + h) * xs)
                                 : zero_bf16x8();
  };
  auto load = [&](int s, WR(&bw)[U][NW], bf16x8(&ax)[U][KP * MT]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int b = 0; b < NW; ++b) bw[u][b] = __builtin_nontemporal_load(wp[b] + (size_t)(s + u) * 64);
      loadx(s + u, ax[u]);
    }
  };
  auto compute1 = [&](const WR(&bwr)[NW], const bf16x8(&ax)[KP * MT]) {
#pragma unroll
    for (int h = 0; h < KP; ++h) {
      bf16x8 bw[NW];
#pragma unroll
      for (int b = 0; b < NW; ++b) bw[b] = widen(bwr[b], h);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8& a = ax[h * MT + mt];
#pragma unroll
        for (int b = 0; b < NW; ++b)
          acc[b][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[b], acc[b][mt], 0, 0, 0);
        if constexpr (NORM) ss[mt] = sumsq8(a, ss[mt]);
      }
    }
  };
  auto compute = [&](WR(&bw)[U][NW], bf16x8(&ax)[U][KP * MT]) {
#pragma unroll
    for (int u = 0; u < U; ++u) compute1(bw[u], ax[u]);
  };

  const int n = s1 - s0;
  const int nb = n / U;
  if (nb > 0) {
    WR bA[U][NW], bB[U][NW];
    bf16x8 aA[U][KP * MT], aB[U][KP * MT];
    load(s0, bA, aA);
    int b = 0;
    for (; b + 2 < nb; b += 2) {
      load(s0 + (b + 1) * U, bB, aB);
      compute(bA, aA);
      load(s0 + (b + 2) * U, bA, aA);
      compute(bB, aB);
    }
    if (b + 1 < nb) {
      load(s0 + (b + 1) * U, bB, aB);
      compute(bA, aA);
      compute(bB, aB);
    } else {
      compute(bA, aA);
    }
  }
  for (int s = s0 + nb * U; s < s1; ++s) {
    WR b1[NW];
    bf16x8 a1[KP * MT];
#pragma unroll
    for (int b = 0; b < NW; ++b) b1[b] = __builtin_nontemporal_load(wp[b] + (size_t)s * 64);
    loadx(s, a1);
    compute1(b1, a1);
  }

  // ---- epilogue operands (when not loaded before the stream), issued by the finishing wave
  // (0) right after its main loop as one batch, so they land during the split-K reduction:
  // the residual values (EPI_RESID at MT > 1) and, at NG > 1, the rows' (cos, sin)
  // (EPI_QKV_ROPE).  Loaded element by element inside the store loop they were a chain of
  // NG x MT x 4 dependent round trips (each store may alias the next load): +7 us on the
  // 44-row qkv, +1 us per row-quad on the residual GEMMs.
  if constexpr (!kEarlyResid) load_epi_operands();

  // ---- split-K reduction across the block's waves ----
  if constexpr (NORM) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      ss[mt] += __shfl_xor(ss[mt], 16, 64);
      ss[mt] += __shfl_xor(ss[mt], 32, 64);
    }
  }
  float rstd[MT][4];
  if constexpr (WAVES > 1) {
    __shared__ float red[WAVES - 1][NW * MT * 4][64];
    __shared__ float red_ss[WAVES][MT][16];
    if (w > 0) {
#pragma unroll
      for (int b = 0; b < NW; ++b)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int j = 0; j < 4; ++j) red[w - 1][(b * MT + mt) * 4 + j][lane] = acc[b][mt][j];
    }
    if constexpr (NORM) {
      if (q == 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) red_ss[w][mt][r] = ss[mt];
      }
    }
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int ww = 0; ww < WAVES - 1; ++ww)
#pragma unroll
      for (int b = 0; b < NW; ++b)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[b][mt][j] += red[ww][(b * MT + mt) * 4 + j][lane];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rstd[mt][j] = 1.f;
        if constexpr (NORM) {
          float t = 0.f;
#pragma unroll
          for (int ww = 0; ww < WAVES; ++ww) t += red_ss[ww][mt][q * 4 + j];
          rstd[mt][j] = rsqrtf(t / (float)K + eps);
        }
      }
  } else {
    // single wave: rstd for row m lives in lane (m & 15) of the same m-tile.
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rstd[mt][j] = 1.f;
        if constexpr (NORM) {
          const float t = __shfl(ss[mt], q * 4 + j, 64);
          rstd[mt][j] = rsqrtf(t / (float)K + eps);
        }
      }
  }

  // ---- epilogue (wave 0) ----
  if constexpr (EPI == EPI_AR) {  // TP row-parallel: push, wait, sum + residual (fused_ar.h)
    static_assert(NG == 1 && !MOE, "fused all-reduce: one column group per block");
    float v[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float s = rstd[mt][j];
        if constexpr (F8) s *= ea.wscale[(size_t)g0 * 16 + r];
        v[mt][j] = acc[0][mt][j] * s;
      }
    far::epilogue<MT>(v, M, g0, lane, reinterpret_cast<bf16*>(out), ldo, ea.far,
                      MT == 1 ? &h_pre : nullptr);
    return;
  }
#pragma unroll
  for (int c = 0; c < NG; ++c) {
    const int g = g0 + c;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mt * 16 + q * 4 + j;
        float scale = rstd[mt][j];
        int orow = m;
        if constexpr (MOE) {
          orow = m < M ? mrows[m] : 0;
          if (ea.row_w && m < M) scale *= ea.row_w[orow];
        }
        float s0 = scale, s1 = scale;  // F8: per-output-channel weight scales
        if constexpr (F8) {
          s0 *= ea.wscale[(size_t)g * 16 + r];
          if constexpr (NB == 2) s1 *= ea.wscale[(size_t)(g + up_group_offset) * 16 + r];
          else s1 = s0;
        }
        if constexpr (EPI == EPI_QKV_ROPE) {
          const float2 cs = NG == 1 ? rc[mt][j] : csv[c][mt][j];
          epi_store<EPI>(orow, m < M, g, r, acc[c][mt][j] * s0, 0.f, out, ldo, ea, cs,
                         rslot[mt][j]);
        } else if constexpr (EPI == EPI_RESID && !MOE) {
          if (m < M)
            reinterpret_cast<bf16*>(out)[(size_t)orow * ldo + g * 16 + r] =
                f2bf(resv[c][mt][j] + acc[c * NB][mt][j] * s0);
        } else {
          epi_store<EPI>(orow, m < M, g, r, acc[c * NB][mt][j] * s0,
                         acc[c * NB + NB - 1][mt][j] * s1, out, ldo, ea);
        }
      }
    }
  }
}

// EPI_AR (TP row-parallel + fused all-reduce): every column group's epilogue waits in place
// for the same column group of every peer rank, so all ranks' blocks of a call must be able
// to be resident at once.  On its own device a rank's grid always is; ranks sharing a device
// (virtual-rank tests) are not, and in round 5 a TP=4 engine on one device deadlocked until the
// spin bound (4 ranks x 256 blocks x 8 waves > the device's 4096 wave slots at 128 VGPRs).  So
// the launch is capped to the blocks the device holds for its share of co-resident ranks
// (p2p_far_set_coresident) and each block walks column groups gb, gb + grid, ...: no block
// ever waits on one that cannot be scheduled.
template <int MT, int WAVES, int EPI, bool NORM, int U, bool MOE = false, int NG = 1, bool F8 = false>
__global__ __launch_bounds__(WAVES * 64) void skinny_gemm_kernel(
    const bf16x8* __restrict__ Wt, const bf16* __restrict__ X, int ldx, int M, int K,
    int up_group_offset, void* __restrict__ out, int ldo, float eps, EpiArgs ea) {
  if constexpr (EPI == EPI_AR) {
    for (int gb = blockIdx.x; gb < ea.far.groups; gb += gridDim.x) {
      skinny_body<MT, WAVES, EPI, NORM, U, MOE, NG, F8>(Wt, X, ldx, M, K, up_group_offset, out,
                                                        ldo, eps, ea, gb);
      __syncthreads();  // the split-K reduction buffer is reused by the next group
    }
  } else {
    skinny_body<MT, WAVES, EPI, NORM, U, MOE, NG, F8>(Wt, X, ldx, M, K, up_group_offset, out, ldo,
                                                      eps, ea, blockIdx.x);
  }
}

// k-steps per pipeline batch for MT=1: ONE setting for every instantiation unit (defined in
// skinny_gemm.hip, set by p2p_skinny_gemm_tune)
}  // namespace
extern int g_skinny_u_mt1;
namespace {

template <int MT, int WAVES, int EPI, bool NORM, int U>
int launch_mwu(const void* Wt, const void* X, int ldx, int M, int K, int groups, int up_off,
               void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st);

}  // namespace
// Blocks of the EPI_AR launch: the column groups, capped to what the device holds for its
// share of the ranks resident on it (skinny_gemm.hip, p2p_far_set_coresident).
int far_grid(int groups, const void* kernel, int threads);
namespace {

template <int MT, int WAVES, int EPI, bool NORM>
int launch_mw(const void* Wt, const void* X, int ldx, int M, int K, int groups, int up_off,
              void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  // pipeline depth: MT=1 -> 4 or 8 k-steps per batch; MT>1 holds MT A fragments per
  // k-step, so batches of 2 (4 at MT=2) keep it under ~128 VGPRs (no scratch)
  int u = ea.u ? ea.u : (MT == 1 ? g_skinny_u_mt1 : 2);
  // FP8 holds KP = 2 A fragments per weight load: the deep batch spills to scratch at
  // 8 waves (<= 128 VGPRs) and at MT = 4, so those take the shallow one.
  if (ea.wscale && (WAVES == 8 || MT == 4)) u = MT == 1 ? 4 : 2;
  if (WAVES == 16) u = 4;
  if constexpr (MT == 1) {
    if (u == 8)
      return launch_mwu<MT, WAVES, EPI, NORM, 8>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    return launch_mwu<MT, WAVES, EPI, NORM, 4>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  } else {
    if (u >= 4)
      return launch_mwu<MT, WAVES, EPI, NORM, 4>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    return launch_mwu<MT, WAVES, EPI, NORM, 2>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  }
}

template <int MT, int WAVES, int EPI, bool NORM, int U>
int launch_mwu(const void* Wt, const void* X, int ldx, int M, int K, int groups, int up_off,
               void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  if constexpr (WAVES == 16) {
    // 16 waves (batch 1, bf16, one column group per block, 4-deep batches: <= 128 VGPRs with
    // no scratch; not SwiGLU, whose two weight streams per wave spill): a weight stream
    // reaches HBM speed only with ~16 waves per CU (bench/stream_probe.py,
    // profiles/r6_stream_probe.md), and the N = 4096 row-parallel projections have just 256
    // column groups, one per CU
    if constexpr (MT != 1 || U != 4 || EPI == EPI_SILU) {
      return (int)hipErrorInvalidValue;
    } else {
      if (ea.wscale || ea.moe_cnt) return (int)hipErrorInvalidValue;
      int grid = groups;
      if constexpr (EPI == EPI_AR) grid = far_grid(groups, (const void*)skinny_gemm_kernel<MT, WAVES, EPI, NORM, U>, WAVES * 64);
      hipLaunchKernelGGL((skinny_gemm_kernel<MT, WAVES, EPI, NORM, U>), dim3(grid), dim3(WAVES * 64), 0,
                         st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, up_off, out, ldo, eps, ea);
      return (int)hipGetLastError();
    }
  } else {
  if (ea.wscale) {  // FP8 weights (dense projections, one column group per block)
    if (ea.moe_cnt || (K % 64) != 0) return (int)hipErrorInvalidValue;  // k-step pairs
    int grid = groups;
    if constexpr (EPI == EPI_AR)
      grid = far_grid(groups, (const void*)skinny_gemm_kernel<MT, WAVES, EPI, NORM, U, false, 1, true>, WAVES * 64);
    hipLaunchKernelGGL((skinny_gemm_kernel<MT, WAVES, EPI, NORM, U, false, 1, true>), dim3(grid),
                       dim3(WAVES * 64), 0, st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K,
                       up_off, out, ldo, eps, ea);
    return (int)hipGetLastError();
  }
  if (ea.moe_cnt) {
    if constexpr (EPI == EPI_SILU || EPI == EPI_STORE) {
      hipLaunchKernelGGL((skinny_gemm_kernel<MT, WAVES, EPI, NORM, U, true>),
                         dim3(groups, ea.n_experts),
                         dim3(WAVES * 64), 0, st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K,
                         up_off, out, ldo, eps, ea);
      return (int)hipGetLastError();
    }
    return (int)hipErrorInvalidValue;
  }
  if constexpr (MT > 1 || U == 4) {
    // two column groups per block (shared A fragments at MT > 1; at MT = 1, twice the
    // weight bytes in flight per wave); only where the split-K reduction buffer still
    // fits the 64 KiB static LDS window (MT = 1: the 4-deep batch, 8 would spill)
    constexpr int NW2 = 2 * ((EPI == EPI_SILU) ? 2 : 1);
    constexpr size_t lds2 = (size_t)(WAVES - 1) * NW2 * MT * 4 * 64 * 4;
    if constexpr (lds2 <= 56 * 1024 && EPI != EPI_AR) {
      if (ea.ng == 2 && groups % 2 == 0) {
        hipLaunchKernelGGL((skinny_gemm_kernel<MT, WAVES, EPI, NORM, U, false, 2>),
                           dim3(groups / 2), dim3(WAVES * 64), 0, st, (const bf16x8*)Wt,
                           (const bf16*)X, ldx, M, K, up_off, out, ldo, eps, ea);
        return (int)hipGetLastError();
      }
    }
  }
  int grid = groups;
  if constexpr (EPI == EPI_AR) grid = far_grid(groups, (const void*)skinny_gemm_kernel<MT, WAVES, EPI, NORM, U>, WAVES * 64);
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, WAVES, EPI, NORM, U>), dim3(grid), dim3(WAVES * 64), 0,
                     st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, up_off, out, ldo, eps, ea);
  return (int)hipGetLastError();
  }  // WAVES != 16
}

template <int MT, int EPI, bool NORM>
int launch_m(int waves, const void* Wt, const void* X, int ldx, int M, int K, int groups,
             int up_off, void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  switch (waves) {
    case 1: return launch_mw<MT, 1, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 2: return launch_mw<MT, 2, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 4: return launch_mw<MT, 4, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 8: return launch_mw<MT, 8, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 16:
      if constexpr (MT == 1)
        return launch_mw<MT, 16, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
      break;
  }
  return (int)hipErrorInvalidValue;
}

template <int EPI, bool NORM>
int launch_e(int mt, int waves, const void* Wt, const void* X, int ldx, int M, int K, int groups,
             int up_off, void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  switch (mt) {
    case 1: return launch_m<1, EPI, NORM>(waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 2: return launch_m<2, EPI, NORM>(waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 4: return launch_m<4, EPI, NORM>(waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  }
  return (int)hipErrorInvalidValue;
}

}  // namespace

// One instantiation unit per epilogue: the dispatcher calls these through a table.  EpiArgs
// lives in an anonymous namespace (one identical definition per unit), so it crosses
// units as a pointer to the caller's copy.
#define SKINNY_UNIT_ARGS int norm, int mt, int waves, const void *Wt, const void *X, int ldx, \
    int M, int K, int groups, int up_off, void *out, int ldo, float eps, const void *ea_p,     \
    hipStream_t st
typedef int (*skinny_unit_fn)(SKINNY_UNIT_ARGS);
