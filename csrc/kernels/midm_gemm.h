// Mid-M GEMM (16 < M <= 64 rows: chat-length prompt prefill, mixed batches) on an
// LDS-DMA pipeline, one 16-column group per workgroup and the WHOLE K per workgroup.
//
//   out[m, 16 g + r] = epilogue( rstd[m] * sum_k X[m, k] * W[16 g + r, k] )
//
// Why a third family next to skinny_gemm.hip (register-staged GEMV) and
// prefill_gemm.h (LDS-tiled, split-K for few tiles):
//   * at M = 44 the skinny kernel reads MT = 3-4 activation fragments per weight
//     fragment, all through VGPRs, so its bytes in flight per CU (~60 KB) leave both
//     the L2 (activations) and HBM (weights) streams latency-bound (qkv 28-41 us for a
//     50 MB stream that takes 11 us at M = 1);
//   * the tiled kernel fills the chip only by splitting K over workgroups, and pays a
//     cross-workgroup reduction (write-through slabs + tickets) per tile.
// Here a workgroup (4 waves) owns one column group (NB = 1, or 2 for SwiGLU gate/up)
// for all of K and streams K in chunks of KC = 4 k-steps through a STAGES-deep ring of
// LDS-DMA fills (global_load_lds_dwordx4: one wave instruction = one 1 KiB MFMA
// fragment, no VGPRs): the activation fragments (MT x KC KiB per chunk, L2-resident
// after the first workgroups) and the weight fragments (NB x KC KiB, HBM, fragment-
// major so every fill is 1 KiB contiguous).  Two workgroups per CU keep ~100 KB of
// loads in flight per CU.  Wave w consumes k-step w of every chunk (MT x NB MFMAs
// 16x16x32); the four partial accumulators meet in LDS at the end, and the epilogue
// (gemm_epilogue.h: RMSNorm rstd, RoPE + KV write, SwiGLU, residual, argmax) runs on
// the reduced tile with its m-tiles spread over the waves.  No cross-workgroup
// communication at all.
#pragma once
#include "gemm_epilogue.h"

namespace midm {

constexpr int NT = 256;      // 4 waves
constexpr int KC = 4;        // k-steps (x 32) per chunk: one per wave
// chunks in flight: 4 (3 ahead of the one being consumed) for one weight fragment per
// k-step (<= 80 KiB: two workgroups per CU), 3 for SwiGLU's two (<= 72 KiB)
template <int NB>
constexpr int stages() { return NB == 2 ? 3 : 4; }
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MT, int EPI, bool NORM>
__global__ __launch_bounds__(NT, 2) void midm_kernel(const bf16x8* __restrict__ Wt,
                                                     const bf16* __restrict__ X, int ldx, int M,
                                                     int K, int up_off, void* __restrict__ out,
                                                     int ldo, float eps, EpiArgs ea) {
  constexpr int NB = EPI == EPI_SILU ? 2 : 1;
  constexpr int FR = (MT + NB) * KC;  // 1 KiB fragments per chunk
  static_assert(FR % 4 == 0, "fills per chunk must split evenly over the 4 waves");
  constexpr int L = FR / 4;           // LDS-DMA instructions per wave per chunk
  constexpr int STAGE = FR * 64;      // bf16x8 per stage
  constexpr int STAGES = stages<NB>();
  __shared__ __attribute__((aligned(16))) bf16x8 lds[STAGES * STAGE];

  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int S = K >> 5;      // k-steps
  const int n = S / KC;      // chunks (host guarantees K % (32 * KC) == 0)

  // per-lane DMA sources of this wave's L fragments per chunk (chunk offset added later)
  const bf16* asrc[L];
  const bf16x8* wsrc[L];
  bool is_a[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int f = w + 4 * i;
    is_a[i] = f < MT * KC;
    if (f < MT * KC) {
      const int mt = f / KC, ks = f % KC;
      const int row = min(16 * mt + (lane & 15), M - 1);
      asrc[i] = X + (size_t)row * ldx + 32 * ks + 8 * (lane >> 4);
      wsrc[i] = nullptr;
    } else {
      const int b = (f - MT * KC) / KC, ks = (f - MT * KC) % KC;
      const int gg = b == 0 ? g : g + up_off;
      wsrc[i] = Wt + ((size_t)gg * S + ks) * 64 + lane;
      asrc[i] = nullptr;
    }
  }
  auto issue = [&](int c, int st) {
    bf16x8* base = lds + st * STAGE;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int f = w + 4 * i;
      if (is_a[i])
        __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (size_t)c * KC * 32),
                                         (lds_ptr_t)(base + f * 64), 16, 0, 0);
      else  // weights: read once, non-temporal (aux bit 1 = nt)
        __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + (size_t)c * KC * 64),
                                         (lds_ptr_t)(base + f * 64), 16, 0, 2);
    }
  };

  f32x4 acc[NB][MT];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[b][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ss[mt] = 0.f;

#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < n) issue(t, t);
  for (int t = 0; t < n; ++t) {
    // this wave's fills of chunk t have landed (younger chunks may stay in flight) ...
    const int pending = min(STAGES - 2, n - 1 - t);
    if (STAGES >= 4 && pending >= 2) wait_vmcnt<2 * L>();
    else if (pending >= 1) wait_vmcnt<L>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // chunk t-1's LDS reads are done
    __builtin_amdgcn_s_barrier();  // ... and every other wave's: chunk t is complete,
                                   // and slot (t - 1) % STAGES is free again
    if (t + STAGES - 1 < n) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    const bf16x8* st = lds + (t % STAGES) * STAGE;
    bf16x8 af[MT], bw[NB];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) af[mt] = st[(mt * KC + w) * 64 + lane];
#pragma unroll
    for (int b = 0; b < NB; ++b) bw[b] = st[((MT + b) * KC + w) * 64 + lane];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[b][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[b], acc[b][mt], 0, 0, 0);
      if constexpr (NORM) ss[mt] = sumsq8(af[mt], ss[mt]);
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // every wave is done with the ring: LDS becomes the reduction buffer

  // ---- reduce the 4 waves' partial tiles; wave w finishes m-tiles w, w+4, ... ----
  float* red = reinterpret_cast<float*>(lds);  // [4 waves][NB][MT][4][64]
  float* red_ss = red + 4 * NB * MT * 4 * 64;  // [4 waves][MT][16]
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(((w * NB + b) * MT + mt) * 4 + j) * 64 + lane] = acc[b][mt][j];
  if constexpr (NORM) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v = ss[mt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red_ss[(w * MT + mt) * 16 + lane] = v;
    }
  }
  __syncthreads();
  const int r = lane & 15, q = lane >> 4;
  for (int mt = w; mt < MT; mt += 4) {
    float tot[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) v += red[(((ww * NB + b) * MT + mt) * 4 + j) * 64 + lane];
        tot[b][j] = v;
      }
    // epilogue operands of the 4 rows as one batch (residual values / rows' KV slot and
    // (cos, sin)): loaded per element between the stores they were 4 dependent round trips
    float resv[4];
    float2 csv[4];
    int slotv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * mt + 4 * q + j;
      resv[j] = 0.f;
      csv[j] = float2{1.f, 0.f};
      slotv[j] = -1;
      if constexpr (EPI == EPI_RESID)
        if (m < M) resv[j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + g * 16 + r];
      if constexpr (EPI == EPI_QKV_ROPE) {
        if (m < M) {
          const int kk = g & 7;
          const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
          csv[j] = ea.cs[(size_t)ea.pos[m] * 64 + dd];
          slotv[j] = ea.slots[m];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * mt + 4 * q + j;
      const bool valid = m < M;
      float scale = 1.f;
      if constexpr (NORM) {
        float t2 = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) t2 += red_ss[(ww * MT + mt) * 16 + 4 * q + j];
        scale = rsqrtf(t2 / (float)K + eps);
      }
      if constexpr (EPI == EPI_QKV_ROPE) {
        epi_store<EPI>(m, valid, g, r, tot[0][j] * scale, 0.f, out, ldo, ea, csv[j], slotv[j]);
      } else if constexpr (EPI == EPI_RESID) {
        if (valid)
          reinterpret_cast<bf16*>(out)[(size_t)m * ldo + g * 16 + r] = f2bf(resv[j] + tot[0][j] * scale);
      } else {
        epi_store<EPI>(m, valid, g, r, tot[0][j] * scale, tot[NB - 1][j] * scale, out, ldo, ea);
      }
    }
  }
}

template <int MT, int EPI, bool NORM>
int launch_mt(const void* Wt, const void* X, int ldx, int M, int K, int groups, int up_off,
              void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  hipLaunchKernelGGL((midm_kernel<MT, EPI, NORM>), dim3(groups), dim3(NT), 0, st,
                     (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, up_off, out, ldo, eps, ea);
  return (int)hipGetLastError();
}

// M <= 64 rows, K % 128 == 0; groups = column groups (SwiGLU: gate/up pairs).
template <int EPI, bool NORM>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int groups, int up_off,
           void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  if (M <= 0 || M > 64 || K % (32 * KC) != 0) return (int)hipErrorInvalidValue;
  switch ((M + 15) / 16) {
    case 1: return launch_mt<1, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 2: return launch_mt<2, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 3: return launch_mt<3, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
    case 4: return launch_mt<4, EPI, NORM>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  }
  return (int)hipErrorInvalidValue;
}

}  // namespace midm
