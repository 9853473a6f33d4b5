// Tall mid-M SwiGLU GEMM: gate_up of a batched prompt chunk (65..384 rows: several peers'
// prompts, or prompts plus riders, in one prefill step).
//
// MEASURED NEGATIVE (round 5, profiles/r5_tall_silu_negative.jsonl; opt-in P2P_TALL_SILU=1):
// correct, but 1.4-1.6x slower than the split-K tiled kernel at 96-384 rows (384: 152 vs 105
// us; hipBLASLt 78).  Streaming the weights once does not pay: at these heights every kernel
// is bound by what one CU takes in (weights + the activation block it re-reads from L2, ~2 MB
// per 128 output columns at K 4096), and this form takes in ~22 GB/s per CU against the tiled
// kernel's ~37 and hipBLASLt's ~45 -- one barrier per 2 k-steps with all rows resident leaves
// too few bytes in flight per wave.
//
//   act[m, c] = silu(rstd[m] * x[m] . Wg[c]) * (rstd[m] * x[m] . Wu[c])
//
// Where the split-K tiled kernel (prefill_gemm.h) loses at these heights (round 5,
// bench/prefill_gemm_bench.py, profiles/r5_prefill_gemm_midm.jsonl): its 256 x 256 tiles
// pad 288-384 rows to 512 (a third of the MFMA work is padding) and its 128- / 192-row tiles
// re-read the weights once per row tile; at 288-384 rows it runs 0.64-0.73x hipBLASLt.
// Here ONE workgroup holds ALL the chunk's rows and 64 output columns (4 gate + the 4
// matching up groups of 16 columns), so every weight byte is streamed exactly once
// (224 workgroups for the 8B gate_up, no split-K, no seam):
//   * the activation chunks (all rows x KC k-steps) go to an LDS ring by LDS-DMA, each
//     wave DMA-ing its share of the fragments, read by all 8 waves;
//   * waves are 2 row halves x 4 column pairs: wave (h, p) streams its gate group and up
//     group (one 1 KiB fragment each per k-step, non-temporal, DW chunks ahead in VGPRs) and
//     multiplies them with the A fragments of its row half -- per k-step and wave MTW A
//     reads feed 2 x MTW MFMAs (one wave per column group would read every A fragment 8
//     times per workgroup, the LDS read port's limit);
//   * gate and up of one output column end in the same lanes: SwiGLU in registers;
//   * RMSNorm: each row's sum of squares from the A fragments already in LDS (m-tile i of a
//     row half by column pair i % 4), rstd applied in the epilogue (gain folded into W).
#include "common.h"

namespace tall {

constexpr int NT = 512;        // 8 waves
constexpr int KC = 2;          // k-steps per chunk
constexpr int LDS_RING = 144 * 1024;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MTW>
struct Cfg {
  static constexpr int MT = 2 * MTW;                 // m-tiles (16 rows each) of the block
  static constexpr int SLOT = MT * KC * 64;          // bf16x8 per ring slot
  static constexpr int NSLOT_MAX = LDS_RING / (SLOT * 16);
  static constexpr int NSLOT = NSLOT_MAX > 6 ? 6 : NSLOT_MAX;
  static constexpr int DA = NSLOT - 2;               // activation chunks in flight ahead
  static constexpr int FPW = MT * KC / 8;            // activation DMA fragments per wave per chunk
  // weight chunks in flight ahead (per wave 2 x KC KiB each; DW + 1 register sets beside
  // the 8 x MTW accumulators: 3 ahead from 8 m-tiles per wave, else 4)
  static constexpr int DW = MTW == 10 ? 2 : (MTW >= 8 ? 3 : 4);
  static_assert(DA >= 1, "ring too small");
  static_assert((MT * KC) % 8 == 0, "fragments per chunk a multiple of the waves");
};

template <int MTW>
__global__ __launch_bounds__(NT) void tall_silu_kernel(const bf16x8* __restrict__ Wt,
                                                       const bf16* __restrict__ X, int ldx, int M,
                                                       int K, int up_off, bf16* __restrict__ out,
                                                       int ldo, float eps) {
  using C = Cfg<MTW>;
  constexpr int MT = C::MT, SLOT = C::SLOT, NSLOT = C::NSLOT, DA = C::DA, FPW = C::FPW, DW = C::DW;
  __shared__ __attribute__((aligned(16))) bf16x8 ring[NSLOT * SLOT];
  __shared__ float ss_row[MT * 16];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rh = w >> 2, cp = w & 3;  // row half, column pair
  const int S = K >> 5, nc = S / KC;
  const int gg = tile * 4 + cp;       // gate group (output columns 16 gg ..)
  const bf16x8* wg = Wt + (size_t)gg * S * 64 + lane;
  const bf16x8* wu = Wt + (size_t)(gg + up_off) * S * 64 + lane;

  // this wave's activation DMA fragments f = w + 8 j of each chunk: m-tile f / KC, k f % KC
  const bf16* asrc[FPW];
  int aoff[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int f = w + 8 * j, i = f / KC, k = f % KC;
    const int row = min(16 * i + (lane & 15), M - 1);
    asrc[j] = X + (size_t)row * ldx + 32 * k + 8 * (lane >> 4);
    aoff[j] = (i * KC + k) * 64;
  }
  auto issue_a = [&](int c) {
    bf16x8* base = ring + (c % NSLOT) * SLOT;
#pragma unroll
    for (int j = 0; j < FPW; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[j] + (size_t)c * KC * 32),
                                       (lds_ptr_t)(base + aoff[j]), 16, 0, 0);
  };
  bf16x8 wr[DW + 1][KC][2];
  auto issue_w = [&](int c, bf16x8(&d)[KC][2]) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      d[k][0] = __builtin_nontemporal_load(wg + (size_t)(c * KC + k) * 64);
      d[k][1] = __builtin_nontemporal_load(wu + (size_t)(c * KC + k) * 64);
    }
  };

  f32x4 acc[MTW][2];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    acc[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int NSS = (MTW + 3) / 4;  // this wave's m-tiles for the row sums: i % 4 == cp
  float ss[NSS];
#pragma unroll
  for (int i = 0; i < NSS; ++i) ss[i] = 0.f;

  auto compute = [&](int c, const bf16x8(&wv)[KC][2]) {
    const bf16x8* base = ring + (c % NSLOT) * SLOT + (rh * MTW * KC) * 64 + lane;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const bf16x8 a = base[(i * KC + k) * 64];
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wv[k][0], acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wv[k][1], acc[i][1], 0, 0, 0);
        if ((i & 3) == cp) ss[i >> 2] = sumsq8(a, ss[i >> 2]);
      }
    }
  };

  // Issue order per step t: A(t + DA) then W(t + DW).  Steady state (t >= DA, every step
  // issues both): A(t) is the later of the two loads chunk t needs, and the loads issued after
  // it are the W(t + DW - DA) of its own step plus DA full steps -- a compile-time count; the
  // first DA steps and the tail (fewer loads issued) wait for everything.
  constexpr int PA = FPW, PW = 2 * KC;
  constexpr int STEADY = PW + DA * (PA + PW);
#pragma unroll
  for (int c = 0; c < DA; ++c)
    if (c < nc) issue_a(c);
#pragma unroll
  for (int c = 0; c < DW; ++c)
    if (c < nc) issue_w(c, wr[c]);
  // unrolled by the DW + 1 register sets, so every set index is a compile-time constant
  for (int tb = 0; tb < nc; tb += DW + 1) {
#pragma unroll
    for (int j = 0; j <= DW; ++j) {
      const int t = tb + j;
      if (t >= nc) break;
      // (t < DA: A(t) and W(t) both came from the prologue, W(t) last -- wait for everything)
      const bool full = t >= DA && t + DW < nc && t + DA < nc;
      if (t + DA < nc) issue_a(t + DA);
      if (t + DW < nc) issue_w(t + DW, wr[(j + DW) % (DW + 1)]);
      if (full && DW >= DA)
        wait_vmcnt<STEADY>();
      else
        wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's DMA part of chunk t is in LDS
      // (the slot A(t + 1 + DA) refills next step held chunk t - 1: every wave finished it
      // before this step's barrier)
      compute(t, wr[j]);
    }
  }

  // ---- row rstd: lanes l, l ^ 16, l ^ 32, l ^ 48 hold row (l & 15) of an m-tile ----
#pragma unroll
  for (int n = 0; n < NSS; ++n) {
    float v = ss[n];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const int i = 4 * n + cp;
    if (i < MTW && lane < 16) ss_row[(rh * MTW + i) * 16 + lane] = v;
  }
  __syncthreads();
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int mt = rh * MTW + i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * mt + 4 * q + j;
      if (m < M) {
        const float rs = rsqrtf(ss_row[16 * mt + 4 * q + j] / (float)K + eps);
        out[(size_t)m * ldo + 16 * gg + r] = f2bf(silu(acc[i][0][j] * rs) * (acc[i][1][j] * rs));
      }
    }
  }
}

template <int MTW>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int N, void* out, int ldo,
           float eps, hipStream_t st) {
  const int n_tiles = N / 2 / 64;
  hipLaunchKernelGGL(tall_silu_kernel<MTW>, dim3(n_tiles), dim3(NT), 0, st, (const bf16x8*)Wt,
                     (const bf16*)X, ldx, M, K, N / 32, (bf16*)out, ldo, eps);
  return (int)hipGetLastError();
}

}  // namespace tall

// 1 if the tall kernel tiles this gate_up shape: M rows (65..384), N = 2 x output columns
// (a multiple of 128), K a multiple of 64.
P2P_API int p2p_tall_silu_ok(int M, int K, int N) {
  return M > 64 && M <= 384 && K % (32 * tall::KC) == 0 && N % 128 == 0 && K >= 32 * tall::KC * 8;
}

// act[M][N / 2] = silu(rstd x Wg^T) * (rstd x Wu^T): Wt fragment-major [N / 16][K / 32][64][8]
// (gate groups first, up groups from N / 32), x [M][ldx] bf16, out [M][ldo] bf16.
P2P_API int p2p_tall_silu(const void* Wt, const void* X, int ldx, int M, int K, int N, void* out,
                          int ldo, float eps, hipStream_t st) {
  if (!p2p_tall_silu_ok(M, K, N)) return (int)hipErrorInvalidValue;
  const int mtw = (M + 31) / 32;
  switch (mtw) {
    case 3:
    case 4: return tall::launch<4>(Wt, X, ldx, M, K, N, out, ldo, eps, st);
    case 5: return tall::launch<6>(Wt, X, ldx, M, K, N, out, ldo, eps, st);
    case 6: return tall::launch<6>(Wt, X, ldx, M, K, N, out, ldo, eps, st);
    case 7:
    case 8: return tall::launch<8>(Wt, X, ldx, M, K, N, out, ldo, eps, st);
    case 9:
    case 10: return tall::launch<10>(Wt, X, ldx, M, K, N, out, ldo, eps, st);
    case 11:
    case 12: return tall::launch<12>(Wt, X, ldx, M, K, N, out, ldo, eps, st);
  }
  return (int)hipErrorInvalidValue;
}
