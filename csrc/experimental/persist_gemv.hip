// Persistent decode GEMV (M <= 16 rows, bf16 weights): one workgroup of 4 waves per CU
// walks a balanced list of 16-column units and keeps the weight stream going across them.
//
// The skinny kernel (skinny_gemm.hip) launches one workgroup per column group and lets the
// dispatcher balance them; each workgroup's stream starts cold, and the launch ends with
// a tail of partially filled CUs.  Measured inside the persistent decode engine
// (decode_engine.hip, profiles/r4_decode_engine_negative.jsonl) the same weight streams
// ran faster when a workgroup issues the next unit's first 16 k-steps per wave (16 KiB)
// as soon as the current unit's last batch is in flight: gate_up ~32 us and down ~16 us
// per 8B layer against the skinny kernel's 37.4 / 19.8 us.  This kernel is that stream
// on its own -- no hand-offs -- as a launch-code candidate the autotuner times against the
// skinny / mid-M kernels (ops.gemm.PERSIST_FLAG).
//
// Units (same fragment-major weights as the skinny kernel, [N / 16][K / 32][64][8]):
//   EPI_RESID / EPI_STORE / EPI_F32 : column group g (16 weight rows)
//   EPI_SILU (gate rows then up rows): half pair (p, hf) -- lanes r < 8 hold gate column
//     8 hf + r of pair p, lanes r >= 8 the up column 8 hf + r - 8, so one MFMA B operand
//     carries both halves of SwiGLU for 8 output columns (a lane shuffle pairs them)
// Workgroup b takes units b, b + NB, ...; the k-steps of a unit are split over the 4 waves
// (each a multiple of U = 8 and >= PFK = 16: K % 1024 == 0) and summed in LDS by wave 0,
// which runs the epilogue while the other waves stream the next unit.
#include "gemm_epilogue.h"

namespace {

constexpr int W = 4;
constexpr int NT = W * 64;
constexpr int PFK = 16;
constexpr int U = 8;

struct PStream {
  const bf16x8* wp;
  int s0, s1;
};

__device__ __forceinline__ PStream unit_stream(const bf16x8* Wt, int u, int K, bool silu, int NP) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int S = K >> 5;
  int g = u, li = lane;
  if (silu) {  // half pair (u >> 1, u & 1)
    const int p = u >> 1, hf = u & 1;
    g = r < 8 ? p : p + NP;
    li = q * 16 + 8 * hf + (r & 7);
  }
  PStream st;
  st.wp = Wt + (size_t)g * S * 64 + li;
  st.s0 = (S * w) / W;
  st.s1 = (S * (w + 1)) / W;
  return st;
}

__device__ __forceinline__ void prefetch(const PStream& st, bf16x8 (&pf)[PFK]) {
#pragma unroll
  for (int i = 0; i < PFK; ++i) pf[i] = __builtin_nontemporal_load(st.wp + (size_t)(st.s0 + i) * 64);
}

template <bool NORM>
__device__ __forceinline__ void gemv(const PStream& st, const PStream& next, bool has_next,
                                     bf16x8 (&pf)[PFK], const bf16* X, int ldx, int M, f32x4& acc,
                                     float& ss) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const bool xv = r < M;
  const bf16* xp = X + (size_t)(xv ? r : 0) * ldx + 8 * q;
  auto step = [&](const bf16x8& bw, int at) {
    const bf16x8 a = xv ? *reinterpret_cast<const bf16x8*>(xp + at * 32) : zero_bf16x8();
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw, acc, 0, 0, 0);
    if constexpr (NORM) ss = sumsq8(a, ss);
  };
  acc = f32x4{0.f, 0.f, 0.f, 0.f};
  ss = 0.f;
  const int s1 = st.s1;
  bf16x8 bA[U], bB[U];
  auto load = [&](bf16x8(&bw)[U], int at) {
#pragma unroll
    for (int u = 0; u < U; ++u) bw[u] = __builtin_nontemporal_load(st.wp + (size_t)(at + u) * 64);
  };
  auto compute = [&](const bf16x8(&bw)[U], int at) {
#pragma unroll
    for (int u = 0; u < U; ++u) step(bw[u], at + u);
  };
  int s = st.s0 + PFK;
  if (s < s1) load(bA, s);
#pragma unroll
  for (int i = 0; i < PFK; ++i) step(pf[i], st.s0 + i);
  bool pend = has_next;
  if (s >= s1 && pend) {
    prefetch(next, pf);
    pend = false;
  }
  while (s < s1) {
    const int sB = s + U;
    if (sB < s1) {
      load(bB, sB);
    } else if (pend) {
      prefetch(next, pf);
      pend = false;
    }
    compute(bA, s);
    if (sB >= s1) break;
    s = sB + U;
    if (s < s1) {
      load(bA, s);
    } else if (pend) {
      prefetch(next, pf);
      pend = false;
    }
    compute(bB, sB);
  }
}

template <int EPI, bool NORM>
__global__ __launch_bounds__(NT) void persist_gemv_kernel(const bf16x8* __restrict__ Wt,
                                                          const bf16* __restrict__ X, int ldx,
                                                          int M, int K, int units, int NP,
                                                          void* __restrict__ out, int ldo,
                                                          float eps) {
  __shared__ float red[2][W - 1][4][64];
  __shared__ float red_ss[2][W][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int b = blockIdx.x, NB = gridDim.x;
  constexpr bool SILU = EPI == EPI_SILU;
  bf16x8 pf[PFK];
  if (b < units) prefetch(unit_stream(Wt, b, K, SILU, NP), pf);
  int rb = 0;
  for (int u = b; u < units; u += NB) {
    const PStream st = unit_stream(Wt, u, K, SILU, NP);
    const bool more = u + NB < units;
    f32x4 acc;
    float ss;
    gemv<NORM>(st, unit_stream(Wt, more ? u + NB : u, K, SILU, NP), more, pf, X, ldx, M, acc, ss);
    // split-K sum over the waves (double-buffered: the other waves go straight on)
    if (w > 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red[rb][w - 1][j][lane] = acc[j];
    }
    if constexpr (NORM) {
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (q == 0) red_ss[rb][w][r] = ss;
    }
    __syncthreads();
    const int rr = rb;
    rb ^= 1;
    if (w != 0) continue;
#pragma unroll
    for (int ww = 0; ww < W - 1; ++ww)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += red[rr][ww][j][lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 4 * q + j;
      float rstd = 1.f;
      if constexpr (NORM) {
        float t = 0.f;
#pragma unroll
        for (int ww = 0; ww < W; ++ww) t += red_ss[rr][ww][m];
        rstd = rsqrtf(t / (float)K + eps);
      }
      const float v = acc[j] * rstd;
      if constexpr (SILU) {
        const float up = __shfl_xor(v, 8, 64);
        const int col = (u >> 1) * 16 + 8 * (u & 1) + r;
        if (m < M && r < 8) reinterpret_cast<bf16*>(out)[(size_t)m * ldo + col] = f2bf(silu(v) * up);
      } else if constexpr (EPI == EPI_RESID) {
        if (m < M) {
          bf16* o = reinterpret_cast<bf16*>(out) + (size_t)m * ldo + u * 16 + r;
          *o = f2bf((float)*o + v);
        }
      } else if constexpr (EPI == EPI_STORE) {
        if (m < M) reinterpret_cast<bf16*>(out)[(size_t)m * ldo + u * 16 + r] = f2bf(v);
      } else {
        if (m < M) reinterpret_cast<float*>(out)[(size_t)m * ldo + u * 16 + r] = v;
      }
    }
  }
}

int n_cus() {
  static int c = 0;
  if (!c) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      c = 256;
  }
  return c;
}

template <int EPI, bool NORM>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int units, int NP, void* out,
           int ldo, float eps, int grid, hipStream_t st) {
  hipLaunchKernelGGL((persist_gemv_kernel<EPI, NORM>), dim3(grid), dim3(NT), 0, st,
                     (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, units, NP, out, ldo, eps);
  return (int)hipGetLastError();
}

}  // namespace

// 1 if the persistent GEMV runs this shape (bf16 weights, M <= 16).
extern "C" int p2p_persist_gemv_ok(int M, int K, int N, int epi) {
  if (M < 1 || M > 16 || K % (32 * W * U) || K / 32 / W < PFK || N % 16) return 0;
  if (epi == EPI_SILU) return N % 32 == 0;
  return epi == EPI_RESID || epi == EPI_STORE || epi == EPI_F32;
}

// grid_mult: workgroups per CU (0 = 1).  Called by the skinny dispatcher for launch codes
// with PERSIST_FLAG (ops.gemm).
extern "C" int p2p_persist_gemv(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                                int norm, void* out, int ldo, float eps, int grid_mult,
                                hipStream_t st) {
  if (!p2p_persist_gemv_ok(M, K, N, epi)) return (int)hipErrorInvalidValue;
  const int units = N / 16;  // SILU: half pairs = N / 16 as well (N = 2 F)
  const int NP = N / 32;
  int grid = n_cus() * (grid_mult > 0 ? grid_mult : 1);
  if (grid > units) grid = units;
  switch (epi) {
    case EPI_RESID:
      if (norm) return (int)hipErrorInvalidValue;
      return launch<EPI_RESID, false>(Wt, X, ldx, M, K, units, NP, out, ldo, eps, grid, st);
    case EPI_SILU:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_SILU, true>(Wt, X, ldx, M, K, units, NP, out, ldo, eps, grid, st);
    case EPI_STORE:
      return norm ? launch<EPI_STORE, true>(Wt, X, ldx, M, K, units, NP, out, ldo, eps, grid, st)
                  : launch<EPI_STORE, false>(Wt, X, ldx, M, K, units, NP, out, ldo, eps, grid, st);
    case EPI_F32:
      return norm ? launch<EPI_F32, true>(Wt, X, ldx, M, K, units, NP, out, ldo, eps, grid, st)
                  : launch<EPI_F32, false>(Wt, X, ldx, M, K, units, NP, out, ldo, eps, grid, st);
  }
  return (int)hipErrorInvalidValue;
}
