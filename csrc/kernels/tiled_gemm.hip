// LDS-tiled MFMA GEMM for prefill-sized M (> 64 rows): compute-bound regime.
//
//   out[m, n] = epilogue( rstd[m] * sum_k X[m, k] * W[n, k] )   (same epilogues as
//   the skinny kernel: gemm_epilogue.h -- RoPE/KV write, SwiGLU, residual, argmax)
//
// Block tile 128 (rows) x 128 (cols) x 64 (k), 4 waves in a 2x2 grid, each wave
// 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 accumulators.  Both operands sit in LDS
// in *fragment-major* order, so every MFMA operand is one conflict-free
// ds_read_b128 at lane*16:
//   * W is already stored fragment-major in HBM (ops.tile_weight), so its 16 KiB
//     slab per k-tile is a straight lane-linear copy;
//   * X rows are re-ordered on the way in (register staging): chunk (row, k8)
//     goes to m-tile row/16, k-step k8/4, lane (row%16) + 16*(k8%4).
// Double-buffered LDS, next k-tile prefetched into registers during the MFMAs,
// one barrier per k-tile.  Blocks that stream the same weight columns are
// consecutive after an XCD-aware bijective remap, so they share an XCD's L2.
// NORM: each thread always loads the same 4 rows at the same k offset, so it
// accumulates their sum of squares on the fly; 3 xor-shuffles finish each row.
#include "gemm_epilogue.h"
#include "prefill_gemm.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NT = 256;

template <int EPI, bool NORM>
__global__ __launch_bounds__(NT) void tiled_gemm_kernel(const bf16x8* __restrict__ Wt,
                                                        const bf16* __restrict__ X, int ldx, int M,
                                                        int K, int m_tiles, int n_tiles,
                                                        int up_off, void* __restrict__ out,
                                                        int ldo, float eps, EpiArgs ea) {
  __shared__ __attribute__((aligned(16))) bf16x8 As[2][BM / 16][2][64];
  __shared__ __attribute__((aligned(16))) bf16x8 Bs[2][BN / 16][2][64];
  __shared__ float ss_row[BM];

  const int nb = m_tiles * n_tiles;
  const int b = xcd_remap(blockIdx.x, nb);
  const int mt_i = b % m_tiles, nt_i = b / m_tiles;
  const int m0 = mt_i * BM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int S = K >> 5;
  const int nk = K / BK;

  // global group index of B slab gi (0..7) of this n-tile
  auto group_of = [&](int gi) -> int {
    if constexpr (EPI == EPI_SILU) return gi < 4 ? nt_i * 4 + gi : nt_i * 4 + (gi - 4) + up_off;
    return nt_i * 8 + gi;
  };

  // ---- staging assignment ----
  // B: chunk c = tid + 256*i  ->  gi = c >> 7, ks = (c >> 6) & 1, ln = c & 63
  const bf16x8* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    bsrc[i] = Wt + ((size_t)group_of(c >> 7) * S + ((c >> 6) & 1)) * 64 + (c & 63);
  }
  // A: row = tid/8 + 32*i, k8 = tid%8
  const int k8 = tid & 7;
  const bf16* asrc[4];
  bool aval[4];
  int adst[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    aval[i] = m0 + row < M;
    asrc[i] = X + (size_t)(aval[i] ? m0 + row : 0) * ldx + k8 * 8;
    adst[i] = ((row >> 4) * 2 + (k8 >> 2)) * 64 + (row & 15) + 16 * (k8 & 3);
  }
  float ss[4] = {0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[4], rb[4];
  auto load_regs = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) rb[i] = bsrc[i][(size_t)kt * 2 * 64];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      ra[i] = aval[i] ? *reinterpret_cast<const bf16x8*>(asrc[i] + kt * BK) : zero_bf16x8();
  };
  auto store_lds = [&](int buf) {
    bf16x8* a = &As[buf][0][0][0];
    bf16x8* bb = &Bs[buf][0][0][0];
#pragma unroll
    for (int i = 0; i < 4; ++i) bb[tid + NT * i] = rb[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[adst[i]] = ra[i];
      if constexpr (NORM) ss[i] = sumsq8(ra[i], ss[i]);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // wave's B slabs: SILU -> gate {2wn, 2wn+1} and up {4+2wn, 4+2wn+1}; else {4wn..4wn+3}
  int bgi[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr (EPI == EPI_SILU) bgi[j] = j < 2 ? 2 * wn + j : 4 + 2 * wn + (j - 2);
    else bgi[j] = 4 * wn + j;
  }

  load_regs(0);
  store_lds(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_regs(kt + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = As[cur][wm * 4 + i][ks][lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = Bs[cur][bgi[j]][ks][lane];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_lds(cur ^ 1);
    __syncthreads();
  }

  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (k8 == 0) ss_row[(tid >> 3) + 32 * i] = v;
    }
    __syncthreads();
  }

  // ---- epilogue ----
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int rl = wm * 64 + i * 16 + q * 4 + jj;
      const int m = m0 + rl;
      const bool valid = m < M;
      float scale = 1.f;
      if constexpr (NORM) scale = rsqrtf(ss_row[rl] / (float)K + eps);
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          epi_store<EPI>(m, valid, nt_i * 4 + 2 * wn + j, r, acc[i][j][jj] * scale,
                         acc[i][j + 2][jj] * scale, out, ldo, ea);
      } else if constexpr (EPI == EPI_QKV_ROPE) {
        float2 c = float2{1.f, 0.f};
        int slot = -1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int g = nt_i * 8 + 4 * wn + j;
          const int kk = g & 7;
          const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
          if (valid) {
            c = ea.cs[(size_t)ea.pos[m] * 64 + dd];
            slot = ea.slots[m];
          }
          epi_store<EPI>(m, valid, g, r, acc[i][j][jj] * scale, 0.f, out, ldo, ea, c, slot);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          epi_store<EPI>(m, valid, nt_i * 8 + 4 * wn + j, r, acc[i][j][jj] * scale, 0.f, out, ldo,
                         ea);
      }
    }
  }
}

template <int EPI, bool NORM>
int launch_tiled(const void* Wt, const void* X, int ldx, int M, int K, int n_tiles, int up_off,
                 void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  const int m_tiles = (M + BM - 1) / BM;
  hipLaunchKernelGGL((tiled_gemm_kernel<EPI, NORM>), dim3(m_tiles * n_tiles), dim3(NT), 0, st,
                     (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off, out,
                     ldo, eps, ea);
  return (int)hipGetLastError();
}

}  // namespace

// Same contract as p2p_skinny_gemm (+ the fused qkv/argmax variants through `ea`
// fields set by the wrappers below) for any M; requires K % 64 == 0 and N % 128 == 0
// (SiLU: (N/2) % 64 == 0).  Returns hipErrorInvalidValue if the shape does not tile.
static int g_tiled_version = 2;  // 2 = LDS-DMA 8-wave kernel (prefill_gemm.h), 1 = register-staged

// Benchmarks / A-B tests: version 1|2, tile 0 (heuristic) or 1..7 (256x256, 128x256, 128x128,
// 64x128, 64x256, 320x128, 192x128, 192x256),
// splitk 0 (heuristic), 1 (off) or a forced K-slice count.
// 256x256 prefill tiles: 1 = phased pipeline (default), 0 = the 2-stage kernel (A/B).
P2P_API void p2p_prefill_phased(int on) { pgemm::g_phased = on ? 1 : 0; }

// Deep LDS pipeline (A/B): 0 = shallow stages only, 1 = deep variant for grids of at most
// one block per CU (default), 2 = deep variant always.
// Precomputed per-row rstd for normed prefill GEMMs (A/B): 1 = on (default), 0 = in-loop sums.
P2P_API void p2p_prefill_pre_rstd(int on) { pgemm::g_pre_rstd = on ? 1 : 0; }
// 192 x 256 tiles for SwiGLU-width projections in the 384-row bucket (A/B): 1 = on (default)
P2P_API void p2p_prefill_tile8(int on) { pgemm::g_tile8 = on ? 1 : 0; }

P2P_API void p2p_prefill_deep(int mode) { pgemm::g_deep = (mode >= 0 && mode <= 2) ? mode : 1; }

// Split-K reduction mode (A/B): 1 = parallel (every slice reduces a share, default where
// residency allows), 0 = serial (the last arriving slice reduces the whole tile).
P2P_API void p2p_tiled_split_parallel(int on) { pgemm::g_split_parallel = on ? 1 : 0; }

// The split-K fault word of each device (see prefill_gemm.h): allocated once, never moved.
static int* g_fault_word[64];

extern "C" int* p2p_split_fault_word_ptr(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!g_fault_word[dev]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) return nullptr;  // no allocation inside a capture
    int* p = nullptr;
    if (hipMalloc(&p, 256) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, 256, st) != hipSuccess) return nullptr;
    g_fault_word[dev] = p;
  }
  return g_fault_word[dev];
}

// Nonzero if a parallel split-K slice (tiled or wide kernel) waited past its spin bound since
// the last call (its tile's output is invalid); clears the word.  Synchronises the device.
P2P_API int p2p_tiled_split_fault() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_fault_word[dev]) return 0;
  int* w = g_fault_word[dev];
  int v = 0;
  if (hipMemcpy(&v, w, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (v) {
    const int z = 0;
    (void)hipMemcpy(w, &z, sizeof(int), hipMemcpyHostToDevice);
  }
  return v;
}

P2P_API void p2p_tiled_gemm_config(int version, int tile, int splitk) {
  if (version == 1 || version == 2) g_tiled_version = version;
  g_prefill_tile = (tile >= 0 && tile <= 8) ? tile : 0;
  pgemm::g_splitk = splitk >= 0 ? splitk : 0;
}

static int tiled_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                          int norm, void* out, int ldo, float eps, const EpiArgs& ea,
                          hipStream_t st) {
  if (g_tiled_version == 2) {
    const int e = prefill_dispatch(Wt, X, ldx, M, K, N, epi, norm, out, ldo, eps, ea, st);
    if (e != (int)hipErrorInvalidValue) return e;
  }
  if (M <= 0 || K % BK != 0 || N % BN != 0) return (int)hipErrorInvalidValue;
  const int n_tiles = N / BN;
  const int up_off = (epi == EPI_SILU) ? N / 32 : 0;
  switch (epi) {
    case EPI_STORE:
      return norm ? launch_tiled<EPI_STORE, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st)
                  : launch_tiled<EPI_STORE, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st);
    case EPI_RESID:
      return launch_tiled<EPI_RESID, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st);
    case EPI_SILU:
      return launch_tiled<EPI_SILU, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st);
    case EPI_F32:
      return norm ? launch_tiled<EPI_F32, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st)
                  : launch_tiled<EPI_F32, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st);
    case EPI_QKV_ROPE:
      return launch_tiled<EPI_QKV_ROPE, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st);
    case EPI_ARGMAX:
      return launch_tiled<EPI_ARGMAX, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st);
  }
  return (int)hipErrorInvalidValue;
}

P2P_API int p2p_tiled_gemm(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                           int norm, void* out, int ldo, float eps, hipStream_t stream) {
  if (epi == EPI_QKV_ROPE || epi == EPI_ARGMAX) return (int)hipErrorInvalidValue;
  EpiArgs ea = {};
  return tiled_dispatch(Wt, X, ldx, M, K, N, epi, norm, out, ldo, eps, ea, stream);
}

P2P_API int p2p_tiled_gemm_qkv_rope(const void* Wt, const void* X, int ldx, int M, int K, int Hq,
                                    int Hkv, const int* pos, const int* slots, const void* cos_sin,
                                    void* q_out, int ldq, void* k_cache, void* v_cache, float eps,
                                    hipStream_t stream) {
  EpiArgs ea = {};
  ea.pos = pos;
  ea.slots = slots;
  ea.cs = (const float2*)cos_sin;
  ea.q_out = (bf16*)q_out;
  ea.ldq = ldq;
  ea.kc = (bf16*)k_cache;
  ea.vc = (bf16*)v_cache;
  ea.Hq = Hq;
  ea.Hkv = Hkv;
  return tiled_dispatch(Wt, X, ldx, M, K, (Hq + 2 * Hkv) * HD, EPI_QKV_ROPE, 1, nullptr, 0, eps,
                        ea, stream);
}

P2P_API int p2p_tiled_gemm_argmax(const void* Wt, const void* X, int ldx, int M, int K, int N,
                                  unsigned long long* keys, int col_offset, float eps,
                                  hipStream_t stream) {
  EpiArgs ea = {};
  ea.col_offset = col_offset;
  return tiled_dispatch(Wt, X, ldx, M, K, N, EPI_ARGMAX, 1, keys, 0, eps, ea, stream);
}

// Grouped (MoE) expert GEMM on the LDS-tiled MFMA kernel (prefill_gemm.h, MOE mode):
// one launch, grid (m-tiles x n-tiles, experts); see p2p_grouped_gemm for the
// arguments.  Every expert's weights stream once per m-tile of its own rows.
P2P_API int p2p_grouped_gemm_tiled(const void* Wt, long long w_stride, int n_experts,
                                   const int* cnt, const int* rows, int rows_stride, int x_div,
                                   const float* row_w, const void* X, int ldx, int max_rows,
                                   int K, int N, int epi, int norm, void* out, int ldo, float eps,
                                   hipStream_t stream) {
  using namespace pgemm;
  if (n_experts <= 0 || max_rows <= 0 || K % pgemm::BK || N % 128) return (int)hipErrorInvalidValue;
  EpiArgs ea = {};
  ea.moe_cnt = cnt;
  ea.moe_rows = rows;
  ea.rows_stride = rows_stride;
  ea.x_div = x_div > 0 ? x_div : 1;
  ea.row_w = row_w;
  ea.w_stride = w_stride;
  ea.n_experts = n_experts;
  // normed (w13): the token rows' rstd once (X has max_rows rows), then the NORM = false
  // kernel with the rstd applied per slot in the epilogue (prefill_gemm.h, pre_rstd)
  if (norm && (epi == EPI_SILU || epi == EPI_STORE)) {
    if (const float* r = pre_rstd(X, ldx, max_rows, K, eps, stream)) {
      if (epi == EPI_SILU && N % 256) return (int)hipErrorInvalidValue;
      ea.rstd_in = r;
      return epi == EPI_SILU
                 ? launch_moe<128, 128, EPI_SILU, false>(Wt, X, ldx, max_rows, K, N, N / 32, out,
                                                         ldo, eps, ea, stream)
                 : launch_moe<128, 128, EPI_STORE, false>(Wt, X, ldx, max_rows, K, N, 0, out, ldo,
                                                          eps, ea, stream);
    }
  }
  if (epi == EPI_SILU) {
    if (!norm || N % 256) return (int)hipErrorInvalidValue;
    return launch_moe<128, 128, EPI_SILU, true>(Wt, X, ldx, max_rows, K, N, N / 32, out, ldo, eps,
                                                ea, stream);
  }
  if (epi == EPI_STORE)
    return norm ? launch_moe<128, 128, EPI_STORE, true>(Wt, X, ldx, max_rows, K, N, 0, out, ldo,
                                                        eps, ea, stream)
                : launch_moe<128, 128, EPI_STORE, false>(Wt, X, ldx, max_rows, K, N, 0, out, ldo,
                                                         eps, ea, stream);
  return (int)hipErrorInvalidValue;
}
