// Prefill GEMM v2: 8-wave MFMA GEMM with direct global->LDS (LDS-DMA) staging.
//
//   out[m, n] = epilogue( rstd[m] * sum_k X[m, k] * W[n, k] )   (gemm_epilogue.h)
//
// Tile BM x BN x 64 (BM, BN in {128, 256}), 512 threads = 8 waves in a 2 (M) x 4 (N)
// grid; wave tile (BM/2) x (BN/4) of v_mfma_f32_16x16x32_bf16 accumulators.
// Both operands are staged with `global_load_lds_dwordx4` (one wave-instruction
// = one 1 KiB MFMA fragment block): the LDS image is fragment-major, so every
// operand read is a lane-linear, conflict-free ds_read_b128 and no VGPRs or
// VALU are spent on staging:
//   * W is fragment-major in HBM already (ops.tile_weight): a block is 1 KiB
//     contiguous;
//   * X is row-major: lane l of a block fetches X[row0 + (l&15)][k0 + 8(l>>4) ..]
//     (per-lane source address, lane-linear destination).
// Two LDS stages (2 x (BM+BN) x 64 bf16 <= 128 KiB, one __shared__ array):
// stage kt+1 is in flight while the MFMAs consume stage kt; one barrier per
// k-tile.  Blocks sharing a weight n-tile are consecutive after the XCD remap.
// NORM: the waves of column 0 also square the A fragments they read; a lane
// sees 8 of every 32 k of one row, 3 shuffles finish the row's sum.
#pragma once
#include <algorithm>

#include "gemm_epilogue.h"

namespace pgemm {

constexpr int BK = 64;
constexpr int NT = 512;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct SplitArgs {
  int splitk;          // K slices per output tile (1 = no split)
  f32x4* slab;         // [tiles][splitk][FM*FN][NT] partial accumulators
  float* ss_slab;      // [tiles][splitk][BM] partial row sums of squares
  unsigned* counters;  // [tiles], zeroed before the launch
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Waits until at most `pending` x L of this thread's LDS-DMA loads are in flight.
template <int L, int STAGES>
__device__ __forceinline__ void wait_tiles(int pending) {
  if constexpr (STAGES >= 4) {
    if (pending >= 2) { wait_vmcnt<2 * L>(); return; }
  }
  if constexpr (STAGES >= 3) {
    if (pending >= 1) { wait_vmcnt<L>(); return; }
  }
  wait_vmcnt<0>();
}

// MOE: grouped expert GEMM (ea.moe_*): blockIdx.y = local expert e, whose rows are the
// slots rows[e][i] (i < min(cnt[e], M)); A row of slot s = X[s / x_div], output row s
// (scaled by row_w[s]).  m-tiles past the expert's count exit at once, so one launch
// covers every expert at any M and each expert's weights stream once per m-tile.
template <int BM, int BN, int EPI, bool NORM, bool SPLIT, int STAGES, bool MOE = false>
__global__ __launch_bounds__(NT) void prefill_gemm_kernel(const bf16x8* __restrict__ Wt,
                                                          const bf16* __restrict__ X, int ldx,
                                                          int M, int K, int m_tiles, int n_tiles,
                                                          int up_off, void* __restrict__ out,
                                                          int ldo, float eps, EpiArgs ea,
                                                          SplitArgs sp) {
  constexpr int FM = BM / 32;        // 16-row fragments per wave (2 x 4 wave grid)
  constexpr int FN = BN / 64;        // 16-col groups per wave
  constexpr int AB = BM / 16 * 2;    // A fragment blocks per stage (x 1 KiB)
  constexpr int BB = BN / 16 * 2;    // B fragment blocks per stage
  constexpr int STAGE = (AB + BB) * 64;  // bf16x8 per stage
  constexpr int AI = AB / 8, BI = BB / 8;  // blocks per wave per stage
  constexpr int L = AI + BI;               // LDS-DMA instructions per thread per stage
  static_assert(AB % 8 == 0 && BB % 8 == 0, "tile");
  static_assert(FM >= 1 && FN >= 2, "tile");
  __shared__ __attribute__((aligned(16))) bf16x8 lds[STAGES * STAGE];

  const int splitk = SPLIT ? sp.splitk : 1;
  const int nb = m_tiles * n_tiles * splitk;
  const int b = xcd_remap(blockIdx.x, nb);
  // a tile's K slices are consecutive (same XCD: the reducer reads them from its L2)
  const int tile = b / splitk, split = b % splitk;
  const int mt_i = tile % m_tiles, nt_i = tile / m_tiles;
  const int m0 = mt_i * BM;
  const int* mrows = nullptr;
  if constexpr (MOE) {
    const int e = blockIdx.y;
    M = min(ea.moe_cnt[e], M);
    if (m0 >= M) return;  // block-uniform: this expert has fewer rows
    Wt += (size_t)e * ea.w_stride;
    mrows = ea.moe_rows + (size_t)e * ea.rows_stride;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int S = K >> 5;
  const int nk_all = K / BK;
  const int kt0 = split * nk_all / splitk, kt1 = (split + 1) * nk_all / splitk;
  const int n = kt1 - kt0;

  auto group_of = [&](int gi) -> int {  // LDS group slot -> global 16-col group
    if constexpr (EPI == EPI_SILU) {
      constexpr int H = BN / 32;
      return gi < H ? nt_i * H + gi : nt_i * H + (gi - H) + up_off;
    }
    return nt_i * (BN / 16) + gi;
  };

  // ---- per-lane DMA sources (k offsets added per k-tile) ----
  const bf16* asrc[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int blk = w + 8 * i;  // = mi * 2 + ks
    const int mi = blk >> 1, ks = blk & 1;
    int row = m0 + 16 * mi + (lane & 15);
    row = row < M ? row : M - 1;
    if constexpr (MOE) row = mrows[row] / ea.x_div;
    asrc[i] = X + (size_t)row * ldx + 32 * ks + 8 * (lane >> 4);
  }
  const bf16x8* bsrc[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int blk = w + 8 * i;  // = gi * 2 + ks
    bsrc[i] = Wt + ((size_t)group_of(blk >> 1) * S + (blk & 1)) * 64 + lane;
  }

  auto issue = [&](int kt, int st) {
    bf16x8* base = lds + st * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + kt * BK),
                                       (lds_ptr_t)(base + (w + 8 * i) * 64), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + (size_t)kt * 2 * 64),
                                       (lds_ptr_t)(base + (AB + w + 8 * i) * 64), 16, 0, 0);
  };

  int bgi[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    if constexpr (EPI == EPI_SILU) {
      constexpr int H = FN / 2;
      bgi[j] = j < H ? wn * H + j : BN / 32 + wn * H + (j - H);
    } else {
      bgi[j] = wn * FN + j;
    }
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) ss[i] = 0.f;
  const bool do_ss = NORM && wn == 0;

  // ---- STAGES-deep LDS-DMA pipeline: counted vmcnt + raw barriers, so the
  // younger stages stay in flight across the barrier (no vmcnt(0) drain) ----
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < n) issue(kt0 + t, t);
  for (int t = 0; t < n; ++t) {
    wait_tiles<L, STAGES>(min(STAGES - 2, n - 1 - t));  // tile t landed (this thread's part)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                       // ... and every other wave's part
    if (t + STAGES - 1 < n) issue(kt0 + t + STAGES - 1, (t + STAGES - 1) % STAGES);
    const bf16x8* sa = lds + (t % STAGES) * STAGE;
    const bf16x8* sb = sa + AB * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = sb[(bgi[j] * 2 + ks) * 64 + lane];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = sa[((wm * FM + i) * 2 + ks) * 64 + lane];
      // keep the MFMA cluster together against the co-resident wave (guide T5)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (do_ss) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = (float)af[i][e];
            ss[i] = fmaf(v, v, ss[i]);
          }
      }
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // every wave done reading the stages before LDS is reused below

  // ---- row rstd (NORM): column-0 waves publish through LDS (stages are free now) ----
  float* ss_row = reinterpret_cast<float*>(lds);
  if constexpr (NORM) {
    if (wn == 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        float v = ss[i];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) {
          if constexpr (SPLIT)
            sp.ss_slab[((size_t)tile * splitk + split) * BM + wm * (BM / 2) + 16 * i + lane] = v;
          else
            ss_row[wm * (BM / 2) + 16 * i + lane] = v;
        }
      }
    }
    if constexpr (!SPLIT) __syncthreads();
  }
  if constexpr (SPLIT) {
    // split-K hand-off (agent-scope release/acquire through a per-tile ticket):
    // every slice stores its fp32 partial tile, the last arriver reduces all
    // slices in slice order (deterministic) and runs the epilogue.
    f32x4* my = sp.slab + ((size_t)tile * splitk + split) * (FM * FN) * NT;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) my[(i * FN + j) * NT + tid] = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds) + BM;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(&sp.counters[tile], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      *flag = (t == (unsigned)splitk - 1);
    }
    __syncthreads();
    if (!*flag) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const f32x4* base = sp.slab + (size_t)tile * splitk * (FM * FN) * NT;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < splitk; ++s2) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] += base[((size_t)s2 * FM * FN + i * FN + j) * NT + tid];
    }
    if constexpr (NORM) {
      if (tid < BM) {
        float t = 0.f;
        for (int s2 = 0; s2 < splitk; ++s2) t += sp.ss_slab[((size_t)tile * splitk + s2) * BM + tid];
        ss_row[tid] = t;
      }
      __syncthreads();
    }
    // every slice has arrived: re-arm the ticket for the next launch (the workspace
    // counters are zeroed once at allocation, so no per-launch memset node is needed)
    if (tid == 0) sp.counters[tile] = 0;
  }

  // ---- epilogue ----
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int rl = wm * (BM / 2) + 16 * i + 4 * q + jj;
      int m = m0 + rl;
      const bool valid = m < M;
      float scale = 1.f;
      if constexpr (NORM) scale = rsqrtf(ss_row[rl] / (float)K + eps);
      if constexpr (MOE) {
        m = valid ? mrows[m] : 0;  // output row = the slot
        if (ea.row_w && valid) scale *= ea.row_w[m];
      }
      if constexpr (EPI == EPI_SILU) {
        constexpr int H = FN / 2;
#pragma unroll
        for (int j = 0; j < H; ++j)
          epi_store<EPI>(m, valid, nt_i * (BN / 32) + wn * H + j, r, acc[i][j][jj] * scale,
                         acc[i][j + H][jj] * scale, out, ldo, ea);
      } else if constexpr (EPI == EPI_QKV_ROPE) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int g = nt_i * (BN / 16) + bgi[j];
          const int kk = g & 7;
          const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
          float2 c = float2{1.f, 0.f};
          int slot = -1;
          if (valid) {
            c = ea.cs[(size_t)ea.pos[m] * 64 + dd];
            slot = ea.slots[m];
          }
          epi_store<EPI>(m, valid, g, r, acc[i][j][jj] * scale, 0.f, out, ldo, ea, c, slot);
        }
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j)
          epi_store<EPI>(m, valid, nt_i * (BN / 16) + bgi[j], r, acc[i][j][jj] * scale, 0.f, out,
                         ldo, ea);
      }
    }
  }
}

// split-K workspace (device, grown on demand outside graph capture)
struct SplitWs {
  void* buf = nullptr;
  size_t bytes = 0;
};
static SplitWs g_split_ws;

// ticket counters: a fixed region at the end of the workspace, zeroed when the
// workspace is (re)allocated and re-armed by each tile's last arriver
constexpr size_t kCounterBytes = 64 * 1024;  // 16384 tiles

// A grown workspace never frees the previous buffer: a hipGraph captured earlier (the
// decode graph of a mid-M batch bucket routed to this kernel) holds its address and its
// ticket counters and replays against it for the life of the process.  Growth is
// geometric, so the retired buffers total less than the live one.
static bool split_ws(size_t bytes, hipStream_t st, char** out) {
  bytes += kCounterBytes;
  if (g_split_ws.bytes < bytes) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) return false;  // cannot allocate while capturing
    const size_t want = std::max(bytes, 2 * g_split_ws.bytes);
    void* buf = nullptr;
    if (hipMalloc(&buf, want) != hipSuccess) return false;
    if (hipMemsetAsync(buf, 0, want, st) != hipSuccess) return false;
    g_split_ws.buf = buf;  // the old buffer stays allocated (see above)
    g_split_ws.bytes = want;
  }
  *out = (char*)g_split_ws.buf;
  return true;
}

static int g_splitk = 0;  // 0 = heuristic, 1 = never split, >1 = forced

// LDS stages per tile shape.  Measured on MI355X (bench/prefill_gemm_bench.py): the
// 64-row tiles are latency-bound streams and want 3-4 stages in flight; the 128/256-row
// tiles are MFMA-bound and lose more to 1-block/CU occupancy than they gain from depth.
template <int BM, int BN>
constexpr int stages_for() {
  if constexpr (BM >= 128) return 2;
  return BN <= 128 ? 4 : 3;
}

template <int BM, int BN, int EPI, bool NORM>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off, void* out,
           int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  constexpr int STAGES = stages_for<BM, BN>();
  const int m_tiles = (M + BM - 1) / BM;
  const int n_tiles = N / BN;
  const int tiles = m_tiles * n_tiles;
  const int nk = K / BK;
  // too few tiles to fill 256 CUs: split K so every CU gets work (>= 4 k-tiles per slice)
  // (measured on MI355X at 8B shapes: ~400 blocks, >= 16 k-tiles per slice)
  int splitk = g_splitk ? g_splitk : std::min(8, std::max(1, std::min(400 / tiles, nk / 16)));
  splitk = std::max(1, std::min(splitk, nk / 4));
  if (splitk > 1 && (size_t)tiles * sizeof(unsigned) <= kCounterBytes) {
    constexpr int FM = BM / 32, FN = BN / 64;
    const size_t slab = (size_t)tiles * splitk * FM * FN * NT * sizeof(f32x4);
    const size_t ssb = (size_t)tiles * splitk * BM * sizeof(float);
    char* ws = nullptr;
    if (split_ws(slab + ssb, st, &ws)) {
      // counters live at the END of the workspace at a fixed offset from the end so a
      // grown workspace keeps them zeroed; see split_ws
      SplitArgs sp{splitk, (f32x4*)ws, (float*)(ws + slab),
                   (unsigned*)(ws + g_split_ws.bytes - kCounterBytes)};
      hipLaunchKernelGGL((prefill_gemm_kernel<BM, BN, EPI, NORM, true, STAGES>),
                         dim3(tiles * splitk), dim3(NT), 0, st, (const bf16x8*)Wt,
                         (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off, out, ldo, eps, ea, sp);
      return (int)hipGetLastError();
    }
  }
  SplitArgs none{1, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL((prefill_gemm_kernel<BM, BN, EPI, NORM, false, STAGES>), dim3(tiles), dim3(NT), 0,
                     st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off,
                     out, ldo, eps, ea, none);
  return (int)hipGetLastError();
}

template <int BM, int BN, int EPI, bool NORM>
int launch_moe(const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off, void* out,
               int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  constexpr int STAGES = stages_for<BM, BN>();
  const int m_tiles = (M + BM - 1) / BM;
  const int n_tiles = N / BN;
  SplitArgs none{1, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL((prefill_gemm_kernel<BM, BN, EPI, NORM, false, STAGES, true>),
                     dim3(m_tiles * n_tiles, ea.n_experts), dim3(NT), 0, st, (const bf16x8*)Wt,
                     (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off, out, ldo, eps, ea, none);
  return (int)hipGetLastError();
}

template <int EPI, bool NORM>
int launch_tile(int tile, const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off,
                void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  switch (tile) {
    case 1: return launch<256, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 2: return launch<128, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 3: return launch<128, 128, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 4: return launch<64, 128, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 5: return launch<64, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
  }
  return (int)hipErrorInvalidValue;
}

// Largest tile that still gives about one block per CU; N must divide.  M <= 64
// uses the 64-row tiles (no MFMA work or DMA on padding rows beyond one tile).
int pick_tile(int M, int N) {
  if (M <= 64) return N % 128 == 0 ? 4 : 0;
  const int cand[3][3] = {{1, 256, 256}, {2, 128, 256}, {3, 128, 128}};
  int best = 0;
  for (auto& c : cand) {
    if (N % c[2]) continue;
    const long blocks = (long)((M + c[1] - 1) / c[1]) * (N / c[2]);
    if (!best) best = c[0];
    if (blocks >= 200) return c[0];
    best = c[0];
  }
  return best;
}

}  // namespace pgemm

static int g_prefill_tile = 0;  // 0 = heuristic (benchmarks can force 1..3)

// Used by the p2p_tiled_gemm* entry points (tiled_gemm.hip).  Returns
// hipErrorInvalidValue if the shape does not tile (caller falls back).
static int prefill_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                         int norm, void* out, int ldo, float eps, const EpiArgs& ea,
                         hipStream_t st) {
  using namespace pgemm;
  if (M <= 0 || K % BK) return (int)hipErrorInvalidValue;
  int tile = g_prefill_tile ? g_prefill_tile : pick_tile(M, N);
  const int bn = (tile == 3 || tile == 4) ? 128 : 256;
  if (!tile || N % bn) return (int)hipErrorInvalidValue;
  const int up_off = (epi == EPI_SILU) ? N / 32 : 0;
  switch (epi) {
    case EPI_STORE:
      return norm ? launch_tile<EPI_STORE, true>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st)
                  : launch_tile<EPI_STORE, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case EPI_RESID:
      return launch_tile<EPI_RESID, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case EPI_SILU:
      return launch_tile<EPI_SILU, true>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case EPI_F32:
      return norm ? launch_tile<EPI_F32, true>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st)
                  : launch_tile<EPI_F32, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case EPI_QKV_ROPE:
      return launch_tile<EPI_QKV_ROPE, true>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case EPI_ARGMAX:
      return launch_tile<EPI_ARGMAX, true>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
  }
  return (int)hipErrorInvalidValue;
}
