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
#include "lds_pipe.h"

// The split-K fault word of the current device (tiled_gemm.hip): one int per device,
// allocated with the first split-K workspace and never moved, so a captured graph, the
// Python check (ops.gemm.tiled_split_fault) and the native loop (EngineLoop::set_aux_fault)
// all see the same word.  nullptr while a capture is in progress and it does not exist yet.
extern "C" int* p2p_split_fault_word_ptr(hipStream_t st);

namespace pgemm {

constexpr int BK = 64;
constexpr int NT = 512;
typedef int v4i __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct SplitArgs {
  int splitk;          // K slices per output tile (1 = no split)
  f32x4* slab;         // [tiles][splitk][FM*FN][NT] partial accumulators
  float* ss_slab;      // [tiles][splitk][BM] partial row sums of squares
  unsigned* counters;  // [tiles], zeroed before the launch
  // parallel reduction (every slice reduces 8/splitk of the tile's waves; all slices of a
  // tile must be resident together -- the host enables it only for grids <= the CU count):
  unsigned* gen;       // [tiles] generation, bumped by each tile's last arriver
  int* err;            // set if a slice waited past the spin bound (results invalid)
  int parallel;
};

constexpr long long SPLIT_SPIN_TICKS = 20000000;  // 200 ms at the 100 MHz constant clock

// Write-through (sc1) 16-byte store / load through a raw buffer resource (aux 16 = sc1):
// hand-off payload that needs no release fence and is read past stale L1/L2 copies
// (cdna_hip_programming.md Guideline 16, R1).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFFF,
                                           0x00020000);
}
__device__ __forceinline__ void store_sc1(__amdgpu_buffer_rsrc_t r, int off, const f32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, off, 0, 16);
}
__device__ __forceinline__ f32x4 load_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// Tile coordinates of linear tile index t in GROUP_M-row bands: consecutive indices walk
// GROUP_M m-tiles of one n-tile, then the next n-tile.  After xcd_remap an XCD's ~32
// concurrent blocks (one per CU) therefore cover 8 m-tiles x 4 n-tiles -- per k-step 12
// distinct 32 KiB operand slices instead of 33 with m innermost over every m-tile (L2 hit
// rate ~50 % -> ~80 %), and each XCD streams its A rows once instead of once per n-tile.
// Identical to (t % m_tiles, t / m_tiles) for m_tiles <= GROUP_M.
constexpr int GROUP_M = 8;
__device__ __forceinline__ void grouped_tile(int t, int m_tiles, int n_tiles, int& mt, int& nt) {
  const int per_group = GROUP_M * n_tiles;
  const int g = t / per_group, first = g * GROUP_M;
  const int gm = min(m_tiles - first, GROUP_M);
  const int r = t - g * per_group;
  mt = first + r % gm;
  nt = r / gm;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Waits until at most `pending` x L of this thread's LDS-DMA loads are in flight.
template <int L, int STAGES>
__device__ __forceinline__ void wait_tiles(int pending) {
  if constexpr (STAGES >= 6) {
    if (pending >= 4) { wait_vmcnt<4 * L>(); return; }
  }
  if constexpr (STAGES >= 5) {
    if (pending >= 3) { wait_vmcnt<3 * L>(); return; }
  }
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
  int mt_i, nt_i;
  grouped_tile(tile, m_tiles, n_tiles, mt_i, nt_i);
  const int m0 = mt_i * BM;
  const int* mrows = nullptr;
  if constexpr (MOE) {
    const int e = blockIdx.y;
    M = min(ea.moe_cnt[e], M);
    if (m0 >= M) return;  // block-uniform: this expert has fewer rows
    Wt += (size_t)e * ea.w_stride;
    mrows = ea.moe_rows + (size_t)e * ea.rows_stride;
  }
  // rows' RMSNorm rstd precomputed by row_rstd_kernel (ea.rstd_in): the host launches the
  // NORM = false instantiation, so no sums of squares ride in the k loop (they cost
  // 12-22 % of the GEMM, profiles/r2_norm_cost.jsonl); applied in the epilogue
  const bool pre = !NORM && ea.rstd_in != nullptr;
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

  // asm DMA + asm LDS reads (lds_pipe.h): with the builtins the compiler put vmcnt(0)
  // before every stage read, draining the STAGES-deep pipeline at every k-tile
  auto issue = [&](int kt, int st) {
    bf16x8* base = lds + st * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i) ldsp::dma_lds<16>(asrc[i] + kt * BK, base + (w + 8 * i) * 64);
#pragma unroll
    for (int i = 0; i < BI; ++i) ldsp::dma_lds<16>(bsrc[i] + (size_t)kt * 2 * 64, base + (AB + w + 8 * i) * 64);
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
      for (int j = 0; j < FN; ++j) bfr[j] = ldsp::lds_rd(sb + (bgi[j] * 2 + ks) * 64 + lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = ldsp::lds_rd(sa + ((wm * FM + i) * 2 + ks) * 64 + lane);
      ldsp::lds_wait(af, bfr);
      // keep the MFMA cluster together against the co-resident wave (guide T5)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (NORM) {  // RMSNorm sums: fragment i by wave wn == i % 4 (VALU spread)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          if ((i & 3) != wn) continue;
          ss[i] = sumsq8(af[i], ss[i]);
        }
      }
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // every wave done reading the stages before LDS is reused below

  // ---- row rstd (NORM): column-0 waves publish through LDS (stages are free now) ----
  float* ss_row = reinterpret_cast<float*>(lds);
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if ((i & 3) != wn) continue;
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) {
        if constexpr (SPLIT)
          __hip_atomic_store(&sp.ss_slab[((size_t)tile * splitk + split) * BM + wm * (BM / 2) + 16 * i + lane],
                             v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through
        else
          ss_row[wm * (BM / 2) + 16 * i + lane] = v;
      }
    }
    if constexpr (!SPLIT) __syncthreads();
  }
  // ---- epilogue of one wave's accumulators (wave grid position wm_, wn_) ----
  const int r = lane & 15, q = lane >> 4;
  auto epilogue = [&](int wm_, int wn_, const f32x4 (&ac)[FM][FN], auto&& scale_of) {
    int bg[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (EPI == EPI_SILU) {
        constexpr int H = FN / 2;
        bg[j] = j < H ? wn_ * H + j : BN / 32 + wn_ * H + (j - H);
      } else {
        bg[j] = wn_ * FN + j;
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      // one fragment row's epilogue operands as one batch (residual values; the rows'
      // positions -> (cos, sin) and KV slots): per element, between the stores they may
      // alias, they were FN x 4 dependent round trips per fragment row
      float resv[4][FN];
      float2 csv[4][FN];
      int slotv[4];
      if constexpr (EPI == EPI_RESID || EPI == EPI_QKV_ROPE) {
        int posv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int m = m0 + wm_ * (BM / 2) + 16 * i + 4 * q + jj;
          posv[jj] = 0;
          slotv[jj] = -1;
          if constexpr (EPI == EPI_QKV_ROPE && !MOE)
            if (m < M) {
              posv[jj] = ea.pos[m];
              slotv[jj] = ea.slots[m];
            }
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            resv[jj][j] = 0.f;
            if constexpr (EPI == EPI_RESID && !MOE)
              if (m < M) resv[jj][j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + (nt_i * (BN / 16) + bg[j]) * 16 + r];
          }
        }
        if constexpr (EPI == EPI_QKV_ROPE && !MOE) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              const int g = nt_i * (BN / 16) + bg[j];
              const int kk = g & 7;
              const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
              const bool ok = m0 + wm_ * (BM / 2) + 16 * i + 4 * q + jj < M;
              csv[jj][j] = ok ? ea.cs[(size_t)posv[jj] * 64 + dd] : float2{1.f, 0.f};
            }
        }
      }
      float scv[4];  // the rows' rstd (loads, with the operands above)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) scv[jj] = scale_of(i, jj);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int rl = wm_ * (BM / 2) + 16 * i + 4 * q + jj;
        int m = m0 + rl;
        const bool valid = m < M;
        float scale = scv[jj];
        if constexpr (MOE) {
          m = valid ? mrows[m] : 0;  // output row = the slot
          if (ea.row_w && valid) scale *= ea.row_w[m];
        }
        if constexpr (EPI == EPI_SILU) {
          constexpr int H = FN / 2;
#pragma unroll
          for (int j = 0; j < H; ++j)
            epi_store<EPI>(m, valid, nt_i * (BN / 32) + wn_ * H + j, r, ac[i][j][jj] * scale,
                           ac[i][j + H][jj] * scale, out, ldo, ea);
        } else if constexpr (EPI == EPI_QKV_ROPE && !MOE) {
#pragma unroll
          for (int j = 0; j < FN; ++j)
            epi_store<EPI>(m, valid, nt_i * (BN / 16) + bg[j], r, ac[i][j][jj] * scale, 0.f, out,
                           ldo, ea, csv[jj][j], valid ? slotv[jj] : -1);
        } else if constexpr (EPI == EPI_RESID && !MOE) {
#pragma unroll
          for (int j = 0; j < FN; ++j)
            if (valid)
              reinterpret_cast<bf16*>(out)[(size_t)m * ldo + (nt_i * (BN / 16) + bg[j]) * 16 + r] =
                  f2bf(resv[jj][j] + ac[i][j][jj] * scale);
        } else {
#pragma unroll
          for (int j = 0; j < FN; ++j)
            epi_store<EPI>(m, valid, nt_i * (BN / 16) + bg[j], r, ac[i][j][jj] * scale, 0.f, out,
                           ldo, ea);
        }
      }
    }
  };
  auto rstd_of = [&](float t) { return rsqrtf(t / (float)K + eps); };
  auto rstd_pre = [&](int rl) {
    if (!pre) return 1.f;
    int m = min(m0 + rl, M - 1);
    if constexpr (MOE) m = mrows[m] / ea.x_div;  // the slot's token row of X
    return ea.rstd_in[m];
  };

  if constexpr (SPLIT) {
    f32x4* my = sp.slab + ((size_t)tile * splitk + split) * (FM * FN) * NT;
    // (the 256x256 tile keeps the serial reduction: a second set of 128 accumulator
    // registers for the shared reduction would spill its main loop)
    if (BM * BN <= 128 * 256 && sp.parallel) {
      // ---- parallel split-K: write-through slabs, one generation flip per tile, then
      // every slice reduces and stores 8/splitk of the tile's waves (no serial reducer,
      // no release fence) ----
      const __amdgpu_buffer_rsrc_t rsl = raw_rsrc(sp.slab);
      const size_t tile_v = (size_t)tile * splitk * (FM * FN) * NT;  // f32x4 index of slice 0
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          store_sc1(rsl, (int)((tile_v + ((size_t)split * FM * FN + i * FN + j) * NT + tid) * 16),
                    acc[i][j]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
      __syncthreads();
      if (tid == 0) {
        const unsigned g0 = __hip_atomic_load(&sp.gen[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // read the generation BEFORE arriving
        const unsigned t = __hip_atomic_fetch_add(&sp.counters[tile], 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        if (t == (unsigned)splitk - 1) {
          (void)__hip_atomic_exchange(&sp.counters[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // re-armed before the flip
          __hip_atomic_store(&sp.gen[tile], g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          const long long t0 = wall_clock64();
          while (__hip_atomic_load(&sp.gen[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
            if (wall_clock64() - t0 > SPLIT_SPIN_TICKS) {
              __hip_atomic_store(sp.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
      }
      __syncthreads();
      constexpr int kWavesPerTile = NT / 64;
      const int vw_n = kWavesPerTile / splitk;  // host guarantees splitk | 8
      if (w >= vw_n) return;
      const int vw = split * vw_n + w;  // the tile wave whose accumulators this wave finishes
      // acc is dead after the slab stores: it becomes the total (one fragment row of
      // loads in flight at a time keeps the 256x256 tile inside its register budget)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < splitk; ++s2) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          f32x4 part[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j)
            part[j] = load_sc1(rsl, (int)((tile_v + ((size_t)s2 * FM * FN + i * FN + j) * NT +
                                           vw * 64 + lane) * 16));
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] += part[j];
        }
      }
      epilogue(vw >> 2, vw & 3, acc, [&](int i, int jj) {
        const int rl = (vw >> 2) * (BM / 2) + 16 * i + 4 * q + jj;
        if constexpr (!NORM) return rstd_pre(rl);
        float t = 0.f;
        for (int s2 = 0; s2 < splitk; ++s2)
          t += __hip_atomic_load(&sp.ss_slab[((size_t)tile * splitk + s2) * BM + rl],
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return rstd_of(t);
      });
      return;
    }
    // ---- serial split-K: agent-scope release/acquire through a per-tile ticket; every
    // slice stores its fp32 partial tile, the last arriver reduces all slices in slice
    // order (deterministic) and runs the epilogue ----
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

  epilogue(wm, wn, acc, [&](int i, int jj) {
    const int rl = wm * (BM / 2) + 16 * i + 4 * q + jj;
    if constexpr (!NORM) return rstd_pre(rl);
    return rstd_of(ss_row[rl]);
  });
}

// ---------------------------------------------------------------------------------
// 256 x 256 tile, phased pipeline (cdna_hip_programming.md §5 "The 256² 8-phase
// template", re-derived for the fragment-major LDS image).  A K-tile (BK = 64) is
// staged as four 16 KiB units -- A0/A1 (the two 64-row halves of every wave's 128
// rows) and B0/B1 (the two 32-column halves of every wave's 64 columns) -- and
// consumed in four phases of 16 MFMAs per wave, one C quadrant each:
//   p0: (A0, B0)   p1: (A0, B1)   p2: (A1, B1)   p3: (A1, B0)
// (B0 fragments stay in registers from p0 to p3).  Each phase issues ONE unit's
// LDS-DMA (2 instructions per thread), in the order
//   p0: A1(t+1)   p1: A0(t+2)   p2: B0(t+2)   p3: B1(t+2)
// so a unit is re-staged one phase after its last read (behind that phase's
// lgkmcnt(0) + barrier) and lands about five phases (> 1 K-tile) before it is
// read: the counted vmcnt before a reading phase leaves 10 DMA instructions in
// flight in the steady state and never drains the queue inside the loop.
template <int EPI, bool NORM>
__global__ __launch_bounds__(NT) void prefill_gemm8_kernel(const bf16x8* __restrict__ Wt,
                                                           const bf16* __restrict__ X, int ldx,
                                                           int M, int K, int m_tiles, int n_tiles,
                                                           int up_off, void* __restrict__ out,
                                                           int ldo, float eps, EpiArgs ea) {
  constexpr int BM = 256, BN = 256, FM = 8, FN = 4;
  constexpr int AB = 32, BB = 32, STAGE = (AB + BB) * 64;
  __shared__ __attribute__((aligned(16))) bf16x8 lds[2 * STAGE];
  const bool pre = !NORM && ea.rstd_in != nullptr;  // rows' rstd precomputed (see above)

  const int nb = m_tiles * n_tiles;
  const int b = xcd_remap(blockIdx.x, nb);
  int mt_i, nt_i;
  grouped_tile(b, m_tiles, n_tiles, mt_i, nt_i);
  const int m0 = mt_i * BM;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int S = K >> 5;
  const int n = K / BK;

  auto group_of = [&](int gi) -> int {
    if constexpr (EPI == EPI_SILU) {
      constexpr int H = BN / 32;
      return gi < H ? nt_i * H + gi : nt_i * H + (gi - H) + up_off;
    }
    return nt_i * (BN / 16) + gi;
  };
  int bgi[FN];  // LDS B group slot of the wave's column fragment j
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    if constexpr (EPI == EPI_SILU) {
      bgi[j] = j < 2 ? wn * 2 + j : BN / 32 + wn * 2 + (j - 2);
    } else {
      bgi[j] = wn * FN + j;
    }
  }
  // this thread's two DMA instructions of each unit: list index l = w + 8k (k = 0, 1)
  //   A unit qa (full 128-B lines): 8 rows (l>>3)*128 + 64qa + 8(l&7) .. +7, lane ->
  //     row + (lane>>3), LDS chunk p = lane&7 holding global chunk p ^ (row & 7)
  //     (XOR swizzle: the A-fragment ds_read_b128 of 16 rows is conflict-free)
  //   B unit qb: l = (wnb*2 + j2)*2 + ks -> slot of (wn = wnb, j = 2qb + j2)
  const bf16* asrc[2][2];
  int aslot[2][2];  // A: LDS offset in bf16x8 units
  const bf16x8* bsrc[2][2];
  int bslot[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int l = w + 8 * k, ks = l & 1, x = l >> 1;
      const int R = (l >> 3) * 128 + 64 * q + 8 * (l & 7) + (lane >> 3);
      int row = m0 + R;
      row = row < M ? row : M - 1;
      asrc[q][k] = X + (size_t)row * ldx + 8 * ((lane & 7) ^ (R & 7));
      aslot[q][k] = R * 8 + (lane & 7) - lane;  // + lane (per-lane DMA slot) = R*8 + p
      const int wnb = x >> 1, j = 2 * q + (x & 1);
      int gs;
      if constexpr (EPI == EPI_SILU) gs = j < 2 ? wnb * 2 + j : BN / 32 + wnb * 2 + (j - 2);
      else gs = wnb * FN + j;
      bsrc[q][k] = Wt + ((size_t)group_of(gs) * S + ks) * 64 + lane;
      bslot[q][k] = AB + gs * 2 + ks;
    }
  auto issue_a = [&](int q, int kt) {
    bf16x8* base = lds + (kt & 1) * STAGE;
#pragma unroll
    for (int k = 0; k < 2; ++k)  // wave-uniform LDS base: lane 0's slot (lane*16 B added by HW)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[q][k] + kt * BK),
                                       (lds_ptr_t)(base + __builtin_amdgcn_readfirstlane(aslot[q][k])),
                                       16, 0, 0);
  };
  auto issue_b = [&](int q, int kt) {
    bf16x8* base = lds + (kt & 1) * STAGE;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[q][k] + (size_t)kt * 2 * 64),
                                       (lds_ptr_t)(base + bslot[q][k] * 64), 16, 0, 0);
  };
  auto wait_units = [&](int units) {  // at most `units` of this thread's units in flight
    switch (units) {
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<2>(); break;
      case 2: wait_vmcnt<4>(); break;
      case 3: wait_vmcnt<6>(); break;
      case 4: wait_vmcnt<8>(); break;
      default: wait_vmcnt<10>(); break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) ss[i] = 0.f;

  // prologue: A0 B0 B1 A1 of tile 0, A0 B0 B1 of tile 1 (the steady-state order)
  issue_a(0, 0);
  issue_b(0, 0);
  issue_b(1, 0);
  issue_a(1, 0);
  if (n > 1) {
    issue_a(0, 1);
    issue_b(0, 1);
    issue_b(1, 1);
  }
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];
  const int ar = lane & 15, aq = lane >> 4;
  auto read_a = [&](const bf16x8* sa, int q) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)  // row (rg*16 + ar), global chunk 4ks + aq, swizzled
        af[i][ks] = sa[((wm * FM + 4 * q + i) * 16 + ar) * 8 + ((4 * ks + aq) ^ (ar & 7))];
    if constexpr (NORM) {  // RMSNorm sums: fragment i of a quadrant by wave wn == i
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i != wn) continue;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          ss[4 * q + i] = sumsq8(af[i][ks], ss[4 * q + i]);
      }
    }
  };
  auto read_b = [&](const bf16x8* sb, int q, bf16x8(&bfr)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bfr[j][ks] = sb[(bgi[2 * q + j] * 2 + ks) * 64 + lane];
  };
  auto mma = [&](int qa, int qb, const bf16x8(&bfr)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qa + i][2 * qb + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[i][ks], bfr[j][ks], acc[4 * qa + i][2 * qb + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  for (int t = 0; t < n; ++t) {
    const bf16x8* sa = lds + (t & 1) * STAGE;
    const bf16x8* sb = sa + AB * 64;
    const int more1 = t + 1 < n, more2 = t + 2 < n;
    // p0: A0, B0
    wait_units(2 + 3 * more1);
    read_a(sa, 0);
    read_b(sb, 0, bf0);
    if (more1) issue_a(1, t + 1);
    mma(0, 0, bf0);
    // p1: B1 (A0 kept)
    wait_units(1 + 4 * more1);
    read_b(sb, 1, bf1);
    if (more2) issue_a(0, t + 2);
    mma(0, 1, bf1);
    // p2: A1 (B1 kept)
    wait_units(4 * more1 + more2);
    read_a(sa, 1);
    if (more2) issue_b(0, t + 2);
    mma(1, 1, bf1);
    // p3: (A1, B0), both in registers
    if (more2) issue_b(1, t + 2);
    mma(1, 0, bf0);
  }
  wait_vmcnt<0>();
  __syncthreads();

  float* ss_row = reinterpret_cast<float*>(lds);
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if ((i & 3) != wn) continue;  // fragment i's rows were squared by wave (wm, i & 3)
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) ss_row[wm * (BM / 2) + 16 * i + lane] = v;
    }
    __syncthreads();
  }
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    // one fragment row's epilogue operands as one batch (see prefill_gemm_kernel)
    float resv[4][FN];
    float2 csv[4][FN];
    int slotv[4];
    if constexpr (EPI == EPI_RESID || EPI == EPI_QKV_ROPE) {
      int posv[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int m = m0 + wm * (BM / 2) + 16 * i + 4 * q + jj;
        posv[jj] = 0;
        slotv[jj] = -1;
        if constexpr (EPI == EPI_QKV_ROPE)
          if (m < M) {
            posv[jj] = ea.pos[m];
            slotv[jj] = ea.slots[m];
          }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          resv[jj][j] = 0.f;
          if constexpr (EPI == EPI_RESID)
            if (m < M) resv[jj][j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + (nt_i * (BN / 16) + bgi[j]) * 16 + r];
        }
      }
      if constexpr (EPI == EPI_QKV_ROPE) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int g = nt_i * (BN / 16) + bgi[j];
            const int kk = g & 7;
            const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
            const bool ok = m0 + wm * (BM / 2) + 16 * i + 4 * q + jj < M;
            csv[jj][j] = ok ? ea.cs[(size_t)posv[jj] * 64 + dd] : float2{1.f, 0.f};
          }
      }
    }
    float scv[4];  // the rows' precomputed rstd, loaded with the operands above
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      scv[jj] = pre ? ea.rstd_in[min(m0 + wm * (BM / 2) + 16 * i + 4 * q + jj, M - 1)] : 1.f;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int rl = wm * (BM / 2) + 16 * i + 4 * q + jj;
      const int m = m0 + rl;
      const bool valid = m < M;
      float scale = scv[jj];
      if constexpr (NORM) scale = rsqrtf(ss_row[rl] / (float)K + eps);
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          epi_store<EPI>(m, valid, nt_i * (BN / 32) + wn * 2 + j, r, acc[i][j][jj] * scale,
                         acc[i][j + 2][jj] * scale, out, ldo, ea);
      } else if constexpr (EPI == EPI_QKV_ROPE) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
          epi_store<EPI>(m, valid, nt_i * (BN / 16) + bgi[j], r, acc[i][j][jj] * scale, 0.f, out,
                         ldo, ea, csv[jj][j], valid ? slotv[jj] : -1);
      } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
          if (valid)
            reinterpret_cast<bf16*>(out)[(size_t)m * ldo + (nt_i * (BN / 16) + bgi[j]) * 16 + r] =
                f2bf(resv[jj][j] + acc[i][j][jj] * scale);
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
    if (!p2p_split_fault_word_ptr(st)) return false;
    g_split_ws.buf = buf;  // the old buffer stays allocated (see above)
    g_split_ws.bytes = want;
  }
  *out = (char*)g_split_ws.buf;
  return true;
}

static int g_splitk = 0;  // 0 = heuristic, 1 = never split, >1 = forced
static int g_split_parallel = 1;  // parallel split-K reduction where residency allows

// CUs of the current device (cached per device): the parallel reduction needs every slice
// of a tile resident at once, so it is used only for grids of at most one block per CU.
static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cached[dev] = n > 0 ? n : -1;
  }
  return cached[dev] > 0 ? cached[dev] : 0;
}

// LDS stages per tile shape.  Measured on MI355X (bench/prefill_gemm_bench.py): the
// 64-row tiles are latency-bound streams and want 3-4 stages in flight; the 128/256-row
// tiles are MFMA-bound at large M, where two blocks share a CU and hide each other's
// loads, and lose more to 1-block/CU occupancy than they gain from depth.
template <int BM, int BN>
constexpr int stages_for() {
  if constexpr (BM >= 128) return 2;
  return BN <= 128 ? 4 : 3;
}

// Deep variant for grids of at most one block per CU (mid-M prompts, split-K tiles): one
// resident block per CU is bound by its own bytes in flight (Little's law: one 128x128
// stage is 32 KiB, a k-tile's MFMAs take ~0.05 us, an L2/MALL round trip ~1.5 us), so the
// block keeps as many stages in flight as 160 KiB of LDS holds.
// The 64-row tiles already run 3-4 stages and measured 4-9 % slower with 4-6
// (profiles/r2_prefill_gemm_deep_stages.jsonl): deep applies from 128 rows.
template <int BM, int BN>
constexpr int deep_stages_for() {
  if constexpr (BM < 128) return stages_for<BM, BN>();
  constexpr int stage_bytes = (BM + BN) * BK * 2;
  constexpr int most = (160 * 1024) / stage_bytes;
  return most > 6 ? 6 : (most < 2 ? 2 : most);
}

// 0 = shallow stages only, 1 = deep variant when the grid is <= one block per CU (default),
// 2 = deep variant always (A/B).
static int g_deep = 1;

template <int BM, int BN, int EPI, bool NORM, int STAGES>
int launch_stages(const void* Wt, const void* X, int ldx, int M, int K, int m_tiles, int n_tiles,
                  int up_off, void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st,
                  int splitk, char* ws, int par) {
  const int tiles = m_tiles * n_tiles;
  if (splitk > 1) {
    constexpr int FM = BM / 32, FN = BN / 64;
    const size_t slab = (size_t)tiles * splitk * FM * FN * NT * sizeof(f32x4);
    // counters live at the END of the workspace at a fixed offset from the end so a
    // grown workspace keeps them zeroed; see split_ws.  Layout of that region (u32):
    // [0, n/2) arrival tickets, [n/2, n-1) generations, [n-1] the fault word.
    unsigned* ctr = (unsigned*)(ws + g_split_ws.bytes - kCounterBytes);
    constexpr size_t nw = kCounterBytes / sizeof(unsigned);
    int* fw = p2p_split_fault_word_ptr(st);
    SplitArgs sp{splitk, (f32x4*)ws, (float*)(ws + slab), ctr, ctr + nw / 2,
                 fw ? fw : (int*)(ctr + nw - 1), par};
    hipLaunchKernelGGL((prefill_gemm_kernel<BM, BN, EPI, NORM, true, STAGES>),
                       dim3(tiles * splitk), dim3(NT), 0, st, (const bf16x8*)Wt,
                       (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off, out, ldo, eps, ea, sp);
    return (int)hipGetLastError();
  }
  SplitArgs none{1, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  hipLaunchKernelGGL((prefill_gemm_kernel<BM, BN, EPI, NORM, false, STAGES>), dim3(tiles), dim3(NT), 0,
                     st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off,
                     out, ldo, eps, ea, none);
  return (int)hipGetLastError();
}

template <int BM, int BN, int EPI, bool NORM>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off, void* out,
           int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  constexpr int SHALLOW = stages_for<BM, BN>();
  constexpr int DEEP = deep_stages_for<BM, BN>();
  const int m_tiles = (M + BM - 1) / BM;
  const int n_tiles = N / BN;
  const int tiles = m_tiles * n_tiles;
  const int nk = K / BK;
  const int cus = cu_count();
  const bool deep_auto = DEEP > SHALLOW && g_deep == 1 && cus > 0 && tiles <= cus;
  // too few tiles to fill 256 CUs: split K so every CU gets work (>= 4 k-tiles per slice)
  // (measured on MI355X at 8B shapes: ~400 blocks, >= 16 k-tiles per slice); the deep
  // variant keeps the grid at one block per CU instead (power-of-two slices <= CUs/tiles)
  int splitk;
  if (g_splitk) {
    splitk = g_splitk;
  } else if (deep_auto) {
    const int cap = std::min(8, std::max(1, std::min(cus / tiles, nk / 16)));
    splitk = 1;
    while (splitk * 2 <= cap) splitk *= 2;
  } else {
    splitk = std::min(8, std::max(1, std::min(400 / tiles, nk / 16)));
  }
  splitk = std::max(1, std::min(splitk, nk / 4));
  char* ws = nullptr;
  int par = 0;
  if (splitk > 1 && (size_t)tiles * sizeof(unsigned) < kCounterBytes / 2) {
    constexpr int FM = BM / 32, FN = BN / 64;
    const size_t slab = (size_t)tiles * splitk * FM * FN * NT * sizeof(f32x4);
    const size_t ssb = (size_t)tiles * splitk * BM * sizeof(float);
    if (!(split_ws(slab + ssb, st, &ws) && slab + ssb < 0x7FFFFFFF)) splitk = 1;
    par = g_split_parallel && (8 % splitk) == 0 && cus > 0 && tiles * splitk <= cus;
  } else {
    splitk = 1;
  }
  const bool deep = DEEP > SHALLOW && (g_deep == 2 || (g_deep == 1 && cus > 0 && tiles * splitk <= cus));
  if constexpr (DEEP > SHALLOW) {
    if (deep)
      return launch_stages<BM, BN, EPI, NORM, DEEP>(Wt, X, ldx, M, K, m_tiles, n_tiles, up_off, out,
                                                    ldo, eps, ea, st, splitk, ws, par);
  }
  return launch_stages<BM, BN, EPI, NORM, SHALLOW>(Wt, X, ldx, M, K, m_tiles, n_tiles, up_off, out,
                                                   ldo, eps, ea, st, splitk, ws, par);
}

template <int BM, int BN, int EPI, bool NORM>
int launch_moe(const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off, void* out,
               int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  constexpr int STAGES = stages_for<BM, BN>();
  const int m_tiles = (M + BM - 1) / BM;
  const int n_tiles = N / BN;
  SplitArgs none{1, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  hipLaunchKernelGGL((prefill_gemm_kernel<BM, BN, EPI, NORM, false, STAGES, true>),
                     dim3(m_tiles * n_tiles, ea.n_experts), dim3(NT), 0, st, (const bf16x8*)Wt,
                     (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off, out, ldo, eps, ea, none);
  return (int)hipGetLastError();
}

static int g_phased = 1;  // 256x256 tiles: phased pipeline (1) or the 2-stage kernel (0)

template <int EPI, bool NORM>
int launch_phased(const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off,
                  void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  const int m_tiles = (M + 255) / 256, n_tiles = N / 256;
  hipLaunchKernelGGL((prefill_gemm8_kernel<EPI, NORM>), dim3(m_tiles * n_tiles), dim3(NT), 0, st,
                     (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, m_tiles, n_tiles, up_off, out,
                     ldo, eps, ea);
  return (int)hipGetLastError();
}

template <int EPI, bool NORM>
int launch_tile(int tile, const void* Wt, const void* X, int ldx, int M, int K, int N, int up_off,
                void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st) {
  switch (tile) {
    case 1:
      // the phased kernel has no split-K: take it where the tiles already fill the chip
      if (g_phased && (g_splitk == 1 || (!g_splitk && ((M + 255) / 256) * (N / 256) >= 160)))
        return launch_phased<EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
      return launch<256, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 2: return launch<128, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 3: return launch<128, 128, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 4: return launch<64, 128, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 5: return launch<64, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 6: return launch<320, 128, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 7: return launch<192, 128, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
    case 8: return launch<192, 256, EPI, NORM>(Wt, X, ldx, M, K, N, up_off, out, ldo, eps, ea, st);
  }
  return (int)hipErrorInvalidValue;
}

// Largest tile that still gives about one block per CU; N must divide.  M <= 64
// uses the 64-row tiles (no MFMA work or DMA on padding rows beyond one tile).
// 129-192 and 257-320 rows (batched chat prompts: 8 peers x ~36-44 tokens) take ONE
// m-tile of 192 / 320 rows: at these M the tiles are bound by the per-CU LDS-DMA fill
// rate, so the bytes staged per useful output decide, and 128-row tiles would stream
// every weight column 2-3 times (25 % padding) while 256x256 pads up to 44 %.
static int g_tile8 = 1;  // the 192 x 256 gate_up pick below (A/B switch: p2p_prefill_tile8)
static int pick_tile(int M, int N, int K) {
  if (M <= 64) return N % 128 == 0 ? 4 : 0;
  // (one-m-tile 384 / 448-row tiles for 321-448 rows measured 1.1-1.3x SLOWER than the
  // 128x128 split-K / phased 256x256 picks below and were removed:
  // profiles/r3_prefill_tiles_384_448.jsonl)
  // (257-320 rows: the one-m-tile 320x128 pays on the wide gate_up only; o_proj at 288 rows
  // took 64 us with it and 39 with 128x128 split-K, cold weights:
  // profiles/r5_prefill_gemm_cold_vs_hipblaslt.jsonl)
  // (129-192 rows, N <= 4096 with K <= 4096 -- o_proj: 32 one-m-tile tiles take split-K 4 at
  // most, 128 blocks; 128 x 128 split-K 4 fills the 256 CUs: 30.8 vs 37.7 us for llama3.1-8B
  // o_proj at 192 rows, cold weights, profiles/r6_prefill_gemm_sweep_cold.jsonl)
  const bool short_k = N <= 4096 && K <= 4096;
  if (N % 128 == 0 && ((M > 128 && M <= 192 && !short_k) || (M > 256 && M <= 320 && N >= 16384)))
    return M <= 192 ? 7 : 6;
  // qkv-width projections (4096 < N <= 8192) in the 384-row bucket (8 peers x ~44-token
  // prompts): 192 x 128 tiles, split-K 2 by launch()'s rule -- llama3.1-8B qkv+RoPE 49.2 vs
  // 57.0 us with 128 x 128 (144 tiles on 256 CUs, unsplit), cold weights
  // (profiles/r6_prefill_gemm_384_cold.jsonl); o_proj / down (N = 4096) and gate_up measured
  // best on their picks below
  if (N % 128 == 0 && M > 320 && M <= 384 && N > 4096 && N <= 8192) return 7;
  // SwiGLU-width projections (N >= 16384: gate_up) in the 384-row bucket: 192 x 256 tiles (2 x
  // N/256, no padding rows) instead of the phased 256 x 256 (384 -> 512 rows): 2-8 us faster
  // per launch in every round of an order-balanced A/B (bench/tile_ab.py,
  // profiles/r6_tile_ab_gate_up_384.jsonl)
  if (g_tile8 && N % 256 == 0 && M > 320 && M <= 384 && N >= 16384) return 8;
  const int cand[3][3] = {{1, 256, 256}, {2, 128, 256}, {3, 128, 128}};
  int best = 0;
  for (auto& c : cand) {
    if (N % c[2]) continue;
    const long blocks = (long)((M + c[1] - 1) / c[1]) * (N / c[2]);
    if (!best) best = c[0];
    // the phased 256x256 kernel pays from ~160 tiles (profiles/r2_prefill_gemm_phased.jsonl)
    if (blocks >= (c[0] == 1 ? 160 : 200)) return c[0];
    best = c[0];
  }
  return best;
}

// Per-row RMSNorm statistics for the prefill GEMMs (one wave per row, every 16-byte load
// of the row issued before the first use): rstd[m] = rsqrt(mean_k X[m,k]^2 + eps).  Run
// once per normed projection instead of inside every n-tile's k loop.
static __global__ __launch_bounds__(256) void row_rstd_kernel(const bf16* __restrict__ X, int ldx, int M,
                                                       int K, float eps, float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const bf16x8* p = reinterpret_cast<const bf16x8*>(X + (size_t)row * ldx);
  const int nv = K / 8;
  float s = 0.f;
  for (int c0 = 0; c0 < nv; c0 += 64 * 16) {
    bf16x8 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = c0 + 64 * j + lane;
      v[j] = c < nv ? p[c] : zero_bf16x8();
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      s = sumsq8(v[j], s);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[row] = rsqrtf(s / (float)K + eps);
}

// rstd workspace: grow-only like the split-K workspace (a captured graph keeps its address);
// never grown while capturing (the GEMM then keeps the in-loop sums)
static SplitWs g_rstd_ws;
static int g_pre_rstd = 1;  // 0: always in-loop sums (A/B)
static const float* pre_rstd(const void* X, int ldx, int M, int K, float eps, hipStream_t st) {
  if (!g_pre_rstd || M < 128 || (ldx % 8) || (K % 8) || ((uintptr_t)X % 16)) return nullptr;
  const size_t bytes = (size_t)M * sizeof(float);
  if (g_rstd_ws.bytes < bytes) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    void* buf = nullptr;
    const size_t want = std::max(bytes, 2 * g_rstd_ws.bytes);
    if (hipMalloc(&buf, want) != hipSuccess) return nullptr;
    g_rstd_ws.buf = buf;  // the old buffer stays allocated (see split_ws)
    g_rstd_ws.bytes = want;
  }
  float* out = (float*)g_rstd_ws.buf;
  hipLaunchKernelGGL(row_rstd_kernel, dim3((M + 3) / 4), dim3(256), 0, st, (const bf16*)X, ldx, M,
                     K, eps, out);
  return hipGetLastError() == hipSuccess ? out : nullptr;
}

}  // namespace pgemm

#ifndef PGEMM_NO_DISPATCH  // (wide_gemm.hip uses the split-K helpers only)
static int g_prefill_tile = 0;  // 0 = heuristic (benchmarks can force 1..3)

// Used by the p2p_tiled_gemm* entry points (tiled_gemm.hip).  Returns
// hipErrorInvalidValue if the shape does not tile (caller falls back).
static int prefill_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                         int norm, void* out, int ldo, float eps, const EpiArgs& ea,
                         hipStream_t st) {
  using namespace pgemm;
  if (M <= 0 || K % BK) return (int)hipErrorInvalidValue;
  int tile = g_prefill_tile ? g_prefill_tile : pick_tile(M, N, K);
  const int bn = (tile == 3 || tile == 4 || tile == 6 || tile == 7) ? 128 : 256;
  if (!tile || N % bn) return (int)hipErrorInvalidValue;
  const int up_off = (epi == EPI_SILU) ? N / 32 : 0;
  // normed projections from 128 rows: rstd by row_rstd_kernel, GEMM without in-loop sums
  if (norm && !ea.moe_cnt) {
    if (const float* r = pre_rstd(X, ldx, M, K, eps, st)) {
      EpiArgs e2 = ea;
      e2.rstd_in = r;
      switch (epi) {
        case EPI_STORE: return launch_tile<EPI_STORE, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, e2, st);
        case EPI_SILU: return launch_tile<EPI_SILU, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, e2, st);
        case EPI_F32: return launch_tile<EPI_F32, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, e2, st);
        case EPI_QKV_ROPE: return launch_tile<EPI_QKV_ROPE, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, e2, st);
        case EPI_ARGMAX: return launch_tile<EPI_ARGMAX, false>(tile, Wt, X, ldx, M, K, N, up_off, out, ldo, eps, e2, st);
      }
    }
  }
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
#endif  // PGEMM_NO_DISPATCH
