// Wide mid-M GEMM (1 < M <= 64 rows: chat-length prompt prefill, batched decode).
//
//   out[m, n] = epilogue( rstd[m] * sum_k X[m, k] * W[n, k] )   (gemm_epilogue.h)
//
// Where the two older mid-M families lose (profiles/r2_midm_split_parallel.jsonl,
// r1_midM_gemm_families.jsonl):
//   * skinny_gemm.hip (one 16-column group per workgroup) and midm_gemm.h (same, K in an
//     LDS ring) re-read the whole activation block for every 16 output columns: at
//     M = 44 that is 3 activation KiB per weight KiB, and the activation stream, not the
//     weight stream, sets the time (qkv 24-28 us for a 50 MB weight stream);
//   * the split-K tiled kernel (prefill_gemm.h, 64 x 128 tiles) stages the weights
//     through LDS as well and fills only 192 of 256 CUs at the qkv shape.
// Here a workgroup of 8 waves owns 128 output columns (SwiGLU: 64 gate + the matching
// 64 up columns) and a K slice:
//   * the activation slice streams through an LDS ring of D + 2 chunk slots by LDS-DMA
//     (global_load_lds_dwordx4, fragment-major image, conflict-free ds_read_b128), or sits
//     in LDS whole when it fits (RES), and is read by all 8 waves: 16 activation rows cost
//     1/8 of a weight byte, not 1;
//   * each wave streams its OWN 16-column weight group straight into VGPRs (one 1 KiB
//     non-temporal load per k-step, fragment-major in HBM), 2-3 chunks of 8 k-steps ahead
//     (128-192 KiB of weights + the activation chunks in flight per CU: a one-chunk-ahead
//     first version was latency-bound at ~2.6 TB/s);
//   * the grid is column blocks x K slices, with the slice count picked so the grid is
//     <= one block per CU and close to the CU count (qkv at 8B: 48 x 5 = 240 blocks);
//     the K slices of a tile meet through write-through slabs and a generation flip
//     (the parallel split-K reduction of prefill_gemm.h), and slice s finishes the
//     waves w with w % splitk == s, summing the slices in slice order (deterministic).
// RMSNorm: the block squares the activation fragments it already holds in LDS (one
// m-tile per wave pair); the row sums of the slices meet in the reduction.
// Measured (docs/ARCHITECTURE.md "Wide mid-M family"): the autotuner's pick at 33-64 rows
// for gate_up, down and qkv; the split-K seam (~5-6 us) is what it still pays on N <= 6144.
#define PGEMM_NO_DISPATCH
#include "prefill_gemm.h"

namespace wide {

#ifdef WIDE_STAMP
// probe builds only (csrc/experimental/wide_stamp.hip): per-block wall-clock stamps
// [entry, first chunk ready, main loop done, slabs drained, slices met, end, tile, split]
__device__ long long* wide_stamp_buf;
#define WSTAMP(i, v) do { if (wide_stamp_buf && threadIdx.x == 0) wide_stamp_buf[(size_t)blockIdx.x * 8 + (i)] = (v); } while (0)
#else
#define WSTAMP(i, v) do { } while (0)
#endif

constexpr int NT = 512;   // 8 waves
constexpr int KC = 8;     // k-steps per chunk: wave w DMA-loads k-step w of every m-tile
constexpr int MAX_SPLIT = 16;  // K slices per tile (the rstd reduction unrolls over them)
typedef __attribute__((address_space(3))) void* lds_ptr_t;
using pgemm::SplitArgs;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// chunks of a K slice whose activations fit LDS at once (the RES variant): <= 144 KiB
template <int MT>
constexpr int res_chunks() { return 18 / MT; }

// tile = column block: 8 groups of 16 columns (SILU: waves 0-3 gate groups 4t..4t+3,
// waves 4-7 the up groups 4t..4t+3 + up_off; output columns 64t..64t+63).
// RES: the slice's whole activation block is DMA'd into LDS up front (one barrier), so the
// waves never meet again in the k loop and each streams its weights at its own pace;
// otherwise the activations stream through a ring with a barrier per chunk.
template <int MT, int EPI, bool NORM, bool SPLIT, bool RES>
__global__ __launch_bounds__(NT) void wide_gemm_kernel(const bf16x8* __restrict__ Wt,
                                                       const bf16* __restrict__ X, int ldx, int M,
                                                       int K, int n_tiles, int up_off,
                                                       void* __restrict__ out, int ldo, float eps,
                                                       EpiArgs ea, SplitArgs sp) {
  constexpr bool SILU = EPI == EPI_SILU;
  // pipeline depth: D chunks ahead (RS = D + 1 register sets of KC weight fragments: 128
  // VGPRs at D = 3), activation ring of D + 2 slots (<= 128 KiB of LDS at every MT)
  constexpr int D = MT >= 4 ? 2 : 3;
  constexpr int RS = D + 1;
  constexpr int RING = D + 2;
  constexpr int SLOT = MT * KC * 64;  // bf16x8 per ring slot
  constexpr int PER_CHUNK = MT + KC;  // vmem instructions per thread per chunk
  constexpr int NSLOT = RES ? res_chunks<MT>() : RING;
  __shared__ __attribute__((aligned(16))) bf16x8 ring[NSLOT * SLOT];
  __shared__ float ss_l[2][4][16];

  const int splitk = SPLIT ? sp.splitk : 1;
  const int b = xcd_remap(blockIdx.x, n_tiles * splitk);
  const int tile = b / splitk, split = b % splitk;  // a tile's slices are consecutive
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int S = K >> 5;
  const int nc_all = S / KC;
  const int c0 = split * nc_all / splitk, c1 = (split + 1) * nc_all / splitk;
  const int n = c1 - c0;
  WSTAMP(0, wall_clock64());
  WSTAMP(6, tile);
  WSTAMP(7, split);

  const int gw = SILU ? (w < 4 ? tile * 4 + w : tile * 4 + (w - 4) + up_off) : tile * 8 + w;
  const bf16x8* wsrc = Wt + (size_t)gw * S * 64 + lane;
  const bf16* asrc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = min(16 * i + (lane & 15), M - 1);
    asrc[i] = X + (size_t)row * ldx + 32 * w + 8 * (lane >> 4);
  }

  auto issue_a = [&](int c) {
    bf16x8* base = ring + ((c - c0) % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < MT; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (size_t)c * KC * 32),
                                       (lds_ptr_t)(base + (i * KC + w) * 64), 16, 0, 0);
  };
  auto issue_w = [&](int c, bf16x8(&wr)[KC]) {
#pragma unroll
    for (int k = 0; k < KC; ++k) wr[k] = __builtin_nontemporal_load(wsrc + (size_t)(c * KC + k) * 64);
  };
  auto issue = [&](int c, bf16x8(&wr)[KC]) {
    if constexpr (!RES) issue_a(c);
    issue_w(c, wr);
  };

  constexpr int PC = RES ? KC : PER_CHUNK;  // vmem instructions per chunk in the k loop
  auto wait_chunks = [&](int k) {  // at most k chunks of this thread's loads in flight
    switch (k) {
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<PC>(); break;
      case 2: wait_vmcnt<2 * PC>(); break;
      default: wait_vmcnt<(D >= 3 ? 3 : 2) * PC>(); break;
    }
  };

  // The output group this wave finishes, if any: group w (SILU: gate/up pair w < 4); under
  // split-K only slice (w % splitk) finishes it.
  const int r = lane & 15, q = lane >> 4;
  const bool fin = w < (SILU ? 4 : 8) && (!SPLIT || (w % splitk) == split);
  const int g = SILU ? tile * 4 + w : tile * 8 + w;
  // Epilogue operands, issued as ONE batch per lane BEFORE the weight stream (they are the
  // oldest loads in flight, so the counted chunk waits below still hold, and they have long
  // landed when the epilogue runs): the residual values (EPI_RESID), the rows' KV slots and
  // positions (EPI_QKV_ROPE; the (cos, sin) loads that depend on the positions go out right
  // after the main loop).  Issued after the main loop, the residual loads held up the slab
  // drain of the split-K seam by ~1.6 us (bench/wide_stamp_probe.py, r5); loaded element by
  // element in the epilogue they were a chain of MT x 4 dependent round trips per lane.
  float res[MT][4];
  float2 csv[MT][4];
  int slotv[MT][4];
  int posv[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * i + 4 * q + j;
      const bool ok = fin && m < M;
      res[i][j] = 0.f;
      slotv[i][j] = -1;
      posv[i][j] = -1;
      csv[i][j] = float2{1.f, 0.f};
      if constexpr (EPI == EPI_RESID)
        if (ok) res[i][j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + g * 16 + r];
      if constexpr (EPI == EPI_QKV_ROPE)
        if (ok) {
          slotv[i][j] = ea.slots[m];
          posv[i][j] = ea.pos[m];
        }
    }

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;  // NORM: rows of m-tile (w & 3), k-steps of parity (w >> 2), this lane's 8 k
  const int sq_mt = w & 3, sq_par = w >> 2;

  auto compute = [&](int c, const bf16x8(&wr)[KC]) {
    const bf16x8* base = ring + ((c - c0) % NSLOT) * SLOT;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      bf16x8 a[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = base[(i * KC + k) * 64 + lane];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], wr[k], acc[i], 0, 0, 0);
    }
    if constexpr (NORM) {
      if (sq_mt < MT) {
#pragma unroll
        for (int k = 0; k < KC; k += 2) {
          ss = sumsq8(base[(sq_mt * KC + k + sq_par) * 64 + lane], ss);
        }
      }
    }
  };

  // D chunks (activation DMA + this wave's weights) are in flight ahead of the one being
  // computed; the counted wait + barrier makes chunk t complete (every wave's DMA part), and
  // the ring slot refilled at step t (chunk t+D's) was last read at t-2, before barrier t-1
  bf16x8 wr[RS][KC];
  if constexpr (RES)  // the whole slice's activations first (host: n <= res_chunks)
    for (int c = 0; c < n; ++c) issue_a(c0 + c);
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < n) issue(c0 + j, wr[j]);
  for (int tb = 0; tb < n; tb += RS) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const int t = tb + j;
      if (t >= n) break;
      if (t + D < n) issue(c0 + t + D, wr[(j + D) % RS]);
      wait_chunks(min(D, n - 1 - t));
      if (!RES || t == 0) {  // RES: chunk 0's weights landed => this wave's DMA parts too
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (t == 0) WSTAMP(1, wall_clock64());
      }
      compute(c0 + t, wr[j]);
    }
  }

  WSTAMP(2, wall_clock64());
  // ---- this slice's row sums of squares: wave pair (w, w ^ 4) holds m-tile w & 3 ----
  if constexpr (NORM) {
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (sq_mt < MT && lane < 16) ss_l[sq_par][sq_mt][lane] = ss;
  }
  if constexpr (EPI == EPI_QKV_ROPE) {
    const int kk = g & 7;
    const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (posv[i][j] >= 0) csv[i][j] = ea.cs[(size_t)posv[i][j] * 64 + dd];
  }

  auto epilogue = [&](const f32x4 (&v)[MT], const f32x4 (&u)[MT], auto&& rstd_of) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 16 * i + 4 * q + j;
        const bool valid = m < M;
        const float sc = rstd_of(i, j);
        if constexpr (EPI == EPI_QKV_ROPE) {
          epi_store<EPI>(m, valid, g, r, v[i][j] * sc, 0.f, out, ldo, ea, csv[i][j], slotv[i][j]);
        } else if constexpr (EPI == EPI_RESID) {
          if (valid)
            reinterpret_cast<bf16*>(out)[(size_t)m * ldo + g * 16 + r] = f2bf(res[i][j] + v[i][j] * sc);
        } else {
          epi_store<EPI>(m, valid, g, r, v[i][j] * sc, u[i][j] * sc, out, ldo, ea);
        }
      }
    }
  };
  auto rstd_from = [&](float t) { return rsqrtf(t / (float)K + eps); };

  if constexpr (!SPLIT) {
    // the up waves hand their accumulators to the gate waves through LDS (ring is free)
    float* xch = reinterpret_cast<float*>(ring);
    __syncthreads();  // every wave is past its last ring read; ss_l complete
    if constexpr (SILU) {
      if (w >= 4) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) xch[(((w - 4) * MT + i) * 4 + j) * 64 + lane] = acc[i][j];
      }
      __syncthreads();
      if (w >= 4) return;
    }
    f32x4 up[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) up[i][j] = SILU ? xch[((w * MT + i) * 4 + j) * 64 + lane] : 0.f;
    }
    epilogue(acc, up, [&](int i, int j) {
      if constexpr (!NORM) return 1.f;
      const int rr = 4 * q + j;
      return rstd_from(ss_l[0][i][rr] + ss_l[1][i][rr]);
    });
#ifdef WIDE_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    WSTAMP(5, wall_clock64());
    return;
  } else {
    // ---- parallel split-K: write-through slabs [tile][split][wave][MT] (f32x4 per lane) ----
    const __amdgpu_buffer_rsrc_t rsl = pgemm::raw_rsrc(sp.slab);
    const size_t tile_v = (size_t)tile * splitk * 8 * MT * 64;  // f32x4 index of slice 0
#pragma unroll
    for (int i = 0; i < MT; ++i)
      pgemm::store_sc1(rsl, (int)((tile_v + (((size_t)split * 8 + w) * MT + i) * 64 + lane) * 16),
                       acc[i]);
    if constexpr (NORM) {
      __syncthreads();  // ss_l complete
      if (tid < 16 * MT) {
        const int i = tid >> 4, rr = tid & 15;
        __hip_atomic_store(&sp.ss_slab[((size_t)tile * splitk + split) * 64 + 16 * i + rr],
                           ss_l[0][i][rr] + ss_l[1][i][rr], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);  // write-through
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    WSTAMP(3, wall_clock64());
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
          if (wall_clock64() - t0 > pgemm::SPLIT_SPIN_TICKS) {
            __hip_atomic_store(sp.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    WSTAMP(4, wall_clock64());
    // every slice's partials are visible.  Rows' rstd: one lane per row sums the slices'
    // row sums (all loads issued before the first add) into LDS
    __shared__ float rstd_l[64];
    if constexpr (NORM) {
      if (tid < 16 * MT) {
        float pv[MAX_SPLIT];
#pragma unroll
        for (int s2 = 0; s2 < MAX_SPLIT; ++s2)
          pv[s2] = __hip_atomic_load(&sp.ss_slab[((size_t)tile * splitk + min(s2, splitk - 1)) * 64 + tid],
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float t2 = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < MAX_SPLIT; ++s2) t2 += s2 < splitk ? pv[s2] : 0.f;
        rstd_l[tid] = rstd_from(t2);
      }
      __syncthreads();
    }
    if (!fin) return;
    // the finished group's partials, summed in slice order; loads in batches of SB slices
    // (clamped indices: straight-line code, one wait per batch).  SB = 8 covers the usual
    // 5-8 slices in ONE round trip (batches of 4 cost a second one, ~1 us, r5 stamps); the
    // SwiGLU form loads gate and up partials, so it keeps 4 (VGPRs)
    constexpr int SB = SILU ? 4 : 8;
    f32x4 tot[MT], up[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      tot[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      up[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int s0 = 0; s0 < splitk; s0 += SB) {
      f32x4 pt[SB][MT], pu[SB][MT];
#pragma unroll
      for (int s = 0; s < SB; ++s) {
        const int s2 = min(s0 + s, splitk - 1);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          pt[s][i] = pgemm::load_sc1(rsl, (int)((tile_v + (((size_t)s2 * 8 + w) * MT + i) * 64 + lane) * 16));
          if constexpr (SILU)
            pu[s][i] = pgemm::load_sc1(rsl, (int)((tile_v + (((size_t)s2 * 8 + w + 4) * MT + i) * 64 + lane) * 16));
        }
      }
#pragma unroll
      for (int s = 0; s < SB; ++s) {
        if (s0 + s >= splitk) break;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          tot[i] += pt[s][i];
          if constexpr (SILU) up[i] += pu[s][i];
        }
      }
    }
    epilogue(tot, up, [&](int i, int j) {
      if constexpr (!NORM) return 1.f;
      return rstd_l[16 * i + 4 * q + j];
    });
#ifdef WIDE_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    WSTAMP(5, wall_clock64());
  }
}

static int g_max_split = MAX_SPLIT;
static int g_res = 1;  // RES variant where a slice's activations fit LDS (A/B: 0 = ring only)

template <int MT, int EPI, bool NORM, bool SPLIT, bool RES>
int launch_v(const void* Wt, const void* X, int ldx, int M, int K, int n_tiles, int up_off,
             void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st,
             const SplitArgs& sp) {
  hipLaunchKernelGGL((wide_gemm_kernel<MT, EPI, NORM, SPLIT, RES>), dim3(n_tiles * sp.splitk),
                     dim3(NT), 0, st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, n_tiles, up_off,
                     out, ldo, eps, ea, sp);
  return (int)hipGetLastError();
}

template <int MT, int EPI, bool NORM>
int launch_mt(const void* Wt, const void* X, int ldx, int M, int K, int n_tiles, int up_off,
              void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st, int splitk) {
  using namespace pgemm;
  const int nc = K / (32 * KC);
  const bool res = g_res && (nc + splitk - 1) / splitk <= res_chunks<MT>();
  if (splitk > 1) {
    const size_t slab = (size_t)n_tiles * splitk * 8 * MT * 64 * sizeof(f32x4);
    const size_t ssb = (size_t)n_tiles * splitk * 64 * sizeof(float);
    char* ws = nullptr;
    if ((size_t)n_tiles * sizeof(unsigned) >= kCounterBytes / 2 || slab + ssb >= 0x7FFFFFFF ||
        !split_ws(slab + ssb, st, &ws))  // (no workspace growth while a graph is captured)
      return launch_mt<MT, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, 1);
    unsigned* ctr = (unsigned*)(ws + g_split_ws.bytes - kCounterBytes);
    constexpr size_t nw = kCounterBytes / sizeof(unsigned);
    SplitArgs sp{splitk, (f32x4*)ws, (float*)(ws + slab), ctr, ctr + nw / 2, (int*)(ctr + nw - 1), 1};
    return res ? launch_v<MT, EPI, NORM, true, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, sp)
               : launch_v<MT, EPI, NORM, true, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, sp);
  }
  SplitArgs none{1, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  return res ? launch_v<MT, EPI, NORM, false, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, none)
             : launch_v<MT, EPI, NORM, false, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, none);
}

// K slices: the grid must stay <= one block per CU (every slice of a tile resident for the
// parallel reduction) and each slice keeps >= 2 chunks; otherwise as many as fill the CUs.
static int pick_split(int n_tiles, int nc, int req) {
  const int cus = pgemm::cu_count();
  if (cus <= 0) return 1;
  int s = req > 0 ? std::min(std::min(req, nc), MAX_SPLIT)
                  : std::min(cus / n_tiles, std::min(g_max_split, nc / 2));
  while (s > 1 && n_tiles * s > cus) --s;
  return std::max(1, s);
}

template <int EPI, bool NORM>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int N, void* out, int ldo,
           float eps, const EpiArgs& ea, hipStream_t st, int req_split) {
  const int cols = EPI == EPI_SILU ? 64 : 128;  // output columns per tile
  const int n_out = EPI == EPI_SILU ? N / 2 : N;
  if (M <= 0 || M > 64 || K % (32 * KC) || n_out % cols) return (int)hipErrorInvalidValue;
  const int n_tiles = n_out / cols;
  const int up_off = EPI == EPI_SILU ? N / 32 : 0;
  const int splitk = pick_split(n_tiles, K / (32 * KC), req_split);
  switch ((M + 15) / 16) {
    case 1: return launch_mt<1, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk);
    case 2: return launch_mt<2, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk);
    case 3: return launch_mt<3, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk);
    case 4: return launch_mt<4, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk);
  }
  return (int)hipErrorInvalidValue;
}

}  // namespace wide

// Called by skinny_dispatch (skinny_gemm.hip) for launch codes with the WIDE bit; ea_p points
// at the caller's EpiArgs (one identical definition per translation unit).  req_split: K
// slices (0 = heuristic).  Dense bf16 weights only (no FP8, no grouped MoE mode).
extern "C" int p2p_wide_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N,
                                 int epi, int norm, void* out, int ldo, float eps, const void* ea_p,
                                 int req_split, hipStream_t st) {
  const EpiArgs& ea = *reinterpret_cast<const EpiArgs*>(ea_p);
  if (ea.wscale || ea.moe_cnt) return (int)hipErrorInvalidValue;
  using namespace wide;
  switch (epi) {
    case EPI_STORE:
      return norm ? launch<EPI_STORE, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split)
                  : launch<EPI_STORE, false>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split);
    case EPI_RESID:
      if (norm) return (int)hipErrorInvalidValue;
      return launch<EPI_RESID, false>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split);
    case EPI_SILU:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_SILU, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split);
    case EPI_F32:
      return norm ? launch<EPI_F32, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split)
                  : launch<EPI_F32, false>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split);
    case EPI_QKV_ROPE:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_QKV_ROPE, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split);
    case EPI_ARGMAX:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_ARGMAX, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split);
  }
  return (int)hipErrorInvalidValue;
}

// Nonzero if a split slice of the wide kernel waited past its spin bound since the last call
// (that tile's output is invalid); clears the word.  Synchronises the current device.
extern "C" int p2p_wide_split_fault() {
  if (!pgemm::g_split_ws.buf) return 0;
  int* w = (int*)((char*)pgemm::g_split_ws.buf + pgemm::g_split_ws.bytes - sizeof(unsigned));
  int v = 0;
  if (hipMemcpy(&v, w, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (v) {
    const int z = 0;
    (void)hipMemcpy(w, &z, sizeof(int), hipMemcpyHostToDevice);
  }
  return v;
}

// Benchmarks: cap on the K-slice count of the heuristic (1 = never split).
// A/B: 1 = activations resident in LDS where a slice fits (default), 0 = the ring always.
P2P_API void p2p_wide_resident(int on) { wide::g_res = on ? 1 : 0; }

P2P_API void p2p_wide_max_split(int s) {
  wide::g_max_split = (s >= 1 && s <= wide::MAX_SPLIT) ? s : wide::MAX_SPLIT;
}

#ifdef WIDE_STAMP
P2P_API int p2p_wide_stamp_set(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(wide::wide_stamp_buf), &p, sizeof(p));
}
#endif
