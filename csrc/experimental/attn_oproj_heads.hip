// Decode attention fused with o_proj (+ residual), split over KV heads: no hand-off
// between attention and GEMM workgroups.
//
// At batch 1 and chat-length contexts the attention step is a ~2 us chain of dependent
// loads that costs a whole kernel boundary plus ramp (~7 us as its own launch), and
// o_proj is a 33.5 MB weight stream whose first bytes arrive only after that launch
// has drained.  Here ONE launch does both without any cross-workgroup wait:
//
//   grid = (N / 128 column blocks) x Hkv; workgroup (cb, g), 8 waves:
//   1. every wave issues its whole o_proj weight slice first -- 16 output columns of
//      block cb x the K range of kv head g (G*128 dims; fragment-major, 1 KiB per wave
//      instruction, non-temporal) -- so the weight stream is in flight from the start;
//   2. meanwhile it computes the attention of kv head g (its G query heads, GQA-packed)
//      for every row: redundantly in all N/128 workgroups of head g, which is cheap at
//      <= 256 keys (54 KB of K/V per head, L2-resident: with Hkv = 8 the workgroups of
//      head g all sit on XCD g under the round-robin dispatch);
//   3. MFMA of the attention rows (LDS) with the slice: a partial o_proj over head g's
//      K range, stored write-through (sc1) to the head's fp32 slab;
//   4. an arrival ticket per column block: the last of the Hkv workgroups sums the Hkv
//      partials in head order (deterministic) + the residual and writes h.
// The ticket follows cdna_hip_programming.md Guideline 16 (R1): sc1 stores, every
// storing wave drains vmcnt, then one agent-scope atomic add per workgroup; the last
// arriver reads the slabs with sc1 loads.  Nobody spins, so nothing can hang.
//
// SURVEY §2D K6 + K7 (the reference's decode path is Ollama's, web/streamlit_app.py:91).
#include "common.h"

namespace {

constexpr int PAGE = 64, HD = 128;
constexpr int WAVES = 8, NT = WAVES * 64;
constexpr int KPW = 32;                 // keys per wave: 8 waves x 32 = 256-key contexts
constexpr int CB_COLS = WAVES * 16;     // output columns per workgroup (one 16-col group / wave)
constexpr int VS = HD + 8;              // V row stride in LDS (bf16): conflict-free 16-B writes

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFFF,
                                           0x00020000);
}

template <int G>
struct Smem {
  static constexpr int KSH = G * HD / 32;   // o_proj k-steps of one kv head
  static constexpr int AS = KSH * 32 + 8;   // attention row stride (bf16), padded
  bf16x2 qs[G][HD / 2];
  float ps[WAVES][G][KPW];
  float sm[WAVES][G], sl[WAVES][G];
  union {
    bf16 vs[WAVES][KPW][VS];
    float so[WAVES][G][HD];
  } u;
};

template <int G, bool KV_FIRST>
__global__ __launch_bounds__(NT) void attn_oproj_heads_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ bt, int bt_stride, const int* __restrict__ row_bt,
    const int* __restrict__ ctx_lens, int R, int Hkv, float scale, const bf16x8* __restrict__ Wo,
    int N, bf16* __restrict__ h, int ldh, float* __restrict__ slab, unsigned* __restrict__ tickets,
    bf16* __restrict__ attn_out, int lda, int flags) {
  constexpr int KSH = Smem<G>::KSH;
  constexpr int AS = Smem<G>::AS;
  __shared__ Smem<G> S;
  __shared__ __attribute__((aligned(16))) bf16 a_lds[16][AS];
  __shared__ int s_last;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blockIdx.x % Hkv, cb = blockIdx.x / Hkv;
  const int Ssteps = Hkv * KSH;  // k-steps of the whole o_proj (K = Hq * 128)

  // K/V rows of row r: wave w's 32 keys sit in one page (32 | 64), so the page index is
  // wave-uniform (scalar loads: they do not queue behind the vector weight loads)
  const int t = lane >> 2, quarter = lane & 3;
  auto load_kv = [&](int r, bf16x8(&kr)[2][4], bf16x8(&vr)[2][4]) {
    const int rb = row_bt ? row_bt[r] : r;
    const int page = bt[(size_t)rb * bt_stride + min(w * KPW / PAGE, bt_stride - 1)];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int key = w * KPW + p * 16 + t;
      const size_t off = (((size_t)page * Hkv + g) * PAGE + (key % PAGE)) * HD + quarter * 32;
      const bf16x8* kp = reinterpret_cast<const bf16x8*>(kc + off);
      const bf16x8* vp = reinterpret_cast<const bf16x8*>(vc + off);
#pragma unroll
      for (int i = 0; i < 4; ++i) kr[p][i] = kp[i];
#pragma unroll
      for (int i = 0; i < 4; ++i) vr[p][i] = vp[i];
    }
  };
  // q of row r -> LDS (one 4-byte load per thread)
  auto load_q = [&](int r) {
    const bf16x2* qrow = reinterpret_cast<const bf16x2*>(q + (size_t)r * ldq + (size_t)g * G * HD);
    return tid < G * HD / 2 ? qrow[tid] : bf16x2{};
  };

  // 1) the weight slice: column group cb*8 + w, k-steps [g*KSH, (g+1)*KSH).  Vector loads
  // return in issue order, so row 0's K/V and q are issued FIRST (KV_FIRST): the attention
  // then starts after one memory latency instead of after the whole 128 KiB slice
  bf16x8 kr[2][4], vr[2][4];
  bf16x2 qv0 = {};
  if constexpr (KV_FIRST) {
    load_kv(0, kr, vr);
    qv0 = load_q(0);
  }
  bf16x8 wr[KSH];
  {
    const bf16x8* wp = Wo + ((size_t)(cb * WAVES + w) * Ssteps + (size_t)g * KSH) * 64 + lane;
#pragma unroll
    for (int i = 0; i < KSH; ++i) wr[i] = __builtin_nontemporal_load(wp + (size_t)i * 64);
  }

  // MFMA rows past R read zeros (zeroed here, so the A loads below are unconditional)
  for (int i = R * AS + tid; i < 16 * AS; i += NT) (&a_lds[0][0])[i] = f2bf(0.f);

  // 2) attention of kv head g for every row.  Wave w owns keys [32w, 32w + 32) as two
  // 16-key passes; lane = (key t = lane >> 2, quarter = lane & 3 of the 128 dims), so a
  // lane holds 32 dims of q per head (the register budget: the weight slice is live).
  for (int r = 0; r < R; ++r) {
    const int ctx = ctx_lens[r];
    bf16x2 qv;
    if (!KV_FIRST || r > 0) {
      load_kv(r, kr, vr);
      qv = load_q(r);
    } else {
      qv = qv0;
    }
    if (tid < G * HD / 2) S.qs[tid / (HD / 2)][tid % (HD / 2)] = qv;
    const int n_valid = min(max(ctx - w * KPW, 0), KPW);
    __syncthreads();

    float o[G][2], mg[G], lg[G];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      o[gg][0] = o[gg][1] = 0.f;
      mg[gg] = -INFINITY;
      lg[gg] = 0.f;
    }
    if (n_valid > 0) {  // wave-uniform
      float s[2][G];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int gg = 0; gg < G; ++gg) s[p][gg] = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int d2 = quarter * 16 + i * 4 + j;
#pragma unroll
          for (int gg = 0; gg < G; ++gg) {
            const bf16x2 qv = S.qs[gg][d2];
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              const bf16x2 k2 = {kr[p][i][2 * j], kr[p][i][2 * j + 1]};
              s[p][gg] = __builtin_amdgcn_fdot2_f32_bf16(qv, k2, s[p][gg], false);
            }
          }
        }
#pragma unroll
      for (int p = 0; p < 2; ++p)
        if (p * 16 + t < n_valid) {
          bf16x8* vrow = reinterpret_cast<bf16x8*>(&S.u.vs[w][p * 16 + t][quarter * 32]);
#pragma unroll
          for (int i = 0; i < 4; ++i) vrow[i] = vr[p][i];
        }
#pragma unroll
      for (int gg = 0; gg < G; ++gg) {
        float sv[2];
        float m = -INFINITY;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          float x = s[p][gg];
          x += __shfl_xor(x, 1, 64);
          x += __shfl_xor(x, 2, 64);
          sv[p] = p * 16 + t < n_valid ? x * scale : -INFINITY;
          m = fmaxf(m, sv[p]);
        }
#pragma unroll
        for (int o2 = 4; o2 < 64; o2 <<= 1) m = fmaxf(m, __shfl_xor(m, o2, 64));
        float l = 0.f;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const float pr = p * 16 + t < n_valid ? __expf(sv[p] - m) : 0.f;
          l += pr;
          if (quarter == 0) S.ps[w][gg][p * 16 + t] = pr;
        }
#pragma unroll
        for (int o2 = 4; o2 < 64; o2 <<= 1) l += __shfl_xor(l, o2, 64);  // one lane per key
        mg[gg] = m;
        lg[gg] = l;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's V rows and p are in LDS
      __builtin_amdgcn_wave_barrier();
#pragma unroll 4
      for (int k = 0; k < n_valid; ++k) {
        const bf16x2 vv = *reinterpret_cast<const bf16x2*>(&S.u.vs[w][k][2 * lane]);
        const float v0 = (float)vv[0], v1 = (float)vv[1];
#pragma unroll
        for (int gg = 0; gg < G; ++gg) {
          const float p = S.ps[w][gg][k];
          o[gg][0] = fmaf(p, v0, o[gg][0]);
          o[gg][1] = fmaf(p, v1, o[gg][1]);
        }
      }
    }
    __syncthreads();  // every wave's P.V is done: the V region becomes the O partials
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      S.u.so[w][gg][2 * lane] = o[gg][0];
      S.u.so[w][gg][2 * lane + 1] = o[gg][1];
      if (lane == 0) {
        S.sm[w][gg] = mg[gg];
        S.sl[w][gg] = lg[gg];
      }
    }
    __syncthreads();
    for (int i = tid; i < G * HD; i += NT) {
      const int gg = i / HD, d = i % HD;
      float M = -INFINITY;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) M = fmaxf(M, S.sm[ww][gg]);
      float num = 0.f, den = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) {
          const float e = __expf(S.sm[ww][gg] - M);
          num = fmaf(e, S.u.so[ww][gg][d], num);
          den = fmaf(e, S.sl[ww][gg], den);
        }
      }
      const bf16 a = f2bf(den > 0.f ? num / den : 0.f);
      a_lds[r][i] = a;
      if (attn_out && cb == 0) attn_out[(size_t)r * lda + (size_t)g * G * HD + i] = a;
    }
    __syncthreads();  // before the next row reuses the LDS regions
  }

  // 3) partial o_proj over head g's K range: rows on the MFMA M axis (R <= 16)
  const int m = lane & 15, kq = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < KSH; ++i) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(&a_lds[m][32 * i + 8 * kq]);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wr[i], acc, 0, 0, 0);
  }
  const int col = (cb * WAVES + w) * 16 + m;  // accumulator column = lane & 15
  const __amdgpu_buffer_rsrc_t rs = raw_rsrc(slab);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 4 * kq + j;
    const float v = acc[j];  // (bit_cast of the vector element acc[j] itself compiled to
                             // element 0 for every j on ROCm 7.2: go through a scalar)
    if (row < R)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), rs,
                                            (int)((((size_t)g * R + row) * N + col) * 4), 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains (sc1)
  __syncthreads();

  if (flags & 2) return;  // timing probe: no fan-in (results incomplete)
  // 4) one arrival per workgroup; the last of the column block's Hkv heads reduces
  if (tid == 0) {
    const unsigned tk = __hip_atomic_fetch_add(&tickets[cb], 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == (unsigned)Hkv - 1;
    if (last)  // every head arrived: re-arm for the next launch / graph replay
      (void)__hip_atomic_exchange(&tickets[cb], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  for (int i = tid; i < R * CB_COLS; i += NT) {
    const int row = i / CB_COLS, c = cb * CB_COLS + i % CB_COLS;
    float v = 0.f;
    for (int gg = 0; gg < Hkv; ++gg)  // head order: the same sum whoever arrives last
      v += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                         rs, (int)((((size_t)gg * R + row) * N + c) * 4), 0, 16));
    bf16* p = h + (size_t)row * ldh + c;
    *p = f2bf((float)*p + v);
  }
}

static int g_heads_flags = 1;  // bit 0: K/V + q of row 0 issued before the weight slice

template <int G>
int launch(const void* q, int ldq, const void* kc, const void* vc, const int* bt, int bt_stride,
           const int* row_bt, const int* ctx, int R, int Hkv, float scale, const void* Wo, int N,
           void* h, int ldh, float* slab, unsigned* tickets, void* attn, int lda, hipStream_t st) {
  const int f = g_heads_flags;
  if (f & 1)
    hipLaunchKernelGGL((attn_oproj_heads_kernel<G, true>), dim3((N / CB_COLS) * Hkv), dim3(NT), 0,
                       st, (const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, bt, bt_stride,
                       row_bt, ctx, R, Hkv, scale, (const bf16x8*)Wo, N, (bf16*)h, ldh, slab,
                       tickets, (bf16*)attn, lda, f);
  else
    hipLaunchKernelGGL((attn_oproj_heads_kernel<G, false>), dim3((N / CB_COLS) * Hkv), dim3(NT), 0,
                       st, (const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, bt, bt_stride,
                       row_bt, ctx, R, Hkv, scale, (const bf16x8*)Wo, N, (bf16*)h, ldh, slab,
                       tickets, (bf16*)attn, lda, f);
  return (int)hipGetLastError();
}

}  // namespace

// Launch flags (benchmarks): bit 0 = K/V-first issue order (default on), bit 1 = skip the
// fan-in (timing probe only: h is not updated).
P2P_API void p2p_attn_oproj_heads_tune(int flags) { g_heads_flags = flags; }

// Workspace of p2p_attn_oproj_heads: fp32 slab floats (Hkv * R * N) and u32 tickets
// (N / 128, zeroed once; the kernel re-arms them).
P2P_API long long p2p_attn_oproj_heads_slab_floats(int R, int Hkv, int N) {
  return (long long)Hkv * R * N;
}

// h[R, N] += attention(q) @ Wo^T for decode rows (R <= 16, every context <= 256 keys,
// head_dim 128, G = Hq / Hkv in {1, 2, 4}, N % 128 == 0); Wo fragment-major
// [N/16][Hq*128/32][64][8] bf16.  row_bt null = row r uses block-table row r.
// attn (optional, may be null): [R, Hq*128] copy of the attention output.
P2P_API int p2p_attn_oproj_heads(const void* q, int ldq, const void* k_cache, const void* v_cache,
                                 const int* block_tables, int bt_stride, const int* row_bt,
                                 const int* ctx_lens, int R, int Hq, int Hkv, int head_dim,
                                 float scale, int max_ctx, const void* Wo, int N, void* h, int ldh,
                                 float* slab, unsigned* tickets, void* attn, int lda,
                                 hipStream_t stream) {
  if (head_dim != HD || Hkv <= 0 || Hq % Hkv || R <= 0 || R > 16 || max_ctx > WAVES * KPW ||
      N % CB_COLS || !slab || !tickets)
    return (int)hipErrorInvalidValue;
  switch (Hq / Hkv) {
    case 1: return launch<1>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, Wo, N, h, ldh, slab, tickets, attn, lda, stream);
    case 2: return launch<2>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, Wo, N, h, ldh, slab, tickets, attn, lda, stream);
    case 4: return launch<4>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, Wo, N, h, ldh, slab, tickets, attn, lda, stream);
    // G = 8 (70B at TP=1) would spill: the weight slice (32 k-steps) stays live across the
    // attention -- callers run the two kernels
  }
  return (int)hipErrorInvalidValue;
}
