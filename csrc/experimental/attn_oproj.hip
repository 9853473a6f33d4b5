// Decode attention fused with the o_proj GEMM (+ residual) in one launch.
//
// At batch <= 16 and short contexts the attention step is latency-bound (a
// chain of dependent loads on 8 workgroups) while the next kernel, o_proj, is a
// pure weight stream (33.5 MB for 8B).  Here both run in one grid:
//   blocks [0, R*Hkv)        attention for (row, kv head), GQA-packed, one 256-key
//                            chunk; write attn[row] and post an arrival
//                            (agent-scope release + atomic);
//   blocks [R*Hkv, +N/16)    o_proj column group g: the 16 waves FIRST load their
//                            split-K slice of W_o (fragment-major, 1 KiB per wave
//                            instruction) into registers, THEN wait for all
//                            attention arrivals (agent-scope acquire), then MFMA
//                            over the attention rows, reduce across waves in LDS,
//                            and add into the residual h.
// The o_proj weight stream therefore overlaps the attention latency instead of
// following it.  Attention blocks have the lowest ids, so they are dispatched
// before any waiting block (no residency deadlock); every wait is bounded in
// time (error flag, never a hang).  The last o_proj block re-arms the counters
// for the next launch (graph replay).  SURVEY §2D K6+K7.
#include "common.h"

namespace {

constexpr int PAGE = 64, HD = 128, WAVES = 16, KPW = 16, NT = WAVES * 64;
constexpr long long SPIN_TICKS = 2000000;  // 20 ms at the 100 MHz constant clock

template <int G>
struct AttnSmem {
  bf16x2 qs[G][HD / 2];
  float ps[WAVES][G][KPW];
  float sm[WAVES][G], sl[WAVES][G];
  float so[WAVES][G][HD];
};
struct OprojSmem {
  float red[WAVES][4][64];
};
template <int G>
constexpr int smem_floats() {
  return (sizeof(AttnSmem<G>) > sizeof(OprojSmem) ? sizeof(AttnSmem<G>) : sizeof(OprojSmem)) / 4;
}

template <int G, int KS>
__global__ __launch_bounds__(NT) void attn_oproj_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ bt, int bt_stride, const int* __restrict__ row_bt,
    const int* __restrict__ ctx_lens, int R, int Hkv, float scale, bf16* __restrict__ attn,
    int lda, const bf16x8* __restrict__ Wo, bf16* __restrict__ h, int ldh,
    unsigned* __restrict__ sync, int* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) float smem[smem_floats<G>()];
  const int n_attn = R * Hkv;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  if ((int)blockIdx.x < n_attn) {
    // ------------------------------------------------------------- attention
    AttnSmem<G>& S = *reinterpret_cast<AttnSmem<G>*>(smem);
    const int r = blockIdx.x / Hkv, hh = blockIdx.x % Hkv;
    const int t = lane >> 2, quarter = lane & 3;
    const int ctx = ctx_lens[r];
    const int rb = row_bt[r];
    const int key0 = w * KPW;
    // a wave's 16 keys sit in one page (16 | 64)
    const int page = bt[(size_t)rb * bt_stride + min(key0 / PAGE, bt_stride - 1)];
    const size_t head_base = ((size_t)page * Hkv + hh) * PAGE * HD;
    bf16x8 kr[4];
    {
      const bf16x8* kp = reinterpret_cast<const bf16x8*>(
          kc + head_base + (size_t)((key0 + t) % PAGE) * HD + quarter * 32);
#pragma unroll
      for (int i = 0; i < 4; ++i) kr[i] = kp[i];
    }
    // V: lane owns output dims 2*lane, 2*lane+1 of the wave's 16 keys (4 B per key)
    bf16x2 vv[KPW];
#pragma unroll
    for (int k = 0; k < KPW; ++k)
      vv[k] = *reinterpret_cast<const bf16x2*>(vc + head_base + (size_t)((key0 + k) % PAGE) * HD +
                                               2 * lane);
    const bf16x2* qrow =
        reinterpret_cast<const bf16x2*>(q + (size_t)r * ldq + (size_t)hh * G * HD);
    for (int i = tid; i < G * HD / 2; i += NT) S.qs[i / (HD / 2)][i % (HD / 2)] = qrow[i];
    __syncthreads();

    const int n_valid = min(max(ctx - key0, 0), KPW);
    const bool mine = t < n_valid;
    float o[G][2], mg[G], lg[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      o[g][0] = o[g][1] = 0.f;
      mg[g] = -INFINITY;
      lg[g] = 0.f;
    }
    if (n_valid > 0) {
      float s[G];
#pragma unroll
      for (int g = 0; g < G; ++g) s[g] = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x2 k2 = {kr[i][2 * j], kr[i][2 * j + 1]};
          const int d2 = quarter * 16 + i * 4 + j;
#pragma unroll
          for (int g = 0; g < G; ++g) s[g] = __builtin_amdgcn_fdot2_f32_bf16(S.qs[g][d2], k2, s[g], false);
        }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        s[g] += __shfl_xor(s[g], 1, 64);
        s[g] += __shfl_xor(s[g], 2, 64);
        const float sv = mine ? s[g] * scale : -INFINITY;
        float m = sv;
#pragma unroll
        for (int o2 = 4; o2 < 64; o2 <<= 1) m = fmaxf(m, __shfl_xor(m, o2, 64));
        const float p = mine ? __expf(sv - m) : 0.f;
        float l = p;
#pragma unroll
        for (int o2 = 4; o2 < 64; o2 <<= 1) l += __shfl_xor(l, o2, 64);
        mg[g] = m;
        lg[g] = l;
        if (quarter == 0) S.ps[w][g][t] = p;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's ps writes landed
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < KPW; ++k) {
        if (k < n_valid) {
          const float v0 = (float)vv[k][0], v1 = (float)vv[k][1];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const float p = S.ps[w][g][k];
            o[g][0] = fmaf(p, v0, o[g][0]);
            o[g][1] = fmaf(p, v1, o[g][1]);
          }
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      S.so[w][g][2 * lane] = o[g][0];
      S.so[w][g][2 * lane + 1] = o[g][1];
      if (lane == 0) {
        S.sm[w][g] = mg[g];
        S.sl[w][g] = lg[g];
      }
    }
    __syncthreads();
    // two dims per thread, one 4-byte write-through (sc1) store each: the hand-off below
    // needs no release fence (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1)
    for (int i = tid; i < G * HD / 2; i += NT) {
      const int g = i / (HD / 2), d = 2 * (i % (HD / 2));
      float M = -INFINITY;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) M = fmaxf(M, S.sm[ww][g]);
      float n0 = 0.f, n1 = 0.f, den = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) {
          const float e = __expf(S.sm[ww][g] - M);
          n0 = fmaf(e, S.so[ww][g][d], n0);
          n1 = fmaf(e, S.so[ww][g][d + 1], n1);
          den = fmaf(e, S.sl[ww][g], den);
        }
      }
      const float inv = den > 0.f ? 1.f / den : 0.f;
      bf16x2 o2 = {f2bf(n0 * inv), f2bf(n1 * inv)};
      unsigned bits;
      __builtin_memcpy(&bits, &o2, 4);
      __hip_atomic_store(reinterpret_cast<unsigned*>(attn + (size_t)r * lda + (size_t)(hh * G + g) * HD + d),
                         bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // publish: every storing wave's write-through stores retired -> barrier -> one arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_fetch_add(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }

  // ----------------------------------------------------------------- o_proj
  OprojSmem& S = *reinterpret_cast<OprojSmem*>(smem);
  const int g = blockIdx.x - n_attn;  // 16-column group
  const int Ssteps = Hkv * G * HD / 32;
  // 1) this wave's split-K weight slice, before the dependency (overlaps attention)
  bf16x8 wr[KS];
  const bf16x8* wp = Wo + ((size_t)g * Ssteps + (size_t)w * KS) * 64 + lane;
#pragma unroll
  for (int i = 0; i < KS; ++i) wr[i] = load_nt(wp + (size_t)i * 64);
  // 2) wait for every attention block (bounded): an sc1 poll by one lane, the block's
  //    other waves behind the barrier; no acquire fence -- every load of the handed-off
  //    rows below is an sc1 (L1-bypassing) load of write-through-stored data
  if (tid == 0) {
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           (unsigned)n_attn) {
      if (wall_clock64() - t0 > SPIN_TICKS) {
        atomicOr(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // 3) MFMA over the attention rows (A fragment: row lane&15, k 8(lane>>4)..+8)
  const int m = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bf16* arow = attn + (size_t)(m < R ? m : 0) * lda + (size_t)w * KS * 32 + 8 * (lane >> 4);
  bf16x8 af[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) {  // two 8-byte sc1 loads per fragment, all in flight
    const unsigned long long* p8 = reinterpret_cast<const unsigned long long*>(arow + i * 32);
    unsigned long long lo = 0, hi = 0;
    if (m < R) {
      lo = __hip_atomic_load(p8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      hi = __hip_atomic_load(p8 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned long long two[2] = {lo, hi};
    __builtin_memcpy(&af[i], two, 16);
  }
#pragma unroll
  for (int i = 0; i < KS; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wr[i], acc, 0, 0, 0);
  // 4) split-K reduction across the 16 waves, residual epilogue by wave 0
#pragma unroll
  for (int j = 0; j < 4; ++j) S.red[w][j][lane] = acc[j];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) v += S.red[ww][j][lane];
      const int row = 4 * (lane >> 4) + j;
      if (row < R) {
        bf16* p = h + (size_t)row * ldh + g * 16 + (lane & 15);
        *p = f2bf((float)*p + v);
      }
    }
  }
  // 5) the last o_proj block re-arms the counters for the next launch
  if (tid == 0) {
    const unsigned n_o = gridDim.x - n_attn;
    const unsigned tk = __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    if (tk == n_o - 1) {
      __hip_atomic_store(&sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sync[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int G, int KS>
int launch(const void* q, int ldq, const void* kc, const void* vc, const int* bt, int bt_stride,
           const int* row_bt, const int* ctx, int R, int Hkv, float scale, void* attn, int lda,
           const void* Wo, int N, void* h, int ldh, unsigned* sync, int* err, hipStream_t st) {
  hipLaunchKernelGGL((attn_oproj_kernel<G, KS>), dim3(R * Hkv + N / 16), dim3(NT), 0, st,
                     (const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, bt, bt_stride, row_bt,
                     ctx, R, Hkv, scale, (bf16*)attn, lda, (const bf16x8*)Wo, (bf16*)h, ldh, sync,
                     err);
  return (int)hipGetLastError();
}

template <int G>
int launch_g(int ks, const void* q, int ldq, const void* kc, const void* vc, const int* bt,
             int bt_stride, const int* row_bt, const int* ctx, int R, int Hkv, float scale,
             void* attn, int lda, const void* Wo, int N, void* h, int ldh, unsigned* sync,
             int* err, hipStream_t st) {
  switch (ks) {
    case 1: return launch<G, 1>(q, ldq, kc, vc, bt, bt_stride, row_bt, ctx, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, st);
    case 2: return launch<G, 2>(q, ldq, kc, vc, bt, bt_stride, row_bt, ctx, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, st);
    case 4: return launch<G, 4>(q, ldq, kc, vc, bt, bt_stride, row_bt, ctx, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, st);
    case 8: return launch<G, 8>(q, ldq, kc, vc, bt, bt_stride, row_bt, ctx, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, st);
    case 16: return launch<G, 16>(q, ldq, kc, vc, bt, bt_stride, row_bt, ctx, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, st);
  }
  return (int)hipErrorInvalidValue;
}

}  // namespace

// Fused decode attention + o_proj + residual.  Preconditions (else hipErrorInvalidValue,
// the caller runs the two kernels): R <= 16 rows, every context <= 256 keys (max_ctx),
// head_dim 128, G = Hq/Hkv in {1,2,4}, K = Hq*128 with (K/32) % 16 == 0 and K/512 in
// {1,2,4,8,16}, N % 16 == 0.
// attn: [R, Hq*128] scratch output of the attention; Wo: fragment-major [N/16][K/32][64][8];
// h: [R, N] residual, updated in place; sync: 2 zeroed u32 (re-armed by the kernel);
// err: int, set nonzero if a wait timed out.
P2P_API int p2p_attn_oproj(const void* q, int ldq, const void* k_cache, const void* v_cache,
                           const int* block_tables, int bt_stride, const int* row_bt,
                           const int* ctx_lens, int R, int Hq, int Hkv, int head_dim, float scale,
                           int max_ctx, void* attn, int lda, const void* Wo, int N, void* h,
                           int ldh, unsigned* sync, int* err, hipStream_t stream) {
  if (head_dim != HD || Hkv <= 0 || Hq % Hkv || R <= 0 || R > 16 || max_ctx > WAVES * KPW ||
      N % 16)
    return (int)hipErrorInvalidValue;
  const int S = Hq * HD / 32;
  if (S % WAVES) return (int)hipErrorInvalidValue;
  const int ks = S / WAVES;
  switch (Hq / Hkv) {
    case 1: return launch_g<1>(ks, q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, stream);
    case 2: return launch_g<2>(ks, q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, stream);
    case 4: return launch_g<4>(ks, q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, attn, lda, Wo, N, h, ldh, sync, err, stream);
    // G = 8 (70B) would spill the attention role's registers: callers use the two kernels
  }
  return (int)hipErrorInvalidValue;
}
