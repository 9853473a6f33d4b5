// Paged-KV attention for decode ("flash-decoding", split over the context).
//
// KV cache layout (engine/kv_cache.py): K and V are each
//     [num_pages][n_kv_heads][PAGE=64][D=128] bf16
// so one page of one kv head is a contiguous 16 KiB tile.  Every query row r
// carries a block-table row (its sequence) and a context length; a query row
// is either one decode token or one prefill token (causal: ctx = pos + 1).
//
// Grid: (chunk, kv_head, row); a chunk = 4 pages = 256 keys (16 waves x 16 keys).
// GQA packing: all G = Hq / Hkv query heads of a kv head are scored against the
// same K/V bytes in one pass (K/V read once per group, not once per q head).
// With one chunk the block writes the final bf16 output, otherwise fp32
// partials (m, l, o) for the combine kernel.
#include "common.h"

namespace {

constexpr int PAGE = 64;
constexpr int HD = 128;
constexpr int CHUNK = 4 * PAGE;

// Block = 16 waves = one 256-key chunk of one (row, kv head); wave w owns keys
// [16w, 16w+16).  QK: lane = (key t = lane>>2, quarter c = lane&3) holds 32 dims of
// K row t (four 16-B loads) and dots them with the G query heads; the four
// quarter partials meet by two xor-shuffles.  Softmax over the wave's 16 keys by
// xor-shuffles over the key bits.  PV: the wave's V rows go to LDS (row stride 272 B:
// conflict-free 16-B writes and 4-B column reads) and lane owns output dims
// 2*lane, 2*lane+1 over the 16 keys.  The 16 wave partials (m, l, o) merge
// through LDS.  Every global load of a wave is issued before any math, so the
// kernel pays one memory latency; the serial per-lane work is 16 keys deep.
constexpr int WAVES = 16;
constexpr int KPW = CHUNK / WAVES;  // keys per wave = 16

template <int G>
__global__ __launch_bounds__(WAVES * 64) void paged_attn_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ bt, int bt_stride, const int* __restrict__ row_bt,
    const int* __restrict__ ctx_lens, int Hkv, float scale, int n_chunks, bf16* __restrict__ out,
    int ldo, float* __restrict__ part_o, float* __restrict__ part_ml) {
  const int c = blockIdx.x, h = blockIdx.y, r = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int t = lane >> 2, quarter = lane & 3;
  // The context length, the block-table row and q are independent loads: issue them
  // together, and issue the K/V loads before looking at ctx (keys past the context
  // read the zero-initialised block-table tail = null page 0, always mapped), so the
  // kernel's dependent-latency chain is row_bt -> page -> K/V, not ctx -> ... -> K/V.
  const int ctx = ctx_lens[r];
  const int rb = row_bt ? row_bt[r] : r;  // null: row r uses block-table row r (decode)

  constexpr int VS = HD + 8;
  __shared__ bf16x2 qs[G][HD / 2];
  // V staging (P.V) and the wave partials of O (merge) share one region: the V rows are
  // dead once every wave has finished its P.V (barrier below), and the union keeps the
  // block under 80 KiB, i.e. two blocks per CU on long contexts (one block's loads in
  // flight while the other one computes).
  constexpr int kVsBytes = WAVES * KPW * VS * 2;
  constexpr int kSoBytes = WAVES * G * HD * 4;
  __shared__ __attribute__((aligned(16))) char vs_so[kVsBytes > kSoBytes ? kVsBytes : kSoBytes];
  auto& vs = *reinterpret_cast<bf16(*)[WAVES][KPW][VS]>(vs_so);
  auto& so = *reinterpret_cast<float(*)[WAVES][G][HD]>(vs_so);
  __shared__ float ps[WAVES][G][KPW];
  __shared__ float sm[WAVES][G], sl[WAVES][G];

  const int key0 = c * CHUNK + w * KPW;  // first key of this wave

  // 1) all global loads first: 32 dims (4 x 16 B) of K and V row `t` per lane
  bf16x8 kr[4], vr[4];
  {
    const int key = key0 + t;
    const int pcol = min(key / PAGE, bt_stride - 1);
    const int page = bt[(size_t)rb * bt_stride + pcol];
    const size_t off = (((size_t)page * Hkv + h) * PAGE + (key % PAGE)) * HD + quarter * 32;
    const bf16x8* kp = reinterpret_cast<const bf16x8*>(kc + off);
    const bf16x8* vp = reinterpret_cast<const bf16x8*>(vc + off);
#pragma unroll
    for (int i = 0; i < 4; ++i) kr[i] = kp[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) vr[i] = vp[i];
  }
  const bf16x2* qrow = reinterpret_cast<const bf16x2*>(q + (size_t)r * ldq + (size_t)h * G * HD);
  for (int i = tid; i < G * HD / 2; i += WAVES * 64) qs[i / (HD / 2)][i % (HD / 2)] = qrow[i];
  if (c * CHUNK >= ctx) return;  // block-uniform: the whole chunk is past the context
  const int n_valid = min(max(ctx - key0, 0), KPW);
  const bool mine = t < n_valid;
  __syncthreads();

  float o[G][2];
  float mg[G], lg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    o[g][0] = o[g][1] = 0.f;
    mg[g] = -INFINITY;
    lg[g] = 0.f;
  }
  if (n_valid > 0) {
    // 2) scores
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    if (mine) {
      // bf16 dot2 (v_dot2_f32_bf16): K stays packed, 2 MACs per instruction
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x2 k2 = {kr[i][2 * j], kr[i][2 * j + 1]};
          const int d2 = quarter * 16 + i * 4 + j;
#pragma unroll
          for (int g = 0; g < G; ++g) s[g] = __builtin_amdgcn_fdot2_f32_bf16(qs[g][d2], k2, s[g], false);
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) s[g] *= scale;
      bf16x8* vrow = reinterpret_cast<bf16x8*>(&vs[w][t][quarter * 32]);
#pragma unroll
      for (int i = 0; i < 4; ++i) vrow[i] = vr[i];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      s[g] += __shfl_xor(s[g], 1, 64);
      s[g] += __shfl_xor(s[g], 2, 64);
      float sv = mine ? s[g] : -INFINITY;
      float m = sv;
#pragma unroll
      for (int o2 = 4; o2 < 64; o2 <<= 1) m = fmaxf(m, __shfl_xor(m, o2, 64));
      const float p = mine ? __expf(sv - m) : 0.f;
      float l = p;
#pragma unroll
      for (int o2 = 4; o2 < 64; o2 <<= 1) l += __shfl_xor(l, o2, 64);
      mg[g] = m;
      lg[g] = l;  // the xor-4..32 sum runs over one lane per key (same quarter)
      if (quarter == 0) ps[w][g][t] = p;
    }
    // 3) P.V over the wave's keys (same-wave LDS ops stay in order)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll 4
    for (int k = 0; k < n_valid; ++k) {
      const bf16x2 vv = *reinterpret_cast<const bf16x2*>(&vs[w][k][2 * lane]);
      const float v0 = (float)vv[0], v1 = (float)vv[1];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = ps[w][g][k];
        o[g][0] = fmaf(p, v0, o[g][0]);
        o[g][1] = fmaf(p, v1, o[g][1]);
      }
    }
  }
  __syncthreads();  // every wave's P.V has read its V rows: the region becomes `so`
#pragma unroll
  for (int g = 0; g < G; ++g) {
    so[w][g][2 * lane] = o[g][0];
    so[w][g][2 * lane + 1] = o[g][1];
    if (lane == 0) {
      sm[w][g] = mg[g];
      sl[w][g] = lg[g];
    }
  }
  __syncthreads();
  const int Hq = Hkv * G;
  for (int i = tid; i < G * HD; i += WAVES * 64) {
    const int g = i / HD, d = i % HD;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) M = fmaxf(M, sm[ww][g]);
    float num = 0.f, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        const float e = __expf(sm[ww][g] - M);
        num = fmaf(e, so[ww][g][d], num);
        den = fmaf(e, sl[ww][g], den);
      }
    }
    const int hq = h * G + g;
    if (n_chunks == 1) {
      out[(size_t)r * ldo + (size_t)hq * HD + d] = f2bf(num / den);
    } else {
      const size_t pidx = ((size_t)r * Hq + hq) * n_chunks + c;
      part_o[pidx * HD + d] = num;
      if (d == 0) {
        part_ml[pidx * 2] = M;
        part_ml[pidx * 2 + 1] = den;
      }
    }
  }
}

// Split-K combine: one block per (row, q head).  The chunk statistics go to LDS first
// (one load per chunk, all in flight together), then CG groups of HD threads each sum
// the partial outputs of every CG-th chunk with 8 loads in flight per thread, and the
// groups meet in LDS.  (A serial per-dimension loop over the chunks leaves one load
// in flight per thread: ~85 us per layer at a 32K context.)
constexpr int CG = 8;                  // chunk groups per block
constexpr int MAX_CHUNKS = 131072 / CHUNK;  // 128K-token contexts
__global__ __launch_bounds__(HD * CG) void attn_combine_kernel(const float* __restrict__ part_o,
                                                               const float* __restrict__ part_ml,
                                                               const int* __restrict__ ctx_lens,
                                                               int Hq, int n_chunks,
                                                               bf16* __restrict__ out, int ldo) {
  __shared__ float s_e[MAX_CHUNKS];  // exp(m_c - M)
  __shared__ float s_l[MAX_CHUNKS];
  __shared__ float s_red[CG][HD];
  __shared__ float s_wmax[HD * CG / 64];
  const int r = blockIdx.x, hq = blockIdx.y, tid = threadIdx.x;
  const int d = tid % HD, grp = tid / HD;
  const int nc = min(min((ctx_lens[r] + CHUNK - 1) / CHUNK, n_chunks), MAX_CHUNKS);
  const size_t base = ((size_t)r * Hq + hq) * n_chunks;
  float mloc = -INFINITY;
  for (int c = tid; c < nc; c += HD * CG) {
    const float m = part_ml[(base + c) * 2];
    s_e[c] = m;
    s_l[c] = part_ml[(base + c) * 2 + 1];
    mloc = fmaxf(mloc, m);
  }
  mloc = wave_max(mloc);
  if ((tid & 63) == 0) s_wmax[tid >> 6] = mloc;
  __syncthreads();
  float M = -INFINITY;
#pragma unroll
  for (int i = 0; i < HD * CG / 64; ++i) M = fmaxf(M, s_wmax[i]);
  __syncthreads();
  for (int c = tid; c < nc; c += HD * CG) s_e[c] = s_e[c] == -INFINITY ? 0.f : __expf(s_e[c] - M);
  __syncthreads();
  float num = 0.f;
  const float* po = part_o + base * HD + d;
  int c = grp;
  for (; c + 7 * CG < nc; c += 8 * CG) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = po[(size_t)(c + u * CG) * HD];
#pragma unroll
    for (int u = 0; u < 8; ++u) num = fmaf(s_e[c + u * CG], v[u], num);
  }
  for (; c < nc; c += CG) num = fmaf(s_e[c], po[(size_t)c * HD], num);
  s_red[grp][d] = num;
  __syncthreads();
  if (grp == 0) {
    float tot = 0.f, den = 0.f;
#pragma unroll
    for (int g = 0; g < CG; ++g) tot += s_red[g][d];
    for (int i = 0; i < nc; ++i) den = fmaf(s_e[i], s_l[i], den);
    out[(size_t)r * ldo + (size_t)hq * HD + d] = f2bf(den > 0.f ? tot / den : 0.f);
  }
}

// ---- single-chunk decode attention on MFMA (contexts <= 256 keys: chat decode) ----
// The 16-wave kernel above spends its time in a serial per-lane P.V loop over LDS and a
// 16-way cross-wave merge; here 4 waves x 64 keys (= one KV page per wave, so one
// block-table load per wave) run both products on v_mfma_f32_16x16x32_bf16 with the
// query heads on the MFMA's N axis (G <= 16, padded with zero rows):
//   S^T[key][head] = K . Q^T   (A = 16 keys x 32 dims straight from the page, 16 B per
//                               lane; B = q fragments, loaded once)
//   O[head][dim]  += P . V     (A = P: the S^T accumulator registers after the softmax ARE
//                               the A fragment -- lane (head, key group) -- with the 32
//                               keys of a k-step taken as two 16-key blocks; B = V^T
//                               fragments read from the wave's V rows in LDS with the
//                               same key permutation)
// and the 4 wave partials merge once through LDS.
constexpr int MW = 4;            // waves
constexpr int MKPW = 64;         // keys per wave = one page
constexpr int MVS = HD + 8;      // V row stride (bf16) in LDS: conflict-free 16-B writes

template <int G>
__global__ __launch_bounds__(MW * 64) void paged_attn_mfma_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ bt, int bt_stride, const int* __restrict__ row_bt,
    const int* __restrict__ ctx_lens, int Hkv, float scale, bf16* __restrict__ out, int ldo) {
  static_assert(G >= 1 && G <= 16, "query heads on the MFMA N axis");
  __shared__ __attribute__((aligned(16))) bf16 vs[MW][MKPW][MVS];
  __shared__ float so[MW][G][HD];
  __shared__ float sm[MW][G], sl[MW][G];
  const int h = blockIdx.x, r = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kk = lane & 15, qd = lane >> 4;
  const int ctx = ctx_lens[r];
  const int rb = row_bt ? row_bt[r] : r;
  const int page = bt[(size_t)rb * bt_stride + min(w, bt_stride - 1)];  // wave-uniform
  const size_t pbase = ((size_t)page * Hkv + h) * PAGE * HD;

  // loads: K and V rows of this wave's 64 keys (block b = keys 16b.., lane row kk, dims
  // 32s + 8qd..), q fragments of the G heads (rows kk >= G are zero)
  bf16x8 kr[4][4], vr[4][4], qf[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const bf16x8* kp = reinterpret_cast<const bf16x8*>(kc + pbase + (size_t)(16 * b + kk) * HD + 8 * qd);
    const bf16x8* vp = reinterpret_cast<const bf16x8*>(vc + pbase + (size_t)(16 * b + kk) * HD + 8 * qd);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) kr[b][s2] = kp[4 * s2];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) vr[b][s2] = vp[4 * s2];
  }
  {
    const bf16x8* qp = reinterpret_cast<const bf16x8*>(q + (size_t)r * ldq +
                                                       (size_t)(h * G + min(kk, G - 1)) * HD + 8 * qd);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) qf[s2] = kk < G ? qp[4 * s2] : zero_bf16x8();
  }
  const int n_valid = min(max(ctx - w * MKPW, 0), MKPW);  // wave-uniform

  // V rows -> LDS (this wave's region only: a wave barrier orders them for its reads)
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
      *reinterpret_cast<bf16x8*>(&vs[w][16 * b + kk][32 * s2 + 8 * qd]) = vr[b][s2];

  float mg = -INFINITY, lg = 0.f;  // per head kk (every lane of column kk agrees)
  f32x4 o[HD / 16];
#pragma unroll
  for (int c = 0; c < HD / 16; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (n_valid > 0) {
    // S^T blocks: lane holds keys 16b + 4qd + j (j < 4) of head kk
    f32x4 st[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      st[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        st[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr[b][s2], qf[s2], st[b], 0, 0, 0);
    }
    float m = -INFINITY;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = 16 * b + 4 * qd + j < n_valid;
        st[b][j] = ok ? st[b][j] * scale : -INFINITY;
        m = fmaxf(m, st[b][j]);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __expf(st[b][j] - m);  // -inf -> 0
        st[b][j] = p;
        l += p;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    mg = m;
    lg = l;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's V rows are in LDS
    __builtin_amdgcn_wave_barrier();
    // P.V: k-step t covers key blocks 2t (A slots 0-3) and 2t+1 (slots 4-7)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = f2bf(st[2 * t][j]);
        pa[4 + j] = f2bf(st[2 * t + 1][j]);
      }
#pragma unroll
      for (int c = 0; c < HD / 16; ++c) {
        bf16x8 vb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vb[j] = vs[w][32 * t + 4 * qd + j][16 * c + kk];
          vb[4 + j] = vs[w][32 * t + 16 + 4 * qd + j][16 * c + kk];
        }
        o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[c], 0, 0, 0);
      }
    }
  }
  // O accumulators: lane holds O[head 4qd + j][dim 16c + kk]
#pragma unroll
  for (int c = 0; c < HD / 16; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int hd = 4 * qd + j;
      if (hd < G) so[w][hd][16 * c + kk] = o[c][j];
    }
  if (qd == 0 && kk < G) {
    sm[w][kk] = mg;
    sl[w][kk] = lg;
  }
  __syncthreads();
  for (int i = tid; i < G * HD; i += MW * 64) {
    const int hd = i / HD, d = i % HD;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < MW; ++ww) M = fmaxf(M, sm[ww][hd]);
    float num = 0.f, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < MW; ++ww) {
        const float e = __expf(sm[ww][hd] - M);
        num = fmaf(e, so[ww][hd][d], num);
        den = fmaf(e, sl[ww][hd], den);
      }
    }
    out[(size_t)r * ldo + (size_t)(h * G + hd) * HD + d] = f2bf(den > 0.f ? num / den : 0.f);
  }
}

// Opt-in (p2p_paged_attention_mfma(1)): measured on MI355X it is 7.7-7.9 us per launch
// at 44-256 keys vs 6.3-8.1 us for the 16-wave kernel (profiles/r2_decode_attn_mfma.jsonl):
// both are bound by the block-table -> K/V load chain, not by the arithmetic.
static int g_attn_mfma = 0;

template <int G>
int launch_attn(const void* q, int ldq, const void* kc, const void* vc, const int* bt,
                int bt_stride, const int* row_bt, const int* ctx, int R, int Hkv, float scale,
                int n_chunks, void* out, int ldo, float* part_o, float* part_ml, hipStream_t st) {
  if (n_chunks == 1 && g_attn_mfma) {
    hipLaunchKernelGGL((paged_attn_mfma_kernel<G>), dim3(Hkv, R), dim3(MW * 64), 0, st,
                       (const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, bt, bt_stride, row_bt,
                       ctx, Hkv, scale, (bf16*)out, ldo);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((paged_attn_kernel<G>), dim3(n_chunks, Hkv, R), dim3(WAVES * 64), 0, st,
                     (const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, bt, bt_stride, row_bt,
                     ctx, Hkv, scale, n_chunks, (bf16*)out, ldo, part_o, part_ml);
  int e = (int)hipGetLastError();
  if (e || n_chunks == 1) return e;
  hipLaunchKernelGGL(attn_combine_kernel, dim3(R, Hkv * G), dim3(HD * CG), 0, st, part_o, part_ml, ctx,
                     Hkv * G, n_chunks, (bf16*)out, ldo);
  return (int)hipGetLastError();
}

}  // namespace

// 1: contexts <= 256 keys run the 4-wave MFMA kernel; 0 (default): the 16-wave kernel.
P2P_API void p2p_paged_attention_mfma(int on) { g_attn_mfma = on; }

// row_bt null = identity (decode batches: row r is sequence r), one dependent load less
// on the kernel's critical path (row_bt -> page -> K/V becomes page -> K/V).
// max_ctx bounds the number of 256-key chunks (grid.x); rows whose context is
// shorter exit early.  part_o / part_ml: workspace of R*Hq*n_chunks*(128 | 2) floats,
// unused when max_ctx <= 256.
P2P_API int p2p_paged_attention(const void* q, int ldq, const void* k_cache, const void* v_cache,
                                const int* block_tables, int bt_stride, const int* row_bt,
                                const int* ctx_lens, int R, int Hq, int Hkv, int head_dim,
                                float scale, int max_ctx, void* out, int ldo, float* part_o,
                                float* part_ml, hipStream_t stream) {
  if (head_dim != HD || Hkv <= 0 || Hq % Hkv != 0 || R <= 0) return (int)hipErrorInvalidValue;
  const int n_chunks = (max_ctx + CHUNK - 1) / CHUNK;
  if (n_chunks > 1 && (!part_o || !part_ml)) return (int)hipErrorInvalidValue;
  if (n_chunks > MAX_CHUNKS) return (int)hipErrorInvalidValue;
  switch (Hq / Hkv) {
    case 1: return launch_attn<1>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, n_chunks, out, ldo, part_o, part_ml, stream);
    case 2: return launch_attn<2>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, n_chunks, out, ldo, part_o, part_ml, stream);
    case 4: return launch_attn<4>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, n_chunks, out, ldo, part_o, part_ml, stream);
    case 8: return launch_attn<8>(q, ldq, k_cache, v_cache, block_tables, bt_stride, row_bt, ctx_lens, R, Hkv, scale, n_chunks, out, ldo, part_o, part_ml, stream);
  }
  return (int)hipErrorInvalidValue;
}
