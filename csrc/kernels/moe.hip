// Mixtral sparse-MoE glue kernels (the expert GEMMs themselves are the grouped
// mode of skinny_gemm.hip, so an expert nobody routed to streams no weights):
//   moe_route   : softmax over the router logits, top-k, renormalised weights,
//                 per-local-expert slot lists (slot = token * top_k + k)
//   moe_combine : h[token] += sum_k o[slot]  (or a partial for the EP/TP all-reduce)
#include "common.h"

namespace {

constexpr int MAX_E = 64;
constexpr int MAX_K = 8;

__global__ __launch_bounds__(256) void moe_route_kernel(const float* __restrict__ logits, int ldl,
                                                        int R, int E, int K, int e_lo, int e_local,
                                                        int* __restrict__ topk_ids,
                                                        float* __restrict__ topk_w,
                                                        int* __restrict__ cnt, int* __restrict__ rows,
                                                        int rows_stride) {
  __shared__ int s_cnt[MAX_E];
  for (int i = threadIdx.x; i < MAX_E; i += blockDim.x) s_cnt[i] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const float* l = logits + (size_t)r * ldl;
    float m = -INFINITY;
    for (int e = 0; e < E; ++e) m = fmaxf(m, l[e]);
    float p[MAX_E];
    float sum = 0.f;
    for (int e = 0; e < E; ++e) {
      p[e] = __expf(l[e] - m);
      sum += p[e];
    }
    int sel[MAX_K];
    float ws[MAX_K];
    float wsum = 0.f;
    for (int k = 0; k < K; ++k) {
      int best = -1;
      float bv = -1.f;
      for (int e = 0; e < E; ++e) {
        bool taken = false;
        for (int j = 0; j < k; ++j) taken |= (sel[j] == e);
        if (!taken && p[e] > bv) {
          bv = p[e];
          best = e;
        }
      }
      sel[k] = best;
      ws[k] = bv / sum;
      wsum += ws[k];
    }
    for (int k = 0; k < K; ++k) {
      const int slot = r * K + k;
      topk_ids[slot] = sel[k];
      topk_w[slot] = ws[k] / wsum;
      const int le = sel[k] - e_lo;
      if (le >= 0 && le < e_local) {
        const int pos = atomicAdd(&s_cnt[le], 1);
        rows[(size_t)le * rows_stride + pos] = slot;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < e_local; i += blockDim.x) cnt[i] = s_cnt[i];
}

// Fused router + route for decode/prefill chunks (R <= 64 rows): one wave per row
// computes rstd(h) and the E router logits (norm gain folded into Wr) with 16-byte
// loads and wave reductions, then softmax / top-k / renormalisation in registers
// (no scratch arrays), and the per-local-expert slot lists through LDS atomics.
// Replaces the padded router GEMM + moe_route pair (two dependent launches).
template <int E>
__global__ __launch_bounds__(512) void moe_router_route_kernel(
    const bf16* __restrict__ h, int ldh, int R, int H, const bf16* __restrict__ wr, float eps,
    int K, int e_lo, int e_local, int* __restrict__ topk_ids, float* __restrict__ topk_w,
    int* __restrict__ cnt, int* __restrict__ rows, int rows_stride) {
  __shared__ int s_cnt[E];
  __shared__ float s_part[64][E + 1];  // per (row, H slice): E logit partials + sum of squares
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x < E) s_cnt[threadIdx.x] = 0;
  // phase 1: logits.  With few rows the H reduction is split over the waves (a batch-1
  // decode step would otherwise leave 7 of 8 waves idle behind one serial load chain).
  const int ns = R >= nw ? 1 : nw / R;  // H slices per row
  const int C = H / 8;                  // 16-byte chunks per row
  for (int item = w; item < R * ns; item += nw) {
    const int r = item / ns, sl = item % ns;
    const bf16x8* hp = reinterpret_cast<const bf16x8*>(h + (size_t)r * ldh);
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    float ss = 0.f;
    const int c1 = (sl + 1) * C / ns;
#pragma unroll 2
    for (int c = sl * C / ns + lane; c < c1; c += 64) {
      const bf16x8 x = hp[c];
      float xf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xf[j] = (float)x[j];
        ss = fmaf(xf[j], xf[j], ss);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const bf16x8 wv = reinterpret_cast<const bf16x8*>(wr + (size_t)e * H)[c];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[e] = fmaf(xf[j], (float)wv[j], acc[e]);
      }
    }
    ss = wave_sum(ss);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = wave_sum(acc[e]);
    if (lane == 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) s_part[item][e] = acc[e];
      s_part[item][E] = ss;
    }
  }
  __syncthreads();
  // phase 2: softmax / top-k / slot lists, one wave per row
  for (int r = w; r < R; r += nw) {
    float acc[E];
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    for (int sl = 0; sl < ns; ++sl) {
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += s_part[r * ns + sl][e];
      ss += s_part[r * ns + sl][E];
    }
    const float rstd = rsqrtf(ss / (float)H + eps);
    float m = -INFINITY;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      acc[e] *= rstd;
      m = fmaxf(m, acc[e]);
    }
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      acc[e] = __expf(acc[e] - m);
      sum += acc[e];
    }
    // top-k by repeated arg-max over a taken mask (all indices compile-time)
    unsigned taken = 0;
    float wsum = 0.f;
    int sel[MAX_K];
    float wk[MAX_K];
    for (int k = 0; k < K; ++k) {
      int best = 0;
      float bv = -1.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (!(taken >> e & 1u) && acc[e] > bv) {
          bv = acc[e];
          best = e;
        }
      }
      taken |= 1u << best;
      sel[k] = best;
      wk[k] = bv / sum;
      wsum += wk[k];
    }
    if (lane == 0) {
      for (int k = 0; k < K; ++k) {
        const int slot = r * K + k;
        topk_ids[slot] = sel[k];
        topk_w[slot] = wk[k] / wsum;
        const int le = sel[k] - e_lo;
        if (le >= 0 && le < e_local) {
          const int pos = atomicAdd(&s_cnt[le], 1);
          rows[(size_t)le * rows_stride + pos] = slot;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < e_local) cnt[threadIdx.x] = s_cnt[threadIdx.x];
}

// Router logits for prefill-size chunks: one workgroup per row (the fused single-block
// kernel above serialises ~R/8 rows per wave -- 69 us per layer at 43 rows); 4 waves
// split H, LDS combines.  logits[r][e] = rstd(h_r) * h_r . wr_e  (gain folded into wr).
template <int E>
__global__ __launch_bounds__(256) void moe_router_logits_kernel(const bf16* __restrict__ h, int ldh,
                                                                int H, const bf16* __restrict__ wr,
                                                                float eps, float* __restrict__ logits,
                                                                int ldl) {
  __shared__ float s_part[4][E + 1];
  const int r = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bf16x8* hp = reinterpret_cast<const bf16x8*>(h + (size_t)r * ldh);
  const int C = H / 8;
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  float ss = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const bf16x8 x = hp[c];
    float xf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xf[j] = (float)x[j];
      ss = fmaf(xf[j], xf[j], ss);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const bf16x8 wv = reinterpret_cast<const bf16x8*>(wr + (size_t)e * H)[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[e] = fmaf(xf[j], (float)wv[j], acc[e]);
    }
  }
  ss = wave_sum(ss);
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = wave_sum(acc[e]);
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < E; ++e) s_part[w][e] = acc[e];
    s_part[w][E] = ss;
  }
  __syncthreads();
  if (threadIdx.x < E) {
    const float t = s_part[0][E] + s_part[1][E] + s_part[2][E] + s_part[3][E];
    const float v = s_part[0][threadIdx.x] + s_part[1][threadIdx.x] + s_part[2][threadIdx.x] +
                    s_part[3][threadIdx.x];
    logits[(size_t)r * ldl + threadIdx.x] = v * rsqrtf(t / (float)H + eps);
  }
}

// accumulate=1: h[r] += sum_k o[r*K+k] over local experts;  0: out[r] = that sum.
__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16* __restrict__ o, int ldo_,
                                                          const int* __restrict__ topk_ids, int K,
                                                          int e_lo, int e_local, int H,
                                                          bf16* __restrict__ out, int ld_out,
                                                          int accumulate) {
  const int r = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const int le = topk_ids[r * K + k] - e_lo;
      if (le < 0 || le >= e_local) continue;
      const bf16x8 v = reinterpret_cast<const bf16x8*>(o + (size_t)(r * K + k) * ldo_)[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
    bf16x8* dst = reinterpret_cast<bf16x8*>(out + (size_t)r * ld_out) + c;
    bf16x8 res;
    if (accumulate) {
      const bf16x8 h = *dst;
#pragma unroll
      for (int j = 0; j < 8; ++j) res[j] = f2bf((float)h[j] + acc[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) res[j] = f2bf(acc[j]);
    }
    *dst = res;
  }
}

// ---- expert-parallel all-to-all (DP attention + EP): dispatch, slot grouping, combine ----
// Slot s = token * K + k goes to rank dest = expert / El.  Its send row is
//   static capacity C > 0 : dest * C + pos      (graph-capturable, padded)
//   exact (C == 0)        : off[dest] + pos     (packed; off = exclusive prefix of counts)
// where pos is drawn with an atomic per destination (row order inside a destination is
// free: every expert row is computed independently, and the combine sums a token's K
// returns in k order, so results do not depend on it).
__global__ __launch_bounds__(256) void a2a_assign_kernel(const int* __restrict__ topk_ids,
                                                         int n_slots, int El,
                                                         int* __restrict__ dest_cnt,
                                                         int* __restrict__ slot_pos) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  const int dest = topk_ids[s] / El;
  slot_pos[s] = atomicAdd(&dest_cnt[dest], 1);
}

__global__ __launch_bounds__(256) void a2a_pack_kernel(const bf16* __restrict__ h, int ldh, int H,
                                                       const int* __restrict__ topk_ids,
                                                       const float* __restrict__ topk_w, int K,
                                                       int El, int W, int C,
                                                       const int* __restrict__ dest_cnt,
                                                       const int* __restrict__ slot_pos,
                                                       bf16* __restrict__ send_x,
                                                       int* __restrict__ send_meta,
                                                       int* __restrict__ send_map) {
  const int s = blockIdx.x;
  const int e = topk_ids[s];
  const int dest = e / El;
  int off = 0;
  if (C > 0) {
    off = dest * C;
  } else {
    for (int d = 0; d < dest; ++d) off += dest_cnt[d];
  }
  const int row = off + slot_pos[s];
  const bf16x8* src = reinterpret_cast<const bf16x8*>(h + (size_t)(s / K) * ldh);
  bf16x8* dst = reinterpret_cast<bf16x8*>(send_x + (size_t)row * H);
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) dst[c] = src[c];
  if (threadIdx.x == 0) {
    send_meta[2 * row] = e % El;
    send_meta[2 * row + 1] = __float_as_int(topk_w[s]);
    send_map[s] = row;
  }
}

// received rows -> per-local-expert slot lists (rows whose expert id is < 0 are padding)
__global__ __launch_bounds__(1024) void a2a_group_kernel(const int* __restrict__ meta, int n,
                                                         int El, int* __restrict__ cnt,
                                                         int* __restrict__ rows, int rows_stride) {
  __shared__ int s_cnt[MAX_E];
  for (int i = threadIdx.x; i < MAX_E; i += blockDim.x) s_cnt[i] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    const int le = meta[2 * r];
    if (le < 0 || le >= El) continue;
    const int pos = atomicAdd(&s_cnt[le], 1);
    rows[(size_t)le * rows_stride + pos] = r;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < El; i += blockDim.x) cnt[i] = s_cnt[i];
}

// h[token] += sum_k back[send_map[token * K + k]]  (fp32 sum in k order, one rounding)
__global__ __launch_bounds__(256) void a2a_combine_kernel(const bf16* __restrict__ back, int H,
                                                          const int* __restrict__ send_map, int K,
                                                          bf16* __restrict__ h, int ldh) {
  const int r = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const bf16x8 v = reinterpret_cast<const bf16x8*>(back + (size_t)send_map[r * K + k] * H)[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
    bf16x8* dst = reinterpret_cast<bf16x8*>(h + (size_t)r * ldh) + c;
    const bf16x8 hv = *dst;
    bf16x8 res;
#pragma unroll
    for (int j = 0; j < 8; ++j) res[j] = f2bf((float)hv[j] + acc[j]);
    *dst = res;
  }
}

}  // namespace

// Dispatch for the EP all-to-all.  dest_cnt [W] (zeroed by this call), slot_pos [R*K]
// scratch; send_x [W*C | R*K, H], send_meta [same, 2] int (static mode: pre-filled with
// -1 by this call so padding rows group nowhere), send_map [R*K].
P2P_API int p2p_moe_a2a_dispatch(const void* h, int ldh, int R, int H, const int* topk_ids,
                                 const float* topk_w, int K, int El, int W, int C, int* dest_cnt,
                                 int* slot_pos, void* send_x, int* send_meta, int* send_map,
                                 hipStream_t st) {
  if (R <= 0 || H % 8 || K <= 0 || El <= 0 || W <= 0 || C < 0) return (int)hipErrorInvalidValue;
  const int n = R * K;
  hipError_t e = hipMemsetAsync(dest_cnt, 0, sizeof(int) * W, st);
  if (e != hipSuccess) return (int)e;
  if (C > 0) {
    e = hipMemsetAsync(send_meta, 0xFF, sizeof(int) * 2 * (size_t)W * C, st);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(a2a_assign_kernel, dim3((n + 255) / 256), dim3(256), 0, st, topk_ids, n, El,
                     dest_cnt, slot_pos);
  hipLaunchKernelGGL(a2a_pack_kernel, dim3(n), dim3(256), 0, st, (const bf16*)h, ldh, H, topk_ids,
                     topk_w, K, El, W, C, dest_cnt, slot_pos, (bf16*)send_x, send_meta, send_map);
  return (int)hipGetLastError();
}

P2P_API int p2p_moe_a2a_group(const int* meta, int n, int El, int* cnt, int* rows, int rows_stride,
                              hipStream_t st) {
  if (n <= 0 || El <= 0 || El > MAX_E || rows_stride < n) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(a2a_group_kernel, dim3(1), dim3(1024), 0, st, meta, n, El, cnt, rows,
                     rows_stride);
  return (int)hipGetLastError();
}

P2P_API int p2p_moe_a2a_combine(const void* back, int H, const int* send_map, int R, int K,
                                void* h, int ldh, hipStream_t st) {
  if (R <= 0 || H % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(a2a_combine_kernel, dim3(R), dim3(256), 0, st, (const bf16*)back, H, send_map,
                     K, (bf16*)h, ldh);
  return (int)hipGetLastError();
}

P2P_API int p2p_moe_route(const float* logits, int ldl, int R, int E, int K, int e_lo, int e_local,
                          int* topk_ids, float* topk_w, int* cnt, int* rows, int rows_stride,
                          hipStream_t st) {
  if (E > MAX_E || K > MAX_K || K > E || R <= 0 || rows_stride < R) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(256), 0, st, logits, ldl, R, E, K, e_lo,
                     e_local, topk_ids, topk_w, cnt, rows, rows_stride);
  return (int)hipGetLastError();
}

// h: [R, H] bf16 residual rows (raw); wr: [E, H] bf16 router with the RMSNorm gain folded.
P2P_API int p2p_moe_router_route(const void* h, int ldh, int R, int H, const void* wr, float eps,
                                 int E, int K, int e_lo, int e_local, int* topk_ids, float* topk_w,
                                 int* cnt, int* rows, int rows_stride, hipStream_t st) {
  if (K > MAX_K || K > E || R <= 0 || R > 64 || H % 8 || rows_stride < R || e_local > E)
    return (int)hipErrorInvalidValue;
  const auto* hb = (const bf16*)h;
  const auto* wb = (const bf16*)wr;
#define P2P_ROUTER_CASE(EE)                                                                      \
  case EE:                                                                                      \
    hipLaunchKernelGGL(moe_router_route_kernel<EE>, dim3(1), dim3(512), 0, st, hb, ldh, R, H, wb, \
                       eps, K, e_lo, e_local, topk_ids, topk_w, cnt, rows, rows_stride);         \
    return (int)hipGetLastError();
  switch (E) {
    P2P_ROUTER_CASE(4)
    P2P_ROUTER_CASE(8)
    P2P_ROUTER_CASE(16)
  }
#undef P2P_ROUTER_CASE
  return (int)hipErrorInvalidValue;
}

// logits [R, >= E] fp32 of rstd(h) h Wr^T, one workgroup per row (prefill chunks).
P2P_API int p2p_moe_router_logits(const void* h, int ldh, int R, int H, const void* wr, int E,
                                  float eps, float* logits, int ldl, hipStream_t st) {
  if (R <= 0 || H % 8 || ldl < E) return (int)hipErrorInvalidValue;
  const auto* hb = (const bf16*)h;
  const auto* wb = (const bf16*)wr;
  switch (E) {
    case 4: hipLaunchKernelGGL(moe_router_logits_kernel<4>, dim3(R), dim3(256), 0, st, hb, ldh, H, wb, eps, logits, ldl); break;
    case 8: hipLaunchKernelGGL(moe_router_logits_kernel<8>, dim3(R), dim3(256), 0, st, hb, ldh, H, wb, eps, logits, ldl); break;
    case 16: hipLaunchKernelGGL(moe_router_logits_kernel<16>, dim3(R), dim3(256), 0, st, hb, ldh, H, wb, eps, logits, ldl); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

P2P_API int p2p_moe_combine(const void* o, int ldo_, const int* topk_ids, int R, int K, int e_lo,
                            int e_local, int H, void* out, int ld_out, int accumulate,
                            hipStream_t st) {
  if (H % 8 != 0 || R <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(R), dim3(256), 0, st, (const bf16*)o, ldo_, topk_ids,
                     K, e_lo, e_local, H, (bf16*)out, ld_out, accumulate);
  return (int)hipGetLastError();
}
