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

}  // namespace

P2P_API int p2p_moe_route(const float* logits, int ldl, int R, int E, int K, int e_lo, int e_local,
                          int* topk_ids, float* topk_w, int* cnt, int* rows, int rows_stride,
                          hipStream_t st) {
  if (E > MAX_E || K > MAX_K || K > E || R <= 0 || rows_stride < R) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(256), 0, st, logits, ldl, R, E, K, e_lo,
                     e_local, topk_ids, topk_w, cnt, rows, rows_stride);
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
