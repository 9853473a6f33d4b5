// Small memory-bound kernels of the decode/prefill step: embedding / row gather,
// RoPE (llama3-scaled table) + paged KV-cache write, greedy argmax, and the
// graph-resident "advance" step that lets many decode steps replay from one
// hipGraph without a host round trip.
#include "common.h"

namespace {

constexpr int PAGE = 64;
constexpr int HD = 128;
constexpr int KEY_SHARDS = 32;

// max over the KEY_SHARDS argmax keys of row m, resetting them; -> token id
__device__ __forceinline__ int reduce_keys(unsigned long long* keys, int m) {
  unsigned long long best = 0;
  unsigned long long* k = keys + (size_t)m * KEY_SHARDS;
#pragma unroll
  for (int i = 0; i < KEY_SHARDS; ++i) {
    const unsigned long long v = k[i];
    best = v > best ? v : best;
    k[i] = 0ull;
  }
  return (int)(0xFFFFFFFFu - (unsigned)(best & 0xFFFFFFFFull));
}

// out[t, :] = src[idx[t], :]  (H bf16 per row, 16-B vectors)
// An index outside [0, n_src) -- e.g. a token id decoded from the argmax keys of a step
// whose collective timed out -- yields a zero row instead of a wild read (the fault word
// already makes the host raise; this keeps the device from faulting first).
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16* __restrict__ src,
                                                          const int* __restrict__ idx, int H,
                                                          int n_src, bf16* __restrict__ out,
                                                          int ldo) {
  const int t = blockIdx.x;
  const int r = idx[t];
  bf16x8* o = reinterpret_cast<bf16x8*>(out + (size_t)t * ldo);
  if (r < 0 || r >= n_src) {
    for (int i = threadIdx.x; i < H / 8; i += 256) o[i] = zero_bf16x8();
    return;
  }
  const bf16x8* s = reinterpret_cast<const bf16x8*>(src + (size_t)r * H);
  for (int i = threadIdx.x; i < H / 8; i += 256) o[i] = s[i];
}

// qkv: [T, (Hq + 2 Hkv) * 128]; one wave per head; lane l rotates the pair (l, l + 64)
// (HF rotate_half convention).  cs: float2 [max_pos][64] = (cos, sin).
// q heads -> q_out [T, Hq*128]; k heads (rotated) and v heads -> paged cache at slot[t]
// (slot = page * 64 + offset; slot < 0 skips the cache write, e.g. padding rows).
__global__ __launch_bounds__(256) void rope_cache_kernel(
    const bf16* __restrict__ qkv, int ldqkv, const int* __restrict__ pos,
    const int* __restrict__ slots, const float2* __restrict__ cs, int Hq, int Hkv,
    bf16* __restrict__ q_out, int ldq, bf16* __restrict__ kc, bf16* __restrict__ vc) {
  const int t = blockIdx.y;
  const int hh = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (hh >= Hq + 2 * Hkv) return;
  const bf16* row = qkv + (size_t)t * ldqkv + (size_t)hh * HD;
  const float x1 = (float)row[l], x2 = (float)row[l + 64];
  if (hh < Hq + Hkv) {
    const float2 c = cs[(size_t)pos[t] * 64 + l];
    const float y1 = x1 * c.x - x2 * c.y;
    const float y2 = x2 * c.x + x1 * c.y;
    if (hh < Hq) {
      bf16* o = q_out + (size_t)t * ldq + (size_t)hh * HD;
      o[l] = f2bf(y1);
      o[l + 64] = f2bf(y2);
    } else {
      const int slot = slots[t];
      if (slot < 0) return;
      const int h = hh - Hq;
      bf16* o = kc + (((size_t)(slot / PAGE) * Hkv + h) * PAGE + (slot % PAGE)) * HD;
      o[l] = f2bf(y1);
      o[l + 64] = f2bf(y2);
    }
  } else {
    const int slot = slots[t];
    if (slot < 0) return;
    const int h = hh - Hq - Hkv;
    bf16* o = vc + (((size_t)(slot / PAGE) * Hkv + h) * PAGE + (slot % PAGE)) * HD;
    o[l] = row[l];
    o[l + 64] = row[l + 64];
  }
}

// Greedy sampling: out[m] = argmax_v logits[m, v] (first index on ties, like torch).
__global__ __launch_bounds__(1024) void argmax_kernel(const float* __restrict__ logits, int V,
                                                      int ld, int* __restrict__ out) {
  const int m = blockIdx.x;
  const float* row = logits + (size_t)m * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const int V4 = V / 4;
  const float4* r4 = reinterpret_cast<const float4*>(row);
  for (int i = threadIdx.x; i < V4; i += 1024) {
    const float4 v = r4[i];
    const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (a[j] > best) { best = a[j]; bi = 4 * i + j; }
  }
  for (int i = V4 * 4 + threadIdx.x; i < V; i += 1024)
    if (row[i] > best) { best = row[i]; bi = i; }
  // NaN-free inputs assumed; ties -> smaller index.
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  __shared__ float sb[16];
  __shared__ int si[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sb[w] = best; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 16; ++k)
      if (sb[k] > best || (sb[k] == best && si[k] < bi)) { best = sb[k]; bi = si[k]; }
    out[m] = bi;
  }
}

// Graph-resident decode-state advance for B sequences (one thread each):
//   hist[b, *step] = ids[b]; pos[b] += 1; ctx[b] = pos[b] + 1;
//   slot[b] = bt[b][pos / 64] * 64 + pos % 64;  then (*step)++ by thread 0.
__global__ void advance_kernel(int* __restrict__ ids, unsigned long long* __restrict__ keys,
                               int* __restrict__ pos, int* __restrict__ ctx,
                               int* __restrict__ slots, const int* __restrict__ bt, int bt_stride,
                               int* __restrict__ hist, int hist_stride, int* __restrict__ step,
                               int B) {
  const int b = threadIdx.x;
  const int st = *step;
  if (b < B) {
    if (keys) {  // greedy keys from the fused LM-head argmax -> token ids; reset for next step
      ids[b] = reduce_keys(keys, b);
    }
    if (hist) hist[(size_t)b * hist_stride + st] = ids[b];
    const int p = pos[b] + 1;
    pos[b] = p;
    ctx[b] = p + 1;
    slots[b] = bt[(size_t)b * bt_stride + p / PAGE] * PAGE + (p % PAGE);
  }
  __syncthreads();
  if (b == 0) *step = st + 1;
}

__global__ void argmax_finalize_kernel(unsigned long long* __restrict__ keys, int* __restrict__ ids,
                                       int M) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) ids[m] = reduce_keys(keys, m);
}

}  // namespace

P2P_API int p2p_argmax_finalize(unsigned long long* keys, int* ids, int M, hipStream_t st) {
  if (M <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(argmax_finalize_kernel, dim3((M + 255) / 256), dim3(256), 0, st, keys, ids, M);
  return (int)hipGetLastError();
}

P2P_API int p2p_gather_rows(const void* src, const int* idx, int T, int H, int n_src, void* out,
                            int ldo, hipStream_t st) {
  if (H % 8 != 0 || T <= 0 || n_src <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(T), dim3(256), 0, st, (const bf16*)src, idx, H,
                     n_src, (bf16*)out, ldo);
  return (int)hipGetLastError();
}

P2P_API int p2p_rope_cache(const void* qkv, int ldqkv, const int* pos, const int* slots,
                           const void* cos_sin, int T, int Hq, int Hkv, int head_dim, void* q_out,
                           int ldq, void* k_cache, void* v_cache, hipStream_t st) {
  if (head_dim != HD || T <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rope_cache_kernel, dim3((Hq + 2 * Hkv + 3) / 4, T), dim3(256), 0, st,
                     (const bf16*)qkv, ldqkv, pos, slots, (const float2*)cos_sin, Hq, Hkv,
                     (bf16*)q_out, ldq, (bf16*)k_cache, (bf16*)v_cache);
  return (int)hipGetLastError();
}

P2P_API int p2p_argmax(const float* logits, int M, int V, int ld, int* out, hipStream_t st) {
  if (M <= 0 || V <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(argmax_kernel, dim3(M), dim3(1024), 0, st, logits, V, ld, out);
  return (int)hipGetLastError();
}

P2P_API int p2p_advance(int* ids, unsigned long long* keys, int* pos, int* ctx, int* slots,
                        const int* bt, int bt_stride, int* hist, int hist_stride, int* step, int B,
                        hipStream_t st) {
  if (B <= 0 || B > 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(((B + 63) / 64) * 64), 0, st, ids, keys, pos,
                     ctx, slots, bt, bt_stride, hist, hist_stride, step, B);
  return (int)hipGetLastError();
}

// Row-major X [M, K] -> fragment-major Xf: 16-row m-tiles, each K/32 MFMA A fragments of
// 1 KiB (lane l of fragment (mt, s) holds X[16 mt + (l & 15)][32 s + 8 (l >> 4) .. + 7]);
// rows past M are zero.  One thread per 16-byte chunk.
__global__ __launch_bounds__(256) void pack_frag_kernel(const bf16* __restrict__ X, int ldx, int M,
                                                         int S, int chunks, bf16x8* __restrict__ Xf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= chunks) return;
  const int lane = i & 63, s = (i >> 6) % S, mt = (i >> 6) / S;
  const int row = mt * 16 + (lane & 15);
  Xf[i] = row < M ? *reinterpret_cast<const bf16x8*>(X + (size_t)row * ldx + 32 * s + 8 * (lane >> 4))
                  : zero_bf16x8();
}

P2P_API int p2p_pack_frag(const void* X, int ldx, int M, int K, void* Xf, hipStream_t st) {
  if (M <= 0 || K % 32 || ldx % 8) return (int)hipErrorInvalidValue;
  const int S = K / 32, chunks = ((M + 15) / 16) * S * 64;
  hipLaunchKernelGGL(pack_frag_kernel, dim3((chunks + 255) / 256), dim3(256), 0, st, (const bf16*)X,
                     ldx, M, S, chunks, (bf16x8*)Xf);
  return (int)hipGetLastError();
}
