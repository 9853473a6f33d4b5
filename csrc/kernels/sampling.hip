// Ollama-style stochastic sampling on the GPU: temperature -> top-k ->
// top-p -> multinomial draw, one workgroup per row, graph-capturable (all
// per-row parameters live in device memory; the random stream is a counter-based
// hash of (seed, position, token id), so a replayed graph draws fresh numbers
// every step without host state).
//
// Per row (1024 threads = 16 waves, the logits row stays L2-resident across passes):
//   1. top-k threshold by an MSB-first radix select over the order-preserving
//      32-bit keys of the fp32 logits: 4 passes of 8 bits, per-wave LDS histograms
//      (16 x 256 bins) summed, wave 0 finds the bin holding the k-th largest by a
//      shuffle suffix-scan.  The k-th largest key T is exact after 4 passes.  A
//      prefilter first bounds T from below by the k-th largest per-thread maximum,
//      so the passes run over a few hundred LDS-resident entries, not the row.
//   2. collect the k candidates: every key > T, then the keys == T with the lowest
//      ids (a second radix select over ~id, only when the k-th value is tied).
//   3. bitonic sort of the (<= 128) candidates in LDS, descending value, ascending id.
//   4. softmax(v / temperature) over them, inclusive cumsum; keep the smallest
//      prefix whose mass reaches top_p (drop i when cum_i - p_i > top_p).
//   5. exponential race: token = argmax_i p_i / E_i with E_i ~ Exp(1) -- exactly a
//      draw from the renormalised kept distribution.
// temperature <= 0 rows are greedy (argmax, lowest id on ties, like torch).
// The same semantics as engine/sampling.py (the CPU reference and the test oracle).
#include "common.h"

namespace {

constexpr int THREADS = 1024;
constexpr int NWAVES = THREADS / 64;
constexpr int KMAX = 128;
constexpr int CAP = 4096;  // prefiltered candidates held in LDS

__device__ __forceinline__ unsigned ord_key(float v) {
  unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float key_float(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// splitmix64 finaliser: a well-mixed 64-bit hash of the draw's coordinates
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// uniform in (0, 1) from (seed, pos, token): 24 random bits, centred in their cell
__device__ __forceinline__ float uniform01(unsigned long long seed, int pos, int tok) {
  const unsigned long long h =
      mix64(seed ^ mix64(((unsigned long long)(unsigned)pos << 32) | (unsigned)tok));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// Entry sources of one row: a dense logits row (ids = column + id_off), or -- vocab-
// parallel TP -- the gathered per-shard candidates: entry i of row r is slot i % seg of
// segment i / seg (one per rank), at vals/ids[(i / seg) * seg_stride + r * seg + i % seg].
struct Src {
  const float* vals;
  const int* ids;  // null: dense row
  int ld, seg;
  long long seg_stride;
  int id_off;
};

__global__ __launch_bounds__(THREADS) void sample_kernel(
    Src src, int V, const float* __restrict__ temp,
    const int* __restrict__ topk, const float* __restrict__ topp,
    const unsigned long long* __restrict__ seeds, const int* __restrict__ pos,
    int* __restrict__ out, float* __restrict__ cand_v, int* __restrict__ cand_id) {
  // cand_v != null: emit mode -- write this row's top-KMAX (value, id) pairs, sorted
  // (descending value, ascending id; padding -inf / INT_MAX) instead of drawing
  const int r = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool emit = cand_v != nullptr;
  const float* row = src.vals + (size_t)r * src.ld;
  const bool vec = !src.ids && ((src.ld | V) & 3) == 0;
  const float T = emit ? 1.f : temp[r];
  auto for_each_key = [&](const float* __restrict__, int, bool, auto&& f) {
    if (src.ids) {
      for (int i = threadIdx.x; i < V; i += THREADS) {
        const size_t o = (size_t)(i / src.seg) * src.seg_stride + (size_t)r * src.seg + i % src.seg;
        f(src.ids[o], src.vals[o]);
      }
    } else if (vec) {
      const float4* r4 = reinterpret_cast<const float4*>(row);
      for (int i = threadIdx.x; i < (V >> 2); i += THREADS) {
        const float4 x = r4[i];
        f(src.id_off + 4 * i + 0, x.x);
        f(src.id_off + 4 * i + 1, x.y);
        f(src.id_off + 4 * i + 2, x.z);
        f(src.id_off + 4 * i + 3, x.w);
      }
    } else {
      for (int i = threadIdx.x; i < V; i += THREADS) f(src.id_off + i, row[i]);
    }
  };

  __shared__ int hist[NWAVES][256];
  __shared__ float cv[KMAX];
  __shared__ int ci[KMAX];
  __shared__ int s_bin, s_kr, s_cnt, s_ngt, s_ntie, s_nc;
  __shared__ unsigned s_tmk[THREADS];  // per-thread max keys (prefilter)
  __shared__ unsigned s_ck[CAP];       // prefiltered candidates: key, id
  __shared__ int s_ci[CAP];
  __shared__ float s_bestv[NWAVES];
  __shared__ int s_besti[NWAVES];

  if (!(T > 0.f)) {  // greedy
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for_each_key(row, V, vec, [&](int i, float x) {
      if (x > bv || (x == bv && i < bi)) { bv = x; bi = i; }
    });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { s_bestv[w] = bv; s_besti[w] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int i = 1; i < NWAVES; ++i)
        if (s_bestv[i] > bv || (s_bestv[i] == bv && s_besti[i] < bi)) { bv = s_bestv[i]; bi = s_besti[i]; }
      out[r] = bi == 0x7fffffff ? 0 : bi;
    }
    return;
  }

  int k = emit ? KMAX : topk[r];
  if (k <= 0 || k > KMAX) k = KMAX;
  if (k > V) k = V;

  // ---- 1. radix select of the k-th largest (value, -id) pair ----
  // One MSB-first 8-bit digit per pass over the keys that match the prefix so far
  // (per-wave LDS histograms; wave 0 finds the bin by a shuffle suffix-scan).  Phase
  // A selects on the value key; if the k-th value is tied with more keys than remain
  // to be taken, phase B selects among those ties on ~id (ascending ids win), so the
  // candidate set is exact and deterministic.  `each(f)` enumerates (id, key) pairs.
  auto radix_pass = [&](auto&& each, auto&& digit_of) {  // -> s_bin / s_kr / s_cnt
    for (int i = lane; i < 256; i += 64) hist[w][i] = 0;
    __syncthreads();
    each([&](int i, unsigned key) {
      unsigned d;
      if (digit_of(i, key, &d)) atomicAdd(&hist[w][d], 1);
    });
    __syncthreads();
    if (w == 0) {
      int c[4];
      int s = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int t = 0;
#pragma unroll
        for (int ww = 0; ww < NWAVES; ++ww) t += hist[ww][4 * lane + j];
        c[j] = t;
        s += t;
      }
      int suf = s;  // keys in bins >= 4*lane
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_down(suf, o, 64);
        if (lane + o < 64) suf += t;
      }
      int above = suf - s;  // keys in bins > 4*lane+3
      const int kr0 = s_kr;
      if (above < kr0 && suf >= kr0) {  // the kr-th largest lies in this lane's 4 bins
#pragma unroll
        for (int j = 3; j >= 0; --j) {
          if (above + c[j] >= kr0) {
            s_bin = 4 * lane + j;
            s_cnt = c[j];
            s_kr = kr0 - above;
            break;
          }
          above += c[j];
        }
      }
    }
    __syncthreads();
  };
  // k-th largest (value key, ~id) among `each`'s pairs: returns (value key, ties taken,
  // id threshold: ties with ~id >= thr are in)
  auto select = [&](auto&& each, int kk, unsigned* vkey, int* kr_out, unsigned* idthr) {
    if (tid == 0) s_kr = kk;
    unsigned prefix = 0u, mask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
      radix_pass(each, [&](int, unsigned u, unsigned* d) {
        *d = (u >> shift) & 255u;
        return (u & mask) == prefix;
      });
      prefix |= (unsigned)s_bin << shift;
      mask |= 255u << shift;
    }
    const int kr = s_kr;
    unsigned thr = 0u;
    if (s_cnt > kr) {
      unsigned ip = 0u, im = 0u;
      for (int shift = 24; shift >= 0; shift -= 8) {
        radix_pass(each, [&](int i, unsigned u, unsigned* d) {
          const unsigned ni = ~(unsigned)i;
          *d = (ni >> shift) & 255u;
          return u == prefix && (ni & im) == ip;
        });
        ip |= (unsigned)s_bin << shift;
        im |= 255u << shift;
      }
      thr = ip;
    }
    *vkey = prefix;
    *kr_out = kr;
    *idthr = thr;
  };
  auto each_row = [&](auto&& f) {
    for_each_key(row, V, vec, [&](int i, float x) { f(i, ord_key(x)); });
  };

  // Prefilter: the k-th largest of the 1024 per-thread maxima is a key with at least
  // k row entries at or above it, so only those entries (typically a few hundred)
  // can be in the top k.  They are gathered to LDS and selected there; a row with
  // more than CAP such entries (massive ties) is selected over the whole row instead.
  float tmax = -INFINITY;
  for_each_key(row, V, vec, [&](int, float x) { tmax = fmaxf(tmax, x); });
  s_tmk[tid] = ord_key(tmax);
  unsigned t0key;
  {
    int kr_;
    unsigned thr_;
    select([&](auto&& f) { f(tid, s_tmk[tid]); }, min(k, THREADS), &t0key, &kr_, &thr_);
  }
  if (tid == 0) s_nc = 0;
  __syncthreads();
  each_row([&](int i, unsigned u) {
    if (u >= t0key) {
      const int sidx = atomicAdd(&s_nc, 1);
      if (sidx < CAP) { s_ck[sidx] = u; s_ci[sidx] = i; }
    }
  });
  __syncthreads();
  const int nc = s_nc;
  const bool small = nc <= CAP;
  auto each_cand = [&](auto&& f) {
    for (int j = tid; j < nc; j += THREADS) f(s_ci[j], s_ck[j]);
  };
  unsigned prefix, idthr;
  int kr;
  if (small)
    select(each_cand, k, &prefix, &kr, &idthr);
  else
    select(each_row, k, &prefix, &kr, &idthr);
  const int n_gt = k - kr;

  // ---- 2. collect the k candidates ----
  if (tid == 0) {
    s_ngt = 0;
    s_ntie = 0;
  }
  __syncthreads();
  auto take = [&](int i, unsigned u) {
    if (u > prefix) {
      const int sidx = atomicAdd(&s_ngt, 1);
      if (sidx < KMAX) { cv[sidx] = key_float(u); ci[sidx] = i; }
    } else if (u == prefix && ~(unsigned)i >= idthr) {
      const int sidx = atomicAdd(&s_ntie, 1);
      if (sidx < kr) { cv[n_gt + sidx] = key_float(u); ci[n_gt + sidx] = i; }
    }
  };
  if (small)
    each_cand(take);
  else
    each_row(take);
  __syncthreads();

  // ---- 3. bitonic sort (descending value, ascending id), KMAX slots padded ----
  if (tid < KMAX && tid >= k) {
    cv[tid] = -INFINITY;
    ci[tid] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= KMAX; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (tid < KMAX) {
        const int j = tid ^ stride;
        if (j > tid) {
          const bool desc = (tid & size) == 0;  // descending overall
          const float a = cv[tid], b = cv[j];
          const int ia = ci[tid], ib = ci[j];
          // "a before b" in the final (descending value, ascending id) order
          const bool a_first = a > b || (a == b && ia < ib);
          if (desc != a_first) {
            cv[tid] = b; cv[j] = a;
            ci[tid] = ib; ci[j] = ia;
          }
        }
      }
      __syncthreads();
    }
  }

  if (emit) {
    if (tid < KMAX) {
      cand_v[(size_t)r * KMAX + tid] = cv[tid];
      cand_id[(size_t)r * KMAX + tid] = ci[tid];
    }
    return;
  }

  // ---- 4 + 5. softmax / top-p / exponential race, wave 0 (2 slots per lane) ----
  if (w == 0) {
    const float vmax = cv[0];
    const float invT = 1.f / T;
    float p[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * lane + j;
      p[j] = i < k ? __expf((cv[i] - vmax) * invT) : 0.f;
    }
    const float tot = wave_sum(p[0] + p[1]);
    p[0] /= tot;
    p[1] /= tot;
    // inclusive prefix sum over slots 0..127 (lane-major: slot 2*lane + j)
    float ls = p[0] + p[1];
    float inc = ls;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    const float base = inc - ls;  // mass of slots before 2*lane
    const float cum0 = base + p[0], cum1 = cum0 + p[1];
    const float top_p = topp[r];
    const bool keep0 = 2 * lane < k && (cum0 - p[0]) <= top_p;
    const bool keep1 = 2 * lane + 1 < k && (cum1 - p[1]) <= top_p;
    const unsigned long long seed = seeds[r];
    const int ps = pos[r];
    float best = -1.f;
    int bid = 0x7fffffff;
    if (keep0) {
      best = p[0] / -__logf(uniform01(seed, ps, ci[2 * lane]));
      bid = ci[2 * lane];
    }
    if (keep1) {
      const float sc = p[1] / -__logf(uniform01(seed, ps, ci[2 * lane + 1]));
      if (sc > best) { best = sc; bid = ci[2 * lane + 1]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bid, o, 64);
      if (ob > best || (ob == best && oi < bid)) { best = ob; bid = oi; }
    }
    if (lane == 0) out[r] = bid == 0x7fffffff ? ci[0] : bid;
  }
}

}  // namespace

// ids[r] <- a draw from row r of logits [B, V] (row stride ld) with per-row
// temperature (<= 0: greedy), top_k (<= 0 or > 128: 128), top_p, and a random
// stream keyed by (seeds[r], pos[r], token id).
P2P_API int p2p_sample(const float* logits, int ld, int B, int V, const float* temp,
                       const int* topk, const float* topp, const unsigned long long* seeds,
                       const int* pos, int* ids, hipStream_t st) {
  if (B <= 0 || V <= 0 || ld < V) return (int)hipErrorInvalidValue;
  Src src{logits, nullptr, ld, 0, 0, 0};
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(THREADS), 0, st, src, V, temp, topk, topp,
                     seeds, pos, ids, (float*)nullptr, (int*)nullptr);
  return (int)hipGetLastError();
}

// Vocab-parallel sampling, step 1 (every TP rank, its logits shard [B, V] at columns
// id_off ..): the shard's top-128 (value, global id) pairs per row, sorted, into
// cand_v / cand_id [B][128].  The global top-k (k <= 128, the sampler's cap) of a row is
// contained in the union of the shards' sets, ties included (lowest ids first).
P2P_API int p2p_topk_candidates(const float* logits, int ld, int B, int V, int id_off,
                                float* cand_v, int* cand_id, hipStream_t st) {
  if (B <= 0 || V <= 0 || ld < V || !cand_v || !cand_id) return (int)hipErrorInvalidValue;
  Src src{logits, nullptr, ld, 0, 0, id_off};
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(THREADS), 0, st, src, V, (const float*)nullptr,
                     (const int*)nullptr, (const float*)nullptr,
                     (const unsigned long long*)nullptr, (const int*)nullptr, (int*)nullptr,
                     cand_v, cand_id);
  return (int)hipGetLastError();
}

// Step 2 (after the all-gather of every rank's candidates, rank-major [W][B][128]):
// the same draw as p2p_sample over the full vocabulary row -- identical token for
// the same (seed, position), since only ids in the union can be drawn.
P2P_API int p2p_sample_candidates(const float* cand_v, const int* cand_id, int W, int B,
                                  const float* temp, const int* topk, const float* topp,
                                  const unsigned long long* seeds, const int* pos, int* ids,
                                  hipStream_t st) {
  if (B <= 0 || W <= 0) return (int)hipErrorInvalidValue;
  Src src{cand_v, cand_id, 0, KMAX, (long long)B * KMAX, 0};
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(THREADS), 0, st, src, W * KMAX, temp, topk,
                     topp, seeds, pos, ids, (float*)nullptr, (int*)nullptr);
  return (int)hipGetLastError();
}
