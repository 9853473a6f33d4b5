// Decode step: qkv projection + RoPE + KV-cache write + attention in ONE launch
// (batch rows M <= 16, contexts <= 256 keys: the chat decode regime).
//
// Unfused, a decode layer runs the qkv GEMV (weight stream, ~11 us at 8B) and then the
// paged-attention kernel, whose ~7 us are a launch plus a serial load chain (block table
// -> page -> K/V) and a short computation.  Here the same grid holds two kinds of
// workgroup:
//   * consumers (the first M x Hkv blocks, dispatched first): one per (row, kv head).
//     At kernel start they load the block table and the K/V rows of every CACHED key of
//     their context -- that latency now hides behind the weight stream -- then wait for
//     the current token's q (G heads), k and v, compute the attention and write it.
//   * producers (one per 16-column group of the permuted qkv weight, as the skinny
//     kernel's EPI_QKV_ROPE): stream the weights, apply RMSNorm (rstd from the A
//     fragments) and RoPE, write k/v of the current token to the cache for later steps,
//     and publish the rotated q/k and v to the consumers as 8-byte tagged granules
//     {tag << 32 | two bf16} (cdna_hip_programming.md publish/consume recipe R2: the
//     data is the flag, no fence, one relaxed agent-scope 64-bit store per granule).
// The tag of (row, kv head) is counters[row * Hkv + h] + 1: producers read it before they
// publish, the consumer advances it after it has every granule, so a granule left by an
// earlier call or layer never carries the current tag.  Consumers only wait on producers,
// producers never wait, and consumer blocks are few (M x Hkv <= 128): the grid always
// drains.  Spins are bounded; a timeout sets the fault word (LlamaModel.check_faults).
//
// K-split producers (launch code bits 8..15 = ks > 1, round 5): a producer unit is one
// k-slice of one column group -- groups x ks units, so the weight stream is spread evenly
// over the CUs where whole groups are not (the 8B qkv: 384 groups = 1.5 per CU, 768 halves
// = 3; the 70B TP=8 shard: 80 groups on 256 CUs, 160 halves; qa_ksplit picks).  Units publish fp32 partial
// sums as {tag, fp32} granules; the consumer of (row, kv head) sums the slices in slice
// order (deterministic), applies the row's rstd (it sums the squares of the row itself,
// behind the weight stream), RoPE, writes this token's k / v to the cache and goes on with
// the attention.
#include "common.h"

#include <cstdlib>

namespace {

constexpr int PAGE = 64;
constexpr int HD = 128;
constexpr int QA_U = 4;       // producer: k-steps per pipeline batch
constexpr int VT = 64 + 8;    // V^T row stride in LDS (keys, bf16): one row per head dim
constexpr long long QA_SPIN_TICKS = 500000000ll;  // default spin bound: 5 s at the 100 MHz wall clock

typedef unsigned long long u64;

struct QAArgs {
  const bf16x8* Wt;
  const bf16* X;
  int ldx, M, K;
  float eps;
  const int* pos;
  const int* slots;
  const float2* cs;  // [max_pos][64] (cos, sin)
  bf16* kc;
  bf16* vc;
  int Hq, Hkv;
  const int* bt;
  int bt_stride;
  const int* ctx_lens;
  float scale;
  bf16* out;
  int ldo;
  u64* gran;          // [M][Hkv][G + 2][64] granules
  unsigned* counters; // [M][Hkv]
  int* err;
  int n_cons;         // consumer blocks = M * Hkv
  int probe;          // bench probe: 2 = consumers stop after the granule sweep, 4 = they
                      // wait for their K / V page loads before it
  long long spin_ticks;  // hand-off spin bound (P2P_QA_TIMEOUT_MS; 5 s default)
  // o_proj role (p2p_qkv_attn_oproj; null Wo = the attention output goes to `out`)
  const bf16x8* Wo;   // o_proj weight, fragment-major [No / 16][Ko / 32][64][8]
  bf16* h;            // residual [M][ldh]: h += attention @ Wo^T
  int ldh, No, Ko;    // Ko = Hq * 128
  u64* gran2;         // [M][Ko / 2] attention-output granules {epoch, two bf16}
  unsigned* epoch;    // [2]: launch epoch, o_proj arrival ticket
  int n_prod;         // producer blocks (groups x ks)
  int n_o;            // o_proj blocks = No / 16
  int ks;             // k-slices per column group (1: whole-group producers)
};

__device__ __forceinline__ unsigned bits16(float x) {
  const bf16 b = f2bf(x);
  unsigned short u;
  __builtin_memcpy(&u, &b, 2);
  return u;
}

__device__ __forceinline__ bf16x2 as_bf16x2(unsigned u) {
  bf16x2 r;
  __builtin_memcpy(&r, &u, 4);
  return r;
}

// ---------------------------------------------------------------- producer
template <int G, int W>
__device__ __forceinline__ void producer(const QAArgs& a, int g, char* smem) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int S = a.K >> 5;
  const int s0 = (S * w) / W, s1 = (S * (w + 1)) / W;
  const bf16x8* wp = a.Wt + (size_t)g * S * 64 + lane;
  const bool xv = r < a.M;
  const bf16* xp = a.X + (size_t)(xv ? r : 0) * a.ldx + 8 * q;
  const int head = g >> 3, kk = g & 7;
  const int d = (r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8);
  // epilogue rows m = 4q + j: their positions / slots / (cos, sin) now, behind the stream
  float2 rc[4];
  int rslot[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = 4 * q + j;
    const bool ok = m < a.M && w == 0;
    rslot[j] = ok ? a.slots[m] : -1;
    rc[j] = ok ? a.cs[(size_t)a.pos[m] * 64 + (d & 63)] : float2{1.f, 0.f};
  }

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  auto load = [&](int s, bf16x8(&bw)[QA_U], bf16x8(&ax)[QA_U]) {
#pragma unroll
    for (int u = 0; u < QA_U; ++u) {
      bw[u] = __builtin_nontemporal_load(wp + (size_t)(s + u) * 64);
      ax[u] = xv ? *reinterpret_cast<const bf16x8*>(xp + (s + u) * 32) : zero_bf16x8();
    }
  };
  auto compute = [&](const bf16x8(&bw)[QA_U], const bf16x8(&ax)[QA_U]) {
#pragma unroll
    for (int u = 0; u < QA_U; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[u], bw[u], acc, 0, 0, 0);
      ss = sumsq8(ax[u], ss);
    }
  };
  const int n = s1 - s0, nb = n / QA_U;
  if (nb > 0) {
    bf16x8 bA[QA_U], bB[QA_U], aA[QA_U], aB[QA_U];
    load(s0, bA, aA);
    int b = 0;
    for (; b + 2 < nb; b += 2) {
      load(s0 + (b + 1) * QA_U, bB, aB);
      compute(bA, aA);
      load(s0 + (b + 2) * QA_U, bA, aA);
      compute(bB, aB);
    }
    if (b + 1 < nb) {
      load(s0 + (b + 1) * QA_U, bB, aB);
      compute(bA, aA);
      compute(bB, aB);
    } else {
      compute(bA, aA);
    }
  }
  for (int s = s0 + nb * QA_U; s < s1; ++s) {
    const bf16x8 b1 = __builtin_nontemporal_load(wp + (size_t)s * 64);
    const bf16x8 a1 = xv ? *reinterpret_cast<const bf16x8*>(xp + s * 32) : zero_bf16x8();
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss = fmaf((float)a1[j], (float)a1[j], ss);
  }
  // split-K over the block's waves
  ss += __shfl_xor(ss, 16, 64);
  ss += __shfl_xor(ss, 32, 64);
  float* red = reinterpret_cast<float*>(smem);  // [W - 1][4][64]
  float* red_ss = red + (W - 1) * 4 * 64;       // [W][16]
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[((w - 1) * 4 + j) * 64 + lane] = acc[j];
  }
  if (q == 0) red_ss[w * 16 + r] = ss;
  __syncthreads();
  if (w != 0) return;  // (every wave returns together to the o_proj phase, if any)
#pragma unroll
  for (int ww = 0; ww < W - 1; ++ww)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += red[(ww * 4 + j) * 64 + lane];
  const int Hq = a.Hq, Hkv = a.Hkv;
  int kvh, sl;
  if (head < Hq) {
    kvh = head / G;
    sl = head % G;
  } else if (head < Hq + Hkv) {
    kvh = head - Hq;
    sl = G;
  } else {
    kvh = head - Hq - Hkv;
    sl = G + 1;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = 4 * q + j;
    float t = 0.f;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) t += red_ss[ww * 16 + (m & 15)];
    const float v = acc[j] * rsqrtf(t / (float)a.K + a.eps);
    const float vp = __shfl_xor(v, 8, 64);
    float y = v;
    if (head < Hq + Hkv) y = (r < 8) ? (v * rc[j].x - vp * rc[j].y) : (v * rc[j].x + vp * rc[j].y);
    const float y1 = __shfl_xor(y, 1, 64);
    if (m < a.M) {
      const int slot = rslot[j];
      if (head >= Hq && slot >= 0) {  // k / v of the current token -> cache (later steps)
        bf16* cache = head < Hq + Hkv ? a.kc : a.vc;
        cache[(((size_t)(slot / PAGE) * Hkv + kvh) * PAGE + slot % PAGE) * HD + d] = f2bf(y);
      }
      if ((r & 1) == 0) {  // lanes r, r + 1 hold dims d, d + 1: one granule
        const unsigned tag = a.counters[m * Hkv + kvh] + 1;
        const u64 gr = ((u64)tag << 32) | ((u64)bits16(y1) << 16) | bits16(y);
        __hip_atomic_store(a.gran + (((size_t)m * Hkv + kvh) * (G + 2) + sl) * 64 + (d >> 1), gr,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// K-split producer: unit pg = k-slice (pg / groups) of column group (pg % groups); the
// block's waves split the slice's k-steps; the summed partial (no rstd, no RoPE: the
// consumer finishes those) goes out as {tag, fp32} granules [M][Hkv][G + 2][ks][128].
template <int G, int W>
__device__ __forceinline__ void producer_split(const QAArgs& a, int pg, char* smem) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int groups = a.n_prod / a.ks;
  const int g = pg % groups, sk = pg / groups;
  const int S = a.K >> 5;
  const int u0 = (S * sk) / a.ks, u1 = (S * (sk + 1)) / a.ks;
  const int s0 = u0 + ((u1 - u0) * w) / W, s1 = u0 + ((u1 - u0) * (w + 1)) / W;
  const bf16x8* wp = a.Wt + (size_t)g * S * 64 + lane;
  const bool xv = r < a.M;
  const bf16* xp = a.X + (size_t)(xv ? r : 0) * a.ldx + 8 * q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  auto load = [&](int s, bf16x8(&bw)[QA_U], bf16x8(&ax)[QA_U]) {
#pragma unroll
    for (int u = 0; u < QA_U; ++u) {
      bw[u] = __builtin_nontemporal_load(wp + (size_t)(s + u) * 64);
      ax[u] = xv ? *reinterpret_cast<const bf16x8*>(xp + (s + u) * 32) : zero_bf16x8();
    }
  };
  auto compute = [&](const bf16x8(&bw)[QA_U], const bf16x8(&ax)[QA_U]) {
#pragma unroll
    for (int u = 0; u < QA_U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[u], bw[u], acc, 0, 0, 0);
  };
  const int n = s1 - s0, nb = n / QA_U;
  if (nb > 0) {
    bf16x8 bA[QA_U], bB[QA_U], aA[QA_U], aB[QA_U];
    load(s0, bA, aA);
    int b = 0;
    for (; b + 2 < nb; b += 2) {
      load(s0 + (b + 1) * QA_U, bB, aB);
      compute(bA, aA);
      load(s0 + (b + 2) * QA_U, bA, aA);
      compute(bB, aB);
    }
    if (b + 1 < nb) {
      load(s0 + (b + 1) * QA_U, bB, aB);
      compute(bA, aA);
      compute(bB, aB);
    } else {
      compute(bA, aA);
    }
  }
  for (int s = s0 + nb * QA_U; s < s1; ++s) {
    const bf16x8 b1 = __builtin_nontemporal_load(wp + (size_t)s * 64);
    const bf16x8 a1 = xv ? *reinterpret_cast<const bf16x8*>(xp + s * 32) : zero_bf16x8();
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
  }
  float* red = reinterpret_cast<float*>(smem);  // [W - 1][4][64]
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[((w - 1) * 4 + j) * 64 + lane] = acc[j];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int ww = 0; ww < W - 1; ++ww)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += red[(ww * 4 + j) * 64 + lane];
  const int head = g >> 3, kk = g & 7;
  const int d = (r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8);
  const int Hq = a.Hq, Hkv = a.Hkv;
  int kvh, sl;
  if (head < Hq) {
    kvh = head / G;
    sl = head % G;
  } else if (head < Hq + Hkv) {
    kvh = head - Hq;
    sl = G;
  } else {
    kvh = head - Hq - Hkv;
    sl = G + 1;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = 4 * q + j;
    if (m < a.M) {
      const unsigned tag = a.counters[m * Hkv + kvh] + 1;
      const u64 gr = ((u64)tag << 32) | (u64)__float_as_uint(acc[j]);
      __hip_atomic_store(a.gran + ((((size_t)m * Hkv + kvh) * (G + 2) + sl) * a.ks + sk) * HD + d, gr,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- consumer
// Wave w owns the 64 keys of page w of the row (contexts <= 256 keys).  The math is the
// MFMA form of decode attention (v_mfma_f32_16x16x32_bf16, query heads on the N axis,
// G <= 16 padded with zero rows):
//   S^T[key][head] = K . Q^T   (A = 16 keys x 32 dims, prefetched from the page into
//                               registers at kernel start; B = q fragments)
//   O[head][dim]  += P . V     (A = P: the S^T accumulators after the softmax; B = V^T
//                               fragments from the wave's V rows in LDS)
// so the per-wave work after the hand-off is 32 MFMAs and a 4-way LDS merge (a scalar
// P.V loop over 64 keys per wave took ~7 us here).  This step's token (key ctx - 1) is
// not in the prefetched rows: its k row is patched into the K fragments and its v row
// into the LDS V rows from the granules.
constexpr int MKPW = 64;  // keys per wave = one page
// key waves KW: one page of 64 keys each -- 4 (256 keys) by default, 2 (128 keys) when the
// caller bounds the contexts (launch-code bits 16..23): half the consumer's LDS, so the
// grid's workgroups (all sized for a consumer) fit the CUs 3-4 at a time instead of 2
// (waves >= KW only join the barriers)
template <int G, int W, int KW = 4>
__device__ __forceinline__ void consumer(const QAArgs& a, int b, char* smem) {
  static_assert(G >= 1 && G <= 16, "query heads on the MFMA N axis");
  static_assert(W >= KW, "one page per key wave");
  const int Hkv = a.Hkv;
  const int r = b / Hkv, h = b % Hkv;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kk = lane & 15, qd = lane >> 4;
  const int ctx = a.ctx_lens[r];
  const int nprev = ctx - 1;  // keys already in the cache; key nprev is this step's token
  // V is kept TRANSPOSED per wave (vt[w][dim][key]): the P.V B operand of lane (kk, qd) is
  // then 4 + 4 consecutive keys of one dim -- two 8-byte LDS reads per column block after
  // the hand-off, where [key][dim] rows took eight 2-byte reads.  The transpose (scalar
  // writes) happens at kernel start, behind the producers' weight stream.
  auto& vt = *reinterpret_cast<bf16(*)[KW][HD][VT]>(smem);
  auto& so = *reinterpret_cast<float(*)[KW][G][HD]>(smem);  // after P.V (aliases vt)
  char* p = smem + (sizeof(bf16) * KW * HD * VT > sizeof(float) * KW * G * HD
                        ? sizeof(bf16) * KW * HD * VT
                        : sizeof(float) * KW * G * HD);
  auto& cur = *reinterpret_cast<unsigned(*)[G + 2][64]>(p);  // q heads, k, v: bf16 pairs
  p += sizeof(unsigned) * (G + 2) * 64;
  auto& sm = *reinterpret_cast<float(*)[KW][G]>(p);
  p += sizeof(float) * KW * G;
  auto& sl = *reinterpret_cast<float(*)[KW][G]>(p);

  // 1. this wave's page: K fragments to registers, V rows to LDS (all loads in flight)
  const int n_valid = w < KW ? min(max(ctx - w * MKPW, 0), MKPW) : 0;  // wave-uniform
  bf16x8 kr[4][4];
  // a page holding only this step's token is still loaded whole: its other rows (stale or
  // zero, always finite) keep the masked P.V lanes finite (0 x NaN would poison O)
  if (n_valid > 0) {
    const int page = a.bt[(size_t)r * a.bt_stride + w];
    const size_t pbase = ((size_t)page * Hkv + h) * PAGE * HD;
    bf16x8 vr[4][4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const bf16x8* kp = reinterpret_cast<const bf16x8*>(a.kc + pbase + (size_t)(16 * bb + kk) * HD + 8 * qd);
      const bf16x8* vp = reinterpret_cast<const bf16x8*>(a.vc + pbase + (size_t)(16 * bb + kk) * HD + 8 * qd);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) kr[bb][s2] = kp[4 * s2];
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) vr[bb][s2] = vp[4 * s2];
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) vt[w][32 * s2 + 8 * qd + j][16 * bb + kk] = vr[bb][s2][j];
  } else {
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) kr[bb][s2] = zero_bf16x8();
  }
  if (a.probe & 4) __builtin_amdgcn_s_waitcnt(0);  // probe: this wave's pages landed first
  // 2. the current token's q (G heads), k and v from the producers' granules
  const unsigned tag = a.counters[r * Hkv + h] + 1;
  const unsigned o_epoch =
      a.gran2 ? __hip_atomic_load(&a.epoch[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 : 0;
  const int failed = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long t0 = wall_clock64();
  if (a.ks > 1) {
    // k-split producers: this row's rstd first (its squares, behind the weight stream) ...
    const bf16* xr = a.X + (size_t)r * a.ldx;
    float ss = 0.f;
    for (int i = tid; i < (a.K >> 3); i += W * 64)
      ss = sumsq8(*reinterpret_cast<const bf16x8*>(xr + 8 * i), ss);
    ss = wave_sum(ss);
    float* rs = &sm[0][0];  // (free until the softmax merge)
    if (lane == 0) rs[w] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) tot += rs[ww];
    const float rstd = rsqrtf(tot / (float)a.K + a.eps);
    // ... then per dim pair (d, d + 64) of a head: the slices' partials summed in slice
    // order, rstd, RoPE (q heads and k), this token's k / v to the cache
    const u64* gb = a.gran + ((size_t)r * Hkv + h) * (G + 2) * a.ks * HD;
    const int slot = a.slots[r];
    const float2* csr = a.cs + (size_t)a.pos[r] * 64;
    bf16* cb = reinterpret_cast<bf16*>(&cur[0][0]);
    constexpr int KSM = 8;
    for (int i = tid; i < (G + 2) * 64; i += W * 64) {
      const int sl = i >> 6, d = i & 63;
      const u64* base = gb + (size_t)sl * a.ks * HD;
      u64 lo[KSM], hi[KSM];
#pragma unroll
      for (int k = 0; k < KSM; ++k)
        if (k < a.ks) {
          lo[k] = __hip_atomic_load(base + k * HD + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          hi[k] = __hip_atomic_load(base + k * HD + d + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      for (;;) {
        bool stale = false;
#pragma unroll
        for (int k = 0; k < KSM; ++k)
          if (k < a.ks) stale |= (unsigned)(lo[k] >> 32) != tag || (unsigned)(hi[k] >> 32) != tag;
        if (!stale || failed) break;
        if (wall_clock64() - t0 > a.spin_ticks) {
          atomicOr(a.err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (int k = 0; k < KSM; ++k)
          if (k < a.ks) {
            if ((unsigned)(lo[k] >> 32) != tag)
              lo[k] = __hip_atomic_load(base + k * HD + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(hi[k] >> 32) != tag)
              hi[k] = __hip_atomic_load(base + k * HD + d + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
      }
      float vlo = 0.f, vhi = 0.f;
#pragma unroll
      for (int k = 0; k < KSM; ++k)
        if (k < a.ks) {
          vlo += __uint_as_float((unsigned)lo[k]);
          vhi += __uint_as_float((unsigned)hi[k]);
        }
      vlo *= rstd;
      vhi *= rstd;
      float ylo = vlo, yhi = vhi;
      if (sl <= G) {  // q heads and k: rotate the pair (d, d + 64)
        const float2 c = csr[d];
        ylo = vlo * c.x - vhi * c.y;
        yhi = vhi * c.x + vlo * c.y;
      }
      cb[sl * HD + d] = f2bf(ylo);
      cb[sl * HD + d + 64] = f2bf(yhi);
      if (sl >= G && slot >= 0) {  // k / v of the current token -> cache (later steps)
        bf16* cache = sl == G ? a.kc : a.vc;
        bf16* dst = cache + (((size_t)(slot / PAGE) * Hkv + h) * PAGE + slot % PAGE) * HD;
        dst[d] = f2bf(ylo);
        dst[d + 64] = f2bf(yhi);
      }
    }
  } else {
    const u64* gb = a.gran + ((size_t)r * Hkv + h) * (G + 2) * 64;
    for (int i = tid; i < (G + 2) * 64; i += W * 64) {
      u64 x = __hip_atomic_load(gb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((unsigned)(x >> 32) != tag && !failed) {
        if (wall_clock64() - t0 > a.spin_ticks) {
          atomicOr(a.err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        x = __hip_atomic_load(gb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      cur[i >> 6][i & 63] = (unsigned)x;
    }
  }
  __syncthreads();
  if (a.probe & 2) {  // probe: hand-off only (no attention math)
    if (tid == 0) a.counters[r * Hkv + h] = tag;
    return;
  }
  auto frag = [&](int row, int s2) {  // 8 dims (32 s2 + 8 qd ..) of a granule row, as bf16x8
    bf16x8 f;
    const unsigned* src = &cur[row][16 * s2 + 4 * qd];
    __builtin_memcpy(&f, src, 16);
    return f;
  };
  // this step's token: k row into the K fragments, v row into the LDS V rows
  if (w < KW && nprev >= w * MKPW && nprev < (w + 1) * MKPW) {
    const int rn = nprev - w * MKPW;
    if (kk == (rn & 15)) {
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
        if (bb == (rn >> 4)) {
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) kr[bb][s2] = frag(G, s2);
        }
    }
    const bf16x2 v2 = as_bf16x2(cur[G + 1][lane]);
    vt[w][2 * lane][rn] = v2[0];
    vt[w][2 * lane + 1][rn] = v2[1];
  }
  bf16x8 qf[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) qf[s2] = kk < G ? frag(min(kk, G - 1), s2) : zero_bf16x8();

  float mg = -INFINITY, lg = 0.f;  // per head kk (every lane of column kk agrees)
  f32x4 o[HD / 16];
#pragma unroll
  for (int c = 0; c < HD / 16; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (n_valid > 0) {
    // S^T blocks: lane holds keys 16 bb + 4 qd + j (j < 4) of head kk
    f32x4 st[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      st[bb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        st[bb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr[bb][s2], qf[s2], st[bb], 0, 0, 0);
    }
    float m = -INFINITY;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = 16 * bb + 4 * qd + j < n_valid;
        st[bb][j] = ok ? st[bb][j] * a.scale : -INFINITY;
        m = fmaxf(m, st[bb][j]);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float pr = __expf(st[bb][j] - m);  // -inf -> 0
        st[bb][j] = pr;
        l += pr;
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
        const bf16x4 v0 = *reinterpret_cast<const bf16x4*>(&vt[w][16 * c + kk][32 * t + 4 * qd]);
        const bf16x4 v1 = *reinterpret_cast<const bf16x4*>(&vt[w][16 * c + kk][32 * t + 16 + 4 * qd]);
        bf16x8 vb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vb[j] = v0[j];
          vb[4 + j] = v1[j];
        }
        o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[c], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // every wave's P.V has read its V rows: the region becomes `so`
  // O accumulators: lane holds O[head 4 qd + j][dim 16 c + kk]
  if (w < KW) {
#pragma unroll
    for (int c = 0; c < HD / 16; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int hd = 4 * qd + j;
        if (hd < G) so[w][hd][16 * c + kk] = o[c][j];
      }
  }
  if (w < KW && qd == 0 && kk < G) {
    sm[w][kk] = mg;
    sl[w][kk] = lg;
  }
  __syncthreads();
  auto merged = [&](int hd, int dd) {
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < KW; ++ww) M = fmaxf(M, sm[ww][hd]);
    float num = 0.f, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < KW; ++ww) {
        const float e = __expf(sm[ww][hd] - M);
        num = fmaf(e, so[ww][hd][dd], num);
        den = fmaf(e, sl[ww][hd], den);
      }
    }
    return den > 0.f ? num / den : 0.f;
  };
  if (a.gran2 != nullptr) {
    // o_proj role in this launch: publish the attention output as {epoch, two bf16}
    // granules (R2: the data is the flag) for the o_proj workgroups to sweep
    for (int i = tid; i < G * HD / 2; i += W * 64) {
      const int hd = i / (HD / 2), dd = 2 * (i % (HD / 2));
      const u64 gr = ((u64)o_epoch << 32) | ((u64)bits16(merged(hd, dd + 1)) << 16) |
                     bits16(merged(hd, dd));
      __hip_atomic_store(a.gran2 + (size_t)r * (a.Ko >> 1) + (((h * G + hd) * HD + dd) >> 1), gr,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {
    for (int i = tid; i < G * HD; i += W * 64) {
      const int hd = i / HD, dd = i % HD;
      a.out[(size_t)r * a.ldo + (size_t)(h * G + hd) * HD + dd] = f2bf(merged(hd, dd));
    }
  }
  if (tid == 0) a.counters[r * Hkv + h] = tag;  // every granule of this call was consumed
}

// ---------------------------------------------------------------- o_proj
// 16 output columns of o_proj per workgroup (p2p_qkv_attn_oproj): producer workgroup
// g < No / 16 continues with column group g once its qkv slice is published.  Its waves
// load their k-range of the o_proj weight into the registers the qkv stream just freed (nt
// loads: this stream runs while the attention does, when the weight stream would
// otherwise idle).  Then the whole workgroup sweeps the attention-output granules of
// up to OROWS batch rows into LDS -- every thread's loads issued at once, one round trip
// once the consumers have published -- and each wave runs its k-range of MFMAs from LDS,
// the waves' partial tiles are summed and added to the residual h: the unfused path's
// o_proj launch (skinny GEMM, EPI_RESID) without its launch, weight-stream ramp and
// boundary.  The launch epoch (epoch[0] + 1, read by every consumer and o_proj block at its
// start) tags the granules; the last o_proj block to finish advances it.
constexpr int OQ = 32;     // max k-steps per wave held in registers (Ko / 32 / W)
constexpr int OROWS = 8;   // batch rows staged in LDS per sweep pass
constexpr int OGPT = 8;    // granules in flight per thread per sweep round

template <int W>
__device__ __forceinline__ void oproj_load(const QAArgs& a, int g, bf16x8 (&wr)[OQ]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int S = a.Ko >> 5;
  const int s0 = (S * w) / W, n = (S * (w + 1)) / W - s0;
  const bf16x8* wp = a.Wo + ((size_t)g * S + s0) * 64 + lane;
#pragma unroll
  for (int i = 0; i < OQ; ++i)
    if (i < n) wr[i] = __builtin_nontemporal_load(wp + (size_t)i * 64);
}

template <int W>
__device__ __forceinline__ void oproj(const QAArgs& a, int g, char* smem, const bf16x8 (&wr)[OQ]) {
  constexpr int NT = W * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int S = a.Ko >> 5;
  const int s0 = (S * w) / W, n = (S * (w + 1)) / W - s0;
  const unsigned e = __hip_atomic_load(&a.epoch[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const int failed = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int r = lane & 15, q = lane >> 4;
  const int KG = a.Ko >> 1;        // granules per row
  const int LDR = a.Ko + 8;        // LDS row stride (bf16): 16 B pad, rows on distinct banks
  unsigned* st = reinterpret_cast<unsigned*>(smem);  // [OROWS][LDR / 2] bf16 pairs
  const long long t0 = wall_clock64();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int m0 = 0; m0 < a.M; m0 += OROWS) {
    const int mb = min(OROWS, a.M - m0);
    const int total = mb * KG;
    __syncthreads();  // the previous pass's LDS reads are done
    for (int base = 0; base < total; base += NT * OGPT) {
      u64 x[OGPT];
#pragma unroll
      for (int j = 0; j < OGPT; ++j) {  // independent loads: one round trip
        const int i = base + j * NT + (int)threadIdx.x;
        x[j] = i < total ? __hip_atomic_load(a.gran2 + (size_t)m0 * KG + i, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                         : ((u64)e << 32);
      }
      bool ok = true;
#pragma unroll
      for (int j = 0; j < OGPT; ++j) ok &= (unsigned)(x[j] >> 32) == e;
      while (!ok && !failed) {  // the consumers have not published yet: re-poll the missing
        if (wall_clock64() - t0 > a.spin_ticks) {
          atomicOr(a.err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        ok = true;
#pragma unroll
        for (int j = 0; j < OGPT; ++j) {
          const int i = base + j * NT + (int)threadIdx.x;
          if ((unsigned)(x[j] >> 32) != e && i < total)
            x[j] = __hip_atomic_load(a.gran2 + (size_t)m0 * KG + i, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(x[j] >> 32) == e;
        }
      }
#pragma unroll
      for (int j = 0; j < OGPT; ++j) {
        const int i = base + j * NT + (int)threadIdx.x;
        if (i < total) st[(i / KG) * (LDR >> 1) + i % KG] = (unsigned)x[j];
      }
    }
    __syncthreads();
    // this wave's k-range: A fragment of k-step s = row r, dims 32 s + 8 q .. + 7
    const bool rv = r >= m0 && r < m0 + mb;
    const bf16* arow = reinterpret_cast<const bf16*>(st) + (size_t)(rv ? r - m0 : 0) * LDR + 8 * q;
#pragma unroll
    for (int i = 0; i < OQ; ++i) {
      if (i < n) {
        const bf16x8 af = rv ? *reinterpret_cast<const bf16x8*>(arow + 32 * (s0 + i)) : zero_bf16x8();
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wr[i], acc, 0, 0, 0);
      }
    }
  }
  __syncthreads();  // the staging area becomes the reduction buffer
  float* red = reinterpret_cast<float*>(smem);  // [W - 1][4][64]
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[((w - 1) * 4 + j) * 64 + lane] = acc[j];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int ww = 0; ww < W - 1; ++ww)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += red[(ww * 4 + j) * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // acc[j]: row 4 q + j, column 16 g + r
      const int m = 4 * q + j;
      if (m < a.M) {
        bf16* hp = a.h + (size_t)m * a.ldh + 16 * g + r;
        *hp = f2bf((float)*hp + acc[j]);
      }
    }
    if (lane == 0 &&
        atomicAdd(&a.epoch[1], 1u) == (unsigned)a.n_o - 1) {  // every block swept: next epoch
      a.epoch[1] = 0;
      __hip_atomic_store(&a.epoch[0], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int G, int KW = 4>
constexpr size_t consumer_lds() {
  const size_t v = sizeof(bf16) * KW * HD * VT;
  const size_t o = sizeof(float) * KW * G * HD;
  return (v > o ? v : o) + sizeof(unsigned) * (G + 2) * 64 + 2 * sizeof(float) * KW * G;
}

// FO: the launch also holds the o_proj workgroups (blocks after the producers)
size_t consumer_lds_for(int G) {
  switch (G) {
    case 1: return consumer_lds<1>();
    case 2: return consumer_lds<2>();
    case 4: return consumer_lds<4>();
    case 8: return consumer_lds<8>();
  }
  return 0;
}

template <int G, int W, bool FO, int KW = 4>
__global__ __launch_bounds__(W * 64) void qkv_attn_kernel(QAArgs a) {
  constexpr size_t kProd = sizeof(float) * ((W - 1) * 4 * 64 + W * 16);
  constexpr size_t kCons = consumer_lds<G, KW>();
  __shared__ __attribute__((aligned(16))) char smem[kCons > kProd ? kCons : kProd];
  if ((int)blockIdx.x < a.n_cons) {
    consumer<G, W, KW>(a, blockIdx.x, smem);
  } else {
    const int pg = blockIdx.x - a.n_cons;
    if (!FO && a.ks > 1) {
      producer_split<G, W>(a, pg, smem);
      return;
    }
    producer<G, W>(a, pg, smem);
    // FO: the first n_o producers go on to an o_proj column group, their registers free
    // once the qkv stream is done (no extra workgroups competing for residency).  Loading
    // the o_proj slice before the qkv stream instead needs ~250 VGPRs + spills: one wave
    // per SIMD, and the grid no longer fits the device at once
    if constexpr (FO) {
      if (pg < a.n_o) {
        bf16x8 wr[OQ];
        oproj_load<W>(a, pg, wr);
        oproj<W>(a, pg, smem, wr);
      }
    }
  }
}

template <int W, bool FO, int KW = 4>
int launch_qa(const QAArgs& a, int G, int groups, hipStream_t stream) {
  const dim3 grid(a.n_cons + (FO ? groups : a.n_prod)), block(W * 64);
  switch (G) {
    case 1: hipLaunchKernelGGL((qkv_attn_kernel<1, W, FO, KW>), grid, block, 0, stream, a); break;
    case 2: hipLaunchKernelGGL((qkv_attn_kernel<2, W, FO, KW>), grid, block, 0, stream, a); break;
    case 4: hipLaunchKernelGGL((qkv_attn_kernel<4, W, FO, KW>), grid, block, 0, stream, a); break;
    case 8: hipLaunchKernelGGL((qkv_attn_kernel<8, W, FO, KW>), grid, block, 0, stream, a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

static int g_qa_probe = 0;

// Bench probes (bench/qkv_attn_bench.py): 1 = producers only, 2 = hand-off without the
// attention math, 4 (with 2) = the consumers wait for their K / V pages before the hand-off;
// 0 = the real kernel.
P2P_API void p2p_qkv_attn_probe(int mode) { g_qa_probe = mode; }

// Fused decode qkv + RoPE + KV write + attention (see the file header).  Wt: the qkv
// weight in fragment-major order with rope_row_perm rows (as p2p_skinny_gemm_qkv_rope),
// bf16 only; M <= 16 rows, row r uses block-table row r and attends to ctx_lens[r] <= 256
// keys (this step's token at position ctx - 1, its slot in slots[r]).  gran: u64
// [M][Hkv][Hq / Hkv + 2][64], counters: u32 [M][Hkv] (zeroed once, private to this call
// site's buffers), err: device int (fault word).
// workgroups of the fused-o_proj kernel the device holds at once (occupancy x CUs)
static int oproj_capacity(int W, int G) {
  static int cache[2][9] = {};
  int& c = cache[W == 8][G];
  if (c) return c;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const void* k = nullptr;
#define P2P_QA_K(WW, GG) (const void*)qkv_attn_kernel<GG, WW, true>
  switch (G) {
    case 1: k = W == 8 ? P2P_QA_K(8, 1) : P2P_QA_K(4, 1); break;
    case 2: k = W == 8 ? P2P_QA_K(8, 2) : P2P_QA_K(4, 2); break;
    case 4: k = W == 8 ? P2P_QA_K(8, 4) : P2P_QA_K(4, 4); break;
    case 8: k = W == 8 ? P2P_QA_K(8, 8) : P2P_QA_K(4, 8); break;
    default: return 0;
  }
#undef P2P_QA_K
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, W * 64, 0) != hipSuccess) return 0;
  c = per * cus;
  return c;
}

// The hand-off spin bound: P2P_QA_TIMEOUT_MS (default 5000).  Virtual ranks time-sharing
// one device (tests/test_world8_gpu.py) raise it like P2P_CAR_TIMEOUT_MS: a rank's
// producers can wait behind its peers' spinning grids there, which a real node never sees.
static long long qa_spin_ticks() {
  static const long long t = [] {
    const char* e = std::getenv("P2P_QA_TIMEOUT_MS");
    const long long ms = e && *e ? std::atoll(e) : 0;
    return ms > 0 ? ms * 100000ll : QA_SPIN_TICKS;  // 100 MHz wall clock
  }();
  return t;
}

// k-slices per column group.  Measured (bench/qkv_attn_bench.py, profiles/r5_qkv_attn_ksplit.jsonl):
// the 70B TP=8 shard (80 groups on 256 CUs) runs 10.1 us with 2 slices against 11.4 with
// whole groups (8 waves); the 8B qkv (384 groups) loses with any split (13.4 -> 15.7 us at 2:
// 768 units no longer fit the device at once next to the consumers' LDS).  So: 2 slices
// where whole groups leave more than half of the CUs without one; P2P_QA_KSPLIT overrides.
static int qa_ksplit(int groups, int K) {
  static const int env = [] {
    const char* e = std::getenv("P2P_QA_KSPLIT");
    return e && *e ? std::atoi(e) : 0;
  }();
  if (env >= 1 && env <= 8) return env;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 1;
  return (2 * groups <= cus && (K / 32) / 2 >= 16) ? 2 : 1;
}

static int qkv_attn_impl(const void* Wt, const void* X, int ldx, int M, int K, int Hq, int Hkv,
                         const int* pos, const int* slots, const void* cos_sin, void* k_cache,
                         void* v_cache, const int* block_tables, int bt_stride,
                         const int* ctx_lens, float scale, void* out, int ldo, float eps,
                         void* gran, unsigned* counters, int* err, int waves, const void* Wo,
                         int No, void* h, int ldh, void* gran2, unsigned* epoch,
                         hipStream_t stream) {
  if (M < 1 || M > 16 || K % 32 || Hkv <= 0 || Hq % Hkv || bt_stride * PAGE < 1)
    return (int)hipErrorInvalidValue;
  QAArgs a = {};
  a.Wt = (const bf16x8*)Wt;
  a.X = (const bf16*)X;
  a.ldx = ldx;
  a.M = M;
  a.K = K;
  a.eps = eps;
  a.pos = pos;
  a.slots = slots;
  a.cs = (const float2*)cos_sin;
  a.kc = (bf16*)k_cache;
  a.vc = (bf16*)v_cache;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.bt = block_tables;
  a.bt_stride = bt_stride;
  a.ctx_lens = ctx_lens;
  a.scale = scale;
  a.out = (bf16*)out;
  a.ldo = ldo;
  a.gran = (u64*)gran;
  a.counters = counters;
  a.err = err;
  a.n_cons = (g_qa_probe & 1) ? 0 : M * Hkv;  // probe 1: producers only
  a.probe = g_qa_probe;
  a.spin_ticks = qa_spin_ticks();
  const int groups = (Hq + 2 * Hkv) * (HD / 16);
  // producer waves per block (split-K): 8 when the projection has few column groups (the
  // 70B TP=8 shard: 80), as the skinny kernel's heuristic would pick; else 4.
  // Launch-code bits 8..15: k-slices per group (0 = qa_ksplit's pick; 1 = whole groups)
  int ks = (waves >> 8) & 0xff;
  int W = waves & 0xff;
  if (ks == 0) ks = qa_ksplit(groups, K);
  if (ks < 1 || ks > 8 || (K / 32) / ks < 4) return (int)hipErrorInvalidValue;
  if (W != 4 && W != 8) W = (groups * ks * 8 * 2 <= 4096 && (K / 32) / ks / 8 >= 8) ? 8 : 4;
  a.ks = Wo != nullptr ? 1 : ks;  // (the o_proj role keeps whole groups)
  a.n_prod = groups * a.ks;
  if (Wo != nullptr) {
    a.Wo = (const bf16x8*)Wo;
    a.h = (bf16*)h;
    a.ldh = ldh;
    a.No = No;
    a.Ko = Hq * HD;
    a.gran2 = (u64*)gran2;
    a.epoch = epoch;
    a.n_o = No / 16;
    // the o_proj weights live in registers: at most OQ k-steps per wave
    const size_t stage = (size_t)OROWS * (a.Ko + 8) * sizeof(bf16);
    const size_t lds = consumer_lds_for(Hq / Hkv);
    if (No % 16 || No <= 0 || !h || !gran2 || !epoch || (a.Ko / 32 + W - 1) / W > OQ ||
        stage > lds || a.n_o > groups || (g_qa_probe & 1))
      return (int)hipErrorInvalidValue;
    // producers that went on to o_proj wait for the consumers, which wait for EVERY
    // producer: the whole grid must be resident at once or it only ends at the spin bound
    if (a.n_cons + groups > oproj_capacity(W, Hq / Hkv)) return (int)hipErrorInvalidConfiguration;
    return W == 8 ? launch_qa<8, true>(a, Hq / Hkv, groups, stream)
                  : launch_qa<4, true>(a, Hq / Hkv, groups, stream);
  }
  if (((waves >> 16) & 0xff) == 2)  // the caller bounds every context to 128 keys
    return W == 8 ? launch_qa<8, false, 2>(a, Hq / Hkv, groups, stream)
                  : launch_qa<4, false, 2>(a, Hq / Hkv, groups, stream);
  return W == 8 ? launch_qa<8, false>(a, Hq / Hkv, groups, stream)
                : launch_qa<4, false>(a, Hq / Hkv, groups, stream);
}

P2P_API int p2p_qkv_attn(const void* Wt, const void* X, int ldx, int M, int K, int Hq, int Hkv,
                         const int* pos, const int* slots, const void* cos_sin, void* k_cache,
                         void* v_cache, const int* block_tables, int bt_stride,
                         const int* ctx_lens, float scale, void* out, int ldo, float eps,
                         void* gran, unsigned* counters, int* err, int waves, hipStream_t stream) {
  return qkv_attn_impl(Wt, X, ldx, M, K, Hq, Hkv, pos, slots, cos_sin, k_cache, v_cache,
                       block_tables, bt_stride, ctx_lens, scale, out, ldo, eps, gran, counters, err,
                       waves, nullptr, 0, nullptr, 0, nullptr, nullptr, stream);
}

// 1 if p2p_qkv_attn_oproj can run M rows of this shape (every workgroup resident at once).
P2P_API int p2p_qkv_attn_oproj_fits(int M, int K, int Hq, int Hkv, int waves) {
  if (M < 1 || M > 16 || Hkv <= 0 || Hq % Hkv) return 0;
  const int groups = (Hq + 2 * Hkv) * (HD / 16);
  int W = waves;
  if (W != 4 && W != 8) W = (groups * 8 * 2 <= 4096 && (K / 32) / 8 >= 8) ? 8 : 4;
  return M * Hkv + groups <= oproj_capacity(W, Hq / Hkv) ? 1 : 0;
}

// p2p_qkv_attn with the o_proj projection + residual in the same launch (TP = 1 decode):
// h[M][ldh] += attention @ Wo^T, Wo fragment-major [No / 16][Hq * 128 / 32][64][8] (bf16),
// Hq * 128 / 32 / waves <= 32.  gran2: u64 [M][Hq * 64], epoch: u32 [2] (zeroed once,
// private to this call site's buffers).  `out` is not written.
P2P_API int p2p_qkv_attn_oproj(const void* Wt, const void* X, int ldx, int M, int K, int Hq,
                               int Hkv, const int* pos, const int* slots, const void* cos_sin,
                               void* k_cache, void* v_cache, const int* block_tables,
                               int bt_stride, const int* ctx_lens, float scale, float eps,
                               void* gran, unsigned* counters, int* err, int waves,
                               const void* Wo, int No, void* h, int ldh, void* gran2,
                               unsigned* epoch, hipStream_t stream) {
  if (!Wo) return (int)hipErrorInvalidValue;
  return qkv_attn_impl(Wt, X, ldx, M, K, Hq, Hkv, pos, slots, cos_sin, k_cache, v_cache,
                       block_tables, bt_stride, ctx_lens, scale, nullptr, 0, eps, gran, counters,
                       err, waves, Wo, No, h, ldh, gran2, epoch, stream);
}
