// Shared GEMM epilogues (skinny_gemm.hip, tiled_gemm.hip): what happens to one
// fp32 accumulator element (row m, column 16*g + r) after the K reduction.
#pragma once
#include "common.h"
#include "fused_ar.h"

namespace {

// EPI_AR: TP row-parallel projection with the all-reduce + residual add fused into the
// epilogue (skinny kernel only; fused_ar.h)
enum : int { EPI_STORE = 0, EPI_RESID = 1, EPI_SILU = 2, EPI_F32 = 3, EPI_QKV_ROPE = 4,
             EPI_ARGMAX = 5, EPI_AR = 6 };

constexpr int PAGE = 64;
constexpr int HD = 128;
constexpr int KEY_SHARDS = 32;  // keys buffer: [M][KEY_SHARDS] u64 (see EPI_ARGMAX)

struct EpiArgs {
  // EPI_QKV_ROPE
  const int* pos;
  const int* slots;
  const float2* cs;  // [max_pos][64] (cos, sin)
  bf16* q_out;
  int ldq;
  bf16* kc;
  bf16* vc;
  int Hq, Hkv;
  // EPI_ARGMAX: global column offset of this shard (vocab-parallel LM head)
  int col_offset;
  // Grouped (MoE) mode: blockIdx.y = local expert e.  Its rows are the slot ids
  // rows[e * rows_stride + i], i < cnt[e]; the A row of slot s is X[s / x_div]
  // (x_div = top_k when X holds token rows), the output row is s, scaled by
  // row_w[s] when row_w != null.  Expert weights are w_stride bf16x8 apart.
  const int* moe_cnt;
  const int* moe_rows;
  int rows_stride;
  int x_div;
  const float* row_w;
  long long w_stride;
  int n_experts;
  const float* wscale;  // FP8 weights: per-output-channel scale [N] (null = bf16 weights)
  int u;   // requested pipeline depth (0 = default)
  int ng;  // requested column groups per block (skinny GEMM, M > 16; 0/1 = one)
  const float* rstd_in;  // prefill GEMM NORM: per-row rstd precomputed (null = in-loop sums)
  int afrag;  // skinny GEMM: X is fragment-major (p2p_pack_frag), 16-row m-tiles of K/32 x 1 KiB
  FusedArArgs far;       // EPI_AR: the group's fused all-reduce buffers
};

__device__ __forceinline__ unsigned long long argmax_key(float v, unsigned idx) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}

// Stores one accumulator element (row m, local column r of group g).  Called by
// all 64 lanes of the epilogue wave (the QKV/ARGMAX epilogues shuffle).
template <int EPI>
__device__ __forceinline__ void epi_store(int m, bool valid, int g, int r, float v, float u,
                                          void* __restrict__ out, int ldo, const EpiArgs& ea,
                                          float2 c = float2{1.f, 0.f}, int slot = -1) {
  if constexpr (EPI == EPI_QKV_ROPE) {
    // c (cos, sin) and slot were prefetched before the main loop (rope_prefetch)
    const float vp = __shfl_xor(v, 8, 64);
    if (!valid) return;
    const int head = g >> 3;
    const int k = g & 7;
    const int d = (r < 8) ? 8 * k + r : 64 + 8 * k + (r - 8);
    if (head < ea.Hq + ea.Hkv) {
      const float y = (r < 8) ? (v * c.x - vp * c.y) : (v * c.x + vp * c.y);
      if (head < ea.Hq) {
        ea.q_out[(size_t)m * ea.ldq + (size_t)head * HD + d] = f2bf(y);
      } else {
        if (slot >= 0)
          ea.kc[(((size_t)(slot / PAGE) * ea.Hkv + (head - ea.Hq)) * PAGE + slot % PAGE) * HD + d] =
              f2bf(y);
      }
    } else {
      if (slot >= 0)
        ea.vc[(((size_t)(slot / PAGE) * ea.Hkv + (head - ea.Hq - ea.Hkv)) * PAGE + slot % PAGE) *
                  HD + d] = f2bf(v);
    }
  } else if constexpr (EPI == EPI_ARGMAX) {
    unsigned long long key = argmax_key(v, (unsigned)(ea.col_offset + g * 16 + r));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const unsigned long long ok = __shfl_xor(key, o, 64);
      key = ok > key ? ok : key;
    }
    // sharded by block id: one 64-bit atomic per (row, shard) keeps contention at
    // ~groups/KEY_SHARDS arrivals per word instead of all groups on one word.  The 32 words
    // of a row share two cache lines, so the atomics of a launch still serialise at one
    // memory-side channel (8016 of them at the 8B LM head: +25 us over the fp32-logits
    // epilogue, bench/lmhead_probe.py).  A word only grows within a launch and is reset
    // between launches (argmax_finalize / advance, a kernel boundary apart), so any value
    // read back is a lower bound of the word: a key not above it can never win and its
    // atomic is skipped -- exact, and most groups after the first few skip.
    if (valid && r == 0) {
      unsigned long long* kp =
          reinterpret_cast<unsigned long long*>(out) + (size_t)m * KEY_SHARDS + (g % KEY_SHARDS);
      if (key > __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(kp, key);
    }
  } else {
    if (!valid) return;
    const size_t o = (size_t)m * ldo + g * 16 + r;
    if constexpr (EPI == EPI_STORE) {
      reinterpret_cast<bf16*>(out)[o] = f2bf(v);
    } else if constexpr (EPI == EPI_RESID) {
      bf16* p = reinterpret_cast<bf16*>(out) + o;
      *p = f2bf((float)*p + v);
    } else if constexpr (EPI == EPI_SILU) {
      reinterpret_cast<bf16*>(out)[o] = f2bf(silu(v) * u);
    } else {
      reinterpret_cast<float*>(out)[o] = v;
    }
  }
}


}  // namespace
