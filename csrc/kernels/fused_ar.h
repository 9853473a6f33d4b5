// All-reduce fused into the epilogue of a row-parallel projection (TP o_proj / down at
// decode sizes; SURVEY §5 "distributed comm backend" (a)).
//
// Unfused, a TP row-parallel projection is two dependent launches: the GEMM stores its
// bf16 partial, then the one-shot kernel (custom_allreduce.hip) pushes it to every peer,
// waits and sums into the residual.  Fused, the GEMM's own epilogue does that work for
// the tile it just produced, with the payload carrying its own flag (low-latency "LL"
// granules, cdna_hip_programming.md publish/consume recipe R2):
//   1. the block's [M x 16] bf16 partial (the values the unfused GEMM would store) goes
//      out as 8-byte granules {seq << 32 | two bf16}, one relaxed system-scope 64-bit
//      store per granule, into slot [parity][rank] of EVERY rank's fused buffer (xGMI
//      writes, all peers at once).  No release fence (the first version fenced with
//      __threadfence_system, i.e. an L2 write-back per workgroup: +15 us per call on the
//      70B TP=8 proxy), no separate flag word;
//   2. the block sweeps the granules of ITS columns from every source on its own buffer
//      until every tag == seq (relaxed polls, bounded) -- block b only waits for block b
//      of the peers (same grid and column mapping on every rank), never a grid barrier;
//   3. h[m, cols] += sum over ranks in rank order (fp32, one rounding): the unfused
//      formula, so the two paths are bit-identical on every rank.
// seq is the call index of this column group (counters[group] + 1, never 0); group 0's
// block keeps the counters of groups a narrower call does not have in step, as the one-shot
// kernel does.  A granule left from an earlier call carries an older seq, so it is never
// taken for this call's.  Slot reuse: a rank writes parity p in call k+2 only after its
// call-(k+1) kernel saw call-(k+1) granules of every peer, which each peer writes only
// after its call-k kernel (the last reader of parity p) completed.  Spins are bounded; a
// timeout sets the error word and later calls skip their waits (check_faults raises).
//
// Own buffer, separate from the one-shot kernel's (their call sequences interleave):
//   data : [2 parities][FAR_MAX_RANKS src][max_bytes]   granule (m, c) at (m * ldh / 2 + c)
//          for column pair c = col / 2 -- twice the bytes of the bf16 partial
#pragma once
#include <stddef.h>

#include "common.h"

constexpr int FAR_MAX_RANKS = 8;
constexpr int FAR_MAX_BLOCKS = 1024;  // column groups of 16: hidden sizes up to 16384
constexpr size_t FAR_FLAG_BYTES = 0;  // no flag words: the granules carry the tags

struct FusedArArgs {
  char* base[FAR_MAX_RANKS];  // every rank's fused buffer mapped here (own at [rank])
  int rank, world;
  size_t max_bytes;           // data bytes per (parity, src) slot
  unsigned* counters;         // [FAR_MAX_BLOCKS] private per-block call counters
  int* err;                   // [4]: nonzero when a peer never arrived (+ where, see below)
  long long spin_ticks;       // spin bound (100 MHz wall clock)
  int groups;                 // column groups of the call (the launch may have fewer blocks)
};

// Host-side spin bound shared with the one-shot kernels (p2p_car_set_timeout_ms).
extern "C" long long p2p_car_spin_ticks();

namespace far {

typedef unsigned long long u64;

__device__ __forceinline__ u64* data(char* base, size_t max_bytes, int parity, int src) {
  return reinterpret_cast<u64*>(base + FAR_FLAG_BYTES + ((size_t)parity * FAR_MAX_RANKS + src) * max_bytes);
}

__device__ __forceinline__ unsigned bf16_bits(float x) {
  const bf16 b = f2bf(x);
  unsigned short u;
  __builtin_memcpy(&u, &b, 2);
  return u;
}

__device__ __forceinline__ float bits_bf16(unsigned u) {
  const unsigned short s = (unsigned short)u;
  bf16 b;
  __builtin_memcpy(&b, &s, 2);
  return (float)b;
}

// Epilogue of ONE wave (the block's wave 0, after the split-K reduction).  v[mt][j] is the
// fp32 value of row m = 16 mt + 4 (lane >> 4) + j, column 16 g + (lane & 15) -- the MFMA
// 16x16 accumulator layout.  h: the residual [M, ldh] bf16, updated in place.
// h_pre: the lane's first residual pair (i = lane), when the caller loaded it before its
// weight stream (nullptr: read here).
template <int MT>
__device__ __forceinline__ void epilogue(const float (&v)[MT][4], int M, int g, int lane,
                                         bf16* __restrict__ h, int ldh, const FusedArArgs& fa,
                                         const unsigned* h_pre = nullptr) {
  const int r = lane & 15, q = lane >> 4;
  // per column group: the call's group g is finished by exactly one block (the launch may
  // walk several groups per block: skinny_gemm_kernel, EPI_AR)
  const int blk = g, nblk = fa.groups;
  const unsigned seq = fa.counters[blk] + 1;
  const int parity = seq & 1;
  const int failed = __hip_atomic_load(fa.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const size_t row_g = (size_t)ldh / 2;  // granules per row
  const size_t c0 = (size_t)g * 8;       // first granule (column pair) of this block
  // 1. publish: lanes with an even column pack (col, col + 1) with the tag
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = mt * 16 + q * 4 + j;
      const float hi = __shfl_xor(v[mt][j], 1, 64);
      if (m < M && (r & 1) == 0) {
        const u64 gr = ((u64)seq << 32) | ((u64)bf16_bits(hi) << 16) | bf16_bits(v[mt][j]);
        const size_t off = (size_t)m * row_g + c0 + (r >> 1);
        for (int p = 0; p < fa.world; ++p)
          __hip_atomic_store(data(fa.base[p], fa.max_bytes, parity, fa.rank) + off, gr,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  // 2. + 3. sweep this block's granules of every source, then h += rank-ordered sum
  const long long t0 = wall_clock64();
  for (int i = lane; i < 8 * M; i += 64) {
    const int m = i >> 3, c = i & 7;
    const size_t off = (size_t)m * row_g + c0 + c;
    unsigned* hp = reinterpret_cast<unsigned*>(h + (size_t)m * ldh + 2 * (c0 + c));
    const unsigned hv = (h_pre && i == lane) ? *h_pre : *hp;
    float a0 = bits_bf16(hv & 0xffff), a1 = bits_bf16(hv >> 16);
    u64 x[FAR_MAX_RANKS];
#pragma unroll
    for (int p = 0; p < FAR_MAX_RANKS; ++p)  // every source's granule in flight at once
      x[p] = p < fa.world ? __hip_atomic_load(data(fa.base[fa.rank], fa.max_bytes, parity, p) + off,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                          : ((u64)seq << 32);
    for (;;) {  // re-read the granules whose tag is not this call's yet (bounded)
      bool ok = true;
#pragma unroll
      for (int p = 0; p < FAR_MAX_RANKS; ++p) ok &= (unsigned)(x[p] >> 32) == seq;
      if (ok || failed) break;
      if (wall_clock64() - t0 > fa.spin_ticks) {
        atomicOr(fa.err, 2);  // bit 1: a fused epilogue timed out (one-shot kernels set bit 0)
        // the first timeout of this rank records where it waited: err[1] = column group + 1,
        // err[2] = the call's seq, err[3] = the sources whose granule never carried it
        unsigned miss = 0;
#pragma unroll
        for (int p = 0; p < FAR_MAX_RANKS; ++p)
          if (p < fa.world && (unsigned)(x[p] >> 32) != seq) miss |= 1u << p;
        if (atomicCAS(fa.err + 1, 0, blk + 1) == 0) {
          __hip_atomic_store(fa.err + 2, (int)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(fa.err + 3, (int)miss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int p = 0; p < FAR_MAX_RANKS; ++p)
        if (p < fa.world && (unsigned)(x[p] >> 32) != seq)
          x[p] = __hip_atomic_load(data(fa.base[fa.rank], fa.max_bytes, parity, p) + off,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
    for (int p = 0; p < FAR_MAX_RANKS; ++p) {  // fixed rank order: identical sums on every rank
      if (p < fa.world) {
        a0 += bits_bf16((unsigned)x[p] & 0xffff);
        a1 += bits_bf16(((unsigned)x[p] >> 16) & 0xffff);
      }
    }
    *hp = bf16_bits(a0) | (bf16_bits(a1) << 16);
  }
  if (lane == 0) fa.counters[blk] = seq;
  if (blk == 0)  // keep the counters of groups a narrower call does not have in step
    for (int j = nblk + lane; j < FAR_MAX_BLOCKS; j += 64) fa.counters[j] = seq;
}

}  // namespace far
