// All-reduce fused into the epilogue of a row-parallel projection (TP o_proj / down at
// decode sizes; SURVEY §5 "distributed comm backend" (a)).
//
// Unfused, a TP row-parallel projection is two dependent launches: the GEMM stores its
// bf16 partial, then the one-shot kernel (custom_allreduce.hip) pushes it to every peer,
// waits and sums into the residual.  Fused, the GEMM's own epilogue does that work for
// the tile it just produced:
//   1. the block's [M x 16] bf16 partial (the value the unfused GEMM would store) is
//      staged in LDS and pushed, 16 bytes per lane, into slot [parity][rank] of EVERY
//      rank's fused buffer (xGMI writes, all peers at once);
//   2. fence (system scope), then flag [parity][rank][block] := seq on every rank;
//   3. wait for flag [parity][src][block] == seq of every source on the OWN buffer --
//      block b only waits for block b of the peers (same grid and column mapping on
//      every rank), never for a grid barrier;
//   4. h[m, cols] += sum over ranks in rank order (fp32, one rounding): the unfused
//      formula, so the two paths are bit-identical on every rank.
// seq is the group's call index of this block (counters[block] + 1); block 0 keeps the
// counters of blocks a narrower call does not launch in step, as the one-shot kernel
// does.  Slot reuse: a rank writes parity p in call k+2 only after its call-(k+1) kernel
// saw call-(k+1) flags of every peer, which each peer posts only after its call-k kernel
// (the last reader of parity p) completed.  Spins are bounded; a timeout sets the error
// word and later calls skip their waits (LlamaModel.check_faults raises on it).
//
// Own buffer, separate from the one-shot kernel's (their call sequences interleave):
//   flags : [2 parities][FAR_MAX_RANKS src][FAR_MAX_BLOCKS] u32
//   data  : [2 parities][FAR_MAX_RANKS src][max_bytes]   (row-major [M, ldo] bf16)
#pragma once
#include <stddef.h>

#include "common.h"

constexpr int FAR_MAX_RANKS = 8;
constexpr int FAR_MAX_BLOCKS = 1024;  // column groups of 16: hidden sizes up to 16384
constexpr size_t FAR_FLAG_BYTES = 2ull * FAR_MAX_RANKS * FAR_MAX_BLOCKS * 4;

struct FusedArArgs {
  char* base[FAR_MAX_RANKS];  // every rank's fused buffer mapped here (own at [rank])
  int rank, world;
  size_t max_bytes;           // data bytes per (parity, src) slot
  unsigned* counters;         // [FAR_MAX_BLOCKS] private per-block call counters
  int* err;                   // set nonzero when a peer never arrived
  long long spin_ticks;       // spin bound (100 MHz wall clock)
};

// Host-side spin bound shared with the one-shot kernels (p2p_car_set_timeout_ms).
extern "C" long long p2p_car_spin_ticks();

namespace far {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned* flag(char* base, int parity, int src, int blk) {
  return reinterpret_cast<unsigned*>(base) + ((size_t)parity * FAR_MAX_RANKS + src) * FAR_MAX_BLOCKS + blk;
}

__device__ __forceinline__ bf16* data(char* base, size_t max_bytes, int parity, int src) {
  return reinterpret_cast<bf16*>(base + FAR_FLAG_BYTES + ((size_t)parity * FAR_MAX_RANKS + src) * max_bytes);
}

// Epilogue of ONE wave (the block's wave 0, after the split-K reduction).  v[mt][j] is the
// fp32 value of row m = 16 mt + 4 (lane >> 4) + j, column 16 g + (lane & 15) -- the MFMA
// 16x16 accumulator layout.  h: the residual [M, ldh] bf16, updated in place.
template <int MT>
__device__ __forceinline__ void epilogue(const float (&v)[MT][4], int M, int g, int lane,
                                         bf16* __restrict__ h, int ldh, const FusedArArgs& fa) {
  __shared__ __attribute__((aligned(16))) bf16 tile[MT * 16][16];
  const int r = lane & 15, q = lane >> 4;
  const int blk = blockIdx.x, nblk = gridDim.x;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = mt * 16 + q * 4 + j;
      if (m < M) tile[m][r] = f2bf(v[mt][j]);  // the partial the unfused GEMM would store
    }
  const unsigned seq = fa.counters[blk] + 1;
  const int parity = seq & 1;
  const int failed = __hip_atomic_load(fa.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // LDS tile complete before other lanes read it (single wave: fence + wave barrier)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const int nch = 2 * M;  // 16-byte chunks: 8 columns of one row
  const size_t col0 = (size_t)g * 16;
  // 1. push to every rank (including this one)
  for (int c = lane; c < nch; c += 64) {
    const int m = c >> 1, hf = c & 1;
    const v4u val = *reinterpret_cast<const v4u*>(&tile[m][hf * 8]);
    const size_t off = (size_t)m * ldh + col0 + hf * 8;
    for (int p = 0; p < fa.world; ++p)
      *reinterpret_cast<v4u*>(data(fa.base[p], fa.max_bytes, parity, fa.rank) + off) = val;
  }
  __threadfence_system();
  // 2. post
  if (lane < fa.world)
    __hip_atomic_store(flag(fa.base[lane], parity, fa.rank, blk), seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for block `blk` of every source (bounded; skipped once a peer is known dead)
  if (lane < fa.world && !failed) {
    unsigned* f = flag(fa.base[fa.rank], parity, lane, blk);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      if (wall_clock64() - t0 > fa.spin_ticks) {
        atomicOr(fa.err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_wave_barrier();
  // 4. h += sum in rank order (identical on every rank, = the unfused kernel's formula)
  for (int c = lane; c < nch; c += 64) {
    const int m = c >> 1, hf = c & 1;
    const size_t off = (size_t)m * ldh + col0 + hf * 8;
    bf16x8* hp = reinterpret_cast<bf16x8*>(h + off);
    const bf16x8 hv = *hp;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (float)hv[j];
    for (int p = 0; p < fa.world; ++p) {
      const v4u raw = __builtin_nontemporal_load(
          reinterpret_cast<const v4u*>(data(fa.base[fa.rank], fa.max_bytes, parity, p) + off));
      bf16x8 pv;
      __builtin_memcpy(&pv, &raw, 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)pv[j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *hp = o;
  }
  if (lane == 0) fa.counters[blk] = seq;
  if (blk == 0)  // keep the counters of blocks a narrower call does not launch in step
    for (int j = nblk + lane; j < FAR_MAX_BLOCKS; j += 64) fa.counters[j] = seq;
}

}  // namespace far
