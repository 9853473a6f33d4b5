// Wide mid-M GEMM (1 < M <= 64 rows: chat-length prompt prefill, batched decode).
//
//   out[m, n] = epilogue( rstd[m] * sum_k X[m, k] * W[n, k] )   (gemm_epilogue.h)
//
// Where the two older mid-M families lose (profiles/r2_midm_split_parallel.jsonl,
// r1_midM_gemm_families.jsonl):
//   * skinny_gemm.hip (one 16-column group per workgroup) and midm_gemm.h (same, K in an
//     LDS ring) re-read the whole activation block for every 16 output columns: at
//     M = 44 that is 3 activation KiB per weight KiB, and the activation stream, not the
//     weight stream, sets the time (qkv 24-28 us for a 50 MB weight stream);
//   * the split-K tiled kernel (prefill_gemm.h, 64 x 128 tiles) stages the weights
//     through LDS as well and fills only 192 of 256 CUs at the qkv shape.
// Here a workgroup of 8 waves owns 128 output columns (SwiGLU: 64 gate + the matching
// 64 up columns) and a K slice:
//   * the activation slice streams through an LDS ring of D + 2 chunk slots by LDS-DMA
//     (global_load_lds_dwordx4, fragment-major image, conflict-free ds_read_b128), or sits
//     in LDS whole when it fits (RES), and is read by all 8 waves: 16 activation rows cost
//     1/8 of a weight byte, not 1;
//   * each wave streams its OWN 16-column weight group straight into VGPRs (one 1 KiB
//     non-temporal load per k-step, fragment-major in HBM), 2-3 chunks of 8 k-steps ahead
//     (128-192 KiB of weights + the activation chunks in flight per CU: a one-chunk-ahead
//     first version was latency-bound at ~2.6 TB/s);
//   * the grid is column blocks x K slices, with the slice count picked so the grid is
//     <= one block per CU and close to the CU count (qkv at 8B: 48 x 5 = 240 blocks);
//     the K slices of a tile meet through tagged 8-byte granules (GranArgs below): unit
//     (column group w, m-tile i) is finished by slice (w * MT + i) % splitk, summing the
//     slices in slice order (deterministic);
// RMSNorm: the block squares the activation fragments it already holds in LDS (one
// m-tile per wave pair); the row sums of the slices meet as granules too.
// Measured (docs/ARCHITECTURE.md "Wide mid-M family"): the autotuner's pick at 33-64 rows
// for gate_up, down and qkv; the split-K seam (~5-6 us) is what it still pays on N <= 6144.
#include <cstdlib>
#include <type_traits>
#define PGEMM_NO_DISPATCH
#include "prefill_gemm.h"

namespace wide {

#ifdef WIDE_STAMP
// probe builds only (csrc/experimental/wide_stamp.hip): per-block wall-clock stamps
// [entry, first chunk ready, main loop done, granules stored (split) / -, polls done (split,
//  wave 0 only where it finishes a unit), end, tile, split]; the stores before a stamp
//  wait for completion in this build only (the stamp's own global load)
__device__ long long* wide_stamp_buf;
#define WSTAMP(i, v) do { if (wide_stamp_buf && threadIdx.x == 0) wide_stamp_buf[(size_t)blockIdx.x * 8 + (i)] = (v); } while (0)
#else
#define WSTAMP(i, v) do { } while (0)
#endif

constexpr int KC = 8;     // k-steps per chunk: wave w DMA-loads k-step w of every m-tile
constexpr int MAX_SPLIT = 16;  // K slices per tile (the rstd reduction unrolls over them)
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned long long u64;

// Split-K seam (r5): the K slices of a tile meet through 8-byte tagged granules
// {tag << 32 | fp32} (cdna_hip_programming.md R2: the data is the flag).  Each slice stores
// its partials once and moves on; the wave finishing an (output group, m-tile) unit polls
// the granules of every slice and needs no ticket, generation flip or second load.
// Tags: a block takes ticket[tile] (64-bit, monotonic) BEFORE its weight stream and shares
// it through LDS at the chunk-0 barrier; the splitk blocks of launch L of a (splitk, tile)
// pair draw L*splitk .. L*splitk + splitk-1, so tag = ticket / splitk + 1 is the same in all
// of them and new to every granule of the tile's region (each splitk value owns its tickets
// and its regions; stale granules carry older tags).  (A ticket per WAVE measured 2x slower:
// 64 agent-scope atomics per address serialise at the memory side, and the first chunk's
// loads queue behind them.)  No wave waits for the other waves of its block after its
// stream: each publishes its partials and its k-parity's row sums of squares at once.
// Replaces the write-through slabs + arrival ticket + generation flip, whose ~6 serial
// round trips cost 4-5 us per launch at 48 rows (r5 stamps).
struct GranArgs {
  int splitk;
  u64* gran;      // [tile][splitk][8 waves][4 m-tiles][4][64 lanes] partials
  u64* ssg;       // [tile][splitk][2 k parities][64 rows] RMSNorm row sums of squares
  u64* ticket;    // [tile]
  int* err;       // set if a finishing wave waited past the spin bound (results invalid)
  int align;      // slice boundaries rounded to multiples of this many k-steps (1 or KC)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS reads of the k loop as inline asm.  The activations reach LDS by DMA
// (global_load_lds), and the compiler cannot tell which ring slot a pending DMA writes: it
// put an s_waitcnt vmcnt(0) before every ds_read of the ring, so each chunk's compute waited
// for ALL loads in flight (the next D chunks' weights and activations too) and the pipeline
// drained at every chunk (r6 disassembly; gate_up 16 x 2.8 us per chunk on the ring path).
// The kernel's own counted vmcnt wait + barrier already makes chunk t's slot complete, so
// the reads go out as asm (the compiler inserts no wait for them) and lds_wait holds their
// results until they land.
__device__ __forceinline__ unsigned lds_off(const void* p) { return (unsigned)(uintptr_t)(lds_ptr_t)p; }
__device__ __forceinline__ bf16x8 lds_rd(const bf16x8* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_off(p)));
  return v;
}
// The LDS DMA itself goes out as asm too: with the builtin's DMA events pending, the
// compiler's own vmcnt tracking of the weight loads gave up (mixed event kinds on one
// counter) and put vmcnt(0) before every MFMA of the ring path, draining the pipeline just the
// same.  M0 = the wave's LDS destination; lane i's BYTES land at M0 + i * BYTES.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <int BYTES>
__device__ __forceinline__ void dma_lds(const void* g, const void* l) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_off(l));
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
}
#pragma clang diagnostic pop
// The weight stream as asm as well: the compiler does not count the asm DMAs, so its own
// waits for the weight registers came out AD x D loads short -- each MFMA waited for part of
// the NEXT chunk.  With every k-loop load and LDS read in asm, the kernel's counted
// wait_chunks + barrier + lds_wait are the only waits (an MFMA needs its A fragments from
// lds_wait, which follows the chunk's wait, so it never runs on a weight still in flight).
// KW loads of one chunk, skipped inside the asm when c >= n (past the slice): the compiler
// sees every register set written at every step, so it never merges an in-flight set with an
// older one (a branch around the loads made it copy in-flight registers), and no dummy load
// ever goes out (the slice's last chunk is the last thing waited for).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <int KW>
__device__ __forceinline__ void gload_chunk(bf16x8 (&w)[KW], const bf16x8* const (&p)[KW], int c, int n) {
  static_assert(KW == 4 || KW == 8, "gload_chunk: 4 or 8 k-steps per wave");
  if constexpr (KW == 4)
    asm volatile(
        "s_cmp_lt_i32 %8, %9\n\ts_cbranch_scc0 1f\n\t"
        "global_load_dwordx4 %0, %4, off nt\n\tglobal_load_dwordx4 %1, %5, off nt\n\t"
        "global_load_dwordx4 %2, %6, off nt\n\tglobal_load_dwordx4 %3, %7, off nt\n1:"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
        : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "s"(c), "s"(n)
        : "scc");
  else
    asm volatile(
        "s_cmp_lt_i32 %16, %17\n\ts_cbranch_scc0 1f\n\t"
        "global_load_dwordx4 %0, %8, off nt\n\tglobal_load_dwordx4 %1, %9, off nt\n\t"
        "global_load_dwordx4 %2, %10, off nt\n\tglobal_load_dwordx4 %3, %11, off nt\n\t"
        "global_load_dwordx4 %4, %12, off nt\n\tglobal_load_dwordx4 %5, %13, off nt\n\t"
        "global_load_dwordx4 %6, %14, off nt\n\tglobal_load_dwordx4 %7, %15, off nt\n1:"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]),
          "=&v"(w[6]), "=&v"(w[7])
        : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]),
          "s"(c), "s"(n)
        : "scc");
}
#pragma clang diagnostic pop
// after a chunk's counted wait: its registers re-defined, so no use (or copy) of them can be
// scheduled before the wait
template <int KW>
__device__ __forceinline__ void landed(bf16x8 (&w)[KW]) {
#pragma unroll
  for (int k = 0; k < KW; ++k) asm volatile("" : "+v"(w[k]));
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8 (&a)[N]) {
  static_assert(N >= 1 && N <= 4, "lds_wait: 1-4 fragments");
  if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]));
  if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]));
  if constexpr (N == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]));
  if constexpr (N == 4)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
}

// chunks of a K slice whose activations fit LDS at once (the RES variant): <= 144 KiB
template <int MT>
constexpr int res_chunks() { return 18 / MT; }

// tile = column block: 8 groups of 16 columns (SILU: waves 0-3 gate groups 4t..4t+3,
// waves 4-7 the up groups 4t..4t+3 + up_off; output columns 64t..64t+63).
// RES: the slice's whole activation block is DMA'd into LDS up front (one barrier), so the
// waves never meet again in the k loop and each streams its weights at its own pace;
// otherwise the activations stream through a ring with a barrier per chunk.
// NW = 16 (r6): two waves per column group, splitting every chunk's k-steps by parity (wave
// w and w + 8 stream group w & 7, k-steps of parity w >> 3), summed through LDS after the k
// loop.  A pure weight stream of these sizes reaches ~6.4 TB/s with 16 waves per CU and only
// ~5.3 with 8 (bench/stream_probe.py, profiles/r6_stream_probe.md): the 8-wave grid, one
// workgroup per CU, could not feed HBM however many bytes each wave kept in flight.
template <int MT, int EPI, bool NORM, bool SPLIT, bool RES, int NW>
__global__ __launch_bounds__(NW * 64) void wide_gemm_kernel(const bf16x8* __restrict__ Wt,
                                                            const bf16* __restrict__ X, int ldx, int M,
                                                            int K, int n_tiles, int up_off,
                                                            void* __restrict__ out, int ldo, float eps,
                                                            EpiArgs ea, GranArgs ga) {
  constexpr bool SILU = EPI == EPI_SILU;
  constexpr int NPAR = NW / 8;   // waves per column group (k-step parities)
  constexpr int KW = KC / NPAR;  // k-steps of a chunk per wave
  constexpr int NQ = NW / 4;     // NORM: k-step classes (mod NQ) x 4 m-tiles = NW waves
  constexpr int NQ2 = 2;         // classes left after the pair exchange (NW = 16: 2 + 2 -> 2)
  // pipeline depth: D chunks ahead (RS = D + 1 register sets of KW weight fragments: 128
  // VGPRs at NW = 8, D = 3; 32 at NW = 16, D = 1), activation ring of D + 2 slots (<= 128 KiB).
  // NW = 16 keeps ONE chunk (4 KiB per wave, 64 KiB per CU) ahead: the stream probe's best
  // in-flight depth at 16 waves per CU (deeper queues let every chunk of every CU arrive at
  // once, late, and the MFMAs start only then: r5 stamps, 6-10 us to the first chunk)
  constexpr int D = NW == 16 ? 1 : (MT >= 4 ? 2 : 3);
  constexpr int RS = D + 1;
  constexpr int RING = D + 2;
  constexpr int SLOT = MT * KC * 64;  // bf16x8 per ring slot
  constexpr int AD = (MT + NPAR - 1) / NPAR;  // activation DMA instructions per wave per chunk
  constexpr int PER_CHUNK = AD + KW;  // vmem instructions per thread per chunk
  constexpr int NSLOT = RES ? res_chunks<MT>() : RING;
  constexpr int NSV = NQ2 * MAX_SPLIT / 4;  // row-sum granules polled per lane (split-K NORM)
  __shared__ __attribute__((aligned(16))) bf16x8 ring[NSLOT * SLOT];
  __shared__ float ss_l[NQ2][4][16];
  __shared__ int slot_l[64], pos_l[64];  // EPI_QKV_ROPE: the rows' KV slots and positions

  const int splitk = SPLIT ? ga.splitk : 1;
  const int b = xcd_remap(blockIdx.x, n_tiles * splitk);
  const int tile = b / splitk, split = b % splitk;  // a tile's slices are consecutive
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wg = w & 7, par = w >> 3;  // column group of the tile, k-step parity
  const int S = K >> 5;
  // K slices in k-step units (r5: chunk-unit slices left qkv's 16 chunks in 5 slices as
  // 3/3/3/3/4 and the seam waited ~2.7 us for the long one); chunk c of the slice covers
  // k-steps ks0 + 8c .. + kv(c) - 1, only the last one partial.  A partial chunk still issues
  // full-count loads (clamped to its last k-step) so the counted vmcnt waits hold.
  const int al = SPLIT ? ga.align : 1;
  const int ks0 = split * (S / al) / splitk * al, nks = (split + 1) * (S / al) / splitk * al - ks0;
  const int n = (nks + KC - 1) / KC;
  auto kv_of = [&](int c) { return min(KC, nks - c * KC); };
  WSTAMP(0, wall_clock64());
  WSTAMP(6, tile);
  WSTAMP(7, split);
  // this launch's tag: the ticket load is the oldest in flight, long landed at the seam
  __shared__ unsigned tag_l;
  u64 tkt = 0;
  if constexpr (SPLIT)
    if (tid == 0) tkt = __hip_atomic_fetch_add(&ga.ticket[tile], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  const int gw = SILU ? (wg < 4 ? tile * 4 + wg : tile * 4 + (wg - 4) + up_off) : tile * 8 + wg;
  const bf16x8* wsrc = Wt + (size_t)gw * S * 64 + lane;
  const bf16* asrc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = min(16 * i + (lane & 15), M - 1);
    asrc[i] = X + (size_t)row * ldx + 8 * (lane >> 4);
  }

  // Chunk c's loads (nothing past the slice, c >= n).  Activations: wave w loads k-step
  // w & 7 of the m-tiles of its parity (NW = 16: the odd wave of a pair repeats its last
  // m-tile when MT is odd, so every wave issues AD instructions -- the same bytes to the same
  // LDS place -- and the counted waits hold).  The weights go out through gload_chunk.
  auto issue_a = [&](int c) {
    bf16x8* base = ring + (c % NSLOT) * SLOT;
    const int kk = ks0 + c * KC + min(wg, kv_of(c) - 1);
#pragma unroll
    for (int a = 0; a < AD; ++a) {
      const int i = min(par + NPAR * a, MT - 1);
      dma_lds<16>(asrc[i] + (size_t)kk * 32, base + (i * KC + wg) * 64);
    }
  };
  auto issue_w = [&](int c, bf16x8(&wr)[KW]) {
    const int cc = min(c, n - 1);  // (addresses only; no load goes out for c >= n)
    const int kb = ks0 + cc * KC, kl = kv_of(cc) - 1;
    const bf16x8* p[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) p[j] = wsrc + (size_t)(kb + min(par + NPAR * j, kl)) * 64;
    gload_chunk<KW>(wr, p, c, n);
  };
  auto issue = [&](int c, bf16x8(&wr)[KW]) {
    if constexpr (!RES)
      if (c < n) issue_a(c);
    issue_w(c, wr);
  };

  constexpr int PC = RES ? KW : PER_CHUNK;  // vmem instructions per chunk in the k loop
  auto wait_chunks = [&](int k) {  // at most k chunks of this thread's loads in flight
    switch (k) {
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<PC>(); break;
      case 2: wait_vmcnt<2 * PC>(); break;
      default: wait_vmcnt<(D >= 3 ? 3 : D) * PC>(); break;
    }
  };

  // The units this wave finishes: output group wg (SILU: gate/up pair wg < 4) at m-tile i;
  // under split-K unit (wg, i) belongs to slice (wg * MT + i) % splitk, so the 8 * MT units
  // of a tile spread over all its slices' waves (at most one each from splitk >= MT).  Only
  // the even wave of a parity pair finishes (it holds the pair's sum).
  const int r = lane & 15, q = lane >> 4;
  auto owns = [&](int i) {
    return par == 0 && wg < (SILU ? 4 : 8) && (!SPLIT || (wg * MT + i) % splitk == split);
  };
  const int g = SILU ? tile * 4 + wg : tile * 8 + wg;
  // Epilogue operands, issued as ONE batch per lane BEFORE the weight stream (they are the
  // oldest loads in flight, so the counted chunk waits below still hold, and they have long
  // landed when the epilogue runs): the residual values (EPI_RESID), the rows' KV slots and
  // positions (EPI_QKV_ROPE; the (cos, sin) loads that depend on the positions go out right
  // after the main loop).  Issued after the main loop, the residual loads held up the slab
  // drain of the split-K seam by ~1.6 us (bench/wide_stamp_probe.py, r5); loaded element by
  // element in the epilogue they were a chain of MT x 4 dependent round trips per lane.
  // (r6: the rows' slots / positions land in LDS by DMA from wave 0, not in 24 VGPRs per lane
  // held across the k loop -- the 16-wave variant has 128 VGPRs per lane in all)
  float res[MT][4];
  float2 csv[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * i + 4 * q + j;
      const bool ok = owns(i) && m < M;
      res[i][j] = 0.f;
      csv[i][j] = float2{1.f, 0.f};
      if constexpr (EPI == EPI_RESID && !(SPLIT && NW == 16))
        if (ok) res[i][j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + g * 16 + r];
    }
  if constexpr (EPI == EPI_QKV_ROPE)
    if (w == 0) {
      const int mm = min(lane, M - 1);
      dma_lds<4>(ea.slots + mm, slot_l);
      dma_lds<4>(ea.pos + mm, pos_l);
    }

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;  // NORM: rows of m-tile (w & 3), k-steps = (w >> 2) mod NQ, this lane's 8 k
  const int sq_mt = w & 3, sq_q = w >> 2;

  auto compute_kv = [&](const bf16x8* base, const bf16x8(&wr)[KW], int kv, auto full) {
    constexpr bool FULL = decltype(full)::value;
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const int k = par + NPAR * j;
      if (!FULL && k >= kv) break;
      // A fragments in flight together: every m-tile's (one at a time for MT = 4 at NW = 16)
      constexpr int AB = (NW == 16 && MT == 4) ? 1 : MT;
#pragma unroll
      for (int i0 = 0; i0 < MT; i0 += AB) {
        bf16x8 a[AB];
#pragma unroll
        for (int i = 0; i < AB; ++i) a[i] = lds_rd(base + ((i0 + i) * KC + k) * 64 + lane);
        lds_wait(a);
#pragma unroll
        for (int i = 0; i < AB; ++i)
          acc[i0 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], wr[j], acc[i0 + i], 0, 0, 0);
      }
    }
    if constexpr (NORM) {
      if (sq_mt < MT) {
        // reads in flight together: all of the chunk's at NW = 8, one at NW = 16 (128 VGPRs)
        constexpr int NS = KC / NQ, NB = NW == 16 ? 1 : NS;
#pragma unroll
        for (int u0 = 0; u0 < NS; u0 += NB) {
          bf16x8 x[NB];
#pragma unroll
          for (int u = 0; u < NB; ++u)  // a partial chunk reads a stale k-step, not summed
            x[u] = lds_rd(base + (sq_mt * KC + (u0 + u) * NQ + sq_q) * 64 + lane);
          lds_wait(x);
#pragma unroll
          for (int u = 0; u < NB; ++u)
            if (FULL || (u0 + u) * NQ + sq_q < kv) ss = sumsq8(x[u], ss);
        }
      }
    }
  };
  auto compute = [&](int c, const bf16x8(&wr)[KW]) {
    const bf16x8* base = ring + (c % NSLOT) * SLOT;
    const int kv = kv_of(c);
    if (kv == KC)
      compute_kv(base, wr, KC, std::true_type{});
    else  // a slice's last chunk, partial
      compute_kv(base, wr, kv, std::false_type{});
  };

  // D chunks (activation DMA + this wave's weights) are in flight ahead of the one being
  // computed; the counted wait + barrier makes chunk t complete (every wave's DMA part), and
  // the ring slot refilled at step t (chunk t+D's) was last read at t-2, before barrier t-1
  bf16x8 wr[RS][KW];
  if constexpr (RES)  // the whole slice's activations first (host: n <= res_chunks)
    for (int c = 0; c < n; ++c) issue_a(c);
  // Every real chunk's registers are read after its wait (landed + compute), so none is
  // dead while its load is in flight; past the slice no load goes out at all.
#pragma unroll
  for (int j = 0; j < D; ++j) issue(j, wr[j]);
  for (int tb = 0; tb < n; tb += RS) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const int t = tb + j;
      if (t >= n) break;
      issue(t + D, wr[(j + D) % RS]);
      wait_chunks(min(D, n - 1 - t));  // the chunks that went out after chunk t
      landed(wr[j]);
      if (!RES || t == 0) {  // RES: chunk 0's weights landed => this wave's DMA parts too
        if (SPLIT && t == 0 && tid == 0) tag_l = (unsigned)(tkt / (u64)splitk) + 1u;  // landed (oldest load)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (t == 0) WSTAMP(1, wall_clock64());
      }
      compute(t, wr[j]);
    }
  }

  WSTAMP(2, wall_clock64());
  // ---- this wave's row sums of squares: the NQ waves w = sq_mt + 4 x hold m-tile sq_mt ----
  if constexpr (NORM) {
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
  }
  if constexpr (NPAR > 1) {
    // the odd wave of each pair hands its partial sums (and its row sums of squares: k
    // classes 2, 3 -> 0, 1) to the even one through LDS (the activation buffer is free once
    // every wave is past its last read of it)
    float* xp = reinterpret_cast<float*>(ring);
    float* xs = xp + 8 * MT * 4 * 64;
    __syncthreads();
    if (par == 1) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) xp[((wg * MT + i) * 4 + j) * 64 + lane] = acc[i][j];
      if constexpr (NORM) xs[(w - 8) * 64 + lane] = ss;
    }
    __syncthreads();
    if (par == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += xp[((wg * MT + i) * 4 + j) * 64 + lane];
      if constexpr (NORM) ss += xs[w * 64 + lane];
    }
  }
  if constexpr (NORM)
    if (!SPLIT && par == 0 && sq_mt < MT && lane < 16) ss_l[sq_q & 1][sq_mt][lane] = ss;
  int slotv[MT][4];
  // EPI_QKV_ROPE: unit (i)'s KV slots and (cos, sin) -- issued right before the unit's poll
  // (split-K) or its stores; the slots / positions DMA was wave 0's first load, landed at the
  // chunk-0 barrier
  auto rope_operands = [&](int i) {
    if constexpr (EPI == EPI_QKV_ROPE) {
      const int kk = g & 7;
      const int dd = ((r < 8) ? 8 * kk + r : 64 + 8 * kk + (r - 8)) & 63;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 16 * i + 4 * q + j;
        const bool ok = owns(i) && m < M;
        slotv[i][j] = ok ? slot_l[m] : -1;
        if (ok) csv[i][j] = ea.cs[(size_t)pos_l[m] * 64 + dd];
      }
    }
  };
  if constexpr (!SPLIT) {
#pragma unroll
    for (int i = 0; i < MT; ++i) rope_operands(i);
  }

  auto epilogue = [&](const f32x4 (&v)[MT], const f32x4 (&u)[MT], auto&& rstd_of) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 16 * i + 4 * q + j;
        const bool valid = m < M;
        const float sc = rstd_of(i, j);
        if constexpr (EPI == EPI_QKV_ROPE) {
          epi_store<EPI>(m, valid, g, r, v[i][j] * sc, 0.f, out, ldo, ea, csv[i][j], slotv[i][j]);
        } else if constexpr (EPI == EPI_RESID) {
          if (valid)
            reinterpret_cast<bf16*>(out)[(size_t)m * ldo + g * 16 + r] = f2bf(res[i][j] + v[i][j] * sc);
        } else {
          epi_store<EPI>(m, valid, g, r, v[i][j] * sc, u[i][j] * sc, out, ldo, ea);
        }
      }
    }
  };
  auto rstd_from = [&](float t) { return rsqrtf(t / (float)K + eps); };

  if constexpr (!SPLIT) {
    // the up waves hand their accumulators to the gate waves through LDS (ring is free)
    float* xch = reinterpret_cast<float*>(ring);
    __syncthreads();  // every wave is past its last ring read (and the pair sums); ss_l complete
    if constexpr (SILU) {
      if (par == 0 && wg >= 4) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) xch[(((wg - 4) * MT + i) * 4 + j) * 64 + lane] = acc[i][j];
      }
      __syncthreads();
      if (wg >= 4) return;
    }
    if (par != 0) return;
    f32x4 up[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) up[i][j] = SILU ? xch[((wg * MT + i) * 4 + j) * 64 + lane] : 0.f;
    }
    epilogue(acc, up, [&](int i, int j) {
      if constexpr (!NORM) return 1.f;
      const int rr = 4 * q + j;
      return rstd_from(ss_l[0][i][rr] + ss_l[1][i][rr]);
    });
#ifdef WIDE_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    WSTAMP(5, wall_clock64());
    return;
  } else {
    // ---- split-K seam over tagged granules (see GranArgs) ----
    const unsigned tag = tag_l;  // written before the chunk-0 barrier
    const u64 tg = (u64)tag << 32;
    u64* gt = ga.gran + (size_t)tile * splitk * 8 * 4 * 256;  // this tile's region
    auto gidx = [&](int s2, int wv, int i, int j) { return (((s2 * 8 + wv) * 4 + i) * 4 + j) * 64 + lane; };
    if (par == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __hip_atomic_store(gt + gidx(split, wg, i, j), tg | __float_as_uint(acc[i][j]),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    u64* st = ga.ssg + (size_t)tile * splitk * NQ2 * 64;  // [split][k class][64 rows]
    if constexpr (NORM)
      if (par == 0 && sq_mt < MT && lane < 16)
        __hip_atomic_store(st + (split * NQ2 + (sq_q & 1)) * 64 + 16 * sq_mt + lane, tg | __float_as_uint(ss),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    WSTAMP(3, wall_clock64());
    bool any = false;
#pragma unroll
    for (int i = 0; i < MT; ++i) any |= owns(i);
    if (!any) return;
    // Finish the owned units.  One poll sweep re-reads a batch of SB slices' granules (and,
    // for the first batch, the rows' sum-of-squares granules) until every tag is this
    // launch's; the partials are summed in slice order (deterministic).
    constexpr int SB = NW == 16 ? (SILU ? 2 : 4) : (SILU ? 4 : 8);  // (NW = 16: 128 VGPRs)
    const long long t0 = wall_clock64();
    bool failed = false;
    auto ready = [&](u64 x) { return (unsigned)(x >> 32) == tag; };
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (!owns(i)) continue;
      rope_operands(i);
      if constexpr (EPI == EPI_RESID && NW == 16)  // (16 waves: loaded here, behind the poll)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = 16 * i + 4 * q + j;
          if (m < M) res[i][j] = (float)reinterpret_cast<const bf16*>(out)[(size_t)m * ldo + g * 16 + r];
        }
      f32x4 tot = f32x4{0.f, 0.f, 0.f, 0.f}, upv = f32x4{0.f, 0.f, 0.f, 0.f};
      float rowss = 0.f;  // NORM: lane l holds row 16 i + (l & 15) after the shuffles
      for (int s0 = 0; s0 < splitk; s0 += SB) {
        u64 pt[SB][4], pu[SB][4], sv[NSV];
        for (;;) {
          bool ok = true;
#pragma unroll
          for (int s = 0; s < SB; ++s) {
            if (s0 + s >= splitk) break;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              pt[s][j] = __hip_atomic_load(gt + gidx(s0 + s, wg, i, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if constexpr (SILU)
                pu[s][j] = __hip_atomic_load(gt + gidx(s0 + s, wg + 4, i, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          if constexpr (NORM)
            if (s0 == 0) {
              // lane l: row 16 i + (l & 15), (slice, k class) pairs c = (l >> 4) + 4 k
#pragma unroll
              for (int k = 0; k < NSV; ++k) {
                const int c = q + 4 * k;
                sv[k] = c < NQ2 * splitk ? __hip_atomic_load(st + c * 64 + 16 * i + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                        : tg;
              }
            }
#pragma unroll
          for (int s = 0; s < SB; ++s) {
            if (s0 + s >= splitk) break;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              ok &= ready(pt[s][j]);
              if constexpr (SILU) ok &= ready(pu[s][j]);
            }
          }
          if constexpr (NORM)
            if (s0 == 0) {
#pragma unroll
              for (int k = 0; k < NSV; ++k) ok &= ready(sv[k]);
            }
          if (__all(ok) || failed) break;
          const long long waited = wall_clock64() - t0;
          if (waited > pgemm::SPLIT_SPIN_TICKS) {
            if (lane == 0) __hip_atomic_store(ga.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            failed = true;
          }
          // a sweep re-reads up to 40 granules per lane: past ~5 us (a late slice, not the
          // usual skew) back off so a long wait does not load the memory system
          if (waited > 500) __builtin_amdgcn_s_sleep(32);
          else __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int s = 0; s < SB; ++s) {
          if (s0 + s >= splitk) break;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            tot[j] += __uint_as_float((unsigned)pt[s][j]);
            if constexpr (SILU) upv[j] += __uint_as_float((unsigned)pu[s][j]);
          }
        }
        if constexpr (NORM)
          if (s0 == 0) {
#pragma unroll
            for (int k = 0; k < NSV; ++k)
              if (q + 4 * k < NQ2 * splitk) rowss += __uint_as_float((unsigned)sv[k]);
          }
      }
      WSTAMP(4, wall_clock64());
      if constexpr (NORM) {
        rowss += __shfl_xor(rowss, 16, 64);
        rowss += __shfl_xor(rowss, 32, 64);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 16 * i + 4 * q + j;
        float sc = 1.f;
        if constexpr (NORM) sc = rstd_from(__shfl(rowss, 4 * q + j, 64));
        const float v = tot[j] * sc;
        if constexpr (EPI == EPI_QKV_ROPE) {
          epi_store<EPI>(m, m < M, g, r, v, 0.f, out, ldo, ea, csv[i][j], slotv[i][j]);
        } else if constexpr (EPI == EPI_RESID) {
          if (m < M) reinterpret_cast<bf16*>(out)[(size_t)m * ldo + g * 16 + r] = f2bf(res[i][j] + v);
        } else {
          epi_store<EPI>(m, m < M, g, r, v, upv[j] * sc, out, ldo, ea);
        }
      }
    }
#ifdef WIDE_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    WSTAMP(5, wall_clock64());
  }
}

static int g_max_split = MAX_SPLIT;
static int g_res = 1;  // RES variant where a slice's activations fit LDS (A/B: 0 = ring only)

// Granule workspaces, one per K-slice count (GranArgs: tickets and granule regions of one
// splitk value are never shared with another).  Sized for the most tiles that splitk allows
// on this device (grid <= one block per CU), zeroed at allocation; a grown workspace never
// frees the previous buffer (a captured hipGraph replays against it, see pgemm::split_ws).
struct GranWs {
  void* buf = nullptr;
  int tiles = 0;
};
static GranWs g_gran_ws[MAX_SPLIT + 1];

// P2P_WIDE_KSTEP=0: K slices on chunk boundaries (8 k-steps; r5 A/B against k-step slices)
static int kstep_align() {
  static int a = [] {
    const char* e = std::getenv("P2P_WIDE_KSTEP");
    return (e && e[0] == '0') ? KC : 1;
  }();
  return a;
}

static bool gran_ws(int splitk, int n_tiles, hipStream_t st, GranArgs* ga) {
  if (splitk < 2 || splitk > MAX_SPLIT) return false;
  char* ws = nullptr;  // the fault word lives at the end of the split-K workspace
  if (!pgemm::split_ws(0, st, &ws)) return false;
  GranWs& g = g_gran_ws[splitk];
  // tickets | row sums of squares [tile][split][<= 4 k classes][64] | partials
  auto bytes_for = [&](int tiles) {
    return (size_t)tiles * 8 + (size_t)tiles * splitk * 256 * 8 + (size_t)tiles * splitk * 8192 * 8 + 256;
  };
  if (g.tiles < n_tiles) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) return false;  // cannot allocate while capturing
    const int tiles = std::max(n_tiles, pgemm::cu_count() / splitk);
    void* buf = nullptr;
    if (hipMalloc(&buf, bytes_for(tiles)) != hipSuccess) return false;
    if (hipMemsetAsync(buf, 0, bytes_for(tiles), st) != hipSuccess) return false;
    g.buf = buf;
    g.tiles = tiles;
  }
  char* base = (char*)g.buf;
  const size_t tk = ((size_t)g.tiles * 8 + 255) / 256 * 256;
  ga->splitk = splitk;
  ga->ticket = (u64*)base;
  ga->ssg = (u64*)(base + tk);
  ga->gran = (u64*)(base + tk + (size_t)g.tiles * splitk * 256 * 8);
  int* fw = p2p_split_fault_word_ptr(st);
  ga->err = fw ? fw : (int*)(ws + pgemm::g_split_ws.bytes - sizeof(unsigned));
  ga->align = kstep_align();
  return true;
}

template <int MT, int EPI, bool NORM, bool SPLIT, bool RES>
int launch_v(const void* Wt, const void* X, int ldx, int M, int K, int n_tiles, int up_off,
             void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st,
             const GranArgs& ga, int nw) {
  if (nw == 16)
    hipLaunchKernelGGL((wide_gemm_kernel<MT, EPI, NORM, SPLIT, RES, 16>), dim3(n_tiles * ga.splitk),
                       dim3(16 * 64), 0, st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, n_tiles,
                       up_off, out, ldo, eps, ea, ga);
  else
    hipLaunchKernelGGL((wide_gemm_kernel<MT, EPI, NORM, SPLIT, RES, 8>), dim3(n_tiles * ga.splitk),
                       dim3(8 * 64), 0, st, (const bf16x8*)Wt, (const bf16*)X, ldx, M, K, n_tiles,
                       up_off, out, ldo, eps, ea, ga);
  return (int)hipGetLastError();
}

template <int MT, int EPI, bool NORM>
int launch_mt(const void* Wt, const void* X, int ldx, int M, int K, int n_tiles, int up_off,
              void* out, int ldo, float eps, const EpiArgs& ea, hipStream_t st, int splitk, int nw) {
  const int al = splitk > 1 ? kstep_align() : 1;
  const int S = K / 32, slice_ks = ((S / al + splitk - 1) / splitk) * al;  // the longest slice's k-steps
  const bool res = g_res && (slice_ks + KC - 1) / KC <= res_chunks<MT>();
  if (splitk > 1) {
    GranArgs ga{};
    if (!gran_ws(splitk, n_tiles, st, &ga))  // (no workspace growth while a graph is captured)
      return launch_mt<MT, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, 1, nw);
    return res ? launch_v<MT, EPI, NORM, true, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, ga, nw)
               : launch_v<MT, EPI, NORM, true, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, ga, nw);
  }
  GranArgs none{1, nullptr, nullptr, nullptr, nullptr, 1};
  return res ? launch_v<MT, EPI, NORM, false, true>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, none, nw)
             : launch_v<MT, EPI, NORM, false, false>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, none, nw);
}

// K slices: the grid must stay <= one block per CU (every slice of a tile resident for the
// parallel reduction) and each slice keeps >= 2 chunks; otherwise as many as fill the CUs.
// P2P_WIDE_SPLIT_CAP: hard cap on the K slices of every launch, requested ones included.  The
// slices of a tile meet in the kernel, so they must be resident together: true for a grid of
// at most one workgroup per CU on a device of its own, not for several processes sharing one
// device (virtual-rank tests), where the other processes' spinning grids can hold the CUs a
// late slice needs; those tests set the cap to 1.
static int split_cap() {
  static int c = [] {
    const char* e = std::getenv("P2P_WIDE_SPLIT_CAP");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 ? v : MAX_SPLIT;
  }();
  return c;
}

static int pick_split(int n_tiles, int nc, int req) {
  const int cus = pgemm::cu_count();
  if (cus <= 0) return 1;
  int s = req > 0 ? std::min(std::min(req, nc), MAX_SPLIT)
                  : std::min(cus / n_tiles, std::min(g_max_split, nc / 2));
  s = std::min(s, split_cap());
  while (s > 1 && n_tiles * s > cus) --s;
  return std::max(1, s);
}

template <int EPI, bool NORM>
int launch(const void* Wt, const void* X, int ldx, int M, int K, int N, void* out, int ldo,
           float eps, const EpiArgs& ea, hipStream_t st, int req_split, int nw) {
  const int cols = EPI == EPI_SILU ? 64 : 128;  // output columns per tile
  const int n_out = EPI == EPI_SILU ? N / 2 : N;
  if (M <= 0 || M > 64 || K % (32 * KC) || n_out % cols) return (int)hipErrorInvalidValue;
  const int n_tiles = n_out / cols;
  const int up_off = EPI == EPI_SILU ? N / 32 : 0;
  const int splitk = pick_split(n_tiles, K / (32 * KC), req_split);
  switch ((M + 15) / 16) {
    case 1: return launch_mt<1, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk, nw);
    case 2: return launch_mt<2, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk, nw);
    case 3: return launch_mt<3, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk, nw);
    case 4: return launch_mt<4, EPI, NORM>(Wt, X, ldx, M, K, n_tiles, up_off, out, ldo, eps, ea, st, splitk, nw);
  }
  return (int)hipErrorInvalidValue;
}

}  // namespace wide

// Called by skinny_dispatch (skinny_gemm.hip) for launch codes with the WIDE bit; ea_p points
// at the caller's EpiArgs (one identical definition per translation unit).  code: bits 0..7
// the K slices (0 = heuristic), bit 8 set = 16 waves per workgroup (two per column group,
// ops.gemm.WIDE16), else 8.  Dense bf16 weights only (no FP8, no grouped MoE mode).
extern "C" int p2p_wide_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N,
                                 int epi, int norm, void* out, int ldo, float eps, const void* ea_p,
                                 int code, hipStream_t st) {
  const EpiArgs& ea = *reinterpret_cast<const EpiArgs*>(ea_p);
  if (ea.wscale || ea.moe_cnt) return (int)hipErrorInvalidValue;
  using namespace wide;
  const int req_split = code & 0xff, nw = (code >> 8) & 1 ? 16 : 8;
  switch (epi) {
    case EPI_STORE:
      return norm ? launch<EPI_STORE, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw)
                  : launch<EPI_STORE, false>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw);
    case EPI_RESID:
      if (norm) return (int)hipErrorInvalidValue;
      return launch<EPI_RESID, false>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw);
    case EPI_SILU:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_SILU, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw);
    case EPI_F32:
      return norm ? launch<EPI_F32, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw)
                  : launch<EPI_F32, false>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw);
    case EPI_QKV_ROPE:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_QKV_ROPE, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw);
    case EPI_ARGMAX:
      if (!norm) return (int)hipErrorInvalidValue;
      return launch<EPI_ARGMAX, true>(Wt, X, ldx, M, K, N, out, ldo, eps, ea, st, req_split, nw);
  }
  return (int)hipErrorInvalidValue;
}

// Nonzero if a split slice of the wide kernel waited past its spin bound since the last call
// (that tile's output is invalid); clears the word.  The wide and tiled kernels share the
// device's split-K fault word (p2p_split_fault_word_ptr), so this is p2p_tiled_split_fault.
extern "C" int p2p_tiled_split_fault();
extern "C" int p2p_wide_split_fault() { return p2p_tiled_split_fault(); }

// Benchmarks: cap on the K-slice count of the heuristic (1 = never split).
// A/B: 1 = activations resident in LDS where a slice fits (default), 0 = the ring always.
P2P_API void p2p_wide_resident(int on) { wide::g_res = on ? 1 : 0; }

P2P_API void p2p_wide_max_split(int s) {
  wide::g_max_split = (s >= 1 && s <= wide::MAX_SPLIT) ? s : wide::MAX_SPLIT;
}

#ifdef WIDE_STAMP
P2P_API int p2p_wide_stamp_set(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(wide::wide_stamp_buf), &p, sizeof(p));
}
#endif
