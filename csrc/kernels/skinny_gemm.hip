#include <dlfcn.h>
// Skinny (M <= 64) bf16 GEMM on MFMA for decode / short-prefill projections.
//
//   out[m, n] = epilogue( rstd[m] * sum_k X[m, k] * W[n, k] )
//
// This is the hot loop of suggest-reply decode: at batch 1 every projection is
// a pure weight stream (16 GB / token for Llama-3.1-8B), so the kernel is built
// around one contiguous 1 KiB non-temporal load per wave per k-step.
//
// Weight layout ("fragment-major", produced once at load time by
// ops.gemm.tile_weight):
//     Wt[g][s][lane][j] = W[16*g + (lane & 15)][32*s + 8*(lane >> 4) + j]
// i.e. every 16x32 (n x k) block is stored exactly as the 64 lanes hold the B
// operand of v_mfma_f32_16x16x32_bf16.  The activation fragment (A operand,
// lane l holds X[l & 15][8*(l >> 4) + j]) is read straight from global memory
// (it is a few KiB and L2-resident).
//
// Fusions (epilogues), all replacing separate kernels of a naive decoder layer:
//   NORM      : RMSNorm of the input row.  The RMSNorm gain is folded into the
//               weight at load time, so only rstd[m] = rsqrt(mean(x^2)+eps)
//               remains; the sum of squares is accumulated from the same A
//               fragments the MFMA consumes and applied to the accumulator.
//   EPI_RESID : residual add in place (o_proj / down_proj).
//   EPI_SILU  : SwiGLU: the block owns gate rows g and up rows g+F/16 and
//               writes silu(gate) * up (gate_up_proj -> act -> [M, F]).
//   EPI_F32   : fp32 logits (LM head).
//   EPI_QKV_ROPE : qkv projection + RoPE + paged KV-cache write.  Weight rows of
//               every head are permuted at load time (ops.gemm.rope_row_perm) so
//               that each 16-row group holds dims {8k..8k+7} and {64+8k..64+8k+7};
//               the rotate_half partner of lane r is lane r^8 (one shuffle).  q goes
//               to q_out, k (rotated) and v to their pages -- no qkv round trip.
//   EPI_ARGMAX: greedy sampling fused into the LM head: per-row max over the
//               block's 16 columns, then one 64-bit atomicMax of
//               (ordered(value) << 32 | ~index) per row and block (ties -> lowest id).
// Split-K across the waves of a block (WAVES), reduced through LDS.
#include <map>
#include <mutex>

#include "skinny_gemm_impl.h"
#include "midm_gemm.h"

int g_skinny_u_mt1 = 4;
int skinny_unit_store(SKINNY_UNIT_ARGS);
int skinny_unit_resid(SKINNY_UNIT_ARGS);
int skinny_unit_silu(SKINNY_UNIT_ARGS);
int skinny_unit_f32(SKINNY_UNIT_ARGS);
int skinny_unit_qkv_rope(SKINNY_UNIT_ARGS);
int skinny_unit_argmax(SKINNY_UNIT_ARGS);
int skinny_unit_ar(SKINNY_UNIT_ARGS);

constexpr int MIDM_FLAG = 1 << 25;  // launch-code bit (ops.gemm.MIDM_FLAG)
constexpr int WIDE_FLAG = 1 << 26;  // launch-code bit (ops.gemm.WIDE_FLAG), K slices in bits 8..15,
                                     // bit 16: 16 waves per workgroup (ops.gemm.WIDE16)
constexpr int PERSIST_FLAG = 1 << 28;  // ops.gemm.PERSIST_FLAG: persist_gemv.hip, CU multiple in 8..15
// the persistent GEMV lives in the experimental library (measured slower than the skinny
// launches, profiles/r4_persist_gemv_negative.jsonl): resolved when that library is loaded
typedef int (*persist_gemv_fn)(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                               int norm, void* out, int ldo, float eps, int grid_mult,
                               hipStream_t st);
static persist_gemv_fn persist_gemv() {
  return (persist_gemv_fn)dlsym(RTLD_DEFAULT, "p2p_persist_gemv");
}
extern "C" int p2p_wide_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N,
                                 int epi, int norm, void* out, int ldo, float eps, const void* ea_p,
                                 int req_split, hipStream_t st);

// Picks the split-K factor: enough waves to keep ~8+ MB of weight loads in flight,
// but every wave resident in the first dispatch round (256 CUs x 4 SIMDs x
// g_resident waves/SIMD) and streaming >= 8 k-steps.
static int g_resident = 4;
static int pick_waves(int groups, int K, int mt) {
  const int S = K / 32;
  const int cap = 1024 * g_resident;
  int waves = 1;
  while (waves < 8 && groups * waves * 2 <= cap && S / (waves * 2) >= 8) waves *= 2;
  // LDS budget for the reduction buffer at the largest tile (SiLU, MT=4): keep <= 64 KiB.
  (void)mt;
  return waves;
}

// epi: 0 store bf16, 1 residual add (bf16, in place), 2 silu(gate)*up, 3 fp32 store,
//      4 qkv+rope+kv-cache (see p2p_skinny_gemm_qkv_rope), 5 greedy argmax keys (u64 [M]).
// N: number of weight rows (for epi 2: 2*F, gate rows then up rows).
// waves: 0 = heuristic.
static int skinny_dispatch(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                           int norm, void* out, int ldo, float eps, int waves, const EpiArgs& ea,
                           hipStream_t stream) {
  if (M <= 0 || M > 64 || (K % 32) != 0 || (N % 16) != 0) return (int)hipErrorInvalidValue;
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  int groups = N / 16;
  int up_off = 0;
  if (epi == EPI_SILU) {
    if ((N % 32) != 0) return (int)hipErrorInvalidValue;
    groups = N / 32;
    up_off = groups;
  }
  // bit 28: the persistent GEMV (persist_gemv.hip; bf16 dense weights, M <= 16)
  if ((waves & PERSIST_FLAG) && !ea.wscale && !ea.moe_cnt) {
    const persist_gemv_fn f = persist_gemv();
    if (!f) return (int)hipErrorNotSupported;  // experimental library not loaded
    return f(Wt, X, ldx, M, K, N, epi, norm, out, ldo, eps, (waves >> 8) & 0xff, stream);
  }
  // bit 26: the wide mid-M kernel (wide_gemm.hip; bf16 dense weights, K % 256 == 0)
  if ((waves & WIDE_FLAG) && epi != EPI_AR)
    return p2p_wide_dispatch(Wt, X, ldx, M, K, N, epi, norm, out, ldo, eps, &ea, (waves >> 8) & 0x1ff,
                             stream);
  // bit 25: the mid-M LDS-DMA kernel (midm_gemm.h; bf16 dense weights, K % 128 == 0)
  if ((waves & MIDM_FLAG) && !ea.wscale && !ea.moe_cnt && K % 128 == 0) {
    switch (epi) {
      case EPI_STORE:
        return norm ? midm::launch<EPI_STORE, true>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream)
                    : midm::launch<EPI_STORE, false>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream);
      case EPI_RESID:
        if (norm) return (int)hipErrorInvalidValue;
        return midm::launch<EPI_RESID, false>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream);
      case EPI_SILU:
        if (!norm) return (int)hipErrorInvalidValue;
        return midm::launch<EPI_SILU, true>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream);
      case EPI_F32:
        return norm ? midm::launch<EPI_F32, true>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream)
                    : midm::launch<EPI_F32, false>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream);
      case EPI_QKV_ROPE:
        if (!norm) return (int)hipErrorInvalidValue;
        return midm::launch<EPI_QKV_ROPE, true>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream);
      case EPI_ARGMAX:
        if (!norm) return (int)hipErrorInvalidValue;
        return midm::launch<EPI_ARGMAX, true>(Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, stream);
    }
    return (int)hipErrorInvalidValue;
  }
  // waves: low 8 bits = split-K waves (0 = heuristic), bits 8..15 = pipeline depth U
  // (0 = default), bits 16..23 = column groups per block (M > 16 only; 0 = 1)
  const int u_req = (waves >> 8) & 0xff;
  const int ng_req = (waves >> 16) & 0xff;
  const int afrag = (waves >> 27) & 1;  // bit 27: X is fragment-major (p2p_pack_frag)
  waves &= 0xff;
  if (waves <= 0) waves = pick_waves(groups, K, mt);
  if (epi == EPI_SILU && mt == 4 && waves > 4) waves = 4;
  if (waves == 16 && (mt != 1 || ea.wscale || ea.moe_cnt || epi == EPI_SILU))
    waves = 8;  // 16 waves: batch-1 bf16 projections other than SwiGLU
  EpiArgs ea2 = ea;
  ea2.u = u_req;
  ea2.ng = ng_req;
  ea2.afrag = afrag && !ea.moe_cnt;
  static const skinny_unit_fn units[] = {skinny_unit_store, skinny_unit_resid, skinny_unit_silu,
                                          skinny_unit_f32, skinny_unit_qkv_rope,
                                          skinny_unit_argmax, skinny_unit_ar};
  // the norm variants each epilogue is built with (the units return an error otherwise)
  switch (epi) {
    case EPI_RESID:
    case EPI_AR:
      if (norm) return (int)hipErrorInvalidValue;
      break;
    case EPI_SILU:
    case EPI_QKV_ROPE:
    case EPI_ARGMAX:
      if (!norm) return (int)hipErrorInvalidValue;
      break;
  }
  if (epi == EPI_AR) {
    if (ea.moe_cnt) return (int)hipErrorInvalidValue;
    ea2.ng = 0;  // one column group per block: block b owns the same columns on every rank
  }
  if (epi < EPI_STORE || epi > EPI_AR) return (int)hipErrorInvalidValue;
  return units[epi](norm, mt, waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, &ea2, stream);
  return (int)hipErrorInvalidValue;
}

// Tuning knobs (benchmarks): u_mt1 = k-steps per pipeline batch at M<=16 (4|8);
// resident = waves/SIMD assumed resident when picking the split-K factor.
P2P_API void p2p_skinny_gemm_tune(int u_mt1, int resident) {
  if (u_mt1 == 4 || u_mt1 == 8) g_skinny_u_mt1 = u_mt1;
  if (resident >= 1 && resident <= 8) g_resident = resident;
}

// wscale (all three entry points): null = bf16 fragment-major weights; else FP8 e4m3
// weights in the same fragment order, k-steps paired (ops.gemm.pair_f8), and their
// per-output-channel fp32 scales.
P2P_API int p2p_skinny_gemm(const void* Wt, const void* X, int ldx, int M, int K, int N, int epi,
                            int norm, void* out, int ldo, float eps, int waves,
                            const float* wscale, hipStream_t stream) {
  if (epi == EPI_QKV_ROPE) return (int)hipErrorInvalidValue;
  EpiArgs ea = {};
  ea.wscale = wscale;
  return skinny_dispatch(Wt, X, ldx, M, K, N, epi, norm, out, ldo, eps, waves, ea, stream);
}

// Greedy LM head: keys[m][shard] = atomicMax over columns of (ordered(logit) << 32 | ~(col+off)).
// keys ([M][32] u64) must be zero before the call (p2p_argmax_finalize / p2p_advance reduce
// the shards and reset them).
P2P_API int p2p_skinny_gemm_argmax(const void* Wt, const void* X, int ldx, int M, int K, int N,
                                   unsigned long long* keys, int col_offset, float eps, int waves,
                                   const float* wscale, hipStream_t stream) {
  EpiArgs ea = {};
  ea.col_offset = col_offset;
  ea.wscale = wscale;
  return skinny_dispatch(Wt, X, ldx, M, K, N, EPI_ARGMAX, 1, keys, 0, eps, waves, ea, stream);
}

// Fused qkv projection (rows permuted per head, see header) + RoPE + KV-cache write.
P2P_API int p2p_skinny_gemm_qkv_rope(const void* Wt, const void* X, int ldx, int M, int K,
                                     int Hq, int Hkv, const int* pos, const int* slots,
                                     const void* cos_sin, void* q_out, int ldq, void* k_cache,
                                     void* v_cache, float eps, int waves, const float* wscale,
                                     hipStream_t stream) {
  EpiArgs ea = {};
  ea.wscale = wscale;
  ea.pos = pos;
  ea.slots = slots;
  ea.cs = (const float2*)cos_sin;
  ea.q_out = (bf16*)q_out;
  ea.ldq = ldq;
  ea.kc = (bf16*)k_cache;
  ea.vc = (bf16*)v_cache;
  ea.Hq = Hq;
  ea.Hkv = Hkv;
  const int N = (Hq + 2 * Hkv) * HD;
  return skinny_dispatch(Wt, X, ldx, M, K, N, EPI_QKV_ROPE, 1, nullptr, 0, eps, waves, ea, stream);
}

// Ranks of a TP group resident on this device (1 on a node with a GPU per rank; the group
// size for virtual ranks): the fused all-reduce launch holds at most 1 / n of the device's
// block slots (skinny_gemm_impl.h skinny_gemm_kernel, EPI_AR).
static int g_far_coresident = 1;
P2P_API void p2p_far_set_coresident(int n) { g_far_coresident = n >= 1 ? n : 1; }

int far_grid(int groups, const void* kernel, int threads) {
  static std::map<const void*, int> occ;  // blocks per CU of each instantiation (host side)
  static std::mutex mu;
  int per_cu;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = occ.find(kernel);
    if (it == occ.end()) {
      int b = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, threads, 0) != hipSuccess || b < 1) b = 1;
      it = occ.emplace(kernel, b).first;
    }
    per_cu = it->second;
  }
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // ranks sharing the device: half of their share (the occupancy query can read one block
  // per CU high, MI355X_MICROARCH.md "Residency"; and a late rank's earlier kernels hold
  // slots until they drain), so a rank's waiting blocks never fill what a late peer needs
  const int share = g_far_coresident > 1 ? 2 * g_far_coresident : 1;
  const int cap = std::max(1, per_cu * std::max(cus, 1) / share);
  return std::min(groups, cap);
}

// TP row-parallel projection with the all-reduce fused into the epilogue (fused_ar.h):
//   h[m, :N] += sum over the group's ranks of (X @ W^T)[m, :N]   (bf16 partials, rank order)
// bases: every rank's fused buffer (p2p_far_buffer_bytes(max_bytes), own at [rank]);
// counters: device u32 [FAR_MAX_BLOCKS] (zeroed, private); err: device int.  Every rank
// of the group must make the same sequence of calls with the same N and M.  The tiled /
// mid-M launch-code bits are ignored (skinny kernel only; M <= 64).
P2P_API int p2p_skinny_gemm_ar(const void* Wt, const void* X, int ldx, int M, int K, int N,
                               void* h, int ldh, void* const* bases, int rank, int world,
                               size_t max_bytes, unsigned* counters, int* err, int waves,
                               const float* wscale, hipStream_t stream) {
  if (world < 1 || world > FAR_MAX_RANKS || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
  if (N % 16 || N / 16 > FAR_MAX_BLOCKS || ldh % 8 || ldh < N || M < 1 || M > 64 || max_bytes % 16)
    return (int)hipErrorInvalidValue;
  if (((size_t)(M - 1) * ldh + N) * 4 > max_bytes) return (int)hipErrorInvalidValue;  // granules
  EpiArgs ea = {};
  ea.wscale = wscale;
  for (int p = 0; p < world; ++p) ea.far.base[p] = (char*)bases[p];
  ea.far.rank = rank;
  ea.far.world = world;
  ea.far.max_bytes = max_bytes;
  ea.far.counters = counters;
  ea.far.err = err;
  ea.far.spin_ticks = p2p_car_spin_ticks();
  ea.far.groups = N / 16;
  waves &= ~(WIDE_FLAG | MIDM_FLAG | (1 << 24));  // skinny only
  return skinny_dispatch(Wt, X, ldx, M, K, N, EPI_AR, 0, h, ldh, 0.f, waves, ea, stream);
}

// tiled_gemm.hip: the grouped mode of the LDS-tiled MFMA kernel (rows > 64)
extern "C" int p2p_grouped_gemm_tiled(const void* Wt, long long w_stride, int n_experts,
                                      const int* cnt, const int* rows, int rows_stride, int x_div,
                                      const float* row_w, const void* X, int ldx, int max_rows,
                                      int K, int N, int epi, int norm, void* out, int ldo, float eps,
                                      hipStream_t stream);

// Grouped (MoE) projection over the local experts (blockIdx.y = expert):
//   expert e multiplies rows slot = rows[e*rows_stride + i] (i < cnt[e], <= max_rows) of
//   X (row slot / x_div) with its weights (Wt + e*w_stride) and writes output row slot.
// epi: 0 store (scaled by row_w[slot] if row_w) | 2 silu(gate)*up with RMSNorm (norm=1).
P2P_API int p2p_grouped_gemm(const void* Wt, long long w_stride, int n_experts, const int* cnt,
                             const int* rows, int rows_stride, int x_div, const float* row_w,
                             const void* X, int ldx, int max_rows, int K, int N, int epi, int norm,
                             void* out, int ldo, float eps, int waves, hipStream_t stream) {
  if (n_experts <= 0 || !cnt || !rows) return (int)hipErrorInvalidValue;
  if (epi != EPI_STORE && epi != EPI_SILU) return (int)hipErrorInvalidValue;
  if (max_rows > 64)  // prefill / big batches: the LDS-tiled MFMA kernel, grouped mode
    return p2p_grouped_gemm_tiled(Wt, w_stride, n_experts, cnt, rows, rows_stride, x_div, row_w,
                                  X, ldx, max_rows, K, N, epi, norm, out, ldo, eps, stream);
  EpiArgs ea = {};
  ea.moe_cnt = cnt;
  ea.moe_rows = rows;
  ea.rows_stride = rows_stride;
  ea.x_div = x_div > 0 ? x_div : 1;
  ea.row_w = row_w;
  ea.w_stride = w_stride;
  ea.n_experts = n_experts;
  return skinny_dispatch(Wt, X, ldx, max_rows, K, N, epi, norm, out, ldo, eps, waves, ea, stream);
}
