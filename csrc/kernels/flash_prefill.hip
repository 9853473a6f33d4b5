// Causal prefill attention on MFMA (flash-attention style) over the paged KV
// cache, GQA-packed: one workgroup = one KV head x one tile of <= 16
// consecutive query tokens of one sequence; wave w of the G = Hq/Hkv waves
// owns q-head kvh*G + w, so every K/V tile staged in LDS feeds G heads.
//
// Per 32-key tile and wave (everything transposed so no register shuffles are
// needed between the two GEMMs):
//   S^T[32 keys x 16 tok] = K[keys x 128] . Q^T          8 x mfma_16x16x32_bf16
//   (online softmax per token column; lane owns one token and 8 keys)
//   O^T[128 x 16 tok]   += V^T[128 x 32 keys] . P^T      8 x mfma_16x16x32_bf16
// The MFMA reduction index k is a permutation of the 32 keys chosen so that
// the S^T accumulator registers of a lane ARE its P^T B-operand (slot (g, j)
// <-> key 4g+j for j<4, 16+4g+j-4 otherwise); V^T uses the same permutation.
//
// Replaces the per-row decode kernel for long prompts, whose K/V traffic is
// O(T^2): here each K/V tile is read once per 16 query tokens x G heads.
// Behavioural parity: the reference delegates prompt processing to an external
// Ollama server (`web/streamlit_app.py:89-101`), see SURVEY.md §2B.2 B2.3.
#include "common.h"

namespace {

constexpr int PAGE = 64, HD = 128, KT = 32, QT = 16;
constexpr int KLD = HD + 8;   // K tile row stride (bf16), breaks LDS bank aliasing
constexpr int VLD = KT + 4;   // V^T tile row stride (bf16), 8-byte aligned rows

struct Tile {
  int row0, n, seq, pos0;
};

template <int G>
__global__ __launch_bounds__(64 * G) void flash_prefill_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ kc,
    const bf16* __restrict__ vc, const int* __restrict__ bt, int bt_stride,
    const Tile* __restrict__ tiles, int n_tiles, int Hkv, float scale_log2,
    bf16* __restrict__ out, int ldo) {
  constexpr int NTH = 64 * G;
  constexpr int CH = KT * HD / 8;          // 16-byte chunks per K (or V) tile
  constexpr int PER = (CH + NTH - 1) / NTH;
  __shared__ __attribute__((aligned(16))) bf16 Ks[KT * KLD];
  __shared__ __attribute__((aligned(16))) bf16 Vt[HD * VLD];

  const int nb = n_tiles * Hkv;
  const int b = xcd_remap(blockIdx.x, nb);
  const int ti = b / Hkv, kvh = b % Hkv;  // consecutive ids: same tile, all heads
  const Tile T = tiles[ti];
  if (T.n <= 0) return;  // padding tile of a graph-captured prefill (fixed grid)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, col = lane & 15;
  const int h = kvh * G + w;

  // Q^T B-operand fragments: token col, d = 32s + 8g + j
  const int tok = col < T.n ? col : T.n - 1;
  const int my_pos = T.pos0 + tok;
  bf16x8 qf[4];
  {
    const bf16* qp = q + (size_t)(T.row0 + tok) * ldq + h * HD + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
  }

  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  const int last = T.pos0 + T.n - 1;
  const int n_kt = last / KT + 1;
  const int* btr = bt + (size_t)T.seq * bt_stride;
  const size_t head_off = (size_t)kvh * PAGE * HD;
  const size_t page_sz = (size_t)Hkv * PAGE * HD;

  bf16x8 kr[PER], vr[PER];
  auto fetch = [&](int kt) {
    const int k0 = kt * KT;
    const size_t base = (size_t)btr[k0 / PAGE] * page_sz + head_off + (size_t)(k0 % PAGE) * HD;
    const bf16x8* kp = reinterpret_cast<const bf16x8*>(kc + base);
    const bf16x8* vp = reinterpret_cast<const bf16x8*>(vc + base);
    // V chunk c = key (c % KT), dims 8 (c / KT)..+7: 32 consecutive lanes hold the 32
    // keys of one 8-dim block, so the transposed b16 stores below are bank-conflict free
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTH;
      if (c < CH) {
        kr[i] = kp[c];
        vr[i] = vp[(c % KT) * (HD / 8) + c / KT];
      }
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTH;
      if (c < CH) {
        *reinterpret_cast<bf16x8*>(&Ks[(c >> 4) * KLD + (c & 15) * 8]) = kr[i];
        const int key = c % KT, d0 = (c / KT) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) Vt[(d0 + j) * VLD + key] = vr[i][j];
      }
    }
  };

  fetch(0);
  for (int kt = 0; kt < n_kt; ++kt) {
    __syncthreads();  // previous tile fully consumed
    stash();
    __syncthreads();
    if (kt + 1 < n_kt) fetch(kt + 1);  // overlap next tile's HBM reads with the math

    // S^T = K Q^T : two 16-key row tiles
    f32x4 s[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      s[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 a =
            *reinterpret_cast<const bf16x8*>(&Ks[(16 * mt + col) * KLD + 32 * ks + 8 * g]);
        s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[ks], s[mt], 0, 0, 0);
      }
    }
    // online softmax for token `col`; this lane holds keys 16mt + 4g + j
    const int k0 = kt * KT;
    float mx = -INFINITY;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = k0 + 16 * mt + 4 * g + j;
        const float v = key <= my_pos ? s[mt][j] * scale_log2 : -INFINITY;
        s[mt][j] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);  // m - mn <= 0; -inf -> 0
    m = mn;
    bf16x8 pf;
    float ps = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __builtin_amdgcn_exp2f(s[mt][j] - mn);
        ps += p;
        pf[4 * mt + j] = f2bf(p);
      }
    l = l * alpha + ps;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) acc[dt] *= alpha;

    // O^T += V^T P^T ; A row = d (16dt + col), k-slot (g, j) -> key 16(j>>2) + 4g + (j&3)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const bf16* vrow = &Vt[(16 * dt + col) * VLD + 4 * g];
      const bf16x4 lo = *reinterpret_cast<const bf16x4*>(vrow);
      const bf16x4 hi = *reinterpret_cast<const bf16x4*>(vrow + 16);
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = lo[j];
        a[4 + j] = hi[j];
      }
      acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pf, acc[dt], 0, 0, 0);
    }
  }

  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (col < T.n) {
    const float inv = 1.f / l;
    bf16* op = out + (size_t)(T.row0 + col) * ldo + h * HD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[dt][j] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt) = o;
    }
  }
}

template <int G>
int launch(const bf16* q, int ldq, const bf16* kc, const bf16* vc, const int* bt, int bt_stride,
           const Tile* tiles, int n_tiles, int Hkv, float scale, bf16* out, int ldo,
           hipStream_t st) {
  const float sl2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(flash_prefill_kernel<G>, dim3(n_tiles * Hkv), dim3(64 * G), 0, st, q, ldq,
                     kc, vc, bt, bt_stride, tiles, n_tiles, Hkv, sl2, out, ldo);
  P2P_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------
// v2: 256 query rows per workgroup (8 waves x 32 rows), one 64-key page per K/V tile,
// v_mfma_f32_32x32x16_bf16 throughout.
//
// A workgroup = one KV head x QT = 256/G consecutive tokens of one sequence; wave w
// owns q head kvh*G + w/(8/G) and 32 of the tokens, so every K/V page staged in LDS
// feeds 256 (token, head) rows -- 16x the reuse of v1 (16 tokens x G heads).
// Per 64-key tile and wave, both products keep the query row on the lane:
//   S^T[32 keys x 32 rows] = K . Q^T   (per 32-key half: 8 MFMAs over d = 128)
//   O^T[128 d  x 32 rows] += V^T . P^T (4 d-blocks x 2 halves x 2 k-steps = 16 MFMAs)
// so the online-softmax statistics and the O rescale are per lane (no cross-lane
// moves but one xor-32 for the row max / sum).  The S^T accumulator registers are
// directly the P^T B operand (cdna_hip_programming.md §3 "An accumulator tile as the
// next MFMA's operand"): register 8s+j of lane half h holds S^T row
// 16s + 8(j>>2) + 4h + (j&3); the K rows are loaded permuted (row rho <- key
// kappa(rho)) so that this row is key 16s + 8h + j, i.e. the eight keys a lane
// contributes to one k-step are CONSECUTIVE -- the V^T A-fragment is then a single
// 16-byte LDS read of a [d][key] image.  K is staged row-major [key][d] (272-B rows:
// conflict-free b128 reads), V transposed to [d][key] (144-B rows) while staging.
// The next page's global loads are issued right after the barrier and land in
// registers while the MFMAs run (one barrier per tile, two LDS stages).
constexpr int KLD2 = HD + 8;  // K image row stride (bf16)
constexpr int VLD2 = 64 + 8;  // V^T image row stride (bf16)
constexpr int KS_ELEMS = 64 * KLD2, VS_ELEMS = HD * VLD2;

typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int kperm(int rho) {  // S^T row rho -> key within the 32-key half
  const int s = rho >> 4, r = rho & 15;
  return 16 * s + 8 * ((r >> 2) & 1) + 4 * (r >> 3) + (r & 3);
}

template <int G>
__global__ __launch_bounds__(512) void flash_prefill2_kernel(
    const bf16* __restrict__ q, int ldq, const bf16* __restrict__ kc,
    const bf16* __restrict__ vc, const int* __restrict__ bt, int bt_stride,
    const Tile* __restrict__ tiles, int n_tiles, int Hkv, float scale_log2,
    bf16* __restrict__ out, int ldo) {
  constexpr int WPH = 8 / G;  // waves per q head
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * (KS_ELEMS + VS_ELEMS)];

  // heads outermost, heaviest (latest) tiles first; one head's tiles share an XCD's L2
  const int nb = n_tiles * Hkv;
  const int b = xcd_remap(blockIdx.x, nb);
  const int kvh = b / n_tiles, ti = n_tiles - 1 - b % n_tiles;
  const Tile T = tiles[ti];
  if (T.n <= 0) return;  // padding tile of a graph-captured prefill (fixed grid)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int r32 = lane & 31, hh = lane >> 5;
  const int h = kvh * G + w / WPH;
  const int t = (w % WPH) * 32 + r32;      // token of this lane's query row
  const int tok = t < T.n ? t : T.n - 1;
  const int my_pos = T.pos0 + tok;
  const int row = T.row0 + tok;

  // Q^T B fragments: k-step s covers d = 16s .. 16s+15, lane half hh holds 8hh .. 8hh+7
  bf16x8 qf[8];
  {
    const bf16* qp = q + (size_t)row * ldq + h * HD + 8 * hh;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s);
  }
  f32x16_t o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[db][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  const int last = T.pos0 + T.n - 1;
  const int n_kt = last / PAGE + 1;
  const int* btr = bt + (size_t)T.seq * bt_stride;
  const size_t head_off = (size_t)kvh * PAGE * HD;
  const size_t page_sz = (size_t)Hkv * PAGE * HD;
  const int krow = kperm(r32);

  // K/V of a page travel global -> registers -> LDS.  Two register sets, so a page's
  // loads are issued two tiles before it is staged: a fetch has two tiles of MFMA work
  // (~2 us at 8 waves) to land instead of one, which left the loop waiting on L2/HBM.
  bf16x8 kA[2], vA[2], kB[2], vB[2];
  auto fetch = [&](int kt, bf16x8 (&kr)[2], bf16x8 (&vr)[2]) {
    const size_t base = (size_t)btr[kt] * page_sz + head_off;
    const bf16x8* kp = reinterpret_cast<const bf16x8*>(kc + base);
    const bf16x8* vp = reinterpret_cast<const bf16x8*>(vc + base);
  // K: chunk c = key (c >> 4), dims 8 (c & 15)..+7 (row-major image, b128 stores).
  // V: chunk c = key (c & 63), dims 8 (c >> 6)..+7 -- the 64 lanes of a wave hold the 64
  // keys of ONE 8-dim column block, so each of the eight transposed b16 stores writes 128
  // contiguous bytes of one V^T row (bank-conflict free; with a lane per dim chunk instead
  // they hit 2 banks, 8-16 way conflicts that cost more than the tile's MFMAs).
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 512 * i;
      kr[i] = kp[c];
      vr[i] = vp[(c & 63) * (HD / 8) + (c >> 6)];
    }
  };
  auto stash = [&](int st, const bf16x8 (&kr)[2], const bf16x8 (&vr)[2]) {
    bf16* Ks = lds + st * (KS_ELEMS + VS_ELEMS);
    bf16* Vt = Ks + KS_ELEMS;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 512 * i;
      *reinterpret_cast<bf16x8*>(&Ks[(c >> 4) * KLD2 + (c & 15) * 8]) = kr[i];
      const int key = c & 63, d0 = (c >> 6) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(d0 + j) * VLD2 + key] = vr[i][j];
    }
  };
  auto tile = [&](int kt, int st) {
    const bf16* Ks = lds + st * (KS_ELEMS + VS_ELEMS);
    const bf16* Vt = Ks + KS_ELEMS;

    // ---- S^T = K . Q^T, two 32-key halves ----
    f32x16_t sc[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[kh][i] = 0.f;
      const bf16* kp = Ks + (32 * kh + krow) * KLD2 + 8 * hh;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        sc[kh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            *reinterpret_cast<const bf16x8*>(kp + 16 * s), qf[s], sc[kh], 0, 0, 0);
    }
    // ---- online softmax for this lane's query row (keys of reg rr: 16(rr>>3)+8hh+(rr&7)) ----
    // m is the running max of the RAW scores; p = exp2(s * c - m * c) is one FMA + exp.
    // Deferred rescale (cdna_hip_programming.md T13): O and l are rescaled only when some
    // row's max grew by more than RESCALE_THR (log2 units) -- wave-uniform decision, each
    // lane with its own factor -- so most tiles skip the 64-register multiply; the
    // unrescaled p stay <= 2^RESCALE_THR, exact in fp32 and safe in bf16.
    constexpr float RESCALE_THR = 8.f;
    const int k0 = kt * PAGE;
    // some key of the tile may be in the future (workgroup-uniform: a real branch, so the
    // mask's compares and selects run on diagonal tiles only)
    if (__builtin_amdgcn_readfirstlane(k0 + PAGE - 1 > T.pos0)) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int key = k0 + 32 * kh + 16 * (rr >> 3) + 8 * hh + (rr & 7);
          if (key > my_pos) sc[kh][rr] = -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) mx = fmaxf(mx, sc[kh][rr]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__any((mx - m) * scale_log2 > RESCALE_THR)) {
      const float mn = fmaxf(m, mx);
      const float alpha = exp2f((m - mn) * scale_log2);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
    const float mc = m * scale_log2;
    float ps = 0.f;
    bf16x8 pf[2][2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        // raw v_exp_f32 (arguments <= RESCALE_THR; underflow to 0 is what we want)
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[kh][rr], scale_log2, -mc));
        ps += p;
        pf[kh][rr >> 3][rr & 7] = f2bf(p);
      }
    l += ps;
    // ---- O^T += V^T . P^T ----
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const bf16* vp = Vt + (32 * db + r32) * VLD2 + 8 * hh;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              *reinterpret_cast<const bf16x8*>(vp + 32 * kh + 16 * s2), pf[kh][s2], o[db], 0, 0, 0);
    }
  };

  fetch(0, kA, vA);
  if (n_kt > 1) fetch(1, kB, vB);
  for (int kt = 0; kt < n_kt; kt += 2) {
    stash(0, kA, vA);
    __syncthreads();  // stage 0 complete; every wave is past tile kt-1 (WAR on stage 1)
    if (kt + 2 < n_kt) fetch(kt + 2, kA, vA);
    tile(kt, 0);
    if (kt + 1 >= n_kt) break;
    stash(1, kB, vB);
    __syncthreads();
    if (kt + 3 < n_kt) fetch(kt + 3, kB, vB);
    tile(kt + 1, 1);
  }

  l += __shfl_xor(l, 32, 64);
  if (t < T.n) {
    const float inv = 1.f / l;
    bf16* op = out + (size_t)row * ldo + h * HD + 4 * hh;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {  // regs 4g4..4g4+3 = d 32db + 8g4 + 4hh + 0..3
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = f2bf(o[db][4 * g4 + j] * inv);
        *reinterpret_cast<bf16x4*>(op + 32 * db + 8 * g4) = v;
      }
  }
}

template <int G>
int launch2(const bf16* q, int ldq, const bf16* kc, const bf16* vc, const int* bt, int bt_stride,
            const Tile* tiles, int n_tiles, int Hkv, float scale, bf16* out, int ldo,
            hipStream_t st) {
  const float sl2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(flash_prefill2_kernel<G>, dim3(n_tiles * Hkv), dim3(512), 0, st, q, ldq, kc,
                     vc, bt, bt_stride, tiles, n_tiles, Hkv, sl2, out, ldo);
  P2P_CHECK_LAUNCH();
}

}  // namespace

// v2 entry: tiles of at most 256 / (Hq/Hkv) tokens (p2p_flash_prefill_tile), otherwise as
// p2p_flash_prefill.  K/V pages must be whole 64-key pages of the block table.
P2P_API int p2p_flash_prefill_tile(int Hq, int Hkv) {
  if (Hkv <= 0 || Hq % Hkv) return 0;
  const int G = Hq / Hkv;
  return (G == 1 || G == 2 || G == 4 || G == 8) ? 256 / G : 0;
}

P2P_API int p2p_flash_prefill2(const void* q, int ldq, const void* kc, const void* vc,
                               const int* bt, int bt_stride, const int* tiles, int n_tiles,
                               int Hq, int Hkv, int head_dim, float scale, void* out, int ldo,
                               void* stream) {
  if (head_dim != HD || Hkv <= 0 || Hq % Hkv) return 1;
  if (n_tiles <= 0) return 0;
  auto Q = (const bf16*)q;
  auto K = (const bf16*)kc;
  auto V = (const bf16*)vc;
  auto T = (const Tile*)tiles;
  auto O = (bf16*)out;
  auto st = (hipStream_t)stream;
  switch (Hq / Hkv) {
    case 1: return launch2<1>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    case 2: return launch2<2>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    case 4: return launch2<4>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    case 8: return launch2<8>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    default: return 2;
  }
}

// tiles: int32 [n_tiles, 4] = (first row, n tokens <= 16, sequence, first position);
// n = 0 marks a padding tile (a captured prefill graph launches a fixed tile count);
// a tile's rows are consecutive positions of one sequence whose K/V (positions
// 0 .. pos0+n-1) are already in the paged cache.  head_dim must be 128.
P2P_API int p2p_flash_prefill(const void* q, int ldq, const void* kc, const void* vc,
                              const int* bt, int bt_stride, const int* tiles, int n_tiles,
                              int Hq, int Hkv, int head_dim, float scale, void* out, int ldo,
                              void* stream) {
  if (head_dim != HD || Hkv <= 0 || Hq % Hkv) return 1;
  if (n_tiles <= 0) return 0;
  auto Q = (const bf16*)q;
  auto K = (const bf16*)kc;
  auto V = (const bf16*)vc;
  auto T = (const Tile*)tiles;
  auto O = (bf16*)out;
  auto st = (hipStream_t)stream;
  switch (Hq / Hkv) {
    case 1: return launch<1>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    case 2: return launch<2>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    case 4: return launch<4>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    case 8: return launch<8>(Q, ldq, K, V, bt, bt_stride, T, n_tiles, Hkv, scale, O, ldo, st);
    default: return 2;
  }
}
