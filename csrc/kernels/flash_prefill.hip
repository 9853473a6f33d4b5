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
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTH;
      if (c < CH) {
        kr[i] = kp[c];
        vr[i] = vp[c];
      }
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTH;
      if (c < CH) {
        const int key = c >> 4, d0 = (c & 15) * 8;
        *reinterpret_cast<bf16x8*>(&Ks[key * KLD + d0]) = kr[i];
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
    const float alpha = exp2f(m - mn);
    m = mn;
    bf16x8 pf;
    float ps = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = exp2f(s[mt][j] - mn);
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

}  // namespace

// tiles: int32 [n_tiles, 4] = (first row, n tokens <= 16, sequence, first position);
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
