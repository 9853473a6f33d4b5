// Expert-parallel all-to-all over IPC-mapped peer buffers (xGMI), for decode-size MoE
// layers in the DP-attention + EP layout (models/moe.py a2a mode; BASELINE config 5,
// Mixtral EP=8 runs 2 all-to-alls per layer, dispatch + combine).
//
// RCCL's all_to_all_single with a static per-destination capacity moves W x R·K rows per
// rank (at W = 8 that wire is 8x padding) and, being a host-driven collective, was never
// captured in the decode hipGraph.  Here every exchange is a kernel on the compute stream:
//
//   ep_dispatch (W x NB blocks): block (d, j) picks this rank's slots routed to rank d's
//       experts (a ballot prefix over the slot list, deterministic order), writes those
//       token rows + (local expert, weight) straight into rank d's receive region (xGMI
//       stores), fences, and posts ONE 64-bit flag {seq, count} per (source, block) on d.
//       Only routed rows travel; no padding on the wire.
//   ep_recv (W blocks): block s waits for source s's flags, copies its rows into a local
//       (cached) [W][C][H] buffer and marks the unused capacity as padding (expert -1),
//       so a2a_group + the grouped expert GEMMs run on it unchanged.
//   ep_return (W x NB blocks): the owner pushes every expert output row back to the
//       source's return region at the row the source chose, then posts {seq}.
//   ep_combine (R blocks): block r waits for the owners of its K slots and adds the K
//       returned rows (fp32 sum in k order, one rounding) into the residual h.
//
// Sequencing (one call = dispatch, recv, return, combine; every rank makes the same calls
// in the same order): seq = state[0] + 1, parity = seq & 1 selects one of two copies of
// every region.  The last combine block (arrival ticket state[1]) advances state[0], so
// every kernel of the next call reads the next seq.  A rank writes a peer's parity-p
// region for call k+2 only after its own call k+1 combine saw that peer's call k+1
// return, which the peer posted after its call k+1 recv -- i.e. after it finished reading
// the call-k data: two copies suffice.  Every spin is bounded (5 s default); a timeout
// sets the error word, later calls skip their waits, and the host raises
// (LlamaModel.check_faults).  No counters live in the peers' memory, only flags.
#include <cstring>

#include "common.h"

namespace {

typedef unsigned long long u64;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr int EP_MAX_RANKS = 8;
constexpr int EP_MAX_NB = 4;    // blocks per (source, destination) pair
constexpr int EP_MAX_SLOTS = 4096;
constexpr int NT = 256;
constexpr size_t EP_FLAG_BYTES = 4096;

__device__ long long g_ep_spin_ticks = 500000000ll;  // 5 s at the 100 MHz wall clock

struct EpPeers {
  char* base[EP_MAX_RANKS];
};

struct EpLayout {
  size_t cmax, H;
  // flags: disp [2][src][NB] u64 | ret [2][owner][NB] u64
  __device__ u64* disp_flag(char* b, int par, int src, int j) const {
    return reinterpret_cast<u64*>(b) + ((size_t)par * EP_MAX_RANKS + src) * EP_MAX_NB + j;
  }
  __device__ u64* ret_flag(char* b, int par, int owner, int j) const {
    return reinterpret_cast<u64*>(b) + 2 * EP_MAX_RANKS * EP_MAX_NB +
           ((size_t)par * EP_MAX_RANKS + owner) * EP_MAX_NB + j;
  }
  __device__ size_t region() const { return 2ull * EP_MAX_RANKS * cmax * H * 2; }
  // dispatch rows [2][src][cmax][H] bf16, then their meta [2][src][cmax] int2
  __device__ bf16* disp_x(char* b, int par, int src) const {
    return reinterpret_cast<bf16*>(b + EP_FLAG_BYTES) + (((size_t)par * EP_MAX_RANKS + src) * cmax) * H;
  }
  __device__ int2* disp_meta(char* b, int par, int src) const {
    return reinterpret_cast<int2*>(b + EP_FLAG_BYTES + 2 * region()) +
           ((size_t)par * EP_MAX_RANKS + src) * cmax;
  }
  // returned rows [2][owner][cmax][H] bf16
  __device__ bf16* ret_x(char* b, int par, int owner) const {
    return reinterpret_cast<bf16*>(b + EP_FLAG_BYTES + region()) +
           (((size_t)par * EP_MAX_RANKS + owner) * cmax) * H;
  }
};

__device__ __forceinline__ bool wait_seq(u64* f, unsigned seq, int* err, u64* got) {
  const long long t0 = wall_clock64();
  const long long bound = g_ep_spin_ticks;
  while (true) {
    const u64 v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((unsigned)(v >> 32) == seq) {
      *got = v;
      return true;
    }
    if (wall_clock64() - t0 > bound) {
      atomicOr(err, 1);
      *got = 0;
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// copy one H-wide bf16 row with the whole block (16-byte chunks)
__device__ __forceinline__ void copy_row(bf16* dst, const bf16* src, int H) {
  const v4u* s = reinterpret_cast<const v4u*>(src);
  v4u* d = reinterpret_cast<v4u*>(dst);
  for (int c = threadIdx.x; c < H / 8; c += NT) d[c] = s[c];
}

__global__ __launch_bounds__(NT) void ep_dispatch_kernel(
    EpPeers peers, EpLayout L, int rank, const bf16* __restrict__ h, int ldh, int n_slots, int K,
    int El, const int* __restrict__ topk_ids, const float* __restrict__ topk_w, int NB,
    int* __restrict__ send_map, const unsigned* __restrict__ state) {
  const int d = blockIdx.x / NB, j = blockIdx.x % NB;
  const unsigned seq = state[0] + 1;
  const int par = seq & 1;
  __shared__ short s_pos[EP_MAX_SLOTS];
  __shared__ int s_cnt;
  // deterministic per-destination positions: ballot prefix over the slot list (wave 0)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int base = 0;
    for (int s0 = 0; s0 < n_slots; s0 += 64) {
      const int s = s0 + lane;
      const bool mine = s < n_slots && topk_ids[s] / El == d;
      const u64 m = __ballot(mine);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      if (s < n_slots) s_pos[s] = mine ? (short)(base + before) : (short)-1;
      base += __popcll(m);
    }
    if (lane == 0) s_cnt = base;
  }
  __syncthreads();
  char* peer = peers.base[d];
  bf16* dx = L.disp_x(peer, par, rank);
  int2* dm = L.disp_meta(peer, par, rank);
  for (int s = 0; s < n_slots; ++s) {
    const int p = s_pos[s];
    if (p < 0 || p % NB != j) continue;
    copy_row(dx + (size_t)p * L.H, h + (size_t)(s / K) * ldh, (int)L.H);
    if (threadIdx.x == 0) {
      dm[p] = make_int2(topk_ids[s] % El, __float_as_int(topk_w[s]));
      send_map[s] = (d << 16) | p;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(L.disp_flag(peer, par, rank, j), ((u64)seq << 32) | (unsigned)s_cnt,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(NT) void ep_recv_kernel(
    EpPeers peers, EpLayout L, int rank, int C, int NB, bf16* __restrict__ recv_x,
    int* __restrict__ recv_meta, float* __restrict__ recv_w, int* __restrict__ recv_cnt,
    const unsigned* __restrict__ state, int* __restrict__ err) {
  const int src = blockIdx.x;
  const unsigned seq = state[0] + 1;
  const int par = seq & 1;
  char* own = peers.base[rank];
  __shared__ int s_cnt;
  __shared__ int s_bad;
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_bad = 0;
  }
  __syncthreads();
  const bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (threadIdx.x < NB) {
    u64 v = 0;
    if (!failed && wait_seq(L.disp_flag(own, par, src, threadIdx.x), seq, err, &v)) {
      if (threadIdx.x == 0) s_cnt = (int)(unsigned)v;
    } else {
      s_bad = 1;
    }
  }
  __syncthreads();
  const int cnt = (s_bad || s_cnt > C) ? 0 : s_cnt;
  const bf16* sx = L.disp_x(own, par, src);
  const int2* sm = L.disp_meta(own, par, src);
  for (int p = 0; p < cnt; ++p) copy_row(recv_x + ((size_t)src * C + p) * L.H, sx + (size_t)p * L.H, (int)L.H);
  for (int p = threadIdx.x; p < C; p += NT) {
    int2 m = p < cnt ? sm[p] : make_int2(-1, 0);
    recv_meta[2 * ((size_t)src * C + p)] = m.x;
    recv_meta[2 * ((size_t)src * C + p) + 1] = m.y;
    recv_w[(size_t)src * C + p] = __int_as_float(m.y);
  }
  if (threadIdx.x == 0) recv_cnt[src] = cnt;
}

__global__ __launch_bounds__(NT) void ep_return_kernel(
    EpPeers peers, EpLayout L, int rank, int C, int NB, const bf16* __restrict__ o,
    const int* __restrict__ recv_cnt, const unsigned* __restrict__ state) {
  const int src = blockIdx.x / NB, j = blockIdx.x % NB;
  const unsigned seq = state[0] + 1;
  const int par = seq & 1;
  char* peer = peers.base[src];
  bf16* rx = L.ret_x(peer, par, rank);
  const int cnt = recv_cnt[src];
  for (int p = j; p < cnt; p += NB) copy_row(rx + (size_t)p * L.H, o + ((size_t)src * C + p) * L.H, (int)L.H);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(L.ret_flag(peer, par, rank, j), (u64)seq << 32, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(NT) void ep_combine_kernel(
    EpPeers peers, EpLayout L, int rank, int K, int NB, const int* __restrict__ send_map,
    bf16* __restrict__ h, int ldh, unsigned* __restrict__ state, int* __restrict__ err) {
  const int r = blockIdx.x;
  const unsigned seq = state[0] + 1;
  const int par = seq & 1;
  char* own = peers.base[rank];
  const bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (threadIdx.x < K && !failed) {
    const int sm = send_map[r * K + threadIdx.x];
    u64 v;
    wait_seq(L.ret_flag(own, par, sm >> 16, (sm & 0xffff) % NB), seq, err, &v);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < (int)L.H / 8; c += NT) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const int sm = send_map[r * K + k];
      const v4u raw = __builtin_nontemporal_load(
          reinterpret_cast<const v4u*>(L.ret_x(own, par, sm >> 16) + (size_t)(sm & 0xffff) * L.H) + c);
      bf16x8 v;
      memcpy(&v, &raw, 16);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += (float)v[q];
    }
    bf16x8* dst = reinterpret_cast<bf16x8*>(h + (size_t)r * ldh) + c;
    const bf16x8 hv = *dst;
    bf16x8 res;
#pragma unroll
    for (int q = 0; q < 8; ++q) res[q] = f2bf((float)hv[q] + acc[q]);
    *dst = res;
  }
  // the last block to finish advances the call sequence (every block read it already)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (atomicAdd(&state[1], 1u) == gridDim.x - 1) {
      state[1] = 0;
      __hip_atomic_store(&state[0], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

bool peers_from(void* const* bases, int world, EpPeers* p) {
  if (world < 1 || world > EP_MAX_RANKS) return false;
  *p = {};
  for (int r = 0; r < world; ++r) p->base[r] = (char*)bases[r];
  return true;
}

}  // namespace

// Bytes of one rank's EP exchange buffer for up to `cmax` slot rows per (source,
// destination) pair of `H` bf16 (allocate / export / map with p2p_car_alloc & co.).
P2P_API size_t p2p_ep_buffer_bytes(int cmax, int H) {
  const size_t region = 2ull * EP_MAX_RANKS * (size_t)cmax * H * 2;
  return EP_FLAG_BYTES + 2 * region + 2ull * EP_MAX_RANKS * cmax * sizeof(int2);
}

P2P_API int p2p_ep_set_timeout_ms(int ms) {
  long long t = (long long)ms * 100000ll;  // 100 MHz wall clock
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ep_spin_ticks), &t, sizeof(t));
}

// Dispatch of this rank's R*K slots (topk_ids / topk_w from moe_route): rows go to the
// owners' receive regions; send_map[s] = owner << 16 | row (for ep_combine).
// state: this rank's device u32 [2] (zeroed once); nb: blocks per destination (1..4).
P2P_API int p2p_ep_dispatch(void* const* bases, int rank, int world, int cmax, int H,
                            const void* h, int ldh, int R, int K, int El, const int* topk_ids,
                            const float* topk_w, int* send_map, unsigned* state, int nb,
                            void* stream) {
  EpPeers P;
  const int n = R * K;
  if (!peers_from(bases, world, &P) || rank < 0 || rank >= world || n <= 0 || n > cmax ||
      n > EP_MAX_SLOTS || H % 8 || El <= 0 || nb < 1 || nb > EP_MAX_NB || cmax > 65535)
    return (int)hipErrorInvalidValue;
  EpLayout L{(size_t)cmax, (size_t)H};
  hipLaunchKernelGGL(ep_dispatch_kernel, dim3(world * nb), dim3(NT), 0, (hipStream_t)stream, P, L,
                     rank, (const bf16*)h, ldh, n, K, El, topk_ids, topk_w, nb, send_map, state);
  P2P_CHECK_LAUNCH();
}

// Receive: recv_x [world * C, H] bf16, recv_meta [world * C, 2] int (expert -1 = padding),
// recv_w [world * C] f32, recv_cnt [world] int (rows per source); C = R * K of the call.
P2P_API int p2p_ep_recv(void* const* bases, int rank, int world, int cmax, int H, int C,
                        void* recv_x, int* recv_meta, float* recv_w, int* recv_cnt,
                        const unsigned* state, int* err, int nb, void* stream) {
  EpPeers P;
  if (!peers_from(bases, world, &P) || C <= 0 || C > cmax || H % 8 || nb < 1 || nb > EP_MAX_NB)
    return (int)hipErrorInvalidValue;
  EpLayout L{(size_t)cmax, (size_t)H};
  hipLaunchKernelGGL(ep_recv_kernel, dim3(world), dim3(NT), 0, (hipStream_t)stream, P, L, rank, C,
                     nb, (bf16*)recv_x, recv_meta, recv_w, recv_cnt, state, err);
  P2P_CHECK_LAUNCH();
}

// Return the expert outputs o [world * C, H] (row src * C + p answers source src's row p).
P2P_API int p2p_ep_return(void* const* bases, int rank, int world, int cmax, int H, int C,
                          const void* o, const int* recv_cnt, const unsigned* state, int nb,
                          void* stream) {
  EpPeers P;
  if (!peers_from(bases, world, &P) || C <= 0 || C > cmax || H % 8 || nb < 1 || nb > EP_MAX_NB)
    return (int)hipErrorInvalidValue;
  EpLayout L{(size_t)cmax, (size_t)H};
  hipLaunchKernelGGL(ep_return_kernel, dim3(world * nb), dim3(NT), 0, (hipStream_t)stream, P, L,
                     rank, C, nb, (const bf16*)o, recv_cnt, state);
  P2P_CHECK_LAUNCH();
}

// Combine: h[r] += sum_k returned row of slot r * K + k; ends the call (advances state).
P2P_API int p2p_ep_combine(void* const* bases, int rank, int world, int cmax, int H, int R, int K,
                           const int* send_map, void* h, int ldh, unsigned* state, int* err,
                           int nb, void* stream) {
  EpPeers P;
  if (!peers_from(bases, world, &P) || R <= 0 || K <= 0 || K > NT || H % 8 || nb < 1 ||
      nb > EP_MAX_NB)
    return (int)hipErrorInvalidValue;
  EpLayout L{(size_t)cmax, (size_t)H};
  hipLaunchKernelGGL(ep_combine_kernel, dim3(R), dim3(NT), 0, (hipStream_t)stream, P, L, rank, K,
                     nb, send_map, (bf16*)h, ldh, state, err);
  P2P_CHECK_LAUNCH();
}
