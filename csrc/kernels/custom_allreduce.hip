// One-shot all-reduce over IPC-mapped peer buffers (xGMI) for decode-size
// tensor-parallel messages (SURVEY.md §2C "Collective backend", §5 last row,
// kernel K12).  The reference has no collectives at all; this replaces RCCL's
// ring for the 2 x L per-token all-reduces of TP decode (16 KiB at B=1 for
// 70B), where a ring's 2(W-1) latency-bound hops dominate.
//
// Every rank owns one uncached (MTYPE UC) buffer, hipIpc-exported to the other
// ranks of the group:
//   flags : [2 parities][MAX_RANKS src][MAX_BLOCKS] u32   (one 4-byte word each)
//   data  : [2 parities][MAX_RANKS src][max_bytes]
// Call k of block b on rank r (seq = per-block counter, parity = seq & 1):
//   1. push its chunk of `partial` into slot [parity][r] of EVERY rank's buffer
//      (xGMI writes; all 7 links of a rank are used at once),
//   2. fence (system scope), then store seq into flag [parity][r][b] of every rank,
//   3. spin on its OWN flags [parity][*][b] until all ranks posted seq,
//   4. h[chunk] += sum over ranks in rank order (bit-identical on every rank).
// No grid barrier: block b only waits for block b of the peers (same chunk).
// Parity double-buffering makes slot reuse safe: a rank can only start call
// k+2 after every peer posted call k+1, i.e. finished reading call k.
// Every spin is bounded: on timeout the kernel records an error and finishes
// (wrong numbers, never a hung GPU); the host checks the error word.
#include <cstring>

#include "common.h"

namespace {

constexpr int MAX_RANKS = 8;
constexpr int MAX_BLOCKS = 64;
constexpr int NT = 256;
constexpr size_t FLAG_BYTES = 2ull * MAX_RANKS * MAX_BLOCKS * 4;
// spin bound in wall-clock ticks (100 MHz constant clock): 5 s; a healthy call waits microseconds
constexpr long long SPIN_TICKS = 500000000ll;

struct Peers {
  char* base[MAX_RANKS];  // every rank's buffer, mapped into this process
};

__device__ __forceinline__ unsigned* flag_ptr(char* base, int parity, int src, int blk) {
  return reinterpret_cast<unsigned*>(base) + ((size_t)parity * MAX_RANKS + src) * MAX_BLOCKS + blk;
}

__device__ __forceinline__ bf16x8* data_ptr(char* base, size_t max_bytes, int parity, int src) {
  return reinterpret_cast<bf16x8*>(base + FLAG_BYTES + ((size_t)parity * MAX_RANKS + src) * max_bytes);
}

__global__ __launch_bounds__(NT) void car_allreduce_add_kernel(
    Peers peers, int rank, int world, size_t max_bytes, const bf16x8* __restrict__ partial,
    bf16x8* __restrict__ h, int n_vec, unsigned* __restrict__ counters, int* __restrict__ err) {
  const int blk = blockIdx.x, nblk = gridDim.x;
  const int per = (n_vec + nblk - 1) / nblk;
  const int v0 = blk * per, v1 = min(n_vec, v0 + per);
  __shared__ unsigned s_seq;
  if (threadIdx.x == 0) s_seq = counters[blk] + 1;
  __syncthreads();
  const unsigned seq = s_seq;
  const int parity = seq & 1;

  // 1. push this rank's chunk to every rank (including itself)
  for (int i = v0 + threadIdx.x; i < v1; i += NT) {
    const bf16x8 v = partial[i];
    for (int p = 0; p < world; ++p) data_ptr(peers.base[p], max_bytes, parity, rank)[i] = v;
  }
  __threadfence_system();
  __syncthreads();
  // 2. post
  if (threadIdx.x < world)
    __hip_atomic_store(flag_ptr(peers.base[threadIdx.x], parity, rank, blk), seq,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every source rank's block `blk`
  if (threadIdx.x < world) {
    unsigned* f = flag_ptr(peers.base[rank], parity, threadIdx.x, blk);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      if (wall_clock64() - t0 > SPIN_TICKS) {
        atomicOr(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // 4. reduce in fixed rank order
  for (int i = v0 + threadIdx.x; i < v1; i += NT) {
    float acc[8];
    const bf16x8 hv = h[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (float)hv[j];
    for (int p = 0; p < world; ++p) {
      const bf16x8 v = __builtin_nontemporal_load(data_ptr(peers.base[rank], max_bytes, parity, p) + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    h[i] = o;
  }
  if (threadIdx.x == 0) counters[blk] = seq;
}

}  // namespace

// Buffer bytes needed for messages of up to max_bytes (per rank).
P2P_API size_t p2p_car_buffer_bytes(size_t max_bytes) {
  return FLAG_BYTES + 2ull * MAX_RANKS * max_bytes;
}

// Allocate an uncached, zeroed buffer on the current device; returns hipError_t.
P2P_API int p2p_car_alloc(size_t bytes, void** out) {
  hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*out, 0, bytes);
}

P2P_API int p2p_car_free(void* p) { return (int)hipFree(p); }

// 64-byte IPC handle of a buffer from p2p_car_alloc.
P2P_API int p2p_car_get_handle(void* p, void* handle_out) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), p);
}

P2P_API int p2p_car_open_handle(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

P2P_API int p2p_car_close_handle(void* p) { return (int)hipIpcCloseMemHandle(p); }

P2P_API int p2p_car_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// h[n] += sum over the group's ranks of partial[n] (bf16, n % 8 == 0,
// n * 2 <= max_bytes).  bases: world device pointers (this rank's own buffer at
// index rank).  counters: device u32 [64] (zeroed, private to this rank and
// buffer); err: device int, set nonzero if a peer never arrived.
P2P_API int p2p_car_allreduce_add(void* const* bases, int rank, int world, size_t max_bytes,
                                  const void* partial, void* h, int n, unsigned* counters,
                                  int* err, int blocks, void* stream) {
  if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (n % 8 || (size_t)n * 2 > max_bytes) return 1;
  Peers peers = {};
  for (int p = 0; p < world; ++p) peers.base[p] = (char*)bases[p];
  const int n_vec = n / 8;
  if (blocks <= 0) blocks = (n_vec + NT * 2 - 1) / (NT * 2);
  blocks = max(1, min(blocks, MAX_BLOCKS));
  hipLaunchKernelGGL(car_allreduce_add_kernel, dim3(blocks), dim3(NT), 0, (hipStream_t)stream,
                     peers, rank, world, max_bytes, (const bf16x8*)partial, (bf16x8*)h, n_vec,
                     counters, err);
  P2P_CHECK_LAUNCH();
}
