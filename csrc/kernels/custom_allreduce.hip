// One-shot collectives over IPC-mapped peer buffers (xGMI) for decode-size
// tensor-parallel messages (SURVEY.md §2C "Collective backend", §5 last row,
// kernel K12).  The reference has no collectives at all; this replaces RCCL's
// ring for the 2 x L per-token all-reduces of TP decode (16 KiB at B=1 for
// 70B), where a ring's 2(W-1) latency-bound hops dominate, and for the two
// small per-step exchanges of vocab-parallel sampling (greedy argmax keys:
// MAX of u64; sampled decode: all-gather of per-shard top-k candidates).
//
// Every rank owns one uncached (MTYPE UC) buffer, hipIpc-exported to the other
// ranks of the group:
//   flags : [2 parities][MAX_RANKS src][MAX_BLOCKS] u32   (one 4-byte word each)
//   data  : [2 parities][MAX_RANKS src][max_bytes]
// Call k (k = the group's call index, identical on every rank and every block:
// seq = k + 1, parity = seq & 1), block b, rank r:
//   1. push its slice of the input into slot [parity][r] of EVERY rank's buffer
//      (xGMI writes; all 7 links of a rank are used at once),
//   2. fence (system scope), then store seq into flag [parity][r][b] of every rank,
//   3. spin on its OWN flags [parity][*][b] until all ranks posted seq,
//   4. combine: h += sum in rank order (bit-identical on every rank) | max | gather.
// No grid barrier: block b only waits for block b of the peers.
//
// Slot reuse: a rank starts call k+2 only after its whole call-(k+1) kernel
// finished, i.e. after it saw a call-(k+1) flag of every peer; a peer posts
// call k+1 only after its call-k kernel completed (same stream).  So every peer
// is done reading parity k&1 before anyone rewrites it -- for ANY mapping of
// data to blocks, because seq is the call index on every block: block 0 keeps
// the counters of the blocks a small call does not launch in step
// (counters[nblk..MAX_BLOCKS) = seq), so a later call with more blocks still
// agrees on seq and parity.
//
// Every spin is bounded: on timeout the kernel sets the error word and finishes
// (wrong numbers, never a hung GPU).  Once the error word is set, later calls
// skip their waits (a dead peer costs one timeout, not one per call); the host
// raises on it (LlamaModel.check_faults).
#include <cstring>

#include "common.h"
#include "fused_ar.h"

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // one 16-byte lane payload

constexpr int MAX_RANKS = 8;
constexpr int MAX_BLOCKS = 64;
constexpr int NT = 256;
// two flag regions: A = one-shot flags and two-shot phase 1 (src -> owner), B = two-shot
// phase 2 (owner -> every rank)
constexpr size_t FLAG_REGION = 2ull * MAX_RANKS * MAX_BLOCKS * 4;
constexpr size_t FLAG_BYTES = 2 * FLAG_REGION;
// default spin bound in wall-clock ticks (100 MHz constant clock): 5 s; a healthy call
// waits microseconds (p2p_car_set_timeout_ms overrides, e.g. for fault-injection tests)
__device__ long long g_spin_ticks = 500000000ll;

enum { OP_ADD_BF16 = 0, OP_MAX_U64 = 1, OP_GATHER = 2 };

struct Peers {
  char* base[MAX_RANKS];  // every rank's buffer, mapped into this process
};

__device__ __forceinline__ unsigned* flag_ptr(char* base, int parity, int src, int blk) {
  return reinterpret_cast<unsigned*>(base) + ((size_t)parity * MAX_RANKS + src) * MAX_BLOCKS + blk;
}

__device__ __forceinline__ unsigned* flag2_ptr(char* base, int parity, int src, int blk) {
  return flag_ptr(base + FLAG_REGION, parity, src, blk);
}

// bounded wait until *f == seq (system-scope acquire polls, s_sleep between them)
__device__ __forceinline__ void wait_flag(unsigned* f, unsigned seq, int* err) {
  const long long t0 = wall_clock64();
  const long long bound = g_spin_ticks;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
    if (wall_clock64() - t0 > bound) {
      atomicOr(err, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ v4u* data_ptr(char* base, size_t max_bytes, int parity, int src) {
  return reinterpret_cast<v4u*>(base + FLAG_BYTES + ((size_t)parity * MAX_RANKS + src) * max_bytes);
}

template <int OP>
__global__ __launch_bounds__(NT) void car_kernel(Peers peers, int rank, int world, size_t max_bytes,
                                                 const v4u* __restrict__ in, void* __restrict__ out,
                                                 int n_vec, unsigned* __restrict__ counters,
                                                 int* __restrict__ err) {
  const int blk = blockIdx.x, nblk = gridDim.x;
  const int per = (n_vec + nblk - 1) / nblk;
  const int v0 = blk * per, v1 = min(n_vec, v0 + per);
  __shared__ unsigned s_seq;
  __shared__ int s_failed;
  if (threadIdx.x == 0) {
    s_seq = counters[blk] + 1;
    s_failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned seq = s_seq;
  const int parity = seq & 1;

  // 1. push this rank's slice to every rank (including itself)
  for (int i = v0 + threadIdx.x; i < v1; i += NT) {
    const v4u v = in[i];
    for (int p = 0; p < world; ++p) data_ptr(peers.base[p], max_bytes, parity, rank)[i] = v;
  }
  __threadfence_system();
  __syncthreads();
  // 2. post
  if (threadIdx.x < world)
    __hip_atomic_store(flag_ptr(peers.base[threadIdx.x], parity, rank, blk), seq,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every source rank's block `blk` (skipped once a peer is known dead)
  if (threadIdx.x < world && !s_failed) {
    unsigned* f = flag_ptr(peers.base[rank], parity, threadIdx.x, blk);
    const long long t0 = wall_clock64();
    const long long bound = g_spin_ticks;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      if (wall_clock64() - t0 > bound) {
        atomicOr(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // 4. combine
  if constexpr (OP == OP_ADD_BF16) {
    bf16x8* h = reinterpret_cast<bf16x8*>(out);
    for (int i = v0 + threadIdx.x; i < v1; i += NT) {
      float acc[8];
      const bf16x8 hv = h[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = (float)hv[j];
      for (int p = 0; p < world; ++p) {  // fixed rank order: identical sums on every rank
        const v4u raw = __builtin_nontemporal_load(data_ptr(peers.base[rank], max_bytes, parity, p) + i);
        bf16x8 v;
        memcpy(&v, &raw, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
      h[i] = o;
    }
  } else if constexpr (OP == OP_MAX_U64) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(out);
    for (int i = v0 + threadIdx.x; i < v1; i += NT) {
      unsigned long long a = 0, b = 0;
      for (int p = 0; p < world; ++p) {
        const v4u raw = __builtin_nontemporal_load(data_ptr(peers.base[rank], max_bytes, parity, p) + i);
        const unsigned long long x = ((unsigned long long)raw.y << 32) | raw.x;
        const unsigned long long y = ((unsigned long long)raw.w << 32) | raw.z;
        a = x > a ? x : a;
        b = y > b ? y : b;
      }
      o[2 * i] = a;
      o[2 * i + 1] = b;
    }
  } else {  // OP_GATHER: out[p * n_vec + i] = rank p's input[i]
    v4u* o = reinterpret_cast<v4u*>(out);
    for (int p = 0; p < world; ++p)
      for (int i = v0 + threadIdx.x; i < v1; i += NT)
        o[(size_t)p * n_vec + i] =
            __builtin_nontemporal_load(data_ptr(peers.base[rank], max_bytes, parity, p) + i);
  }
  if (threadIdx.x == 0) {
    counters[blk] = seq;
    if (blk == 0)
      for (int j = nblk; j < MAX_BLOCKS; ++j) counters[j] = seq;  // keep idle blocks in step
  }
}

// Two-shot sum (reduce-scatter + all-gather) for mid-size messages: rank s owns shard s
// of the vectors.  Per call, block b of rank r:
//   1. pushes its part of every shard s of `partial` to OWNER s only (slot [parity][r] of
//      s's buffer, at the shard's offsets) and posts flag A[parity][r][b] on s;
//   2. as owner of shard r: waits for flag A of every source, sums h + partials in rank
//      order (the one-shot formula, so both forms are bit-identical), and pushes the
//      result to every rank (slot [parity][r], shard r's offsets), posting flag B;
//   3. waits for flag B of every owner and copies the reduced shards into h.
// Each rank sends 2 (W-1)/W of the message over xGMI instead of the one-shot's (W-1),
// in two dependent hops instead of one.  Slot reuse follows the one-shot argument: a
// rank writes parity k&1 in call k+2 only after every peer posted a call-(k+1) flag.
__global__ __launch_bounds__(NT) void car2_kernel(Peers peers, int rank, int world,
                                                  size_t max_bytes, const v4u* __restrict__ in,
                                                  bf16x8* __restrict__ h, int n_vec,
                                                  unsigned* __restrict__ counters,
                                                  int* __restrict__ err) {
  const int blk = blockIdx.x, nblk = gridDim.x;
  const int ns = (n_vec + world - 1) / world;  // vectors per shard (the last may be short)
  const int per = (ns + nblk - 1) / nblk;      // this block's part of every shard
  __shared__ unsigned s_seq;
  __shared__ int s_failed;
  if (threadIdx.x == 0) {
    s_seq = counters[blk] + 1;
    s_failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned seq = s_seq;
  const int parity = seq & 1;
  auto range = [&](int s, int& a, int& b) {
    a = min(n_vec, s * ns + blk * per);
    b = min(min(n_vec, (s + 1) * ns), a + per);
  };
  // 1. scatter: my part of shard s -> owner s
  for (int s = 0; s < world; ++s) {
    int a, b;
    range(s, a, b);
    v4u* dst = data_ptr(peers.base[s], max_bytes, parity, rank);
    for (int i = a + threadIdx.x; i < b; i += NT) dst[i] = in[i];
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < world)
    __hip_atomic_store(flag_ptr(peers.base[threadIdx.x], parity, rank, blk), seq,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 2. reduce my shard, push the result to every rank
  if (threadIdx.x < world && !s_failed)
    wait_flag(flag_ptr(peers.base[rank], parity, threadIdx.x, blk), seq, err);
  __syncthreads();
  {
    int a, b;
    range(rank, a, b);
    for (int i = a + threadIdx.x; i < b; i += NT) {
      float acc[8];
      const bf16x8 hv = h[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = (float)hv[j];
      for (int p = 0; p < world; ++p) {  // fixed rank order (= the one-shot sum)
        const v4u raw = __builtin_nontemporal_load(data_ptr(peers.base[rank], max_bytes, parity, p) + i);
        bf16x8 v;
        memcpy(&v, &raw, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
      v4u ov;
      memcpy(&ov, &o, 16);
      for (int q = 0; q < world; ++q) data_ptr(peers.base[q], max_bytes, parity, rank)[i] = ov;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < world)
    __hip_atomic_store(flag2_ptr(peers.base[threadIdx.x], parity, rank, blk), seq,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. gather every owner's reduced shard into h
  if (threadIdx.x < world && !s_failed)
    wait_flag(flag2_ptr(peers.base[rank], parity, threadIdx.x, blk), seq, err);
  __syncthreads();
  for (int s = 0; s < world; ++s) {
    int a, b;
    range(s, a, b);
    const v4u* src = data_ptr(peers.base[rank], max_bytes, parity, s);
    for (int i = a + threadIdx.x; i < b; i += NT) {
      const v4u raw = __builtin_nontemporal_load(src + i);
      memcpy(&h[i], &raw, 16);
    }
  }
  if (threadIdx.x == 0) {
    counters[blk] = seq;
    if (blk == 0)
      for (int j = nblk; j < MAX_BLOCKS; ++j) counters[j] = seq;  // keep idle blocks in step
  }
}

int launch(int op, void* const* bases, int rank, int world, size_t max_bytes, const void* in,
           void* out, int n_vec, unsigned* counters, int* err, int blocks, void* stream) {
  if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world || n_vec <= 0) return 1;
  if ((size_t)n_vec * 16 > max_bytes) return 1;
  Peers peers = {};
  for (int p = 0; p < world; ++p) peers.base[p] = (char*)bases[p];
  if (blocks <= 0) blocks = (n_vec + NT * 2 - 1) / (NT * 2);
  blocks = max(1, min(blocks, MAX_BLOCKS));
  hipStream_t st = (hipStream_t)stream;
  switch (op) {
    case OP_ADD_BF16:
      hipLaunchKernelGGL(car_kernel<OP_ADD_BF16>, dim3(blocks), dim3(NT), 0, st, peers, rank,
                         world, max_bytes, (const v4u*)in, out, n_vec, counters, err);
      break;
    case OP_MAX_U64:
      hipLaunchKernelGGL(car_kernel<OP_MAX_U64>, dim3(blocks), dim3(NT), 0, st, peers, rank,
                         world, max_bytes, (const v4u*)in, out, n_vec, counters, err);
      break;
    case OP_GATHER:
      hipLaunchKernelGGL(car_kernel<OP_GATHER>, dim3(blocks), dim3(NT), 0, st, peers, rank,
                         world, max_bytes, (const v4u*)in, out, n_vec, counters, err);
      break;
    default:
      return 1;
  }
  P2P_CHECK_LAUNCH();
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

// Spin bound of every later call on the current device (ms > 0).
static long long g_host_spin_ticks = 500000000ll;  // = g_spin_ticks, for the fused epilogue

P2P_API int p2p_car_set_timeout_ms(int ms) {
  if (ms <= 0) return 1;
  const long long ticks = (long long)ms * 100000ll;  // 100 MHz constant clock
  g_host_spin_ticks = ticks;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_spin_ticks), &ticks, sizeof(ticks));
}

P2P_API long long p2p_car_spin_ticks() { return g_host_spin_ticks; }

// Bytes of one rank's fused-epilogue all-reduce buffer (fused_ar.h) for partials of up to
// max_bytes; allocate / export / map it with p2p_car_alloc / _get_handle / _open_handle.
P2P_API size_t p2p_far_buffer_bytes(size_t max_bytes) {
  return FAR_FLAG_BYTES + 2ull * FAR_MAX_RANKS * max_bytes;
}

// h[n] += sum over the group's ranks of partial[n] (bf16, n % 8 == 0,
// n * 2 <= max_bytes).  bases: world device pointers (this rank's own buffer at
// index rank).  counters: device u32 [64] (zeroed, private to this rank and
// buffer, shared by every op of the group); err: device int, set nonzero if a
// peer never arrived.
P2P_API int p2p_car_allreduce_add(void* const* bases, int rank, int world, size_t max_bytes,
                                  const void* partial, void* h, int n, unsigned* counters,
                                  int* err, int blocks, void* stream) {
  if (n % 8) return 1;
  return launch(OP_ADD_BF16, bases, rank, world, max_bytes, partial, h, n / 8, counters, err,
                blocks, stream);
}

// Two-shot form of p2p_car_allreduce_add (same contract and bit-identical result): for
// messages where pushing the whole partial to every peer costs more link time than a
// second hop (see parallel/custom_ar.py for the crossover).
P2P_API int p2p_car_allreduce_add_2shot(void* const* bases, int rank, int world, size_t max_bytes,
                                        const void* partial, void* h, int n, unsigned* counters,
                                        int* err, int blocks, void* stream) {
  if (n % 8 || world < 1 || world > MAX_RANKS || rank < 0 || rank >= world || n <= 0) return 1;
  const int n_vec = n / 8;
  if ((size_t)n_vec * 16 > max_bytes) return 1;
  Peers peers = {};
  for (int p = 0; p < world; ++p) peers.base[p] = (char*)bases[p];
  const int ns = (n_vec + world - 1) / world;
  if (blocks <= 0) blocks = (ns + NT * 2 - 1) / (NT * 2);
  blocks = max(1, min(blocks, MAX_BLOCKS));
  hipLaunchKernelGGL(car2_kernel, dim3(blocks), dim3(NT), 0, (hipStream_t)stream, peers, rank,
                     world, max_bytes, (const v4u*)partial, (bf16x8*)h, n_vec, counters, err);
  P2P_CHECK_LAUNCH();
}

// keys[n] = max over ranks of keys[n] (u64, n even, in place allowed).
P2P_API int p2p_car_allreduce_max_u64(void* const* bases, int rank, int world, size_t max_bytes,
                                      const void* keys_in, void* keys_out, int n,
                                      unsigned* counters, int* err, int blocks, void* stream) {
  if (n % 2) return 1;
  return launch(OP_MAX_U64, bases, rank, world, max_bytes, keys_in, keys_out, n / 2, counters,
                err, blocks, stream);
}

// out[world][nbytes] = every rank's in[nbytes] (nbytes % 16 == 0), rank-major.
P2P_API int p2p_car_all_gather(void* const* bases, int rank, int world, size_t max_bytes,
                               const void* in, void* out, long long nbytes, unsigned* counters,
                               int* err, int blocks, void* stream) {
  if (nbytes % 16) return 1;
  return launch(OP_GATHER, bases, rank, world, max_bytes, in, out, (int)(nbytes / 16), counters,
                err, blocks, stream);
}
