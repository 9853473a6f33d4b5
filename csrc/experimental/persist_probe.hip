// Feasibility probe for a persistent batch-1 decode layer (bench/persist_probe.py):
// does one launch per layer -- phases separated by grid barriers, each workgroup
// pulling the first <= 128 KiB of its NEXT phase's weight slice into LDS by LDS-DMA
// before it arrives at the barrier -- stream a layer's bytes faster than one launch per
// phase?  Pure data movement with the decode layer's shapes (qkv, attention stand-in,
// o_proj, gate_up, down); no math, nothing is handed between workgroups.  Every spin
// is bounded (error word, never a hang).
#include "common.h"

namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int NT = 512;
constexpr int NPH = 5;
constexpr int LDS_V = 8192;  // 128 KiB of 16-byte vectors
constexpr long long SPIN = 20000000;  // 200 ms at 100 MHz

struct Phases {
  const v4u* w[NPH];
  long long n16[NPH];  // 0 = the attention stand-in (busy loop on 8 workgroups)
};

__device__ __forceinline__ void slice(long long n, int b, int nb, long long& s0, long long& s1) {
  const long long per = (n + nb - 1) / nb;
  s0 = min(n, (long long)b * per);
  s1 = min(n, s0 + per);
}

// two register batches of 8 loads: batch B is issued before batch A is folded, so a
// wave always has 8-16 KiB in flight (the skinny GEMV's pipelining)
__device__ __forceinline__ v4u stream(const v4u* __restrict__ w, long long a, long long e) {
  v4u acc = {0u, 0u, 0u, 0u};
  long long i = a + threadIdx.x;
  v4u A[8], B[8];
  auto ld = [&](v4u (&r)[8], long long j) {
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = __builtin_nontemporal_load(w + j + u * NT);
  };
  if (i + 7 * NT < e) {
    ld(A, i);
    i += 8 * NT;
    for (; i + 7 * NT < e; i += 8 * NT) {
      ld(B, i);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= A[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) A[u] = B[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= A[u];
  }
  for (; i < e; i += NT) acc ^= __builtin_nontemporal_load(w + i);
  return acc;
}

__device__ __forceinline__ v4u busy(int iters) {
  v4u acc = {1u, 2u, 3u, 4u};
  for (int k = 0; k < iters; ++k) acc = acc * 1664525u + 1013904223u;
  return acc;
}

// Two-level barrier (the guide's barrier-xcd): workgroups of one XCD (blockIdx % 8 under
// round-robin dispatch; placement only affects speed) arrive on their group's counter, the
// group's last arriver on the top counter, the top's last arriver bumps the generation
// word every workgroup polls.  bar: [0..7] group counters, [8] top, [9] generation.
__device__ __forceinline__ void grid_barrier(unsigned* bar, int nb, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    const unsigned g = __hip_atomic_load(&bar[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int grp = blockIdx.x & 7;
    const int in_grp = (nb - grp + 7) / 8;  // workgroups with this blockIdx % 8
    const int n_grp = nb < 8 ? nb : 8;
    bool last = false;
    const unsigned t = __hip_atomic_fetch_add(&bar[grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)in_grp - 1) {
      (void)__hip_atomic_exchange(&bar[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned tt = __hip_atomic_fetch_add(&bar[8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = tt == (unsigned)n_grp - 1;
    }
    if (last) {
      (void)__hip_atomic_exchange(&bar[8], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&bar[9], g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (!failed) {  // after a timeout every later barrier falls through
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(&bar[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (wall_clock64() - t0 > SPIN) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void persist_kernel(Phases ph, int layers, int pf_v, int attn_iters,
                                                     unsigned* bar, int* err, v4u* sink) {
  __shared__ __attribute__((aligned(16))) v4u lds[LDS_V];
  const int b = blockIdx.x, nb = gridDim.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  v4u acc = {0u, 0u, 0u, 0u};
  int have = 0;  // vectors of the current phase already in LDS
  for (int l = 0; l < layers; ++l) {
    for (int p = 0; p < NPH; ++p) {
      if (ph.n16[p] == 0) {
        if (b < 8) acc ^= busy(attn_iters);
      } else {
        long long s0, s1;
        slice(ph.n16[p], b, nb, s0, s1);
        if (have) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          for (int i = threadIdx.x; i < have; i += NT) acc ^= lds[i];
        }
        acc ^= stream(ph.w[p], s0 + have, s1);
      }
      // prefetch the first pf_v vectors of this workgroup's next-phase slice into LDS
      const int np = p + 1 < NPH ? p + 1 : 0;
      have = 0;
      if (pf_v > 0 && ph.n16[np] > 0) {
        long long t0, t1;
        slice(ph.n16[np], b, nb, t0, t1);
        const int n = (int)min((long long)pf_v, t1 - t0) & ~(NT - 1);  // whole wave blocks
        __syncthreads();  // every wave is done reading the previous LDS contents
        for (int i = w * 64; i < n; i += NT)
          __builtin_amdgcn_global_load_lds((const void*)(ph.w[np] + t0 + i + lane),
                                           (lds_ptr_t)(lds + i), 16, 0, 0);
        have = n;
      }
      grid_barrier(bar, nb, err);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(NT) void phase_kernel(const v4u* __restrict__ w, long long n16,
                                                   int attn_iters, v4u* sink) {
  v4u acc;
  if (n16 == 0) {
    acc = busy(attn_iters);
  } else {
    long long s0, s1;
    slice(n16, blockIdx.x, gridDim.x, s0, s1);
    acc = stream(w, s0, s1);
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc;
}

}  // namespace

// mode 0: one launch per phase (attention stand-in: 8 workgroups), mode 1: one persistent
// launch for all layers with grid barriers, prefetching pf_bytes of the next phase.
P2P_API int p2p_persist_probe(int mode, const void* const* w, const long long* bytes, int layers,
                              int grid, int pf_bytes, int attn_iters, unsigned* bar, int* err,
                              void* sink, hipStream_t st) {
  Phases ph;
  for (int p = 0; p < NPH; ++p) {
    ph.w[p] = (const v4u*)w[p];
    ph.n16[p] = bytes[p] / 16;
  }
  if (mode == 0) {
    for (int l = 0; l < layers; ++l)
      for (int p = 0; p < NPH; ++p)
        hipLaunchKernelGGL(phase_kernel, dim3(ph.n16[p] ? grid : 8), dim3(NT), 0, st, ph.w[p],
                           ph.n16[p], attn_iters, (v4u*)sink);
    return (int)hipGetLastError();
  }
  const int pf_v = min(pf_bytes / 16, LDS_V);
  hipLaunchKernelGGL(persist_kernel, dim3(grid), dim3(NT), 0, st, ph, layers, pf_v, attn_iters,
                     bar, err, (v4u*)sink);
  return (int)hipGetLastError();
}
