// Inline-asm pieces of the LDS-DMA GEMM pipelines (wide_gemm.hip, prefill_gemm.h).
//
// Those kernels stage operands into LDS with global_load_lds (LDS DMA) several k-tiles
// ahead, wait with a COUNTED s_waitcnt vmcnt(N) + s_barrier, and read the landed tile with
// ds_read.  Written with the builtins, the compiler cannot tell which LDS bytes a pending
// DMA writes, and with DMA events pending it gives up on counting: it puts s_waitcnt
// vmcnt(0) before every ds_read (and every use of a register loaded after a DMA), so each
// k-tile waited for ALL loads in flight and the pipeline drained at every step (round-6
// disassembly of both kernels).  Issued as asm, these loads and reads are invisible to the
// compiler's wait insertion: the kernels' own counted waits are the only ones.
//
// Rules for a kernel using them:
//  * every load the k loop depends on is issued here (dma_lds / gload_nt) and waited for by
//    the kernel's own counted s_waitcnt vmcnt + s_barrier before its data is read;
//  * a register from gload_nt is consumed only by instructions that also consume a value
//    from lds_wait (issued after the chunk's wait), so it is never read in flight;
//  * the translation unit compiles with ZERO scratch: a spill would read an in-flight
//    register (p2p_llm_chat_go_amd/_build.py NO_SCRATCH refuses the build otherwise).
#pragma once

#include "common.h"

namespace ldsp {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ unsigned lds_off(const void* p) { return (unsigned)(uintptr_t)(lds_ptr_t)p; }

// 16 bytes of this lane from LDS (result valid after lds_wait)
__device__ __forceinline__ bf16x8 lds_rd(const bf16x8* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_off(p)));
  return v;
}

// wait for every outstanding LDS read; the empty asms re-define each fragment AFTER the wait,
// so nothing that uses them can be scheduled before it
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8 (&a)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i]));
}

// the same for two fragment arrays read together (one wait)
template <int N1, int N2>
__device__ __forceinline__ void lds_wait(bf16x8 (&a)[N1], bf16x8 (&b)[N2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N1; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int i = 0; i < N2; ++i) asm volatile("" : "+v"(b[i]));
}

// LDS DMA: lane i's BYTES (4 or 16) from g land at l + i * BYTES (l wave-uniform)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <int BYTES>
__device__ __forceinline__ void dma_lds(const void* g, const void* l) {
  static_assert(BYTES == 4 || BYTES == 16, "dma_lds: 4 or 16 bytes per lane");
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_off(l));
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// a streamed (non-temporal) 16-byte global load into registers, counted like the DMAs
__device__ __forceinline__ bf16x8 gload_nt(const bf16x8* p) {
  bf16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p));
  return v;
}

}  // namespace ldsp
