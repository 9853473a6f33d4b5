// Shared device helpers for the gfx950 (CDNA4) kernels of the in-process engine.
//
// Everything here is written for 64-lane wavefronts and the CDNA4 MFMA
// register layouts (see /opt/skills/guides/cdna_hip_programming.md §3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define P2P_API extern "C" __attribute__((visibility("default")))

static constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.0f;
  return z;
}

// acc + sum of squares of 8 bf16 values: four v_dot2c_f32_bf16 (the RMSNorm statistics
// ride in the GEMM k loops; 8 widen + 8 FMA per fragment made them VALU-heavy there)
__device__ __forceinline__ float sumsq8(const bf16x8& v, float acc) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const bf16x2 t = {v[2 * p], v[2 * p + 1]};
    acc = __builtin_amdgcn_fdot2_f32_bf16(t, t, acc, false);
  }
  return acc;
}

// x * sigmoid(x) with v_rcp_f32 (~1 ulp) instead of an IEEE division: the division
// sequence (div_scale / div_fmas / div_fixup, ~10 VALU) dominated the SwiGLU epilogue of
// the prefill GEMM (a 256x256 tile stores 128 outputs per thread)
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

// Non-temporal 16-byte load for once-read weight streams (decode GEMV).
__device__ __forceinline__ bf16x8 load_nt(const bf16x8* p) {
  return __builtin_nontemporal_load(p);
}

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2).
// Bijective remap so that logically consecutive blocks (which share operands)
// land on the same XCD: physical blocks b and b+8 get logical ids i and i+1.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = b % 8, idx = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

#define P2P_CHECK_LAUNCH() return (int)hipGetLastError()
