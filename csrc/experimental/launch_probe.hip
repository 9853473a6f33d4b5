// Launch-shape probe (benchmarks only, bench/launch_shape_probe.py): what a dependent
// kernel boundary costs as a function of the workgroup shape (threads, LDS) and of a
// chain of dependent loads inside the kernel -- the decode attention kernel runs 8
// workgroups of 1024 threads with ~75 KB of LDS and its waves live ~1.65 us of a
// ~6.4 us launch (profiles/r2_decode_attention_pmc.json).
#include "common.h"

namespace {

template <int NT>
__global__ __launch_bounds__(NT) void launch_probe_kernel(const int* __restrict__ chain, int depth,
                                                          int start, float* __restrict__ out) {
  extern __shared__ int lds_dyn[];
  int idx = start;
  for (int i = 0; i < depth; ++i) idx = chain[idx];
  if (threadIdx.x == 0) lds_dyn[0] = idx;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)lds_dyn[0];
}

template <int NT>
int launch(int blocks, int lds, const int* chain, int depth, int start, float* out, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)launch_probe_kernel<NT>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(launch_probe_kernel<NT>, dim3(blocks), dim3(NT), max(lds, 4), st, chain, depth,
                     start, out);
  return (int)hipGetLastError();
}

}  // namespace

P2P_API int p2p_launch_probe(int blocks, int threads, int lds_bytes, const int* chain, int depth,
                             int start, float* out, hipStream_t stream) {
  if (blocks <= 0 || lds_bytes < 0 || lds_bytes > 160 * 1024) return (int)hipErrorInvalidValue;
  switch (threads) {
    case 64: return launch<64>(blocks, lds_bytes, chain, depth, start, out, stream);
    case 256: return launch<256>(blocks, lds_bytes, chain, depth, start, out, stream);
    case 512: return launch<512>(blocks, lds_bytes, chain, depth, start, out, stream);
    case 1024: return launch<1024>(blocks, lds_bytes, chain, depth, start, out, stream);
  }
  return (int)hipErrorInvalidValue;
}
