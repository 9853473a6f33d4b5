// Infinity-Cache (L3, 256 MiB) warm-up of a byte range: a streaming read whose values
// are discarded, so a later kernel that reads the same bytes is served on-die instead
// of from HBM.  Used on a side branch of the decode graph: while a latency-bound phase
// (paged attention, kernel boundaries) leaves HBM idle, the next weight matrix is
// pulled into L3 and the GEMV that consumes it streams from there.
#include "common.h"

namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// UNROLL 16-B loads in flight per lane; the xor keeps them live (the sink store is
// taken only if the folded value hits a 128-bit constant, i.e. never in practice).
template <int UNROLL>
__global__ __launch_bounds__(256) void l3_prefetch_kernel(const v4u* __restrict__ p, size_t n16,
                                                          v4u* __restrict__ sink) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  v4u acc = {0u, 0u, 0u, 0u};
  for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
    v4u v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u];
  }
  for (; i < n16; i += stride) acc ^= p[i];
  if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == 0xF39CC060u && acc.w == 0x5CEDC834u)
    sink[threadIdx.x] = acc;
}

}  // namespace

// bytes: rounded down to 16; grid 0 = one workgroup per CU (256).
P2P_API int p2p_l3_prefetch(const void* p, size_t bytes, int grid, void* sink, hipStream_t st) {
  if (!p || !sink || ((uintptr_t)p & 15)) return (int)hipErrorInvalidValue;
  const size_t n16 = bytes / 16;
  if (n16 == 0) return 0;
  if (grid <= 0) grid = 256;
  hipLaunchKernelGGL(l3_prefetch_kernel<8>, dim3(grid), dim3(256), 0, st, (const v4u*)p, n16,
                     (v4u*)sink);
  return (int)hipGetLastError();
}
