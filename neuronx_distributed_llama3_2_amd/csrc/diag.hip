// Diagnostics kernels (not on any training path).
//
// cu_stream: a copy kernel of exactly `blocks` workgroups, each streaming its `bytes_per_block`
// region over and over until `ticks` of the 100 MHz real-time counter have passed -- a stand-in for RCCL's copy kernels (one workgroup per
// channel, HBM-streaming) that occupies a chosen number of CUs for a chosen time, used to measure
// how much a concurrent collective slows a GEMM on the compute stream (tools/bench_cu_interference.py).
#include "common.h"

namespace nxd {
namespace diag {

__global__ void __launch_bounds__(512) cu_stream_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst,
                                                        int64_t vec_per_block, int64_t ticks) {
  const int64_t base = (int64_t)blockIdx.x * vec_per_block;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int pass = 0; pass < (1 << 20); ++pass) {
    // wave-uniform exit (every wave of the block reads the same counter value's decision)
    const uint64_t now = __builtin_amdgcn_readfirstlane((uint32_t)(__builtin_amdgcn_s_memrealtime() - t0));
    if ((int64_t)now > ticks) break;
    for (int64_t i = threadIdx.x; i < vec_per_block; i += blockDim.x) {
      u32x4_t v = src[base + i];
      v[0] += (uint32_t)pass;   // keep each pass's loads live
      dst[base + i] = v;
    }
  }
}

}  // namespace diag

int cu_stream_launch(const void* src, void* dst, int64_t bytes_per_block, int blocks, int64_t ticks, hipStream_t stream) {
  if (blocks <= 0 || ticks <= 0 || ticks > 1000000000 || bytes_per_block < 16 || bytes_per_block % 16) return -1;
  hipLaunchKernelGGL(diag::cu_stream_kernel, dim3(blocks), dim3(512), 0, stream, (const u32x4_t*)src, (u32x4_t*)dst,
                     bytes_per_block / 16, ticks);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace nxd
