// bf16 matrix transpose dst[C][R] = src[R][C] through a 64x64 LDS tile (MI355X: HBM-bound).
//
// Used for the K-major weight copies of the dgrad GEMMs (ops/gemm.py: dX = dY W runs 10-20 %
// faster on hipBLASLt with W^T stored K-major, profiles/r2_gemm_layouts.jsonl) and the
// T-contiguous operands of the weight-gradient GEMMs.  256 threads per tile; every global access
// is a 16-byte vector (8 bf16) — the tile is read as 64 rows x 8 vectors and written as 64
// rows x 8 vectors of the transposed image; each 64-element LDS row is padded by 2 elements so the
// column gather of the store phase spreads over the banks.
#include "common.h"

namespace nxd {
namespace tr {

constexpr int T = 64;
constexpr int PAD = 2;   // elements of padding per LDS row

__global__ void __launch_bounds__(256) transpose_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                        int64_t R, int64_t C, int64_t lds_src, int64_t ld_dst) {
  __shared__ uint16_t tile[T][T + PAD];
  const int64_t r0 = (int64_t)blockIdx.y * T, c0 = (int64_t)blockIdx.x * T;
  const int tid = threadIdx.x;
  // load: 64 rows x 8 vectors = 512 vectors, 2 per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    const int row = v >> 3, cv = (v & 7) * 8;
    const int64_t gr = r0 + row, gc = c0 + cv;
    u32x4_t x = {0, 0, 0, 0};
    if (gr < R && gc < C) x = *reinterpret_cast<const u32x4_t*>(src + gr * lds_src + gc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[row][cv + 2 * j] = (uint16_t)(x[j] & 0xffffu);
      tile[row][cv + 2 * j + 1] = (uint16_t)(x[j] >> 16);
    }
  }
  __syncthreads();
  // store: output rows are input columns; 64 out-rows x 8 vectors
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    const int orow = v >> 3, ov = (v & 7) * 8;   // out row = input column c0+orow; out cols = input rows r0+ov..
    const int64_t gr = c0 + orow, gc = r0 + ov;
    if (gr < C && gc < R) {
      u32x4_t y;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        y[j] = (uint32_t)tile[ov + 2 * j][orow] | ((uint32_t)tile[ov + 2 * j + 1][orow] << 16);
      *reinterpret_cast<u32x4_t*>(dst + gr * ld_dst + gc) = y;
    }
  }
}

}  // namespace tr

// dst [C, R] (row stride ld_dst) = src [R, C] (row stride ld_src)^T; R, C, strides multiples of 8
int transpose_bf16_launch(const void* src, void* dst, int64_t R, int64_t C, int64_t ld_src, int64_t ld_dst,
                          hipStream_t stream) {
  if ((R % 8) || (C % 8) || (ld_src % 8) || (ld_dst % 8)) return -1;
  if (R == 0 || C == 0) return 0;
  const dim3 grid((unsigned)((C + tr::T - 1) / tr::T), (unsigned)((R + tr::T - 1) / tr::T));
  if (grid.y > 65535) return -2;
  hipLaunchKernelGGL(tr::transpose_kernel, grid, dim3(256), 0, stream, (const uint16_t*)src, (uint16_t*)dst, R, C,
                     ld_src, ld_dst);
  return (int)hipGetLastError();
}

}  // namespace nxd
