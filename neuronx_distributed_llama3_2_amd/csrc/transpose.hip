// bf16 matrix transpose dst[C][R] = src[R][C] through a 64x64 LDS tile (MI355X: HBM-bound).
//
// Used for the K-major weight copies of the dgrad GEMMs (ops/gemm.py: dX = dY W runs 10-20 %
// faster on hipBLASLt with W^T stored K-major, profiles/r2_gemm_layouts.jsonl) and the
// T-contiguous operands of the weight-gradient GEMMs.  256 threads per tile; every global access
// is a 16-byte vector (8 bf16) — the tile is read as 64 rows x 8 vectors and written as 64
// rows x 8 vectors of the transposed image; each 64-element LDS row is padded by 2 elements so the
// column gather of the store phase spreads over the banks.
#include "common.h"

#include <cstdlib>

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

// v2: the LDS tile is written with ds_write_b128 and read back TRANSPOSED by ds_read_b64_tr_b16
// (cdna_hip_programming.md T10): per 16-lane group a 4-row x 16-column block arrives column-major,
// two such reads give a lane 8 consecutive input rows of one input column = one 16-byte output
// vector.  The v1 kernel above moved every element through LDS as a 16-bit store and a 16-bit
// gather (16 + 16 LDS instructions per 16-byte vector) and ran at ~1.1 TB/s on 8192 x 4096
// (profiles/r2_gemm_layouts.jsonl transpose_x_ms 0.124).
// Image: 64 rows x 128 B, 16-byte chunk ch of row r stored at chunk ch ^ f(r), f(r) = (r & 2) | ((r >> 1) & 4):
// conflict-free for both the row-wise 128-bit writes and the transposed 64-bit reads (exhaustive
// search over XOR masks of the row bits with a bank model of both instructions).
typedef __attribute__((address_space(3))) short4_t lds_short4_t;

__device__ __forceinline__ int swz(int r) { return (r & 2) | ((r >> 1) & 4); }

__global__ void __launch_bounds__(256) transpose_tr_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                           int64_t R, int64_t C, int64_t ld_src, int64_t ld_dst) {
  __shared__ __attribute__((aligned(16))) char tile[T * 128];
  const int64_t r0 = (int64_t)blockIdx.y * T, c0 = (int64_t)blockIdx.x * T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i;
    const int row = v >> 3, ch = v & 7;
    const int64_t gr = r0 + row, gc = c0 + 8 * ch;
    u32x4_t x = {0, 0, 0, 0};
    if (gr < R && gc < C) x = *reinterpret_cast<const u32x4_t*>(src + gr * ld_src + gc);
    *reinterpret_cast<u32x4_t*>(tile + row * 128 + 16 * (ch ^ swz(row))) = x;
  }
  __syncthreads();
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = 16 * w + 4 * p;   // this lane's address column (its group's block row q)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int kb = 4 * s + g;       // 8-row block of the input = 16-byte chunk of the output row
    short4_t h[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int r = 8 * kb + 4 * hh + q;
      h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_short4_t*)(tile + r * 128 + 16 * ((col >> 3) ^ swz(r)) + 2 * (col & 7)));
    }
    const int64_t orow = c0 + 16 * w + i, ocol = r0 + 8 * kb;
    if (orow < C && ocol < R) {
      const short __attribute__((ext_vector_type(8))) o = {h[0][0], h[0][1], h[0][2], h[0][3],
                                                          h[1][0], h[1][1], h[1][2], h[1][3]};
      *reinterpret_cast<u32x4_t*>(dst + orow * ld_dst + ocol) = __builtin_bit_cast(u32x4_t, o);
    }
  }
}

static int g_v2 = -1;   // NXD_TRANSPOSE_TR (default 0); transpose_set_variant for in-process A/B

}  // namespace tr

void transpose_set_variant(int v2) { tr::g_v2 = v2 ? 1 : 0; }

// dst [C, R] (row stride ld_dst) = src [R, C] (row stride ld_src)^T; R, C, strides multiples of 8
int transpose_bf16_launch(const void* src, void* dst, int64_t R, int64_t C, int64_t ld_src, int64_t ld_dst,
                          hipStream_t stream) {
  if ((R % 8) || (C % 8) || (ld_src % 8) || (ld_dst % 8)) return -1;
  if (R == 0 || C == 0) return 0;
  const dim3 grid((unsigned)((C + tr::T - 1) / tr::T), (unsigned)((R + tr::T - 1) / tr::T));
  if (grid.y > 65535) return -2;
  if (tr::g_v2 < 0) {
    const char* e = getenv("NXD_TRANSPOSE_TR");
    tr::g_v2 = e ? (atoi(e) != 0) : 0;   // opt-in: 5.2 vs 5.7 TB/s at 8192 x 4096 (profiles/r5_transpose_tr_vs_lds16.jsonl)
  }
  if (tr::g_v2)
    hipLaunchKernelGGL(tr::transpose_tr_kernel, grid, dim3(256), 0, stream, (const uint16_t*)src, (uint16_t*)dst, R,
                       C, ld_src, ld_dst);
  else
    hipLaunchKernelGGL(tr::transpose_kernel, grid, dim3(256), 0, stream, (const uint16_t*)src, (uint16_t*)dst, R, C,
                       ld_src, ld_dst);
  return (int)hipGetLastError();
}

}  // namespace nxd
