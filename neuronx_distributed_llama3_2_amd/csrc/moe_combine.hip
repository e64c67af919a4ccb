// Dropless-MoE token un-permute + affinity-weighted combine, and its backward
// (reference: the un-permute and `expert_affinities`-weighted sum of
// src/neuronx_distributed/modules/moe/expert_mlps.py:169-265).
//
//   ys   [M = T*k, H] expert outputs in expert-sorted row order (bf16)
//   inv  [T*k] int64: flat (token, choice) slot i sits at sorted row inv[i]
//   aff  [T, k] fp32 chosen affinities, or null for unit weights
//   fwd:  out[t, :] = sum_j aff[t, j] * ys[inv[t*k + j], :]
//   bwd:  dys[inv[t*k + j], :] = aff[t, j] * dout[t, :]      (inv is a permutation: plain stores)
//         daff[t, j] = <dout[t, :], ys[inv[t*k + j], :]>
//
// With aff = null the forward kernel is also the backward of the dispatch gather
// x_sorted = x[order // k]: dx[t] = sum_j dxs[inv[t*k + j]] -- a gather-sum, no atomics.
// Replaces an einsum that became a batch-T (1 x k) @ (k x H) batched GEMM (18 ms per Mixtral layer
// at 16k tokens, profiles/r2_moe_layer_v1.md) plus an atomic index_add in backward.
#include "common.h"

namespace nxd {
namespace moe {

constexpr int kMaxK = 8;

// grid (ceil(H / 2048), rows): 256 threads x 8 bf16 per row slice, rows strided by gridDim.y.
__global__ void __launch_bounds__(256) combine_fwd_kernel(const uint16_t* __restrict__ ys, const int64_t* __restrict__ inv,
                                                           const float* __restrict__ aff, uint16_t* __restrict__ out,
                                                           int64_t T, int k, int H) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= H) return;
  for (int64_t t = blockIdx.y; t < T; t += gridDim.y) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int64_t r = inv[t * k + j];
      const float w = aff ? aff[t * k + j] : 1.f;
      float v[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(ys + r * H + c), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(w, v[e], acc[e]);
    }
    *reinterpret_cast<u32x4_t*>(out + t * H + c) = pack8(acc);
  }
}

// One 256-thread block per token row (rows strided by gridDim.x).
__global__ void __launch_bounds__(256) combine_bwd_kernel(const uint16_t* __restrict__ dout, const uint16_t* __restrict__ ys,
                                                           const int64_t* __restrict__ inv, const float* __restrict__ aff,
                                                           uint16_t* __restrict__ dys, float* __restrict__ daff,
                                                           int64_t T, int k, int H) {
  __shared__ float red[4][kMaxK];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
    int64_t rows[kMaxK];
    float w[kMaxK], dot[kMaxK];
#pragma unroll
    for (int j = 0; j < kMaxK; ++j) {
      rows[j] = j < k ? inv[t * k + j] : 0;
      w[j] = j < k ? aff[t * k + j] : 0.f;
      dot[j] = 0.f;
    }
    for (int c = threadIdx.x * 8; c < H; c += 2048) {
      float d[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(dout + t * H + c), d);
#pragma unroll
      for (int j = 0; j < kMaxK; ++j) {
        if (j < k) {
          float y[8], g[8];
          unpack8(*reinterpret_cast<const u32x4_t*>(ys + rows[j] * H + c), y);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            dot[j] = fmaf(d[e], y[e], dot[j]);
            g[e] = w[j] * d[e];
          }
          *reinterpret_cast<u32x4_t*>(dys + rows[j] * H + c) = pack8(g);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kMaxK; ++j) {
      if (j < k) {
        const float s = wave_sum(dot[j]);
        if (lane == 0) red[wid][j] = s;
      }
    }
    __syncthreads();
    if (threadIdx.x < k) daff[t * k + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    __syncthreads();
  }
}

}  // namespace moe

int moe_combine_fwd_launch(const void* ys, const int64_t* inv, const float* aff, void* out, int64_t T, int k, int H,
                           hipStream_t stream) {
  if (H % 8 || k < 1 || k > moe::kMaxK) return -1;
  if (T == 0) return 0;
  const dim3 grid((unsigned)((H / 8 + 255) / 256), (unsigned)(T < 65535 ? T : 65535));
  hipLaunchKernelGGL(moe::combine_fwd_kernel, grid, dim3(256), 0, stream, (const uint16_t*)ys, inv, aff, (uint16_t*)out, T,
                     k, H);
  return (int)hipGetLastError();
}

int moe_combine_bwd_launch(const void* dout, const void* ys, const int64_t* inv, const float* aff, void* dys, float* daff,
                           int64_t T, int k, int H, hipStream_t stream) {
  if (H % 8 || k < 1 || k > moe::kMaxK) return -1;
  if (T == 0) return 0;
  const unsigned grid = (unsigned)(T < 1048576 ? T : 1048576);
  hipLaunchKernelGGL(moe::combine_bwd_kernel, dim3(grid), dim3(256), 0, stream, (const uint16_t*)dout, (const uint16_t*)ys,
                     inv, aff, (uint16_t*)dys, daff, T, k, H);
  return (int)hipGetLastError();
}

}  // namespace nxd
