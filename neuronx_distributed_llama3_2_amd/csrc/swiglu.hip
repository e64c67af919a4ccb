// SwiGLU activation of a fused gate_up projection (reference: LlamaMLP with
// `gate_up_proj` ColumnParallelLinear(stride=2), examples/training/llama/modeling_llama_nxd.py:183-211).
//
//   gu: [N, 2I] with gate = gu[:, :I], up = gu[:, I:]   (the per-TP-shard layout of stride=2)
//   fwd: h = silu(g) * u
//   bwd: dg = dh * u * s * (1 + g (1 - s)),  du = dh * silu(g)        (s = sigmoid(g))
// Pure streaming: 16-byte vectors, fp32 math, one row slice per thread and row stride in y.
#include "common.h"

namespace nxd {
namespace swiglu {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// 2-D grid: x covers the I/8 column vectors of a row, y strides over rows — no 64-bit div/mod
// in the address math (the former flat grid-stride loop spent more issue slots on the int64
// index division than on the data and reached only ~3.4 TB/s).
__global__ void __launch_bounds__(256) fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ h, int64_t N, int I) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= I) return;
  for (int64_t row = blockIdx.y; row < N; row += gridDim.y) {
    const uint16_t* src = gu + row * 2 * I + c;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(src), g);
    unpack8(*reinterpret_cast<const u32x4_t*>(src + I), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigm(g[j]) * u[j];
    *reinterpret_cast<u32x4_t*>(h + row * I + c) = pack8(o);
  }
}

__global__ void __launch_bounds__(256) bwd_kernel(const uint16_t* __restrict__ gu, const uint16_t* __restrict__ dh,
                                                  uint16_t* __restrict__ dgu, int64_t N, int I) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= I) return;
  for (int64_t row = blockIdx.y; row < N; row += gridDim.y) {
    const uint16_t* src = gu + row * 2 * I + c;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(src), g);
    unpack8(*reinterpret_cast<const u32x4_t*>(src + I), u);
    unpack8(*reinterpret_cast<const u32x4_t*>(dh + row * I + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigm(g[j]);
      du[j] = d[j] * g[j] * s;
      dg[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
    }
    uint16_t* dst = dgu + row * 2 * I + c;
    *reinterpret_cast<u32x4_t*>(dst) = pack8(dg);
    *reinterpret_cast<u32x4_t*>(dst + I) = pack8(du);
  }
}

// Backward with a second, transposed copy of d(gate_up) for the weight gradient: the gate_up
// wgrad runs as a TN GEMM on T-contiguous operands, which otherwise costs a separate transpose of
// the [T, 2I] gradient (read + write of the largest activation gradient of the layer).  Each
// workgroup owns a 64-row x 64-column tile of the gate and up halves: the row-major result is
// written straight from registers, the transposed one goes through LDS and leaves as 16-byte
// vectors of 8 consecutive rows (tokens).  N % 64 == 0 and I % 64 == 0 (checked by the launcher).
constexpr int TT = 64;         // tile columns (of each half)
constexpr int LDT = TT + 8;   // LDS row stride (elements): 16-B aligned rows, offset banks

// TR = tile rows (tokens): 128 gives 256-B contiguous runs per transposed row, 64 covers N % 128 != 0
template <int TR>
__global__ void __launch_bounds__(256) bwd_dual_kernel(const uint16_t* __restrict__ gu, const uint16_t* __restrict__ dh,
                                                       uint16_t* __restrict__ dgu, uint16_t* __restrict__ dgu_t, int64_t N,
                                                       int I) {
  __shared__ __attribute__((aligned(16))) uint16_t sdg[TR * LDT];
  __shared__ __attribute__((aligned(16))) uint16_t sdu[TR * LDT];
  constexpr int NV = TR * TT / 8 / 256;   // 16-B vectors per thread per phase
  const int tid = threadIdx.x;
  const int col0 = blockIdx.x * TT;
  const int64_t row0 = (int64_t)blockIdx.y * TR;
#pragma unroll
  for (int it = 0; it < NV; ++it) {
    const int v = tid + 256 * it, r = v >> 3, c = (v & 7) * 8;
    const int64_t row = row0 + r;
    const uint16_t* src = gu + row * 2 * I + col0 + c;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(src), g);
    unpack8(*reinterpret_cast<const u32x4_t*>(src + I), u);
    unpack8(*reinterpret_cast<const u32x4_t*>(dh + row * I + col0 + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigm(g[j]);
      du[j] = d[j] * g[j] * s;
      dg[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
    }
    const u32x4_t pg = pack8(dg), pu = pack8(du);
    uint16_t* dst = dgu + row * 2 * I + col0 + c;
    *reinterpret_cast<u32x4_t*>(dst) = pg;
    *reinterpret_cast<u32x4_t*>(dst + I) = pu;
    *reinterpret_cast<u32x4_t*>(sdg + r * LDT + c) = pg;
    *reinterpret_cast<u32x4_t*>(sdu + r * LDT + c) = pu;
  }
  __syncthreads();
  constexpr int RV = TR / 8;   // 8-token vectors per transposed row
#pragma unroll
  for (int it = 0; it < NV; ++it) {
    const int v = tid + 256 * it, c = v / RV, r = (v % RV) * 8;   // column c, tokens r .. r + 7
    uint32_t wg[4], wu[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wg[j] = (uint32_t)sdg[(r + 2 * j) * LDT + c] | ((uint32_t)sdg[(r + 2 * j + 1) * LDT + c] << 16);
      wu[j] = (uint32_t)sdu[(r + 2 * j) * LDT + c] | ((uint32_t)sdu[(r + 2 * j + 1) * LDT + c] << 16);
    }
    *reinterpret_cast<u32x4_t*>(dgu_t + (int64_t)(col0 + c) * N + row0 + r) = u32x4_t{wg[0], wg[1], wg[2], wg[3]};
    *reinterpret_cast<u32x4_t*>(dgu_t + (int64_t)(I + col0 + c) * N + row0 + r) = u32x4_t{wu[0], wu[1], wu[2], wu[3]};
  }
}

// Forward with a second, transposed copy of h ([I, N], token-contiguous): the down projection's
// weight gradient (TN GEMM) reads it instead of transposing the saved activation in backward.
template <int TR>
__global__ void __launch_bounds__(256) fwd_dual_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ h,
                                                       uint16_t* __restrict__ h_t, int64_t N, int I) {
  __shared__ __attribute__((aligned(16))) uint16_t sh[TR * LDT];
  constexpr int NV = TR * TT / 8 / 256;
  const int tid = threadIdx.x;
  const int col0 = blockIdx.x * TT;
  const int64_t row0 = (int64_t)blockIdx.y * TR;
#pragma unroll
  for (int it = 0; it < NV; ++it) {
    const int v = tid + 256 * it, r = v >> 3, c = (v & 7) * 8;
    const int64_t row = row0 + r;
    const uint16_t* src = gu + row * 2 * I + col0 + c;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(src), g);
    unpack8(*reinterpret_cast<const u32x4_t*>(src + I), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigm(g[j]) * u[j];
    const u32x4_t po = pack8(o);
    *reinterpret_cast<u32x4_t*>(h + row * I + col0 + c) = po;
    *reinterpret_cast<u32x4_t*>(sh + r * LDT + c) = po;
  }
  __syncthreads();
  constexpr int RV = TR / 8;
#pragma unroll
  for (int it = 0; it < NV; ++it) {
    const int v = tid + 256 * it, c = v / RV, r = (v % RV) * 8;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)sh[(r + 2 * j) * LDT + c] | ((uint32_t)sh[(r + 2 * j + 1) * LDT + c] << 16);
    *reinterpret_cast<u32x4_t*>(h_t + (int64_t)(col0 + c) * N + row0 + r) = u32x4_t{w[0], w[1], w[2], w[3]};
  }
}

}  // namespace swiglu

static inline dim3 row_grid(int64_t N, int I) {
  const unsigned gx = (unsigned)((I / 8 + 255) / 256);
  const unsigned gy = (unsigned)(N < 32768 ? N : 32768);
  return dim3(gx, gy);
}

int swiglu_fwd_launch(const void* gu, void* h, int64_t N, int I, hipStream_t stream) {
  if (I % 8) return -1;
  const int64_t nv = N * (I / 8);
  if (nv == 0) return 0;
  hipLaunchKernelGGL(swiglu::fwd_kernel, row_grid(N, I), dim3(256), 0, stream, (const uint16_t*)gu, (uint16_t*)h, N, I);
  return (int)hipGetLastError();
}

int swiglu_bwd_launch(const void* gu, const void* dh, void* dgu, int64_t N, int I, hipStream_t stream) {
  if (I % 8) return -1;
  const int64_t nv = N * (I / 8);
  if (nv == 0) return 0;
  hipLaunchKernelGGL(swiglu::bwd_kernel, row_grid(N, I), dim3(256), 0, stream, (const uint16_t*)gu, (const uint16_t*)dh,
                     (uint16_t*)dgu, N, I);
  return (int)hipGetLastError();
}

// h [N, I] and h_t [I, N] in one pass; -1 if the shape is not tiled.
int swiglu_fwd_dual_launch(const void* gu, void* h, void* h_t, int64_t N, int I, hipStream_t stream) {
  if (I % swiglu::TT || N % 64 || N / 64 > 65535) return -1;
  if (N == 0) return 0;
  static const int rows_knob = [] { const char* e = getenv("NXD_SWIGLU_DUAL_ROWS"); return e ? atoi(e) : 64; }();
  const bool big = rows_knob == 128 && N % 128 == 0;
  const dim3 grid((unsigned)(I / swiglu::TT), (unsigned)(N / (big ? 128 : 64)));
  if (big)
    hipLaunchKernelGGL(swiglu::fwd_dual_kernel<128>, grid, dim3(256), 0, stream, (const uint16_t*)gu, (uint16_t*)h,
                       (uint16_t*)h_t, N, I);
  else
    hipLaunchKernelGGL(swiglu::fwd_dual_kernel<64>, grid, dim3(256), 0, stream, (const uint16_t*)gu, (uint16_t*)h,
                       (uint16_t*)h_t, N, I);
  return (int)hipGetLastError();
}

// dgu [N, 2I] row-major and dgu_t [2I, N] (its transpose) in one pass; -1 if the shape is not tiled.
int swiglu_bwd_dual_launch(const void* gu, const void* dh, void* dgu, void* dgu_t, int64_t N, int I, hipStream_t stream) {
  if (I % swiglu::TT || N % 64 || N / 64 > 65535) return -1;
  if (N == 0) return 0;
  // 64-row tiles measured faster than 128 (379 vs 387-397 us at T=8192, I=14336; 34.6 vs 39.5 at the
  // TP=8 shard, profiles/r2_swiglu_dual_kernel_ab.jsonl); NXD_SWIGLU_DUAL_ROWS=128 selects the other; read once
  static const int rows_knob = [] { const char* e = getenv("NXD_SWIGLU_DUAL_ROWS"); return e ? atoi(e) : 64; }();
  const bool big = rows_knob == 128 && N % 128 == 0;
  const dim3 grid((unsigned)(I / swiglu::TT), (unsigned)(N / (big ? 128 : 64)));
  if (big)
    hipLaunchKernelGGL(swiglu::bwd_dual_kernel<128>, grid, dim3(256), 0, stream, (const uint16_t*)gu, (const uint16_t*)dh,
                       (uint16_t*)dgu, (uint16_t*)dgu_t, N, I);
  else
    hipLaunchKernelGGL(swiglu::bwd_dual_kernel<64>, grid, dim3(256), 0, stream, (const uint16_t*)gu, (const uint16_t*)dh,
                       (uint16_t*)dgu, (uint16_t*)dgu_t, N, I);
  return (int)hipGetLastError();
}

}  // namespace nxd
