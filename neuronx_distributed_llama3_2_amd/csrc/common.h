// Shared device helpers for the CDNA4 (gfx950 / MI355X) kernels of this package.
//
// Conventions used by every kernel TU in csrc/:
//   * wave = 64 lanes (hard-coded, never warpSize-derived);
//   * bf16 tensors travel as raw 16-bit storage (uint16_t) and are widened with a shift,
//     narrowed with the hardware round-to-nearest-even cast (v_cvt_pk_bf16_f32);
//   * all global loads/stores of bf16 are vectorised to 16 B per lane (8 elements);
//   * launchers take raw pointers + hipStream_t so they can be captured into hipGraphs
//     (no allocation, no synchronisation inside a launcher).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NXD_WAVE 64

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

namespace nxd {

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32 at -O3)
  return __builtin_bit_cast(uint16_t, b);
}

// Pack two floats into one dword of two bf16 (lo in bits 0..15).
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 8 bf16 <-> 8 floats through one 16-byte vector.
__device__ __forceinline__ void unpack8(const u32x4_t& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4_t pack8(const float* f) {
  u32x4_t v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack2bf(f[2 * i], f[2 * i + 1]);
  return v;
}

// acc + sum_i a[i] * b[i] over 8 bf16 pairs by 4 v_dot2c_f32_bf16 (products exact in f32, the bf16
// operands never widened in VGPRs): the decode GEMVs' inner product
// (The pairs are taken with __builtin_shufflevector from the bf16x8 view: bit-casting the extracted
// dword a[i] to bf16x2 made hipcc (ROCm 7.2) feed element 0's registers to all four instructions.)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot8_bf16(const u32x4_t& a, const u32x4_t& b, float acc) {
  const bf16x8_t av = __builtin_bit_cast(bf16x8_t, a), bv = __builtin_bit_cast(bf16x8_t, b);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 0, 1), __builtin_shufflevector(bv, bv, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 2, 3), __builtin_shufflevector(bv, bv, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 4, 5), __builtin_shufflevector(bv, bv, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 6, 7), __builtin_shufflevector(bv, bv, 6, 7), acc, false);
  return acc;
}

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

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024); `red` must hold 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md T1): consecutive
// logical ids land on the same XCD (blocks b and b+8 share an XCD under round-robin dispatch).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Attention-dropout keep mask: a counter hash of (seed, batch, global head, query, key), so nothing
// is stored and the backward regenerates the forward's mask.  Same definition as the host
// reference ops/attention_dropout.py:dropout_keep_mask (keep iff hash >= p * 2^32).
__host__ __device__ __forceinline__ uint32_t drop_hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  return x ^ (x >> 16);
}
__device__ __forceinline__ uint32_t drop_row_hash(uint32_t seed, int b, int head, int q) {
  const uint32_t x = drop_hash32(seed ^ ((uint32_t)b * 0x9E3779B1u) ^ ((uint32_t)head * 0x85EBCA6Bu));
  return drop_hash32(x ^ ((uint32_t)q * 0xC2B2AE35u));
}
__device__ __forceinline__ bool drop_keep(uint32_t row_hash, int key, uint32_t thresh) {
  return drop_hash32(row_hash ^ ((uint32_t)key * 0x27D4EB2Fu)) >= thresh;
}
struct DropoutArgs {
  uint32_t thresh = 0;      // keep iff hash >= thresh (= p * 2^32)
  float scale = 1.f;        // 1 / (1 - p)
  uint32_t seed = 0;
  int head_offset = 0;      // global index of local head 0 (tensor-parallel ranks draw the global masks)
  bool enabled() const { return thresh != 0; }
};

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace nxd
