// Optimizer / gradient kernels over FLAT contiguous buffers (the native replacement of
// torch_xla's ZeroRedundancyOptimizer internals and of the reference's per-parameter Python
// loops: src/neuronx_distributed/utils/adamw_fp32_optim_params.py:91-155,
// src/neuronx_distributed/parallel_layers/grads.py:33-240).
//
// Parameters, fp32 master weights, Adam moments and gradients each live in ONE flat buffer
// (or one ZeRO-1 shard of it), so a whole optimizer step is a handful of launches regardless of
// the number of tensors:
//   * sumsq:  sum(x^2) (or max|x|) of a flat bf16/fp32 range -> fp32 partials -> one scalar
//             (the grad-norm; no per-tensor torch.norm launches);
//   * adamw:  fused decoupled-weight-decay Adam with bias correction, grad scaling (clip
//             coefficient read from device memory, so no host sync for clipping), fp32 master
//             update and bf16 copy-out of the model weights in the same pass.
#include "common.h"

namespace nxd {
namespace optim {

template <bool BF16>
__device__ __forceinline__ void ld4(const void* p, int64_t i, float* f) {
  if constexpr (BF16) {
    const u32x2_t v = *reinterpret_cast<const u32x2_t*>((const uint16_t*)p + i);
    f[0] = __uint_as_float(v[0] << 16);
    f[1] = __uint_as_float(v[0] & 0xffff0000u);
    f[2] = __uint_as_float(v[1] << 16);
    f[3] = __uint_as_float(v[1] & 0xffff0000u);
  } else {
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>((const float*)p + i);
    f[0] = v[0]; f[1] = v[1]; f[2] = v[2]; f[3] = v[3];
  }
}

template <bool BF16>
__device__ __forceinline__ float ld1(const void* p, int64_t i) {
  if constexpr (BF16) return bf2f(((const uint16_t*)p)[i]);
  else return ((const float*)p)[i];
}

// mode 0: sum of squares, mode 1: max |x|
template <bool BF16, int MODE>
__global__ void __launch_bounds__(256) partial_kernel(const void* __restrict__ x, int64_t n, float* __restrict__ part) {
  __shared__ float red[16];
  float acc = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float f[4];
    ld4<BF16>(x, i * 4, f);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = MODE == 0 ? acc + f[j] * f[j] : fmaxf(acc, fabsf(f[j]));
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) {
      const float f = ld1<BF16>(x, i);
      acc = MODE == 0 ? acc + f * f : fmaxf(acc, fabsf(f));
    }
  const float t = MODE == 0 ? block_sum(acc, red) : block_max(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <int MODE>
__global__ void __launch_bounds__(256) final_kernel(const float* __restrict__ part, int np, float* __restrict__ out, int accumulate) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) acc = MODE == 0 ? acc + part[i] : fmaxf(acc, part[i]);
  const float t = MODE == 0 ? block_sum(acc, red) : block_max(acc, red);
  if (threadIdx.x == 0) out[0] = accumulate ? (MODE == 0 ? out[0] + t : fmaxf(out[0], t)) : t;
}

struct AdamHyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2;  // bc = 1 - beta^t
  uint32_t sr_seed;                           // != 0: stochastic rounding of the bf16 copy-out
};

// Stochastic rounding fp32 -> bf16 (reference: NEURON_RT_STOCHASTIC_ROUNDING_EN for the bf16
// weights): add 16 uniform random bits below the bf16 mantissa, then truncate, so an update smaller
// than half a bf16 ulp still moves the weight with the right probability.  Counter-based hash of
// (seed, element index): no RNG state, identical on every replica of a parameter.
__device__ __forceinline__ uint32_t sr_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint16_t f2bf_sr(float f, uint32_t seed, int64_t idx) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return f2bf(f);   // inf / nan: round as usual
  const uint32_t r = sr_hash((uint32_t)idx * 0x9E3779B1u ^ (uint32_t)(idx >> 32) ^ seed) & 0xffffu;
  return (uint16_t)((u + r) >> 16);
}

// hyper (nullable): device [lr, 1 - beta1^t, 1 - beta2^t] overriding h.lr / h.bc1 / h.bc2, so a
// captured optimizer step (hipGraph) replays with the current step's values.
template <bool GBF16, bool HAS_OUT>
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const void* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, uint16_t* __restrict__ p16, int64_t n, AdamHyper h,
                                                    const float* __restrict__ gscale_ptr, float gscale_host,
                                                    const float* __restrict__ hyper) {
  if (hyper) {
    h.lr = hyper[0];
    h.bc1 = hyper[1];
    h.bc2 = hyper[2];
  }
  const float gs = gscale_ptr ? gscale_ptr[0] * gscale_host : gscale_host;
  const float step = h.lr / h.bc1;
  const float rbc2 = rsqrtf(h.bc2);
  const float decay = 1.f - h.lr * h.wd;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float gf[4];
    ld4<GBF16>(g, i * 4, gf);
    f32x4_t pv = *reinterpret_cast<f32x4_t*>(p + i * 4);
    f32x4_t mv = *reinterpret_cast<f32x4_t*>(m + i * 4);
    f32x4_t vv = *reinterpret_cast<f32x4_t*>(v + i * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gr = gf[j] * gs;
      mv[j] = h.beta1 * mv[j] + (1.f - h.beta1) * gr;
      vv[j] = h.beta2 * vv[j] + (1.f - h.beta2) * gr * gr;
      const float denom = sqrtf(vv[j]) * rbc2 + h.eps;
      pv[j] = pv[j] * decay - step * mv[j] / denom;
    }
    *reinterpret_cast<f32x4_t*>(p + i * 4) = pv;
    *reinterpret_cast<f32x4_t*>(m + i * 4) = mv;
    *reinterpret_cast<f32x4_t*>(v + i * 4) = vv;
    if constexpr (HAS_OUT) {
      u32x2_t o;
      if (h.sr_seed) {
        const int64_t e = i * 4;
        o[0] = (uint32_t)f2bf_sr(pv[0], h.sr_seed, e) | ((uint32_t)f2bf_sr(pv[1], h.sr_seed, e + 1) << 16);
        o[1] = (uint32_t)f2bf_sr(pv[2], h.sr_seed, e + 2) | ((uint32_t)f2bf_sr(pv[3], h.sr_seed, e + 3) << 16);
      } else {
        o[0] = pack2bf(pv[0], pv[1]);
        o[1] = pack2bf(pv[2], pv[3]);
      }
      *reinterpret_cast<u32x2_t*>(p16 + i * 4) = o;
    }
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) {
      const float gr = ld1<GBF16>(g, i) * gs;
      m[i] = h.beta1 * m[i] + (1.f - h.beta1) * gr;
      v[i] = h.beta2 * v[i] + (1.f - h.beta2) * gr * gr;
      p[i] = p[i] * decay - step * m[i] / (sqrtf(v[i]) * rbc2 + h.eps);
      if constexpr (HAS_OUT) p16[i] = h.sr_seed ? f2bf_sr(p[i], h.sr_seed, i) : f2bf(p[i]);
    }
}

// clip coefficient on device: coef = min(1, max_norm / (sqrt(sumsq) + 1e-6)) (or from max-norm)
__global__ void clip_coef_kernel(const float* __restrict__ stat, float* __restrict__ coef, float max_norm, int is_sumsq) {
  const float norm = is_sumsq ? sqrtf(stat[0]) : stat[0];
  const float c = max_norm / (norm + 1e-6f);
  coef[0] = c < 1.f ? c : 1.f;
  coef[1] = norm;
}

__global__ void __launch_bounds__(256) scale_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ s) {
  const float sc = s[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] *= sc;
}

}  // namespace optim

static inline int grid_for(int64_t n4) {
  int64_t g = (n4 + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

// out[0] = sum(x^2) (mode 0) or max|x| (mode 1); part must hold >= 2048 floats.
int flat_reduce_launch(const void* x, int is_bf16, int64_t n, int mode, float* part, float* out, int accumulate, hipStream_t stream) {
  using namespace optim;
  const int grid = grid_for(n / 4);
#define PK(B, M) hipLaunchKernelGGL((partial_kernel<B, M>), dim3(grid), dim3(256), 0, stream, x, n, part)
  if (is_bf16) { if (mode == 0) PK(true, 0); else PK(true, 1); }
  else { if (mode == 0) PK(false, 0); else PK(false, 1); }
#undef PK
  if (mode == 0) hipLaunchKernelGGL(final_kernel<0>, dim3(1), dim3(256), 0, stream, part, grid, out, accumulate);
  else hipLaunchKernelGGL(final_kernel<1>, dim3(1), dim3(256), 0, stream, part, grid, out, accumulate);
  return (int)hipGetLastError();
}

int adamw_flat_launch(float* p, const void* g, int g_is_bf16, float* m, float* v, void* p16, int64_t n, float lr, float beta1,
                      float beta2, float eps, float wd, float bc1, float bc2, const float* gscale_ptr, float gscale_host,
                      uint32_t sr_seed, const float* hyper, hipStream_t stream) {
  using namespace optim;
  if (n == 0) return 0;
  AdamHyper h{lr, beta1, beta2, eps, wd, bc1, bc2, sr_seed};
  const int grid = grid_for(n / 4);
#define AK(B, O) hipLaunchKernelGGL((adamw_kernel<B, O>), dim3(grid), dim3(256), 0, stream, p, g, m, v, (uint16_t*)p16, n, h, gscale_ptr, gscale_host, hyper)
  if (g_is_bf16) { if (p16) AK(true, true); else AK(true, false); }
  else { if (p16) AK(false, true); else AK(false, false); }
#undef AK
  return (int)hipGetLastError();
}

int clip_coef_launch(const float* stat, float* coef, float max_norm, int is_sumsq, hipStream_t stream) {
  hipLaunchKernelGGL(optim::clip_coef_kernel, dim3(1), dim3(1), 0, stream, stat, coef, max_norm, is_sumsq);
  return (int)hipGetLastError();
}

int scale_flat_launch(float* x, int64_t n, const float* s, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(optim::scale_kernel, dim3(grid_for(n)), dim3(256), 0, stream, x, n, s);
  return (int)hipGetLastError();
}

}  // namespace nxd
