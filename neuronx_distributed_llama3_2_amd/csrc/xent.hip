// Vocab-parallel cross-entropy for CDNA4.  Replaces the reference's `_ParallelCrossEntropy`
// (src/neuronx_distributed/parallel_layers/loss_functions.py:11-130) which runs three separate
// TP all-reduces (MAX, target logit, SUM exp) on fp64 logits (modeling_llama_nxd.py:731).
//
// Here one streaming pass per row computes the shard-local online-softmax statistics
//   stats[row] = {local max m, sum exp(x - m), target logit (0 if the label is not in this
//                 shard), sum x (for label smoothing)}
// so the TP combine is ONE all-gather of [N, 4] fp32 (instead of three all-reduces), and the
// backward writes softmax - onehot (optionally in place over the logits) in a second pass.
#include "common.h"

namespace nxd {
namespace xent {

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* f);
template <>
__device__ __forceinline__ void load8<uint16_t>(const uint16_t* p, float* f) {
  unpack8(*reinterpret_cast<const u32x4_t*>(p), f);
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p), b = *reinterpret_cast<const f32x4_t*>(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}

template <typename T>
__global__ void __launch_bounds__(256) stats_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                    float* __restrict__ stats, int64_t N, int V, int64_t ld,
                                                    int64_t vocab_start) {
  __shared__ float red_m[4], red_s[4], red_x[4];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  const int nvec = V / 8;
  for (int c = threadIdx.x; c < nvec; c += 256) {
    float f[8];
    load8<T>(x + c * 8, f);
    float lm = f[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, f[j]);
    const float nm = fmaxf(m, lm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc += __expf(f[j] - nm);
      sx += f[j];
    }
    s = s * __expf(m - nm) + acc;
    m = nm;
  }
  for (int c = nvec * 8 + threadIdx.x; c < V; c += 256) {  // tail (V % 8)
    float f;
    if constexpr (sizeof(T) == 2) f = bf2f(((const uint16_t*)x)[c]); else f = ((const float*)x)[c];
    const float nm = fmaxf(m, f);
    s = s * __expf(m - nm) + __expf(f - nm);
    m = nm;
    sx += f;
  }
  // wave combine of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
    sx += __shfl_xor(sx, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red_m[wid] = m; red_s[wid] = s; red_x[wid] = sx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red_m[0], S = red_s[0], X = red_x[0];
    for (int i = 1; i < 4; ++i) {
      const float nm = fmaxf(M, red_m[i]);
      S = (M == -INFINITY ? 0.f : S * __expf(M - nm)) + (red_m[i] == -INFINITY ? 0.f : red_s[i] * __expf(red_m[i] - nm));
      M = nm;
      X += red_x[i];
    }
    const int64_t lab = labels[row] - vocab_start;
    float tgt = 0.f;
    if (lab >= 0 && lab < V) {
      if constexpr (sizeof(T) == 2) tgt = bf2f(((const uint16_t*)x)[lab]); else tgt = ((const float*)x)[lab];
    }
    f32x4_t out = {M, S, tgt, X};
    *reinterpret_cast<f32x4_t*>(stats + row * 4) = out;
  }
}

// grad[row, j] = (exp(x - M) / S - (1-eps)[j == label] - eps / Vtot) * g[row]
// gstat[row] = {M, 1/S, g}, written by the host-side combine.
template <typename T>
__global__ void __launch_bounds__(256) bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                  const float* __restrict__ gstat, uint16_t* __restrict__ grad, int64_t N,
                                                  int V, int64_t ld, int64_t gld, int64_t vocab_start, float eps, float inv_vtot) {
  const int gx = gridDim.x / (unsigned)N;  // blocks per row
  const int64_t row = blockIdx.x / gx;
  const int bx = blockIdx.x % gx;
  const float M = gstat[row * 4], invS = gstat[row * 4 + 1], g = gstat[row * 4 + 2];
  const int64_t lab = labels[row] - vocab_start;
  const T* x = logits + row * ld;
  uint16_t* d = grad + row * gld;
  const int nvec = V / 8;
  for (int c = bx * 256 + threadIdx.x; c < nvec; c += gx * 256) {
    float f[8], o[8];
    load8<T>(x + c * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t col = (int64_t)c * 8 + j;
      float pv = __expf(f[j] - M) * invS - eps * inv_vtot;
      if (col == lab) pv -= (1.f - eps);
      o[j] = pv * g;
    }
    *reinterpret_cast<u32x4_t*>(d + c * 8) = pack8(o);
  }
  if (bx == 0) {
    for (int c = nvec * 8 + threadIdx.x; c < V; c += 256) {
      float f;
      if constexpr (sizeof(T) == 2) f = bf2f(((const uint16_t*)x)[c]); else f = ((const float*)x)[c];
      float pv = __expf(f - M) * invS - eps * inv_vtot;
      if (c == lab) pv -= (1.f - eps);
      d[c] = f2bf(pv * g);
    }
  }
}

}  // namespace xent

int xent_stats_launch(const void* logits, int is_fp32, const int64_t* labels, float* stats, int64_t N, int V, int64_t ld,
                      int64_t vocab_start, hipStream_t stream) {
  if (N == 0) return 0;
  if (is_fp32)
    hipLaunchKernelGGL(xent::stats_kernel<float>, dim3((unsigned)N), dim3(256), 0, stream, (const float*)logits, labels, stats, N, V, ld, vocab_start);
  else
    hipLaunchKernelGGL(xent::stats_kernel<uint16_t>, dim3((unsigned)N), dim3(256), 0, stream, (const uint16_t*)logits, labels, stats, N, V, ld, vocab_start);
  return (int)hipGetLastError();
}

int xent_bwd_launch(const void* logits, int is_fp32, const int64_t* labels, const float* gstat, void* grad, int64_t N, int V,
                    int64_t ld, int64_t gld, int64_t vocab_start, float eps, int64_t vocab_total, hipStream_t stream) {
  if (N == 0) return 0;
  const int nvec = V / 8;
  int gx = (nvec + 255) / 256;
  if (gx < 1) gx = 1;
  if (gx > 64) gx = 64;
  const dim3 grid((unsigned)(gx * N));
  const float inv_vtot = 1.f / (float)vocab_total;
  if (is_fp32)
    hipLaunchKernelGGL(xent::bwd_kernel<float>, grid, dim3(256), 0, stream, (const float*)logits, labels, gstat, (uint16_t*)grad, N, V, ld, gld, vocab_start, eps, inv_vtot);
  else
    hipLaunchKernelGGL(xent::bwd_kernel<uint16_t>, grid, dim3(256), 0, stream, (const uint16_t*)logits, labels, gstat, (uint16_t*)grad, N, V, ld, gld, vocab_start, eps, inv_vtot);
  return (int)hipGetLastError();
}

}  // namespace nxd
