// Inference kernels for the decode (token-generation / speculation) path on CDNA4.
// Reference behaviour: examples/inference/modules/attention/attention_base.py:141-170 (decode
// attention split into prior-cache and active parts), model_base.py:388-422 (KV-cache scatter,
// continuous batching by seq_ids), src/neuronx_distributed/utils/sampling.py:27-77 (argmax /
// top-k multinomial sampling custom calls).
//
//  * decode attention = flash-decoding: grid (batch x kv-head x key-split) so even batch 1
//    fills the chip; every workgroup serves all G = Hq/Hkv query heads x T new tokens of its kv
//    head (GQA-native: each K/V byte is read once per step), writes (m, l, o) partials, and a
//    combine kernel merges the splits.  All shapes are static for a given max cache length and
//    the valid length is read from device memory, so the step is hipGraph-capturable.
//  * KV-cache write is an in-place scatter into the persistent [B, Hkv, Lmax, D] cache.
//  * sampling: block argmax; top-k by an exact 4-pass 8-bit radix select on order-preserving
//    32-bit keys (no full sort of the 128k vocabulary), then softmax / CDF / uniform draw over
//    the k survivors in LDS.
#include "common.h"

namespace nxd {
namespace dec {

constexpr int kChunk = 128;

struct DecodeParams {
  const uint16_t* q;
  int64_t q_sb, q_st, q_sh;
  const uint16_t* kc;
  const uint16_t* vc;
  int64_t c_sb, c_sh, c_sl;  // cache strides (batch, head, position); d contiguous
  const int* cache_idx;      // [B] cache row per batch entry (nullable: identity)
  const int* seq_len;        // [B] valid keys for the LAST new token
  float* po;                 // [B, Hkv, nsplit, M, D]
  float* pm;                 // [B, Hkv, nsplit, M]
  float* pl;
  int B, T, Hq, Hkv, nsplit;
  float scale;
};

template <int D>
__global__ void __launch_bounds__(256) partial_kernel(DecodeParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = p.Hq / p.Hkv;
  const int M = G * p.T;
  float* qs = reinterpret_cast<float*>(smem);  // [M][D]
  float* ss = qs + M * D;                      // [M][kChunk]

  const int split = blockIdx.x % p.nsplit;
  const int bh = blockIdx.x / p.nsplit;
  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int cb = p.cache_idx ? p.cache_idx[b] : b;
  const int slen = p.seq_len[b];
  const int k0 = split * kChunk;
  const int64_t pbase = ((int64_t)bh * p.nsplit + split) * M;

  if (k0 >= slen) {  // nothing valid in this split
    for (int m = threadIdx.x; m < M; m += 256) {
      p.pm[pbase + m] = -INFINITY;
      p.pl[pbase + m] = 0.f;
    }
    return;
  }
  // q rows m = tt * G + gg -> head hkv*G + gg, token tt
  for (int i = threadIdx.x; i < M * (D / 8); i += 256) {
    const int m = i / (D / 8), c = i % (D / 8);
    const int tt = m / G, gg = m % G;
    const uint16_t* src = p.q + (int64_t)b * p.q_sb + (int64_t)tt * p.q_st + (int64_t)(hkv * G + gg) * p.q_sh + c * 8;
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(src), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) qs[m * D + c * 8 + j] = f[j] * p.scale;
  }
  __syncthreads();
  const uint16_t* kbase = p.kc + (int64_t)cb * p.c_sb + (int64_t)hkv * p.c_sh;
  const uint16_t* vbase = p.vc + (int64_t)cb * p.c_sb + (int64_t)hkv * p.c_sh;
  {
    const int kk = threadIdx.x & (kChunk - 1);
    const int rp = threadIdx.x >> 7;
    const int key = k0 + kk;
    float kr[D];
    if (key < slen) {
#pragma unroll
      for (int c = 0; c < D / 8; ++c) unpack8(*reinterpret_cast<const u32x4_t*>(kbase + (int64_t)key * p.c_sl + c * 8), kr + c * 8);
    }
    for (int m = rp; m < M; m += 2) {
      const int tt = m / G;
      const int lim = slen - (p.T - 1 - tt);  // causal among the new tokens
      float s = -INFINITY;
      if (key < lim) {
        s = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) s += qs[m * D + d] * kr[d];
      }
      ss[m * kChunk + kk] = s;
    }
  }
  __syncthreads();
  {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int m = wid; m < M; m += 4) {
      const float a = ss[m * kChunk + lane], c = ss[m * kChunk + 64 + lane];
      const float mx = wave_max(fmaxf(a, c));
      const float mu = mx == -INFINITY ? 0.f : mx;
      const float ea = __expf(a - mu), ec = __expf(c - mu);
      ss[m * kChunk + lane] = ea;
      ss[m * kChunk + 64 + lane] = ec;
      const float sum = wave_sum(ea + ec);
      if (lane == 0) {
        p.pm[pbase + m] = mx;
        p.pl[pbase + m] = sum;
      }
    }
  }
  __syncthreads();
  const int nk = min(kChunk, slen - k0);
  for (int i = threadIdx.x; i < M * (D / 8); i += 256) {
    const int m = i / (D / 8), c = i % (D / 8);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int kk = 0; kk < nk; ++kk) {
      const float pv = ss[m * kChunk + kk];
      float vf[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(vbase + (int64_t)(k0 + kk) * p.c_sl + c * 8), vf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += pv * vf[j];
    }
    float* dst = p.po + (pbase + m) * D + c * 8;
    *reinterpret_cast<f32x4_t*>(dst) = f32x4_t{acc[0], acc[1], acc[2], acc[3]};
    *reinterpret_cast<f32x4_t*>(dst + 4) = f32x4_t{acc[4], acc[5], acc[6], acc[7]};
  }
}

// one workgroup of D threads per (b, hkv, m) row
__global__ void combine_kernel(const float* __restrict__ po, const float* __restrict__ pm, const float* __restrict__ pl,
                               uint16_t* __restrict__ out, int64_t o_sb, int64_t o_st, int64_t o_sh, int Hq, int Hkv,
                               int T, int nsplit, int D) {
  const int G = Hq / Hkv, M = G * T;
  const int row = blockIdx.x;  // (b*Hkv + hkv)*M + m
  const int m = row % M;
  const int bh = row / M;
  const int b = bh / Hkv, hkv = bh % Hkv;
  const int tt = m / G, gg = m % G;
  const int64_t base = (int64_t)bh * nsplit * M + m;
  float mx = -INFINITY;
  for (int s = 0; s < nsplit; ++s) mx = fmaxf(mx, pm[base + (int64_t)s * M]);
  float l = 0.f;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    l = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      const float ms = pm[base + (int64_t)s * M];
      if (ms == -INFINITY) continue;
      const float wgt = __expf(ms - mx);
      l += wgt * pl[base + (int64_t)s * M];
      acc += wgt * po[(base + (int64_t)s * M) * D + d];
    }
    const float o = l > 0.f ? acc / l : 0.f;
    out[(int64_t)b * o_sb + (int64_t)tt * o_st + (int64_t)(hkv * G + gg) * o_sh + d] = f2bf(o);
  }
}

// cache[cb, h, pos[b] + t, :] = new[b, t, h, :]
__global__ void __launch_bounds__(256) kv_write_kernel(const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
                                                       int64_t n_sb, int64_t n_st, int64_t n_sh, uint16_t* __restrict__ kc,
                                                       uint16_t* __restrict__ vc, int64_t c_sb, int64_t c_sh, int64_t c_sl,
                                                       const int* __restrict__ cache_idx, const int* __restrict__ pos,
                                                       int B, int T, int H, int D, int Lmax) {
  const int nv = D / 8;
  const int64_t total = (int64_t)B * T * H * nv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = i % nv;
    const int h = (i / nv) % H;
    const int t = (i / ((int64_t)nv * H)) % T;
    const int b = i / ((int64_t)nv * H * T);
    const int cb = cache_idx ? cache_idx[b] : b;
    const int ps = pos[b] + t;
    if (ps < 0 || ps >= Lmax) continue;
    const int64_t src = (int64_t)b * n_sb + (int64_t)t * n_st + (int64_t)h * n_sh + c * 8;
    const int64_t dst = (int64_t)cb * c_sb + (int64_t)h * c_sh + (int64_t)ps * c_sl + c * 8;
    *reinterpret_cast<u32x4_t*>(kc + dst) = *reinterpret_cast<const u32x4_t*>(k + src);
    *reinterpret_cast<u32x4_t*>(vc + dst) = *reinterpret_cast<const u32x4_t*>(v + src);
  }
}

template <typename T>
__device__ __forceinline__ float ldv(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2) return bf2f(((const uint16_t*)p)[i]);
  else return ((const float*)p)[i];
}

template <typename T>
__global__ void __launch_bounds__(1024) argmax_kernel(const T* __restrict__ x, int64_t ld, int V, int64_t* __restrict__ out) {
  __shared__ float bv[16];
  __shared__ int bi[16];
  const T* row = x + (int64_t)blockIdx.x * ld;
  float best = -INFINITY;
  int idx = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = ldv<T>(row, i);
    if (v > best) { best = v; idx = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > best || (ov == best && oi < idx)) { best = ov; idx = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { bv[wid] = best; bi[wid] = idx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = bv[0];
    int ii = bi[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (bv[w] > b || (bv[w] == b && bi[w] < ii)) { b = bv[w]; ii = bi[w]; }
    out[blockIdx.x] = ii == 0x7fffffff ? 0 : ii;
  }
}

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int kMaxTopK = 1024;

template <typename T>
__global__ void __launch_bounds__(1024) topk_sample_kernel(const T* __restrict__ x, int64_t ld, int V, int K, float inv_temp,
                                                           const float* __restrict__ uniform, int64_t* __restrict__ out,
                                                           float* __restrict__ out_vals, int64_t* __restrict__ out_idx) {
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix, s_mask;
  __shared__ int s_rem, s_cnt_gt, s_cnt_eq;
  __shared__ float cv[kMaxTopK];
  __shared__ int ci[kMaxTopK];
  __shared__ float cp[kMaxTopK];
  __shared__ int si[kMaxTopK];
  const T* row = x + (int64_t)blockIdx.x * ld;
  if (threadIdx.x == 0) { s_prefix = 0; s_mask = 0; s_rem = K; s_cnt_gt = 0; s_cnt_eq = 0; }
  __syncthreads();
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const uint32_t pre = s_prefix, msk = s_mask;
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const uint32_t kk = fkey(ldv<T>(row, i));
      if ((kk & msk) == pre) atomicAdd(&hist[(kk >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int rem = s_rem, cum = 0, bin = 0;
      for (bin = 255; bin >= 0; --bin) {
        if (cum + hist[bin] >= rem) break;
        cum += hist[bin];
      }
      if (bin < 0) bin = 0;
      s_rem = rem - cum;
      s_prefix = pre | ((uint32_t)bin << shift);
      s_mask = msk | (255u << shift);
    }
    __syncthreads();
  }
  const uint32_t thr = s_prefix;
  const int need_eq = s_rem;          // elements equal to thr to take
  const int n_gt = K - need_eq;       // elements strictly greater
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = ldv<T>(row, i);
    const uint32_t kk = fkey(v);
    if (kk > thr) {
      const int slot = atomicAdd(&s_cnt_gt, 1);
      if (slot < n_gt) { cv[slot] = v; ci[slot] = i; }
    } else if (kk == thr) {
      const int slot = atomicAdd(&s_cnt_eq, 1);
      if (slot < need_eq) { cv[n_gt + slot] = v; ci[n_gt + slot] = i; }
    }
  }
  __syncthreads();
  // rank = position in descending (value, then lower index) order; O(K^2 / threads) compares
  for (int i = threadIdx.x; i < K; i += blockDim.x) {
    const float v = cv[i];
    const int id = ci[i];
    int rank = 0;
    for (int j = 0; j < K; ++j) rank += (cv[j] > v) || (cv[j] == v && ci[j] < id);
    cp[rank] = v;
    si[rank] = id;
  }
  __syncthreads();
  if (out_idx || out_vals)
    for (int i = threadIdx.x; i < K; i += blockDim.x) {
      if (out_idx) out_idx[(int64_t)blockIdx.x * K + i] = si[i];
      if (out_vals) out_vals[(int64_t)blockIdx.x * K + i] = cp[i];
    }
  if (threadIdx.x == 0) {
    // softmax(top-k / temperature) -> CDF -> count of CDF entries below the uniform draw
    // (the reference's cumsum / subtract / count_nonzero formulation, sampling.py:66-77)
    const float mx = cp[0];
    float sum = 0.f;
    for (int j = 0; j < K; ++j) sum += __expf((cp[j] - mx) * inv_temp);
    const float u = uniform ? uniform[blockIdx.x] : 0.5f;
    float cdf = 0.f;
    int pick = 0;
    for (int j = 0; j < K; ++j) {
      cdf += __expf((cp[j] - mx) * inv_temp) / sum;
      pick += cdf < u;
    }
    if (pick >= K) pick = K - 1;
    out[blockIdx.x] = si[pick];
  }
}

}  // namespace dec

int decode_attn_launch(const void* q, const int64_t* qs, const void* kc, const void* vc, const int64_t* cs,
                       const int* cache_idx, const int* seq_len, float* po, float* pm, float* pl, void* out,
                       const int64_t* os, int B, int T, int Hq, int Hkv, int D, int nsplit, float scale, hipStream_t stream) {
  using namespace dec;
  if (Hkv <= 0 || Hq % Hkv) return -1;
  const int M = (Hq / Hkv) * T;
  DecodeParams p;
  p.q = (const uint16_t*)q; p.q_sb = qs[0]; p.q_st = qs[1]; p.q_sh = qs[2];
  p.kc = (const uint16_t*)kc; p.vc = (const uint16_t*)vc;
  p.c_sb = cs[0]; p.c_sh = cs[1]; p.c_sl = cs[2];
  p.cache_idx = cache_idx; p.seq_len = seq_len; p.po = po; p.pm = pm; p.pl = pl;
  p.B = B; p.T = T; p.Hq = Hq; p.Hkv = Hkv; p.nsplit = nsplit; p.scale = scale;
  const size_t lds = (size_t)M * D * 4 + (size_t)M * kChunk * 4;
  if (lds > 160 * 1024) return -3;
  const dim3 grid(B * Hkv * nsplit);
  if (D == 64) hipLaunchKernelGGL(partial_kernel<64>, grid, dim3(256), lds, stream, p);
  else if (D == 128) hipLaunchKernelGGL(partial_kernel<128>, grid, dim3(256), lds, stream, p);
  else return -2;
  hipLaunchKernelGGL(combine_kernel, dim3(B * Hkv * M), dim3(D < 256 ? D : 256), 0, stream, po, pm, pl, (uint16_t*)out,
                     os[0], os[1], os[2], Hq, Hkv, T, nsplit, D);
  return (int)hipGetLastError();
}

int kv_cache_write_launch(const void* k, const void* v, const int64_t* ns, void* kc, void* vc, const int64_t* cs,
                          const int* cache_idx, const int* pos, int B, int T, int H, int D, int Lmax, hipStream_t stream) {
  const int64_t total = (int64_t)B * T * H * (D / 8);
  if (total == 0) return 0;
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(dec::kv_write_kernel, dim3((unsigned)g), dim3(256), 0, stream, (const uint16_t*)k, (const uint16_t*)v,
                     ns[0], ns[1], ns[2], (uint16_t*)kc, (uint16_t*)vc, cs[0], cs[1], cs[2], cache_idx, pos, B, T, H, D, Lmax);
  return (int)hipGetLastError();
}

int topk_sample_launch(const void* x, int is_fp32, int64_t ld, int B, int V, int K, float temperature, const float* uniform,
                       int64_t* out, float* out_vals, int64_t* out_idx, hipStream_t stream) {
  if (B == 0) return 0;
  if (K < 1 || K > dec::kMaxTopK || K > V) return -1;
  const float inv_t = temperature > 0.f ? 1.f / temperature : 1.f;
  if (is_fp32)
    hipLaunchKernelGGL(dec::topk_sample_kernel<float>, dim3(B), dim3(1024), 0, stream, (const float*)x, ld, V, K, inv_t, uniform, out, out_vals, out_idx);
  else
    hipLaunchKernelGGL(dec::topk_sample_kernel<uint16_t>, dim3(B), dim3(1024), 0, stream, (const uint16_t*)x, ld, V, K, inv_t, uniform, out, out_vals, out_idx);
  return (int)hipGetLastError();
}

int argmax_launch(const void* x, int is_fp32, int64_t ld, int B, int V, int64_t* out, hipStream_t stream) {
  if (B == 0) return 0;
  if (is_fp32) hipLaunchKernelGGL(dec::argmax_kernel<float>, dim3(B), dim3(1024), 0, stream, (const float*)x, ld, V, out);
  else hipLaunchKernelGGL(dec::argmax_kernel<uint16_t>, dim3(B), dim3(1024), 0, stream, (const uint16_t*)x, ld, V, out);
  return (int)hipGetLastError();
}

}  // namespace nxd
