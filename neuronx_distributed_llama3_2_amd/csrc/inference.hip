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
  int fused_merge;           // 1: last workgroup merges the splits; 0: separate merge_kernel
};

// Merge the (m, l, o) partials of all splits of one (batch, kv head): every phase parallel over the
// workgroup (split maxima/sums in LDS, (row, 8-dim chunk) x split-group partial sums, LDS reduction).
template <int D>
__device__ void merge_splits(const DecodeParams& p, int bh, float* red, float* ss, uint16_t* __restrict__ out,
                             int64_t o_sb, int64_t o_st, int64_t o_sh) {
  constexpr int NC = D / 8;
  const int G = p.Hq / p.Hkv;
  const int M = G * p.T;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int64_t base0 = (int64_t)bh * p.nsplit * M;
  // (1) all (split, row) maxima / sums in parallel -> LDS; per-row max and split weights
  float* wsp = red + 4 * 8 * D;                      // [nsplit][M] split weights
  float* rowl = ss;                                  // [M] total l per row
  const int NSM = p.nsplit * M;
  for (int i = tid; i < NSM; i += 256) wsp[i] = p.pm[base0 + i];
  __syncthreads();
  for (int m = wid; m < M; m += 4) {
    float mx = -INFINITY;
    for (int s2 = lane; s2 < p.nsplit; s2 += 64) mx = fmaxf(mx, wsp[s2 * M + m]);
    mx = wave_max(mx);
    float l = 0.f;
    for (int s2 = lane; s2 < p.nsplit; s2 += 64) {
      const float ms = wsp[s2 * M + m];
      const float w = ms == -INFINITY ? 0.f : __expf(ms - mx);
      l += w * p.pl[base0 + s2 * M + m];
      wsp[s2 * M + m] = w;
    }
    l = wave_sum(l);
    if (lane == 0) rowl[m] = l;
  }
  __syncthreads();
  // (2) weighted sum of the split outputs: (row, 8-dim chunk) items x split groups, LDS reduction
  const int items = M * NC;
  const int SG = 256 / (items < 256 ? items : 256) > 0 ? 256 / (items < 256 ? items : 256) : 1;
  float* part = red;                                 // [SG][items][8] (fits: SG * items <= 256)
  for (int i0 = 0; i0 < items; i0 += 256 / SG) {
    const int it = i0 + tid % (256 / SG), sg = tid / (256 / SG);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (it < items && sg < SG) {
      const int m = it / NC, c = it % NC;
      for (int s2 = sg; s2 < p.nsplit; s2 += SG) {
        const float w = wsp[s2 * M + m];
        if (w == 0.f) continue;
        const float* src = p.po + (base0 + (int64_t)s2 * M + m) * D + c * 8;
        const f32x4_t a0 = *reinterpret_cast<const f32x4_t*>(src);
        const f32x4_t a1 = *reinterpret_cast<const f32x4_t*>(src + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] += w * a0[e];
          acc[4 + e] += w * a1[e];
        }
      }
    }
    __syncthreads();
    if (it < items && sg < SG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) part[(sg * (256 / SG) + (it - i0)) * 8 + e] = acc[e];
    }
    __syncthreads();
    if (tid < 256 / SG && i0 + tid < items) {
      const int itm = i0 + tid, m = itm / NC, c = itm % NC;
      float o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int g = 0; g < SG; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += part[(g * (256 / SG) + tid) * 8 + e];
      const float inv = rowl[m] > 0.f ? 1.f / rowl[m] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= inv;
      const int tt = m / G, gg = m % G;
      *reinterpret_cast<u32x4_t*>(out + (int64_t)b * o_sb + (int64_t)tt * o_st + (int64_t)(hkv * G + gg) * o_sh + c * 8) =
          pack8(o);
    }
    __syncthreads();
  }
}

template <int D>
__global__ void __launch_bounds__(256) merge_kernel(DecodeParams p, uint16_t* __restrict__ out, int64_t o_sb,
                                                    int64_t o_st, int64_t o_sh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = (p.Hq / p.Hkv) * p.T;
  float* ss = reinterpret_cast<float*>(smem);   // [M] row sums
  float* red = ss + ((M + 3) & ~3);             // [4][8][D] + [nsplit][M]
  merge_splits<D>(p, blockIdx.x, red, ss, out, o_sb, o_st, o_sh);
}

// One workgroup per (batch, kv head, 128-key split); the LAST workgroup of a (batch, kv head) to
// finish merges every split's (m, l, o) partials (agent-scope release/acquire fences around one
// atomic counter, which that workgroup resets) — one launch per attention call, every phase fully
// parallel over the 256 threads:
//   scores: 2 threads per key (half the head dim each), q rows broadcast from LDS;
//   softmax: one wave per q row over the 128 keys;
//   P.V: thread (key group, 8-dim chunk) accumulates its keys for 8 q rows at a time, then a
//        shuffle + LDS reduction over the key groups.
template <int D>
__global__ void __launch_bounds__(256) attn_kernel(DecodeParams p, int* __restrict__ counters, uint16_t* __restrict__ out,
                                                   int64_t o_sb, int64_t o_st, int64_t o_sh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NC = D / 8;          // 16-byte chunks per head row
  constexpr int KG = 256 / NC;       // key groups in the P.V phase
  constexpr int MB = 8;              // q rows per P.V pass
  const int G = p.Hq / p.Hkv;
  const int M = G * p.T;
  float* qs = reinterpret_cast<float*>(smem);   // [M][D]
  float* ss = qs + M * D;                       // [M][kChunk]
  float* red = ss + M * kChunk;                 // [4][MB][D]
  __shared__ int last_flag;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int split = blockIdx.x % p.nsplit;
  const int bh = blockIdx.x / p.nsplit;
  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int cb = p.cache_idx ? p.cache_idx[b] : b;
  const int slen = p.seq_len[b];
  const int k0 = split * kChunk;
  const int64_t pbase = ((int64_t)bh * p.nsplit + split) * M;
  const uint16_t* kbase = p.kc + (int64_t)cb * p.c_sb + (int64_t)hkv * p.c_sh;
  const uint16_t* vbase = p.vc + (int64_t)cb * p.c_sb + (int64_t)hkv * p.c_sh;

  if (k0 < slen) {
    // ---- V chunk for the P.V phase: issue the loads early (independent of the scores)
    const int c = tid % NC, kg = tid / NC;
    constexpr int VPT = kChunk / KG;   // keys per thread
    u32x4_t vv[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int key = k0 + kg + j * KG;
      vv[j] = key < slen ? *reinterpret_cast<const u32x4_t*>(vbase + (int64_t)key * p.c_sl + c * 8) : u32x4_t{0, 0, 0, 0};
    }
    // ---- K half-row per thread
    const int kk = tid >> 1, half = tid & 1;
    const int key = k0 + kk;
    float kr[D / 2];
    if (key < slen) {
#pragma unroll
      for (int cc = 0; cc < D / 16; ++cc)
        unpack8(*reinterpret_cast<const u32x4_t*>(kbase + (int64_t)key * p.c_sl + half * (D / 2) + cc * 8), kr + cc * 8);
    } else {
#pragma unroll
      for (int d = 0; d < D / 2; ++d) kr[d] = 0.f;
    }
    // ---- q rows (pre-scaled) -> LDS
    for (int i = tid; i < M * NC; i += 256) {
      const int m = i / NC, c = i % NC;
      const int tt = m / G, gg = m % G;
      const uint16_t* src = p.q + (int64_t)b * p.q_sb + (int64_t)tt * p.q_st + (int64_t)(hkv * G + gg) * p.q_sh + c * 8;
      float f[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(src), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) qs[m * D + c * 8 + j] = f[j] * p.scale;
    }
    __syncthreads();
    for (int m = 0; m < M; ++m) {
      const float* qr = qs + m * D + half * (D / 2);
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D / 2; ++d) s += qr[d] * kr[d];
      s += __shfl_xor(s, 1, 64);
      const int tt = m / G;
      const int lim = slen - (p.T - 1 - tt);  // causal among the new tokens
      if (half == 0) ss[m * kChunk + kk] = key < lim ? s : -INFINITY;
    }
    __syncthreads();
    // ---- softmax per row (wave per row)
    for (int m = wid; m < M; m += 4) {
      const float a = ss[m * kChunk + lane], e = ss[m * kChunk + 64 + lane];
      const float mx = wave_max(fmaxf(a, e));
      const float mu = mx == -INFINITY ? 0.f : mx;
      const float ea = __expf(a - mu), ee = __expf(e - mu);
      ss[m * kChunk + lane] = ea;
      ss[m * kChunk + 64 + lane] = ee;
      const float sum = wave_sum(ea + ee);
      if (lane == 0) {
        p.pm[pbase + m] = mx;
        p.pl[pbase + m] = sum;
      }
    }
    __syncthreads();
    // ---- P.V
    for (int m0 = 0; m0 < M; m0 += MB) {
      float acc[MB][8];
#pragma unroll
      for (int mm = 0; mm < MB; ++mm)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[mm][j] = 0.f;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        float vf[8];
        unpack8(vv[j], vf);
        const int kidx = kg + j * KG;
#pragma unroll
        for (int mm = 0; mm < MB; ++mm) {
          if (m0 + mm < M) {
            const float pv = ss[(m0 + mm) * kChunk + kidx];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[mm][e] += pv * vf[e];
          }
        }
      }
      // reduce over the key groups of this wave (lanes differing in the kg bits), then across waves
#pragma unroll
      for (int mm = 0; mm < MB; ++mm)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = acc[mm][e];
#pragma unroll
          for (int o = NC; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
          acc[mm][e] = v;
        }
      if (lane < NC) {
#pragma unroll
        for (int mm = 0; mm < MB; ++mm)
#pragma unroll
          for (int e = 0; e < 8; ++e) red[(wid * MB + mm) * D + c * 8 + e] = acc[mm][e];
      }
      __syncthreads();
      for (int i = tid; i < MB * D; i += 256) {
        const int mm = i / D, d = i % D;
        if (m0 + mm < M)
          p.po[(pbase + m0 + mm) * D + d] = red[(0 * MB + mm) * D + d] + red[(1 * MB + mm) * D + d] +
                                            red[(2 * MB + mm) * D + d] + red[(3 * MB + mm) * D + d];
      }
      __syncthreads();
    }
  } else {
    for (int m = tid; m < M; m += 256) {
      p.pm[pbase + m] = -INFINITY;
      p.pl[pbase + m] = 0.f;
    }
  }
  // ---- last workgroup of this (b, hkv) merges the splits
  if (!p.fused_merge) return;
  __threadfence();
  __syncthreads();
  if (tid == 0) {
    const int prev = atomicAdd(counters + bh, 1);
    last_flag = prev == p.nsplit - 1;
  }
  __syncthreads();
  if (!last_flag) return;
  __threadfence();
  merge_splits<D>(p, bh, red, ss, out, o_sb, o_st, o_sh);
  if (tid == 0) counters[bh] = 0;  // ready for the next launch / graph replay
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
  if (sizeof(T) == 2 && (V % 8) == 0 && (reinterpret_cast<uintptr_t>(row) % 16) == 0) {
    // 16-byte loads, 4 in flight per thread
    const u32x4_t* rv = reinterpret_cast<const u32x4_t*>(row);
    const int nv = V / 8;
    for (int i0 = threadIdx.x; i0 < nv; i0 += 4 * blockDim.x) {
      u32x4_t q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * blockDim.x;
        q[u] = i < nv ? rv[i] : u32x4_t{0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u};
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(q[u], f);
        const int base = (i0 + u * blockDim.x) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (f[e] > best) { best = f[e]; idx = base + e; }
      }
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float v = ldv<T>(row, i);
      if (v > best) { best = v; idx = i; }
    }
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

// ---- greedy decode step tail: argmax over the vocabulary split across many workgroups (one
// 64-bit atomicMax of (order-preserving value key, ~index) per workgroup: highest logit, lowest
// index on ties, as torch.argmax), then ONE tiny kernel that feeds the token back: out[b, step],
// tokens[b], positions[b] + 1, cache_len[b] + 1, step + 1 and the slot reset -- instead of the
// single-workgroup argmax plus five framework element-wise launches per token.
constexpr int kArgmaxChunk = 2048;   // elements per workgroup (256 threads x 8)

template <typename T>
__global__ void __launch_bounds__(256) argmax_partial_kernel(const T* __restrict__ x, int64_t ld, int V,
                                                             unsigned long long* __restrict__ slot) {
  __shared__ unsigned long long wk[4];
  const int b = blockIdx.y;
  const T* row = x + (int64_t)b * ld;
  const int beg = blockIdx.x * kArgmaxChunk, end = min(V, beg + kArgmaxChunk);
  float best = -INFINITY;
  int idx = -1;
  const int i0 = beg + threadIdx.x * 8;
  if (sizeof(T) == 2 && (reinterpret_cast<uintptr_t>(row) % 16) == 0 && i0 + 8 <= end) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(row + i0), f);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (f[e] > best) { best = f[e]; idx = i0 + e; }
  } else {
    for (int i = i0; i < min(end, i0 + 8); ++i) {
      const float v = ldv<T>(row, i);
      if (idx < 0 || v > best) { best = v; idx = i; }
    }
  }
  unsigned long long key = idx < 0 ? 0ull
                                   : ((unsigned long long)fkey(best) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long ok = __shfl_xor(key, o, 64);
    key = ok > key ? ok : key;
  }
  if ((threadIdx.x & 63) == 0) wk[threadIdx.x >> 6] = key;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long k = wk[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) k = wk[w] > k ? wk[w] : k;
    if (k) atomicMax(slot + b, k);
  }
}

__global__ void __launch_bounds__(64) greedy_advance_kernel(unsigned long long* __restrict__ slot, int64_t* __restrict__ out,
                                                           int64_t ld_out, int max_steps, int64_t* __restrict__ step,
                                                           int64_t* __restrict__ tokens, int64_t* __restrict__ positions,
                                                           int* __restrict__ cache_len, int B) {
  const int64_t s = step[0];
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const unsigned long long k = slot[b];
    const int64_t tok = k ? (int64_t)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : 0;
    if (s >= 0 && s < max_steps) out[(int64_t)b * ld_out + s] = tok;
    tokens[b] = tok;
    positions[b] += 1;
    cache_len[b] += 1;
    slot[b] = 0ull;
  }
  __syncthreads();
  if (threadIdx.x == 0) step[0] = s + 1;
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

int decode_attn2_launch(const void*, const int64_t*, const void*, const void*, const int64_t*, const int*, const int*,
                        float*, float*, float*, void*, const int64_t*, int, int, int, int, int, int, float, int*, hipStream_t);

static int g_attn_v2 = [] { const char* e = getenv("NXD_DECODE_ATTN_V2"); return e ? atoi(e) : 1; }();
void decode_attn_set_v2(int v) { g_attn_v2 = v; }

int decode_attn_launch(const void* q, const int64_t* qs, const void* kc, const void* vc, const int64_t* cs,
                       const int* cache_idx, const int* seq_len, float* po, float* pm, float* pl, int* counters, void* out,
                       const int64_t* os, int B, int T, int Hq, int Hkv, int D, int nsplit, float scale, hipStream_t stream) {
  using namespace dec;
  if (Hkv <= 0 || Hq % Hkv) return -1;
  const int M = (Hq / Hkv) * T;
  // small query groups: the MFMA flash-decoding kernel (decode_attn.hip), merge only past 1024 keys
  if (g_attn_v2) {
    int ns2 = 0;
    const int rc = decode_attn2_launch(q, qs, kc, vc, cs, cache_idx, seq_len, po, pm, pl, out, os, B, T, Hq, Hkv, D,
                                       nsplit * kChunk, scale, &ns2, stream);
    if (rc == 0 && ns2 > 1) {
      DecodeParams mp;
      mp.q = (const uint16_t*)q; mp.q_sb = qs[0]; mp.q_st = qs[1]; mp.q_sh = qs[2];
      mp.kc = (const uint16_t*)kc; mp.vc = (const uint16_t*)vc;
      mp.c_sb = cs[0]; mp.c_sh = cs[1]; mp.c_sl = cs[2];
      mp.cache_idx = cache_idx; mp.seq_len = seq_len; mp.po = po; mp.pm = pm; mp.pl = pl;
      mp.B = B; mp.T = T; mp.Hq = Hq; mp.Hkv = Hkv; mp.nsplit = ns2; mp.scale = scale; mp.fused_merge = 0;
      const size_t mlds = (size_t)((M + 3) & ~3) * 4 + (size_t)4 * 8 * D * 4 + (size_t)ns2 * M * 4;
      if (D == 64)
        hipLaunchKernelGGL(merge_kernel<64>, dim3(B * Hkv), dim3(256), mlds, stream, mp, (uint16_t*)out, os[0], os[1], os[2]);
      else
        hipLaunchKernelGGL(merge_kernel<128>, dim3(B * Hkv), dim3(256), mlds, stream, mp, (uint16_t*)out, os[0], os[1], os[2]);
      return (int)hipGetLastError();
    }
    if (rc != -1) return rc;   // -1: shape not covered by the MFMA kernel
  }
  DecodeParams p{};
  p.q = (const uint16_t*)q; p.q_sb = qs[0]; p.q_st = qs[1]; p.q_sh = qs[2];
  p.kc = (const uint16_t*)kc; p.vc = (const uint16_t*)vc;
  p.c_sb = cs[0]; p.c_sh = cs[1]; p.c_sl = cs[2];
  p.cache_idx = cache_idx; p.seq_len = seq_len; p.po = po; p.pm = pm; p.pl = pl;
  p.B = B; p.T = T; p.Hq = Hq; p.Hkv = Hkv; p.nsplit = nsplit; p.scale = scale;
  // separate merge launch by default: the fused last-workgroup merge needs agent-scope fences (L2
  // write-back / invalidate across the 8 XCDs), measured 2-3x slower on MI355X (tools/bench_decode.py)
  static const int mode = [] { const char* e = getenv("NXD_DECODE_FUSED_MERGE"); return e ? atoi(e) : 0; }();
  p.fused_merge = mode;
  const size_t lds = (size_t)M * D * 4 + (size_t)M * kChunk * 4 + (size_t)4 * 8 * D * 4 + (size_t)nsplit * M * 4;
  if (lds > 160 * 1024) return -3;
  const dim3 grid(B * Hkv * nsplit);
  if (D == 64) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)attn_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(attn_kernel<64>, grid, dim3(256), lds, stream, p, counters, (uint16_t*)out, os[0], os[1], os[2]);
  } else if (D == 128) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)attn_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(attn_kernel<128>, grid, dim3(256), lds, stream, p, counters, (uint16_t*)out, os[0], os[1], os[2]);
  } else {
    return -2;
  }
  if (!p.fused_merge) {
    const size_t mlds = (size_t)((M + 3) & ~3) * 4 + (size_t)4 * 8 * D * 4 + (size_t)nsplit * M * 4;
    if (D == 64) {
      if (mlds > 64 * 1024) (void)hipFuncSetAttribute((const void*)merge_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlds);
      hipLaunchKernelGGL(merge_kernel<64>, dim3(B * Hkv), dim3(256), mlds, stream, p, (uint16_t*)out, os[0], os[1], os[2]);
    } else {
      if (mlds > 64 * 1024) (void)hipFuncSetAttribute((const void*)merge_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlds);
      hipLaunchKernelGGL(merge_kernel<128>, dim3(B * Hkv), dim3(256), mlds, stream, p, (uint16_t*)out, os[0], os[1], os[2]);
    }
  }
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

int greedy_advance_launch(const void* logits, int is_fp32, int64_t ld, int B, int V, unsigned long long* slot, int64_t* out,
                          int64_t ld_out, int max_steps, int64_t* step, int64_t* tokens, int64_t* positions, int* cache_len,
                          hipStream_t stream) {
  if (B == 0) return 0;
  if (B > 65535) return -1;
  const dim3 grid((unsigned)((V + dec::kArgmaxChunk - 1) / dec::kArgmaxChunk), (unsigned)B);
  if (is_fp32)
    hipLaunchKernelGGL(dec::argmax_partial_kernel<float>, grid, dim3(256), 0, stream, (const float*)logits, ld, V, slot);
  else
    hipLaunchKernelGGL(dec::argmax_partial_kernel<uint16_t>, grid, dim3(256), 0, stream, (const uint16_t*)logits, ld, V, slot);
  hipLaunchKernelGGL(dec::greedy_advance_kernel, dim3(1), dim3(64), 0, stream, slot, out, ld_out, max_steps, step, tokens,
                     positions, cache_len, B);
  return (int)hipGetLastError();
}

int argmax_launch(const void* x, int is_fp32, int64_t ld, int B, int V, int64_t* out, hipStream_t stream) {
  if (B == 0) return 0;
  if (is_fp32) hipLaunchKernelGGL(dec::argmax_kernel<float>, dim3(B), dim3(1024), 0, stream, (const float*)x, ld, V, out);
  else hipLaunchKernelGGL(dec::argmax_kernel<uint16_t>, dim3(B), dim3(1024), 0, stream, (const uint16_t*)x, ld, V, out);
  return (int)hipGetLastError();
}

}  // namespace nxd
