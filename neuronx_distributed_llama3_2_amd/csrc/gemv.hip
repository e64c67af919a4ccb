// Skinny GEMM ("GEMV") for token generation: y[M, N] = x[M, K] @ W[N, K]^T for M <= 8, with
// bf16 or int8 weights (int8: symmetric, per-tensor or per-output-row fp32 scale), an optional
// bias, and an optional fused SwiGLU epilogue (y[:, n] = silu(x.W[n]) * (x.W[n + N]) for the fused
// gate_up projection — the [M, 2N] intermediate never touches memory).
//
// Decode is weight-bandwidth bound: every weight byte is read exactly once, 16 B per lane per load
// (8 bf16 or 16 int8), with the tiny activation rows served from L2/LDS-speed caches.  One wave
// owns ROWS output rows; lanes stride over K and the partial dot products are reduced with
// cross-lane shuffles.  int8 halves the bytes per token versus bf16 (the reference's int8
// weight-only inference: src/neuronx_distributed/quantization/quantization_layers.py:342-665).
#include "common.h"

namespace nxd {
namespace gemv {

struct Params {
  const uint16_t* x;
  int64_t ldx;
  const void* w;
  int64_t ldw;
  const float* scale;  // per weight row (nullable)
  float tscale;        // per-tensor scale (used when scale == nullptr)
  const uint16_t* bias;  // [N] (nullable; added after scaling, before the GLU)
  uint16_t* y;
  int64_t ldy;
  int M, N, K;  // N = output columns (GLU: the up rows start at weight row N)
  // expert (MoE decode) mode: blockIdx.y = (token, expert-slot) pair p; it multiplies x row
  // p / xdiv with the weights of expert eidx[p] (base + eidx[p] * estride) into y row p
  const int32_t* eidx;
  int64_t estride;
  int xdiv;
};

template <typename WT>
struct WTraits;
template <>
struct WTraits<uint16_t> {
  static constexpr int EPL = 8;  // elements per 16-byte load
  __device__ static void load(const void* base, int64_t off, float* f) {
    unpack8(*reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(base) + off), f);
  }
};
template <>
struct WTraits<int8_t> {
  static constexpr int EPL = 16;
  __device__ static void load(const void* base, int64_t off, float* f) {
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const int8_t*>(base) + off);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t d = (int32_t)v[i];
      f[4 * i + 0] = (float)((d << 24) >> 24);
      f[4 * i + 1] = (float)((d << 16) >> 24);
      f[4 * i + 2] = (float)((d << 8) >> 24);
      f[4 * i + 3] = (float)(d >> 24);
    }
  }
};

template <typename WT, int MM, int ROWS, bool GLU>
__global__ void __launch_bounds__(256) gemv_kernel(Params p) {
  constexpr int EPL = WTraits<WT>::EPL;
  constexpr int NW = GLU ? 2 * ROWS : ROWS;  // weight rows per wave
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * 4) + (threadIdx.x >> 6);
  const int n0 = wave * ROWS;
  if (n0 >= p.N) return;
  if (p.eidx) {
    const int pair = blockIdx.y;
    p.w = reinterpret_cast<const char*>(p.w) + (int64_t)p.eidx[pair] * p.estride * (int64_t)sizeof(WT);
    p.x += (int64_t)(pair / p.xdiv) * p.ldx;
    p.y += (int64_t)pair * p.ldy;
  }
  int wrow[NW];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int n = min(n0 + r, p.N - 1);
    wrow[r] = n;
    if (GLU) wrow[ROWS + r] = n + p.N;
  }
  float acc[MM][NW];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int r = 0; r < NW; ++r) acc[m][r] = 0.f;

  for (int k = lane * EPL; k < p.K; k += 64 * EPL) {
    float wf[NW][EPL];
#pragma unroll
    for (int r = 0; r < NW; ++r) WTraits<WT>::load(p.w, (int64_t)wrow[r] * p.ldw + k, wf[r]);
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (m < p.M) {
        float xf[EPL];
#pragma unroll
        for (int c = 0; c < EPL / 8; ++c)
          unpack8(*reinterpret_cast<const u32x4_t*>(p.x + (int64_t)m * p.ldx + k + 8 * c), xf + 8 * c);
#pragma unroll
        for (int r = 0; r < NW; ++r)
#pragma unroll
          for (int e = 0; e < EPL; ++e) acc[m][r] += xf[e] * wf[r][e];
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int r = 0; r < NW; ++r) acc[m][r] = wave_sum(acc[m][r]);
  if (lane != 0) return;
#pragma unroll
  for (int m = 0; m < MM; ++m) {
    if (m >= p.M) continue;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const int n = n0 + r;
      if (n >= p.N) continue;
      float v = acc[m][r] * (p.scale ? p.scale[wrow[r]] : p.tscale);
      if (p.bias) v += bf2f(p.bias[wrow[r]]);
      if (GLU) {
        float u = acc[m][ROWS + r] * (p.scale ? p.scale[wrow[ROWS + r]] : p.tscale);
        if (p.bias) u += bf2f(p.bias[wrow[ROWS + r]]);
        v = v / (1.f + __expf(-v)) * u;
      }
      p.y[(int64_t)m * p.ldy + n] = f2bf(v);
    }
  }
}

// W_bf16[n, k] = W_int8[n, k] * scale[n] (or tscale)
__global__ void __launch_bounds__(256) dequant_kernel(const int8_t* __restrict__ w, int64_t ldw,
                                                      const float* __restrict__ scale, float tscale,
                                                      uint16_t* __restrict__ out, int N, int K) {
  const int64_t total = (int64_t)N * (K / 16);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int n = i / (K / 16);
    const int k = (i % (K / 16)) * 16;
    float f[16];
    WTraits<int8_t>::load(w, (int64_t)n * ldw + k, f);
    const float s = scale ? scale[n] : tscale;
#pragma unroll
    for (int e = 0; e < 16; ++e) f[e] *= s;
    *reinterpret_cast<u32x4_t*>(out + (int64_t)n * K + k) = pack8(f);
    *reinterpret_cast<u32x4_t*>(out + (int64_t)n * K + k + 8) = pack8(f + 8);
  }
}

template <typename WT, int MM, bool GLU>
static int launch_m(const Params& p, hipStream_t s, int pairs = 1) {
  const int rows = p.N >= 8192 ? 2 : 1;
  const int waves = (p.N + rows - 1) / rows;
  dim3 grid((waves + 3) / 4, pairs), block(256);
  if (rows == 2)
    hipLaunchKernelGGL((gemv_kernel<WT, MM, 2, GLU>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemv_kernel<WT, MM, 1, GLU>), grid, block, 0, s, p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <typename WT, bool GLU>
static int launch_t(const Params& p, hipStream_t s) {
  if (p.M <= 1) return launch_m<WT, 1, GLU>(p, s);
  if (p.M <= 2) return launch_m<WT, 2, GLU>(p, s);
  if (p.M <= 4) return launch_m<WT, 4, GLU>(p, s);
  if (p.M <= 8) return launch_m<WT, 8, GLU>(p, s);
  return 2;
}

}  // namespace gemv

int gemv_launch(const void* x, int64_t ldx, const void* w, int64_t ldw, int w_is_int8, const float* scale, float tscale,
                const void* bias, void* y, int64_t ldy, int M, int N, int K, int glu, hipStream_t stream) {
  gemv::Params p{reinterpret_cast<const uint16_t*>(x), ldx, w, ldw, scale, tscale,
                 reinterpret_cast<const uint16_t*>(bias), reinterpret_cast<uint16_t*>(y), ldy, M, N, K,
                 nullptr, 0, 1};
  if (w_is_int8) return glu ? gemv::launch_t<int8_t, true>(p, stream) : gemv::launch_t<int8_t, false>(p, stream);
  return glu ? gemv::launch_t<uint16_t, true>(p, stream) : gemv::launch_t<uint16_t, false>(p, stream);
}

// MoE decode: y[p, :N] = x[p / xdiv] . W[eidx[p]]^T  (W [E, Nw, K] bf16, rows ldw apart, experts
// estride elements apart; GLU as above).  Only the selected experts' weights are read.
int expert_gemv_launch(const void* x, int64_t ldx, const void* w, int64_t ldw, int64_t estride, const int32_t* eidx,
                       int pairs, int xdiv, void* y, int64_t ldy, int N, int K, int glu, hipStream_t stream) {
  gemv::Params p{reinterpret_cast<const uint16_t*>(x), ldx, w, ldw, nullptr, 1.f, nullptr,
                 reinterpret_cast<uint16_t*>(y), ldy, 1, N, K, eidx, estride, xdiv};
  return glu ? gemv::launch_m<uint16_t, 1, true>(p, stream, pairs) : gemv::launch_m<uint16_t, 1, false>(p, stream, pairs);
}

int dequant_int8_launch(const void* w, int64_t ldw, const float* scale, float tscale, void* out, int N, int K,
                        hipStream_t stream) {
  const int64_t total = (int64_t)N * (K / 16);
  const int64_t g = (total + 255) / 256;
  const int grid = (int)(g < 8192 ? g : 8192);
  hipLaunchKernelGGL(gemv::dequant_kernel, dim3(grid), dim3(256), 0, stream, reinterpret_cast<const int8_t*>(w), ldw,
                     scale, tscale, reinterpret_cast<uint16_t*>(out), N, K);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace nxd
