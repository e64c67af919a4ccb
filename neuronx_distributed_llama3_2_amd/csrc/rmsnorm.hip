// RMSNorm forward / backward for CDNA4, optionally fused with the residual add of a pre-norm
// transformer block.  Replaces the reference's fp64 LlamaRMSNorm
// (examples/training/llama/modeling_llama_nxd.py:134-149) and the inference RmsNorm custom call
// (examples/inference/modules/custom_calls.py:5-16).
//
//   fwd:  h = x (+ residual);  y = h * rsqrt(mean(h^2) + eps) * w        (bf16 io, fp32 math)
//   bwd:  dh = rstd * (dy*w - xhat * mean(dy*w*xhat)) (+ dres);  dw = sum_rows dy * xhat
//
// Memory-bound: one row per workgroup, 16-byte vector loads (Guideline 13), the row stays in
// registers between the reduction and the normalisation (no re-read).  dw partials are written
// per workgroup ([G, H] fp32) and summed by a column-reduction kernel (no float atomics, so the
// result is bitwise reproducible).
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace nxd {
namespace rms {

template <int VPT>  // 8-element vectors per thread
__global__ void __launch_bounds__(256) fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                  const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                  uint16_t* __restrict__ h_out, float* __restrict__ rstd_out,
                                                  int64_t rows, int H, float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const int nvec = H / 8;
  const uint16_t* xr = x + row * H;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      u32x4_t xv = *reinterpret_cast<const u32x4_t*>(xr + c * 8);
      unpack8(xv, v[i]);
      if (res) {
        float rv[8];
        unpack8(*reinterpret_cast<const u32x4_t*>(res + row * H + c * 8), rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + rv[j]));  // round like the stored h
        *reinterpret_cast<u32x4_t*>(h_out + row * H + c * 8) = pack8(v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  const float tot = block_sum(ss, red);
  const float rstd = rsqrtf(tot / (float)H + eps);
  if (threadIdx.x == 0 && rstd_out) rstd_out[row] = rstd;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float wv[8], o[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(w + c * 8), wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wv[j];
      *reinterpret_cast<u32x4_t*>(y + row * H + c * 8) = pack8(o);
    }
  }
}

// grid-stride over rows; each workgroup accumulates its dw partial in registers.  PIPE: the next
// row's h / dy / dres vectors are loaded before this row's reduction barrier, so a workgroup's
// rows no longer pay one HBM round trip each (512 workgroups x 4 waves = 2 waves per SIMD: the
// per-row latency, not bandwidth, set the time).
template <int VPT, bool PIPE>
__global__ void __launch_bounds__(256) bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ h,
                                                  const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                                                  const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
                                                  float* __restrict__ dw_part, int64_t rows, int H) {
  __shared__ float red[16];
  const int nvec = H / 8;
  float wv[VPT][8], dwa[VPT][8];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwa[i][j] = 0.f;
    if (c < nvec) unpack8(*reinterpret_cast<const u32x4_t*>(w + c * 8), wv[i]);
  }
  u32x4_t hn[VPT], dn[VPT], rn[VPT];
  auto load_row = [&](int64_t row) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
        hn[i] = *reinterpret_cast<const u32x4_t*>(h + row * H + c * 8);
        dn[i] = *reinterpret_cast<const u32x4_t*>(dy + row * H + c * 8);
        if (dres) rn[i] = *reinterpret_cast<const u32x4_t*>(dres + row * H + c * 8);
      }
    }
  };
  if (PIPE && (int64_t)blockIdx.x < rows) load_row(blockIdx.x);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    u32x4_t hc[VPT], dc[VPT], rc[VPT];
    if (!PIPE) load_row(row);
#pragma unroll
    for (int i = 0; i < VPT; ++i) { hc[i] = hn[i]; dc[i] = dn[i]; rc[i] = rn[i]; }
    if (PIPE && row + gridDim.x < rows) load_row(row + gridDim.x);
    const float rs = rstd[row];
    float xh[VPT][8], g[VPT][8];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
        float hv[8], dv[8];
        unpack8(hc[i], hv);
        unpack8(dc[i], dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = hv[j] * rs;
          g[i][j] = dv[j] * wv[i][j];
          dot += g[i][j] * xh[i][j];
          dwa[i][j] += dv[j] * xh[i][j];
        }
      }
    }
    const float mean = block_sum(dot, red) / (float)H;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[i][j] - xh[i][j] * mean);
        if (dres) {
          float rv[8];
          unpack8(rc[i], rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rv[j];
        }
        *reinterpret_cast<u32x4_t*>(dx + row * H + c * 8) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float* dst = dw_part + (int64_t)blockIdx.x * H + c * 8;
      *reinterpret_cast<f32x4_t*>(dst) = f32x4_t{dwa[i][0], dwa[i][1], dwa[i][2], dwa[i][3]};
      *reinterpret_cast<f32x4_t*>(dst + 4) = f32x4_t{dwa[i][4], dwa[i][5], dwa[i][6], dwa[i][7]};
    }
  }
}

// dw[c] = sum_g part[g][c]  (fp32 out; optionally accumulated into an fp32 main_grad).
// 32 columns x 8 row-groups per workgroup (H/32 workgroups), LDS reduction of the 8 partials.
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ part, float* __restrict__ out, int G, int H,
                                                    int accumulate) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < H)
    for (int gi = rg; gi < G; gi += 8) s += part[(int64_t)gi * H + c];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < H) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][cl];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// ---- row-per-wave kernels (H a multiple of 512, H <= 8192: every Llama width to 70B) ----------
// One wave owns one row (SPLIT = 1, H <= 4096) or one half of it (SPLIT = 2, H 4608 .. 8192: the
// 70B hidden size); lane l holds the 16-byte vectors l, l+64, ... of its slice (VPL = H / 512 / SPLIT
// of them, each wave-instruction one contiguous KiB), so a row's sum of squares / dot product is a
// wave reduction (plus, at SPLIT = 2, one LDS exchange between the two waves of the row and one
// workgroup barrier per row step) and the register footprint stays that of a 4096-wide row.  The
// one-row-per-workgroup kernels above paid two block barriers per row and kept little in flight:
// the backward measured 1.98 TB/s at 8192 x 4096 (profiles/r4_rmsnorm_bwd_pipe_ab.txt), and its
// 128-workgroup column sum of 512 per-workgroup partials was latency-bound beside concurrent work.
template <int VPL, bool RES, int SPLIT>
__global__ void __launch_bounds__(256) fwd_rows_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                       const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                       uint16_t* __restrict__ h_out, float* __restrict__ rstd_out,
                                                       int64_t rows, int H, float eps) {
  constexpr int RPW = 4 / SPLIT;   // rows per workgroup step
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int part = wave % SPLIT, slot = wave / SPLIT;
  const int col0 = part * VPL * 512 + lane * 8;
  u32x4_t wv[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) wv[i] = *reinterpret_cast<const u32x4_t*>(w + col0 + i * 512);
  int step = 0;
  // the loop bound is workgroup-uniform (every wave reaches every barrier); rows past the end idle
  for (int64_t base = (int64_t)blockIdx.x * RPW; base < rows; base += (int64_t)gridDim.x * RPW, ++step) {
    const int64_t row = base + slot;
    const bool valid = row < rows;
    const int64_t off = row * H + col0;
    u32x4_t xv[VPL], rv[VPL];
    float ss = 0.f;
    if (valid) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        xv[i] = *reinterpret_cast<const u32x4_t*>(x + off + i * 512);
        if (RES) rv[i] = *reinterpret_cast<const u32x4_t*>(res + off + i * 512);
      }
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        float v[8];
        unpack8(xv[i], v);
        if (RES) {
          float r[8];
          unpack8(rv[i], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] + r[j]));   // round like the stored h
          xv[i] = pack8(v);
          *reinterpret_cast<u32x4_t*>(h_out + off + i * 512) = xv[i];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
      }
    }
    ss = wave_sum(ss);
    if constexpr (SPLIT > 1) {
      // the row's two halves meet in LDS (double-buffered by step parity: one barrier per step)
      if (lane == 0) red[step & 1][wave] = ss;
      __syncthreads();
      ss = red[step & 1][slot * SPLIT] + red[step & 1][slot * SPLIT + 1];
    }
    if (!valid) continue;
    const float rstd = rsqrtf(ss / (float)H + eps);
    if (lane == 0 && part == 0 && rstd_out) rstd_out[row] = rstd;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float v[8], g[8];
      unpack8(xv[i], v);
      unpack8(wv[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * rstd * g[j];
      *reinterpret_cast<u32x4_t*>(y + off + i * 512) = pack8(v);
    }
  }
}

// 8 waves per workgroup, one workgroup per CU (G <= 256 workgroups, grid-stride over rows); each lane
// accumulates dw for its 8 * VPL columns in registers over all of its wave's rows; the waves' sums
// are added through LDS (fixed order) into ONE partial row per workgroup, so the column sum reads
// G <= 256 rows instead of 512.  Bitwise reproducible (no atomics, fixed row -> wave assignment).
template <int VPL, bool RES, int SPLIT>
__global__ void __launch_bounds__(512) bwd_rows_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ h,
                                                       const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                                                       const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
                                                       float* __restrict__ dw_part, int64_t rows, int H) {
  constexpr int RPW = 8 / SPLIT;
  __shared__ float red[8][520];   // one 512-column slice of the 8 waves' dw sums (+8 pad)
  __shared__ float dred[2][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int part = wave % SPLIT, slot = wave / SPLIT;
  const int col0 = part * VPL * 512 + lane * 8;
  u32x4_t wv[VPL];
  float dwa[VPL][8];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    wv[i] = *reinterpret_cast<const u32x4_t*>(w + col0 + i * 512);
#pragma unroll
    for (int j = 0; j < 8; ++j) dwa[i][j] = 0.f;
  }
  int step = 0;
  for (int64_t base = (int64_t)blockIdx.x * RPW; base < rows; base += (int64_t)gridDim.x * RPW, ++step) {
    const int64_t row = base + slot;
    const bool valid = row < rows;
    const int64_t off = row * H + col0;
    u32x4_t hv[VPL], dv[VPL], rv[VPL];
    float rs = 0.f, dot = 0.f;
    if (valid) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        hv[i] = *reinterpret_cast<const u32x4_t*>(h + off + i * 512);
        dv[i] = *reinterpret_cast<const u32x4_t*>(dy + off + i * 512);
        if (RES) rv[i] = *reinterpret_cast<const u32x4_t*>(dres + off + i * 512);
      }
      rs = rstd[row];
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        float a[8], d[8], g[8];
        unpack8(hv[i], a);
        unpack8(dv[i], d);
        unpack8(wv[i], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = a[j] * rs;
          dot += d[j] * g[j] * xh;
          dwa[i][j] += d[j] * xh;
        }
      }
    }
    dot = wave_sum(dot);
    if constexpr (SPLIT > 1) {
      if (lane == 0) dred[step & 1][wave] = dot;
      __syncthreads();
      dot = dred[step & 1][slot * SPLIT] + dred[step & 1][slot * SPLIT + 1];
    }
    if (!valid) continue;
    const float mean = dot / (float)H;
    // re-unpack from the packed registers below instead of keeping the first pass's 3 x 8 x VPL
    // unpacked floats alive (at VPL = 8 that spilled ~100 VGPRs)
#pragma unroll
    for (int i = 0; i < VPL; ++i) asm volatile("" : "+v"(hv[i]), "+v"(dv[i]), "+v"(wv[i]));
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float a[8], d[8], g[8], o[8];
      unpack8(hv[i], a);
      unpack8(dv[i], d);
      unpack8(wv[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rs * (d[j] * g[j] - a[j] * rs * mean);
      if (RES) {
        float r[8];
        unpack8(rv[i], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += r[j];
      }
      *reinterpret_cast<u32x4_t*>(dx + off + i * 512) = pack8(o);
    }
  }
  // workgroup partial: slice i (columns [512 i, 512 i + 512) of each wave's part) of the waves' sums,
  // the waves of one part added in wave order
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = dwa[i][j];
    __syncthreads();
    const int c = threadIdx.x;   // 512 threads = the slice's 512 columns
#pragma unroll
    for (int pp = 0; pp < SPLIT; ++pp) {
      float t = 0.f;
#pragma unroll
      for (int q = pp; q < 8; q += SPLIT) t += red[q][c];
      dw_part[(int64_t)blockIdx.x * H + pp * VPL * 512 + i * 512 + c] = t;
    }
  }
}

// dw[c] (+)= sum_g part[g][c] over G <= 256 partial rows: 64 columns per workgroup, 16 row lanes x 16
// float4 column quads, every row load of a thread in flight at once (G / 16 <= 16), then a fixed-order
// LDS sum of the 16 row lanes.
__global__ void __launch_bounds__(256) colsum4_kernel(const float* __restrict__ part, float* __restrict__ out, int G,
                                                      int H, int accumulate) {
  __shared__ f32x4_t red[16][17];
  const int q = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + q * 4;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  if (c < H) {
#pragma unroll 16
    for (int g = rl; g < G; g += 16) s += *reinterpret_cast<const f32x4_t*>(part + (int64_t)g * H + c);
  }
  red[rl][q] = s;
  __syncthreads();
  if (rl == 0 && c < H) {
    f32x4_t t = red[0][q];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += red[i][q];
#pragma unroll
    for (int j = 0; j < 4; ++j) out[c + j] = accumulate ? out[c + j] + t[j] : t[j];   // out: any 4-B alignment
  }
}

// NXD_RMS_ROWS=0 (or rmsnorm_set_rows_path(0)): the one-row-per-workgroup kernels (A/B)
static int g_rows_mode = -1;
static bool rows_path(int H) {
  if (g_rows_mode < 0) {
    const char* e = getenv("NXD_RMS_ROWS");
    g_rows_mode = e ? (atoi(e) != 0) : 1;
  }
  return g_rows_mode && H % 512 == 0 && H >= 512 && H <= 8192 && (H <= 4096 || H % 1024 == 0);
}

}  // namespace rms

int rmsnorm_fwd_launch(const void* x, const void* res, const void* w, void* y, void* h_out, float* rstd, int64_t rows,
                       int H, float eps, hipStream_t stream) {
  using namespace rms;
  if (H % 8 != 0) return -1;
  if (rows_path(H)) {
    if (rows == 0) return 0;
    const int g = (int)std::min<int64_t>(ceil_div64(rows, H <= 4096 ? 4 : 2), 2048);
#define RMS_FWD_ROWS(V, S)                                                                                     \
  do {                                                                                                         \
    if (res)                                                                                                   \
      hipLaunchKernelGGL((fwd_rows_kernel<V, true, S>), dim3(g), dim3(256), 0, stream, (const uint16_t*)x,      \
                         (const uint16_t*)res, (const uint16_t*)w, (uint16_t*)y, (uint16_t*)h_out, rstd, rows, H, eps); \
    else                                                                                                       \
      hipLaunchKernelGGL((fwd_rows_kernel<V, false, S>), dim3(g), dim3(256), 0, stream, (const uint16_t*)x,     \
                         (const uint16_t*)res, (const uint16_t*)w, (uint16_t*)y, (uint16_t*)h_out, rstd, rows, H, eps); \
  } while (0)
    switch (H / 512) {
      case 1: RMS_FWD_ROWS(1, 1); break;
      case 2: RMS_FWD_ROWS(2, 1); break;
      case 3: RMS_FWD_ROWS(3, 1); break;
      case 4: RMS_FWD_ROWS(4, 1); break;
      case 5: RMS_FWD_ROWS(5, 1); break;
      case 6: RMS_FWD_ROWS(6, 1); break;
      case 7: RMS_FWD_ROWS(7, 1); break;
      case 8: RMS_FWD_ROWS(8, 1); break;
      case 10: RMS_FWD_ROWS(5, 2); break;
      case 12: RMS_FWD_ROWS(6, 2); break;
      case 14: RMS_FWD_ROWS(7, 2); break;
      default: RMS_FWD_ROWS(8, 2); break;   // 16: H = 8192
    }
#undef RMS_FWD_ROWS
    return (int)hipGetLastError();
  }
  const int nvec = H / 8;
  const int threads = nvec >= 256 ? 256 : ((nvec + 63) / 64) * 64;
  const int vpt = (nvec + threads - 1) / threads;
  const dim3 grid((unsigned)rows), block(threads);
#define RMS_FWD(V) hipLaunchKernelGGL(fwd_kernel<V>, grid, block, 0, stream, (const uint16_t*)x, (const uint16_t*)res, \
                                      (const uint16_t*)w, (uint16_t*)y, (uint16_t*)h_out, rstd, rows, H, eps)
  if (vpt <= 1) RMS_FWD(1);
  else if (vpt <= 2) RMS_FWD(2);
  else if (vpt <= 4) RMS_FWD(4);
  else if (vpt <= 8) RMS_FWD(8);
  else return -2;
#undef RMS_FWD
  return (int)hipGetLastError();
}

void rmsnorm_set_rows_path(int on) { rms::g_rows_mode = on ? 1 : 0; }

// dw_part must hold G*H floats where G = rmsnorm_bwd_num_partials(rows)
int rmsnorm_bwd_num_partials(int64_t rows) { return (int)(rows < 512 ? rows : 512); }

int rmsnorm_bwd_launch(const void* dy, const void* h, const void* w, const float* rstd, const void* dres, void* dx,
                       float* dw_part, float* dw, int accumulate_dw, int64_t rows, int H, hipStream_t stream) {
  using namespace rms;
  if (H % 8 != 0) return -1;
  if (rows_path(H)) {
    // G <= 256 <= rmsnorm_bwd_num_partials(rows) for rows >= 256 (and ceil(rows / 8) <= rows below)
    const int G = (int)std::min<int64_t>(ceil_div64(rows, H <= 4096 ? 8 : 4), 256);
    if (G == 0) return 0;
#define RMS_BWD_ROWS(V, S)                                                                                     \
  do {                                                                                                         \
    if (dres)                                                                                                  \
      hipLaunchKernelGGL((bwd_rows_kernel<V, true, S>), dim3(G), dim3(512), 0, stream, (const uint16_t*)dy,     \
                         (const uint16_t*)h, (const uint16_t*)w, rstd, (const uint16_t*)dres, (uint16_t*)dx, dw_part, \
                         rows, H);                                                                             \
    else                                                                                                       \
      hipLaunchKernelGGL((bwd_rows_kernel<V, false, S>), dim3(G), dim3(512), 0, stream, (const uint16_t*)dy,    \
                         (const uint16_t*)h, (const uint16_t*)w, rstd, (const uint16_t*)dres, (uint16_t*)dx, dw_part, \
                         rows, H);                                                                             \
  } while (0)
    switch (H / 512) {
      case 1: RMS_BWD_ROWS(1, 1); break;
      case 2: RMS_BWD_ROWS(2, 1); break;
      case 3: RMS_BWD_ROWS(3, 1); break;
      case 4: RMS_BWD_ROWS(4, 1); break;
      case 5: RMS_BWD_ROWS(5, 1); break;
      case 6: RMS_BWD_ROWS(6, 1); break;
      case 7: RMS_BWD_ROWS(7, 1); break;
      case 8: RMS_BWD_ROWS(8, 1); break;
      case 10: RMS_BWD_ROWS(5, 2); break;
      case 12: RMS_BWD_ROWS(6, 2); break;
      case 14: RMS_BWD_ROWS(7, 2); break;
      default: RMS_BWD_ROWS(8, 2); break;   // 16: H = 8192
    }
#undef RMS_BWD_ROWS
    hipLaunchKernelGGL(colsum4_kernel, dim3((H + 63) / 64), dim3(256), 0, stream, dw_part, dw, G, H, accumulate_dw);
    return (int)hipGetLastError();
  }
  const int nvec = H / 8;
  const int threads = nvec >= 256 ? 256 : ((nvec + 63) / 64) * 64;
  const int vpt = (nvec + threads - 1) / threads;
  const int G = rmsnorm_bwd_num_partials(rows);
  if (G == 0) return 0;
  const dim3 grid(G), block(threads);
  // NXD_RMS_BWD_PIPE=0: the unpipelined loop (A/B; identical results)
  static const bool pipe = [] {
    const char* e = getenv("NXD_RMS_BWD_PIPE");
    return e ? atoi(e) != 0 : true;
  }();
#define RMS_BWD(V)                                                                                          \
  do {                                                                                                      \
    if (pipe)                                                                                               \
      hipLaunchKernelGGL((bwd_kernel<V, true>), grid, block, 0, stream, (const uint16_t*)dy, (const uint16_t*)h,  \
                         (const uint16_t*)w, rstd, (const uint16_t*)dres, (uint16_t*)dx, dw_part, rows, H);       \
    else                                                                                                    \
      hipLaunchKernelGGL((bwd_kernel<V, false>), grid, block, 0, stream, (const uint16_t*)dy, (const uint16_t*)h, \
                         (const uint16_t*)w, rstd, (const uint16_t*)dres, (uint16_t*)dx, dw_part, rows, H);       \
  } while (0)
  if (vpt <= 1) RMS_BWD(1);
  else if (vpt <= 2) RMS_BWD(2);
  else if (vpt <= 4) RMS_BWD(4);
  else if (vpt <= 8) RMS_BWD(8);
  else return -2;
#undef RMS_BWD
  hipLaunchKernelGGL(colsum_kernel, dim3((H + 31) / 32), dim3(256), 0, stream, dw_part, dw, G, H, accumulate_dw);
  return (int)hipGetLastError();
}

}  // namespace nxd
