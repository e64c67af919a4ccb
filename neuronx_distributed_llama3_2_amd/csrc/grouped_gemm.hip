// Grouped (ragged-M) bf16 GEMMs for the dropless MoE expert MLPs on gfx950 MFMA.
//
// Tokens are sorted by expert on the device (argsort of the router's top-k choices); expert e
// owns rows offs[e] .. offs[e+1] of the sorted activations.  The group sizes never travel to the
// host: every launch is sized for the worst case (ceil(M / 128) + E row tiles) and each workgroup
// finds its (expert, row tile) from the device-resident offsets, so the MoE layer has no
// device->host sync and can be captured in a hipGraph (reference: modules/moe/expert_mlps.py
// :169-265 runs every token through every expert, or drops by capacity; this computes only the
// chosen rows).
//
// Three products, one kernel template (C = A.B, reduction over k):
//   FWD   y[m, n]     = x[m, :]  . W[e][:, n]        A row-major [M][K],  B = W[e] stored [K][N]
//   DGRAD dx[m, k]    = dy[m, :] . W[e][k, :]^T      A row-major [M][N],  B = W[e] stored [K][N] read as [n][k]
//   WGRAD dW[e][k, n] (+)= sum_{m in e} x[m, k] dy[m, n]    A = x^T (stored [m][k]), B = dy stored [m][n]
// Workgroup = 4 waves, 128 x 128 output tile (2 x 2 waves of 64 x 64 = 2 x 2 v_mfma_f32_32x32x16_bf16
// tiles each), K-step 64, two LDS buffers (64 KiB): full reduction tiles go global -> LDS by
// LDS-DMA (tile t+1 in flight while tile t runs its 16 MFMAs per wave), a ragged reduction tail
// by zero-filling register staging; workgroups walk the tile grid in L2-sized bands
// (band_raster).  Mixtral shapes: 0.55-0.74 -> 0.80-0.84 PF/s fwd / dgrad (profiles/r2_moe_layer_v1.md).  Operands consumed along their contiguous axis are read with
// ds_read_b128 from a [row][64] image (16-B chunk XOR (row>>1)&7: conflict-free over 16 lanes);
// operands stored reduction-major are read with the hardware transpose ds_read_b64_tr_b16 from a
// [k][128] image (chunk XOR (k&3)<<2: the four rows of one transposed read and the two column
// blocks of a 32-lane half land on disjoint banks).
#include "common.h"

namespace nxd {
namespace gg {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;   // 16 KiB: one operand tile (both images)

enum Mode { FWD = 0, DGRAD = 1, WGRAD = 2 };

struct Params {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  const int* offs;      // [E + 1] device offsets of the expert groups in the sorted rows
  int E;
  int M;                // rows of the sorted activations
  int K;                // reduction length (FWD: in features, DGRAD: out features of W); WGRAD: rows of dW
  int N;                // output columns
  int lda, ldb, ldc;
  int64_t b_estride;    // elements between experts' weights (FWD / DGRAD)
  int64_t c_estride;    // elements between experts' dW (WGRAD)
  int n_tiles, r_tiles; // output tiles along N, and along rows (WGRAD: K / BM) or row-tile slots
  int accumulate;       // WGRAD: dW += (fp32 main_grad) instead of dW =
  int band;             // row tiles per raster band (band_raster)
};

typedef __attribute__((address_space(3))) short4_t lds_short4_t;

// byte offsets inside one 16 KiB image
__device__ __forceinline__ int row_img(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }   // [128][64]
__device__ __forceinline__ int tr_img(int k, int c) { return k * 256 + 16 * (c ^ ((k & 3) << 2)); }     // [64][128]

// Stage a [128 rows][64 k] tile whose rows are contiguous along k: 1024 16-B chunks, 4 per thread.
__device__ __forceinline__ void load_rows(u32x4_t* v, const uint16_t* base, int ld, int rows_valid, int k0, int K) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + NT * i, r = idx >> 3, c = idx & 7;
    const int k = k0 + 8 * c;
    v[i] = u32x4_t{0, 0, 0, 0};
    if (r < rows_valid && k < K) v[i] = *reinterpret_cast<const u32x4_t*>(base + (int64_t)r * ld + k);
  }
}
__device__ __forceinline__ void store_rows(char* img, const u32x4_t* v) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + NT * i, r = idx >> 3, c = idx & 7;
    *reinterpret_cast<u32x4_t*>(img + row_img(r, c)) = v[i];
  }
}
// Stage a [64 k][128 cols] tile stored k-major (rows contiguous along the output columns).
__device__ __forceinline__ void load_tr(u32x4_t* v, const uint16_t* base, int ld, int k_valid, int c0, int C) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + NT * i, k = idx >> 4, c = idx & 15;
    const int col = c0 + 8 * c;
    v[i] = u32x4_t{0, 0, 0, 0};
    if (k < k_valid && col < C) v[i] = *reinterpret_cast<const u32x4_t*>(base + (int64_t)k * ld + col);
  }
}
__device__ __forceinline__ void store_tr(char* img, const u32x4_t* v) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + NT * i, k = idx >> 4, c = idx & 15;
    *reinterpret_cast<u32x4_t*>(img + tr_img(k, c)) = v[i];
  }
}

// LDS-DMA staging (global_load_lds_dwordx4: 1 KiB per wave-instruction, written lane-linearly at
// M0): the XOR swizzle of the LDS images is applied to each lane's SOURCE address instead, so the
// tile never passes through VGPRs or the ds_write path (whose VGPR->LDS transfer, ~79 B/clk/CU,
// cost more LDS cycles per k-step than the MFMA fragment reads).  Issued from inline asm so the
// compiler does not wait for it before every transposed LDS read; completion is a manual
// vmcnt(0) before the k-step's barrier.  Rows / columns past the valid range re-read a valid
// chunk (their outputs are never stored); reduction tails take the zero-filling VGPR path.
typedef __attribute__((address_space(3))) char lds_char_t;
__device__ __forceinline__ uint32_t lds_addr(const char* q) { return (uint32_t)(uintptr_t)(const lds_char_t*)q; }
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_dst) {
  uint32_t sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(sv) : "v"(src), "s"(lds_dst) : "memory");
}
// [128 rows][64 k] row image: piece P (1 KiB) = rows 8P .. 8P + 7; lane l -> row 8P + l / 8, slot l % 8.
__device__ __forceinline__ void dma_rows(uint32_t img, const uint16_t* base, int ld, int rows_valid, int k0) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = w * 4 + i, r = piece * 8 + (l >> 3), c = (l & 7) ^ ((r >> 1) & 7);
    const int rr = min(r, rows_valid - 1);
    dma16(base + (int64_t)rr * ld + k0 + 8 * c, __builtin_amdgcn_readfirstlane(img + piece * 1024));
  }
}
// [64 k][128 cols] k-major image: piece P = k rows 4P .. 4P + 3; lane l -> k 4P + l / 16, slot l % 16.
__device__ __forceinline__ void dma_tr(uint32_t img, const uint16_t* base, int ld, int c0, int C) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = w * 4 + i, k = piece * 4 + (l >> 4), c = (l & 15) ^ ((k & 3) << 2);
    const int col = min(c0 + 8 * c, C - 8);
    dma16(base + (int64_t)k * ld + col, __builtin_amdgcn_readfirstlane(img + piece * 1024));
  }
}

// 32x32x16 operand fragment of rows [rbase, rbase + 32), k-step s: lane (r = l & 31, h = l >> 5)
// needs element j = 0..7 at (row rbase + r, k 16 s + 8 h + j).
__device__ __forceinline__ bf16x8_t frag_rows(const char* img, int rbase, int s) {
  const int l = threadIdx.x & 63;
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4_t*>(img + row_img(rbase + (l & 31), 2 * s + (l >> 5))));
}
// Same fragment from a k-major image: two transposed reads of 4 k-rows x 16 columns per 16-lane
// group; lane 4q + p of group g supplies (k row 16 s + 8 h + q (+4), column rbase + 16 (g & 1) + 4 p).
__device__ __forceinline__ bf16x8_t frag_tr(const char* img, int rbase, int s) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int h = g >> 1;
  const int col = rbase + 16 * (g & 1) + 4 * p;
  const int k = 16 * s + 8 * h + q;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_short4_t*)(img + tr_img(k, col >> 3) + 8 * (p & 1)));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_short4_t*)(img + tr_img(k + 4, col >> 3) + 8 * (p & 1)));
  const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, a8);
}

// L2-aware raster: walk the (row tile, column tile) grid in bands of kBand row tiles, column-major
// inside a band, so the workgroups resident on one XCD at a time (consecutive ids after
// xcd_remap) share both A row tiles and B column tiles in that XCD's 4 MiB L2.  Row-major order
// re-streamed the whole weight matrix W[e] from HBM once per row tile.
__device__ __forceinline__ void band_raster(int id, int rows, int cols, int kBand, int& r, int& c) {
  const int band = id / (kBand * cols), within = id - band * kBand * cols;
  const int h = min(kBand, rows - band * kBand);
  r = band * kBand + within % h;
  c = within / h;
}

template <int MODE, bool DMA>
__global__ void __launch_bounds__(NT) grouped_gemm_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];   // [buf][A | B]
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;

  int e = 0, row0 = 0, row_end = 0, n0 = 0, red0 = 0, red_end = 0;
  if (MODE == WGRAD) {
    const int per_e = p.r_tiles * p.n_tiles;
    e = id / per_e;
    const int rem = id - e * per_e;
    int rt, ct;
    band_raster(rem, p.r_tiles, p.n_tiles, p.band, rt, ct);
    row0 = rt * BM;                           // rows of dW (= input features)
    n0 = ct * BN;
    row_end = p.K;
    int lo = min(max(p.offs[e], 0), p.M), hi = min(max(p.offs[e + 1], 0), p.M);
    red0 = lo;
    red_end = max(hi, lo);
  } else {
    int slot, ct;
    band_raster(id, p.r_tiles, p.n_tiles, p.band, slot, ct);
    n0 = ct * BN;
    // locate (expert, row tile) of this slot from the device offsets (E scalar iterations)
    int acc = 0, prev = 0;
    e = -1;
    for (int x = 0; x < p.E; ++x) {
      int lo = min(max(p.offs[x], prev), p.M), hi = min(max(p.offs[x + 1], lo), p.M);
      prev = hi;
      const int tiles = (hi - lo + BM - 1) / BM;
      if (slot < acc + tiles) {
        e = x;
        row0 = lo + (slot - acc) * BM;
        row_end = hi;
        break;
      }
      acc += tiles;
    }
    if (e < 0) return;                        // past the last real tile: the whole workgroup exits
    red0 = 0;
    red_end = p.K;
  }

  const uint16_t* a_base;
  const uint16_t* b_base;
  if (MODE == FWD) {
    a_base = p.a + (int64_t)row0 * p.lda;                  // x rows, contiguous along k
    b_base = p.b + (int64_t)e * p.b_estride;               // W[e] [K][N], k-major
  } else if (MODE == DGRAD) {
    a_base = p.a + (int64_t)row0 * p.lda;                  // dy rows, contiguous along n (= reduction)
    b_base = p.b + (int64_t)e * p.b_estride + (int64_t)n0 * p.ldb;   // W[e] rows = output columns
  } else {
    a_base = p.a;                                           // x [m][k]: the tile's rows are columns of x
    b_base = p.b;                                           // dy [m][n]
  }
  const int rows_valid = row_end - row0;

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16_t{0};

  const int n_k = (red_end - red0 + BK - 1) / BK;
  u32x4_t va[4], vb[4];
  auto load = [&](int t) {
    const int k0 = red0 + t * BK;
    if (MODE == WGRAD) {
      load_tr(va, a_base + (int64_t)k0 * p.lda, p.lda, red_end - k0, row0, p.K);
      load_tr(vb, b_base + (int64_t)k0 * p.ldb, p.ldb, red_end - k0, n0, p.N);
    } else if (MODE == FWD) {
      load_rows(va, a_base, p.lda, rows_valid, k0, p.K);
      load_tr(vb, b_base + (int64_t)k0 * p.ldb, p.ldb, p.K - k0, n0, p.N);
    } else {
      load_rows(va, a_base, p.lda, rows_valid, k0, p.K);
      load_rows(vb, b_base, p.ldb, p.N - n0, k0, p.K);
    }
  };
  auto store = [&](int buf) {
    char* ia = smem + buf * 2 * TILE_BYTES;
    char* ib = ia + TILE_BYTES;
    if (MODE == WGRAD) store_tr(ia, va); else store_rows(ia, va);
    if (MODE == DGRAD) store_rows(ib, vb); else store_tr(ib, vb);
  };
  // full reduction tile t straight into LDS buffer `buf`
  auto dma = [&](int t, int buf) {
    const int k0 = red0 + t * BK;
    const uint32_t ia = lds_addr(smem + buf * 2 * TILE_BYTES), ib = ia + TILE_BYTES;
    if (MODE == WGRAD) {
      dma_tr(ia, a_base + (int64_t)k0 * p.lda, p.lda, row0, p.K);
      dma_tr(ib, b_base + (int64_t)k0 * p.ldb, p.ldb, n0, p.N);
    } else if (MODE == FWD) {
      dma_rows(ia, a_base, p.lda, rows_valid, k0);
      dma_tr(ib, b_base + (int64_t)k0 * p.ldb, p.ldb, n0, p.N);
    } else {
      dma_rows(ia, a_base, p.lda, rows_valid, k0);
      dma_rows(ib, b_base, p.ldb, p.N - n0, k0);
    }
  };
  // tiles [0, n_full) cover BK full reduction steps; a ragged last tile is zero-filled through VGPRs
  const int n_full = DMA ? (red_end - red0) / BK : 0;

  if (n_k > 0) {
    if (n_full > 0) {
      dma(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      load(0);
      store(0);
    }
    __syncthreads();
  }
  for (int t = 0; t < n_k; ++t) {
    const int buf = t & 1;
    const bool next_dma = t + 1 < n_full, next_stage = t + 1 < n_k && !next_dma;
    if (next_dma) dma(t + 1, buf ^ 1);
    if (next_stage) load(t + 1);
    const char* ia = smem + buf * 2 * TILE_BYTES;
    const char* ib = ia + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = (MODE == WGRAD) ? frag_tr(ia, wm * 64 + 32 * i, s) : frag_rows(ia, wm * 64 + 32 * i, s);
        bfr[i] = (MODE == DGRAD) ? frag_rows(ib, wn * 64 + 32 * i, s) : frag_tr(ib, wn * 64 + 32 * i, s);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (next_stage) store(buf ^ 1);
    if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: acc element v of tile (i, j) is (row (v & 3) + 8 (v >> 2) + 4 (lane >> 5), col lane & 31)
  const int ccol = lane & 31, rsub = 4 * (lane >> 5);
  if (MODE == WGRAD && p.accumulate) {
    // dW += acc: batch the 32 fp32 reads of a tile row pair before any store (a load after a store
    // to a possibly aliasing address is not hoisted, which serialised 64 HBM round trips per lane)
    float* cbase = reinterpret_cast<float*>(p.c) + (int64_t)e * p.c_estride;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float old[2][16];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + 32 * j + ccol;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * 64 + 32 * i + (v & 3) + 8 * (v >> 2) + rsub;
          old[j][v] = (col < p.N && r < rows_valid) ? cbase[(int64_t)(row0 + r) * p.ldc + col] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + 32 * j + ccol;
        if (col >= p.N) continue;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * 64 + 32 * i + (v & 3) + 8 * (v >> 2) + rsub;
          if (r < rows_valid) cbase[(int64_t)(row0 + r) * p.ldc + col] = old[j][v] + acc[i][j][v];
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + 32 * j + ccol;
      if (col >= p.N) continue;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int r = wm * 64 + 32 * i + (v & 3) + 8 * (v >> 2) + rsub;
        if (r >= rows_valid) continue;
        const int64_t grow = row0 + r;
        if (MODE == WGRAD) {
          float* c = reinterpret_cast<float*>(p.c) + (int64_t)e * p.c_estride + grow * p.ldc + col;
          *c = p.accumulate ? (*c + acc[i][j][v]) : acc[i][j][v];
        } else {
          reinterpret_cast<uint16_t*>(p.c)[grow * p.ldc + col] = f2bf(acc[i][j][v]);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Large-tile variant: 256 x 256 output tile per workgroup, 4 waves of 128 x 128 (4 x 4 MFMA tiles,
// 256 fp32 accumulators per lane in AGPRs), BK 64, two 64 KiB LDS stages filled by LDS-DMA one
// tile ahead, one workgroup per CU.  A k-step is 64 MFMAs per wave (~850 ns), long enough to
// cover the LDS-DMA latency that bounds the 128 x 128 kernel (2 x its FLOP per byte staged).
// Reduction tails read a zero chunk (g_zero16); rows / columns past the valid range re-read a
// valid chunk (never stored).
constexpr int BB = 256;                         // tile rows = tile cols
constexpr int BIG_TILE = BB * BK * 2;           // 32 KiB per operand image
__device__ __attribute__((aligned(16))) uint32_t g_zero16[4];   // zero-initialised device global

// k-major [64 k][256 cols] image: 512-B rows, chunk XOR (k & 3) << 2 (as tr_img)
__device__ __forceinline__ int trb_img(int k, int c) { return k * 512 + 16 * (c ^ ((k & 3) << 2)); }
__device__ __forceinline__ bf16x8_t frag_trb(const char* img, int rbase, int s) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int h = g >> 1;
  const int col = rbase + 16 * (g & 1) + 4 * p;
  const int k = 16 * s + 8 * h + q;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_short4_t*)(img + trb_img(k, col >> 3) + 8 * (p & 1)));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_short4_t*)(img + trb_img(k + 4, col >> 3) + 8 * (p & 1)));
  const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, a8);
}
// [256 rows][64 k] row image (row_img): piece P = rows 8P .. 8P + 7, 8 pieces per wave
__device__ __forceinline__ void dma_rows_big(uint32_t img, const uint16_t* base, int ld, int rows_valid, int k0, int k_end) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = w * 8 + i, r = piece * 8 + (l >> 3), c = (l & 7) ^ ((r >> 1) & 7);
    const int rr = min(r, rows_valid - 1), k = k0 + 8 * c;
    const void* src = k < k_end ? (const void*)(base + (int64_t)rr * ld + k) : (const void*)g_zero16;
    dma16(src, __builtin_amdgcn_readfirstlane(img + piece * 1024));
  }
}
// trb image: piece P = k rows 2P, 2P + 1; lane l -> k 2P + l / 32, slot l % 32
__device__ __forceinline__ void dma_tr_big(uint32_t img, const uint16_t* base, int ld, int c0, int C, int k_valid) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = w * 8 + i, k = piece * 2 + (l >> 5), c = (l & 31) ^ ((k & 3) << 2);
    const int col = min(c0 + 8 * c, C - 8);
    const void* src = k < k_valid ? (const void*)(base + (int64_t)k * ld + col) : (const void*)g_zero16;
    dma16(src, __builtin_amdgcn_readfirstlane(img + piece * 1024));
  }
}

template <int MODE>
__global__ void __launch_bounds__(NT, 1) grouped_gemm_big_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * BIG_TILE];   // [stage][A | B], 128 KiB
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;

  int e = 0, row0 = 0, row_end = 0, n0 = 0, red0 = 0, red_end = 0;
  if (MODE == WGRAD) {
    const int per_e = p.r_tiles * p.n_tiles;
    e = id / per_e;
    int rt, ct;
    band_raster(id - e * per_e, p.r_tiles, p.n_tiles, p.band, rt, ct);
    row0 = rt * BB;
    n0 = ct * BB;
    row_end = p.K;
    const int lo = min(max(p.offs[e], 0), p.M), hi = min(max(p.offs[e + 1], 0), p.M);
    red0 = lo;
    red_end = max(hi, lo);
  } else {
    int slot, ct;
    band_raster(id, p.r_tiles, p.n_tiles, p.band, slot, ct);
    n0 = ct * BB;
    int acc_t = 0, prev = 0;
    e = -1;
    for (int x = 0; x < p.E; ++x) {
      const int lo = min(max(p.offs[x], prev), p.M), hi = min(max(p.offs[x + 1], lo), p.M);
      prev = hi;
      const int tiles = (hi - lo + BB - 1) / BB;
      if (slot < acc_t + tiles) {
        e = x;
        row0 = lo + (slot - acc_t) * BB;
        row_end = hi;
        break;
      }
      acc_t += tiles;
    }
    if (e < 0) return;
    red0 = 0;
    red_end = p.K;
  }
  const uint16_t* a_base;
  const uint16_t* b_base;
  if (MODE == FWD) {
    a_base = p.a + (int64_t)row0 * p.lda;
    b_base = p.b + (int64_t)e * p.b_estride;
  } else if (MODE == DGRAD) {
    a_base = p.a + (int64_t)row0 * p.lda;
    b_base = p.b + (int64_t)e * p.b_estride + (int64_t)n0 * p.ldb;
  } else {
    a_base = p.a;
    b_base = p.b;
  }
  const int rows_valid = row_end - row0;

  f32x16_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16_t{0};

  const int n_k = (red_end - red0 + BK - 1) / BK;
  auto issue = [&](int t, int buf) {
    const int k0 = red0 + t * BK;
    const uint32_t ia = lds_addr(smem + buf * 2 * BIG_TILE), ib = ia + BIG_TILE;
    if (MODE == WGRAD) {
      dma_tr_big(ia, a_base + (int64_t)k0 * p.lda, p.lda, row0, p.K, red_end - k0);
      dma_tr_big(ib, b_base + (int64_t)k0 * p.ldb, p.ldb, n0, p.N, red_end - k0);
    } else if (MODE == FWD) {
      dma_rows_big(ia, a_base, p.lda, rows_valid, k0, p.K);
      dma_tr_big(ib, b_base + (int64_t)k0 * p.ldb, p.ldb, n0, p.N, p.K - k0);
    } else {
      dma_rows_big(ia, a_base, p.lda, rows_valid, k0, p.K);
      dma_rows_big(ib, b_base, p.ldb, p.N - n0, k0, p.K);
    }
  };
  if (n_k > 0) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < n_k; ++t) {
    const int buf = t & 1;
    if (t + 1 < n_k) issue(t + 1, buf ^ 1);
    const char* ia = smem + buf * 2 * BIG_TILE;
    const char* ib = ia + BIG_TILE;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = (MODE == WGRAD) ? frag_trb(ia, wm * 128 + 32 * i, s) : frag_rows(ia, wm * 128 + 32 * i, s);
        bfr[i] = (MODE == DGRAD) ? frag_rows(ib, wn * 128 + 32 * i, s) : frag_trb(ib, wn * 128 + 32 * i, s);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const int ccol = lane & 31, rsub = 4 * (lane >> 5);
  if (MODE == WGRAD) {
    float* cbase = reinterpret_cast<float*>(p.c) + (int64_t)e * p.c_estride;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // 16 reads in flight before the tile's 16 stores
        const int col = n0 + wn * 128 + 32 * j + ccol;
        float old[16];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * 128 + 32 * i + (v & 3) + 8 * (v >> 2) + rsub;
          old[v] = (p.accumulate && col < p.N && r < rows_valid) ? cbase[(int64_t)(row0 + r) * p.ldc + col] : 0.f;
        }
        if (col >= p.N) continue;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * 128 + 32 * i + (v & 3) + 8 * (v >> 2) + rsub;
          if (r < rows_valid) cbase[(int64_t)(row0 + r) * p.ldc + col] = old[v] + acc[i][j][v];
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 128 + 32 * j + ccol;
        if (col >= p.N) continue;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = wm * 128 + 32 * i + (v & 3) + 8 * (v >> 2) + rsub;
          if (r < rows_valid) reinterpret_cast<uint16_t*>(p.c)[(int64_t)(row0 + r) * p.ldc + col] = f2bf(acc[i][j][v]);
        }
      }
  }
}

// NXD_GG_DMA=0 selects the VGPR-staged variant (A/B, tools/bench_grouped_gemm.py); read once.
static int band_rows() {
  static const int b = [] {
    const char* e = getenv("NXD_GG_BAND");
    const int v = e ? atoi(e) : 8;
    return v > 0 ? v : 8;
  }();
  return b;
}
// NXD_GG_BIG=1: 256 x 256 tiles (grouped_gemm_big_kernel); read once.
static bool use_big() {
  static const bool on = [] {
    const char* e = getenv("NXD_GG_BIG");
    return e && e[0] == '1';
  }();
  return on;
}
static bool use_dma() {
  static const bool on = [] {
    const char* e = getenv("NXD_GG_DMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace gg

// mode 0 FWD:   a = x [M, K], b = W [E, K, N], c = y [M, N] bf16
// mode 1 DGRAD: a = dy [M, N], b = W [E, K, N], c = dx [M, K] bf16        (launch N := K, K := N)
// mode 2 WGRAD: a = x [M, K], b = dy [M, N], c = dW [E, K, N] fp32 (accumulate: +=)
// All inner dims multiples of 8 elements and 16-byte aligned rows (checked by the binding).
int grouped_gemm_launch(int mode, const void* a, const void* b, void* c, const int* offs, int E, int M, int K, int N,
                        int accumulate, hipStream_t stream) {
  if (E <= 0 || K <= 0 || N <= 0 || M < 0 || (K % 8) || (N % 8)) return -1;
  gg::Params p{};
  p.a = static_cast<const uint16_t*>(a);
  p.b = static_cast<const uint16_t*>(b);
  p.c = c;
  p.offs = offs;
  p.E = E;
  p.M = M;
  p.accumulate = accumulate;
  p.band = gg::band_rows();
  if (gg::use_big()) {
    constexpr int T = gg::BB;
    if (mode == gg::FWD || mode == gg::DGRAD) {
      if (mode == gg::FWD) {
        p.K = K; p.N = N; p.lda = K; p.ldb = N; p.ldc = N;
      } else {
        p.K = N; p.N = K; p.lda = N; p.ldb = N; p.ldc = K;
      }
      p.b_estride = (int64_t)K * N;
      p.n_tiles = ceil_div(p.N, T);
      p.r_tiles = ceil_div(M, T) + E;
      if (M == 0) return 0;
      const int64_t nwg = (int64_t)p.n_tiles * p.r_tiles;
      if (nwg > INT32_MAX) return -2;
      if (mode == gg::FWD)
        hipLaunchKernelGGL(gg::grouped_gemm_big_kernel<gg::FWD>, dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
      else
        hipLaunchKernelGGL(gg::grouped_gemm_big_kernel<gg::DGRAD>, dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
    } else if (mode == gg::WGRAD) {
      p.K = K; p.N = N; p.lda = K; p.ldb = N; p.ldc = N; p.c_estride = (int64_t)K * N;
      p.n_tiles = ceil_div(N, T);
      p.r_tiles = ceil_div(K, T);
      const int64_t nwg = (int64_t)p.n_tiles * p.r_tiles * E;
      if (nwg > INT32_MAX) return -2;
      hipLaunchKernelGGL(gg::grouped_gemm_big_kernel<gg::WGRAD>, dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
    } else {
      return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (mode == gg::FWD) {
    p.K = K; p.N = N; p.lda = K; p.ldb = N; p.ldc = N; p.b_estride = (int64_t)K * N;
    p.n_tiles = ceil_div(N, gg::BN);
    p.r_tiles = ceil_div(M, gg::BM) + E;
    if (M == 0) return 0;
    const int64_t nwg = (int64_t)p.n_tiles * p.r_tiles;
    if (nwg > INT32_MAX) return -2;
    if (gg::use_dma())
      hipLaunchKernelGGL((gg::grouped_gemm_kernel<gg::FWD, true>), dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
    else
      hipLaunchKernelGGL((gg::grouped_gemm_kernel<gg::FWD, false>), dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
  } else if (mode == gg::DGRAD) {
    // dx [M, K] = dy [M, N] . W[e]^T : reduction over N, output columns K
    p.K = N; p.N = K; p.lda = N; p.ldb = N; p.ldc = K; p.b_estride = (int64_t)K * N;
    p.n_tiles = ceil_div(K, gg::BN);
    p.r_tiles = ceil_div(M, gg::BM) + E;
    if (M == 0) return 0;
    const int64_t nwg = (int64_t)p.n_tiles * p.r_tiles;
    if (nwg > INT32_MAX) return -2;
    if (gg::use_dma())
      hipLaunchKernelGGL((gg::grouped_gemm_kernel<gg::DGRAD, true>), dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
    else
      hipLaunchKernelGGL((gg::grouped_gemm_kernel<gg::DGRAD, false>), dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
  } else if (mode == gg::WGRAD) {
    p.K = K; p.N = N; p.lda = K; p.ldb = N; p.ldc = N; p.c_estride = (int64_t)K * N;
    p.n_tiles = ceil_div(N, gg::BN);
    p.r_tiles = ceil_div(K, gg::BM);
    const int64_t nwg = (int64_t)p.n_tiles * p.r_tiles * E;
    if (nwg > INT32_MAX) return -2;
    if (gg::use_dma())
      hipLaunchKernelGGL((gg::grouped_gemm_kernel<gg::WGRAD, true>), dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
    else
      hipLaunchKernelGGL((gg::grouped_gemm_kernel<gg::WGRAD, false>), dim3((unsigned)nwg), dim3(gg::NT), 0, stream, p);
  } else {
    return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace nxd
