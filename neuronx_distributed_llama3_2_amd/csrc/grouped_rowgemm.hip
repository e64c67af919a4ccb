// Grouped (ragged-M) MoE expert GEMMs with 256 x 256 tiles on gfx950 MFMA: the forward and the
// input gradient of the expert MLPs over expert-sorted rows (expert e owns rows offs[e] ..
// offs[e+1], read on the device: no host sync, hipGraph-capturable).
//
//   FWD   y[m, n]  = sum_k x[m, k]  W[e][k, n]       A = x  [rows][K] , B = W[e] [K][N]  (k-major)
//   DGRAD dx[m, k] = sum_n dy[m, n] W[e][k, n]       A = dy [rows][N] , B = W[e] read as [k][n] rows
//
// Reference: the expert MLP of modules/moe/expert_mlps.py:169-265 (all-experts einsum / capacity
// drop); here only the chosen rows are computed.  The weight gradients of the same layer run on the
// token-major wgrad kernel (csrc/wgrad_gemm.hip, grouped mode).
//
// Structure (shared with csrc/wgrad_gemm.hip, cdna_hip_programming.md §5):
//   * 8 waves (512 threads), 256 x 256 output tile, one workgroup per CU; waves 2 (M) x 4 (N) of
//     128 x 64 = 8 x 4 v_mfma_f32_16x16x32_bf16 tiles, 128 fp32 accumulators per lane;
//   * reduction step BK = 32, 4-stage LDS ring (4 x 32 KiB) filled by LDS-DMA (1 KiB lane-linear
//     pieces, swizzle applied to the source address), counted vmcnt; default main loop = the
//     ping-pong one (PP below: wave groups staggered by one barrier, +3-9 % over one barrier per
//     stage, bitwise-identical output, profiles/r3_pp_mainloop_ab.jsonl);
//   * operands consumed along their contiguous axis (A; DGRAD's B) sit in a [256][32] row image
//     (64-B rows, 16-B chunk c stored at c ^ g[(row >> 2) & 3], g = {0, 2, 3, 1}: every 16-lane
//     group of a ds_read_b128 fragment read covers all 64 banks once); FWD's B (reduction along its
//     rows) sits in a [32][256] image read with ds_read_b64_tr_b16 (as the wgrad kernel);
//   * row tiles: worst-case count ceil(rows / 256) + E, each workgroup finds (expert, tile) by a
//     scan of the offsets; the L2 band raster of the wgrad kernel over (row tile, column tile);
//   * epilogue: per wave, 32-row slabs through padded LDS, bf16 pairs stored 128 B per row per
//     wave-instruction, rows outside the expert's range masked.
#include "common.h"

#include <cstdlib>

namespace nxd {
namespace grg {

constexpr int BM = 256, BN = 256, BK = 32, STAGES = 4, NT = 512;
constexpr int IMG_BYTES = 256 * BK * 2;            // 16 KiB: one operand stage
constexpr int STAGE_BYTES = 2 * IMG_BYTES;
constexpr int LDS_BYTES = STAGES * STAGE_BYTES;    // 128 KiB
constexpr int PIECES = IMG_BYTES / 1024 / (NT / 64);   // 2 per wave per operand
constexpr int DMA_PER_STAGE = 2 * PIECES;
enum Mode { FWD = 0, DGRAD = 1 };

struct Params {
  const uint16_t* a;    // [rows][lda]
  const uint16_t* b;    // W [E][K][N]
  uint16_t* c;          // [rows][ldc]
  const int* offs;      // [E + 1]
  int E, rows;
  int red;              // reduction length (FWD: K, DGRAD: N)
  int ncols;            // output columns (FWD: N, DGRAD: K)
  int64_t lda, ldb, ldc, b_es;
  int rt, nt;           // worst-case row tiles, column tiles
  int band;
};

__device__ __forceinline__ int rswz(int row) {   // {0, 2, 3, 1}[(row >> 2) & 3]
  const int j = (row >> 2) & 3;
  return (0x78 >> (2 * j)) & 3;                 // 0b01'11'10'00, two bits per j: 0, 2, 3, 1
}
__device__ __forceinline__ int row_off(int row, int ch) { return row * 64 + 16 * (ch ^ rswz(row)); }
__device__ __forceinline__ int tswz(int t) { return 2 * ((t & 3) | (((t >> 3) & 1) << 2)); }
__device__ __forceinline__ int tr_off(int t, int ch) { return t * 512 + 16 * (ch ^ tswz(t)); }

typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) short4_t lds_short4_t;
__device__ __forceinline__ uint32_t lds_addr(const char* q) { return (uint32_t)(uintptr_t)(const lds_char_t*)q; }

__device__ __forceinline__ void dma16(const void* src, uint32_t lds_dst) {
  uint32_t sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(sv) : "v"(src), "s"(lds_dst) : "memory");
}

// 16x16x32 fragment of rows [r0, r0 + 16) from a row image: lane l -> row r0 + (l & 15), k 8 (l >> 4) .. + 7
__device__ __forceinline__ bf16x8_t frag_row(const char* img, int r0) {
  const int l = threadIdx.x & 63;
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4_t*>(img + row_off(r0 + (l & 15), l >> 4)));
}
// the same fragment of columns [c0, c0 + 16) from a [32 k][256] image (two transposed reads)
__device__ __forceinline__ bf16x8_t frag_tr(const char* img, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  const int t = 8 * g + q;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)(img + tr_off(t, col >> 3) + 8 * (p & 1)));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)(img + tr_off(t + 4, col >> 3) + 8 * (p & 1)));
  const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, a8);
}

// this thread's pieces of the oldest outstanding stage landed (`newer` younger stages left in flight)
__device__ __forceinline__ void wait_vm(int newer) {
  if (newer >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_STAGE) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Measured and not kept (profiles/r3_grouped_rowgemm_variants.jsonl): a 5-stage ring (160 KiB) and
// s_setprio around the MFMA clusters or for the younger wave half -- all within +-2 %.
//
// PP (ping-pong): each 32-deep stage is two phases of 16 MFMAs per wave, every phase
// [LDS-DMA half-stage][fragment reads] barrier [16 MFMAs at raised priority] barrier, and wave group
// 1 (waves 4-7; every SIMD holds one wave of each group) runs one barrier behind group 0, so on each
// SIMD one wave's MFMA burst covers the other wave's reads and DMA issue (cdna_hip_programming.md,
// "The 256^2 8-phase template").  Ring safety, global barrier instances #n (group 0 passes #(4t+2h)
// and #(4t+2h+1) in phase (t, h); group 1 one later):
//   * stage S is read from #(4S-1) on (group 0, phase (S, 0)); both groups retire their pieces of S
//     before arriving there (group 0 after its MFMAs of (S-1, 1), group 1 before its reads of (S-1, 1));
//   * the last reads of stage S complete before #(4S+4) (group 1's MFMAs of (S, 1)); its slot is
//     refilled with S+4 after that: group 1 in (S+1, 0/1), group 0 in (S+1, 1) and (S+2, 0);
//   * pieces issued after stage S's last: S+1 (4) and S+2's first half (2) -> vmcnt(6), less at the tail.
// Measured and not kept: the LDS-DMA issued inside the MFMA bursts instead of the load phases
// (vmcnt(8) / (6) by group) -- 1-5 % slower than this on every MoE / dense shape
// (profiles/r3_pp_dma_in_mfma_rejected.jsonl).
template <int MODE, bool PP>
__global__ void __launch_bounds__(NT, 1) rowgemm_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  int rt, ct;
  {
    const int kb = p.band, bnd = id / (kb * p.nt), rem = id - bnd * kb * p.nt;
    const int h = min(kb, p.rt - bnd * kb);
    rt = bnd * kb + rem % h;
    ct = rem / h;
  }
  // (expert, row range) of row tile rt: tiles are numbered expert by expert
  int e = -1, r0 = 0, r1 = 0;
  {
    int acc = 0;
    for (int i = 0; i < p.E; ++i) {
      const int g0 = p.offs[i], g1 = p.offs[i + 1];
      const int nt_e = g1 > g0 ? (g1 - g0 + BM - 1) / BM : 0;
      if (rt < acc + nt_e) {
        e = i;
        r0 = g0 + (rt - acc) * BM;
        r1 = min(g1, r0 + BM);
        break;
      }
      acc += nt_e;
    }
  }
  if (e < 0) return;   // beyond the real tile count (workgroup-uniform)
  const int n0 = ct * BN;
  const int nk = p.red / BK;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 2, wn = wid & 3;
  const uint16_t* bw = p.b + (int64_t)e * p.b_es;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  // per-lane DMA sources of reduction step 0; step s adds s * BK elements (row images) or s * BK
  // rows (the k-major image)
  const uint16_t* src_a[PIECES];
  const uint16_t* src_b[PIECES];
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    const int piece = wid * PIECES + i;
    {  // row image: piece = rows 16 piece .. + 15, lane -> row 16 piece + l / 4, slot l % 4
      const int row = 16 * piece + (lane >> 2), ch = (lane & 3) ^ rswz(row);
      const int gr = min(r0 + row, r1 - 1);   // rows past the expert's range re-read a valid row (never stored)
      src_a[i] = p.a + (int64_t)gr * p.lda + 8 * ch;
      if (MODE == DGRAD) {
        const int col = min(n0 + row, p.ncols - 1);   // output column k_out = a row of W[e]
        src_b[i] = bw + (int64_t)col * p.ldb + 8 * ch;
      }
    }
    if (MODE == FWD) {  // k-major image: piece = k rows 2 piece, 2 piece + 1; lane -> k 2 piece + l / 32, slot l % 32
      const int t = 2 * piece + (lane >> 5), ch = (lane & 31) ^ tswz(t);
      src_b[i] = bw + (int64_t)t * p.ldb + min(n0 + 8 * ch, p.ncols - 8);
    }
  }
  auto issue = [&](int s) {
    const uint32_t img = lds0 + (s % STAGES) * STAGE_BYTES + wid * PIECES * 1024;
    const int oa = s * BK;
    const int64_t ob = MODE == FWD ? (int64_t)s * BK * p.ldb : (int64_t)s * BK;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      dma16(src_a[i] + oa, __builtin_amdgcn_readfirstlane(img + i * 1024));
      dma16(src_b[i] + ob, __builtin_amdgcn_readfirstlane(img + IMG_BYTES + i * 1024));
    }
  };
  auto bfrag = [&](const char* img, int c0) { return MODE == FWD ? frag_tr(img, c0) : frag_row(img, c0); };

  if constexpr (PP) {
    const int grp = wm;
    auto issue_half = [&](int s, int hh) {
      if (s >= nk) return;
      const uint32_t img = lds0 + (s % STAGES) * STAGE_BYTES + wid * PIECES * 1024;
      const int oa = s * BK;
      const int64_t ob = MODE == FWD ? (int64_t)s * BK * p.ldb : (int64_t)s * BK;
      dma16(src_a[hh] + oa, __builtin_amdgcn_readfirstlane(img + hh * 1024));
      dma16(src_b[hh] + ob, __builtin_amdgcn_readfirstlane(img + IMG_BYTES + hh * 1024));
    };
    auto wait_stage = [&](int S) {   // this thread's pieces of stage S landed
      if (S + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (S + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto barrier = [] {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    issue_half(0, 0); issue_half(0, 1); issue_half(1, 0); issue_half(1, 1); issue_half(2, 0);
    wait_stage(0);
    if (grp == 1) issue_half(2, 1);
    barrier();
    if (grp == 1) barrier();   // the stagger
    bf16x8_t af[4], bf[4];
    for (int t = 0; t < nk; ++t) {
      const char* img = smem + (t % STAGES) * STAGE_BYTES;
      // ---- phase (t, 0): B fragments + A rows 0..63 of the wave
      if (grp == 0) issue_half(t + 2, 1); else issue_half(t + 3, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = bfrag(img + IMG_BYTES, wn * 64 + 16 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag_row(img, wm * 128 + 16 * i);
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- phase (t, 1): A rows 64..127
      if (grp == 1) {
        if (t + 1 < nk) wait_stage(t + 1);
        issue_half(t + 3, 1);
      } else {
        issue_half(t + 3, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag_row(img, wm * 128 + 16 * (4 + i));
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (grp == 0 && t + 1 < nk) wait_stage(t + 1);
      barrier();
    }
    if (grp == 0) barrier();   // equal barrier counts before the epilogue's __syncthreads
  } else {
  for (int s = 0; s < STAGES - 1 && s < nk; ++s) issue(s);
  bf16x8_t af[8], bf[4];
  if (nk > 0) {
    wait_vm(min(STAGES - 2, nk - 1));
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = bfrag(smem + IMG_BYTES, wn * 64 + 16 * j);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag_row(smem, wm * 128 + 16 * i);
  }
  for (int t = 0; t < nk; ++t) {
    const bool more = t + 1 < nk;
    if (more) wait_vm(min(STAGES - 3, nk - 2 - t));
    __builtin_amdgcn_s_barrier();
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    const char* n_img = smem + ((more ? t + 1 : t) % STAGES) * STAGE_BYTES;
    bf16x8_t bn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bn[j] = bfrag(n_img + IMG_BYTES, wn * 64 + 16 * j);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      af[i] = frag_row(n_img, wm * 128 + 16 * i);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = bn[j];
  }
  }

  // ---- epilogue: 4 rounds of 32 rows x 64 columns per wave through a padded LDS slab, then bf16
  // pairs: lane l stores columns 2 (l & 31), +1 of row 2 rr + (l >> 5) (128 B per row per instruction)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int LD = 68;
  float* slab = reinterpret_cast<float*>(smem) + wid * (32 * LD);
  const int ccol = lane & 15, crow = 4 * (lane >> 4);
  const int pc = 2 * (lane & 31), ph = lane >> 5;
  const int col = n0 + wn * 64 + pc;
#pragma unroll
  for (int rnd = 0; rnd < 4; ++rnd) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(16 * ii + crow + r) * LD + 16 * j + ccol] = acc[2 * rnd + ii][j][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll 4
    for (int rr = 0; rr < 16; ++rr) {
      const int lr = 2 * rr + ph;
      const int row = r0 + wm * 128 + 32 * rnd + lr;
      const float v0 = slab[lr * LD + pc], v1 = slab[lr * LD + pc + 1];
      if (row < r1 && col < p.ncols) *reinterpret_cast<uint32_t*>(p.c + (int64_t)row * p.ldc + col) = pack2bf(v0, v1);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

static int g_pp = -1;   // ping-pong variant (NXD_GRG_PP; settable for in-process A/B)
static bool use_pp() {
  if (g_pp < 0) {
    const char* e = getenv("NXD_GRG_PP");
    g_pp = e ? (atoi(e) != 0) : 1;
  }
  return g_pp != 0;
}

static int band_rows() {
  static const int b = [] {
    const char* e = getenv("NXD_GRG_BAND");   // 8: +2..7 % over 4 on most Mixtral shapes (r3_grouped_rowgemm_variants)
    const int v = e ? atoi(e) : 8;
    return v > 0 ? v : 8;
  }();
  return b;
}

}  // namespace grg

void grouped_rowgemm_set_pp(int v) { grg::g_pp = v != 0; }

// mode 0 FWD:   a = x [rows, K],  W [E, K, N], c = y  [rows, N]
// mode 1 DGRAD: a = dy [rows, N], W [E, K, N], c = dx [rows, K]
// Requires the reduction length % 32 == 0 and K, N % 8 == 0 (checked; returns -1 otherwise, the
// caller then takes the 128-tile kernel).  Rows past offs[E] are not written.
int grouped_rowgemm_launch(int mode, const void* a, const void* w, void* c, const int* offs, int E, int rows, int K,
                           int N, hipStream_t stream) {
  if (E <= 0 || K <= 0 || N <= 0 || rows < 0 || K % 8 || N % 8) return -1;
  grg::Params p{};
  p.a = static_cast<const uint16_t*>(a);
  p.b = static_cast<const uint16_t*>(w);
  p.c = static_cast<uint16_t*>(c);
  p.offs = offs;
  p.E = E;
  p.rows = rows;
  p.b_es = (int64_t)K * N;
  p.ldb = N;
  if (mode == grg::FWD) {
    p.red = K; p.ncols = N; p.lda = K; p.ldc = N;
  } else if (mode == grg::DGRAD) {
    p.red = N; p.ncols = K; p.lda = N; p.ldc = K;
  } else {
    return -1;
  }
  if (p.red % grg::BK) return -1;
  if (rows == 0) return 0;
  p.rt = ceil_div(rows, grg::BM) + E;
  p.nt = ceil_div(p.ncols, grg::BN);
  p.band = grg::band_rows();
  const int64_t nwg = (int64_t)p.rt * p.nt;
  if (nwg > INT32_MAX) return -2;
  const bool pp = grg::use_pp();
  if (mode == grg::FWD) {
    if (pp) hipLaunchKernelGGL((grg::rowgemm_kernel<grg::FWD, true>), dim3((unsigned)nwg), dim3(grg::NT), 0, stream, p);
    else hipLaunchKernelGGL((grg::rowgemm_kernel<grg::FWD, false>), dim3((unsigned)nwg), dim3(grg::NT), 0, stream, p);
  } else {
    if (pp) hipLaunchKernelGGL((grg::rowgemm_kernel<grg::DGRAD, true>), dim3((unsigned)nwg), dim3(grg::NT), 0, stream, p);
    else hipLaunchKernelGGL((grg::rowgemm_kernel<grg::DGRAD, false>), dim3((unsigned)nwg), dim3(grg::NT), 0, stream, p);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace nxd
