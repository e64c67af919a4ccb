// Weight-gradient GEMM for the parallel linear layers on gfx950 MFMA:
//
//     main_grad[m, n] (fp32) += sum_t dy[t, m] * x[t, n]        (bf16 operands, fp32 accumulate)
//
// Both operands arrive token-major exactly as the forward / backward produced them (dy = output
// gradient [T, M], x = layer input [T, N], rows contiguous along the features): the reduction runs
// over their ROW index.  hipBLASLt needs both transposed to reach its TN speed (a separate tiled
// transpose per operand per layer, 2-5 % of the step) and runs the skinny tensor-parallel shards
// at 0.55-0.9 PF/s (profiles/r2_gemm_tp8_wgrad_layouts.jsonl); this kernel reads the token-major
// tiles with the hardware transpose read (ds_read_b64_tr_b16) instead, and splits the token range
// over workgroups when the output alone cannot fill the 256 CUs.
// Reference: the weight gradient of LinearWithAsyncCommunication.backward
// (src/neuronx_distributed/parallel_layers/layers.py:391-409) and GQAQKVLinearWithAsyncCommunication
// (src/neuronx_distributed/modules/qkv_linear.py:131-150), fp32 gradient accumulation as in the
// reference's use_fp32_grad_acc ZeRO-1 mode.
//
// Structure (cdna_hip_programming.md §5, "Pipelining across barriers"):
//   * workgroup = 8 waves (512 threads), 256 x 256 output tile, one workgroup per CU (128 KiB LDS);
//     waves 2 (M) x 4 (N), 128 x 64 outputs each = 8 x 4 v_mfma_f32_16x16x32_bf16 tiles, 128 fp32
//     accumulators per lane;
//   * token step BK = 32, a 4-stage LDS ring (4 x 32 KiB): stage t + 3 is issued by LDS-DMA
//     (global_load_lds_dwordx4, lane-linear 1 KiB pieces) while stage t is consumed, each wave
//     waits with a COUNTED vmcnt for its own pieces of stage t only, and one raw s_barrier per
//     stage publishes it (no vmcnt(0) in the loop: two stages stay in flight across every barrier);
//     default: the ping-pong variant of that loop (two 16-MFMA phases per stage, wave groups one
//     barrier apart; +3-16 %, profiles/r3_pp_mainloop_ab.jsonl);
//   * LDS image of an operand stage: [32 tokens][256 features], 512-B rows, 16-B chunk c stored at
//     c ^ 2 * ((t & 3) | ((t >> 3) & 1) << 2): the two 16-lane groups of a transposed read (4 token
//     rows x 16 features each, rows t, t + 8) land on 16 distinct bank quads — conflict-free.  The
//     swizzle is applied to each lane's SOURCE address (the DMA writes lane-linearly, rule 21);
//   * epilogue: the fp32 tile goes through LDS (padded rows) so that every global atomic add covers
//     256 contiguous bytes (MI355X_MICROARCH "Global float atomics": full rate), issued without
//     return and left in flight when the workgroup exits; with one token split per tile each
//     element receives exactly one add (deterministic), with S splits S adds in any order.
//   * grouped (MoE expert weight gradients, dW[e] += x_e^T dy_e over expert-sorted rows): the grid
//     covers (split, expert, tile); each workgroup reads its expert's row range from the device
//     offsets (no host sync) and its ragged token tail DMAs a zero chunk instead of a foreign row.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace nxd {
namespace wg {

constexpr int BM = 256, BN = 256, BK = 32, STAGES = 4, NT = 512;
constexpr int IMG_BYTES = BK * 256 * 2;           // 16 KiB: one operand stage
constexpr int STAGE_BYTES = 2 * IMG_BYTES;        // A | B
constexpr int LDS_BYTES = STAGES * STAGE_BYTES;   // 128 KiB
constexpr int PIECES = IMG_BYTES / 1024 / (NT / 64);   // LDS-DMA pieces per wave per operand stage (2)
constexpr int DMA_PER_STAGE = 2 * PIECES;               // per thread per stage (A and B): 4

struct Params {
  const uint16_t* dy;   // [T, M], row stride ld_dy
  const uint16_t* x;    // [T, N], row stride ld_x
  float* c;             // [M, N] fp32, row stride ldc
  int T, M, N;
  int64_t ld_dy, ld_x, ldc;
  int mt, nt;           // output tiles along M, N
  int splits;           // token splits per tile
  int t_per_split;      // tokens per split (multiple of BK)
  int band;             // row tiles per raster band
  int ablate;           // A/B diagnostics only (wgrad_gemm_set_ablate): 1 = skip the epilogue adds,
                        // 2 = skip the MFMAs, 4 = skip the LDS-DMA refills of stages >= 3
  // grouped mode: expert e owns rows offs[e] .. offs[e+1] of dy / x; c += e * c_es
  const int* offs;
  int E;
  int64_t c_es;
};

__device__ __attribute__((aligned(16))) uint32_t g_zero16[4];   // zero-initialised device global: the DMA
                                                                  // source of token rows past a group's end

__device__ __forceinline__ int swz(int t) { return 2 * ((t & 3) | (((t >> 3) & 1) << 2)); }
__device__ __forceinline__ int img_off(int t, int ch) { return t * 512 + 16 * (ch ^ swz(t)); }

typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) short4_t lds_short4_t;
__device__ __forceinline__ uint32_t lds_addr(const char* q) { return (uint32_t)(uintptr_t)(const lds_char_t*)q; }

// one 1 KiB LDS-DMA piece (16 B per lane) at the wave-uniform LDS address `lds_dst`
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_dst) {
  uint32_t sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(sv) : "v"(src), "s"(lds_dst) : "memory");
}

// 16x16x32 operand fragment of features [c0, c0 + 16) from a token-major image: lane l holds
// feature c0 + (l & 15) at tokens 8 (l >> 4) + j, j = 0..7 -- two transposed reads, each a block
// of 4 token rows x 16 features per 16-lane group (lane 4q + p supplies row q, features 4p .. 4p+3).
__device__ __forceinline__ bf16x8_t frag(const char* img, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  const int t = 8 * g + q;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)(img + img_off(t, col >> 3) + 8 * (p & 1)));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)(img + img_off(t + 4, col >> 3) + 8 * (p & 1)));
  const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, a8);
}

__device__ __forceinline__ void wait_vm(int newer) {   // this thread's pieces of the oldest stage landed
  if (newer >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_STAGE) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// s_setprio around the MFMA clusters or for the younger wave half measured within +-2 % (not kept,
// profiles/r3_wgrad_kernel_prio_rejected.jsonl)
// PP: the ping-pong main loop of csrc/grouped_rowgemm.hip (two 16-MFMA phases per stage, wave group
// 1 one barrier behind group 0; ring-safety argument there).
template <bool GROUPED, bool PP>
__global__ void __launch_bounds__(NT, 1) wgrad_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tiles = p.mt * p.nt;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int groups = GROUPED ? p.E : 1;
  const int split = id / (tiles * groups);   // splits outermost: a tile's partial sums land in different grid waves
  const int ge = GROUPED ? (id / tiles) % groups : 0;
  int rt, ct;
  {
    const int within = id % tiles;
    const int kb = p.band, bnd = within / (kb * p.nt), rem = within - bnd * kb * p.nt;
    const int h = min(kb, p.mt - bnd * kb);
    rt = bnd * kb + rem % h;
    ct = rem / h;
  }
  const int m0 = rt * BM, n0 = ct * BN;
  int t_begin, t_end, nk;
  float* cbase = p.c;
  if constexpr (GROUPED) {
    const int g0 = p.offs[ge], g1 = p.offs[ge + 1];
    const int per = ceil_div(ceil_div(max(g1 - g0, 0), BK), p.splits) * BK;
    t_begin = g0 + split * per;
    t_end = min(g1, t_begin + per);
    if (t_begin >= t_end) return;      // empty group / split: nothing to add (workgroup-uniform)
    nk = ceil_div(t_end - t_begin, BK);
    cbase += ge * p.c_es;
  } else {
    t_begin = split * p.t_per_split;
    t_end = min(p.T, t_begin + p.t_per_split);
    nk = (t_end - t_begin) / BK;
  }
  const int rows = t_end - t_begin;   // grouped: token rows >= rows of the last stage read zeros

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 2, wn = wid & 3;   // 2 x 4 waves: rows 128 wm.., cols 64 wn..

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  // per-lane LDS-DMA source pointers of this tile's first token step (piece i of operand A / B);
  // a stage s reads them advanced by s * BK rows (one scalar 64-bit offset per operand)
  const uint16_t* src_a[PIECES];
  const uint16_t* src_b[PIECES];
  int tt_of[PIECES];
  {
    const int l = lane;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = wid * PIECES + i, tt = piece * 2 + (l >> 5), ch = (l & 31) ^ swz(tt);
      tt_of[i] = tt;
      src_a[i] = p.dy + (int64_t)(t_begin + tt) * p.ld_dy + min(m0 + 8 * ch, p.M - 8);
      src_b[i] = p.x + (int64_t)(t_begin + tt) * p.ld_x + min(n0 + 8 * ch, p.N - 8);
    }
  }
  auto issue = [&](int s) {
    const uint32_t img = lds0 + (s % STAGES) * STAGE_BYTES + wid * PIECES * 1024;
    const int64_t oa = (int64_t)s * BK * p.ld_dy, ob = (int64_t)s * BK * p.ld_x;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const uint16_t* sa = src_a[i] + oa;
      const uint16_t* sb = src_b[i] + ob;
      if constexpr (GROUPED) {
        if (s * BK + tt_of[i] >= rows) sa = sb = reinterpret_cast<const uint16_t*>(g_zero16);   // past the group's end
      }
      dma16(sa, __builtin_amdgcn_readfirstlane(img + i * 1024));
      dma16(sb, __builtin_amdgcn_readfirstlane(img + IMG_BYTES + i * 1024));
    }
  };

  // Software pipeline, one barrier per 32-token stage.  Fragments of stage t sit in registers
  // (read during iteration t-1); iteration t publishes stage t+1 (counted vmcnt for this thread's
  // pieces + barrier), refills the slot of stage t-1 (all reads of t-1 completed before the MFMAs
  // of t-1, i.e. before this barrier) with stage t+3, and runs the 32 MFMAs of stage t with the
  // transposed reads of stage t+1 interleaved (each A fragment is re-read right after its last
  // MFMA; B fragments into a second set) -- the MFMA pipe never waits on an LDS read after a
  // barrier.  LDS-DMA: stages t+1 .. t+3 in flight at most; a stage is waited for two iterations
  // after its issue.
  if constexpr (PP) {
    const int grp = wm;
    auto issue_half = [&](int s, int hh) {
      if (s >= nk || (p.ablate & 4 && s >= STAGES - 1)) return;
      const uint32_t img = lds0 + (s % STAGES) * STAGE_BYTES + wid * PIECES * 1024;
      const uint16_t* sa = src_a[hh] + (int64_t)s * BK * p.ld_dy;
      const uint16_t* sb = src_b[hh] + (int64_t)s * BK * p.ld_x;
      if constexpr (GROUPED) {
        if (s * BK + tt_of[hh] >= rows) sa = sb = reinterpret_cast<const uint16_t*>(g_zero16);
      }
      dma16(sa, __builtin_amdgcn_readfirstlane(img + hh * 1024));
      dma16(sb, __builtin_amdgcn_readfirstlane(img + IMG_BYTES + hh * 1024));
    };
    auto wait_stage = [&](int S) {
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
      if (grp == 0) issue_half(t + 2, 1); else issue_half(t + 3, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = frag(img + IMG_BYTES, wn * 64 + 16 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(img, wm * 128 + 16 * i);
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      if (grp == 1) {
        if (t + 1 < nk) wait_stage(t + 1);
        issue_half(t + 3, 1);
      } else {
        issue_half(t + 3, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(img, wm * 128 + 16 * (4 + i));
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
    if (grp == 0) barrier();
  } else {
  for (int s = 0; s < STAGES - 1 && s < nk; ++s) issue(s);
  bf16x8_t af[8], bf[4];
  if (nk > 0) {
    wait_vm(min(STAGES - 2, nk - 1));
    __builtin_amdgcn_s_barrier();
    const char* a_img = smem;
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = frag(a_img + IMG_BYTES, wn * 64 + 16 * j);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag(a_img, wm * 128 + 16 * i);
  }
  for (int t = 0; t < nk; ++t) {
    const bool more = t + 1 < nk;
    if (more) wait_vm(min(STAGES - 3, nk - 2 - t));
    __builtin_amdgcn_s_barrier();
    if (t + STAGES - 1 < nk && !(p.ablate & 4)) issue(t + STAGES - 1);
    // stage t+1 (or, on the last iteration, stage t again: harmless, never consumed)
    const char* n_img = smem + ((more ? t + 1 : t) % STAGES) * STAGE_BYTES;
    bf16x8_t bn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bn[j] = frag(n_img + IMG_BYTES, wn * 64 + 16 * j);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (!(p.ablate & 2)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      } else {
        asm volatile("" ::"v"(af[i]), "v"(bf[0]), "v"(bf[1]), "v"(bf[2]), "v"(bf[3]));
      }
      af[i] = frag(n_img, wm * 128 + 16 * i);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = bn[j];
  }
  }

  // ---- epilogue: per wave, 4 rounds of 32 rows x 64 columns through a private padded LDS slab
  // ([32][68] fp32: the two row groups of a 32-lane store half are 4 rows apart -> 16 banks apart),
  // then one row (64 floats, 256 contiguous bytes) per atomic wave-instruction.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave is done with the ring
  constexpr int LD = 68;
  float* slab = reinterpret_cast<float*>(smem) + wid * (32 * LD);
  const int ccol = lane & 15, crow = 4 * (lane >> 4);
#pragma unroll
  for (int rnd = 0; rnd < 4; ++rnd) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(16 * ii + crow + r) * LD + 16 * j + ccol] = acc[2 * rnd + ii][j][r];
    __builtin_amdgcn_wave_barrier();
    const int col = n0 + wn * 64 + lane;
#pragma unroll 8
    for (int rr = 0; rr < 32; ++rr) {
      const int row = m0 + wm * 128 + 32 * rnd + rr;
      const float v = slab[rr * LD + lane];
      if (row < p.M && col < p.N && !(p.ablate & 1)) unsafeAtomicAdd(cbase + (int64_t)row * p.ldc + col, v);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

static int band_rows() {
  static const int b = [] {
    const char* e = getenv("NXD_WG_BAND");
    const int v = e ? atoi(e) : 4;
    return v > 0 ? v : 4;
  }();
  return b;
}

static int g_ablate = 0;

static int g_pp = -1;   // ping-pong main loop (NXD_WG_PP; settable for in-process A/B)
static bool use_pp() {
  if (g_pp < 0) {
    const char* e = getenv("NXD_WG_PP");
    g_pp = e ? (atoi(e) != 0) : 1;
  }
  return g_pp != 0;
}

template <bool G>
void launch(const Params& p, int64_t nwg, hipStream_t stream) {
  if (use_pp())
    hipLaunchKernelGGL((wgrad_kernel<G, true>), dim3((unsigned)nwg), dim3(NT), 0, stream, p);
  else
    hipLaunchKernelGGL((wgrad_kernel<G, false>), dim3((unsigned)nwg), dim3(NT), 0, stream, p);
}

}  // namespace wg

void wgrad_gemm_set_ablate(int v) { wg::g_ablate = v; }
void wgrad_gemm_set_pp(int v) { wg::g_pp = v != 0; }

// Token splits per output tile.  Cost model in token steps (BK = 32) of one workgroup: grid waves
// of 256 workgroups x (steps per split + ~10 for the atomic epilogue); the smallest split count
// of minimal cost (fewer splits = fewer fp32 atomic adds per element).
int wgrad_gemm_choose_splits(int T, int M, int N) {
  const int tiles = ceil_div(M, wg::BM) * ceil_div(N, wg::BN);
  const int steps = T / wg::BK;
  int best = 1;
  int64_t best_cost = INT64_MAX;
  for (int s = 1; s <= 32 && s <= steps; ++s) {
    if (s > 1 && steps / s < 16) break;
    const int64_t cost = (int64_t)ceil_div(tiles * s, 256) * (ceil_div(steps, s) + 10);
    if (cost < best_cost) {
      best_cost = cost;
      best = s;
    }
  }
  return best;
}

// c [M, N] fp32 += dy[T, M]^T x[T, N]; T % 32 == 0, M % 8 == 0, N % 8 == 0, 16-B aligned rows.
int wgrad_gemm_launch(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, float* c, int64_t ldc, int T, int M,
                      int N, int splits, hipStream_t stream) {
  if (T <= 0 || M <= 0 || N <= 0) return 0;
  if (T % wg::BK || M % 8 || N % 8 || ld_dy % 8 || ld_x % 8) return -1;
  wg::Params p{};
  p.dy = static_cast<const uint16_t*>(dy);
  p.x = static_cast<const uint16_t*>(x);
  p.c = c;
  p.T = T; p.M = M; p.N = N;
  p.ld_dy = ld_dy; p.ld_x = ld_x; p.ldc = ldc;
  p.mt = ceil_div(M, wg::BM);
  p.nt = ceil_div(N, wg::BN);
  if (splits <= 0) splits = wgrad_gemm_choose_splits(T, M, N);
  const int steps = T / wg::BK;
  splits = splits < 1 ? 1 : (splits > steps ? steps : splits);
  p.t_per_split = ceil_div(steps, splits) * wg::BK;
  p.splits = ceil_div(T, p.t_per_split);
  p.band = wg::band_rows();
  p.ablate = wg::g_ablate;
  const int64_t nwg = (int64_t)p.mt * p.nt * p.splits;
  if (nwg > INT32_MAX) return -2;
  wg::launch<false>(p, nwg, stream);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Grouped: c[e] [M, N] fp32 += dy[g0:g1]^T x[g0:g1] for every expert e, rows g0 = offs[e],
// g1 = offs[e+1] read on the device; splits per group chosen for the mean group size rows / E.
// M % 8 == 0, N % 8 == 0.
int wgrad_gemm_grouped_launch(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, float* c, int64_t ldc,
                              int64_t c_es, const int* offs, int E, int rows, int M, int N, hipStream_t stream) {
  if (E <= 0 || M <= 0 || N <= 0 || rows <= 0) return 0;
  if (M % 8 || N % 8 || ld_dy % 8 || ld_x % 8) return -1;
  wg::Params p{};
  p.dy = static_cast<const uint16_t*>(dy);
  p.x = static_cast<const uint16_t*>(x);
  p.c = c;
  p.T = rows; p.M = M; p.N = N;
  p.ld_dy = ld_dy; p.ld_x = ld_x; p.ldc = ldc;
  p.mt = ceil_div(M, wg::BM);
  p.nt = ceil_div(N, wg::BN);
  p.offs = offs;
  p.E = E;
  p.c_es = c_es;
  // splits for the mean group (all E groups' tiles share the grid)
  const int mean = std::max(wg::BK, (rows / E) / wg::BK * wg::BK);
  p.splits = wgrad_gemm_choose_splits(mean, (int)std::min<int64_t>((int64_t)M * E, INT32_MAX), N);
  p.band = wg::band_rows();
  p.ablate = wg::g_ablate;
  const int64_t nwg = (int64_t)p.mt * p.nt * E * p.splits;
  if (nwg > INT32_MAX) return -2;
  wg::launch<true>(p, nwg, stream);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace nxd
