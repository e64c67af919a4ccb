// Dense bf16 GEMMs of the training hot path on gfx950 MFMA: one main loop, two operand layouts,
// three epilogues.
//
//   NT  C[m, n] = sum_k A[m, k] B[n, k]    A [M][K], B [N][K]  (contraction contiguous in both):
//       the forward y = x W^T and the input gradient dx = dy W (W's K-major copy);
//   TN  C[m, n] = sum_k A[k, m] B[k, n]    A [K][M], B [K][N]  (contraction along the ROWS):
//       the weight gradient dW = dy^T x straight from the token-major activations -- no transposes.
//   Epilogues: BF16 store, F32_ACC (C fp32 += acc, one read-modify-write per element: exact and
//   deterministic), F32_ATOMIC (split-K partial sums into C fp32 by no-return float atomics).
//
// Reference: ColumnParallelLinear / RowParallelLinear forward and LinearWithAsyncCommunication's
// backward matmuls (src/neuronx_distributed/parallel_layers/layers.py:322,348,391-409), which the
// Neuron compiler lowers for its own matrix engine; here they are hand-scheduled for CDNA4.
//
// Structure (cdna_hip_programming.md §5, "The 256^2 8-phase template" and "Pipelining across barriers"):
//   * 256 x 256 output tile, 8 waves (512 threads), one workgroup per CU, reduction step BK = 64;
//     wave (wr, wc) = (wid >> 2, wid & 3) owns rows {wr*64 + [0,64)} and {128 + wr*64 + [0,64)}
//     and columns {wc*32 + [0,32)} and {128 + wc*32 + [0,32)}: four 64 x 32 quadrants, each
//     4 x 2 v_mfma_f32_16x16x32_bf16 tiles x 2 k-halves = 16 MFMAs per K-step;
//   * a K-tile lives in LDS as four 16 KiB REGIONS -- A_lo (tile rows 0..127), A_hi (128..255),
//     B_lo (columns 0..127), B_hi (128..255) -- so every region is a contiguous slab of the source
//     (128-B rows for NT, 256-B token rows for TN: whole cache lines, never half-lines), two
//     K-tiles = 128 KiB;
//   * per K-tile four phases, wave-uniform and identical for all waves:
//       q0: read A_lo + B_lo fragments, MFMA A_lo x B_lo      q1: read B_hi, MFMA A_lo x B_hi
//       q2: read A_hi, MFMA A_hi x B_hi                       q3: (no reads)  MFMA A_hi x B_lo
//     so A_lo / B_lo are dead after q0, B_hi after q1, A_hi after q2, and each region is REFILLED
//     with the K-tile two ahead as soon as it is dead: every phase issues one region (2 LDS-DMA
//     pieces per thread), four regions = eight pieces stay in flight across the barriers, each
//     waited for with a counted vmcnt (never 0 in the loop) ~4.5 phases after its issue;
//   * ping-pong: waves 4..7 run one barrier behind waves 0..3, so on every SIMD one wave's 16-MFMA
//     burst covers its partner's fragment reads and DMA issue; MFMA bursts at s_setprio 1;
//   * LDS images (written lane-linearly by global_load_lds_dwordx4, the swizzle applied to each
//     lane's SOURCE address, rule 21):
//       NT region [128 rows][64 k], 128-B rows, 16-B chunk c of row r stored at c ^ ((r >> 1) & 7):
//          every 16-lane group of a ds_read_b128 fragment read covers all 64 banks once;
//       TN region [64 k][128 features], 256-B rows, chunk c of row t at c ^ swz(t) (the wgrad
//          kernel's swizzle): the two 32-lane groups of ds_read_b64_tr_b16 are conflict-free;
//   * XCD-aware block remap + a raster band of row tiles; split-K outermost in the grid.
// Ring safety (global barrier instance #n; waves 0..3 pass #(2P), #(2P+1) in phase P = 4t + q,
// waves 4..7 one later): a region read in phase P is dead after #(2P+2); the refills are issued in
// phase P + 2 or later (A_lo / B_lo of tile t + 2 in q2 / q3 of t, B_hi / A_hi of t + 1 in q0 / q1
// of t).  Data read in phase P is waited for (vmcnt) by every thread before #(2P-1): waves 0..3 at
// the end of their MFMA burst of P-1, waves 4..7 at the end of their load segment of P-1.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace nxd {
namespace dg {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int REG = 16384;         // one region
constexpr int BUF = 4 * REG;       // one K-tile
constexpr int LDS_BYTES = 2 * BUF; // 128 KiB
// region offsets inside a K-tile buffer, indexed by issue order 0..3 = A_lo, B_lo, B_hi, A_hi
constexpr int R_ALO = 0, R_AHI = REG, R_BLO = 2 * REG, R_BHI = 3 * REG;

enum Layout { LNT = 0, LTN = 1 };
enum Epi { BF16 = 0, F32_ACC = 1, F32_ATOMIC = 2 };

struct Params {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  int M, N, K;
  int64_t lda, ldb, ldc;
  int mt, nt;        // output tiles along M, N
  int splits;        // K splits (F32_ATOMIC only; 1 otherwise)
  int k_per_split;   // multiple of BK
  int band;          // row tiles per raster band
};

typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) short4_t lds_short4_t;
__device__ __forceinline__ uint32_t lds_addr(const char* q) { return (uint32_t)(uintptr_t)(const lds_char_t*)q; }

// one 1 KiB LDS-DMA piece (16 B per lane) at the wave-uniform LDS address `lds_dst`
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_dst) {
  uint32_t sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(sv) : "v"(src), "s"(lds_dst) : "memory");
}

__device__ __forceinline__ int nt_swz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int tn_swz(int t) { return 2 * ((t & 3) | (((t >> 3) & 1) << 2)); }

// NT fragment of region rows [r0, r0 + 16), k-half s: lane l -> row r0 + (l & 15), k 32 s + 8 (l >> 4) .. + 7
__device__ __forceinline__ bf16x8_t frag_nt(const char* reg, int r0, int s) {
  const int l = threadIdx.x & 63, r = r0 + (l & 15), ch = (l >> 4) + 4 * s;
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4_t*>(reg + r * 128 + ((ch ^ nt_swz(r)) << 4)));
}
// TN fragment of region features [f0, f0 + 16), k-half s (two transposed reads): lane l -> feature
// f0 + (l & 15) at k 32 s + 8 (l >> 4) + j
__device__ __forceinline__ bf16x8_t frag_tn(const char* reg, int f0, int s) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int col = f0 + 4 * p, t = 32 * s + 8 * g + q;
  const char* b0 = reg + t * 256 + (((col >> 3) ^ tn_swz(t)) << 4) + 8 * (p & 1);
  const char* b1 = reg + (t + 4) * 256 + (((col >> 3) ^ tn_swz(t + 4)) << 4) + 8 * (p & 1);
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)b0);
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)b1);
  const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, a8);
}

template <int L>
__device__ __forceinline__ bf16x8_t frag(const char* reg, int x0, int s) {
  if constexpr (L == LNT) return frag_nt(reg, x0, s);
  else return frag_tn(reg, x0, s);
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// wait until at most `younger` regions (2 pieces each) issued after the needed one are in flight
__device__ __forceinline__ void wait_regions(int younger) {
  switch (younger) {
    case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int L, int E, int PIPE>
__global__ void __launch_bounds__(NT, 1) gemm_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tiles = p.mt * p.nt;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int split = id / tiles;
  int rt, ct;
  {
    const int within = id - split * tiles;
    const int kb = p.band, bnd = within / (kb * p.nt), rem = within - bnd * kb * p.nt;
    const int h = min(kb, p.mt - bnd * kb);
    rt = bnd * kb + rem % h;
    ct = rem / h;
  }
  const int m0 = rt * BM, n0 = ct * BN;
  const int k_begin = split * p.k_per_split;
  const int k_end = min(p.K, k_begin + p.k_per_split);
  const int nk = (k_end - k_begin) / BK;

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wid >> 2, wc = wid & 3;

  f32x4_t acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // per-lane DMA sources of K-tile 0 of this split, [region lo/hi][piece]; tile s adds s * adv
  const uint16_t* sa[2][2];
  const uint16_t* sb[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = 2 * wid + j;
      if constexpr (L == LNT) {
        const int pr = 8 * piece + (lane >> 3), c = (lane & 7) ^ nt_swz(pr);
        sa[h][j] = p.a + (int64_t)min(m0 + 128 * h + pr, p.M - 1) * p.lda + k_begin + 8 * c;
        sb[h][j] = p.b + (int64_t)min(n0 + 128 * h + pr, p.N - 1) * p.ldb + k_begin + 8 * c;
      } else {
        const int pr = 4 * piece + (lane >> 4), c = (lane & 15) ^ tn_swz(pr);
        sa[h][j] = p.a + (int64_t)(k_begin + pr) * p.lda + min(m0 + 128 * h + 8 * c, p.M - 8);
        sb[h][j] = p.b + (int64_t)(k_begin + pr) * p.ldb + min(n0 + 128 * h + 8 * c, p.N - 8);
      }
    }
  const int64_t adv_a = L == LNT ? (int64_t)BK : (int64_t)BK * p.lda;
  const int64_t adv_b = L == LNT ? (int64_t)BK : (int64_t)BK * p.ldb;
  const uint32_t lds0 = lds_addr(smem);

  // issue region R (issue order 0 A_lo, 1 B_lo, 2 B_hi, 3 A_hi) of K-tile s
  auto issue = [&](auto rc, int s) {
    constexpr int R = decltype(rc)::value;
    if (s >= nk) return;
    const uint32_t dst = lds0 + (s & 1) * BUF + (R == 0 ? R_ALO : R == 1 ? R_BLO : R == 2 ? R_BHI : R_AHI) + wid * 2048;
    if constexpr (R == 0 || R == 3) {
      constexpr int h = R == 0 ? 0 : 1;
      const int64_t o = (int64_t)s * adv_a;
      dma16(sa[h][0] + o, __builtin_amdgcn_readfirstlane(dst));
      dma16(sa[h][1] + o, __builtin_amdgcn_readfirstlane(dst + 1024));
    } else {
      constexpr int h = R == 1 ? 0 : 1;
      const int64_t o = (int64_t)s * adv_b;
      dma16(sb[h][0] + o, __builtin_amdgcn_readfirstlane(dst));
      dma16(sb[h][1] + o, __builtin_amdgcn_readfirstlane(dst + 1024));
    }
  };
  const int last = 4 * nk - 1;   // last issue position (4 s + R)
  // the region at issue position `need` is waited for; nothing to do past the last K-tile
  auto wait_for = [&](int need, int max_younger = 4) {
    if (need > last) return;
    wait_regions(min(max_younger, last - need));
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  bf16x8_t af[4][2], blo[2][2], bhi[2][2];
  auto mfma_q = [&](auto qc, bf16x8_t (&bf)[2][2]) {
    constexpr int qd = decltype(qc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qd][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bf[j][s], acc[qd][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (PIPE == 0) {
  // prologue: K-tile 0 whole, A_lo / B_lo of K-tile 1 (what the loop expects issued before t = 0)
  issue(I0{}, 0); issue(I1{}, 0); issue(I2{}, 0); issue(I3{}, 0); issue(I0{}, 1); issue(I1{}, 1);
  wait_for(1);
  barrier();
  const bool grp1 = wr == 1;
  if (grp1) barrier();   // the stagger
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    // ---- q0: A_lo x B_lo
    issue(I2{}, t + 1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = frag<L>(buf + R_ALO, wr * 64 + 16 * i, s);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) blo[j][s] = frag<L>(buf + R_BLO, wc * 32 + 16 * j, s);
    if (grp1) wait_for(4 * t + 2);
    barrier();
    mfma_q(I0{}, blo);
    if (!grp1) wait_for(4 * t + 2);
    barrier();
    // ---- q1: A_lo x B_hi
    issue(I3{}, t + 1);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) bhi[j][s] = frag<L>(buf + R_BHI, wc * 32 + 16 * j, s);
    if (grp1) wait_for(4 * t + 3);
    barrier();
    mfma_q(I1{}, bhi);
    if (!grp1) wait_for(4 * t + 3);
    barrier();
    // ---- q2: A_hi x B_hi
    issue(I0{}, t + 2);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = frag<L>(buf + R_AHI, wr * 64 + 16 * i, s);
    barrier();
    mfma_q(I2{}, bhi);
    barrier();
    // ---- q3: A_hi x B_lo
    issue(I1{}, t + 2);
    if (grp1) wait_for(4 * t + 5);
    barrier();
    mfma_q(I3{}, blo);
    if (!grp1) wait_for(4 * t + 5);
    barrier();
  }
  if (!grp1) barrier();   // equal barrier counts before the epilogue
  } else {
    // PIPE 1: no wave-group stagger; every phase's MFMA burst carries the fragment reads of the next
    // phase (register-pipelined), one barrier per phase.  Reads: B_hi(t) in q0, A_hi(t) in q1 (each
    // A fragment re-read right after its last use), A_lo(t+1) / B_lo(t+1) in q3; a region read in
    // phase P is consumed by P+1's MFMAs, so it is dead after the barrier ending P+1 and refilled in
    // P+2 or later: phase P issues issue-position P + 7 (A_hi(t+1) in q0, A_lo / B_lo / B_hi(t+2) in
    // q1 / q2 / q3).  Before the barrier ending phase P every thread waits for the regions read in
    // P+1 (4 regions younger stay in flight).
    issue(I0{}, 0); issue(I1{}, 0); issue(I2{}, 0); issue(I3{}, 0); issue(I0{}, 1); issue(I1{}, 1); issue(I2{}, 1);
    wait_for(1, 5);
    barrier();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = frag<L>(smem + R_ALO, wr * 64 + 16 * i, s);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) blo[j][s] = frag<L>(smem + R_BLO, wc * 32 + 16 * j, s);
    wait_for(2);
    barrier();
    for (int t = 0; t < nk; ++t) {
      const char* buf = smem + (t & 1) * BUF;
      const char* nbuf = smem + ((t + 1) & 1) * BUF;
      // ---- q0: A_lo x B_lo, reads B_hi(t)
      issue(I3{}, t + 1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], blo[j][s], acc[0][i][j], 0, 0, 0);
          if (i < 2) bhi[i][s] = frag<L>(buf + R_BHI, wc * 32 + 16 * i, s);
        }
      wait_for(4 * t + 3);
      barrier();
      // ---- q1: A_lo x B_hi, reads A_hi(t) into af as each fragment dies
      issue(I0{}, t + 2);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bhi[j][s], acc[1][i][j], 0, 0, 0);
          af[i][s] = frag<L>(buf + R_AHI, wr * 64 + 16 * i, s);
        }
      barrier();
      // ---- q2: A_hi x B_hi
      issue(I1{}, t + 2);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[2][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bhi[j][s], acc[2][i][j], 0, 0, 0);
      wait_for(4 * t + 5);
      barrier();
      // ---- q3: A_hi x B_lo, reads A_lo(t+1) / B_lo(t+1) as fragments die
      issue(I2{}, t + 2);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[3][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], blo[j][s], acc[3][i][j], 0, 0, 0);
            if (j == 1) af[i][s] = frag<L>(nbuf + R_ALO, wr * 64 + 16 * i, s);
          }
          blo[j][s] = frag<L>(nbuf + R_BLO, wc * 32 + 16 * j, s);
        }
      wait_for(4 * t + 6);
      barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: per wave and quadrant, the 64 x 32 fp32 block through a private padded LDS slab
  constexpr int LD = 36;
  float* slab = reinterpret_cast<float*>(smem) + wid * (64 * LD);
  const int crow = 4 * (lane >> 4), ccol = lane & 15;
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    const int rh = (qd == 2 || qd == 3) ? 1 : 0, ch = (qd == 1 || qd == 2) ? 1 : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(16 * i + crow + r) * LD + 16 * j + ccol] = acc[qd][i][j][r];
    __builtin_amdgcn_wave_barrier();
    const int row0 = m0 + 128 * rh + 64 * wr, col0 = n0 + 128 * ch + 32 * wc;
    if constexpr (E == F32_ATOMIC) {
      // one dword per lane: two rows x 128 contiguous bytes per wave-instruction (full atomic rate)
      const int col = col0 + (lane & 31);
      float* cp = static_cast<float*>(p.c);
#pragma unroll 8
      for (int rr = 0; rr < 32; ++rr) {
        const int lr = 2 * rr + (lane >> 5), row = row0 + lr;
        const float v = slab[lr * LD + (lane & 31)];
        if (row < p.M && col < p.N) unsafeAtomicAdd(cp + (int64_t)row * p.ldc + col, v);
      }
    } else {
      // 8 consecutive columns per lane, 4 lanes per row, 16 rows per pass
#pragma unroll
      for (int ps = 0; ps < 4; ++ps) {
        const int lr = 16 * ps + (lane >> 2), c8 = 8 * (lane & 3);
        const int row = row0 + lr, col = col0 + c8;
        const f32x4_t v0 = *reinterpret_cast<const f32x4_t*>(slab + lr * LD + c8);
        const f32x4_t v1 = *reinterpret_cast<const f32x4_t*>(slab + lr * LD + c8 + 4);
        if (row < p.M && col < p.N) {
          if constexpr (E == BF16) {
            u32x4_t o;
            o[0] = pack2bf(v0[0], v0[1]); o[1] = pack2bf(v0[2], v0[3]);
            o[2] = pack2bf(v1[0], v1[1]); o[3] = pack2bf(v1[2], v1[3]);
            *reinterpret_cast<u32x4_t*>(static_cast<uint16_t*>(p.c) + (int64_t)row * p.ldc + col) = o;
          } else {
            f32x4_t* cp = reinterpret_cast<f32x4_t*>(static_cast<float*>(p.c) + (int64_t)row * p.ldc + col);
            const f32x4_t c0 = cp[0], c1 = cp[1];
            cp[0] = c0 + v0;
            cp[1] = c1 + v1;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- PIPE 2: four waves of 128 x 128 (one per SIMD) on v_mfma_f32_32x32x16_bf16 ------------------
// The 8-wave kernel above spends ~30 % of its wave-cycles parked at barriers and fragment waits
// (MFMA busy 57 % at 8192 x 4096 x 4096, SQ_WAIT_ANY 0.315 of wave cycles: profiles/r6_dense_gemm_pmc.txt).
// Here each wave owns a 128 x 128 quarter of the tile -- 4 x 4 32x32 accumulator tiles, 256 registers
// (a lone wave per SIMD has 512) -- and reads 8 fragments per 16 MFMAs of 32 cycles, each k-step's
// fragments read into the other register set while the current one feeds the MFMAs:
//   tile t, k-steps 0..3 (16 k each):  reads (t, ks+1) -> other set | 16 MFMAs on this set
//   after k-step 2: lgkmcnt(0) + vmcnt(0) (this thread's pieces of tile t+1) + ONE barrier; k-step 3
//   reads (t+1, 0) and issues the LDS-DMA of tile t+2 into tile t's buffer (all its reads retired)
// so a tile's DMA has four k-steps (~2,000 cycles) to land.  (The 16x16x32 form of this structure
// made hipcc shuttle the 64 four-register accumulators between AGPRs and VGPRs every iteration.)
// LDS images as above except the TN swizzle: 256-B rows with chunk c of row t at
// c ^ (((t & 3) << 2) | ((t >> 2) & 3)) (cdna_hip_programming.md T10 (b)), under which the 32-lane
// halves of the 32x32x16 transposed operand reads are conflict-free.
constexpr int NT4 = 256;

__device__ __forceinline__ int tn4_swz(int t) { return ((t & 3) << 2) | ((t >> 2) & 3); }

// 32x32x16 operand of region rows / features [x0, x0 + 32), k-step ks (16 k): lane l -> row / feature
// x0 + (l & 31), k = 16 ks + 8 (l >> 5) + j
template <int L>
__device__ __forceinline__ bf16x8_t frag32(const char* reg, int x0, int ks) {
  const int l = threadIdx.x & 63;
  if constexpr (L == LNT) {
    const int r = x0 + (l & 31), ch = 2 * ks + (l >> 5);
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4_t*>(reg + r * 128 + ((ch ^ nt_swz(r)) << 4)));
  } else {
    const int g = l >> 4, q = (l >> 2) & 3, pp = l & 3;
    const int t = 16 * ks + 8 * (g >> 1) + q;
    const int ch = (x0 >> 3) + 2 * (g & 1) + (pp >> 1);
    const char* b0 = reg + t * 256 + ((ch ^ tn4_swz(t)) << 4) + 8 * (pp & 1);
    const char* b1 = reg + (t + 4) * 256 + ((ch ^ tn4_swz(t + 4)) << 4) + 8 * (pp & 1);
    const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)b0);
    const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)b1);
    const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, a8);
  }
}

template <int L, int E>
__global__ void __launch_bounds__(NT4, 1) gemm4_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tiles = p.mt * p.nt;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int split = id / tiles;
  int rt, ct;
  {
    const int within = id - split * tiles;
    const int kb = p.band, bnd = within / (kb * p.nt), rem = within - bnd * kb * p.nt;
    const int h = min(kb, p.mt - bnd * kb);
    rt = bnd * kb + rem % h;
    ct = rem / h;
  }
  const int m0 = rt * BM, n0 = ct * BN;
  const int k_begin = split * p.k_per_split;
  const int k_end = min(p.K, k_begin + p.k_per_split);
  const int nk = (k_end - k_begin) / BK;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wid >> 1, wc = wid & 1;

  f32x16_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Per-lane DMA sources of K-tile 0.  Full tiles only (M, N % 256 == 0: the launcher checks), so the
  // 4 pieces x 2 halves of one operand differ by uniform row / token offsets, except for the source
  // swizzle: NT's depends on the piece's parity (2 pointers per operand), TN's on the piece (4).
  constexpr int NV = L == LNT ? 2 : 4;
  const uint16_t* sa[NV];
  const uint16_t* sb[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if constexpr (L == LNT) {
      const int pr = 8 * (4 * wid + v) + (lane >> 3), c = (lane & 7) ^ nt_swz(pr);
      sa[v] = p.a + (int64_t)(m0 + pr) * p.lda + k_begin + 8 * c;
      sb[v] = p.b + (int64_t)(n0 + pr) * p.ldb + k_begin + 8 * c;
    } else {
      const int pr = 4 * (4 * wid + v) + (lane >> 4), c = (lane & 15) ^ tn4_swz(pr);
      sa[v] = p.a + (int64_t)(k_begin + pr) * p.lda + m0 + 8 * c;
      sb[v] = p.b + (int64_t)(k_begin + pr) * p.ldb + n0 + 8 * c;
    }
  }
  auto pv = [](int j) { return L == LNT ? (j & 1) : j; };
  auto poff = [&](int h, int j, int64_t ld) -> int64_t {
    if constexpr (L == LNT) return (int64_t)(128 * h + 8 * (j & ~1)) * ld;
    else return (int64_t)128 * h;
  };
  const int64_t adv_a = L == LNT ? (int64_t)BK : (int64_t)BK * p.lda;
  const int64_t adv_b = L == LNT ? (int64_t)BK : (int64_t)BK * p.ldb;
  const uint32_t lds0 = lds_addr(smem);
  // piece q (0..15) of K-tile s: region q / 4 (A_lo, A_hi, B_lo, B_hi), piece j = q % 4
  auto issue_piece = [&](int s, int q) {
    const int r = q >> 2, j = q & 3, h = r & 1;
    const uint32_t dst = lds0 + (s & 1) * BUF + (r == 0 ? R_ALO : r == 1 ? R_AHI : r == 2 ? R_BLO : R_BHI) + wid * 4096 + j * 1024;
    const uint16_t* src = r < 2 ? sa[pv(j)] + (int64_t)s * adv_a + poff(h, j, p.lda)
                                : sb[pv(j)] + (int64_t)s * adv_b + poff(h, j, p.ldb);
    dma16(src, __builtin_amdgcn_readfirstlane(dst));
  };
  const int ra = wr ? R_AHI : R_ALO, rb = wc ? R_BHI : R_BLO;
  bf16x8_t fa0[4], fb0[4], fa1[4], fb1[4];
  auto rd = [&](const char* buf, int ks, bf16x8_t (&fa)[4], bf16x8_t (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag32<L>(buf + ra, 32 * i, ks);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag32<L>(buf + rb, 32 * j, ks);
  };
  auto mm = [&](bf16x8_t (&fa)[4], bf16x8_t (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };

#pragma unroll
  for (int q = 0; q < 16; ++q) issue_piece(0, q);
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) issue_piece(1, q);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  rd(smem, 0, fa0, fb0);
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    rd(buf, 1, fa1, fb1);
    mm(fa0, fb0);
    rd(buf, 2, fa0, fb0);
    mm(fa1, fb1);
    rd(buf, 3, fa1, fb1);
    mm(fa0, fb0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's pieces of tile t+1
    barrier();
    rd(smem + ((t + 1) & 1) * BUF, 0, fa0, fb0);      // past the last tile: stale LDS, never consumed
    if (t + 2 < nk) {
#pragma unroll
      for (int q = 0; q < 16; ++q) issue_piece(t + 2, q);
    }
    mm(fa1, fb1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: per wave 4 passes of 32 rows x 128 columns through a padded fp32 LDS slab
  constexpr int LD = 132;
  float* slab = reinterpret_cast<float*>(smem) + wid * (32 * LD);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        slab[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LD + 32 * j + (lane & 31)] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    const int row0 = m0 + 128 * wr + 32 * i, col0 = n0 + 128 * wc;
    if constexpr (E == F32_ATOMIC) {
      float* cp = static_cast<float*>(p.c);
#pragma unroll 2
      for (int rr = 0; rr < 64; ++rr) {   // half a row (256 contiguous bytes) per wave-instruction
        const int lr = rr >> 1, col = col0 + 64 * (rr & 1) + lane, row = row0 + lr;
        const float v = slab[lr * LD + 64 * (rr & 1) + lane];
        if (row < p.M && col < p.N) unsafeAtomicAdd(cp + (int64_t)row * p.ldc + col, v);
      }
    } else {
#pragma unroll
      for (int ps = 0; ps < 8; ++ps) {   // 16 lanes x 8 columns per row, 4 rows per pass
        const int lr = 4 * ps + (lane >> 4), c8 = 8 * (lane & 15);
        const int row = row0 + lr, col = col0 + c8;
        const f32x4_t v0 = *reinterpret_cast<const f32x4_t*>(slab + lr * LD + c8);
        const f32x4_t v1 = *reinterpret_cast<const f32x4_t*>(slab + lr * LD + c8 + 4);
        if (row < p.M && col < p.N) {
          if constexpr (E == BF16) {
            u32x4_t o;
            o[0] = pack2bf(v0[0], v0[1]); o[1] = pack2bf(v0[2], v0[3]);
            o[2] = pack2bf(v1[0], v1[1]); o[3] = pack2bf(v1[2], v1[3]);
            *reinterpret_cast<u32x4_t*>(static_cast<uint16_t*>(p.c) + (int64_t)row * p.ldc + col) = o;
          } else {
            f32x4_t* cp = reinterpret_cast<f32x4_t*>(static_cast<float*>(p.c) + (int64_t)row * p.ldc + col);
            const f32x4_t c0 = cp[0], c1 = cp[1];
            cp[0] = c0 + v0;
            cp[1] = c1 + v1;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

static int g_pipe = -1;   // main-loop variant override (dense_gemm_set_pipe, in-process A/B)

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

}  // namespace dg

void dense_gemm_set_pipe(int v) { dg::g_pipe = v; }

// K splits of the atomic epilogue: grid waves of 256 workgroups x (K-steps per split + the atomic
// epilogue's cost in K-steps, ~6); splits stay 1 unless they save at least a tenth.
int dense_gemm_choose_splits(int M, int N, int K) {
  const int tiles = ceil_div(M, dg::BM) * ceil_div(N, dg::BN);
  const int steps = K / dg::BK;
  const int64_t base = (int64_t)ceil_div(tiles, 256) * steps;
  int best = 1;
  int64_t best_cost = base;
  for (int s = 2; s <= 8 && s <= steps; ++s) {
    if (steps / s < 8) break;
    const int64_t cost = (int64_t)ceil_div(tiles * s, 256) * (ceil_div(steps, s) + 6);
    if (cost * 10 < best_cost * 9 && cost < best_cost) {
      best_cost = cost;
      best = s;
    }
  }
  return best;
}

// layout 0 NT: a [M][K] (lda), b [N][K] (ldb); layout 1 TN: a [K][M], b [K][N].
// epi 0: c bf16 [M][N] = acc; 1: c fp32 += acc (splits forced to 1); 2: c fp32 += acc by atomics,
// `splits` K splits (<= 0: chosen).  K % 64 == 0, N % 8 == 0, TN also M % 8 == 0, ld* % 8 == 0.
int dense_gemm_launch(int layout, int epi, const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc,
                      int M, int N, int K, int splits, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % dg::BK || N % 8 || lda % 8 || ldb % 8 || ldc % 4) return -1;
  if (layout == dg::LTN && M % 8) return -1;
  if (epi == dg::BF16 && ldc % 8) return -1;
  dg::Params p{};
  p.a = static_cast<const uint16_t*>(a);
  p.b = static_cast<const uint16_t*>(b);
  p.c = c;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.mt = ceil_div(M, dg::BM);
  p.nt = ceil_div(N, dg::BN);
  const int steps = K / dg::BK;
  if (epi != dg::F32_ATOMIC) splits = 1;
  else if (splits <= 0) splits = dense_gemm_choose_splits(M, N, K);
  splits = splits < 1 ? 1 : (splits > steps ? steps : splits);
  p.k_per_split = ceil_div(steps, splits) * dg::BK;
  p.splits = ceil_div(K, p.k_per_split);
  static const int band = [] { const int v = dg::env_int("NXD_DG_BAND", 8); return v > 0 ? v : 8; }();
  p.band = band;
  const int64_t nwg = (int64_t)p.mt * p.nt * p.splits;
  if (nwg > INT32_MAX) return -2;
  // default: the 8-wave register-pipelined loop (PIPE 1), the fastest of the three on every measured
  // shape (profiles/r6_dense_gemm_pipes_vs_hipblaslt.jsonl: PIPE 2 5-20 % slower, PIPE 0 2-9 %)
  static int pipe_env = dg::env_int("NXD_DG_PIPE", 1);
  int pipe = dg::g_pipe >= 0 ? dg::g_pipe : pipe_env;
  if (pipe == 2 && (M % dg::BM || N % dg::BN)) pipe = 1;   // the 4-wave kernel takes whole tiles only
#define NXD_DG_LAUNCH(LY, EP)                                                                                  \
  do {                                                                                                       \
    if (pipe == 2) hipLaunchKernelGGL((dg::gemm4_kernel<LY, EP>), dim3((unsigned)nwg), dim3(dg::NT4), 0, stream, p); \
    else if (pipe) hipLaunchKernelGGL((dg::gemm_kernel<LY, EP, 1>), dim3((unsigned)nwg), dim3(dg::NT), 0, stream, p); \
    else hipLaunchKernelGGL((dg::gemm_kernel<LY, EP, 0>), dim3((unsigned)nwg), dim3(dg::NT), 0, stream, p);      \
  } while (0)
  if (layout == dg::LNT) {
    if (epi == dg::BF16) NXD_DG_LAUNCH(dg::LNT, dg::BF16);
    else if (epi == dg::F32_ACC) NXD_DG_LAUNCH(dg::LNT, dg::F32_ACC);
    else NXD_DG_LAUNCH(dg::LNT, dg::F32_ATOMIC);
  } else {
    if (epi == dg::BF16) NXD_DG_LAUNCH(dg::LTN, dg::BF16);
    else if (epi == dg::F32_ACC) NXD_DG_LAUNCH(dg::LTN, dg::F32_ACC);
    else NXD_DG_LAUNCH(dg::LTN, dg::F32_ATOMIC);
  }
#undef NXD_DG_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace nxd
