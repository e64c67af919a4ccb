// Decode attention on MFMA for small query groups (M = (Hq/Hkv) * T <= 16 rows per kv head):
// one workgroup (8 waves at D 64, 4 at D 128) owns a (batch, kv head, key split); the keys per split
// (128-1,024, keys_per_split) are sized so the grid reaches ~128 workgroups; every wave runs an
// online-softmax flash-decoding loop over 64-key chunks entirely in registers:
//
//   S^T[key][m] = K.Q^T   v_mfma_f32_16x16x32_bf16, K rows straight from the cache (16-B loads),
//                         Q^T fragments held for the whole loop (rows >= M are zero);
//   softmax             16 scores per lane (4 key tiles x 4), row max / sum over the 4 lanes of a
//                         query row with two xor-shuffles, exp2 with the scale folded in;
//   O[m][d] += P.V      P re-packed into the A operand with 16 lane shuffles per chunk, V staged
//                         through a per-wave LDS tile and read transposed (ds_read_b64_tr_b16);
//
// then the waves merge their (max, sum, O) through LDS once.  With one split the workgroup writes
// the final bf16 output; otherwise it writes the (m, l, o) partials that inference.hip's merge kernel
// -- or, fused with o_proj, merge_oproj_kernel below -- combines.  Compared with the 128-key-chunk
// kernel there (four workgroup barriers per chunk and a merge launch at every length) this is one
// barrier per call.
//
// FUSE (attention + o_proj, one launch instead of two; caches up to NXD_DECODE_ATTN_OPROJ_MAXL =
// 1,024 keys): the grid is (batch, kv head, R row chunks
// of the o_proj output); every workgroup of a kv head recomputes that head group's attention (a
// few hundred L2-resident keys at decode lengths) and multiplies it by its Wo block [H/R rows x
// G*D columns], prefetched into registers before the attention starts, then adds the partial
// rows into an fp32 accumulator with float atomics (G*D columns of the o_proj reduction per
// workgroup).  No cross-workgroup wait: the next launch (the GLU projection's RMSNorm prologue and
// the down projection's residual epilogue, decode_fused.hip xadd / yadd) folds the accumulator into
// the residual stream with the rounding of the unfused o_proj epilogue and zeroes it.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace nxd {
namespace dattn {

constexpr int KB = 64;            // keys per chunk (one wave)
constexpr int KPS = 1024;         // most keys per workgroup split (one pass of 8 waves x 2 chunks)

struct Params {
  const uint16_t* q;
  int64_t q_sb, q_st, q_sh;
  const uint16_t* kc;
  const uint16_t* vc;
  int64_t c_sb, c_sh, c_sl;
  const int* cache_idx;
  const int* seq_len;
  uint16_t* out;
  int64_t o_sb, o_st, o_sh;
  float* po;   // [B*Hkv, nsplit, M, D] partials (nsplit > 1)
  float* pm;   // natural-log row max
  float* pl;
  int B, T, Hq, Hkv, nsplit;
  int kps;            // keys per split (multiple of KB; FUSE: unused)
  float scale_log2;   // softmax scale * log2(e)
  // weight prefetch riding on the (tiny) attention grid: workgroups >= attn_wgs stream the two
  // byte ranges through the memory hierarchy so the next projections (o_proj, gate_up) find them
  // in the Infinity Cache instead of cold HBM; the attention itself leaves HBM idle
  const u32x4_t* pf[2];
  int64_t pf_n16[2];   // 16-byte chunks per range
  int attn_wgs;
  // FUSE: o_proj weight [Hout, Hq * D] (row stride ldwo), fp32 accumulator [B * T, Hout]
  const uint16_t* wo;
  int64_t ldwo;
  float* oacc;
  int Hout, R, NP;     // output rows, row chunks per kv head, Wo register passes (<= 4)
  // opt-in phase trace (decode_attn_set_trace): wave 0 of each workgroup stores s_memrealtime (100 MHz)
  // at entry and exit to trace[2 * blockIdx.x + {0, 1}]; null = off.  This is the trailing field whose
  // round-4 version aborted the decode tests: decode_attn2_launch built `Params p;` without value-
  // initialisation, so the field was stack garbage (non-null) there and the kernel stored through it
  // (profiles/r4_decode_attn_trace_abort.txt).  Every launcher now value-initialises its Params.
  uint64_t* trace;
  // SYNC (fused, long caches): per-(batch, kv head) arrival / done counters [2][kSyncHeads] (device
  // globals, zero at load, reset by the last workgroup of each head) and the bounded-spin error word
  unsigned* sync_cnt;
  int* sync_err;
  float* mo;          // SYNC: [B * Hkv, M, D] merged attention rows (the merger's hand-off)
};
static_assert(std::is_trivially_copyable<Params>::value && sizeof(Params) <= 4096, "kernel-argument struct");

static uint64_t* g_trace = nullptr;

constexpr int kSyncHeads = 4096;   // batch x kv heads covered by the SYNC counters
__device__ unsigned g_sync_cnt[3 * kSyncHeads];   // arrivals, done, merged-flag per head
__device__ int g_sync_err;

// Prefetch workgroup body: 4 independent 16-B loads in flight per lane, folded into one value that
// is stored only under a condition the host never creates (pf_n16[0] < 0), so the loads stay live.
__device__ __forceinline__ void prefetch_body(const Params& p, int wg, int nwg) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)nwg * blockDim.x;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const u32x4_t* base = p.pf[r];
    const int64_t n = p.pf_n16[r];
    int64_t i = (int64_t)wg * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      const u32x4_t a = base[i], b = base[i + stride], c = base[i + 2 * stride], d = base[i + 3 * stride];
      acc ^= a[0] ^ b[1] ^ c[2] ^ d[3];
    }
    for (; i < n; i += stride) acc ^= base[i][0];
  }
  if (p.pf_n16[0] < 0) p.pm[threadIdx.x] = __uint_as_float(acc);
}

typedef __attribute__((address_space(3))) short4_t lds_s4_t;
typedef short short8_t __attribute__((ext_vector_type(8)));

// FUSE o_proj pieces: thread (row row0 + pass * rpp, 32-column segment) holds its Wo block in
// registers (<= 4 passes), then adds its rows' dot products with the attention output into oacc.
__device__ __forceinline__ void load_wo_regs(const Params& p, int row0, int col0, int rpp, u32x4_t (&wreg)[4][4]) {
  const uint16_t* wb = p.wo + (int64_t)row0 * p.ldwo + col0;
#pragma unroll
  for (int np = 0; np < 4; ++np) {
    if (np < p.NP) {
#pragma unroll
      for (int j = 0; j < 4; ++j) wreg[np][j] = *reinterpret_cast<const u32x4_t*>(wb + (int64_t)np * rpp * p.ldwo + 8 * j);
    }
  }
}

// out[t][row] += sum_c Wo[row][hkv*G*D + c] o[t][c] over this thread's 32 columns, reduced over the
// tpr threads of a row; of = [M][D] attention output (m = t * G + g)
template <int D>
__device__ __forceinline__ void oproj_tail(const Params& p, const float* of, const u32x4_t (&wreg)[4][4], int b, int row0,
                                           int rpp, int tpr, int seg, int G) {
  const int c0 = 32 * seg, gg = c0 / D, d0 = c0 % D;
#pragma unroll
  for (int np = 0; np < 4; ++np) {
    if (np >= p.NP) break;
    float w[32];
#pragma unroll
    for (int j = 0; j < 4; ++j) unpack8(wreg[np][j], w + 8 * j);
    const int row = row0 + np * rpp;
    for (int tt = 0; tt < p.T; ++tt) {
      const float* orow = of + (tt * G + gg) * D + d0;
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < 32; j += 4) {
        const f32x4_t o4 = *reinterpret_cast<const f32x4_t*>(orow + j);
        dot += w[j] * o4[0] + w[j + 1] * o4[1] + w[j + 2] * o4[2] + w[j + 3] * o4[3];
      }
      for (int off = tpr / 2; off > 0; off >>= 1) dot += __shfl_xor(dot, off, 64);
      if (seg == 0) unsafeAtomicAdd(p.oacc + (int64_t)(b * p.T + tt) * p.Hout + row, dot);
    }
  }
}

// SYNC (with FUSE, caches past one pass): workgroup r of a kv head's R also computes key split r
// (kps keys; splits >= nsplit have none) and publishes its (m, l, o) partial with write-through (sc1)
// stores and an agent-scope arrival count; the split whose arrival completes the count merges the
// head once and publishes the merged rows (write-through) and a flag, which the head's other
// workgroups poll (bounded spin: every workgroup of the grid is resident, the host caps the grid at
// the CU count) before their o_proj slices: split-K attention + merge + o_proj in one launch, the KV
// cache read once.  The last workgroup of a head through the hand-off resets the head's counters.
// Measured SLOWER than the two launches it replaces at the notebook config (16.1 us per layer --
// 17.9 with every workgroup merging all partials itself -- vs 5.7 + 5.6 us; 0.759 vs 0.686
// ms/token; profiles/r6_decode/sync_ab.txt): the in-launch wait on the slowest split of a head costs
// more than a kernel boundary, so it is off by default (NXD_DECODE_ATTN_SYNC=1).
template <int D, int NWV, bool FUSE, bool WO_LATE = true, bool SYNC = false>
__global__ void __launch_bounds__(64 * NWV) attn_kernel(Params p) {
  static_assert(!SYNC || FUSE, "SYNC is a FUSE form");
  constexpr int NS = D / 32;      // k-steps of the score MFMA
  constexpr int NDT = D / 16;     // 16-wide d tiles of the output
  constexpr int VL = D / 8;       // 16-B V loads per lane for 64 keys x D
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mi = lane & 15, g = lane >> 4;
  uint16_t* vt = reinterpret_cast<uint16_t*>(smem) + wid * KB * D;              // this wave's V tile [64][D]
  float* red_o = reinterpret_cast<float*>(smem + NWV * KB * D * 2);             // [NWV][16][D]
  float* red_m = red_o + NWV * 16 * D;                                          // [NWV][16]
  float* red_l = red_m + NWV * 16;

  if (!FUSE && (int)blockIdx.x >= p.attn_wgs) {
    prefetch_body(p, blockIdx.x - p.attn_wgs, gridDim.x - p.attn_wgs);
    return;
  }
  if (p.trace != nullptr && tid == 0) p.trace[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  const int split = FUSE ? (SYNC ? (int)blockIdx.x % p.R : 0) : (int)blockIdx.x % p.nsplit;
  const int bh = FUSE ? (int)blockIdx.x / p.R : (int)blockIdx.x / p.nsplit;
  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int G = p.Hq / p.Hkv, M = G * p.T;
  // FUSE: this workgroup's Wo block (rows rc * NR .., columns of head group hkv) into registers,
  // in flight during the attention so its HBM latency hides behind it.  Thread (row r0 + pass * RPP,
  // 32-column segment seg).
  const int tpr = FUSE ? (G * D) / 32 : 1;
  const int seg = tid % tpr, r0 = tid / tpr, rpp = (64 * NWV) / tpr;
  const int nr = FUSE ? p.Hout / p.R : 0;
  const int row0 = FUSE ? ((int)blockIdx.x % p.R) * nr + r0 : 0;
  u32x4_t wreg[4][4];
  auto load_wo = [&]() { load_wo_regs(p, row0, hkv * G * D + 32 * seg, rpp, wreg); };
  if constexpr (FUSE && !WO_LATE) load_wo();   // round-3 order (A/B: NXD_DECODE_WO_LATE=0)
  const int cb = p.cache_idx ? p.cache_idx[b] : b;
  const int slen = p.seq_len[b];
  const uint16_t* kbase = p.kc + (int64_t)cb * p.c_sb + (int64_t)hkv * p.c_sh;
  const uint16_t* vbase = p.vc + (int64_t)cb * p.c_sb + (int64_t)hkv * p.c_sh;

  // Q^T fragments: lane (mi, g) holds Q[mi][32 s + 8 g .. +7]
  bf16x8_t qf[NS];
  const int tt_q = mi / G, gg_q = mi % G;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    u32x4_t v = {0, 0, 0, 0};
    if (mi < M)
      v = *reinterpret_cast<const u32x4_t*>(p.q + (int64_t)b * p.q_sb + (int64_t)tt_q * p.q_st +
                                             (int64_t)(hkv * G + gg_q) * p.q_sh + 32 * s + 8 * g);
    qf[s] = __builtin_bit_cast(bf16x8_t, v);
  }
  const int lim = slen - (p.T - 1 - tt_q);        // keys visible to query row mi (causal over new tokens)

  float run_m = -INFINITY, run_l = 0.f;           // stats of query row mi (log2 domain)
  f32x4_t o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // FUSE: the whole cache in one pass per workgroup (no key splits, no merge launch)
  const int kend = (FUSE && !SYNC) ? slen : min(slen, (split + 1) * p.kps);
  // K fragments and the V chunk of the NEXT chunk are loaded while this one runs its softmax and P.V
  u32x4_t kf[4][NS], vv[VL];
  auto load_chunk = [&](int k0) {
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int idx = lane + 64 * i, key = idx / (D / 8), c = idx % (D / 8);
      vv[i] = *reinterpret_cast<const u32x4_t*>(vbase + (int64_t)min(k0 + key, slen - 1) * p.c_sl + 8 * c);
    }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const uint16_t* kr = kbase + (int64_t)min(k0 + kt * 16 + mi, slen - 1) * p.c_sl + 8 * g;
#pragma unroll
      for (int s = 0; s < NS; ++s) kf[kt][s] = *reinterpret_cast<const u32x4_t*>(kr + 32 * s);
    }
  };
  int k0 = split * p.kps + wid * KB;
  if (k0 < kend) load_chunk(k0);
  // FUSE: the Wo block is issued AFTER the q and first K / V loads.  vmcnt retires in issue order:
  // issued first (round 3), the cold-HBM Wo loads had to land before the first score MFMA could
  // read its L2-resident K fragments, so their latency was added to the attention instead of
  // hidden behind it (attention + o_proj 7.16 -> 6.92 us, 0.619 -> 0.614 ms/token alternating, profiles/r4_decode_wo_late_ab.txt).
  if constexpr (FUSE && WO_LATE) load_wo();
  for (; k0 < kend; k0 += NWV * KB) {
    // ---- scores S^T[key][m] for 4 key tiles of 16
    f32x4_t sc[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      sc[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s)
        sc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf[kt][s]), qf[s], sc[kt], 0, 0, 0);
    }
    // V tile -> LDS (row-major [key][D]) once the wave's previous transposed reads have retired
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < VL; ++i) {
      const int idx = lane + 64 * i, key = idx / (D / 8), c = idx % (D / 8);
      *reinterpret_cast<u32x4_t*>(vt + key * D + 8 * c) = vv[i];
    }
    if (k0 + NWV * KB < kend) load_chunk(k0 + NWV * KB);
    // ---- online softmax of query row mi over this chunk: lane holds keys k0 + 16 kt + 4 g + v
    float cm = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int key = k0 + kt * 16 + 4 * g + v;
        const float sv = key < lim ? sc[kt][v] * p.scale_log2 : -INFINITY;
        sc[kt][v] = sv;
        cm = fmaxf(cm, sv);
      }
    cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    const float nm = fmaxf(run_m, cm);
    const float mu = nm == -INFINITY ? 0.f : nm;
    const float alpha = run_m == -INFINITY ? 0.f : exp2f(run_m - mu);
    float ls = 0.f;
    uint32_t p2[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float e[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        e[v] = exp2f(sc[kt][v] - mu);
        ls += e[v];
      }
      p2[kt][0] = pack2bf(e[0], e[1]);
      p2[kt][1] = pack2bf(e[2], e[3]);
    }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    run_l = run_l * alpha + ls;
    run_m = nm;
    // rescale O rows 4 g + v by their row's alpha (held by lane 4 g + v)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float a = __shfl(alpha, 4 * g + v, 64);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt][v] *= a;
    }
    // ---- P as the A operand: lane (mi, h) needs P[mi][32 ks + 8 h + j], j = 0..7
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int src0 = (2 * (g & 1)) * 16 + mi, src1 = src0 + 16;
      const bool hi = (g >> 1) != 0;
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t a0 = __shfl(p2[2 * ks][q], src0, 64), b0 = __shfl(p2[2 * ks + 1][q], src0, 64);
        const uint32_t a1 = __shfl(p2[2 * ks][q], src1, 64), b1 = __shfl(p2[2 * ks + 1][q], src1, 64);
        w[q] = hi ? b0 : a0;
        w[2 + q] = hi ? b1 : a1;
      }
      const u32x4_t pw = {w[0], w[1], w[2], w[3]};
      const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, pw);
      // V B-fragments: keys 32 ks + 8 g + (0..3 | 4..7), columns 16 dt + 4 p of the 16-lane group
      const int qrow = (lane & 15) >> 2, pc = lane & 3;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const uint16_t* a = vt + (32 * ks + 8 * g + qrow) * D + 16 * dt + 4 * pc;
        const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)a);
        const short4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a + 4 * D));
        const short8_t v8 = {lo[0], lo[1], lo[2], lo[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8_t, v8), o[dt], 0, 0, 0);
      }
    }
  }

  // ---- merge the 4 waves: stats of row mi from lanes g == 0, O rows 4 g + v, cols 16 dt + (lane & 15)
  if (g == 0) {
    red_m[wid * 16 + mi] = run_m;
    red_l[wid * 16 + mi] = run_l;
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int v = 0; v < 4; ++v) red_o[(wid * 16 + 4 * g + v) * D + 16 * dt + (lane & 15)] = o[dt][v];
  __syncthreads();
  const int64_t pbase = ((int64_t)bh * p.nsplit + split) * M;
  for (int it = tid; it < M * D; it += 64 * NWV) {
    const int m = it / D, d = it % D;
    float gm = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWV; ++w) gm = fmaxf(gm, red_m[w * 16 + m]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float mw = red_m[w * 16 + m];
      const float wt = (mw == -INFINITY) ? 0.f : exp2f(mw - gm);
      L += wt * red_l[w * 16 + m];
      acc += wt * red_o[(w * 16 + m) * D + d];
    }
    if (FUSE && !SYNC) {   // bf16-rounded as the unfused path's attention output, then o_proj below
      reinterpret_cast<float*>(smem)[m * D + d] = bf2f(f2bf(L > 0.f ? acc / L : 0.f));
    } else if (SYNC) {   // write-through partials (the merge reads them from other workgroups)
      if (split < p.nsplit) {
        __hip_atomic_store(p.po + (pbase + m) * D + d, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 0) {
          __hip_atomic_store(p.pm + pbase + m, gm == -INFINITY ? -INFINITY : gm * 0.69314718056f, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(p.pl + pbase + m, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else if (p.nsplit == 1) {
      const int tt = m / G, gg = m % G;
      p.out[(int64_t)b * p.o_sb + (int64_t)tt * p.o_st + (int64_t)(hkv * G + gg) * p.o_sh + d] =
          f2bf(L > 0.f ? acc / L : 0.f);
    } else {
      p.po[(pbase + m) * D + d] = acc;
      if (d == 0) {
        p.pm[pbase + m] = gm == -INFINITY ? -INFINITY : gm * 0.69314718056f;   // log2 -> natural-log domain
        p.pl[pbase + m] = L;
      }
    }
  }
  if constexpr (SYNC) {
    int* flg = reinterpret_cast<int*>(red_m);   // [0] lost, [1] merger: red_m is free once the waves are
                                                // merged (no static __shared__: it would shift the LDS base)
    float* of = reinterpret_cast<float*>(smem);   // [M][D] merged attention output
    float* wts = of + 16 * D;                     // [nsplit][16]
    const int ns = p.nsplit;
    const int64_t pb = (int64_t)bh * ns * M;
    float* mo = p.mo + (int64_t)bh * M * D;       // the head's merged output, handed to its other workgroups
    unsigned* cnt = p.sync_cnt + bh;
    unsigned* done = p.sync_cnt + kSyncHeads + bh;
    unsigned* flag = p.sync_cnt + 2 * kSyncHeads + bh;
    // publish: every storing wave drains its write-through partial stores, then one arrival per split;
    // the split whose arrival completes the count merges the head once
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int merger = 0;
      if (split < ns) merger = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)ns - 1;
      flg[0] = 0;
      flg[1] = merger;
    }
    __syncthreads();
    if (flg[1]) {
      // every split's partial has arrived: merge (write-through / sc1 loads: no stale line from an
      // earlier launch), publish the merged rows write-through, then the head's flag
      for (int m = wid; m < M; m += NWV) {
        float gm = -INFINITY;
        for (int sp = lane; sp < ns; sp += 64)
          gm = fmaxf(gm, __hip_atomic_load(p.pm + pb + (int64_t)sp * M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) gm = fmaxf(gm, __shfl_xor(gm, off, 64));
        float L = 0.f;
        for (int sp = lane; sp < ns; sp += 64) {
          const float ms = __hip_atomic_load(p.pm + pb + (int64_t)sp * M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float w = ms == -INFINITY ? 0.f : __expf(ms - gm);
          wts[sp * 16 + m] = w;
          L += w * __hip_atomic_load(p.pl + pb + (int64_t)sp * M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) L += __shfl_xor(L, off, 64);
        const float inv = L > 0.f ? 1.f / L : 0.f;
        for (int sp = lane; sp < ns; sp += 64) wts[sp * 16 + m] *= inv;
      }
      __syncthreads();
      for (int it = tid; it < M * D; it += 64 * NWV) {
        const int m = it / D;
        const float* src = p.po + (pb + m) * D + it % D;
        const int64_t st = (int64_t)M * D;
        float acc = 0.f;
        int sp = 0;
        for (; sp + 3 < ns; sp += 4) {
          const float a0 = __hip_atomic_load(src + sp * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float a1 = __hip_atomic_load(src + (sp + 1) * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float a2 = __hip_atomic_load(src + (sp + 2) * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float a3 = __hip_atomic_load(src + (sp + 3) * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          acc += wts[sp * 16 + m] * a0 + wts[(sp + 1) * 16 + m] * a1 + wts[(sp + 2) * 16 + m] * a2 + wts[(sp + 3) * 16 + m] * a3;
        }
        for (; sp < ns; ++sp) acc += wts[sp * 16 + m] * __hip_atomic_load(src + sp * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float v = bf2f(f2bf(acc));
        of[it] = v;
        __hip_atomic_store(mo + it, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (tid == 0) {
        for (unsigned spins = 0; __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1u << 24)) {   // ~0.5 s: the head's merge never arrived
            flg[0] = 1;
            __hip_atomic_store(p.sync_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __syncthreads();
      const bool lost = flg[0] != 0;
      for (int it = tid; it < M * D; it += 64 * NWV)
        of[it] = lost ? __builtin_nanf("") : __hip_atomic_load(mo + it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();   // the merged rows are in LDS: this workgroup is done with the hand-off
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == (unsigned)p.R - 1) {   // the head's last workgroup: every peer has read the merged rows
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if constexpr (FUSE) {
    __syncthreads();
    oproj_tail<D>(p, reinterpret_cast<const float*>(smem), wreg, b, row0, rpp, tpr, seg, G);
  }
  if (p.trace != nullptr && tid == 0) p.trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}

// Keys per split: enough splits that the (batch, kv head, split) grid reaches ~NXD_DECODE_ATTN_WGS
// workgroups (default 128) -- the KV cache streams from HBM at the per-CU rate, so 24 workgroups on a
// 2,304-key cache took 9.8 us -- between 128 keys (the caller's partial buffers hold Lmax / 128
// splits) and 1,024 (one pass of the 8 waves x 2 chunks).  0.786 -> 0.726 ms/token at the notebook
// config (profiles/r6_decode/attn_split_ab.txt).
static int keys_per_split(int Lmax, int B, int Hkv) {
  static const int target = [] {
    const char* e = getenv("NXD_DECODE_ATTN_WGS");
    const int v = e ? atoi(e) : 128;
    return v > 0 ? v : 128;
  }();
  int kps = (int)(((int64_t)Lmax * B * Hkv + target - 1) / target);
  kps = (kps + KB - 1) / KB * KB;
  return kps < 128 ? 128 : (kps > KPS ? KPS : kps);
}

// Split attention's partials -> merged attention row block (bf16-rounded, as the merge kernel's
// output the o_proj GEMV would read) -> this workgroup's o_proj partial, fp32 atomics into oacc: the
// long-context form of FUSE (one launch instead of the merge + o_proj pair).  Grid (batch, kv head,
// R row chunks), the split weights of each query row in LDS.
template <int D, int NWV>
__global__ void __launch_bounds__(64 * NWV) merge_oproj_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* of = reinterpret_cast<float*>(smem);   // [M][D] merged attention output
  float* wts = of + 16 * D;                     // [nsplit][16] normalised split weights
  const int tid = threadIdx.x;
  const int bh = (int)blockIdx.x / p.R, b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int G = p.Hq / p.Hkv, M = G * p.T;
  const int tpr = (G * D) / 32, seg = tid % tpr, r0 = tid / tpr, rpp = (64 * NWV) / tpr;
  const int row0 = ((int)blockIdx.x % p.R) * (p.Hout / p.R) + r0;
  const int64_t pb = (int64_t)bh * p.nsplit * M;
  const int ns = p.nsplit, lane = tid & 63, wid = tid >> 6;
  // the splits are divided over H thread groups (partials summed through LDS); when a thread's share
  // fits in registers its partial-row loads are issued first, beside the stats loads below, so the
  // merge costs one memory round trip instead of two
  constexpr int PMAX = 16;
  const int elems = M * D, H = (64 * NWV) / elems >= 2 ? 2 : 1;
  const int64_t st = (int64_t)M * D;   // one split further
  const bool regs = elems * H <= 64 * NWV && (ns + H - 1) / H <= PMAX;
  const int e0 = tid % elems, h0 = tid / elems;
  const float* src0 = p.po + (pb + e0 / D) * D + e0 % D;
  float pv[PMAX];
  if (regs && tid < elems * H) {
#pragma unroll
    for (int i = 0; i < PMAX; ++i)
      if (h0 + i * H < ns) pv[i] = src0[(h0 + i * H) * st];
  }
  // split weights of query row m: one wave per row, one split per lane (all loads in parallel: a
  // serial walk over the splits was a chain of dependent L2 round trips, 7.8 us per launch).  The
  // stats are loaded before the Wo block, whose HBM latency then hides behind the merge (vmcnt
  // retires in issue order: issued first, Wo would gate the first use of the stats)
  constexpr int KM = (16 + NWV - 1) / NWV;   // rows per wave (M <= 16)
  const bool fast = regs && ns <= 64;
  float pmv[KM], plv[KM];
  if (fast) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int m = wid + k * NWV;
      const bool ok = m < M && lane < ns;
      pmv[k] = ok ? p.pm[pb + (int64_t)lane * M + m] : -INFINITY;
      plv[k] = ok ? p.pl[pb + (int64_t)lane * M + m] : 0.f;
    }
  }
  u32x4_t wreg[4][4];
  load_wo_regs(p, row0, hkv * G * D + 32 * seg, rpp, wreg);
  if (fast) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int m = wid + k * NWV;
      if (m >= M) break;   // wave-uniform
      float gm = pmv[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) gm = fmaxf(gm, __shfl_xor(gm, off, 64));
      const float w = pmv[k] == -INFINITY ? 0.f : __expf(pmv[k] - gm);
      float L = w * plv[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) L += __shfl_xor(L, off, 64);
      if (lane < ns) wts[lane * 16 + m] = L > 0.f ? w / L : 0.f;
    }
  } else for (int m = wid; m < M; m += NWV) {
    float gm = -INFINITY;
    for (int s = lane; s < ns; s += 64) gm = fmaxf(gm, p.pm[pb + (int64_t)s * M + m]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) gm = fmaxf(gm, __shfl_xor(gm, off, 64));
    float L = 0.f;
    for (int s = lane; s < ns; s += 64) {
      const float ms = p.pm[pb + (int64_t)s * M + m];
      const float w = ms == -INFINITY ? 0.f : __expf(ms - gm);
      wts[s * 16 + m] = w;
      L += w * p.pl[pb + (int64_t)s * M + m];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) L += __shfl_xor(L, off, 64);
    const float inv = L > 0.f ? 1.f / L : 0.f;
    for (int s = lane; s < ns; s += 64) wts[s * 16 + m] *= inv;
  }
  __syncthreads();
  // weighted sum of the partial rows
  float* part = wts + ns * 16;   // [H][M * D]
  if (regs) {
    if (tid < elems * H) {
      const int m = e0 / D;
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < PMAX; ++i)
        if (h0 + i * H < ns) acc += wts[(h0 + i * H) * 16 + m] * pv[i];
      part[h0 * elems + e0] = acc;
    }
  } else for (int it = tid; it < elems * H; it += 64 * NWV) {   // four independent loads in flight per thread
    const int e = it % elems, h = it / elems, m = e / D, d = e % D;
    const float* src = p.po + (pb + m) * D + d;
    float acc = 0.f;
    int sp = h;
    for (; sp + 3 * H < ns; sp += 4 * H) {
      const float a0 = src[sp * st], a1 = src[(sp + H) * st], a2 = src[(sp + 2 * H) * st], a3 = src[(sp + 3 * H) * st];
      acc += wts[sp * 16 + m] * a0 + wts[(sp + H) * 16 + m] * a1 + wts[(sp + 2 * H) * 16 + m] * a2 +
             wts[(sp + 3 * H) * 16 + m] * a3;
    }
    for (; sp < ns; sp += H) acc += wts[sp * 16 + m] * src[sp * st];
    part[h * elems + e] = acc;
  }
  __syncthreads();
  for (int e = tid; e < elems; e += 64 * NWV) of[e] = bf2f(f2bf(H == 2 ? part[e] + part[elems + e] : part[e]));
  __syncthreads();
  oproj_tail<D>(p, of, wreg, b, row0, rpp, tpr, seg, G);
}

// Pending prefetch of the next decode_attn2 launch (set by decode_attn_set_prefetch, consumed by
// one launch: graph capture records the kernel arguments by value, so every captured layer keeps
// its own ranges).
static const void* g_pf[2] = {nullptr, nullptr};
static int64_t g_pf_bytes[2] = {0, 0};
static int g_pf_wgs = 0;

}  // namespace dattn

// Opt-in phase trace of the following decode attention launches (eager or captured: the pointer is
// recorded by value); null turns it off.  trace must hold 2 x (launch grid) uint64.
void decode_attn_set_trace(uint64_t* trace) { dattn::g_trace = trace; }

void decode_attn_set_prefetch(const void* a, int64_t a_bytes, const void* b, int64_t b_bytes, int wgs) {
  dattn::g_pf[0] = a; dattn::g_pf_bytes[0] = a ? a_bytes : 0;
  dattn::g_pf[1] = b; dattn::g_pf_bytes[1] = b ? b_bytes : 0;
  dattn::g_pf_wgs = wgs;
}

// Returns -1 when the shape is not covered (caller falls back to the 128-key-chunk kernel).
int decode_attn2_launch(const void* q, const int64_t* qs, const void* kc, const void* vc, const int64_t* cs,
                        const int* cache_idx, const int* seq_len, float* po, float* pm, float* pl, void* out,
                        const int64_t* os, int B, int T, int Hq, int Hkv, int D, int Lmax, float scale, int* nsplit_out,
                        hipStream_t stream) {
  if (Hkv <= 0 || Hq % Hkv) return -1;
  const int M = (Hq / Hkv) * T;
  if (M > 16 || (D != 64 && D != 128)) return -1;
  dattn::Params p{};   // value-initialised: every field a launcher does not set is zero / null
  p.q = (const uint16_t*)q; p.q_sb = qs[0]; p.q_st = qs[1]; p.q_sh = qs[2];
  p.kc = (const uint16_t*)kc; p.vc = (const uint16_t*)vc;
  p.c_sb = cs[0]; p.c_sh = cs[1]; p.c_sl = cs[2];
  p.cache_idx = cache_idx; p.seq_len = seq_len;
  p.out = (uint16_t*)out; p.o_sb = os[0]; p.o_st = os[1]; p.o_sh = os[2];
  p.po = po; p.pm = pm; p.pl = pl;
  p.B = B; p.T = T; p.Hq = Hq; p.Hkv = Hkv;
  const int kps = dattn::keys_per_split(Lmax, B, Hkv);
  p.kps = kps;
  p.nsplit = (Lmax + kps - 1) / kps;
  p.scale_log2 = scale * 1.4426950408889634f;
  *nsplit_out = p.nsplit;
  // D = 64: 8 waves (<= 2 chunks each per 1024-key split); D = 128: 4 waves (LDS: V tiles + merge)
  const int nwv = D == 64 ? 8 : 4;
  const size_t lds = (size_t)nwv * dattn::KB * D * 2 + (size_t)nwv * 16 * D * 4 + (size_t)2 * nwv * 16 * 4;
  p.attn_wgs = B * Hkv * p.nsplit;
  p.trace = dattn::g_trace;
  int pf_wgs = 0;
  for (int r = 0; r < 2; ++r) {
    // 16-B aligned start, whole chunks only (a prefetch never needs the ragged tail)
    const bool ok = dattn::g_pf[r] && (reinterpret_cast<uintptr_t>(dattn::g_pf[r]) & 15) == 0 && dattn::g_pf_bytes[r] >= 16;
    p.pf[r] = ok ? static_cast<const u32x4_t*>(dattn::g_pf[r]) : nullptr;
    p.pf_n16[r] = ok ? dattn::g_pf_bytes[r] / 16 : 0;
    if (ok) pf_wgs = dattn::g_pf_wgs > 0 ? dattn::g_pf_wgs : 256;
  }
  dattn::g_pf[0] = dattn::g_pf[1] = nullptr;
  dattn::g_pf_bytes[0] = dattn::g_pf_bytes[1] = 0;
  const dim3 grid(p.attn_wgs + pf_wgs), block(64 * nwv);
  if (D == 64) {
    (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<64, 8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((dattn::attn_kernel<64, 8, false>), grid, block, lds, stream, p);
  } else {
    (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<128, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((dattn::attn_kernel<128, 4, false>), grid, block, lds, stream, p);
  }
  return (int)hipGetLastError();
}

namespace dattn {
int g_oproj_maxl = -1;   // NXD_DECODE_ATTN_OPROJ_MAXL, or decode_attn_set_oproj_maxl
int g_sync_on = -1;      // NXD_DECODE_ATTN_SYNC (default 0: measured slower), or decode_attn_set_sync
}
void decode_attn_set_sync(int v) { dattn::g_sync_on = v ? 1 : 0; }
void decode_attn_set_oproj_maxl(int v) { dattn::g_oproj_maxl = v; }

// Bounded-spin error word of the SYNC launches (a partial never arrived: that launch wrote NaN);
// reset clears it.  Synchronous (reads device memory).
int decode_attn_sync_error(bool reset) {
  int v = 0;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(dattn::g_sync_err), sizeof(int), 0, hipMemcpyDeviceToHost);
  if (reset && v) {
    const int z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(dattn::g_sync_err), &z, sizeof(int), 0, hipMemcpyHostToDevice);
  }
  return v;
}
int decode_attn_oproj_maxl() {
  if (dattn::g_oproj_maxl < 0) {
    const char* e = getenv("NXD_DECODE_ATTN_OPROJ_MAXL");
    dattn::g_oproj_maxl = e ? atoi(e) : 1024;
  }
  return dattn::g_oproj_maxl;
}

// Fused decode attention + o_proj (see FUSE above): oacc [B*T, Hout] fp32 must be zero on entry
// (the down projection's RESID epilogue re-zeroes it).  Returns -1 when the shape is not covered:
// cache capacity Lmax <= NXD_DECODE_ATTN_OPROJ_MAXL (default 1024: every workgroup of a kv head walks
// the whole cache; past that the split attention, whose keys per split fill the GPU, + merge + o_proj
// launches win -- 0.726 vs 0.774 ms/token at the notebook's 2,304-key cache,
// profiles/r6_decode/attn_split_ab.txt), M = G*T <= 16, D in {64, 128}, Wo blocks of <= 4 register
// passes.
int decode_attn_oproj_launch(const void* q, const int64_t* qs, const void* kc, const void* vc, const int64_t* cs,
                             const int* cache_idx, const int* seq_len, const void* wo, int64_t ldwo, int Hout, float* oacc,
                             float* po, float* pm, float* pl, float* mo, int B, int T, int Hq, int Hkv, int D, int Lmax,
                             float scale, hipStream_t stream) {
  if (Hkv <= 0 || Hq % Hkv) return -1;
  const int G = Hq / Hkv, M = G * T;
  const int maxl = decode_attn_oproj_maxl();
  // past maxl: split attention into the partials, then merge + o_proj (needs the partial buffers:
  // [B * Hkv * ceil(Lmax / 128) * M] rows of D, plus the two stats)
  const bool split = Lmax > maxl && po != nullptr && dattn::keys_per_split(Lmax, B, Hkv) < Lmax;
  if (M > 16 || (D != 64 && D != 128) || (Lmax > maxl && !split) || (G * D) % 32 || ldwo % 8) return -1;
  const int nwv = D == 64 ? 8 : 4;
  const int nt = 64 * nwv, tpr = (G * D) / 32;
  if (tpr > 64 || 64 % tpr || nt % tpr) return -1;
  const int rpp = nt / tpr;
  // row chunks per kv head: fill >= target workgroups (NXD_DECODE_OPROJ_WGS, default 256), at most 4
  // register passes per thread
  static const int target = [] {
    const char* e = getenv("NXD_DECODE_OPROJ_WGS");
    const int v = e ? atoi(e) : 256;
    return v > 0 ? v : 256;
  }();
  int R = 1;
  while ((int64_t)B * Hkv * R < target && Hout % (2 * R) == 0 && (Hout / (2 * R)) % rpp == 0) R *= 2;
  while (Hout % R == 0 && (Hout / R) % rpp == 0 && Hout / R / rpp > 4 && Hout % (2 * R) == 0 && (Hout / (2 * R)) % rpp == 0)
    R *= 2;
  if (Hout % R || (Hout / R) % rpp || Hout / R / rpp > 4 || Hout / R / rpp < 1) return -1;
  dattn::Params p{};
  p.q = (const uint16_t*)q; p.q_sb = qs[0]; p.q_st = qs[1]; p.q_sh = qs[2];
  p.kc = (const uint16_t*)kc; p.vc = (const uint16_t*)vc;
  p.c_sb = cs[0]; p.c_sh = cs[1]; p.c_sl = cs[2];
  p.cache_idx = cache_idx; p.seq_len = seq_len;
  p.B = B; p.T = T; p.Hq = Hq; p.Hkv = Hkv; p.nsplit = 1;
  p.scale_log2 = scale * 1.4426950408889634f;
  p.wo = (const uint16_t*)wo; p.ldwo = ldwo; p.oacc = oacc; p.Hout = Hout; p.R = R; p.NP = Hout / R / rpp;
  p.attn_wgs = B * Hkv * R;
  p.trace = dattn::g_trace;
  const dim3 grid(p.attn_wgs), block(nt);
  if (dattn::g_sync_on < 0) {
    const char* e = getenv("NXD_DECODE_ATTN_SYNC");
    dattn::g_sync_on = e ? (atoi(e) != 0) : 0;
  }
  const bool sync_on = dattn::g_sync_on != 0;
  static const int n_cu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  if (split && sync_on && mo != nullptr && B * Hkv <= dattn::kSyncHeads && (int)grid.x <= n_cu) {
    // one launch: workgroup r of a head computes key split r (>= 128 keys, the partial buffers hold
    // Lmax / 128 splits), then merges the head's splits and runs its o_proj slice (SYNC above)
    int kps = (Lmax + R - 1) / R;
    kps = (kps + dattn::KB - 1) / dattn::KB * dattn::KB;
    kps = kps < 128 ? 128 : kps;
    const int ns = (Lmax + kps - 1) / kps;
    const size_t lds = (size_t)nwv * dattn::KB * D * 2 + (size_t)nwv * 16 * D * 4 + (size_t)2 * nwv * 16 * 4;
    if (ns <= R && (size_t)16 * D * 4 + (size_t)ns * 16 * 4 <= (size_t)nwv * dattn::KB * D * 2) {
      static unsigned* cnt = [] { void* a = nullptr; (void)hipGetSymbolAddress(&a, HIP_SYMBOL(dattn::g_sync_cnt)); return (unsigned*)a; }();
      static int* err = [] { void* a = nullptr; (void)hipGetSymbolAddress(&a, HIP_SYMBOL(dattn::g_sync_err)); return (int*)a; }();
      p.kps = kps; p.nsplit = ns; p.po = po; p.pm = pm; p.pl = pl; p.sync_cnt = cnt; p.sync_err = err;
      p.mo = mo;
      if (D == 64) {
        (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<64, 8, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((dattn::attn_kernel<64, 8, true, true, true>), grid, block, lds, stream, p);
      } else {
        (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<128, 4, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((dattn::attn_kernel<128, 4, true, true, true>), grid, block, lds, stream, p);
      }
      return (int)hipGetLastError();
    }
  }
  if (split) {
    const int kps = dattn::keys_per_split(Lmax, B, Hkv), ns = (Lmax + kps - 1) / kps;
    const size_t mlds = (size_t)16 * D * 4 + (size_t)ns * 16 * 4 + (size_t)2 * 16 * D * 4;
    if (mlds > 64 * 1024) return -1;
    int ns2 = 0;
    const int64_t no_out[3] = {0, 0, 0};
    const int rc = decode_attn2_launch(q, qs, kc, vc, cs, cache_idx, seq_len, po, pm, pl, nullptr, no_out, B, T, Hq, Hkv,
                                       D, Lmax, scale, &ns2, stream);
    if (rc != 0) return rc;
    if (ns2 != ns) return 3;   // the attention launch split differently: never write the output through null
    p.nsplit = ns; p.po = po; p.pm = pm; p.pl = pl;
    if (D == 64) {
      (void)hipFuncSetAttribute((const void*)dattn::merge_oproj_kernel<64, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlds);
      hipLaunchKernelGGL((dattn::merge_oproj_kernel<64, 8>), grid, block, mlds, stream, p);
    } else {
      (void)hipFuncSetAttribute((const void*)dattn::merge_oproj_kernel<128, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlds);
      hipLaunchKernelGGL((dattn::merge_oproj_kernel<128, 4>), grid, block, mlds, stream, p);
    }
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)nwv * dattn::KB * D * 2 + (size_t)nwv * 16 * D * 4 + (size_t)2 * nwv * 16 * 4;
  static const bool wo_late = [] {
    const char* e = getenv("NXD_DECODE_WO_LATE");
    return e ? atoi(e) != 0 : true;
  }();
  if (D == 64) {
    if (wo_late) {
      (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<64, 8, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((dattn::attn_kernel<64, 8, true, true>), grid, block, lds, stream, p);
    } else {
      (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<64, 8, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((dattn::attn_kernel<64, 8, true, false>), grid, block, lds, stream, p);
    }
  } else {
    if (wo_late) {
      (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<128, 4, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((dattn::attn_kernel<128, 4, true, true>), grid, block, lds, stream, p);
    } else {
      (void)hipFuncSetAttribute((const void*)dattn::attn_kernel<128, 4, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((dattn::attn_kernel<128, 4, true, false>), grid, block, lds, stream, p);
    }
  }
  return (int)hipGetLastError();
}

}  // namespace nxd
