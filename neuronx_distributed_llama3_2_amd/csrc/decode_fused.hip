// Fused decode-step GEMVs (token generation, M <= 8 rows): each projection of a Llama layer is ONE
// launch that also does the element-wise work around it, so a decode layer is 5 kernels instead of
// 10 (reference: examples/inference/modules/attention/attention_base.py:141-170 and
// model_base.py:388-422 run RMSNorm, QKV, RoPE, the KV-cache scatter, o_proj, the residual adds,
// the MLP as separate graph ops):
//
//   QKV   : RMSNorm(h) prologue -> x.Wqkv^T -> RoPE on q/k (rotate-half pairs d, d + D/2 are the two
//           rows of one wave) -> q to the output buffer, k/v straight into the KV cache at pos[m]
//   O     : a.Wo^T with the residual add as epilogue: h[m, n] = h + bf16(acc) (in place)
//   GATEUP: RMSNorm(h) prologue -> silu(x.Wg^T) * (x.Wu^T)   (fused gate/up weight [2N, K])
//   DOWN  : a.Wd^T + residual add (in place), like O
//   plain : x.W^T, optional RMSNorm prologue (final norm + lm_head)
//
// Decode is weight-streaming bound (every weight byte read once per token): one wave owns NW
// weight rows and issues all of its row segments' 16-byte loads before the FMAs (4 k-steps of 512
// elements per round), so a CU keeps ~48 KB of weight loads in flight.  The normalised activation
// rows are built once per workgroup in LDS (the block recomputes sum(h^2) from L2: K <= 16 K
// elements, negligible next to the weights) and read back by every wave with ds_read_b128.
#include "common.h"

#include <cstdlib>

namespace nxd {
namespace dfused {

enum Epi { PLAIN = 0, RESID = 1, GLU = 2, ROPE_KV = 3 };

struct Params {
  const uint16_t* x;      // [M, K] activations (row stride ldx)
  int64_t ldx;
  const uint16_t* norm_w; // [K] RMSNorm weight (NORM variants)
  float eps;
  const uint16_t* w;      // [Nw, K] weights (row stride ldw)
  int64_t ldw;
  uint16_t* y;            // [M, N] output (RESID: residual stream updated in place)
  int64_t ldy;
  int M, N, K;            // N = output columns (GLU: up rows start at N)
  // ROPE_KV: y rows hold [nq | nkv | nkv] heads of D; k/v also go to the cache
  int nq, nkv, D;
  const float* cos_t;     // [max_pos, D/2]
  const float* sin_t;
  const int64_t* pos;     // [M] absolute position of each row
  int T;                  // rows per sequence (cache row = cache_idx[m / T])
  uint16_t* kc;
  uint16_t* vc;
  int64_t c_sb, c_sh, c_sl;
  const int* cache_idx;   // [M / T] (nullable: identity)
  int Lmax;
  int max_pos;            // rows of the cos/sin tables (positions are clamped into them)
  // pending residual contribution (fp32 [M, K] / [M, N], e.g. o_proj summed by the fused attention
  // kernel's atomics): NORM prologue sees x = bf16(x + bf16(xadd)); RESID epilogue first folds
  // yadd into y exactly as the o_proj RESID epilogue would have (y = bf16(y + bf16(yadd))), then
  // adds its own product, and zeroes yadd for the next layer.  Both nullable.
  const float* xadd;
  float* yadd;
  int pf;                 // issue the epilogue's / prologue's own global reads (residual row, yadd,
                          // position + cos/sin, RMSNorm weight) at kernel start, next to the first
                          // weight round, instead of as dependent round trips after the GEMV
  // XI kernels (first layer's QKV): x is the embedding table [xrows, K] and row m of the input is
  // x[xidx[m]] (the embedding gather folded into the prologue); workgroup 0 also stores the gathered
  // rows to xcopy [M, K] (the residual stream).  Reference: the separate embed_tokens op ahead of the
  // first layer (examples/inference/modules/model_base.py:473)
  const int64_t* xidx;
  int64_t xrows;
  uint16_t* xcopy;
  // PLAIN only: fp32 output [M, N] (row stride ldy) instead of bf16 y -- a row-parallel projection's
  // partial sum kept unrounded for the tensor-parallel all-reduce (decode at TP > 1)
  float* yf;
  int dot2;               // inner product on v_dot2c_f32_bf16 (NXD_DECODE_DOT2, default 1)
  int split;              // dmm_kernel: workgroups per weight tile along K (partials summed in g_sk)
};

constexpr int U = 4;   // 512-element k-steps per load round

// Workgroup = 4 waves = (4 / KS) row groups x KS k-slices: a row group's NW weight rows are split
// over KS waves (partials reduced through LDS), so a short-N / long-K projection (o_proj, down)
// still has thousands of waves streaming.  The first round of weight loads is issued before the
// RMSNorm prologue: the weights do not depend on the activations.
template <int MM, int NW, int EPI, bool NORM, int KS, bool XI = false>
__device__ __forceinline__ void dgemv_body(const Params& p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem);   // NORM: [MM][K] normalised bf16 rows
  __shared__ float red[4][MM];
  __shared__ float part[4][MM][NW];
  // wid is wave-uniform: readfirstlane puts it (and the rows, row pointers and k range derived
  // from it) in SGPRs, so each weight load is one scalar base + the lane's 16-byte offset + an
  // immediate, not a 64-bit per-lane address (the VGPR count sets how many waves stream at once)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rg = wid / KS, ks = wid % KS;
  const int wave = blockIdx.x * (4 / KS) + rg;          // row-group index

  // ---- this row group's weight rows (clamped; inactive groups compute but never store)
  int rows[NW];
  bool active = true;
  if (EPI == GLU) {   // NW / 2 (gate, up) row pairs per wave
    active = wave * (NW / 2) < p.N;
#pragma unroll
    for (int i = 0; i < NW / 2; ++i) {
      rows[2 * i] = min(wave * (NW / 2) + i, p.N - 1);
      rows[2 * i + 1] = rows[2 * i] + p.N;
    }
  } else if (EPI == ROPE_KV) {
    const int half = p.D / 2;
    const int npair = (p.nq + p.nkv) * half;   // rotary (d, d + D/2) row pairs of the q and k heads
    const int nv = p.nkv * p.D;                // v rows, two per wave
    if (wave < npair) {
      const int h = wave / half, d = wave % half;
      rows[0] = h * p.D + d;
      rows[1] = rows[0] + half;
    } else {
      const int r = (p.nq + p.nkv) * p.D + 2 * (wave - npair);
      active = (wave - npair) * 2 < nv;
      rows[0] = min(r, p.N - 1);
      rows[1] = min(r + 1, p.N - 1);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NW; ++i) rows[i] = min(wave * NW + i, p.N - 1);
    active = wave * NW < p.N;
  }

  const int kc = ((p.K + KS - 1) / KS + 7) & ~7;
  const int kbeg = min(ks * kc, p.K), kend = min(p.K, kbeg + kc);
  const uint16_t* wrow[NW];
#pragma unroll
  for (int r = 0; r < NW; ++r) wrow[r] = p.w + (int64_t)rows[r] * p.ldw;
  u32x4_t wv[NW][U];
  // Weight rows are loaded non-temporal (global_load ... nt): decode reads every weight byte once per
  // token (MI355X_MICROARCH.md, nt-weights; Llama-3.2-1B bs=1 0.732 -> 0.712 ms/token,
  // profiles/r4_decode_nt_fn_ab.txt).  Unpredicated: a lane past kend re-reads the slice's last 16 bytes (in
  // bounds) and the FMA loop skips it.  Predicated / zero-filled loads or a runtime choice of load
  // kind made the compiler merge register copies right after the loads, i.e. wait (s_waitcnt
  // vmcnt) for most of them before the prologue could start, and cost 4-8 VGPRs.
  auto load_round = [&](int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(base + u * 512 + lane * 8, kend - 8);
#pragma unroll
      for (int r = 0; r < NW; ++r)
        wv[r][u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wrow[r] + k));
    }
  };

  // ---- bs = 1: the RMSNorm prologue's first chunk of x (+ pending xadd, + norm weight) is issued
  // BEFORE the weight round.  vmcnt retires in issue order, so a load issued after the weights can
  // only be waited for together with all of them: the prologue then started only once the weights
  // had landed, and its own L2 round trip and barriers were added to every wave's critical path.
  // (Left uninitialised where not loaded; only read under the same conditions.)
  // (Rows of bs <= 2 too: at 2 rows the prologue behind the weights cost gate_up / qkv 2-4 us each.)
  constexpr bool PRE = NORM && MM <= 2;
  u32x4_t x0[MM], gw0 = {0, 0, 0, 0};
  f32x4_t xa0[MM], xa1[MM];
  const bool pre_ok = PRE && tid * 8 < p.K;
  // XI: input row m is an embedding-table row picked by a token id (a scalar load).  Its gather is
  // still issued ahead of the weights: waiting for the id delays the weight round by one scalar
  // round trip, while a gather issued after the weights made the prologue wait for all of them
  // (layer-0 QKV 5.89-6.04 vs 5.43-5.45 us for the other layers' launches)
  // An id outside [0, xrows) reads an in-bounds row (clamped address) whose value is then replaced by
  // zeros at its use (xok), as ops.vocab_parallel_embedding returns a zero row for such ids (pad -1,
  // another TP rank's vocabulary slice); masking at the use keeps the load ahead of the weights.
  auto xrow = [&](int m) -> const uint16_t* {
    if constexpr (XI) {
      const int64_t t = p.xidx[m];
      return p.x + (t < 0 ? 0 : (t >= p.xrows ? p.xrows - 1 : t)) * p.ldx;
    } else {
      return p.x + (int64_t)m * p.ldx;
    }
  };
  auto xok = [&](int m) -> bool {
    if constexpr (XI) {
      const int64_t t = p.xidx[m];
      return t >= 0 && t < p.xrows;
    } else {
      return true;
    }
  };
  if (pre_ok) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {   // rows past M re-read the last row (never used)
      const int mm = min(m, p.M - 1);
      x0[m] = *reinterpret_cast<const u32x4_t*>(xrow(mm) + tid * 8);
      if (p.xadd) {
        xa0[m] = *reinterpret_cast<const f32x4_t*>(p.xadd + (int64_t)mm * p.K + tid * 8);
        xa1[m] = *reinterpret_cast<const f32x4_t*>(p.xadd + (int64_t)mm * p.K + tid * 8 + 4);
      }
    }
    gw0 = *reinterpret_cast<const u32x4_t*>(p.norm_w + tid * 8);
  }
  // bs = 1 without a norm prologue (down, o_proj): the first round's activation chunks, likewise
  // ahead of the weights (they were read inside the FMA loop, one L2 round trip after the weights)
  constexpr bool PREX = !NORM && MM == 1;
  u32x4_t xv0[PREX ? U : 1];
  if constexpr (PREX) {
#pragma unroll
    for (int u = 0; u < U; ++u) xv0[u] = *reinterpret_cast<const u32x4_t*>(p.x + min(kbeg + u * 512 + lane * 8, kend - 8));
  }
  // RESID epilogue operands (p.pf), likewise ahead of the weights and kept raw: converting the bf16
  // right after its load made the wave wait (vmcnt) there for every weight load issued before it
  uint16_t y_raw[MM][NW];
  float ya_pre[MM][NW];
  if (EPI == RESID && p.pf && lane == 0 && active) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (m >= p.M) continue;
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        const int n = min(wave * NW + r, p.N - 1);
        y_raw[m][r] = p.y[(int64_t)m * p.ldy + n];
        if (p.yadd) ya_pre[m][r] = p.yadd[(int64_t)m * p.N + n];
      }
    }
  }
  load_round(kbeg);

  // ---- early epilogue / prologue operands (p.pf): independent of the activations, so their
  // latency overlaps the first weight round instead of following the reduction
  if (!PRE && NORM && p.pf && tid * 8 < p.K) gw0 = *reinterpret_cast<const u32x4_t*>(p.norm_w + tid * 8);
  float cs_pre[MM], sn_pre[MM];
  if (EPI == ROPE_KV && p.pf && lane == 0 && active) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (m >= p.M) continue;
      const int half = p.D / 2;
      if (rows[0] < (p.nq + p.nkv) * p.D && rows[1] == rows[0] + half) {
        const int64_t ps = p.pos[m];
        const int64_t pt = ps < 0 ? 0 : (ps >= p.max_pos ? p.max_pos - 1 : ps);
        const int d = rows[0] % p.D;
        cs_pre[m] = p.cos_t[pt * half + d];
        sn_pre[m] = p.sin_t[pt * half + d];
      }
    }
  }

  if (NORM) {
    float ss[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) ss[m] = 0.f;
    for (int k = tid * 8; k < p.K; k += 256 * 8) {
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        if (m < p.M) {
          u32x4_t v;
          f32x4_t a0, a1;
          if (PRE && k == tid * 8) {   // the chunk loaded ahead of the weights
            v = x0[m];
            if (p.xadd) { a0 = xa0[m]; a1 = xa1[m]; }
          } else {
            v = *reinterpret_cast<const u32x4_t*>(xrow(m) + k);
            if (p.xadd) {
              a0 = *reinterpret_cast<const f32x4_t*>(p.xadd + (int64_t)m * p.K + k);
              a1 = *reinterpret_cast<const f32x4_t*>(p.xadd + (int64_t)m * p.K + k + 4);
            }
          }
          if (XI && !xok(m)) v = u32x4_t{0u, 0u, 0u, 0u};
          float f[8];
          unpack8(v, f);
          if (p.xadd) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = bf2f(f2bf(f[j] + bf2f(f2bf(j < 4 ? a0[j] : a1[j - 4]))));
            v = pack8(f);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[m] += f[j] * f[j];
          *reinterpret_cast<u32x4_t*>(xs + m * p.K + k) = v;
          if (XI && blockIdx.x == 0 && p.xcopy) *reinterpret_cast<u32x4_t*>(p.xcopy + (int64_t)m * p.K + k) = v;
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      const float sm = wave_sum(ss[m]);
      if (lane == 0) red[wid][m] = sm;
    }
    __syncthreads();
    float rstd[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) rstd[m] = rsqrtf((red[0][m] + red[1][m] + red[2][m] + red[3][m]) / (float)p.K + p.eps);
    for (int k = tid * 8; k < p.K; k += 256 * 8) {
      float g[8];
      unpack8((PRE || p.pf) && k == tid * 8 ? gw0 : *reinterpret_cast<const u32x4_t*>(p.norm_w + k), g);
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        if (m < p.M) {
          float f[8];
          unpack8(*reinterpret_cast<const u32x4_t*>(xs + m * p.K + k), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] * rstd[m] * g[j];
          *reinterpret_cast<u32x4_t*>(xs + m * p.K + k) = pack8(f);
        }
      }
    }
    __syncthreads();
  }

  float acc[MM][NW];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int r = 0; r < NW; ++r) acc[m][r] = 0.f;

  // inner product: v_dot2c_f32_bf16 on the packed bf16 operands (p.dot2, default), or both operands
  // widened to f32 and multiplied with FMAs (NXD_DECODE_DOT2=0).  The widening costs one VALU op per
  // element per activation row: at 8 rows the GEMVs were VALU-bound, 3-4x the single-row time
  // (gate_up 43.9 vs 12.5 us, profiles/r5k_decode_bs8_kernel_stats_fma.csv)
  auto fma_round = [&](int base, bool first) {
    const bool full = base + 512 * U <= kend;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + lane * 8 + u * 512;
      if (full || k < kend) {
#pragma unroll
        for (int m = 0; m < MM; ++m) {
          if (m < p.M) {
            const u32x4_t xv = (PREX && first) ? xv0[PREX ? u : 0]
                                               : *reinterpret_cast<const u32x4_t*>(NORM ? (xs + m * p.K + k) : (p.x + (int64_t)m * p.ldx + k));
            if (p.dot2) {
#pragma unroll
              for (int r = 0; r < NW; ++r) acc[m][r] = dot8_bf16(xv, wv[r][u], acc[m][r]);
            } else {
              float xf[8];
              unpack8(xv, xf);
#pragma unroll
              for (int r = 0; r < NW; ++r) {
                float wf[8];
                unpack8(wv[r][u], wf);
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[m][r] += xf[e] * wf[e];
              }
            }
          }
        }
      }
    }
  };
  if (kbeg < kend) fma_round(kbeg, true);
  for (int base = kbeg + 512 * U; base < kend; base += 512 * U) {
    load_round(base);
    fma_round(base, false);
  }
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int r = 0; r < NW; ++r) acc[m][r] = wave_sum(acc[m][r]);
  if (KS > 1) {
    if (lane == 0) {
#pragma unroll
      for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int r = 0; r < NW; ++r) part[wid][m][r] = acc[m][r];
    }
    __syncthreads();
    if (ks != 0) return;
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < KS; ++j) t += part[wid + j][m][r];
        acc[m][r] = t;
      }
  }
  if (lane != 0 || !active) return;

#pragma unroll
  for (int m = 0; m < MM; ++m) {
    if (m >= p.M) continue;
    uint16_t* yr = p.y + (int64_t)m * p.ldy;
    if (EPI == GLU) {
#pragma unroll
      for (int i = 0; i < NW / 2; ++i) {
        if (wave * (NW / 2) + i >= p.N) continue;
        const float g = acc[m][2 * i], u = acc[m][2 * i + 1];
        yr[rows[2 * i]] = f2bf(g / (1.f + __expf(-g)) * u);
      }
    } else if (EPI == ROPE_KV) {
      const int half = p.D / 2;
      const int64_t ps = p.pos[m];
      const int b = m / p.T;
      const int cb = p.cache_idx ? p.cache_idx[b] : b;
      const bool in_cache = ps >= 0 && ps < p.Lmax;
      const int qk_rows = (p.nq + p.nkv) * p.D;
      if (rows[0] < qk_rows && rows[1] == rows[0] + half) {
        const int h = rows[0] / p.D, d = rows[0] % p.D;
        const int64_t pt = ps < 0 ? 0 : (ps >= p.max_pos ? p.max_pos - 1 : ps);
        const float c = p.pf ? cs_pre[m] : p.cos_t[pt * half + d];
        const float sn = p.pf ? sn_pre[m] : p.sin_t[pt * half + d];
        const float x1 = bf2f(f2bf(acc[m][0])), x2 = bf2f(f2bf(acc[m][1]));   // bf16 projection output
        const uint16_t o1 = f2bf(x1 * c - x2 * sn), o2 = f2bf(x2 * c + x1 * sn);
        yr[rows[0]] = o1;
        yr[rows[1]] = o2;
        if (h >= p.nq && in_cache) {
          uint16_t* kp = p.kc + (int64_t)cb * p.c_sb + (int64_t)(h - p.nq) * p.c_sh + ps * p.c_sl;
          kp[d] = o1;
          kp[d + half] = o2;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          if (r == 1 && rows[1] == rows[0]) break;
          const uint16_t o = f2bf(acc[m][r]);
          yr[rows[r]] = o;
          const int vr = rows[r] - qk_rows;
          if (in_cache)
            p.vc[(int64_t)cb * p.c_sb + (int64_t)(vr / p.D) * p.c_sh + ps * p.c_sl + vr % p.D] = o;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        const int n = wave * NW + r;
        if (n >= p.N) continue;
        if (EPI == RESID) {
          float yv = p.pf ? bf2f(y_raw[m][r]) : bf2f(yr[n]);
          if (p.yadd) {
            float* ya = p.yadd + (int64_t)m * p.N + n;
            yv = bf2f(f2bf(yv + bf2f(f2bf(p.pf ? ya_pre[m][r] : *ya))));
            *ya = 0.f;
          }
          yr[n] = f2bf(yv + bf2f(f2bf(acc[m][r])));
        }
        else if (EPI == PLAIN && p.yf) p.yf[(int64_t)m * p.ldy + n] = acc[m][r];
        else yr[n] = f2bf(acc[m][r]);
      }
    }
  }
}

template <int MM, int NW, int EPI, bool NORM, int KS, bool XI = false>
__global__ void __launch_bounds__(256) dgemv_kernel(Params p) {
  dgemv_body<MM, NW, EPI, NORM, KS, XI>(p);
}

// The same body at a forced occupancy (WPE waves / SIMD: 7 -> <= 72 VGPRs, 8 -> <= 64).  The bs = 1
// two-row kernels take 74-76 VGPRs (6 waves / SIMD = 1,536 resident workgroups), so gate_up's
// 2,048 workgroups run as a full round plus a partial one, each paying the HBM latency.  Forcing 8
// spills 64-76 bytes / lane and measured 1.17 vs 0.69 ms/token; 7 spills 16-20 (NXD_DECODE_OCC).
template <int MM, int NW, int EPI, bool NORM, int KS, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) dgemv_kernel_occ(Params p) {
  dgemv_body<MM, NW, EPI, NORM, KS>(p);
}


// ---------------------------------------------------------------------------------------------
// M = 2..8 activation rows on v_mfma_f32_16x16x32_bf16.  With the VALU inner product every 16-B
// weight chunk is multiplied by M activation chunks that each wave re-reads (LDS or L2) and the
// FMAs scale with M: at 8 rows the GEMVs ran 3-4x their single-row time (gate_up 35.7 vs 12.4 us
// with dot2, profiles/r5k_decode_bs8_kernel_stats_*).  Here a wave owns a tile of 16 weight rows
// = the 16 columns of the MFMA B operand (lane l loads 16 B of row (l & 15) at k 8 (l >> 4), the
// same 16-B nontemporal loads as the VALU body), the activations are the A operand (rows >= M
// zero), and one MFMA consumes 1 KiB of weights: the arithmetic no longer grows with M.
// Tiles: PLAIN / RESID 16 consecutive rows; GLU 8 gate rows (columns 0-7) + their 8 up rows
// (8-15); ROPE_KV 8 rotary pairs of one q / k head (d0..d0+7 | the same + D/2) or 16 v rows --
// the pair partner is 8 lanes away (one xor-8 shuffle in the epilogue).  KS waves split K and
// reduce through LDS; NWV waves per workgroup (4, or 8 when KS = 8).
// C layout of the 16x16 MFMA: lane l holds rows m = 4 (l >> 4) + i (i < 4) of column l & 15, so
// lanes 0-31 carry the <= 8 real rows.
constexpr int kSkTiles = 1024;   // weight tiles a split launch may have
constexpr int kMaxSplit = 8;     // workgroups per tile
__device__ float g_sk[kSkTiles * kMaxSplit * 128];   // per-part partial slots (overwritten every launch)
__device__ int g_skc[kSkTiles];                      // arrival tickets: zero-initialised, left zero

template <int EPI, bool NORM, int KS, int NWV, bool XI = false>
__global__ void __launch_bounds__(64 * NWV, 4) dmm_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem);   // NORM: [M][K] normalised bf16 rows
  __shared__ float red[NWV][8];
  __shared__ f32x4_t part[KS > 1 ? NWV : 1][32];
  constexpr int G = NWV / KS;
  constexpr int U = 4;                                 // 32-deep k-steps per load round (two rounds in flight)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rg = wid / KS, ks = wid % KS;
  const int spi = (int)blockIdx.x % p.split;            // this workgroup's K part of its tiles
  const int tile = ((int)blockIdx.x / p.split) * G + rg;
  const int c = lane & 15;

  // ---- this lane's weight row (B column c) and the tile's output mapping
  int row = 0;
  bool active = true;   // tile-uniform
  const int half = p.D / 2;
  const int qk_tiles = EPI == ROPE_KV ? (p.nq + p.nkv) * (half / 8) : 0;
  if (EPI == GLU) {
    active = tile * 8 < p.N;
    const int g = min(tile * 8 + (c & 7), p.N - 1);
    row = c < 8 ? g : g + p.N;
  } else if (EPI == ROPE_KV) {
    if (tile < qk_tiles) {
      const int h = tile / (half / 8), d0 = (tile % (half / 8)) * 8;
      row = h * p.D + d0 + (c & 7) + (c < 8 ? 0 : half);
    } else {
      const int v0 = (p.nq + p.nkv) * p.D + (tile - qk_tiles) * 16;
      active = (tile - qk_tiles) * 16 < p.nkv * p.D;
      row = min(v0 + c, p.N - 1);
    }
  } else {
    active = tile * 16 < p.N;
    row = min(tile * 16 + c, p.N - 1);
  }
  const uint16_t* wrow = p.w + (int64_t)row * p.ldw;

  // ---- k range of this slice (32-aligned); the first weight round goes out before the prologue
  const int nparts = p.split * KS;
  const int kc = ((p.K + nparts - 1) / nparts + 31) & ~31;
  const int kbeg = min((spi * KS + ks) * kc, p.K), kend = min(p.K, kbeg + kc);
  const int kq = 8 * (lane >> 4);                      // this lane's k offset inside a 32-step
  u32x4_t wv[U], wn[U];   // double-buffered weight rounds: round r + 1 is in flight while r is consumed
  auto load_into = [&](u32x4_t (&dst)[U], int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(base + 32 * u + kq, kend - 8);
      dst[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wrow + k));
    }
  };
  auto load_round = [&](int base) { load_into(wv, base); };
  auto xrow = [&](int m) -> const uint16_t* {
    if constexpr (XI) {
      const int64_t t = p.xidx[m];
      return p.x + (t < 0 ? 0 : (t >= p.xrows ? p.xrows - 1 : t)) * p.ldx;
    } else {
      return p.x + (int64_t)m * p.ldx;
    }
  };
  auto xok = [&](int m) -> bool {
    if constexpr (XI) {
      const int64_t t = p.xidx[m];
      return t >= 0 && t < p.xrows;
    } else {
      return true;
    }
  };
  // RMSNorm rows of one chunk per thread (K <= 8 x threads): loaded BEFORE the weight round.  vmcnt
  // retires in issue order, so prologue loads issued after the weights wait for all of them and
  // the normalisation only starts once the weights have landed (the VALU body's MM = 1 PRE path)
  constexpr int NTH = 64 * NWV;
  const bool pre = NORM && p.K <= NTH * 8;
  u32x4_t xpre[8];
  if (NORM && pre) {
    const int k = min(tid * 8, p.K - 8);
#pragma unroll
    for (int m = 0; m < 8; ++m) xpre[m] = *reinterpret_cast<const u32x4_t*>(xrow(min(m, p.M - 1)) + k);
  }
  if (kbeg < kend) load_round(kbeg);
  if (kbeg + 32 * U < kend) load_into(wn, kbeg + 32 * U);
  // epilogue operands (residual row + pending fp32 sum; rotary position + cos / sin) issued now,
  // so they land behind the first weight round instead of as round trips after the reduction
  const int m0 = 4 * (lane >> 4);
  uint16_t y_pre[4];
  float ya_pre[4], cs_pre[4], sn_pre[4];
  if (EPI == RESID && active && lane < 32 && ks == 0) {
    const int n = min(tile * 16 + c, p.N - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(m0 + i, p.M - 1);
      y_pre[i] = p.y[(int64_t)m * p.ldy + n];
      ya_pre[i] = p.yadd ? p.yadd[(int64_t)m * p.N + n] : 0.f;
    }
  }
  if (EPI == ROPE_KV && active && lane < 32 && ks == 0 && tile < qk_tiles) {
    const int d = (row % p.D) % half;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t ps = p.pos[min(m0 + i, p.M - 1)];
      const int64_t pt = ps < 0 ? 0 : (ps >= p.max_pos ? p.max_pos - 1 : ps);
      cs_pre[i] = p.cos_t[pt * half + d];
      sn_pre[i] = p.sin_t[pt * half + d];
    }
  }

  // ---- RMSNorm prologue (as the VALU body): rows -> LDS, x += bf16(xadd), normalised in place
  if constexpr (NORM) {
    constexpr int NT = 64 * NWV;
    float ss[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) ss[m] = 0.f;
    for (int k = tid * 8; k < p.K; k += NT * 8) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if (m < p.M) {
          u32x4_t v = pre ? xpre[m] : *reinterpret_cast<const u32x4_t*>(xrow(m) + k);
          if (XI && !xok(m)) v = u32x4_t{0u, 0u, 0u, 0u};
          float f[8];
          unpack8(v, f);
          if (p.xadd) {
            const f32x4_t a0 = *reinterpret_cast<const f32x4_t*>(p.xadd + (int64_t)m * p.K + k);
            const f32x4_t a1 = *reinterpret_cast<const f32x4_t*>(p.xadd + (int64_t)m * p.K + k + 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = bf2f(f2bf(f[j] + bf2f(f2bf(j < 4 ? a0[j] : a1[j - 4]))));
            v = pack8(f);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[m] += f[j] * f[j];
          *reinterpret_cast<u32x4_t*>(xs + m * p.K + k) = v;
          if (XI && blockIdx.x == 0 && p.xcopy) *reinterpret_cast<u32x4_t*>(p.xcopy + (int64_t)m * p.K + k) = v;
        }
      }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float sm = wave_sum(ss[m]);
      if (lane == 0) red[wid][m] = sm;
    }
    __syncthreads();
    float rstd[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t += red[w][m];
      rstd[m] = rsqrtf(t / (float)p.K + p.eps);
    }
    for (int k = tid * 8; k < p.K; k += NT * 8) {
      float g[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(p.norm_w + k), g);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if (m < p.M) {
          float f[8];
          unpack8(*reinterpret_cast<const u32x4_t*>(xs + m * p.K + k), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] * rstd[m] * g[j];
          *reinterpret_cast<u32x4_t*>(xs + m * p.K + k) = pack8(f);
        }
      }
    }
    __syncthreads();
  }

  // ---- main loop: A = activation rows (lane row c < M, k 8 (l >> 4)), B = the weight tile
  const bool arow = c < p.M;
  // activation rows >= M and k >= kend read an in-bounds chunk that is replaced by zeros (an
  // unpredicated load; a predicated one made hipcc spill the whole round)
  const uint16_t* xr = NORM ? xs + min(c, p.M - 1) * p.K : p.x + (int64_t)min(c, p.M - 1) * p.ldx;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  // two weight rounds in flight: rounds 0 and 1 went out before the prologue; after the MFMAs of
  // round r its buffer takes round r + 2.  The activation chunks of round r + 1 are issued before
  // the weights of round r + 2 (vmcnt retires in order: waiting for them never waits for weights)
  auto load_x = [&](u32x4_t (&xa)[U], int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + 32 * u + kq;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(xr + min(k, kend - 8));
      xa[u] = (arow && k < kend) ? v : u32x4_t{0u, 0u, 0u, 0u};
    }
  };
  auto mfma_round = [&](const u32x4_t (&w)[U], const u32x4_t (&xa)[U], int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + 32 * u < kend)   // wave-uniform
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, xa[u]), __builtin_bit_cast(bf16x8_t, w[u]), acc, 0, 0, 0);
    }
  };
  constexpr int RK = 32 * U;   // k per round
  u32x4_t xc[U], xn[U];
  if (kbeg < kend) load_x(xc, kbeg);
#pragma unroll 1
  for (int base = kbeg; base < kend; base += 2 * RK) {
    mfma_round(wv, xc, base);
    if (base + RK < kend) load_x(xn, base + RK);
    if (base + 2 * RK < kend) load_into(wv, base + 2 * RK);
    if (base + RK < kend) {
      mfma_round(wn, xn, base + RK);
      if (base + 2 * RK < kend) load_x(xc, base + 2 * RK);
      if (base + 3 * RK < kend) load_into(wn, base + 3 * RK);
    }
  }

  // ---- k-slice reduction (lanes 0-31 hold the real rows)
  if constexpr (KS > 1) {
    if (lane < 32) part[wid][lane] = acc;
    __syncthreads();
    if (ks != 0) return;
#pragma unroll
    for (int j = 1; j < KS; ++j) {
      const f32x4_t o = part[wid + j][lane & 31];
      acc += o;
    }
  }
  if (!active) return;

  // ---- split-K across workgroups: every part stores its 16 x 8 partial into its own slot with
  // write-through (sc1) stores, drains them (vmcnt) and takes a ticket (relaxed agent atomic); the
  // last part reads the slots back with sc1 loads, sums them in part order (the same bits whichever
  // part arrives last), resets the ticket for the next launch and runs the epilogue.  No fences:
  // a release fence writes back the whole L2 (buffer_wbl2) and cost the step 0.7 ms at batch 8;
  // no workgroup waits on another (cdna_hip_programming.md Guideline 16, recipe R1).
  if (p.split > 1) {
    float* sk = g_sk + (int64_t)tile * (kMaxSplit * 128);   // [part][4][32 lanes]
    if (lane < 32) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __hip_atomic_store(sk + spi * 128 + 32 * i + lane, acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(g_skc + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __shfl(t, 0, 64);
    if (t != p.split - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below the ticket
    if (lane < 32) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
        for (int j = 0; j < p.split; ++j)
          v += __hip_atomic_load(sk + j * 128 + 32 * i + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc[i] = v;
      }
    }
    if (lane == 0) __hip_atomic_store(g_skc + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- epilogue: lane (c, rows 4 (lane >> 4) + i)
  if (EPI == GLU) {
    f32x4_t up;
#pragma unroll
    for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(acc[i], 8, 64);
    const int n = tile * 8 + c;
    if (lane >= 32 || c >= 8 || n >= p.N) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + i;
      if (m < p.M) {
        const float g = acc[i];
        p.y[(int64_t)m * p.ldy + n] = f2bf(g / (1.f + __expf(-g)) * up[i]);
      }
    }
    return;
  }
  if (EPI == ROPE_KV) {
    const int qk_rows = (p.nq + p.nkv) * p.D;
    f32x4_t other;
#pragma unroll
    for (int i = 0; i < 4; ++i) other[i] = __shfl_xor(acc[i], 8, 64);
    if (lane >= 32) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + i;
      if (m >= p.M) continue;
      const int64_t ps = p.pos[m];
      const int b = m / p.T;
      const int cb = p.cache_idx ? p.cache_idx[b] : b;
      const bool in_cache = ps >= 0 && ps < p.Lmax;
      uint16_t* yr = p.y + (int64_t)m * p.ldy;
      if (tile < qk_tiles) {
        const int h = row / p.D;
        const float cs = cs_pre[i], sn = sn_pre[i];
        const float mine = bf2f(f2bf(acc[i])), part2 = bf2f(f2bf(other[i]));   // bf16 projection outputs
        const uint16_t o = c < 8 ? f2bf(mine * cs - part2 * sn) : f2bf(mine * cs + part2 * sn);
        yr[row] = o;
        if (h >= p.nq && in_cache)
          p.kc[(int64_t)cb * p.c_sb + (int64_t)(h - p.nq) * p.c_sh + ps * p.c_sl + (row % p.D)] = o;
      } else {
        const int r = (p.nq + p.nkv) * p.D + (tile - qk_tiles) * 16 + c;
        if (r >= p.N) continue;
        const uint16_t o = f2bf(acc[i]);
        yr[r] = o;
        const int vr = r - qk_rows;
        if (in_cache) p.vc[(int64_t)cb * p.c_sb + (int64_t)(vr / p.D) * p.c_sh + ps * p.c_sl + vr % p.D] = o;
      }
    }
    return;
  }
  const int n = tile * 16 + c;
  if (lane >= 32 || n >= p.N) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + i;
    if (m >= p.M) continue;
    uint16_t* yr = p.y + (int64_t)m * p.ldy;
    if (EPI == RESID) {
      float yv = bf2f(y_pre[i]);
      if (p.yadd) {
        yv = bf2f(f2bf(yv + bf2f(f2bf(ya_pre[i]))));
        p.yadd[(int64_t)m * p.N + n] = 0.f;
      }
      yr[n] = f2bf(yv + bf2f(f2bf(acc[i])));
    } else if (p.yf) {
      p.yf[(int64_t)m * p.ldy + n] = acc[i];
    } else {
      yr[n] = f2bf(acc[i]);
    }
  }
}

int g_mfma_split = -1;   // knob 8: K split over workgroups in dmm launches (NXD_DECODE_MFMA_SPLIT, default 0)
int g_mfma = -1;   // knob 7: dmm_kernel from this many activation rows on (NXD_DECODE_MFMA, default 4; 0 = never)

template <int EPI, bool NORM, bool XI>
static int launch_mfma(Params p, int tiles, hipStream_t s) {
  // K split over KS waves of one workgroup (reduced in LDS), KS doubling until ~2,048 waves stream
  // while every wave keeps >= 256 elements of K (Llama-3.2-1B: qkv / o_proj 8, down 16, gate_up 2,
  // lm_head 1), 4 / 8 / 16 waves per workgroup.  NXD_DECODE_MFMA_SPLIT=1 instead keeps 4-wave
  // workgroups and splits K further over workgroups (hand-off through g_sk) to ~512 workgroups:
  // batch 8 1.135 vs 1.077 ms per step, batch 4 1.09 vs 1.01 (profiles/r5m_decode_mfma_ab.jsonl).
  if (g_mfma_split < 0) {
    const char* e = getenv("NXD_DECODE_MFMA_SPLIT");
    g_mfma_split = e ? atoi(e) : 0;
  }
  const int split_mode = g_mfma_split;
  static const int target = [] {
    const char* e = getenv("NXD_DECODE_MFMA_WGS");
    const int v = e ? atoi(e) : 512;
    return v > 0 ? v : 512;
  }();
  const size_t lds = NORM ? (size_t)p.M * p.K * 2 : 0;
  int ks = 1, split = 1;
  if (split_mode) {
    auto wgs = [&] { return (int64_t)((tiles + (4 / ks) - 1) / (4 / ks)) * split; };
    while (wgs() < target && (int64_t)ks * split * 2 * 256 <= p.K) {
      if (ks < 4) ks *= 2;
      else if (split < kMaxSplit && tiles <= kSkTiles) split *= 2;
      else break;
    }
    p.split = split;
    const unsigned grid = (unsigned)wgs();
    if (ks == 4) hipLaunchKernelGGL((dmm_kernel<EPI, NORM, 4, 4, XI>), dim3(grid), dim3(256), lds, s, p);
    else if (ks == 2) hipLaunchKernelGGL((dmm_kernel<EPI, NORM, 2, 4, XI>), dim3(grid), dim3(256), lds, s, p);
    else hipLaunchKernelGGL((dmm_kernel<EPI, NORM, 1, 4, XI>), dim3(grid), dim3(256), lds, s, p);
    return hipGetLastError() == hipSuccess ? 0 : 1;
  }
  while (ks < 16 && (int64_t)tiles * ks < 2048 && p.K / (ks * 2) >= 256) ks *= 2;
  p.split = 1;
#define NXD_DMM(KSV, NW)                                                                                    \
  hipLaunchKernelGGL((dmm_kernel<EPI, NORM, KSV, NW, XI>), dim3((unsigned)((tiles + (NW / KSV) - 1) / (NW / KSV))), \
                     dim3(64 * NW), lds, s, p)
  if (ks == 16) NXD_DMM(16, 16);
  else if (ks == 8) NXD_DMM(8, 8);
  else if (ks == 4) NXD_DMM(4, 4);
  else if (ks == 2) NXD_DMM(2, 4);
  else NXD_DMM(1, 4);
#undef NXD_DMM
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

static int dispatch_mfma(const Params& p, int epi, bool norm, hipStream_t s) {
  switch (epi) {
    case PLAIN: {
      const int tiles = (p.N + 15) / 16;
      return norm ? launch_mfma<PLAIN, true, false>(p, tiles, s) : launch_mfma<PLAIN, false, false>(p, tiles, s);
    }
    case RESID: {
      const int tiles = (p.N + 15) / 16;
      return norm ? launch_mfma<RESID, true, false>(p, tiles, s) : launch_mfma<RESID, false, false>(p, tiles, s);
    }
    case GLU: {
      const int tiles = (p.N + 7) / 8;
      return norm ? launch_mfma<GLU, true, false>(p, tiles, s) : launch_mfma<GLU, false, false>(p, tiles, s);
    }
    case ROPE_KV: {
      const int tiles = (p.nq + p.nkv) * (p.D / 2 / 8) + (p.nkv * p.D + 15) / 16;
      if (p.xidx) return norm ? launch_mfma<ROPE_KV, true, true>(p, tiles, s) : -4;
      return norm ? launch_mfma<ROPE_KV, true, false>(p, tiles, s) : launch_mfma<ROPE_KV, false, false>(p, tiles, s);
    }
  }
  return -1;
}


// k-slices per row group: split K while the grid stays <= 8192 waves and slices keep >= 1024
// elements (o_proj 2048 x 2048 -> 2, down 2048 x 8192 -> 4, gate_up / lm_head / QKV -> 1)
int g_glu_pairs = 1;   // knob 0: (gate, up) row pairs per wave of the GLU projection (1 | 2)
int g_ks = 0;          // knob 1: k-slices per row group (0 = pick_ks)
int g_pf = -1;         // knob 2: early epilogue / prologue reads (Params::pf; NXD_DECODE_EPI_PF, default 1)
int g_dot2 = -1;       // knob 6: v_dot2c inner product (Params::dot2; NXD_DECODE_DOT2, default 1)
int g_occ = -1;        // knob 5: bs = 1 two-row kernels at 7 | 8 waves / SIMD (dgemv_kernel_occ; NXD_DECODE_OCC, 0 = natural)

// per-projection override (A/B): NXD_DECODE_KS_PLAIN / _RESID / _GLU / _QKV = 1 | 2 | 4
static int g_ks_epi[4] = {-2, -2, -2, -2};

static int pick_ks(int groups, int K, int epi) {
  if (g_ks == 1 || g_ks == 2 || g_ks == 4) return g_ks;
  if (g_ks_epi[0] == -2) {
    const char* names[4] = {"NXD_DECODE_KS_PLAIN", "NXD_DECODE_KS_RESID", "NXD_DECODE_KS_GLU", "NXD_DECODE_KS_QKV"};
    for (int i = 0; i < 4; ++i) {
      const char* e = getenv(names[i]);
      g_ks_epi[i] = e ? atoi(e) : 0;
    }
  }
  const int f = g_ks_epi[epi & 3];
  if (f == 1 || f == 2 || f == 4) return f;
  // QKV + RoPE (two rows per wave, K = hidden): whole rows per wave, no LDS partial reduction --
  // Llama-3.2-1B bs=1 0.6187 / 0.6195 vs 0.6226 / 0.6207 ms/token with 2 slices, alternating
  // (profiles/r4_decode_shape_sweep.txt)
  if (epi == ROPE_KV && K <= 4096) return 1;
  int ks = 1;
  while (ks < 4 && groups * ks * 2 <= 8192 && K / (ks * 2) >= 1024) ks *= 2;
  return ks;
}

template <int MM, int NW, int EPI, bool NORM, bool XI = false>
static int launch(const Params& p, int groups, hipStream_t s) {
  const size_t lds = NORM ? (size_t)MM * p.K * 2 : 0;
  const int ks = pick_ks(groups, p.K, EPI);
  const dim3 grid((unsigned)((groups * ks + 3) / 4)), block(256);
  if constexpr (MM == 1 && NW == 2 && !XI) {
    if (g_occ == 7 || g_occ == 8) {
#define NXD_OCC_LAUNCH(W)                                                                   \
  if (ks == 4)                                                                              \
    hipLaunchKernelGGL((dgemv_kernel_occ<MM, NW, EPI, NORM, 4, W>), grid, block, lds, s, p); \
  else if (ks == 2)                                                                         \
    hipLaunchKernelGGL((dgemv_kernel_occ<MM, NW, EPI, NORM, 2, W>), grid, block, lds, s, p); \
  else                                                                                      \
    hipLaunchKernelGGL((dgemv_kernel_occ<MM, NW, EPI, NORM, 1, W>), grid, block, lds, s, p);
      if (g_occ == 7) { NXD_OCC_LAUNCH(7) } else { NXD_OCC_LAUNCH(8) }
#undef NXD_OCC_LAUNCH
      return hipGetLastError() == hipSuccess ? 0 : 1;
    }
  }
  if (ks == 4)
    hipLaunchKernelGGL((dgemv_kernel<MM, NW, EPI, NORM, 4, XI>), grid, block, lds, s, p);
  else if (ks == 2)
    hipLaunchKernelGGL((dgemv_kernel<MM, NW, EPI, NORM, 2, XI>), grid, block, lds, s, p);
  else
    hipLaunchKernelGGL((dgemv_kernel<MM, NW, EPI, NORM, 1, XI>), grid, block, lds, s, p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <int MM>
static int dispatch(const Params& p, int epi, bool norm, hipStream_t s) {
  switch (epi) {
    case PLAIN: {
      const int nw = p.N >= 16384 ? 2 : 1;
      const int groups = (p.N + nw - 1) / nw;
      if (nw == 2) return norm ? launch<MM, 2, PLAIN, true>(p, groups, s) : launch<MM, 2, PLAIN, false>(p, groups, s);
      return norm ? launch<MM, 1, PLAIN, true>(p, groups, s) : launch<MM, 1, PLAIN, false>(p, groups, s);
    }
    case RESID:
      return norm ? launch<MM, 1, RESID, true>(p, p.N, s) : launch<MM, 1, RESID, false>(p, p.N, s);
    case GLU:
      if (g_glu_pairs == 2) {
        const int groups = (p.N + 1) / 2;
        return norm ? launch<MM, 4, GLU, true>(p, groups, s) : launch<MM, 4, GLU, false>(p, groups, s);
      }
      return norm ? launch<MM, 2, GLU, true>(p, p.N, s) : launch<MM, 2, GLU, false>(p, p.N, s);
    case ROPE_KV: {
      const int groups = (p.nq + p.nkv) * (p.D / 2) + (p.nkv * p.D + 1) / 2;
      if (p.xidx) return norm ? launch<MM, 2, ROPE_KV, true, true>(p, groups, s) : -4;
      return norm ? launch<MM, 2, ROPE_KV, true>(p, groups, s) : launch<MM, 2, ROPE_KV, false>(p, groups, s);
    }
  }
  return -1;
}

}  // namespace dfused

void dgemv_set_knob(int which, int value) {
  if (which == 0) dfused::g_glu_pairs = value == 2 ? 2 : 1;
  else if (which == 1) dfused::g_ks = value;
  else if (which == 2) dfused::g_pf = value != 0;
  else if (which == 5) dfused::g_occ = value;
  else if (which == 6) dfused::g_dot2 = value != 0;
  else if (which == 7) dfused::g_mfma = value;
  else if (which == 8) dfused::g_mfma_split = value;
}

int dgemv_launch(int epi, const void* x, int64_t ldx, const void* norm_w, float eps, const void* w, int64_t ldw, void* y,
                 int64_t ldy, int M, int N, int K, int nq, int nkv, int D, const float* cos_t, const float* sin_t,
                 const int64_t* pos, int T, void* kc, void* vc, int64_t c_sb, int64_t c_sh, int64_t c_sl,
                 const int* cache_idx, int Lmax, int max_pos, const float* xadd, float* yadd, hipStream_t stream,
                 const int64_t* xidx, int64_t xrows, void* xcopy, float* yf) {
  if (yf && epi != dfused::PLAIN) return -5;
  if (M < 1 || M > 8 || N < 1 || K < 8 || (K % 8)) return -1;
  if ((xadd && !norm_w) || (yadd && epi != dfused::RESID)) return -3;
  if (xidx && (epi != dfused::ROPE_KV || !norm_w || xrows < 1)) return -4;
  if (norm_w && (size_t)M * K * 2 > 65536) return -2;
  dfused::Params p{static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(norm_w), eps,
                   static_cast<const uint16_t*>(w), ldw, static_cast<uint16_t*>(y), ldy, M, N, K, nq, nkv, D, cos_t,
                   sin_t, pos, T, static_cast<uint16_t*>(kc), static_cast<uint16_t*>(vc), c_sb, c_sh, c_sl, cache_idx,
                   Lmax, max_pos, xadd, yadd, 1};
  if (dfused::g_pf < 0) {
    const char* e = getenv("NXD_DECODE_EPI_PF");
    dfused::g_pf = e ? (atoi(e) != 0) : 1;
  }
  p.pf = dfused::g_pf;
  p.xidx = xidx;
  p.xrows = xrows;
  p.xcopy = static_cast<uint16_t*>(xcopy);
  p.yf = yf;
  if (dfused::g_dot2 < 0) {
    const char* e = getenv("NXD_DECODE_DOT2");
    dfused::g_dot2 = e ? (atoi(e) != 0) : 1;
  }
  p.dot2 = dfused::g_dot2;
  if (dfused::g_occ < 0) {
    const char* e = getenv("NXD_DECODE_OCC");
    dfused::g_occ = e ? atoi(e) : 0;
    const char* gp = getenv("NXD_DECODE_GLU_PAIRS");
    if (gp && atoi(gp) == 2) dfused::g_glu_pairs = 2;
  }
  const bool norm = norm_w != nullptr;
  if (dfused::g_mfma < 0) {
    const char* e = getenv("NXD_DECODE_MFMA");
    dfused::g_mfma = e ? atoi(e) : 4;
  }
  // MFMA rows need whole rotary 8-pair tiles (D / 2 % 8 == 0) and 16-B aligned 32-deep k-steps
  if (M >= 2 && dfused::g_mfma > 0 && M >= dfused::g_mfma && (epi != dfused::ROPE_KV || (D / 2) % 8 == 0))
    return dfused::dispatch_mfma(p, epi, norm, stream);
  if (M == 1) return dfused::dispatch<1>(p, epi, norm, stream);
  if (M == 2) return dfused::dispatch<2>(p, epi, norm, stream);
  if (M <= 4) return dfused::dispatch<4>(p, epi, norm, stream);
  return dfused::dispatch<8>(p, epi, norm, stream);
}

}  // namespace nxd
