// FlashAttention-2 backward for CDNA4 (gfx950): dQ, dK, dV from Q, K, V, dO, LSE, delta.
// Replaces the reference's NKI `flash_attn_bwd` (src/neuronx_distributed/kernels/flash_attn.py:61-82,130-148).
//
// Structure (cdna_hip_programming.md, "Attention backward"):
//   * one workgroup = 4 waves = 128 keys of one (batch, kv-head); each wave owns 32 keys and
//     keeps dK^T / dV^T for them in accumulators while the workgroup sweeps every q head of the
//     GQA group x every 32-row query tile (GQA reduction of dK/dV happens in registers — no
//     repeat_kv, no second reduction pass);
//   * "key on the lane": S = Q K^T and dP = dO V^T are computed with the key as the MFMA column,
//     so their fp32 accumulators convert in place into the B operands of dV^T += dO^T P and
//     dK^T += Q^T dS (accumulator-as-operand, no LDS round trip);
//   * Q / dO tiles arrive by LDS-DMA one tile ahead into a double-buffered swizzled image that
//     serves both row reads (ds_read_b128) and transposed reads (ds_read_b64_tr_b16);
//   * dQ: dS crosses LDS once (transposed image), each wave computes one 32-wide d block of
//     dS . K over all 128 keys and adds it with f32 atomics (two 128-B row segments per
//     wave-instruction — the full-rate atomic shape) into an fp32 dQ accumulator; a tiny
//     post-pass scales and narrows dQ to bf16.
#include "common.h"

namespace nxd {
namespace fab {

constexpr int kWaves = 4;
constexpr int kThreads = 256;
constexpr int kBlockK = 128;  // keys per workgroup
constexpr int kBlockQ = 32;   // query rows per tile

struct BwdParams {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  const uint16_t* dout;
  const float* lse;    // [B, Hq, Sq]
  const float* delta;  // [B, Hq, Sq]
  float* dq_acc;       // [B, Hq, Sq, D] fp32, zero-initialised
  uint16_t* dk;
  uint16_t* dv;
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t do_sb, do_ss, do_sh;
  int64_t dk_sb, dk_ss, dk_sh;
  int64_t dv_sb, dv_ss, dv_sh;
  int B, Sq, Sk, Hq, Hkv;
  float scale;       // softmax scale
  float scale_log2;  // softmax scale * log2(e)
  int causal;
  int causal_offset;
};

template <int D>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (D == 128) {
    return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  } else {
    return ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
  }
}
template <int D>
__device__ __forceinline__ int lds_off(int row, int ch) {
  return row * (D * 2) + swz<D>(row, ch) * 16;
}

typedef __attribute__((address_space(3))) short4_t* lds_s4_t;

// transposed read of 4 consecutive rows at (row0 + tq, col .. col+3) of a swizzled [rows][D] image
template <int D>
__device__ __forceinline__ short4_t tr_read(const char* base, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(base + lds_off<D>(row, col >> 3) + (col & 7) * 2));
}

// dS^T image: [128 keys][32 q] bf16, 64-B rows, 8-B chunks XOR-swizzled by (row & 7)
__device__ __forceinline__ int ds_off(int key, int q) { return key * 64 + (((q >> 2) ^ (key & 7)) << 3) + (q & 3) * 2; }

template <int D>
__global__ void __launch_bounds__(kThreads, 1) bwd_kernel(BwdParams p) {
  constexpr int CH = D / 8;
  constexpr int KS = D / 16;
  constexpr int NDB = D / 32;
  constexpr int KV_BYTES = kBlockK * D * 2;
  constexpr int QT_BYTES = kBlockQ * D * 2;
  constexpr int OFF_K = 0;                            // K block image (B operand of dQ = dS K)
  constexpr int OFF_Q = KV_BYTES;                     // 2 buffers
  constexpr int OFF_DO = OFF_Q + 2 * QT_BYTES;        // 2 buffers
  constexpr int OFF_DS = OFF_DO + 2 * QT_BYTES;       // 128 x 64 B
  constexpr int OFF_LD = OFF_DS + kBlockK * 64;       // 2 buffers x (32 lse + 32 delta) floats
  constexpr int ROWS_PER_PIECE = 1024 / (2 * D);
  constexpr int QT_PIECES = QT_BYTES / 1024;          // per tile (Q or dO)
  constexpr int QT_PIECES_PER_WAVE = QT_PIECES / kWaves;
  // dQ work split: NDB d-blocks x (4 / NDB) key ranges
  constexpr int KEY_SPLIT = kWaves / NDB;
  constexpr int KEYS_PER_DQ = kBlockK / KEY_SPLIT;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nkb = (p.Sk + kBlockK - 1) / kBlockK;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = L % (p.B * p.Hkv);
  const int jb = L / (p.B * p.Hkv);
  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int G = p.Hq / p.Hkv;
  const int Sq_pad = (p.Sq + kBlockQ - 1) / kBlockQ * kBlockQ;
  // causal: pair the heaviest and the lightest key block in one workgroup (equal work per WG)
  const int npass = (p.causal && (nkb - 1 - jb) != jb) ? 2 : 1;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3, g = lane >> 4;

  const uint16_t* kbase = p.k + (int64_t)b * p.k_sb + (int64_t)hkv * p.k_sh;
  const uint16_t* vbase = p.v + (int64_t)b * p.v_sb + (int64_t)hkv * p.v_sh;

  for (int pass = 0; pass < npass; ++pass) {
    const int kb = pass == 0 ? jb : nkb - 1 - jb;
    const int kb0 = kb * kBlockK;
    const int wkey0 = kb0 + 32 * w;  // this wave's first key
    const int my_key = wkey0 + r;

    // ---- K block -> LDS (for dQ); this wave's K and V rows -> registers (B operands of S, dP)
    for (int idx = tid; idx < kBlockK * CH; idx += kThreads) {
      const int row = idx / CH, ch = idx % CH;
      const int key = kb0 + row;
      u32x4_t kv4 = {0, 0, 0, 0};
      if (key < p.Sk) kv4 = *reinterpret_cast<const u32x4_t*>(kbase + (int64_t)key * p.k_ss + ch * 8);
      *reinterpret_cast<u32x4_t*>(smem + OFF_K + lds_off<D>(row, ch)) = kv4;
    }
    bf16x8_t kf[KS], vf[KS];
    {
      const bool ok = my_key < p.Sk;
      const uint16_t* kr = kbase + (int64_t)(ok ? my_key : 0) * p.k_ss;
      const uint16_t* vr = vbase + (int64_t)(ok ? my_key : 0) * p.v_ss;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const u32x4_t a = ok ? *reinterpret_cast<const u32x4_t*>(kr + 16 * s + 8 * hh) : u32x4_t{0, 0, 0, 0};
        const u32x4_t c = ok ? *reinterpret_cast<const u32x4_t*>(vr + 16 * s + 8 * hh) : u32x4_t{0, 0, 0, 0};
        kf[s] = __builtin_bit_cast(bf16x8_t, a);
        vf[s] = __builtin_bit_cast(bf16x8_t, c);
      }
    }

    // ---- query-tile schedule: every head of the group x tiles of 32 rows
    int qstart = 0;
    if (p.causal) qstart = max(0, kb0 - p.causal_offset);
    qstart = (qstart / kBlockQ) * kBlockQ;
    const int n_qt = qstart < p.Sq ? (p.Sq - qstart + kBlockQ - 1) / kBlockQ : 0;
    const int n_it = G * n_qt;

    auto issue_tile = [&](int it, int buf) {
      const int hq = hkv * G + it / n_qt;
      const int qt0 = qstart + (it % n_qt) * kBlockQ;
      const uint16_t* qb = p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
      const uint16_t* db = p.dout + (int64_t)b * p.do_sb + (int64_t)hq * p.do_sh;
#pragma unroll
      for (int i = 0; i < QT_PIECES_PER_WAVE; ++i) {
        const int piece = w * QT_PIECES_PER_WAVE + i;
        const int row = piece * ROWS_PER_PIECE + lane / CH;
        const int ch = swz<D>(row, lane % CH);
        const int qi = min(qt0 + row, p.Sq - 1);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(qb + (int64_t)qi * p.q_ss + ch * 8),
                                         (__attribute__((address_space(3))) void*)(smem + OFF_Q + buf * QT_BYTES + piece * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(db + (int64_t)qi * p.do_ss + ch * 8),
                                         (__attribute__((address_space(3))) void*)(smem + OFF_DO + buf * QT_BYTES + piece * 1024), 16, 0, 0);
      }
      if (w == 0) {
        const int qi = min(qt0 + (lane & 31), p.Sq - 1);
        const float* src = (lane < 32 ? p.lse : p.delta) + ((int64_t)b * p.Hq + hq) * p.Sq + qi;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(smem + OFF_LD + buf * 256), 4, 0, 0);
      }
    };

    f32x16_t acc_dk[NDB], acc_dv[NDB];
#pragma unroll
    for (int i = 0; i < NDB; ++i) {
      acc_dk[i] = f32x16_t{0};
      acc_dv[i] = f32x16_t{0};
    }

    if (n_it > 0) issue_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // K image + tile 0 visible

    for (int it = 0; it < n_it; ++it) {
      const int buf = it & 1;
      const int hq = hkv * G + it / n_qt;
      const int qt0 = qstart + (it % n_qt) * kBlockQ;
      // buffer buf^1 was last read in iteration it-1, closed by its final barrier
      if (it + 1 < n_it) issue_tile(it + 1, buf ^ 1);

      const char* ql = smem + OFF_Q + buf * QT_BYTES;
      const char* dl = smem + OFF_DO + buf * QT_BYTES;
      const float* lsel = reinterpret_cast<const float*>(smem + OFF_LD + buf * 256);
      const float* dell = lsel + 32;

      const bool active = !p.causal || (wkey0 <= qt0 + kBlockQ - 1 + p.causal_offset);
      if (active) {
        // ---- S = Q K^T, dP = dO V^T (key on the lane; K/V rows in registers)
        f32x16_t s_acc = f32x16_t{0}, dp_acc = f32x16_t{0};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const u32x4_t qa = *reinterpret_cast<const u32x4_t*>(ql + lds_off<D>(r, 2 * s + hh));
          s_acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, qa), kf[s], s_acc, 0, 0, 0);
          const u32x4_t da = *reinterpret_cast<const u32x4_t*>(dl + lds_off<D>(r, 2 * s + hh));
          dp_acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, da), vf[s], dp_acc, 0, 0, 0);
        }
        // ---- P, dS
        bf16x8_t pf[2], dsf[2];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int qrow = 8 * gq + 4 * hh;  // local q of element e = 4gq + i is qrow + i
          const f32x4_t l4 = *reinterpret_cast<const f32x4_t*>(lsel + qrow);
          const f32x4_t d4 = *reinterpret_cast<const f32x4_t*>(dell + qrow);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int e = 4 * gq + i;
            const int qg = qt0 + qrow + i;
            const float lse2 = l4[i] == -INFINITY ? INFINITY : l4[i] * 1.4426950408889634f;
            float pv = exp2f(s_acc[e] * p.scale_log2 - lse2);
            const bool bad = qg >= p.Sq || my_key >= p.Sk || (p.causal && my_key > qg + p.causal_offset);
            pv = bad ? 0.f : pv;
            const float dsv = pv * (dp_acc[e] - d4[i]);
            pf[e >> 3][e & 7] = (__bf16)pv;
            dsf[e >> 3][e & 7] = (__bf16)dsv;
          }
        }
        // ---- dV^T += dO^T P ; dK^T += Q^T dS   (A operands by transposed reads)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int R0 = 16 * s2 + 4 * hh;
#pragma unroll
          for (int dbk = 0; dbk < NDB; ++dbk) {
            const int col = 32 * dbk + 16 * (g & 1) + 4 * tp;
            const short4_t dlo = tr_read<D>(dl, R0 + tq, col);
            const short4_t dhi = tr_read<D>(dl, R0 + 8 + tq, col);
            const short __attribute__((ext_vector_type(8))) da8 = {dlo[0], dlo[1], dlo[2], dlo[3], dhi[0], dhi[1], dhi[2], dhi[3]};
            acc_dv[dbk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, da8), pf[s2], acc_dv[dbk], 0, 0, 0);
            const short4_t qlo = tr_read<D>(ql, R0 + tq, col);
            const short4_t qhi = tr_read<D>(ql, R0 + 8 + tq, col);
            const short __attribute__((ext_vector_type(8))) qa8 = {qlo[0], qlo[1], qlo[2], qlo[3], qhi[0], qhi[1], qhi[2], qhi[3]};
            acc_dk[dbk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, qa8), dsf[s2], acc_dk[dbk], 0, 0, 0);
          }
        }
        // ---- dS -> LDS (transposed image [key][q]): lane stores q = 8gq+4hh .. +3 of its key.
        // (whole-vector bit casts: per-element extraction of bf16 ext_vectors miscompiles on
        // ROCm 7.2 — it replicated element 0 into all four slots)
        const u32x4_t ds_w0 = __builtin_bit_cast(u32x4_t, dsf[0]);
        const u32x4_t ds_w1 = __builtin_bit_cast(u32x4_t, dsf[1]);
        *reinterpret_cast<u32x2_t*>(smem + OFF_DS + ds_off(32 * w + r, 0 + 4 * hh)) = u32x2_t{ds_w0[0], ds_w0[1]};
        *reinterpret_cast<u32x2_t*>(smem + OFF_DS + ds_off(32 * w + r, 8 + 4 * hh)) = u32x2_t{ds_w0[2], ds_w0[3]};
        *reinterpret_cast<u32x2_t*>(smem + OFF_DS + ds_off(32 * w + r, 16 + 4 * hh)) = u32x2_t{ds_w1[0], ds_w1[1]};
        *reinterpret_cast<u32x2_t*>(smem + OFF_DS + ds_off(32 * w + r, 24 + 4 * hh)) = u32x2_t{ds_w1[2], ds_w1[3]};
      } else {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<u32x2_t*>(smem + OFF_DS + ds_off(32 * w + r, 8 * gq + 4 * hh)) = u32x2_t{0, 0};
      }
      // dS^T complete.  Raw barrier: the tile prefetch (LDS-DMA) stays in flight across it.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();

      // ---- dQ[q][d] += dS[q][key] K[key][d] over this wave's (d block, key range)
      const int dbk = w % NDB;
      const int kr0 = (w / NDB) * KEYS_PER_DQ;
      const bool any = !p.causal || (kb0 + kr0 <= qt0 + kBlockQ - 1 + p.causal_offset);
      if (any) {
        f32x16_t acc_dq = f32x16_t{0};
#pragma unroll
        for (int s = 0; s < KEYS_PER_DQ / 16; ++s) {
          const int kr = kr0 + 16 * s + 8 * hh;  // first key of this lane-half's 8
          // A = dS[q][key]: tr reads of the [key][q] image, column q = r
          const int qc = 16 * (g & 1) + 4 * tp;
          const short4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(smem + OFF_DS + ds_off(kr + tq, qc)));
          const short4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(smem + OFF_DS + ds_off(kr + 4 + tq, qc)));
          const short __attribute__((ext_vector_type(8))) a8 = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          // B = K[key][d]: tr reads of the K image, column d = 32 dbk + r
          const int col = 32 * dbk + 16 * (g & 1) + 4 * tp;
          const short4_t b0 = tr_read<D>(smem + OFF_K, kr + tq, col);
          const short4_t b1 = tr_read<D>(smem + OFF_K, kr + 4 + tq, col);
          const short __attribute__((ext_vector_type(8))) b8 = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
          acc_dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), __builtin_bit_cast(bf16x8_t, b8), acc_dq, 0, 0, 0);
        }
        // 16 UNCONDITIONAL atomics per lane (dq_acc has Sq padded to kBlockQ rows), so the
        // counted wait below knows exactly how many of this wave's VM ops are atomics.
        float* dqb = p.dq_acc + (((int64_t)b * p.Hq + hq) * Sq_pad) * D + 32 * dbk + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int qg = qt0 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          atomicAdd(dqb + (int64_t)qg * D, acc_dq[e]);
        }
        // retire the tile prefetch (issued before the atomics) but leave the 16 atomics in flight
        asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // dS^T / Q / dO reads done; next tile landed for every wave
    }

    // ---- dK, dV epilogue: C rows = d, col = key
    if (my_key < p.Sk) {
      uint16_t* dkr = p.dk + (int64_t)b * p.dk_sb + (int64_t)my_key * p.dk_ss + (int64_t)hkv * p.dk_sh;
      uint16_t* dvr = p.dv + (int64_t)b * p.dv_sb + (int64_t)my_key * p.dv_ss + (int64_t)hkv * p.dv_sh;
#pragma unroll
      for (int dbk = 0; dbk < NDB; ++dbk) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int d = 32 * dbk + 8 * gq + 4 * hh;
          u32x2_t kv, vv;
          kv[0] = pack2bf(acc_dk[dbk][4 * gq] * p.scale, acc_dk[dbk][4 * gq + 1] * p.scale);
          kv[1] = pack2bf(acc_dk[dbk][4 * gq + 2] * p.scale, acc_dk[dbk][4 * gq + 3] * p.scale);
          vv[0] = pack2bf(acc_dv[dbk][4 * gq], acc_dv[dbk][4 * gq + 1]);
          vv[1] = pack2bf(acc_dv[dbk][4 * gq + 2], acc_dv[dbk][4 * gq + 3]);
          *reinterpret_cast<u32x2_t*>(dkr + d) = kv;
          *reinterpret_cast<u32x2_t*>(dvr + d) = vv;
        }
      }
    }
    if (pass + 1 < npass) __syncthreads();  // K image reused by the next pass
  }
}

// delta[b, h, q] = sum_d dO * O  (fp32); D/8 lanes per row.
template <int D>
__global__ void __launch_bounds__(256) delta_kernel(const uint16_t* o, const uint16_t* dout, float* delta,
                                                   int64_t o_sb, int64_t o_ss, int64_t o_sh,
                                                   int64_t d_sb, int64_t d_ss, int64_t d_sh, int B, int Sq, int Hq) {
  constexpr int LPR = D / 8;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t nrows = (int64_t)B * Hq * Sq;
  float acc = 0.f;
  int b = 0, h = 0, qi = 0;
  if (row < nrows) {
    b = row / ((int64_t)Hq * Sq);
    h = (row / Sq) % Hq;
    qi = row % Sq;
    const u32x4_t ov = *reinterpret_cast<const u32x4_t*>(o + b * o_sb + (int64_t)qi * o_ss + h * o_sh + c * 8);
    const u32x4_t dv = *reinterpret_cast<const u32x4_t*>(dout + b * d_sb + (int64_t)qi * d_ss + h * d_sh + c * 8);
    float of[8], df[8];
    unpack8(ov, of);
    unpack8(dv, df);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += of[i] * df[i];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < nrows && c == 0) delta[row] = acc;
}

// dq (bf16, strided [B,S,H,D]) = dq_acc ([B,H,S,D] fp32) * scale
template <int D>
__global__ void __launch_bounds__(256) dq_convert_kernel(const float* acc, uint16_t* dq, int64_t sb, int64_t ss, int64_t sh,
                                                        int B, int Sq, int Hq, float scale) {
  constexpr int LPR = D / 8;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t nrows = (int64_t)B * Hq * Sq;
  if (row >= nrows) return;
  const int b = row / ((int64_t)Hq * Sq);
  const int h = (row / Sq) % Hq;
  const int qi = row % Sq;
  const int Sq_pad = (Sq + 31) / 32 * 32;
  const int64_t arow = ((int64_t)b * Hq + h) * Sq_pad + qi;
  const f32x4_t a0 = *reinterpret_cast<const f32x4_t*>(acc + arow * D + c * 8);
  const f32x4_t a1 = *reinterpret_cast<const f32x4_t*>(acc + arow * D + c * 8 + 4);
  float f[8] = {a0[0] * scale, a0[1] * scale, a0[2] * scale, a0[3] * scale,
                a1[0] * scale, a1[1] * scale, a1[2] * scale, a1[3] * scale};
  *reinterpret_cast<u32x4_t*>(dq + b * sb + (int64_t)qi * ss + h * sh + c * 8) = pack8(f);
}

}  // namespace fab

int flash_attn_bwd_launch(const void* q, const void* k, const void* v, const void* o, const void* dout,
                          const float* lse, float* delta, float* dq_acc, void* dq, void* dk, void* dv,
                          const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os,
                          const int64_t* dos, const int64_t* dqs, const int64_t* dks, const int64_t* dvs,
                          int B, int Sq, int Sk, int Hq, int Hkv, int D, float softmax_scale, int causal,
                          int causal_offset, hipStream_t stream) {
  using namespace fab;
  if (Hkv <= 0 || Hq % Hkv != 0 || (D != 64 && D != 128)) return -1;
  const int64_t nrows = (int64_t)B * Hq * Sq;
  const int rows_per_block = 256 / (D / 8);
  const int gpre = (int)((nrows + rows_per_block - 1) / rows_per_block);
  if (D == 128)
    hipLaunchKernelGGL(delta_kernel<128>, dim3(gpre), dim3(256), 0, stream, (const uint16_t*)o, (const uint16_t*)dout, delta,
                       os[0], os[1], os[2], dos[0], dos[1], dos[2], B, Sq, Hq);
  else
    hipLaunchKernelGGL(delta_kernel<64>, dim3(gpre), dim3(256), 0, stream, (const uint16_t*)o, (const uint16_t*)dout, delta,
                       os[0], os[1], os[2], dos[0], dos[1], dos[2], B, Sq, Hq);
  const int64_t Sq_pad = (Sq + kBlockQ - 1) / kBlockQ * kBlockQ;
  (void)hipMemsetAsync(dq_acc, 0, (size_t)B * Hq * Sq_pad * D * sizeof(float), stream);

  BwdParams p;
  p.q = (const uint16_t*)q; p.k = (const uint16_t*)k; p.v = (const uint16_t*)v; p.dout = (const uint16_t*)dout;
  p.lse = lse; p.delta = delta; p.dq_acc = dq_acc; p.dk = (uint16_t*)dk; p.dv = (uint16_t*)dv;
  p.q_sb = qs[0]; p.q_ss = qs[1]; p.q_sh = qs[2];
  p.k_sb = ks[0]; p.k_ss = ks[1]; p.k_sh = ks[2];
  p.v_sb = vs[0]; p.v_ss = vs[1]; p.v_sh = vs[2];
  p.do_sb = dos[0]; p.do_ss = dos[1]; p.do_sh = dos[2];
  p.dk_sb = dks[0]; p.dk_ss = dks[1]; p.dk_sh = dks[2];
  p.dv_sb = dvs[0]; p.dv_ss = dvs[1]; p.dv_sh = dvs[2];
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale = softmax_scale;
  p.scale_log2 = softmax_scale * 1.4426950408889634f;
  p.causal = causal; p.causal_offset = causal_offset;
  const int nkb = (Sk + kBlockK - 1) / kBlockK;
  const int grid = (causal ? (nkb + 1) / 2 : nkb) * B * Hkv;
  if (grid > 0) {
    if (D == 128) {
      const size_t lds = kBlockK * 128 * 2 + 4 * kBlockQ * 128 * 2 + kBlockK * 64 + 512;
      static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once
      if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)bwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
      }
      hipLaunchKernelGGL(bwd_kernel<128>, dim3(grid), dim3(kThreads), lds, stream, p);
    } else {
      const size_t lds = kBlockK * 64 * 2 + 4 * kBlockQ * 64 * 2 + kBlockK * 64 + 512;
      hipLaunchKernelGGL(bwd_kernel<64>, dim3(grid), dim3(kThreads), lds, stream, p);
    }
  }
  if (D == 128)
    hipLaunchKernelGGL(dq_convert_kernel<128>, dim3(gpre), dim3(256), 0, stream, dq_acc, (uint16_t*)dq, dqs[0], dqs[1], dqs[2], B, Sq, Hq, softmax_scale);
  else
    hipLaunchKernelGGL(dq_convert_kernel<64>, dim3(gpre), dim3(256), 0, stream, dq_acc, (uint16_t*)dq, dqs[0], dqs[1], dqs[2], B, Sq, Hq, softmax_scale);
  return (int)hipGetLastError();
}

}  // namespace nxd
