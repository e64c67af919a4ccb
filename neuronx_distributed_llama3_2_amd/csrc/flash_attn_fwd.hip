// FlashAttention-2 forward for CDNA4 (gfx950): causal / non-causal, GQA-native, bf16 in,
// fp32 accumulate, LSE out.  Replaces the reference's NKI `flash_fwd` (reference:
// src/neuronx_distributed/kernels/flash_attn.py:32-58,151-191) and the inference
// `attention_isa_kernel` prefill path (examples/inference/modules/attention/attention_base.py:105-133).
//
// Design (MI355X-first, see cdna_hip_programming.md "Fused attention prefill"):
//   * workgroup = 4 waves (256 threads) = 128 query rows of one (batch, q-head); each wave owns
//     32 rows for the whole key sweep, Q fragments live in VGPRs for the whole kernel;
//   * K/V tiles of 64 keys stream global -> LDS by LDS-DMA (global_load_lds_dwordx4), issued
//     one tile ahead so the copy overlaps the current tile's MFMAs, into a double-buffered,
//     XOR-swizzled LDS image (T2; swizzle applied on the source address) so that K row reads
//     (ds_read_b128) and V transposed reads (ds_read_b64_tr_b16, T10) are both bank-conflict
//     free, and no staging VGPRs are spent (the kernel sits at 2 waves/SIMD, 236 VGPRs);
//   * swapped product S^T = K Q^T with v_mfma_f32_32x32x16_bf16: every lane holds one query row
//     of the score tile, so the online softmax (max / exp2 / sum) is lane-local plus one
//     cross-half exchange, and the fp32 accumulator converts in place into the B operand of
//     O^T += V^T P (no LDS round trip for P);
//   * GQA: K/V are addressed through kv_head = q_head / (Hq/Hkv) — no repeat_kv copies; the
//     block id is remapped so that the q heads sharing a kv head run back to back on one XCD
//     (T1, shared L2), heavy causal q-blocks first.
//   * arbitrary (batch, seq, head) strides, so Q/K/V can be read straight out of a fused
//     [S, B, (Hq+2Hkv)*D] QKV projection output and O written into [S, B, Hq*D].
#include "common.h"

namespace nxd {
namespace fa {

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kBlockM = kWaves * 32;  // q rows per workgroup
constexpr int kBlockN = 64;           // keys per tile

struct FwdParams {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  float* lse;  // [B, Hq, Sq]
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t o_sb, o_ss, o_sh;
  int B, Sq, Sk, Hq, Hkv;
  float scale_log2;  // softmax_scale * log2(e)
  int causal;
  int causal_offset;  // query i attends keys <= i + causal_offset (Sk - Sq for bottom-right alignment)
};

// 16-byte chunk swizzle of a [rows][D] bf16 LDS image (D/8 chunks per row).
template <int D>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (D == 128) {
    return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  } else {
    return ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
  }
}

template <int D>
__device__ __forceinline__ int lds_off(int row, int ch) {  // byte offset of a 16-B chunk
  return row * (D * 2) + swz<D>(row, ch) * 16;
}

template <int D>
__global__ void __launch_bounds__(kThreads, 2) fwd_kernel(FwdParams p) {
  constexpr int CH = D / 8;                       // 16-B chunks per row
  constexpr int KS = D / 16;                      // k-steps of the QK^T product
  constexpr int NDB = D / 32;                     // 32-wide d blocks of O
  constexpr int TILE_BYTES = kBlockN * D * 2;     // one K (or V) tile

  extern __shared__ __attribute__((aligned(16))) char smem[];
  // layout: [buf0: K | V][buf1: K | V]

  const int nblk_m = (p.Sq + kBlockM - 1) / kBlockM;
  const int nwg = gridDim.x;
  const int L = xcd_remap(blockIdx.x, nwg);
  const int bh = L % (p.B * p.Hq);
  const int mblk = nblk_m - 1 - L / (p.B * p.Hq);  // heavy (late) causal blocks first
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int qb0 = mblk * kBlockM;
  const int q0 = qb0 + w * 32;  // this wave's first row
  const int my_q = q0 + r;

  const uint16_t* qbase = p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const uint16_t* kbase = p.k + (int64_t)b * p.k_sb + (int64_t)hkv * p.k_sh;
  const uint16_t* vbase = p.v + (int64_t)b * p.v_sb + (int64_t)hkv * p.v_sh;

  // ---- Q fragments (B operand of S^T = K Q^T): lane (r, hh) holds Q[q0+r][16s + 8hh .. +7]
  bf16x8_t qf[KS];
  {
    const bool ok = my_q < p.Sq;
    const uint16_t* qrow = qbase + (int64_t)(ok ? my_q : 0) * p.q_ss;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = ok ? *reinterpret_cast<const u32x4_t*>(qrow + 16 * s + 8 * hh) : u32x4_t{0, 0, 0, 0};
      qf[s] = __builtin_bit_cast(bf16x8_t, v);
    }
  }

  // ---- key range
  int kend = p.Sk;
  if (p.causal) kend = min(p.Sk, qb0 + kBlockM + p.causal_offset);
  const int ntiles = kend > 0 ? (kend + kBlockN - 1) / kBlockN : 0;
  const int wave_qmax = q0 + 31 + p.causal_offset;  // last key any row of this wave may see
  const int wave_qmin = q0 + p.causal_offset;

  f32x16_t acc_o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) acc_o[i] = f32x16_t{0};
  float m_i = -INFINITY, l_i = 0.f;

  // K/V tiles go global -> LDS directly (global_load_lds_dwordx4, 1 KiB per wave-instruction).
  // The LDS image is lane-linear per instruction, so the XOR swizzle is applied to the per-lane
  // SOURCE address (cdna_hip_programming.md rule 21): LDS slot (row, c) receives logical chunk
  // swz(row, c) (the swizzle is an involution).  Out-of-range keys re-read the last valid row;
  // their scores are masked to -inf so they contribute p = 0.
  constexpr int ROWS_PER_PIECE = 1024 / (2 * D);
  constexpr int PIECES_PER_WAVE = TILE_BYTES / 1024 / kWaves;
  auto issue_tile = [&](int t, int buf) {
    char* kl = smem + buf * 2 * TILE_BYTES;
    char* vl = kl + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < PIECES_PER_WAVE; ++i) {
      const int piece = w * PIECES_PER_WAVE + i;
      const int row = piece * ROWS_PER_PIECE + lane / CH;
      const int ch = swz<D>(row, lane % CH);
      const int key = min(t * kBlockN + row, p.Sk - 1);
      const uint16_t* ks = kbase + (int64_t)key * p.k_ss + ch * 8;
      const uint16_t* vs = vbase + (int64_t)key * p.v_ss + ch * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ks,
                                       (__attribute__((address_space(3))) void*)(kl + piece * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)vs,
                                       (__attribute__((address_space(3))) void*)(vl + piece * 1024), 16, 0, 0);
    }
  };

  if (ntiles > 0) issue_tile(0, 0);
  __syncthreads();  // drains the LDS-DMA (vmcnt(0)) before any wave reads buffer 0

  // per-lane constant parts of the V transposed-read address (T10):
  // group g = lane>>4 covers rows (4 consecutive keys) x 16 columns; lane 4q+pp of the group
  // supplies row q, columns 4pp..4pp+3 of that block.
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int g = lane >> 4;

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    // buffer buf^1 was last read in iteration t-1, which every wave finished before the
    // barrier that closed it: safe to refill now, overlapped with this tile's MFMAs.
    if (t + 1 < ntiles) issue_tile(t + 1, buf ^ 1);

    const int kt0 = t * kBlockN;
    const bool wave_active = kt0 <= wave_qmax || !p.causal;
    if (wave_active) {
      const char* kl = smem + buf * 2 * TILE_BYTES;
      const char* vl = kl + TILE_BYTES;
      // ---- S^T for the two 32-key subtiles
      f32x16_t sacc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sacc[j] = f32x16_t{0};
        const int row = 32 * j + r;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const u32x4_t kv = *reinterpret_cast<const u32x4_t*>(kl + lds_off<D>(row, 2 * s + hh));
          sacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kv), qf[s], sacc[j], 0, 0, 0);
        }
      }
      // ---- mask + tile max on the RAW scores (scale > 0 commutes with max); the scale is folded
      // into one FMA per score below: p = exp2(s * c - m*c)
      const bool need_mask = (kt0 + kBlockN > p.Sk) || (p.causal && kt0 + kBlockN - 1 > wave_qmin);
      float tmax = -INFINITY;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float x = sacc[j][e];
          if (need_mask) {
            const int key = kt0 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * hh;
            const bool bad = key >= p.Sk || (p.causal && key > my_q + p.causal_offset);
            x = bad ? -INFINITY : x;
            sacc[j][e] = x;
          }
          tmax = fmaxf(tmax, x);
        }
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * p.scale_log2;
      // deferred rescale (T13): keep the running max stale while the tile max exceeds it by less
      // than kRescaleThreshold (log2 units); p then stays below 2^threshold, fine in fp32 / bf16,
      // and the 4*NDB*16 accumulator multiplies are skipped on most tiles.
      constexpr float kRescaleThreshold = 8.f;
      if (tmax > m_i + kRescaleThreshold || m_i == -INFINITY) {
        const float m_new = fmaxf(m_i, tmax);
        const float alpha = (m_i == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_i - m_new);
        m_i = m_new;
        l_i *= alpha;
#pragma unroll
        for (int db = 0; db < NDB; ++db) acc_o[db] *= alpha;
      }
      const float m_use = m_i == -INFINITY ? 0.f : m_i;
      float rsum = 0.f;
      bf16x8_t pf[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[j][8 * s2 + e], p.scale_log2, -m_use));
            rsum += pv;
            pf[j][s2][e] = (__bf16)pv;
          }
        }
      }
      rsum += __shfl_xor(rsum, 32, 64);
      l_i += rsum;

      // ---- O^T += V^T P
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int R0 = 32 * j + 16 * s2 + 4 * hh;  // this lane-half's first key of the k-step
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const int col = 32 * db + 16 * (g & 1) + 4 * tp;
            const int ch = col >> 3, sub = (col & 7) * 2;
            const int ra = R0 + tq, rb = R0 + 8 + tq;
            typedef __attribute__((address_space(3))) short4_t* lds_s4;
            const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s4)(vl + lds_off<D>(ra, ch) + sub));
            const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s4)(vl + lds_off<D>(rb, ch) + sub));
            const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            acc_o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), pf[j][s2], acc_o[db], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // vmcnt(0) + barrier: tile t+1 has landed for every wave
  }

  // ---- epilogue: O[q][d] = acc / l ; lse
  if (my_q < p.Sq) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    uint16_t* orow = p.o + (int64_t)b * p.o_sb + (int64_t)my_q * p.o_ss + (int64_t)hq * p.o_sh;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = 32 * db + 8 * gq + 4 * hh;
        u32x2_t v;
        v[0] = pack2bf(acc_o[db][4 * gq + 0] * inv, acc_o[db][4 * gq + 1] * inv);
        v[1] = pack2bf(acc_o[db][4 * gq + 2] * inv, acc_o[db][4 * gq + 3] * inv);
        *reinterpret_cast<u32x2_t*>(orow + d) = v;
      }
    }
    if (hh == 0 && p.lse) {
      const float lse = l_i > 0.f ? (m_i + __log2f(l_i)) * 0.69314718055994531f : -INFINITY;
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + my_q] = lse;
    }
  }
}

}  // namespace fa

int flash_attn_fwd_launch(const void* q, const void* k, const void* v, void* o, float* lse,
                          const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os,
                          int B, int Sq, int Sk, int Hq, int Hkv, int D, float softmax_scale,
                          int causal, int causal_offset, hipStream_t stream) {
  using namespace fa;
  FwdParams p;
  p.q = (const uint16_t*)q;
  p.k = (const uint16_t*)k;
  p.v = (const uint16_t*)v;
  p.o = (uint16_t*)o;
  p.lse = lse;
  p.q_sb = qs[0]; p.q_ss = qs[1]; p.q_sh = qs[2];
  p.k_sb = ks[0]; p.k_ss = ks[1]; p.k_sh = ks[2];
  p.v_sb = vs[0]; p.v_ss = vs[1]; p.v_sh = vs[2];
  p.o_sb = os[0]; p.o_ss = os[1]; p.o_sh = os[2];
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale_log2 = softmax_scale * 1.4426950408889634f;
  p.causal = causal;
  p.causal_offset = causal_offset;
  if (Hkv <= 0 || Hq % Hkv != 0) return -1;
  const int nblk = (Sq + kBlockM - 1) / kBlockM;
  const int grid = nblk * B * Hq;
  if (grid == 0) return 0;
  if (D == 128) {
    const size_t lds = 2 * 2 * kBlockN * 128 * 2;
    hipLaunchKernelGGL(fwd_kernel<128>, dim3(grid), dim3(kThreads), lds, stream, p);
  } else if (D == 64) {
    const size_t lds = 2 * 2 * kBlockN * 64 * 2;
    hipLaunchKernelGGL(fwd_kernel<64>, dim3(grid), dim3(kThreads), lds, stream, p);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

}  // namespace nxd
