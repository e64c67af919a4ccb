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

#include <cstdlib>
#include <type_traits>

namespace nxd {
namespace fa {

// W waves per workgroup (W * 32 query rows share each K/V tile): 4 (two workgroups per CU) or 8
// (one 256-row block per workgroup: half the K/V tile traffic and barriers per query row).
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
  DropoutArgs drop;   // DROP variants only
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

typedef __attribute__((address_space(3))) char lds_char_t;
__device__ __forceinline__ uint32_t lds_addr(const char* ptr) { return (uint32_t)(uintptr_t)(const lds_char_t*)ptr; }

// ds_read_b64_tr_b16 as inline asm: the builtin form makes the compiler put an s_waitcnt vmcnt(0)
// (it cannot tell the read from the in-flight LDS-DMA of the next tile) in front of the first V
// read, which serialises the prefetch with P.V.  The other buffer is being filled; this one was
// completed by the previous barrier.  Results are valid only after tr_wait<N>.
__device__ __forceinline__ short4_t tr_read(uint32_t a) {
  short4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
template <int OFF>
__device__ __forceinline__ short4_t tr_read_off(uint32_t a) {   // + an immediate byte offset
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  short4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}
template <int N>
__device__ __forceinline__ void tr_wait(short4_t (&v)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
               : "n"(N));
}

// lane l <-> l ^ 32 combine by v_permlane32_swap (VALU; the ds_bpermute of __shfl_xor would make
// the compiler wait lgkmcnt(0) on the V reads already in flight) -> max (is_max) or sum of the pair.
__device__ __forceinline__ float xor32(float x, bool is_max) {
  const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float a = __uint_as_float(pr[0]), b = __uint_as_float(pr[1]);
  return is_max ? fmaxf(a, b) : a + b;
}

// Double-buffered LDS ring of 64-key tiles: tile t + 1 is DMA'd while tile t is computed.
// DROP: dropout on the probabilities (reference NKI flash_fwd dropout_p / seed): the row sum l and
// the LSE use the undropped P, the P.V operand is P * keep / (1 - p); the lane's query row hash is
// computed once, each score costs one more hash.
template <int D, int W, bool DROP>
__global__ void __launch_bounds__(W * 64, 8 / W) fwd_kernel(FwdParams p) {
  constexpr int kWaves = W;
  constexpr int kBlockM = W * 32;                 // q rows per workgroup
  constexpr int CH = D / 8;                       // 16-B chunks per row
  constexpr int KS = D / 16;                      // k-steps of the QK^T product
  constexpr int NDB = D / 32;                     // 32-wide d blocks of O
  constexpr int TILE_BYTES = kBlockN * D * 2;     // one K (or V) LDS tile

  extern __shared__ __attribute__((aligned(16))) char smem[];
  // layout: [buf0: K | V][buf1: K | V]

  // block -> (batch, q head, q block), interleaved over the XCDs: the dispatch order IS the
  // heavy-first causal order and consecutive blocks land on different XCDs, so every XCD gets the
  // same mix of block sizes (profiles/r2_fa_xcd_map_ab.jsonl: faster than contiguous ranges per XCD
  // or kv-head-per-XCD maps at the TP=1 and TP=8 shapes)
  const int nblk_m = (p.Sq + kBlockM - 1) / kBlockM;
  const int bh = blockIdx.x % (p.B * p.Hq);
  const int mblk = nblk_m - 1 - blockIdx.x / (p.B * p.Hq);
  const int b = bh / p.Hq;
  const int hq = bh % p.Hq;
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
  uint32_t drow = 0;
  if constexpr (DROP) drow = drop_row_hash(p.drop.seed, b, hq + p.drop.head_offset, my_q);

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
  // static priority for the younger half of an 8-wave workgroup (MI355X_MICROARCH "Two waves per
  // SIMD" item 4); the condition is wave-uniform through readfirstlane (T5 static form)
  if (kWaves == 8 && __builtin_amdgcn_readfirstlane(w) >= kWaves / 2) __builtin_amdgcn_s_setprio(1);
  __syncthreads();  // drains the LDS-DMA (vmcnt(0)) before any wave reads buffer 0

  // per-lane constant parts of the V transposed-read address (T10):
  // group g = lane>>4 covers rows (4 consecutive keys) x 16 columns; lane 4q+pp of the group
  // supplies row q, columns 4pp..4pp+3 of that block.
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int g = lane >> 4;
  // V transposed-read addresses without the tile part: row 32 j + 16 s2 + 4 hh + tq (+ 8) of
  // buffer buf is this per-lane base + the immediate buf * 2 * TILE + TILE + (32 j + 16 s2) * 2D
  // (the swizzle only sees row bits 0-3, which j and s2 do not touch)
  uint32_t vlane[NDB][2];
  {
    const uint32_t s0 = lds_addr(smem);
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const int col = 32 * db + 16 * (g & 1) + 4 * tp;
      const int ch = col >> 3, sub = (col & 7) * 2;
      vlane[db][0] = s0 + lds_off<D>(4 * hh + tq, ch) + sub;
      vlane[db][1] = s0 + lds_off<D>(4 * hh + 8 + tq, ch) + sub;
    }
  }

  // The tile loop is unrolled by the two LDS buffers: with the buffer a compile-time constant every
  // K / V read address is a loop-invariant per-lane offset plus an immediate (buffer, 32-key subtile,
  // 16-row P.V group), instead of a v_add_u32 per read on the tile's base.
  auto tile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    // buffer buf^1 was last read in iteration t-1, which every wave finished before the
    // barrier that closed it: safe to refill now, overlapped with this tile's MFMAs.
    if (t + 1 < ntiles) issue_tile(t + 1, buf ^ 1);

    {
      const int kt0 = t * kBlockN;
      const bool wave_active = kt0 <= wave_qmax || !p.causal;
      if (wave_active) {
        const char* kl = smem + buf * 2 * TILE_BYTES;
        // ---- S^T for the two 32-key subtiles
        f32x16_t sacc[2];
        sacc[0] = f32x16_t{0};
        sacc[1] = f32x16_t{0};
        {
          // K fragments one k-step ahead, both subtiles interleaved (two independent MFMA chains)
          u32x4_t kf[2][2];
          kf[0][0] = *reinterpret_cast<const u32x4_t*>(kl + lds_off<D>(r, hh));
          kf[0][1] = *reinterpret_cast<const u32x4_t*>(kl + lds_off<D>(32 + r, hh));
  #pragma unroll
          for (int s = 0; s < KS; ++s) {
            if (s + 1 < KS) {
              kf[(s + 1) & 1][0] = *reinterpret_cast<const u32x4_t*>(kl + lds_off<D>(r, 2 * (s + 1) + hh));
              kf[(s + 1) & 1][1] = *reinterpret_cast<const u32x4_t*>(kl + lds_off<D>(32 + r, 2 * (s + 1) + hh));
            }
            sacc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf[s & 1][0]), qf[s], sacc[0], 0, 0, 0);
            sacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf[s & 1][1]), qf[s], sacc[1], 0, 0, 0);
          }
        }
        // V reads of the first two P.V groups go out now, hidden behind the softmax VALU work
        short4_t va[8], vb2[8];
          // 4 groups (j, s2) of 8 transposed V reads (4 d-blocks x lo/hi); group g+1 is issued
          // before group g's MFMAs, a counted wait covers exactly group g
          auto issue = [&](auto grpc, short4_t (&v)[8]) {
            constexpr int grp = decltype(grpc)::value;
            constexpr int OFF = buf * 2 * TILE_BYTES + TILE_BYTES + (32 * (grp >> 1) + 16 * (grp & 1)) * D * 2;
  #pragma unroll
            for (int db = 0; db < NDB; ++db) {
              v[2 * db] = tr_read_off<OFF>(vlane[db][0]);
              v[2 * db + 1] = tr_read_off<OFF>(vlane[db][1]);
            }
          };
        static_assert(NDB <= 4, "group size is 8 reads");
        issue(std::integral_constant<int, 0>{}, va);
        issue(std::integral_constant<int, 1>{}, vb2);
        // ---- mask + tile max on the RAW scores (scale > 0 commutes with max); the scale is folded
        // into one FMA per score below: p = exp2(s * c - m*c)
        const bool need_mask = (kt0 + kBlockN > p.Sk) || (p.causal && kt0 + kBlockN - 1 > wave_qmin);
        float tmax = -INFINITY;
        {
          // branch-free select against one per-lane limit: key offset c inside the tile is masked
          // iff c > lim (one compare + select per score, only on tiles that need a mask)
          if (need_mask) {
            const int lim = (p.causal ? min(my_q + p.causal_offset, p.Sk - 1) : p.Sk - 1) - kt0 - 4 * hh;
  #pragma unroll
            for (int j = 0; j < 2; ++j)
  #pragma unroll
              for (int e = 0; e < 16; ++e) {
                const int c = 32 * j + (e & 3) + 8 * (e >> 2);
                sacc[j][e] = c > lim ? -INFINITY : sacc[j][e];
              }
          }
  #pragma unroll
          for (int j = 0; j < 2; ++j)
  #pragma unroll
            for (int e = 0; e < 16; ++e) tmax = fmaxf(tmax, sacc[j][e]);
        }
        tmax = fmaxf(tmax, xor32(tmax, true)) * p.scale_log2;
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
              if constexpr (DROP) {
                const int key = kt0 + 32 * j + (e & 3) + 8 * (2 * s2 + (e >> 2)) + 4 * hh;
                pf[j][s2][e] = (__bf16)(drop_keep(drow, key, p.drop.thresh) ? pv * p.drop.scale : 0.f);
              } else {
                pf[j][s2][e] = (__bf16)pv;
              }
            }
          }
        }
        rsum = xor32(rsum, false);
        l_i += rsum;

        // ---- O^T += V^T P
        {
          auto mma = [&](int grp, short4_t (&v)[8]) {
            const int j = grp >> 1, s2 = grp & 1;
  #pragma unroll
            for (int db = 0; db < NDB; ++db) {
              const short4_t lo = v[2 * db], hi = v[2 * db + 1];
              const short __attribute__((ext_vector_type(8))) a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
              acc_o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), pf[j][s2], acc_o[db], 0, 0, 0);
            }
          };
          tr_wait<2 * NDB>(va);
          mma(0, va);
          issue(std::integral_constant<int, 2>{}, va);
          tr_wait<2 * NDB>(vb2);
          mma(1, vb2);
          issue(std::integral_constant<int, 3>{}, vb2);
          tr_wait<2 * NDB>(va);
          mma(2, va);
          tr_wait<0>(vb2);
          mma(3, vb2);
        }
      }
    }
    __syncthreads();  // vmcnt(0) + barrier: tile t+1 has landed for every wave
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) tile(t + 1, std::integral_constant<int, 1>{});
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
                          int causal, int causal_offset, const DropoutArgs& drop, hipStream_t stream) {
  using namespace fa;
  FwdParams p{};
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
  p.drop = drop;
  if (Hkv <= 0 || Hq % Hkv != 0) return -1;
  if (D != 128 && D != 64) return -2;
  // 8-wave workgroups (256 query rows: half the K/V tile traffic and barriers per row) while the
  // 256-row grid still fills the chip, else 4 waves.  Measured at S=8192 D=128 causal, 32 / 4 heads
  // (profiles/r1_fa_fwd_variants.jsonl, profiles/r2_fa_xcd_map_ab.jsonl): this pipelined body
  // 574-587 / 406-417 TF/s before the XCD map, 955-966 TF/s with it; the non-pipelined body, per-
  // cluster s_setprio, a 3-stage LDS ring and 128-key tiles measured neutral or slower (removed).
  const bool w8 = ((Sq + 255) / 256) * B * Hq >= 512;
  const int rows = w8 ? 256 : 128;
  const int grid = ((Sq + rows - 1) / rows) * B * Hq;
  if (grid == 0) return 0;
  const size_t lds = 2 * 2 * kBlockN * D * 2;
#define NXD_FA_LAUNCH(DD, WW, DR) hipLaunchKernelGGL((fwd_kernel<DD, WW, DR>), dim3(grid), dim3(WW * 64), lds, stream, p)
  if (drop.enabled()) {
    if (D == 128) {
      if (w8) NXD_FA_LAUNCH(128, 8, true); else NXD_FA_LAUNCH(128, 4, true);
    } else {
      if (w8) NXD_FA_LAUNCH(64, 8, true); else NXD_FA_LAUNCH(64, 4, true);
    }
  } else if (D == 128) {
    if (w8) NXD_FA_LAUNCH(128, 8, false); else NXD_FA_LAUNCH(128, 4, false);
  } else {
    if (w8) NXD_FA_LAUNCH(64, 8, false); else NXD_FA_LAUNCH(64, 4, false);
  }
#undef NXD_FA_LAUNCH
  return (int)hipGetLastError();
}

}  // namespace nxd
