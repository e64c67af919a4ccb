// FlashAttention-2 backward for CDNA4 (gfx950): dQ, dK, dV from Q, K, V, dO, LSE.
// Replaces the reference's NKI `flash_attn_bwd` (src/neuronx_distributed/kernels/flash_attn.py:61-82,130-148).
//
// Structure (cdna_hip_programming.md, "Attention backward"):
//   * a key block = 256 keys of one (batch, kv-head); a workgroup = 4 waves, each wave owns 64
//     keys (two 32-key MFMA columns) and keeps their dK / dV in 256 accumulator registers while
//     it sweeps a CHUNK of the block's (q head of the GQA group x 32-row query tile) iteration
//     space.  GQA reduction of dK/dV happens in registers — no repeat_kv, no second pass.
//   * Work items = (key block, chunk): the host sizes chunks so there are >= 2 items per CU even
//     at TP=8 head counts (one kv head per GPU), and the causal triangle is cut into near-equal
//     pieces instead of one workgroup per key block whose runtime is the longest sweep.  Items
//     of one key block write their dK/dV partials (256 KiB per item) with plain stores into
//     per-item slabs that the bf16 convert pass sums (f32 atomics into one accumulator: knob 5).
//   * "key on the lane": S = Q K^T and dP = dO V^T put the key on the MFMA column, so their
//     fp32 accumulators convert in place into the A operands of dV += P^T dO and dK += dS^T Q
//     (accumulator-as-operand: no LDS round trip for P / dS), and the dV / dK accumulators come
//     out [key][d] with d on the lane — the full-rate shape for the f32 atomics (two 128-B row
//     segments per wave-instruction).
//   * row constants as initial accumulators: S starts at -LSE/scale and dP at -delta, so
//     P = exp2(scale*log2e * S) and dS = P * dP need no per-element subtraction;
//   * K of the block lives in LDS (row reads for S, transposed reads for dQ); V rows live in
//     VGPRs; Q / dO tiles arrive by LDS-DMA one tile ahead into a double-buffered swizzled image
//     that serves both row reads (ds_read_b128) and transposed reads (ds_read_b64_tr_b16).
//   * dQ: dS^T crosses LDS once; each wave computes one 32-wide d block of dS . K over the
//     block's 256 keys (D=128; D=64 splits keys in halves and sums the halves in LDS) and adds
//     it with f32 atomics into an fp32 dQ accumulator.  At 256 keys per block the atomic volume
//     is one byte per 640 FLOPs (half of a 128-key design).  At S=8192, 32/8 heads that is 2.21 GB
//     of dQ adds + 0.55 GB of dK/dV adds; at the chip-wide f32 atomic rate (~1.3 TB/s, any adder
//     placement) that alone is ~2.1 ms, the kernel's time (profiles/r2_fab_ablate_after.jsonl: the
//     body with every atomic ablated runs 1.59 ms).  Going lower needs fewer atomic BYTES, not a
//     faster body: 256 keys per workgroup is the register-file maximum for resident dK/dV
//     (256 keys x 128 d x 2 x 4 B = half of a CU's 512 KiB of registers).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <queue>
#include <tuple>
#include <type_traits>
#include <vector>

namespace nxd {
namespace fab {

constexpr int kWaves = 4;
constexpr int kThreads = 256;
constexpr int kBlockK = 256;  // keys per key block (64 per wave)
constexpr int kBlockQ = 32;   // query rows per tile
constexpr int kPipeDq = 3;    // dQ operand reads ahead (one MFMA per step)

struct BwdParams {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  const uint16_t* dout;
  const float* nlse;    // [B, Hq, Sq]: -LSE / scale  (-inf for empty rows)
  const float* ndelta;  // [B, Hq, Sq]: -rowsum(dO * O)
  float* dq_acc;        // [B, Hq, Sq_pad, D] fp32, zero-initialised
  float* dk_acc;        // [B, Hkv, Sk_pad, D] fp32, zero-initialised
  float* dv_acc;        // [B, Hkv, Sk_pad, D] fp32, zero-initialised
  float* dk_slab;       // slab mode (non-null): [B*Hkv, items per bh, kBlockK, D] fp32 per-item partials,
  float* dv_slab;       //   plain stores (no atomics), summed by slab_convert_kernel
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t do_sb, do_ss, do_sh;
  int B, Sq, Sk, Hq, Hkv;
  float scale_log2;  // softmax scale * log2(e)
  int causal;
  int causal_offset;
  int chunk;   // max (q head, q tile) iterations per work item
  int xcd_map; // 0: contiguous item ranges per XCD, 2: interleaved (see bwd_kernel)
  int ablate;  // timing-only ablations (NXD_FAB_ABLATE; outputs wrong): 1 no dQ atomics,
               // 2 no dK/dV atomics, 16 no Q/dO tile loads,
               // 32 no per-tile barriers
  DropoutArgs drop;  // DROP variants only
};

// (q head x q tile) iterations of key block kb
__host__ __device__ inline int kb_iters(int kb, int Sq, int G, int causal, int off) {
  int qstart = 0;
  if (causal) qstart = kb * kBlockK - off > 0 ? kb * kBlockK - off : 0;
  qstart = (qstart / kBlockQ) * kBlockQ;
  const int n_qt = qstart < Sq ? (Sq - qstart + kBlockQ - 1) / kBlockQ : 0;
  return G * n_qt;
}

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

// dS^T image: [256 keys][32 q] bf16, 64-B rows, 8-B chunks XOR-swizzled by (row & 7)
__device__ __forceinline__ int ds_off(int key, int q) { return key * 64 + (((q >> 2) ^ (key & 7)) << 3) + (q & 3) * 2; }

typedef short bf16s8_t __attribute__((ext_vector_type(8)));

// LDS access through a plain 32-bit byte address (the extern LDS symbol's address is folded
// into the per-lane base registers once, so `base + constant` becomes the ds_* immediate offset
// instead of a v_add per access).
typedef __attribute__((address_space(3))) char lds_char_t;
__device__ __forceinline__ uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)(const lds_char_t*)p; }
template <typename T>
__device__ __forceinline__ T lds_ld(uint32_t a) {
  return *(const __attribute__((address_space(3))) T*)(uintptr_t)a;
}
template <typename T>
__device__ __forceinline__ void lds_st(uint32_t a, const T& v) {
  *(__attribute__((address_space(3))) T*)(uintptr_t)a = v;
}
__device__ __forceinline__ short4_t lds_tr(uint32_t a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(uintptr_t)a);
}

// acc += A * B with the accumulator pinned to AGPRs.  The 256 resident dK/dV accumulators must
// live in the AGPR file and every short-lived MFMA chain (S, dP, dQ) in VGPRs; hipcc's allocator
// does not find that split by itself (it either spills two accumulator tiles every tile, or —
// with -amdgpu-mfma-vgpr-form — puts the accumulators in VGPRs and parks addresses in AGPRs).
// The asm is invisible to the hazard recognizer, so it carries the one wait it needs itself: a
// VALU write of a VGPR read as SrcA/SrcB by an MFMA needs 2 wait states (hipcc emits the same
// `s_nop 1` for the builtin form); SrcC/vDst are AGPRs no VALU touches inside the loop, and the
// epilogue waits out the last MFMAs before reading them.
template <typename TA, typename TB>
__device__ __forceinline__ void mfma_acc_agpr(f32x16_t& acc, const TA& a, const TB& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// PIPE: S / dP operand reads issued this many steps ahead of their MFMAs; PIPE_DVDK: the same for
// the dV / dK transposed reads (the first ones go out before the softmax VALU).
// DROP: attention dropout (reference NKI flash_attn_bwd dropout_p / seed): the forward's keep mask m
// (0 or 1/(1-p)) is regenerated from the hash; dV uses P*m, dS = P * (m * dO.V^T - delta), so dP
// starts at 0 instead of -delta and delta is re-read from the tile's LDS row constants.
template <int D, int PIPE, int PIPE_DVDK, bool DROP>
__global__ void __launch_bounds__(kThreads, 1) bwd_kernel(BwdParams p) {
  constexpr int kPipe = PIPE;
  constexpr int CH = D / 8;
  constexpr int KS = D / 16;
  constexpr int NDB = D / 32;
  constexpr int KV_BYTES = kBlockK * D * 2;
  constexpr int QT_BYTES = kBlockQ * D * 2;
  constexpr int OFF_K = 0;                            // K block image
  constexpr int OFF_Q = KV_BYTES;                     // 2 buffers
  constexpr int OFF_DO = OFF_Q + 2 * QT_BYTES;        // 2 buffers
  constexpr int OFF_DS = OFF_DO + 2 * QT_BYTES;       // 256 x 64 B
  constexpr int OFF_LD = OFF_DS + kBlockK * 64;       // 2 buffers x (32 nlse + 32 ndelta) floats
  constexpr int OFF_RED = OFF_LD + 512;               // D=64: dQ key-half partials (2 x 4 KiB)
  constexpr int OFF_V = OFF_RED + (NDB == 2 ? 8192 : 0);  // V rows of every wave's 2nd key column
  constexpr int ROWS_PER_PIECE = 1024 / (2 * D);
  constexpr int QT_PIECES = QT_BYTES / 1024;
  constexpr int QT_PIECES_PER_WAVE = QT_PIECES / kWaves;
  constexpr int KEY_SPLIT = kWaves / NDB;             // 1 (D=128) or 2 (D=64)
  constexpr int KEYS_PER_DQ = kBlockK / KEY_SPLIT;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int G = p.Hq / p.Hkv;
  const int BH = p.B * p.Hkv;
  // work-item order = dispatch order (xcd_map 2: consecutive items on different XCDs, so every XCD
  // gets the same mix of heavy and light items) or contiguous item ranges per XCD (0, round 1: the
  // first XCD received all of the heaviest key blocks' items)
  const int L = p.xcd_map == 2 ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int bh = L % BH;
  int kc = L / BH;
  const int64_t slab = (int64_t)bh * (gridDim.x / BH) + kc;  // this item's dK/dV slab (slab mode)
  // ---- decode (key block, chunk) of this work item: key blocks in order (heaviest first)
  const int nkb = (p.Sk + kBlockK - 1) / kBlockK;
  int kb = 0, it_begin = 0, it_end = 0;
  for (; kb < nkb; ++kb) {
    const int n_it = kb_iters(kb, p.Sq, G, p.causal, p.causal_offset);
    const int nc = (n_it + p.chunk - 1) / p.chunk;
    if (kc < nc) {
      const int per = (n_it + nc - 1) / nc;
      it_begin = kc * per;
      it_end = min(n_it, it_begin + per);
      break;
    }
    kc -= nc;
  }
  if (kb >= nkb || it_begin >= it_end) {  // (host sizes the grid exactly; defensive)
    if (p.dk_slab != nullptr) {  // an empty item's slab still enters the sum
      for (int i = threadIdx.x; i < kBlockK * D; i += kThreads) {
        p.dk_slab[slab * kBlockK * D + i] = 0.f;
        p.dv_slab[slab * kBlockK * D + i] = 0.f;
      }
    }
    return;
  }

  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int Sq_pad = (p.Sq + kBlockQ - 1) / kBlockQ * kBlockQ;
  const int Sk_pad = nkb * kBlockK;
  int qstart = 0;
  if (p.causal) qstart = max(0, kb * kBlockK - p.causal_offset);
  qstart = (qstart / kBlockQ) * kBlockQ;
  const int n_qt = (p.Sq - qstart + kBlockQ - 1) / kBlockQ;

  // (w stays a VGPR value: made scalar, its uniform branches split the tile body into blocks and
  // the allocator spills the V rows)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3, g = lane >> 4;

  const uint16_t* kbase = p.k + (int64_t)b * p.k_sb + (int64_t)hkv * p.k_sh;
  const uint16_t* vbase = p.v + (int64_t)b * p.v_sb + (int64_t)hkv * p.v_sh;
  const int kb0 = kb * kBlockK;
  const int wkey0 = kb0 + 64 * w;  // this wave's first key

  // ---- K block -> LDS; this wave's V rows -> registers (B operands of dP)
  for (int idx = tid; idx < kBlockK * CH; idx += kThreads) {
    const int row = idx / CH, ch = idx % CH;
    const int key = kb0 + row;
    u32x4_t kv4 = {0, 0, 0, 0};
    if (key < p.Sk) kv4 = *reinterpret_cast<const u32x4_t*>(kbase + (int64_t)key * p.k_ss + ch * 8);
    *reinterpret_cast<u32x4_t*>(smem + OFF_K + lds_off<D>(row, ch)) = kv4;
  }
  // V rows: first key column in VGPRs, second in an LDS image (the 256 dK/dV accumulators
  // leave room for only one column of V in registers)
  bf16x8_t vf[KS];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int key = wkey0 + 32 * c + r;
    const bool ok = key < p.Sk;
    const uint16_t* vr = vbase + (int64_t)(ok ? key : 0) * p.v_ss;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const u32x4_t cv = ok ? *reinterpret_cast<const u32x4_t*>(vr + 16 * s + 8 * hh) : u32x4_t{0, 0, 0, 0};
      if (c == 0)
        vf[s] = __builtin_bit_cast(bf16x8_t, cv);
      else
        *reinterpret_cast<u32x4_t*>(smem + OFF_V + lds_off<D>(32 * w + r, 2 * s + hh)) = cv;
    }
  }

  // ---- per-lane LDS byte offsets, computed ONCE (every in-loop LDS access is one of these plus a
  // compile-time constant, so the loop spends no VALU on swizzled address math).  They hold
  // because every image's swizzle depends only on row & 15 (key/query images) or key & 7 (dS^T),
  // and all per-step row strides are multiples of 16 / 8.
  const int dbq = w % NDB;                 // dQ: this wave's 32-wide d block (wave-uniform)
  const int kr0 = (w / NDB) * KEYS_PER_DQ; // dQ: this wave's first key of the block
  // (image bases are folded into the registers: ds_read immediates are 16-bit)
  const uint32_t L0 = lds_addr(smem);
  // row reads of q/dO row r, K row 64w+r, V row 32w+r all use a_q (the dO image is a constant
  // away; K / V a wave-uniform SGPR away, added per read so the registers are not replicated)
  uint32_t a_q[KS];
  uint32_t a_trq[2][NDB];                  // tr reads rows 4hh+tq+8j, col 32dbk+16(g&1)+4tp (Q; dO +const)
  const uint32_t kofs0 = __builtin_amdgcn_readfirstlane((uint32_t)(OFF_K - OFF_Q + 64 * w * (2 * D)));
  const uint32_t vofs0 = __builtin_amdgcn_readfirstlane((uint32_t)(OFF_V - OFF_Q + 32 * w * (2 * D)));
  constexpr int DO_Q = OFF_DO - OFF_Q;
  uint32_t a_dsw[4];                       // dS^T writes: key 64w+r, q 8gq+4hh
  uint32_t a_dsr[2], a_ktr[2];             // dQ tr reads: dS^T keys kr0+8hh+tq+4j / K rows
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int a_row = lds_off<D>(r, 2 * s + hh);
    a_q[s] = L0 + OFF_Q + a_row;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dbk = 0; dbk < NDB; ++dbk) {
      const int col = 32 * dbk + 16 * (g & 1) + 4 * tp;
      const int a_tr = lds_off<D>(4 * hh + tq + 8 * j, col >> 3) + (col & 7) * 2;
      a_trq[j][dbk] = L0 + OFF_Q + a_tr;
    }
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) a_dsw[gq] = L0 + OFF_DS + 64 * w * 64 + ds_off(r, 8 * gq + 4 * hh);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    a_dsr[j] = L0 + OFF_DS + kr0 * 64 + ds_off(8 * hh + tq + 4 * j, 16 * (g & 1) + 4 * tp);
    const int col = 32 * dbq + 16 * (g & 1) + 4 * tp;
    a_ktr[j] = L0 + OFF_K + kr0 * (2 * D) + lds_off<D>(8 * hh + tq + 4 * j, col >> 3) + (col & 7) * 2;
  }
  uint32_t a_ld = L0 + OFF_LD + 16 * hh;  // nlse / ndelta rows 8gq + 4hh
  // opaque: otherwise the compiler re-splits each base into (lane part + big constant) and puts the
  // v_add back into the loop (the big constants do not fit the 16-bit ds offset)
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    asm volatile("" : "+v"(a_q[s]));
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int dbk = 0; dbk < NDB; ++dbk) asm volatile("" : "+v"(a_trq[j][dbk]));
    asm volatile("" : "+v"(a_dsr[j]), "+v"(a_ktr[j]));
  }
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) asm volatile("" : "+v"(a_dsw[gq]));
  asm volatile("" : "+v"(a_ld));
  // per-lane global offsets of the Q / dO tile pieces this lane copies (tile-invariant)
  int q_lane[QT_PIECES_PER_WAVE], do_lane[QT_PIECES_PER_WAVE], row_lane[QT_PIECES_PER_WAVE];
#pragma unroll
  for (int i = 0; i < QT_PIECES_PER_WAVE; ++i) {
    const int piece = w * QT_PIECES_PER_WAVE + i;
    const int row = piece * ROWS_PER_PIECE + lane / CH;
    const int ch = swz<D>(row, lane % CH);
    row_lane[i] = row;
    q_lane[i] = row * (int)p.q_ss + ch * 8;
    do_lane[i] = row * (int)p.do_ss + ch * 8;
  }

  // Q / dO tile + row constants -> LDS by LDS-DMA (global_load_lds), one tile ahead into the other
  // buffer.  Issued from inline asm: when the compiler sees an LDS-DMA in flight it waits for it
  // (vmcnt(0)) before every transposed LDS read, which exposed the whole prefetch once per tile.
  // Completion is tracked by hand (the counted vmcnt wait at the end of each tile).  M0 carries the
  // wave-uniform LDS destination and is restored after the issue.
  auto dma16 = [&](const void* src, uint32_t lds_dst) {
    uint32_t sv;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(sv) : "v"(src), "s"(lds_dst) : "memory");
  };
  auto dma4 = [&](const void* src, uint32_t lds_dst) {
    uint32_t sv;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(sv) : "v"(src), "s"(lds_dst) : "memory");
  };
  auto issue_tile = [&](int it, int buf) {
    const int hq = hkv * G + it / n_qt;
    const int qt0 = qstart + (it % n_qt) * kBlockQ;
    const uint16_t* qb = p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh + (int64_t)qt0 * p.q_ss;
    const uint16_t* db = p.dout + (int64_t)b * p.do_sb + (int64_t)hq * p.do_sh + (int64_t)qt0 * p.do_ss;
    const bool tail = qt0 + kBlockQ > p.Sq;  // wave-uniform
#pragma unroll
    for (int i = 0; i < QT_PIECES_PER_WAVE; ++i) {
      const int piece = w * QT_PIECES_PER_WAVE + i;
      int qo = q_lane[i], dof = do_lane[i];
      if (tail) {  // clamp rows past the end of the sequence (masked later)
        const int rr = min(row_lane[i], p.Sq - 1 - qt0);
        const int ch = swz<D>(row_lane[i], lane % CH);
        qo = rr * (int)p.q_ss + ch * 8;
        dof = rr * (int)p.do_ss + ch * 8;
      }
      dma16(qb + qo, __builtin_amdgcn_readfirstlane(L0 + OFF_Q + buf * QT_BYTES + piece * 1024));
      dma16(db + dof, __builtin_amdgcn_readfirstlane(L0 + OFF_DO + buf * QT_BYTES + piece * 1024));
    }
    if (w == 0) {
      const int qi = min(qt0 + (lane & 31), p.Sq - 1);
      const float* src = (lane < 32 ? p.nlse : p.ndelta) + ((int64_t)b * p.Hq + hq) * p.Sq + qi;
      dma4(src, __builtin_amdgcn_readfirstlane(L0 + OFF_LD + buf * 256));
    }
  };

  f32x16_t acc_dk[2][NDB], acc_dv[2][NDB];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < NDB; ++i) {
      acc_dk[c][i] = f32x16_t{0};
      acc_dv[c][i] = f32x16_t{0};
    }
  bool touched[2] = {false, false};

  issue_tile(it_begin, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // K / V images + first tile visible

  // one tile; BUF (0/1) is a compile-time constant so every LDS offset folds into the instruction
  auto tile = [&](auto BUFC, int it) {
    constexpr int buf = decltype(BUFC)::value;
    constexpr int QB = buf * QT_BYTES, DB = buf * QT_BYTES, LB = buf * 256;  // offsets from the per-lane bases
    const int hq = hkv * G + it / n_qt;
    const int qt0 = qstart + (it % n_qt) * kBlockQ;
    // buffer buf^1 was last read in the previous tile, closed by its final barrier
    if (it + 1 < it_end && !(p.ablate & 16)) issue_tile(it + 1, buf ^ 1);
    uint32_t kofs = kofs0, vofs = vofs0;
    asm volatile("" : "+s"(kofs), "+s"(vofs));  // per tile: the adds stay next to their reads
    const int qlast = qt0 + kBlockQ - 1 + p.causal_offset;  // last key any row of the tile may see

#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kc0 = wkey0 + 32 * c;
      // no branch on the causal diagonal: a fully masked column computes P = dS = 0 (the tile's
      // time is set by wave 0, whose columns are never fully masked), and a branch around MFMAs
      // would need to be a uniform jump -- an MFMA ignores EXEC
      touched[c] = touched[c] || !p.causal || kc0 <= qlast;
      {
        // ---- S = Q K^T - LSE/scale, dP = dO V^T - delta  (key on the lane; row constants as
        // the initial accumulators)
        f32x16_t s_acc, dp_acc;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const f32x4_t l4 = lds_ld<f32x4_t>(a_ld + LB + 32 * gq);
          const f32x4_t d4 = lds_ld<f32x4_t>(a_ld + LB + 128 + 32 * gq);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            s_acc[4 * gq + i] = l4[i];
            dp_acc[4 * gq + i] = DROP ? 0.f : d4[i];
          }
        }
        // operands of step s are read kPipe steps ahead of its MFMAs (explicit software pipeline:
        // each step is fenced for the scheduler, so a read is never sunk next to its consumer and
        // the MFMAs wait only for their own operands -- lgkmcnt(N), not lgkmcnt(0))
        u32x4_t qa[KS], kk[KS], da[KS];
        bf16x8_t vb[KS];
        auto ld_sdp = [&](int s) {
          qa[s] = lds_ld<u32x4_t>(a_q[s] + QB);
          kk[s] = lds_ld<u32x4_t>(a_q[s] + kofs + c * 32 * (2 * D));
          da[s] = lds_ld<u32x4_t>(a_q[s] + DO_Q + DB);
          if (c == 0)
            vb[s] = vf[s];
          else
            vb[s] = __builtin_bit_cast(bf16x8_t, lds_ld<u32x4_t>(a_q[s] + vofs));
        };
#pragma unroll
        for (int s = 0; s < kPipe; ++s) ld_sdp(s);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (s + kPipe < KS) ld_sdp(s + kPipe);
          s_acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, qa[s]), __builtin_bit_cast(bf16x8_t, kk[s]), s_acc, 0, 0, 0);
          dp_acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, da[s]), vb[s], dp_acc, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
        // first dV / dK operands (transposed dO / Q reads) go out before the softmax VALU
        short4_t tr_lo[2 * NDB][2], tr_hi[2 * NDB][2];
        auto ld_dvdk = [&](int st) {
          const int s2 = st / NDB, dbk = st % NDB;
          const int o = s2 * 16 * (2 * D);
          tr_lo[st][0] = lds_tr(a_trq[0][dbk] + DO_Q + DB + o);
          tr_hi[st][0] = lds_tr(a_trq[1][dbk] + DO_Q + DB + o);
          tr_lo[st][1] = lds_tr(a_trq[0][dbk] + QB + o);
          tr_hi[st][1] = lds_tr(a_trq[1][dbk] + QB + o);
        };
#pragma unroll
        for (int st = 0; st < PIPE_DVDK; ++st) ld_dvdk(st);
        __builtin_amdgcn_sched_barrier(0);
        // ---- P, dS (element e of the lane: query row 8(e>>2) + 4hh + (e&3), key kc0 + r).  Rows
        // 0-15 (half 0) first; the exps of half 1 run in the shadow of half 0's dV / dK MFMAs.
        const bool need_mask = (p.causal && kc0 + 31 > qt0 + p.causal_offset) || qt0 + kBlockQ > p.Sq || kc0 + 32 > p.Sk;
        float pv[16];
        bf16x8_t pf[2], dsf[2];
        auto p_fix = [&](int e0) {  // masked tiles only (a VALU-only exec-masked block)
          const int my_key = kc0 + r;
#pragma unroll
          for (int e = e0; e < e0 + 8; ++e) {
            const int qg = qt0 + 8 * (e >> 2) + 4 * hh + (e & 3);
            const bool bad = qg >= p.Sq || my_key >= p.Sk || (p.causal && my_key > qg + p.causal_offset);
            pv[e] = bad ? 0.f : pv[e];
          }
        };
        auto p_half = [&](int h) {  // bf16 P / dS of half h, dS^T rows -> LDS
          if constexpr (DROP) {
            const f32x4_t nd0 = lds_ld<f32x4_t>(a_ld + LB + 128 + 32 * (2 * h));
            const f32x4_t nd1 = lds_ld<f32x4_t>(a_ld + LB + 128 + 32 * (2 * h + 1));
            const int my_key = kc0 + r;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int e = 8 * h + j;
              const int qg = qt0 + 8 * (e >> 2) + 4 * hh + (e & 3);
              const uint32_t rh = drop_row_hash(p.drop.seed, b, hq + p.drop.head_offset, qg);
              const float m = drop_keep(rh, my_key, p.drop.thresh) ? p.drop.scale : 0.f;
              const float nd = j < 4 ? nd0[j] : nd1[j - 4];
              pf[h][j] = (__bf16)(pv[e] * m);
              dsf[h][j] = (__bf16)(pv[e] * __builtin_fmaf(m, dp_acc[e], nd));
            }
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              pf[h][j] = (__bf16)pv[8 * h + j];
              dsf[h][j] = (__bf16)(pv[8 * h + j] * dp_acc[8 * h + j]);
            }
          }
          // whole-vector bit casts (per-element extraction of bf16 ext_vectors miscompiles on ROCm 7.2)
          const u32x4_t dw = __builtin_bit_cast(u32x4_t, dsf[h]);
          lds_st(a_dsw[2 * h] + c * 32 * 64, u32x2_t{dw[0], dw[1]});
          lds_st(a_dsw[2 * h + 1] + c * 32 * 64, u32x2_t{dw[2], dw[3]});
        };
#pragma unroll
        for (int e = 0; e < 8; ++e) pv[e] = __builtin_amdgcn_exp2f(s_acc[e] * p.scale_log2);
        if (need_mask) p_fix(0);
        p_half(0);
        // ---- dV += P^T dO ; dK += dS^T Q   (B operands by transposed reads of the tile images)
        constexpr int EPS = 8 / NDB;  // half-1 exps per half-0 step
#pragma unroll
        for (int st = 0; st < 2 * NDB; ++st) {
          {
            if (st + PIPE_DVDK < 2 * NDB) ld_dvdk(st + PIPE_DVDK);
            const int s2 = st / NDB, dbk = st % NDB;
            const bf16s8_t db8 = {tr_lo[st][0][0], tr_lo[st][0][1], tr_lo[st][0][2], tr_lo[st][0][3],
                                  tr_hi[st][0][0], tr_hi[st][0][1], tr_hi[st][0][2], tr_hi[st][0][3]};
            const bf16s8_t qb8 = {tr_lo[st][1][0], tr_lo[st][1][1], tr_lo[st][1][2], tr_lo[st][1][3],
                                  tr_hi[st][1][0], tr_hi[st][1][1], tr_hi[st][1][2], tr_hi[st][1][3]};
            mfma_acc_agpr(acc_dv[c][dbk], pf[s2], db8);
            mfma_acc_agpr(acc_dk[c][dbk], dsf[s2], qb8);
          }
          if (st < NDB) {
#pragma unroll
            for (int j = 0; j < EPS; ++j) pv[8 + EPS * st + j] = __builtin_amdgcn_exp2f(s_acc[8 + EPS * st + j] * p.scale_log2);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (st == NDB - 1) {
            if (need_mask) p_fix(8);
            p_half(1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
    // dS^T complete.  Raw barrier: the tile prefetch (LDS-DMA) stays in flight across it.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(p.ablate & 32)) __builtin_amdgcn_s_barrier();

    // ---- dQ[q][d] += dS[q][key] K[key][d] over this wave's (d block, key range)
    // all key groups, masked ones included (their dS^T entries are zeros): unguarded MFMAs, and
    // near-diagonal tiles only
    // two independent accumulation chains (even / odd key groups): a single chain of dependent
    // 32x32 MFMAs runs at half rate
    f32x16_t acc_dq = f32x16_t{0}, acc_dq2 = f32x16_t{0};
    constexpr int NKS = KEYS_PER_DQ / 16;
    short4_t qa0[NKS], qa1[NKS], qb0[NKS], qb1[NKS];
    auto ld_dq = [&](int s) {
      qa0[s] = lds_tr(a_dsr[0] + s * 16 * 64);
      qa1[s] = lds_tr(a_dsr[1] + s * 16 * 64);
      qb0[s] = lds_tr(a_ktr[0] + s * 16 * (2 * D));
      qb1[s] = lds_tr(a_ktr[1] + s * 16 * (2 * D));
    };
#pragma unroll
    for (int s = 0; s < kPipeDq; ++s) ld_dq(s);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      if (s + kPipeDq < NKS) ld_dq(s + kPipeDq);
      const bf16s8_t a8 = {qa0[s][0], qa0[s][1], qa0[s][2], qa0[s][3], qa1[s][0], qa1[s][1], qa1[s][2], qa1[s][3]};
      const bf16s8_t b8 = {qb0[s][0], qb0[s][1], qb0[s][2], qb0[s][3], qb1[s][0], qb1[s][1], qb1[s][2], qb1[s][3]};
      if (s & 1)
        acc_dq2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), __builtin_bit_cast(bf16x8_t, b8), acc_dq2, 0, 0, 0);
      else
        acc_dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), __builtin_bit_cast(bf16x8_t, b8), acc_dq, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    acc_dq += acc_dq2;
    bool adder = !(p.ablate & 1);
    if constexpr (KEY_SPLIT == 2) {
      // key-half 1 hands its partial to key-half 0 through LDS (no doubled atomics)
      float* red = reinterpret_cast<float*>(smem + OFF_RED) + (dbq * 64 + lane) * 16;
      if (w >= NDB) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<f32x4_t*>(red + 4 * j) = f32x4_t{acc_dq[4 * j], acc_dq[4 * j + 1], acc_dq[4 * j + 2], acc_dq[4 * j + 3]};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (w < NDB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4_t o = *reinterpret_cast<const f32x4_t*>(red + 4 * j);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc_dq[4 * j + i] += o[i];
        }
      } else {
        adder = false;
      }
    }
    if (adder) {
      // (dq_acc has Sq padded to kBlockQ rows: no bounds checks)
      float* dqb = p.dq_acc + (((int64_t)b * p.Hq + hq) * Sq_pad + qt0 + 4 * hh) * D + 32 * dbq + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) atomicAdd(dqb + ((e & 3) + 8 * (e >> 2)) * D, acc_dq[e]);
      // retire the tile prefetch (issued before the atomics) but leave the 16 atomics in flight
      asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    if (!(p.ablate & 32)) __builtin_amdgcn_s_barrier();  // dS^T / Q / dO reads done; next tile landed
  };

  for (int it = it_begin; it < it_end; it += 2) {
    tile(std::integral_constant<int, 0>{}, it);
    if (it + 1 < it_end) tile(std::integral_constant<int, 1>{}, it + 1);
  }

  // the dK/dV MFMAs are inline asm (invisible to the hazard recognizer): give the last ones their
  // pass latency before the accumulators are read
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  if (p.dk_slab != nullptr) {
    // slab mode: this item's dK / dV partials -> its own slab with plain stores (every column,
    // untouched ones as zeros; the accumulators of a fully masked column stay 0)
    if (p.ablate & 2) return;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t srow0 = slab * kBlockK + 64 * w + 32 * c;
#pragma unroll
      for (int dbk = 0; dbk < NDB; ++dbk) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          int64_t off = (srow0 + 8 * gq + 4 * hh) * D + 32 * dbk + r;
          asm volatile("" : "+v"(off));
          float* dkr = p.dk_slab + off;
          float* dvr = p.dv_slab + off;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            dkr[i * D] = acc_dk[c][dbk][4 * gq + i];
            dvr[i * D] = acc_dv[c][dbk][4 * gq + i];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    return;
  }
  // ---- dK, dV partials -> fp32 workspace: C rows = key, col = d (d on the lane)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (!touched[c] || (p.ablate & 2)) continue;
    const int64_t krow0 = ((int64_t)b * p.Hkv + hkv) * Sk_pad + wkey0 + 32 * c;
#pragma unroll
    for (int dbk = 0; dbk < NDB; ++dbk) {
      // one opaque row base per group of 4 rows, issued group by group: unconstrained, the
      // scheduler precomputes all 256 64-bit atomic addresses next to the 256 live accumulators
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        int64_t off = (krow0 + 8 * gq + 4 * hh) * D + 32 * dbk + r;
        asm volatile("" : "+v"(off));
        float* dkr = p.dk_acc + off;
        float* dvr = p.dv_acc + off;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          atomicAdd(dkr + i * D, acc_dk[c][dbk][4 * gq + i]);
          atomicAdd(dvr + i * D, acc_dv[c][dbk][4 * gq + i]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// nlse = -lse / scale (or -inf), ndelta = -sum_d dO * O  (fp32); D/8 lanes per row.
template <int D>
__global__ void __launch_bounds__(256) prep_kernel(const uint16_t* o, const uint16_t* dout, const float* lse, float* nlse,
                                                  float* ndelta, int64_t o_sb, int64_t o_ss, int64_t o_sh, int64_t d_sb,
                                                  int64_t d_ss, int64_t d_sh, int B, int Sq, int Hq, float inv_scale,
                                                  float* dq_zero, int Sq_pad) {
  constexpr int LPR = D / 8;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t nrows = (int64_t)B * Hq * Sq;
  float acc = 0.f;
  if (row < nrows) {
    const int b = row / ((int64_t)Hq * Sq);
    const int h = (row / Sq) % Hq;
    const int qi = row % Sq;
    if (dq_zero != nullptr) {   // this row's slice of the fp32 dQ accumulator (rows >= Sq are never read)
      float* z = dq_zero + (((int64_t)b * Hq + h) * Sq_pad + qi) * D + c * 8;
      *reinterpret_cast<f32x4_t*>(z) = f32x4_t{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4_t*>(z + 4) = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
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
  if (row < nrows && c == 0) {
    ndelta[row] = -acc;
    const float l = lse[row];
    nlse[row] = l == -INFINITY ? -INFINITY : -l * inv_scale;
  }
}

// out (bf16, strided [B,S,H,D]) = acc ([B,H,S_pad,D] fp32) * scale
template <int D>
__global__ void __launch_bounds__(256) acc_convert_kernel(const float* acc, uint16_t* out, int64_t sb, int64_t ss, int64_t sh,
                                                         int B, int S, int S_pad, int H, float scale) {
  constexpr int LPR = D / 8;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t nrows = (int64_t)B * H * S;
  if (row >= nrows) return;
  const int b = row / ((int64_t)H * S);
  const int h = (row / S) % H;
  const int si = row % S;
  const int64_t arow = ((int64_t)b * H + h) * S_pad + si;
  const f32x4_t a0 = *reinterpret_cast<const f32x4_t*>(acc + arow * D + c * 8);
  const f32x4_t a1 = *reinterpret_cast<const f32x4_t*>(acc + arow * D + c * 8 + 4);
  float f[8] = {a0[0] * scale, a0[1] * scale, a0[2] * scale, a0[3] * scale,
                a1[0] * scale, a1[1] * scale, a1[2] * scale, a1[3] * scale};
  *reinterpret_cast<u32x4_t*>(out + b * sb + (int64_t)si * ss + h * sh + c * 8) = pack8(f);
}

// slab mode: out (bf16, strided [B,S,H,D]) = scale * sum of the per-item partials of the row's
// key block (items of key block kb of one (b, h) are slabs [pre(kb), pre(kb) + nc(kb)) of that
// (b, h): the kernel's item numbering)
template <int D>
__global__ void __launch_bounds__(256) slab_convert_kernel(const float* slab, uint16_t* out, int64_t sb, int64_t ss,
                                                          int64_t sh, int B, int S, int H, float scale, int Sq, int G,
                                                          int causal, int coff, int chunk, int per_bh) {
  constexpr int LPR = D / 8;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t nrows = (int64_t)B * H * S;
  if (row >= nrows) return;
  const int b = row / ((int64_t)H * S);
  const int h = (row / S) % H;
  const int si = row % S;
  const int kb = si / kBlockK;
  int pre = 0;
  for (int k2 = 0; k2 < kb; ++k2) pre += (kb_iters(k2, Sq, G, causal, coff) + chunk - 1) / chunk;
  const int nc = (kb_iters(kb, Sq, G, causal, coff) + chunk - 1) / chunk;
  const float* sp = slab + (((int64_t)(b * H + h) * per_bh + pre) * kBlockK + si % kBlockK) * D + c * 8;
  f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nc; ++j) {
    a0 += *reinterpret_cast<const f32x4_t*>(sp + (int64_t)j * kBlockK * D);
    a1 += *reinterpret_cast<const f32x4_t*>(sp + (int64_t)j * kBlockK * D + 4);
  }
  float f[8] = {a0[0] * scale, a0[1] * scale, a0[2] * scale, a0[3] * scale,
                a1[0] * scale, a1[1] * scale, a1[2] * scale, a1[3] * scale};
  *reinterpret_cast<u32x4_t*>(out + b * sb + (int64_t)si * ss + h * sh + c * 8) = pack8(f);
}

template <int D>
void launch_slab_convert(const float* slab, void* out, const int64_t* st, int B, int S, int H, float scale, int Sq,
                         int G, int causal, int coff, int chunk, int per_bh, hipStream_t stream) {
  const int64_t nrows = (int64_t)B * H * S;
  const int rows_per_block = 256 / (D / 8);
  const int grid = (int)((nrows + rows_per_block - 1) / rows_per_block);
  if (grid > 0)
    hipLaunchKernelGGL(slab_convert_kernel<D>, dim3(grid), dim3(256), 0, stream, slab, (uint16_t*)out, st[0], st[1], st[2],
                       B, S, H, scale, Sq, G, causal, coff, chunk, per_bh);
}

template <int D>
void launch_convert(const float* acc, void* out, const int64_t* st, int B, int S, int S_pad, int H, float scale,
                    hipStream_t stream) {
  const int64_t nrows = (int64_t)B * H * S;
  const int rows_per_block = 256 / (D / 8);
  const int grid = (int)((nrows + rows_per_block - 1) / rows_per_block);
  if (grid > 0)
    hipLaunchKernelGGL(acc_convert_kernel<D>, dim3(grid), dim3(256), 0, stream, acc, (uint16_t*)out, st[0], st[1], st[2],
                       B, S, S_pad, H, scale);
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// Chunk length (iterations per work item) minimising the simulated makespan of the item list on
// `ncu` CUs (one resident workgroup each, greedy dispatch in item order).  An item costs its
// iterations plus a fixed overhead for the K/V block load and the dK/dV atomics (~256 KiB of
// f32 adds = about 16 iterations' worth of dQ atomics).  Cached per shape (host-side, once).
int choose_chunk(int nkb, int Sq, int G, int causal, int off, int BH, int ncu) {
  static std::map<std::tuple<int, int, int, int, int, int, int>, int> cache;
  const auto key = std::make_tuple(nkb, Sq, G, causal, off, BH, ncu);
  auto hit = cache.find(key);
  if (hit != cache.end()) return hit->second;
  constexpr int kOverhead = 18;
  std::vector<int> n_it(nkb);
  int64_t total = 0;
  int max_it = 1;
  for (int kb = 0; kb < nkb; ++kb) {
    n_it[kb] = kb_iters(kb, Sq, G, causal, off);
    total += (int64_t)n_it[kb] * BH;
    max_it = std::max(max_it, n_it[kb]);
  }
  int best = max_it;
  double best_t = 1e300;
  std::vector<double> fin;
  // measured (profiles/r2_fa_batch_chunks.jsonl): long items run far slower per iteration than
  // this model says (32 q / 8 kv heads, B = 2: chunk 991 = 226 TF vs chunk 64 = 496 TF) -- their
  // Q/dO streams lose the cross-item L2 reuse -- so the search is capped at kMaxChunk
  constexpr int kMaxChunk = 160;
  best = std::min(best, kMaxChunk);
  for (int chunk = 8; chunk <= std::min(max_it, kMaxChunk); chunk = chunk < 64 ? chunk + 4 : chunk + chunk / 16) {
    const int64_t approx_items = (total + chunk - 1) / chunk;
    if (approx_items > 64 * (int64_t)ncu) continue;  // far too fine
    // min-heap of CU finish times
    std::priority_queue<double, std::vector<double>, std::greater<double>> cu;
    for (int i = 0; i < ncu; ++i) cu.push(0.0);
    double makespan = 0.0;
    for (int kb = 0; kb < nkb; ++kb) {
      if (n_it[kb] == 0) continue;
      const int nc = (n_it[kb] + chunk - 1) / chunk;
      const int per = (n_it[kb] + nc - 1) / nc;
      for (int c = 0; c < nc; ++c) {
        const int len = std::min(n_it[kb], (c + 1) * per) - c * per;
        for (int bh = 0; bh < BH; ++bh) {
          double t = cu.top();
          cu.pop();
          t += len + kOverhead;
          makespan = std::max(makespan, t);
          cu.push(t);
        }
      }
    }
    if (makespan < best_t * 0.999) {
      best_t = makespan;
      best = chunk;
    }
  }
  cache[key] = best;
  return best;
}

// tuning knobs, resolved once at load (NXD_FAB_ABLATE / NXD_FAB_CHUNK) and settable from Python
// (flash_attn_set_knob) for in-process A/B — no per-launch getenv
static int g_ablate = -1, g_chunk = -1, g_xcd = -1;
int xcd_map_mode() {
  if (g_xcd < 0) {
    const char* e = getenv("NXD_FAB_XCD_MAP");
    g_xcd = e ? atoi(e) : 2;
  }
  return g_xcd;
}
int ablate_flags() {
  if (g_ablate < 0) {
    const char* e = getenv("NXD_FAB_ABLATE");
    g_ablate = e ? atoi(e) : 0;
  }
  return g_ablate;
}
int chunk_override() {
  if (g_chunk < 0) {
    const char* e = getenv("NXD_FAB_CHUNK");
    g_chunk = e ? atoi(e) : 0;
  }
  return g_chunk;
}

// dK/dV reduction across the items of a key block: 0 = f32 atomics into one accumulator, 1 = per-item
// slabs written with plain stores and summed by the convert pass (NXD_FAB_DKV_SLAB, default 1).
// Slabs take the 0.55 GB of dK/dV adds (S=8192, 32/8 heads) off the chip-wide f32 atomic rate the
// kernel is bound by, for 0.55 GB of plain stores plus one read in the convert: 2.117 -> 2.008 ms
// (32/8 heads), 1.072 -> 1.014 (TP=8 shape, B=4), 0.299 -> 0.275 (4/1, B=1); D=64 16/4 neutral
// (profiles/r3_fab_slab_ab.jsonl).
static int g_slab = -1;
int slab_mode() {
  if (g_slab < 0) {
    const char* e = getenv("NXD_FAB_DKV_SLAB");
    g_slab = e ? atoi(e) : 1;
  }
  return g_slab;
}

static int g_pipe = -1;
int pipe_variant() {
  if (g_pipe < 0) {
    const char* e = getenv("NXD_FAB_PIPE");
    g_pipe = e ? atoi(e) : 12;
  }
  return g_pipe;
}

template <int D, int PIPE, int PIPE_DVDK, bool DROP = false>
void launch_bwd(const BwdParams& p, int64_t items, size_t lds, hipStream_t stream) {
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once per instantiation
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)bwd_kernel<D, PIPE, PIPE_DVDK, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((bwd_kernel<D, PIPE, PIPE_DVDK, DROP>), dim3((unsigned)items), dim3(kThreads), lds, stream, p);
}

}  // namespace fab

void flash_attn_bwd_set_knob(int which, int value) {
  if (which == 0) fab::g_ablate = value;
  if (which == 1) fab::g_chunk = value;
  if (which == 3) fab::g_xcd = value;
  if (which == 4) fab::g_pipe = value;  // pipeline depths: 12 (default), 11, 21, 0
  if (which == 5) fab::g_slab = value;  // dK/dV: 0 atomics, 1 per-item slabs
}

namespace fab {
// work-item chunk length and items per (batch, kv head) of a launch (one definition for the
// workspace sizing and the launch)
void plan(int B, int Sq, int Sk, int Hq, int Hkv, int causal, int causal_offset, int* chunk, int64_t* per_bh) {
  const int nkb = (Sk + kBlockK - 1) / kBlockK;
  const int G = Hq / Hkv;
  *chunk = chunk_override() > 0 ? chunk_override() : choose_chunk(nkb, Sq, G, causal, causal_offset, B * Hkv, num_cus());
  int64_t n = 0;
  for (int kb = 0; kb < nkb; ++kb) n += (kb_iters(kb, Sq, G, causal, causal_offset) + *chunk - 1) / *chunk;
  *per_bh = n;
}
}  // namespace fab

// fp32 workspace floats the backward needs: dq_acc + dk_acc + dv_acc + nlse + ndelta (+ the dK / dV
// slabs in slab mode)
int64_t flash_attn_bwd_workspace(int B, int Sq, int Sk, int Hq, int Hkv, int D, int causal, int causal_offset) {
  const int64_t Sq_pad = (Sq + fab::kBlockQ - 1) / fab::kBlockQ * fab::kBlockQ;
  const int64_t Sk_pad = (Sk + fab::kBlockK - 1) / fab::kBlockK * fab::kBlockK;
  int64_t n = (int64_t)B * Hq * Sq_pad * D + 2 * (int64_t)B * Hkv * Sk_pad * D + 2 * (int64_t)B * Hq * Sq;
  if (fab::slab_mode() && Hkv > 0 && Hq % Hkv == 0) {
    int chunk;
    int64_t per_bh;
    fab::plan(B, Sq, Sk, Hq, Hkv, causal, causal_offset, &chunk, &per_bh);
    n += 2 * (int64_t)B * Hkv * per_bh * fab::kBlockK * D;
  }
  return n;
}

int flash_attn_bwd_launch(const void* q, const void* k, const void* v, const void* o, const void* dout,
                          const float* lse, float* ws, void* dq, void* dk, void* dv,
                          const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os,
                          const int64_t* dos, const int64_t* dqs, const int64_t* dks, const int64_t* dvs,
                          int B, int Sq, int Sk, int Hq, int Hkv, int D, float softmax_scale, int causal,
                          int causal_offset, const DropoutArgs& drop, hipStream_t stream) {
  using namespace fab;
  if (Hkv <= 0 || Hq % Hkv != 0 || (D != 64 && D != 128)) return -1;
  const int G = Hq / Hkv;
  const int64_t Sq_pad = (Sq + kBlockQ - 1) / kBlockQ * kBlockQ;
  const int nkb = (Sk + kBlockK - 1) / kBlockK;
  const int64_t Sk_pad = (int64_t)nkb * kBlockK;
  float* dq_acc = ws;
  float* dk_acc = dq_acc + (int64_t)B * Hq * Sq_pad * D;
  float* dv_acc = dk_acc + (int64_t)B * Hkv * Sk_pad * D;
  float* nlse = dv_acc + (int64_t)B * Hkv * Sk_pad * D;
  float* ndelta = nlse + (int64_t)B * Hq * Sq;
  int chunk;
  int64_t per_bh;
  plan(B, Sq, Sk, Hq, Hkv, causal, causal_offset, &chunk, &per_bh);
  const bool slabs = slab_mode() != 0;
  float* dk_slab = slabs ? ndelta + (int64_t)B * Hq * Sq : nullptr;
  float* dv_slab = slabs ? dk_slab + (int64_t)B * Hkv * per_bh * kBlockK * D : nullptr;
  // zeroing: one memset for the accumulators (the slabs are written whole by the kernel), or, opt-in,
  // the dQ rows zeroed by the prep kernel, which visits every (row, head) anyway
  // NXD_FAB_PREP_ZERO=1 zeroes in the prep kernel instead of the memset launch: bench 3,006 / 3,016
  // vs 2,999 / 3,007 ms per step with the memset (profiles/r4_fab_prep_zero_ab.txt), so off
  static int prep_zero = -1;
  if (prep_zero < 0) {
    const char* e = getenv("NXD_FAB_PREP_ZERO");
    prep_zero = e ? (atoi(e) != 0) : 0;
  }
  const bool pz = slabs && prep_zero;
  if (!pz)
    (void)hipMemsetAsync(ws, 0, (size_t)((int64_t)B * Hq * Sq_pad * D + (slabs ? 0 : 2 * (int64_t)B * Hkv * Sk_pad * D)) * sizeof(float), stream);
  float* dq_zero = pz ? dq_acc : nullptr;

  const int64_t nrows = (int64_t)B * Hq * Sq;
  const int rows_per_block = 256 / (D / 8);
  const int gpre = (int)((nrows + rows_per_block - 1) / rows_per_block);
  if (gpre > 0) {
    if (D == 128)
      hipLaunchKernelGGL(prep_kernel<128>, dim3(gpre), dim3(256), 0, stream, (const uint16_t*)o, (const uint16_t*)dout, lse,
                         nlse, ndelta, os[0], os[1], os[2], dos[0], dos[1], dos[2], B, Sq, Hq, 1.f / softmax_scale,
                         dq_zero, (int)Sq_pad);
    else
      hipLaunchKernelGGL(prep_kernel<64>, dim3(gpre), dim3(256), 0, stream, (const uint16_t*)o, (const uint16_t*)dout, lse,
                         nlse, ndelta, os[0], os[1], os[2], dos[0], dos[1], dos[2], B, Sq, Hq, 1.f / softmax_scale,
                         dq_zero, (int)Sq_pad);
  }

  BwdParams p{};
  p.q = (const uint16_t*)q; p.k = (const uint16_t*)k; p.v = (const uint16_t*)v; p.dout = (const uint16_t*)dout;
  p.nlse = nlse; p.ndelta = ndelta; p.dq_acc = dq_acc; p.dk_acc = dk_acc; p.dv_acc = dv_acc;
  p.dk_slab = dk_slab; p.dv_slab = dv_slab;
  p.q_sb = qs[0]; p.q_ss = qs[1]; p.q_sh = qs[2];
  p.k_sb = ks[0]; p.k_ss = ks[1]; p.k_sh = ks[2];
  p.v_sb = vs[0]; p.v_ss = vs[1]; p.v_sh = vs[2];
  p.do_sb = dos[0]; p.do_ss = dos[1]; p.do_sh = dos[2];
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale_log2 = softmax_scale * 1.4426950408889634f;
  p.causal = causal; p.causal_offset = causal_offset;

  p.chunk = chunk;
  const int64_t items = per_bh * B * Hkv;
  p.ablate = ablate_flags();
  p.xcd_map = xcd_map_mode();
  p.drop = drop;
  if (items > 0) {
    if (D == 128) {
      const size_t lds = kBlockK * 128 * 2 + 4 * kBlockQ * 128 * 2 + kBlockK * 64 + 512 + 128 * 128 * 2;
      if (drop.enabled()) {
        launch_bwd<128, 1, 2, true>(p, items, lds, stream);
      } else switch (pipe_variant()) {
        case 11: launch_bwd<128, 1, 1>(p, items, lds, stream); break;
        case 21: launch_bwd<128, 2, 1>(p, items, lds, stream); break;
        case 0: launch_bwd<128, 0, 0>(p, items, lds, stream); break;
        default: launch_bwd<128, 1, 2>(p, items, lds, stream); break;
      }
    } else {
      const size_t lds = kBlockK * 64 * 2 + 4 * kBlockQ * 64 * 2 + kBlockK * 64 + 512 + 2 * 64 * 16 * 4 + 128 * 64 * 2;
      if (drop.enabled())
        launch_bwd<64, 1, 2, true>(p, items, lds, stream);
      else
        launch_bwd<64, 1, 2>(p, items, lds, stream);
    }
  }
  if (D == 128) {
    launch_convert<128>(dq_acc, dq, dqs, B, Sq, (int)Sq_pad, Hq, softmax_scale, stream);
    if (slabs) {
      launch_slab_convert<128>(dk_slab, dk, dks, B, Sk, Hkv, softmax_scale, Sq, G, causal, causal_offset, chunk, (int)per_bh, stream);
      launch_slab_convert<128>(dv_slab, dv, dvs, B, Sk, Hkv, 1.f, Sq, G, causal, causal_offset, chunk, (int)per_bh, stream);
    } else {
      launch_convert<128>(dk_acc, dk, dks, B, Sk, (int)Sk_pad, Hkv, softmax_scale, stream);
      launch_convert<128>(dv_acc, dv, dvs, B, Sk, (int)Sk_pad, Hkv, 1.f, stream);
    }
  } else {
    launch_convert<64>(dq_acc, dq, dqs, B, Sq, (int)Sq_pad, Hq, softmax_scale, stream);
    if (slabs) {
      launch_slab_convert<64>(dk_slab, dk, dks, B, Sk, Hkv, softmax_scale, Sq, G, causal, causal_offset, chunk, (int)per_bh, stream);
      launch_slab_convert<64>(dv_slab, dv, dvs, B, Sk, Hkv, 1.f, Sq, G, causal, causal_offset, chunk, (int)per_bh, stream);
    } else {
      launch_convert<64>(dk_acc, dk, dks, B, Sk, (int)Sk_pad, Hkv, softmax_scale, stream);
      launch_convert<64>(dv_acc, dv, dvs, B, Sk, (int)Sk_pad, Hkv, 1.f, stream);
    }
  }
  return (int)hipGetLastError();
}

}  // namespace nxd
