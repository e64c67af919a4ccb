// Rotary position embedding (rotate-half convention of HF Llama) applied IN PLACE to the q and
// k heads of a fused QKV projection output.  Replaces HF `apply_rotary_pos_emb`
// (examples/training/llama/modeling_llama_nxd.py:398-399, examples/inference/modules/attention/utils.py:27-41).
//
//   x1 = x[:D/2], x2 = x[D/2:];  out1 = x1*cos - x2*sin;  out2 = x2*cos + x1*sin
//   backward = the same rotation with sin negated (pass sign = -1).
//
// Token t of a [T, W] buffer (W = row stride in elements) holds `nheads` heads of D starting at
// column `col0`; its position is pos[t] if a position tensor is given, else (t / pos_div) % pos_mod
// (covers [S, B, W] and [B, S, W] layouts).  cos/sin come from fp32 tables [max_pos, D/2]
// precomputed on the host (Llama-3 frequency scaling included there) — no device trig
// (Appendix B "Element-wise": on-device sin/cos turns the op VALU-bound).
#include "common.h"

namespace nxd {
namespace rope {

template <int D>
__global__ void __launch_bounds__(256) kernel(uint16_t* __restrict__ buf, int64_t T, int64_t W, int col0, int nheads,
                                              const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                              const int64_t* __restrict__ pos, int64_t pos_div, int64_t pos_mod, float sign) {
  constexpr int HALF = D / 2;
  constexpr int TPH = HALF / 8;  // threads per head
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t work = T * nheads * TPH;
  if (gid >= work) return;
  const int c = gid % TPH;
  const int64_t th = gid / TPH;
  const int hd = th % nheads;
  const int64_t t = th / nheads;
  const int64_t p = pos ? pos[t] : (t / pos_div) % pos_mod;
  uint16_t* x = buf + t * W + col0 + (int64_t)hd * D;
  float a[8], bb[8], o1[8], o2[8];
  unpack8(*reinterpret_cast<const u32x4_t*>(x + c * 8), a);
  unpack8(*reinterpret_cast<const u32x4_t*>(x + HALF + c * 8), bb);
  const float* cp = cos_t + p * HALF + c * 8;
  const float* sp = sin_t + p * HALF + c * 8;
  const f32x4_t c0 = *reinterpret_cast<const f32x4_t*>(cp), c1 = *reinterpret_cast<const f32x4_t*>(cp + 4);
  const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(sp), s1 = *reinterpret_cast<const f32x4_t*>(sp + 4);
  const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
  const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float s = sn[j] * sign;
    o1[j] = a[j] * cs[j] - bb[j] * s;
    o2[j] = bb[j] * cs[j] + a[j] * s;
  }
  *reinterpret_cast<u32x4_t*>(x + c * 8) = pack8(o1);
  *reinterpret_cast<u32x4_t*>(x + HALF + c * 8) = pack8(o2);
}

}  // namespace rope

int rope_inplace_launch(void* buf, int64_t T, int64_t W, int col0, int nheads, int D, const float* cos_t,
                        const float* sin_t, const int64_t* pos, int64_t pos_div, int64_t pos_mod, float sign,
                        hipStream_t stream) {
  const int64_t work = T * nheads * (D / 16);
  if (work == 0) return 0;
  const dim3 grid((unsigned)((work + 255) / 256)), block(256);
  if (D == 128)
    hipLaunchKernelGGL(rope::kernel<128>, grid, block, 0, stream, (uint16_t*)buf, T, W, col0, nheads, cos_t, sin_t, pos, pos_div, pos_mod, sign);
  else if (D == 64)
    hipLaunchKernelGGL(rope::kernel<64>, grid, block, 0, stream, (uint16_t*)buf, T, W, col0, nheads, cos_t, sin_t, pos, pos_div, pos_mod, sign);
  else if (D == 256)
    hipLaunchKernelGGL(rope::kernel<256>, grid, block, 0, stream, (uint16_t*)buf, T, W, col0, nheads, cos_t, sin_t, pos, pos_div, pos_mod, sign);
  else
    return -1;
  return (int)hipGetLastError();
}

}  // namespace nxd
