// Vocab-parallel embedding gather / scatter-add (reference: ParallelEmbedding
// `_forward_shard_across_vocab`, src/neuronx_distributed/parallel_layers/layers.py:215-238).
//
//   fwd: out[t] = W[id - start] if start <= id < start + Vl else 0   (mask fused into the gather)
//   bwd: dW[id - start] += dout[t] for in-range tokens, f32 atomics straight into the fp32
//        main_grad of the weight (whole 256-B contiguous row segments per wave-instruction: the
//        full-rate atomic shape; no [V, H] zero-fill + index_add round trip).
#include "common.h"

namespace nxd {
namespace emb {

__global__ void __launch_bounds__(256) fwd_kernel(const int64_t* __restrict__ ids, const uint16_t* __restrict__ w,
                                                  uint16_t* __restrict__ out, int64_t T, int H, int64_t start, int64_t Vl) {
  const int nv = H / 8;
  const int64_t total = T * nv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i / nv;
    const int c = i % nv;
    const int64_t id = ids[t] - start;
    u32x4_t v = {0, 0, 0, 0};
    if (id >= 0 && id < Vl) v = *reinterpret_cast<const u32x4_t*>(w + id * H + c * 8);
    *reinterpret_cast<u32x4_t*>(out + t * H + c * 8) = v;
  }
}

__global__ void __launch_bounds__(256) bwd_kernel(const int64_t* __restrict__ ids, const uint16_t* __restrict__ dout,
                                                  float* __restrict__ dw, int64_t T, int H, int64_t start, int64_t Vl) {
  // one workgroup per token row, lanes over contiguous columns
  for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
    const int64_t id = ids[t] - start;
    if (id < 0 || id >= Vl) continue;
    float* dst = dw + id * H;
    const uint16_t* src = dout + t * H;
    for (int c = threadIdx.x; c < H; c += 256) atomicAdd(dst + c, bf2f(src[c]));
  }
}

}  // namespace emb

int embedding_fwd_launch(const int64_t* ids, const void* w, void* out, int64_t T, int H, int64_t start, int64_t Vl,
                         hipStream_t stream) {
  if (H % 8) return -1;
  const int64_t total = T * (H / 8);
  if (total == 0) return 0;
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(emb::fwd_kernel, dim3((unsigned)g), dim3(256), 0, stream, ids, (const uint16_t*)w, (uint16_t*)out, T, H, start, Vl);
  return (int)hipGetLastError();
}

int embedding_bwd_launch(const int64_t* ids, const void* dout, float* dw, int64_t T, int H, int64_t start, int64_t Vl,
                         hipStream_t stream) {
  if (T == 0) return 0;
  int64_t g = T < 4096 ? T : 4096;
  hipLaunchKernelGGL(emb::bwd_kernel, dim3((unsigned)g), dim3(256), 0, stream, ids, (const uint16_t*)dout, dw, T, H, start, Vl);
  return (int)hipGetLastError();
}

}  // namespace nxd
