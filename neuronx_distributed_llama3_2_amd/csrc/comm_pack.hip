// Multi-tensor pack / unpack for the native collective layer (csrc/comm.cpp): many small tensors
// are copied into (or out of) one persistent staging buffer by ONE launch, so a bucket of N
// gradients costs one collective and two launches instead of N collectives.  Up to kMaxDesc
// (src, dst, bytes) descriptors travel in the kernel argument block (no host->device table copy);
// grid.y = descriptor, grid.x strides over its bytes with 16-byte vectors.
#include "common.h"

namespace nxd {
namespace cpack {

constexpr int kMaxDesc = 64;

struct Desc {
  const char* src;
  char* dst;
  int64_t nbytes;
};
struct DescTable {
  Desc d[kMaxDesc];
};

__global__ void __launch_bounds__(256) multi_copy_kernel(DescTable t) {
  const Desc c = t.d[blockIdx.y];
  const int64_t nvec = c.nbytes / 16;
  const bool aligned = ((reinterpret_cast<uintptr_t>(c.src) | reinterpret_cast<uintptr_t>(c.dst)) & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (aligned) {
    for (int64_t i = t0; i < nvec; i += stride)
      reinterpret_cast<u32x4_t*>(c.dst)[i] = reinterpret_cast<const u32x4_t*>(c.src)[i];
    for (int64_t i = nvec * 16 + t0; i < c.nbytes; i += stride) c.dst[i] = c.src[i];
  } else {
    for (int64_t i = t0; i < c.nbytes; i += stride) c.dst[i] = c.src[i];
  }
}

}  // namespace cpack

// n descriptors (arrays of length n); launches ceil(n / 64) kernels on `stream`.
int multi_copy_launch(const void* const* src, void* const* dst, const int64_t* nbytes, int n, hipStream_t stream) {
  using namespace cpack;
  for (int base = 0; base < n; base += kMaxDesc) {
    const int m = n - base < kMaxDesc ? n - base : kMaxDesc;
    DescTable t{};
    int64_t maxb = 0;
    for (int i = 0; i < m; ++i) {
      t.d[i] = Desc{static_cast<const char*>(src[base + i]), static_cast<char*>(dst[base + i]), nbytes[base + i]};
      maxb = nbytes[base + i] > maxb ? nbytes[base + i] : maxb;
    }
    if (maxb == 0) continue;
    int64_t bx = (maxb / 16 + 255) / 256;
    bx = bx < 1 ? 1 : (bx > 1024 ? 1024 : bx);
    hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)bx, (unsigned)m), dim3(256), 0, stream, t);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace nxd
