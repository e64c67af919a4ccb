// Probe of v_dot2c_f32_bf16 (__builtin_amdgcn_fdot2_f32_bf16) on gfx950 against the exact f32 sum.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <vector>
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__global__ void probe(const uint32_t* a, const uint32_t* b, const float* c, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a[i]), __builtin_bit_cast(bf16x2_t, b[i]), c[i], false);
}
static float bf(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t tobf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
int main() {
  const int n = 4096;
  std::vector<uint32_t> a(n), b(n); std::vector<float> c(n), o(n);
  srand(1);
  for (int i = 0; i < n; ++i) {
    float x0 = (rand() / (float)RAND_MAX - 0.5f) * 4, x1 = (rand() / (float)RAND_MAX - 0.5f) * 4;
    float y0 = (rand() / (float)RAND_MAX - 0.5f) * 0.1f, y1 = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
    a[i] = tobf(x0) | ((uint32_t)tobf(x1) << 16);
    b[i] = tobf(y0) | ((uint32_t)tobf(y1) << 16);
    c[i] = (rand() / (float)RAND_MAX - 0.5f);
  }
  uint32_t *da, *db; float *dc, *dout;
  hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice); hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dout, n);
  hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
  double maxerr = 0; int worst = 0;
  for (int i = 0; i < n; ++i) {
    double ref = (double)bf(a[i] & 0xffff) * bf(b[i] & 0xffff) + (double)bf(a[i] >> 16) * bf(b[i] >> 16) + c[i];
    double e = fabs(o[i] - ref) / (fabs(ref) + 1e-6);
    if (e > maxerr) { maxerr = e; worst = i; }
  }
  int i = worst;
  double ref = (double)bf(a[i] & 0xffff) * bf(b[i] & 0xffff) + (double)bf(a[i] >> 16) * bf(b[i] >> 16) + c[i];
  printf("dot2 probe: max rel err %.3e at %d: got %.8f ref %.8f (a %g %g b %g %g c %g)\n", maxerr, i, o[i], ref,
         bf(a[i] & 0xffff), bf(a[i] >> 16), bf(b[i] & 0xffff), bf(b[i] >> 16), c[i]);
  for (int j = 0; j < 4; ++j) {
    double r = (double)bf(a[j] & 0xffff) * bf(b[j] & 0xffff) + (double)bf(a[j] >> 16) * bf(b[j] >> 16) + c[j];
    printf("  %d: got %.8f ref %.8f\n", j, o[j], r);
  }
  return 0;
}
