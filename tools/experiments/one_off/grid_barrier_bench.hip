// Cost of a device-wide barrier between the phases of a persistent decode kernel, vs a kernel
// boundary.  G co-resident workgroups of 256 threads run N barriers: thread 0 of each workgroup
// adds to an arrival counter (device scope), the last arrival resets it and bumps a generation
// word, the others poll the generation with device-scope acquire loads.  Every poll loop is
// bounded (a timed-out workgroup records it and leaves), so the grid always drains.
//   hipcc --offload-arch=gfx950 -O3 -o grid_barrier_bench tools/grid_barrier_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ bool grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, unsigned* timeouts) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nblocks - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > 20000000) {
          atomicAdd(timeouts, 1u);
          ok = false;
          break;
        }
      }
    }
  }
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = ok;
  __syncthreads();
  return s_ok;
}

__global__ void __launch_bounds__(256) barrier_kernel(unsigned* count, unsigned* gen, unsigned* timeouts, int n, float* sink) {
  float acc = threadIdx.x;
  for (int i = 0; i < n; ++i) {
    acc = acc * 1.0001f + 1.0f;
    if (!grid_barrier(count, gen, gridDim.x, timeouts)) break;
  }
  if (acc == -1.f) sink[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) empty_kernel(float* sink) {
  if (threadIdx.x == 1023) sink[blockIdx.x] = 0.f;
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, dev);
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, barrier_kernel, 256, 0);
  const int max_resident = per_cu * prop.multiProcessorCount;
  printf("{\"cus\": %d, \"resident_blocks_per_cu\": %d}\n", prop.multiProcessorCount, per_cu);
  unsigned *count, *gen, *timeouts;
  float* sink;
  (void)hipMalloc(&count, 4);
  (void)hipMalloc(&gen, 4);
  (void)hipMalloc(&timeouts, 4);
  (void)hipMalloc(&sink, 1 << 20);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int N = 2000;
  for (int G : {64, 256, 512, 1024, 2048}) {
    if (G > max_resident) continue;   // a grid barrier needs every workgroup resident
    (void)hipMemset(count, 0, 4);
    (void)hipMemset(gen, 0, 4);
    (void)hipMemset(timeouts, 0, 4);
    hipLaunchKernelGGL(barrier_kernel, dim3(G), dim3(256), 0, 0, count, gen, timeouts, 10, sink);  // warm-up
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(barrier_kernel, dim3(G), dim3(256), 0, 0, count, gen, timeouts, N, sink);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned to = 0;
    (void)hipMemcpy(&to, timeouts, 4, hipMemcpyDeviceToHost);
    printf("{\"kind\": \"grid_barrier\", \"blocks\": %d, \"us_per_barrier\": %.3f, \"timeouts\": %u}\n", G, 1000.f * ms / N, to);
  }
  // kernel boundaries: N back-to-back launches of an empty kernel (stream-ordered), and the same in a graph
  for (int G : {256, 1024, 2048}) {
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(256), 0, 0, sink);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"kind\": \"launch\", \"blocks\": %d, \"us_per_kernel\": %.3f}\n", G, 1000.f * ms / N);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipGraph_t graph;
    hipGraphExec_t exec;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(256), 0, s, sink);
    (void)hipStreamEndCapture(s, &graph);
    (void)hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphLaunch(exec, s);
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 10; ++r) (void)hipGraphLaunch(exec, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"kind\": \"graph_launch\", \"blocks\": %d, \"us_per_kernel\": %.3f}\n", G, 1000.f * ms / 2000);
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);
    (void)hipStreamDestroy(s);
  }
  return 0;
}
