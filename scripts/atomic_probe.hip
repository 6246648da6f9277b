// Diagnostic: throughput and latency of device-scope atomicAdd with return
// on ONE address, as a grid-wide work counter would use it.  Each of G
// workgroups (one wave each does the work) performs K grabs, waiting for
// each result before the next (like a work queue), with `gap` cycles of
// busy work between grabs.  Prints ns per grab per wave and the aggregate
// grab rate.
//   hipcc --offload-arch=gfx950 -O2 -o build/atomic_probe scripts/atomic_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void probe(unsigned* ctr, unsigned* sink, int k, int gap) {
  if (threadIdx.x >= 64) return;
  unsigned acc = 0;
  for (int i = 0; i < k; ++i) {
    unsigned v = 0;
    if (threadIdx.x == 0)
      v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = __builtin_amdgcn_readfirstlane(v);
    acc += v;
    const long long t0 = clock64();
    while (clock64() - t0 < gap) {
    }
  }
  if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}

int main() {
  unsigned *ctr, *sink;
  if (hipMalloc(&ctr, 4) != hipSuccess || hipMalloc(&sink, 4 * 4096) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grids[] = {1, 8, 64, 256, 1024};
  const int gaps[] = {0, 2000, 10000};
  for (int gap : gaps) {
    for (int g : grids) {
      const int k = 200;
      hipMemset(ctr, 0, 4);
      hipLaunchKernelGGL(probe, dim3(g), dim3(64), 0, 0, ctr, sink, 4, gap);  // warm
      hipMemset(ctr, 0, 4);
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(probe, dim3(g), dim3(64), 0, 0, ctr, sink, k, gap);
      hipEventRecord(b, 0);
      if (hipEventSynchronize(b) != hipSuccess) return 2;
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      unsigned got = 0;
      hipMemcpy(&got, ctr, 4, hipMemcpyDeviceToHost);
      printf("gap %6d cycles  waves %5d  grabs %8u  %8.3f ms  %7.1f ns/grab/wave  %8.1f grabs/us\n",
             gap, g, got, ms, ms * 1e6 / k, got / (ms * 1e3));
    }
  }
  return 0;
}
