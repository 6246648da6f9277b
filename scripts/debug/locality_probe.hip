// Read-bandwidth probe: the same 4 KiB-page loads (one wave per page per
// iteration, 1 KiB per lane-row, 16 waves per CU, 2 pages in flight per
// wave) in two page orders -- interleaved (page k * NW + w: the waves sweep
// one compact front, as run_ea's span deal does) and per-wave contiguous
// (page w * P + k: 4096 separate streams, as run_ps's chunks do).
//   hipcc --offload-arch=gfx950 -O3 -o build/probe/locality scripts/debug/locality_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const uint8_t* __restrict__ base, uint64_t pages,
                                              uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  const uint64_t w = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t per = pages / nw;
  uint32_t acc = 0;
  for (uint64_t k = 0; k + 1 < per; k += 2) {
    const uint64_t p0 = MODE == 0 ? k * nw + w : w * per + k;
    const uint64_t p1 = MODE == 0 ? (k + 1) * nw + w : w * per + k + 1;
    const u32x4* a = reinterpret_cast<const u32x4*>(base + p0 * 4096) + lane;
    const u32x4* b = reinterpret_cast<const u32x4*>(base + p1 * 4096) + lane;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = __builtin_nontemporal_load(a + 64 * i);
      v[4 + i] = __builtin_nontemporal_load(b + 64 * i);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  if (acc == 0x12345678u) out[w] = acc;
}

int main() {
  const uint64_t bytes = 4ull << 30, pages = bytes / 4096;
  uint8_t* d;
  uint32_t* o;
  hipMalloc(&d, bytes);
  hipMalloc(&o, 1 << 20);
  hipMemset(d, 1, bytes);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 2; ++mode) {
      for (int i = 0; i < 3; ++i) {
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(1024), 0, 0, d, pages, o);
        else hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(1024), 0, 0, d, pages, o);
      }
      hipEventRecord(e0);
      const int n = 20;
      for (int i = 0; i < n; ++i) {
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(1024), 0, 0, d, pages, o);
        else hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(1024), 0, 0, d, pages, o);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s: %.1f GiB/s\n", mode == 0 ? "interleaved" : "per-wave contiguous",
             bytes / (ms / n * 1e-3) / (1 << 30));
    }
  }
  return 0;
}
