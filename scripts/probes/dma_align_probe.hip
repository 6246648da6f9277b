// dma_align_probe.hip -- standalone probe (not product code): does
// global_load_lds_dwordx4 from byte-misaligned global addresses deliver the
// right bytes, and what does the misalignment cost a load-only skeleton of
// the spans kernel (per-wave 4 KiB LDS slot, 4 DMAs of 1 KiB per segment,
// 16 waves per CU, one segment in flight per wave)?
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/dma_align_probe.hip \
//         -o build/dma_align_probe && build/dma_align_probe
//
// For skew s in {0, 4, 8, 12, 16, 64}: 1 M blocks of 4 KiB read at
// base + 4096 i + s; every wave compares its slot with the same bytes read
// by plain global loads (first pass) and XOR-reduces (timed passes).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4 l_u32x4;

__device__ __forceinline__ void dma4(uint64_t base, uint32_t slot, uint32_t o0, uint32_t o1,
                                     uint32_t o2, uint32_t o3) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %6 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %6 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %6 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %4, %6 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(o0), "v"(o1), "v"(o2), "v"(o3), "s"(slot), "s"(base)
      : "memory", "scc");
}

// Wave w of workgroup g takes blocks g*16 + w, + 16 * grid, ...; one block
// in flight per wave (the next DMA is issued right after the slot is read).
__global__ __launch_bounds__(1024) void skel_kernel(const uint8_t* __restrict__ data, uint32_t skew,
                                                    uint64_t count, uint32_t* __restrict__ out,
                                                    uint32_t* __restrict__ bad, int check) {
  extern __shared__ uint8_t lds[];
  const uint32_t l = threadIdx.x & 63u, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t slot = 98304u + w * 4096u;
  (void)lds;
  const uint64_t stride = uint64_t(gridDim.x) * 16u;
  uint64_t b = uint64_t(blockIdx.x) * 16u + w;
  if (b >= count) return;
  const uint64_t base = reinterpret_cast<uint64_t>(data) + skew;
  dma4(base + __builtin_amdgcn_readfirstlane(b) * 4096u, slot, 16u * l, 16u * l + 1024u, 16u * l + 2048u, 16u * l + 3072u);
  uint32_t acc = 0;
  for (;;) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(slot + 1024u * q + 16u * l));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t cur = b;
    b += stride;
    if (b < count)
      dma4(base + __builtin_amdgcn_readfirstlane(b) * 4096u, slot, 16u * l, 16u * l + 1024u, 16u * l + 2048u, 16u * l + 3072u);
    if (check) {
      const uint8_t* src = data + skew + cur * 4096u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u32x4 g;
        __builtin_memcpy(&g, src + 1024u * q + 16u * l, 16);
        if (g.x != v[q].x || g.y != v[q].y || g.z != v[q].z || g.w != v[q].w) atomicAdd(bad, 1u);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    if (b >= count) break;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep the loads
}

__global__ void fill_kernel(uint64_t* dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
       i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[i] = z ^ (z >> 31);
  }
}

int main(int argc, char** argv) {
  const uint64_t count = argc > 1 ? strtoull(argv[1], 0, 0) : (1u << 20);
  const int reps = 50;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  uint8_t* d;
  const uint64_t bytes = count * 4096u + 4096u;
  CK(hipMalloc(&d, bytes));
  fill_kernel<<<4096, 256>>>(reinterpret_cast<uint64_t*>(d), bytes / 8);
  uint32_t *out, *bad;
  CK(hipMalloc(&out, grid * 4));
  CK(hipMalloc(&bad, 4));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(skel_kernel),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // precondition (clock settling)
  for (int i = 0; i < 150; ++i) skel_kernel<<<grid, 1024, 163840>>>(d, 0, count, out, bad, 0);
  const uint32_t skews[] = {0, 4, 8, 12, 16, 64, 0};
  for (uint32_t s : skews) {
    CK(hipMemset(bad, 0, 4));
    skel_kernel<<<grid, 1024, 163840>>>(d, s, count, out, bad, 1);
    uint32_t nbad = 0;
    CK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < 10; ++i) skel_kernel<<<grid, 1024, 163840>>>(d, s, count, out, bad, 0);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) skel_kernel<<<grid, 1024, 163840>>>(d, s, count, out, bad, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("{\"skew\": %u, \"ms\": %.4f, \"TBps\": %.3f, \"mismatched_chunks\": %u}\n", s, ms,
           count * 4096.0 / ms / 1e9, nbad);
  }
  CK(hipFree(d));
  return 0;
}
