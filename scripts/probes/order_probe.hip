// order_probe.hip -- standalone probe (not product code): the load-only
// skeleton of the spans kernel (one 4 KiB LDS slot per wave, 4 DMAs of 1 KiB
// per block, the next DMA issued right after the slot is read) over 1 M
// aligned 4 KiB blocks, for several BLOCK ORDERS and wave counts per CU:
//
//   order 0  wave w of workgroup g: units w, w + W, ... (16 waves: blocks
//            (k G + g) 16 + w -- all waves of a CU in one 64 KiB row at a time)
//   order 1  run_lp's desks of 8: wave w takes desks w, w + W, ... of its
//            workgroup; desk j = units 8 j .. 8 j + 7, unit u = block
//            ((u / 16) G + g) 16 + u % 16 (half a row per desk: a CU reads
//            W / 2 rows 16 MiB apart at a time)
//   order 2  desks of 8 whose lanes are 16 units apart: wave w at step i
//            reads block row 8 (i / 8) + i % 8 of round ... (round 3's
//            "rounds of 16")
//   order 3  desks of 4 (order 1 with 4-unit desks)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/order_probe.hip \
//         -o scripts/probes/order_probe && scripts/probes/order_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                       \
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

// the i-th block wave w of workgroup g reads (W waves, G workgroups), or
// >= count when done
__device__ __forceinline__ uint64_t block_of(int order, uint64_t i, uint32_t w, uint32_t W,
                                             uint32_t g, uint32_t G) {
  const uint32_t D = order == 3 ? 4u : 8u;
  uint64_t u;
  if (order == 0) {
    u = i * W + w;  // (16 waves: one row per step)
  } else if (order == 2) {
    // round r = i / 8 holds 16 waves x 8 lanes; lane t of wave w: unit
    // r * 8 W + w + W t
    u = (i / 8u) * 8u * W + w + uint64_t(W) * (i % 8u);
  } else {
    u = (uint64_t(w) + uint64_t(W) * (i / D)) * D + i % D;
  }
  return ((u / 16u) * G + g) * 16u + u % 16u;
}

__global__ __launch_bounds__(1024) void skel_kernel(const uint8_t* __restrict__ data, int order,
                                                    uint64_t count, uint32_t* __restrict__ out) {
  const uint32_t l = threadIdx.x & 63u, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = blockDim.x / 64u, g = blockIdx.x, G = gridDim.x;
  const uint32_t slot = 98304u + w * 4096u;
  const uint64_t base = reinterpret_cast<uint64_t>(data);
  // blocks per wave: the count is a multiple of G * 16 * 8
  const uint64_t per = count / (uint64_t(G) * W);
  uint64_t i = 0;
  uint64_t b = block_of(order, i, w, W, g, G);
  dma4(base + __builtin_amdgcn_readfirstlane(b) * 4096u, slot, 16u * l, 16u * l + 1024u,
       16u * l + 2048u, 16u * l + 3072u);
  uint32_t acc = 0;
  for (;;) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(slot + 1024u * q + 16u * l));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ++i;
    if (i < per) {
      b = block_of(order, i, w, W, g, G);
      dma4(base + __builtin_amdgcn_readfirstlane(b) * 4096u, slot, 16u * l, 16u * l + 1024u,
           16u * l + 2048u, 16u * l + 3072u);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    if (i >= per) break;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep the loads
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  // a multiple of grid * 16 * 8 blocks near 1 M: every order covers each
  // block once for W = 16, 12 and 8 waves (per wave: count / (grid W))
  const uint64_t unit = uint64_t(grid) * 16u * 8u * 3u;
  const uint64_t count = ((uint64_t(1) << 20) / unit) * unit;
  const int reps = 50;
  uint8_t* d;
  CK(hipMalloc(&d, count * 4096u + 4096u));
  CK(hipMemset(d, 0x5a, count * 4096u));
  uint32_t* out;
  CK(hipMalloc(&out, grid * 4));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(skel_kernel),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 150; ++i) skel_kernel<<<grid, 1024, 163840>>>(d, 0, count, out);
  const int waves[] = {16, 12, 8};
  for (int order = 0; order < 4; ++order) {
    for (int W : waves) {
      if (order == 2 && W != 16) continue;
      for (int i = 0; i < 10; ++i) skel_kernel<<<grid, 64 * W, 163840>>>(d, order, count, out);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) skel_kernel<<<grid, 64 * W, 163840>>>(d, order, count, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      printf("{\"order\": %d, \"waves\": %d, \"blocks\": %llu, \"ms\": %.4f, \"TBps\": %.3f}\n", order,
             W, (unsigned long long)count, ms, count * 4096.0 / ms / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(d));
  return 0;
}
