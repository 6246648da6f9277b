// inflight_probe.hip -- standalone probe (not product code): how much does
// per-iteration compute cost the spans kernel's memory pipeline, and would a
// second LDS slot per wave (two segments in flight) buy it back?
//
// The load-only skeleton of the spans kernel (per-wave 4 KiB LDS slots
// filled by 4 global_load_lds_dwordx4 of 1 KiB, waves take 4 KiB blocks
// round robin) with N dependent VALU ops of fake compute after each segment's
// read + next DMA issue; slots = 1 (the kernel today: the next DMA goes out
// when the slot has been read) or 2 (ping-pong: the DMA two segments ahead is
// in flight while a segment computes), waves = 16 or 8 per CU.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/inflight_probe.hip \
//         -o scripts/probes/inflight_probe && scripts/probes/inflight_probe
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

__device__ __forceinline__ void dma4(uint64_t base, uint32_t slot, uint32_t o0) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3 offset:1024 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3 offset:2048 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3 offset:3072 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(o0), "s"(slot), "s"(base)
      : "memory", "scc");
}

__device__ __forceinline__ uint32_t read_slot(uint32_t slot, uint32_t l) {
  u32x4 v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    v[q] = *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(slot + 1024u * q + 16u * l));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint32_t a = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) a ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
  return a;
}

// n (multiple of 8) dependent full-rate VALU ops (rotate + add)
__device__ __forceinline__ uint32_t fake(uint32_t a, uint32_t n) {
  for (uint32_t i = 0; i < n; i += 8) {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) a = __builtin_amdgcn_alignbit(a, a, 31u) + (i + k);
  }
  return a;
}

template <int SLOTS>
__global__ __launch_bounds__(1024) void skel(const uint8_t* __restrict__ data, uint64_t count,
                                             uint32_t n, uint32_t* __restrict__ out) {
  const uint32_t l = threadIdx.x & 63u, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = blockDim.x >> 6;
  const uint32_t slot0 = w * 4096u * SLOTS;
  const uint64_t stride = uint64_t(gridDim.x) * nw;
  uint64_t b = uint64_t(blockIdx.x) * nw + w;
  if (b >= count) return;
  const uint64_t base = reinterpret_cast<uint64_t>(data);
  uint32_t acc = l;
  if (SLOTS == 1) {
    dma4(base + b * 4096u, slot0, 16u * l);
    for (;;) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc ^= read_slot(slot0, l);
      b += stride;
      if (b < count) dma4(base + b * 4096u, slot0, 16u * l);
      acc = fake(acc, n);
      if (b >= count) break;
    }
  } else {
    // ping-pong: slot A holds segment b, slot B segment b + stride
    dma4(base + b * 4096u, slot0, 16u * l);
    uint64_t b1 = b + stride;
    const bool two = b1 < count;
    if (two) dma4(base + b1 * 4096u, slot0 + 4096u, 16u * l);
    uint32_t cur = 0;  // slot index of the oldest segment
    uint64_t pending = two ? 2 : 1;
    uint64_t next = b1 + stride;
    while (pending) {
      if (pending == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t s = slot0 + 4096u * cur;
      acc ^= read_slot(s, l);
      --pending;
      if (next < count) {
        dma4(base + next * 4096u, s, 16u * l);
        next += stride;
        ++pending;
      }
      cur ^= 1u;
      acc = fake(acc, n);
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keep the loads
}

__global__ void fill_kernel(uint64_t* dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
       i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    dst[i] = z ^ (z >> 31);
  }
}

int main(int argc, char** argv) {
  const uint64_t count = argc > 1 ? strtoull(argv[1], 0, 0) : (1u << 20);
  const int reps = 30;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  uint8_t* d;
  const uint64_t bytes = count * 4096u;
  CK(hipMalloc(&d, bytes));
  fill_kernel<<<4096, 256>>>(reinterpret_cast<uint64_t*>(d), bytes / 8);
  uint32_t* out;
  CK(hipMalloc(&out, grid * 4));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(skel<1>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(skel<2>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 150; ++i) skel<1><<<grid, 1024, 163840>>>(d, count, 0, out);
  struct Cfg { int slots, waves; };
  const Cfg cfgs[] = {{1, 16}, {2, 16}, {1, 8}, {2, 8}};
  const uint32_t ns[] = {0, 128, 256, 384, 512, 768, 1024};
  for (const Cfg& c : cfgs) {
    for (uint32_t n : ns) {
      auto launch = [&]() {
        if (c.slots == 1) skel<1><<<grid, 64 * c.waves, 163840>>>(d, count, n, out);
        else skel<2><<<grid, 64 * c.waves, 163840>>>(d, count, n, out);
      };
      for (int i = 0; i < 5; ++i) launch();
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      printf("{\"slots\": %d, \"waves\": %d, \"valu_ops\": %u, \"ms\": %.4f, \"TBps\": %.3f}\n",
             c.slots, c.waves, n, ms, count * 4096.0 / ms / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(d));
  return 0;
}
