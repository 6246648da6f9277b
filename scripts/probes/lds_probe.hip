// lds_probe.hip -- standalone probe (not product code): the LDS-staged
// memory skeleton for the spans kernel rebuild (round 2).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I wipdb_amd/csrc \
//         scripts/probes/lds_probe.hip -o build/lds_probe
//
// Kernels over 1 M x 4 KiB aligned blocks (4 GiB, device-generated):
//   stream   plain read stream, one wave per block (round-1 ceiling)
//   dma<M>   per-wave 4 KiB LDS slot filled by global_load_lds_dwordx4;
//            M=0 load-only (XOR), M=1 full CRC32C (rotated 8-replica
//            slicing-by-4 tables + per-lane fold tables)
// Prints kernel ms per launch (hipEvents, 30 warmup + 50 timed) and the
// CRC check of sampled blocks against a host Sarwate loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "gf2_crc32c.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t l_u32;
typedef __attribute__((address_space(3))) const u32x4 l_u32x4;

constexpr uint32_t kL2 = 0;          // [0, 32K)  L2 fold tables, 128-B rows
constexpr uint32_t kMain = 32768;    // [32K, 96K) slicing tables + L1 fold tables, 256-B rows
constexpr uint32_t kSlots = 98304;   // [96K, 160K) 16 wave slots of 4 KiB
constexpr uint32_t kImage = 98304;   // table image bytes
constexpr uint32_t kLds = 163840;
constexpr int kWaves = 16;

__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {
  return *reinterpret_cast<l_u32*>(static_cast<uintptr_t>(a));
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xF, 0xF, true));
}

struct LaneK {
  uint32_t sel[4];
  uint32_t km, k1, k2;
};

__device__ __forceinline__ LaneK lane_consts(uint32_t l) {
  LaneK k;
  const uint32_t q = (l >> 3) & 3u, rep = l & 7u, a = 7u - (l & 7u), c = 7u - (l >> 3);
  k.km = k.k1 = k.k2 = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t t = (j + q) & 3u;
    k.sel[j] = 0x0c0c0000u | (t << 8) | (4u + j);
    k.km |= (t * 32u + rep * 4u) << (8 * j);
    k.k1 |= (128u + (a * 4u + t) * 4u) << (8 * j);
    k.k2 |= (8u * (c * 4u + t)) << (8 * j);
  }
  return k;
}

// one slicing-by-4 step in x form: returns L(x) ^ wn
__device__ __forceinline__ uint32_t step(const LaneK& k, uint32_t x, uint32_t wn) {
  const uint32_t a0 = lds_ld(kMain + __builtin_amdgcn_perm(k.km, x, k.sel[0]));
  const uint32_t a1 = lds_ld(kMain + __builtin_amdgcn_perm(k.km, x, k.sel[1]));
  const uint32_t a2 = lds_ld(kMain + __builtin_amdgcn_perm(k.km, x, k.sel[2]));
  const uint32_t a3 = lds_ld(kMain + __builtin_amdgcn_perm(k.km, x, k.sel[3]));
  return xor3(xor3(a0, a1, a2), a3, wn);
}
__device__ __forceinline__ uint32_t fold_l1(const LaneK& k, uint32_t r) {
  const uint32_t a0 = lds_ld(kMain + __builtin_amdgcn_perm(k.k1, r, k.sel[0]));
  const uint32_t a1 = lds_ld(kMain + __builtin_amdgcn_perm(k.k1, r, k.sel[1]));
  const uint32_t a2 = lds_ld(kMain + __builtin_amdgcn_perm(k.k1, r, k.sel[2]));
  const uint32_t a3 = lds_ld(kMain + __builtin_amdgcn_perm(k.k1, r, k.sel[3]));
  return xor3(a0, a1, a2) ^ a3;
}
__device__ __forceinline__ uint32_t fold_l2(const LaneK& k, uint32_t r) {
  const uint32_t a0 = lds_ld(kL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[0]) >> 1));
  const uint32_t a1 = lds_ld(kL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[1]) >> 1));
  const uint32_t a2 = lds_ld(kL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[2]) >> 1));
  const uint32_t a3 = lds_ld(kL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[3]) >> 1));
  return xor3(a0, a1, a2) ^ a3;
}

// DMA one 4 KiB segment (16-B aligned at `src`) into the wave's slot:
// 4 x global_load_lds_dwordx4, lane m of load q reads chunk 64q + c_m.
template <bool NT>
__device__ __forceinline__ void dma_seg(const uint8_t* src, uint32_t slot, const uint32_t (&voff)[4]) {
  uint32_t keep;
#define DMA_ASM(NTS)                                        \
  asm volatile(                                             \
      "s_mov_b32 %0, m0\n\t"                                 \
      "s_mov_b32 m0, %5\n\t"                                 \
      "s_nop 0\n\t"                                          \
      "global_load_lds_dwordx4 %1, %6" NTS "\n\t"              \
      "s_add_u32 m0, m0, 0x400\n\t"                          \
      "s_nop 0\n\t"                                          \
      "global_load_lds_dwordx4 %2, %6" NTS "\n\t"              \
      "s_add_u32 m0, m0, 0x400\n\t"                          \
      "s_nop 0\n\t"                                          \
      "global_load_lds_dwordx4 %3, %6" NTS "\n\t"              \
      "s_add_u32 m0, m0, 0x400\n\t"                          \
      "s_nop 0\n\t"                                          \
      "global_load_lds_dwordx4 %4, %6" NTS "\n\t"              \
      "s_mov_b32 m0, %0"                                    \
      : "=&s"(keep)                                         \
      : "v"(voff[0]), "v"(voff[1]), "v"(voff[2]), "v"(voff[3]), "s"(slot), "s"(src) \
      : "memory")
  if (NT) DMA_ASM(" nt");
  else DMA_ASM("");
#undef DMA_ASM
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// MODE 0: load-only, MODE 1: CRC
template <int MODE, bool NT, bool SHARE = false>
__global__ __launch_bounds__(1024) void dma_kernel(const uint8_t* __restrict__ data, uint64_t count,
                                                   const u32x4* __restrict__ image,
                                                   uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x, l = tid & 63u, w = uni(tid >> 6);
  if (MODE == 1) {
    u32x4* li = reinterpret_cast<u32x4*>(lds);
    for (uint32_t i = tid; i < kImage / 16; i += 1024) li[i] = image[i];
  }
  typedef __attribute__((address_space(3))) uint32_t l_u32w;
  l_u32w* ctr = reinterpret_cast<l_u32w*>(static_cast<uintptr_t>(kL2 + 0));  // probe only: clobbers L2 row 0 entry c=0,p=0 (identity, unused)
  if (SHARE && tid == 0) *ctr = 0;
  __syncthreads();
  const uint64_t rstride = uint64_t(gridDim.x) * 16u;
  auto grab = [&]() -> uint64_t {
    uint32_t u = 0;
    if (l == 0) u = __atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED);
    u = uni(u);
    return uint64_t(u >> 4) * rstride + 16u * blockIdx.x + (u & 15u);
  };
  const LaneK k = lane_consts(l);
  const uint32_t slot = kSlots + w * 4096u;
  // lane m of load q: chunk 64q + 4(m>>2) + (((m&3) - (m>>4)) & 3)
  const uint32_t cm = 4u * (l >> 2) + (((l & 3u) - (l >> 4)) & 3u);
  uint32_t voff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) voff[q] = cm * 16u + 1024u * q;
  // read: lane l, step i: position 4l + ((i + (l>>2)) & 3)
  uint32_t rpos[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) rpos[i] = slot + 16u * (4u * l + ((i + (l >> 2)) & 3u));
  const uint64_t nw = uint64_t(gridDim.x) * kWaves;
  uint64_t s = SHARE ? grab() : uint64_t(blockIdx.x) * kWaves + w;
  if (s >= count) return;
  dma_seg<NT>(data + s * 4096u, slot, voff);
  bool first = true;
  for (;;) {
    const uint64_t sn = SHARE ? grab() : s + nw;
    // pending: this span's 4 loads, then (after the first) the previous store
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    first = false;
    u32x4 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(rpos[i]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (sn < count) dma_seg<NT>(data + sn * 4096u, slot, voff);
    uint32_t res;
    if (MODE == 0) {
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) x ^= d[i].x ^ d[i].y ^ d[i].z ^ d[i].w;
      x ^= dpp<0xB1>(x);
      res = uni(x);
    } else {
      uint32_t W[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        W[4 * i] = d[i].x;
        W[4 * i + 1] = d[i].y;
        W[4 * i + 2] = d[i].z;
        W[4 * i + 3] = d[i].w;
      }
      uint32_t x = (l == 0u ? 0xffffffffu : 0u) ^ W[0];
#pragma unroll
      for (int i = 0; i < 15; ++i) x = step(k, x, W[i + 1]);
      uint32_t r = step(k, x, 0u);
      uint32_t v = fold_l1(k, r);
      v ^= dpp<0xB1>(v);
      v ^= dpp<0x4E>(v);
      v ^= dpp<0x104>(v);
      uint32_t wv = 0;
      if ((l & 7u) == 0u) {
        const uint32_t f = fold_l2(k, v);
        wv = (l >> 3) == 7u ? v : f;  // c = 0: identity (its LDS column holds the counter)
      }
      wv ^= dpp<0x108>(wv);
      const uint32_t R = __builtin_amdgcn_readlane(wv, 0) ^ __builtin_amdgcn_readlane(wv, 16) ^
                         __builtin_amdgcn_readlane(wv, 32) ^ __builtin_amdgcn_readlane(wv, 48);
      res = ~R;
    }
    if (l == 0u) out[s] = res;
    if (sn >= count) break;
    s = sn;
  }
}

__global__ __launch_bounds__(1024) void stream_kernel(const uint8_t* __restrict__ data, uint64_t count,
                                                      uint32_t* __restrict__ out) {
  const uint32_t l = threadIdx.x & 63u;
  const uint64_t nw = uint64_t(gridDim.x) * kWaves;
  for (uint64_t s = uint64_t(blockIdx.x) * kWaves + (threadIdx.x >> 6); s < count; s += nw) {
    const u32x4* p = reinterpret_cast<const u32x4*>(data + s * 4096u);
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __builtin_nontemporal_load(p + l + 64 * i);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    x ^= dpp<0xB1>(x);
    if (l == 0) out[s] = x;
  }
}

__global__ void fill_kernel(uint64_t* dst, uint64_t n, uint64_t seed) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[i] = z ^ (z >> 31);
  }
}

static void build_image(std::vector<uint32_t>& img) {
  using namespace wipdb::gf2;
  Tables T;
  BuildTables(&T);
  img.assign(kImage / 4, 0);
  // L2: row b at b*128: (c, p) at (c*4+p)*4, shift by 512c
  for (int c = 0; c < 8; ++c) {
    uint32_t sh[4][256];
    BuildShiftTable(uint64_t(512) * c, sh);
    for (int p = 0; p < 4; ++p)
      for (int b = 0; b < 256; ++b) img[(kL2 + b * 128 + (c * 4 + p) * 4) / 4] = sh[p][b];
  }
  for (int b = 0; b < 256; ++b)
    for (int t = 0; t < 4; ++t)
      for (int rep = 0; rep < 8; ++rep) img[(kMain + b * 256 + t * 32 + rep * 4) / 4] = T.t[3 - t][b];
  for (int a = 0; a < 8; ++a) {
    uint32_t sh[4][256];
    BuildShiftTable(uint64_t(64) * a, sh);
    for (int p = 0; p < 4; ++p)
      for (int b = 0; b < 256; ++b) img[(kMain + b * 256 + 128 + (a * 4 + p) * 4) / 4] = sh[p][b];
  }
}

static uint32_t host_crc(const uint8_t* p, size_t n) {
  static uint32_t t[256];
  static bool init = false;
  if (!init) {
    for (int i = 0; i < 256; ++i) t[i] = wipdb::gf2::ByteStepSlow(0, uint8_t(i));
    init = true;
  }
  uint32_t r = ~0u;
  for (size_t i = 0; i < n; ++i) r = t[(r ^ p[i]) & 0xff] ^ (r >> 8);
  return ~r;
}

int main(int argc, char** argv) {
  const uint64_t count = argc > 1 ? strtoull(argv[1], 0, 0) : (1u << 20);
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  const uint64_t bytes = count * 4096;
  uint8_t* d;
  uint32_t *o, *img_d;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&o, count * 4));
  CK(hipMalloc(&img_d, kImage));
  std::vector<uint32_t> img;
  build_image(img);
  CK(hipMemcpy(img_d, img.data(), kImage, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(d), bytes / 8, 0x4B10C5ull);
  CK(hipDeviceSynchronize());
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipFuncSetAttribute((const void*)dma_kernel<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  CK(hipFuncSetAttribute((const void*)dma_kernel<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  CK(hipFuncSetAttribute((const void*)dma_kernel<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  CK(hipFuncSetAttribute((const void*)dma_kernel<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  CK(hipFuncSetAttribute((const void*)dma_kernel<1, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 30; ++i) launch();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double alg = double(count) * 4100.0;
    printf("%-12s %.4f ms  %.3f TB/s alg  frac %.4f\n", name, ms, alg / ms / 1e9, alg / ms / 1e9 / 8.0);
    fflush(stdout);
  };
  const dim3 grid(ncu), blk(1024);
  run("stream", [&] { hipLaunchKernelGGL(stream_kernel, grid, blk, 0, 0, d, count, o); });
  run("dma0", [&] { hipLaunchKernelGGL((dma_kernel<0, false>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  run("dma0nt", [&] { hipLaunchKernelGGL((dma_kernel<0, true>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  run("dma1", [&] { hipLaunchKernelGGL((dma_kernel<1, false>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  CK(hipDeviceSynchronize());
  // check sampled CRCs
  std::vector<uint32_t> ho(count);
  CK(hipMemcpy(ho.data(), o, count * 4, hipMemcpyDeviceToHost));
  std::vector<uint8_t> blkb(4096);
  int bad = 0, checked = 0;
  for (uint64_t s = 0; s < count; s += (s < 4096 ? 1 : 997)) {
    CK(hipMemcpy(blkb.data(), d + s * 4096, 4096, hipMemcpyDeviceToHost));
    const uint32_t want = host_crc(blkb.data(), 4096);
    if (want != ho[s]) {
      if (bad < 5) printf("mismatch span %llu: got %08x want %08x\n", (unsigned long long)s, ho[s], want);
      ++bad;
    }
    ++checked;
  }
  printf("dma1 check: %d/%d bad\n", bad, checked);
  run("dma1nt", [&] { hipLaunchKernelGGL((dma_kernel<1, true>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  run("dma1ntsh", [&] { hipLaunchKernelGGL((dma_kernel<1, true, true>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ho.data(), o, count * 4, hipMemcpyDeviceToHost));
  for (uint64_t s = 0; s < count; s += (s < 4096 ? 1 : 997)) {
    CK(hipMemcpy(blkb.data(), d + s * 4096, 4096, hipMemcpyDeviceToHost));
    if (host_crc(blkb.data(), 4096) != ho[s]) ++bad;
  }
  printf("dma1ntsh check: %d bad (cumulative)\n", bad);
  run("dma1nt", [&] { hipLaunchKernelGGL((dma_kernel<1, true>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  run("dma1ntsh", [&] { hipLaunchKernelGGL((dma_kernel<1, true, true>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  run("dma0nt", [&] { hipLaunchKernelGGL((dma_kernel<0, true>), grid, blk, kLds, 0, d, count, (const u32x4*)img_d, o); });
  run("stream", [&] { hipLaunchKernelGGL(stream_kernel, grid, blk, 0, 0, d, count, o); });
  return bad ? 1 : 0;
}
