// crc32c_util.hip -- auxiliary device kernels of the library (not the CRC
// path): the seeded bench/test data generator, the read-stream ceiling the
// roofline is compared with, and the bounds check of device descriptors.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wipdb {
namespace util {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Read-stream ceiling: one wave per fixed-size block, 16-byte nontemporal
// loads, XOR-reduced to 4 bytes per block (the same bytes in and out as the
// CRC kernels, no CRC work).  length must be a multiple of 16.
__global__ __launch_bounds__(1024) void readstream_kernel(const uint8_t* __restrict__ base,
                                                          uint64_t stride, uint32_t length,
                                                          uint32_t* __restrict__ out,
                                                          uint64_t count) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  const uint32_t chunks = length >> 4;
  for (uint64_t s = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
       s < count; s += nw) {
    const u32x4* p = reinterpret_cast<const u32x4*>(base + s * stride);
    uint32_t acc = 0;
    for (uint32_t i = lane; i < chunks; i += 64u) {
      const u32x4 v = __builtin_nontemporal_load(p + i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
    if (lane == 0u) out[s] = acc;
  }
}

// Seeded test/bench data: 64-bit word k = splitmix64(seed + (k+1)*gamma)
// (tests/golden/common.py), so any block can be regenerated on the host.
__global__ __launch_bounds__(256) void fill_splitmix64_kernel(uint64_t* __restrict__ dst,
                                                              uint64_t nwords,
                                                              uint64_t first_word,
                                                              uint64_t seed) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nwords;
       i += step) {
    uint64_t z = seed + (first_word + i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[i] = z ^ (z >> 31);
  }
}

// Bounds check of a device descriptor batch (hcrc_check_spans_async): span i
// is bad when offsets[i] + lengths[i] + extra > base_bytes (in 64 bits; an
// offset past base_bytes is bad whatever the length).  result[0] += the bad
// spans, result[1] = min(result[1], the lowest bad index); the caller
// initialises result to {0, ~0}.  One wave-level reduction per 64 spans, one
// pair of atomics per wave that found any.
__global__ __launch_bounds__(256) void check_spans_kernel(const uint64_t* __restrict__ offsets,
                                                          const uint32_t* __restrict__ lengths,
                                                          uint64_t count, uint64_t base_bytes,
                                                          uint32_t extra,
                                                          unsigned long long* result) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  unsigned long long bad = 0, first = ~0ull;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < count;
       i += step) {
    const uint64_t o = offsets[i];
    const uint64_t need = static_cast<uint64_t>(lengths[i]) + extra;
    if (o > base_bytes || need > base_bytes - o) {
      ++bad;
      first = first < i ? first : i;
    }
  }
  // wave reduction (64 lanes), then one atomic pair per wave
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) {
    bad += __shfl_xor(bad, k, 64);
    const unsigned long long f = __shfl_xor(first, k, 64);
    first = first < f ? first : f;
  }
  if ((threadIdx.x & 63u) == 0u && bad) {
    atomicAdd(result, bad);
    atomicMin(result + 1, first);
  }
}

}  // namespace util
}  // namespace wipdb
