// crc32c_util.hip -- auxiliary device kernels of the library: the seeded
// bench/test data generator, the read-stream ceiling the roofline is
// compared with, the bounds check of device descriptors, and the expand /
// combine passes of long spans in device batches (HCRC_SPLIT_LONG).
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

// ---------------------------------------------------------------------------
// Long spans in device batches (HCRC_SPLIT_LONG).  A span's segments are
// chained on one wave (~2.5 GiB/s for a lone span), so a span of at least
// `thresh` bytes is cut into parts of `part` bytes (the first part takes the
// remainder) that run as independent spans on many waves, and their
// registers are combined by linearity, as crc32c_3way's CombineCRC does
// (kv/src/util/crc32c.cc:640-657; gf2_crc32c.h):
//   part 0 runs with the span's init (returns Extend(init, p0) = ~feed(~init, p0)),
//   part j >= 1 from init ~0 (returns ~feed(0, p_j)),
//   feed(~init, span) = XOR_j feed(., p_j) * x^(8 part (m - 1 - j)).
// ---------------------------------------------------------------------------

// a * b mod P, reflected CRC-32C polynomials (gf2::MulMod)
__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    p ^= (a & (0x80000000u >> i)) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? 0x82F63B78u : 0u);
  }
  return p;
}
__device__ __forceinline__ uint32_t powmod(uint32_t k, uint64_t e) {
  uint32_t r = 0x80000000u;  // x^0
  while (e) {
    if (e & 1u) r = mulmod(r, k);
    k = mulmod(k, k);
    e >>= 1;
  }
  return r;
}

// wave-inclusive prefix sum (64 lanes)
__device__ __forceinline__ uint32_t wave_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    if (lane >= static_cast<uint32_t>(d)) v += u;
  }
  return v;
}

// Expand: every span becomes one list entry (id = its index), or -- long
// spans, while the part pool lasts -- its parts (ids count + slot ..).
// first[i] = the span's first part slot, or ~0 if it is not split.  The
// split spans' indices go to split_idx.  counters: [0] list entries,
// [1] part slots taken, [2] split spans.  One atomic per wave per counter.
__global__ __launch_bounds__(256) void split_expand_kernel(
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
    const uint32_t* __restrict__ init, uint64_t count, uint32_t part, uint32_t thresh,
    uint32_t cap, uint64_t* __restrict__ l_off, uint32_t* __restrict__ l_len,
    uint32_t* __restrict__ l_init, uint32_t* __restrict__ l_id, uint32_t* __restrict__ first,
    uint32_t* __restrict__ split_idx, uint32_t* counters) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * blockDim.x + (threadIdx.x & ~63u);
       base < count; base += step) {
    const uint64_t i = base + lane;
    const bool live = i < count;
    const uint32_t n = live ? len[i] : 0u;
    // (64-bit: a length near 4 GiB must not wrap)
    uint32_t m = (live && n >= thresh)
                     ? static_cast<uint32_t>((static_cast<uint64_t>(n) + part - 1u) / part)
                     : (live ? 1u : 0u);
    // part slots for the long ones
    const uint32_t want = m > 1u ? m : 0u;
    const uint32_t incl = wave_scan(want, lane);
    const uint32_t tot = __shfl(incl, 63, 64);
    uint32_t s0 = 0;
    if (lane == 0u && tot) s0 = atomicAdd(counters + 1, tot);
    s0 = __shfl(s0, 0, 64);
    uint32_t slot = s0 + incl - want;
    if (want && slot + want > cap) m = 1u;  // pool exhausted: not split
    const bool split = m > 1u;
    // list entries
    const uint32_t incl2 = wave_scan(m, lane);
    const uint32_t tot2 = __shfl(incl2, 63, 64);
    uint32_t p0 = 0;
    if (lane == 0u && tot2) p0 = atomicAdd(counters, tot2);
    p0 = __shfl(p0, 0, 64);
    uint32_t pos = p0 + incl2 - m;
    // split-span list
    const uint32_t incl3 = wave_scan(split ? 1u : 0u, lane);
    const uint32_t tot3 = __shfl(incl3, 63, 64);
    uint32_t q0 = 0;
    if (lane == 0u && tot3) q0 = atomicAdd(counters + 2, tot3);
    q0 = __shfl(q0, 0, 64);
    if (!live) continue;
    const uint64_t o = off[i];
    const uint32_t ini = init ? init[i] : 0u;
    if (!split) {
      l_off[pos] = o;
      l_len[pos] = n;
      l_init[pos] = ini;
      l_id[pos] = static_cast<uint32_t>(i);
      first[i] = ~0u;
      continue;
    }
    first[i] = slot;
    split_idx[q0 + incl3 - 1u] = static_cast<uint32_t>(i);
    const uint32_t p_first = n - (m - 1u) * part;  // 1 .. part
    const uint32_t id0 = static_cast<uint32_t>(count) + slot;
    l_off[pos] = o;
    l_len[pos] = p_first;
    l_init[pos] = ini;
    l_id[pos] = id0;
    for (uint32_t j = 1; j < m; ++j) {
      l_off[pos + j] = o + p_first + static_cast<uint64_t>(j - 1u) * part;
      l_len[pos + j] = part;
      l_init[pos + j] = ~0u;
      l_id[pos + j] = id0 + j;
    }
  }
}

// Unsplit spans: out[i] = tmp[i] (masked when asked).
__global__ __launch_bounds__(256) void split_copy_kernel(const uint32_t* __restrict__ tmp,
                                                         const uint32_t* __restrict__ first,
                                                         uint32_t* __restrict__ out,
                                                         uint64_t count, uint32_t mask) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < count;
       i += step) {
    if (first[i] != ~0u) continue;
    const uint32_t v = tmp[i];
    out[i] = mask ? ((v >> 15) | (v << 17)) + 0xa282ead8u : v;
  }
}

// Split spans: one wave each.  Lane l takes parts j = l, l + 64, ..., from
// the last one down, with term_j = ~tmp[part j] * K^(m - 1 - j), K =
// x^(8 part) (kpart); the running power steps by K^64.  XOR over the lanes.
__global__ __launch_bounds__(256) void split_combine_kernel(
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ first,
    const uint32_t* __restrict__ split_idx, const uint32_t* __restrict__ counters,
    const uint32_t* __restrict__ tmp, uint32_t* __restrict__ out, uint64_t count, uint32_t part,
    uint32_t kpart, uint32_t mask) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nsplit = counters[2];
  const uint32_t w0 = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (w0 >= nsplit) return;  // (most waves of a batch with few long spans)
  const uint32_t k64 = powmod(kpart, 64);
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t w = w0; w < nsplit; w += nw) {
    const uint32_t i = split_idx[w];
    const uint32_t m = static_cast<uint32_t>((static_cast<uint64_t>(len[i]) + part - 1u) / part);
    const uint32_t* t = tmp + count + first[i];
    uint32_t acc = 0;
    if (lane < m) {
      // this lane's last part: the largest j = lane + 64 k < m
      const uint32_t jl = lane + ((m - 1u - lane) / 64u) * 64u;
      uint32_t pw = powmod(kpart, m - 1u - jl);
      for (int64_t j = jl; j >= 0; j -= 64) {
        acc ^= mulmod(~t[j], pw);
        pw = mulmod(pw, k64);
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc ^= __shfl_xor(acc, d, 64);
    if (lane == 0u) {
      const uint32_t v = ~acc;
      out[i] = mask ? ((v >> 15) | (v << 17)) + 0xa282ead8u : v;
    }
  }
}

}  // namespace util
}  // namespace wipdb
