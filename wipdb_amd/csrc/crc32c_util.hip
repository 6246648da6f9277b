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
  uint64_t s = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (chunks == 256u) {
    // 4 KiB blocks (the headline's): two blocks per iteration, all 8 of a
    // lane's 16-byte loads issued before any is used (a ceiling needs bytes
    // in flight, not one block's 4 loads at a time)
    for (; s + nw < count; s += 2u * nw) {
      const u32x4* p = reinterpret_cast<const u32x4*>(base + s * stride) + lane;
      const u32x4* q = reinterpret_cast<const u32x4*>(base + (s + nw) * stride) + lane;
      u32x4 v[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = __builtin_nontemporal_load(p + 64 * k);
        v[4 + k] = __builtin_nontemporal_load(q + 64 * k);
      }
      uint32_t a = 0, b = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        b ^= v[4 + k].x ^ v[4 + k].y ^ v[4 + k].z ^ v[4 + k].w;
      }
#pragma unroll
      for (int k = 32; k >= 1; k >>= 1) {
        a ^= __shfl_xor(a, k, 64);
        b ^= __shfl_xor(b, k, 64);
      }
      if (lane == 0u) {
        out[s] = a;
        out[s + nw] = b;
      }
    }
  }
  for (; s < count; s += nw) {
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

// ---------------------------------------------------------------------------
// Byte-balanced workgroup ranges (HCRC_BALANCE): workgroup g of the spans
// kernel takes the contiguous spans [bounds[g], bounds[g + 1]), cut where
// the running weight (length + 64 per span: bytes plus a per-span cost)
// crosses g / G of the total.  The default deal (16-span blocks round robin)
// gives every workgroup the same NUMBER of spans; on config 3's Zipf mix
// that is max / mean 1.17 bytes per workgroup over 256 of them
// (scripts/balance_model.py), the measured wave-lifetime spread 1.15.
// Span i goes to the workgroup g with excl(i) in [t(g), t(g + 1)), t(g) =
// g T / G, so bounds[g] = #{i : excl(i) < t(g)} (monotone; every span once).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), d, 64);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), d, 64);
    v += (static_cast<uint64_t>(hi) << 32) | lo;
  }
  return v;
}
// 256 threads: the exclusive prefix of v over the block, and the total.
__device__ __forceinline__ uint64_t block_excl64(uint64_t v, uint64_t* sh, uint64_t& total) {
  const uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
#pragma unroll
  for (uint32_t d = 1; d < 256; d <<= 1) {
    const uint64_t u = t >= d ? sh[t - d] : 0u;
    __syncthreads();
    sh[t] += u;
    __syncthreads();
  }
  total = sh[255];
  const uint64_t incl = sh[t];
  __syncthreads();
  return incl - v;
}

// Pass 1: sums[c] = weight of chunk c (spans [c C, c C + C)).
__global__ __launch_bounds__(256) void balance_sums_kernel(const uint32_t* __restrict__ len,
                                                           uint64_t n, uint32_t C,
                                                           uint64_t* __restrict__ sums) {
  __shared__ uint64_t red[4];
  const uint64_t lo = static_cast<uint64_t>(blockIdx.x) * C;
  const uint64_t hi = lo + C < n ? lo + C : n;
  uint64_t s = 0;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += 256u) s += len[i] + 64u;
  s = wave_sum64(s);
  if ((threadIdx.x & 63u) == 0u) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0u) sums[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Pass 2: one block per cut g = 1 .. G - 1 (bounds[0] = 0, bounds[G] = n
// written by the first).  The chunk holding t(g) from the chunk sums, then
// the spans of that chunk below t(g).
__global__ __launch_bounds__(256) void balance_bounds_kernel(
    const uint32_t* __restrict__ len, uint64_t n, uint32_t C, const uint64_t* __restrict__ sums,
    uint32_t nb, uint32_t G, uint32_t* __restrict__ bounds) {
  __shared__ uint64_t sh[256];
  __shared__ uint32_t cnt_sh[4];
  __shared__ uint64_t chunk_base;
  const uint32_t t = threadIdx.x, g = blockIdx.x + 1u;
  if (g == 1u && t == 0u) {
    bounds[0] = 0u;
    bounds[G] = static_cast<uint32_t>(n);
  }
  // chunk level: thread t holds chunks [b0, b1)
  const uint32_t k = (nb + 255u) / 256u;
  const uint32_t b0 = t * k < nb ? t * k : nb, b1 = b0 + k < nb ? b0 + k : nb;
  uint64_t loc = 0;
  for (uint32_t b = b0; b < b1; ++b) loc += sums[b];
  uint64_t T = 0;
  const uint64_t e0 = block_excl64(loc, sh, T);
  const uint64_t target = (T / G) * g + (T % G) * g / G;
  uint32_t cnt = 0;
  uint64_t e = e0;
  for (uint32_t b = b0; b < b1; ++b) {
    cnt += e < target ? 1u : 0u;
    e += sums[b];
  }
  // chunks with excl < target: count over the block (>= 1: chunk 0 starts at 0)
  uint32_t c = cnt;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((t & 63u) == 0u) cnt_sh[t >> 6] = c;
  __syncthreads();
  const uint32_t chunk = cnt_sh[0] + cnt_sh[1] + cnt_sh[2] + cnt_sh[3] - 1u;
  if (chunk >= b0 && chunk < b1) {  // its owner: the chunk's exclusive weight
    uint64_t x = e0;
    for (uint32_t b = b0; b < chunk; ++b) x += sums[b];
    chunk_base = x;
  }
  __syncthreads();
  const uint64_t base_e = chunk_base;
  __syncthreads();
  // span level inside the chunk: thread t holds spans [s0, s1)
  const uint64_t lo = static_cast<uint64_t>(chunk) * C;
  const uint64_t hi = lo + C < n ? lo + C : n;
  const uint64_t m = (hi - lo + 255u) / 256u;
  const uint64_t s0 = lo + t * m < hi ? lo + t * m : hi, s1 = s0 + m < hi ? s0 + m : hi;
  uint64_t w = 0;
  for (uint64_t i = s0; i < s1; ++i) w += len[i] + 64u;
  uint64_t T2 = 0;
  uint64_t x = base_e + block_excl64(w, sh, T2);
  uint32_t below = 0;
  for (uint64_t i = s0; i < s1; ++i) {
    below += x < target ? 1u : 0u;
    x += len[i] + 64u;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) below += __shfl_xor(below, d, 64);
  if ((t & 63u) == 0u) cnt_sh[t >> 6] = below;
  __syncthreads();
  if (t == 0u)
    bounds[g] = static_cast<uint32_t>(lo) + cnt_sh[0] + cnt_sh[1] + cnt_sh[2] + cnt_sh[3];
}

}  // namespace util
}  // namespace wipdb
