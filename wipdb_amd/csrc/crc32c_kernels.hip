// crc32c_kernels.hip -- hand-written CDNA4 (gfx950) kernels for batched
// CRC32C of WipDB table blocks.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// crc32c.cc:1225-1227) applied to every block span, as WriteRawBlock
// (kv/src/table/table_builder.cc:194-196) and ReadBlock
// (kv/src/table/format.cc:91-93) do one block at a time.
//
// Design (DESIGN.md "Kernels"):
//   * one span per wavefront; 64 lanes each CRC a contiguous stripe of
//     c 16-byte chunks of the span (16-byte loads, all bytes of every
//     fetched line used by the wave);
//   * CRC arithmetic is table-driven from LDS (no carry-less multiply exists
//     on CDNA4 and this is a byte scan, not a contraction: no MFMA):
//     slicing-by-2 tables replicated 32x so lane l always reads bank l --
//     every lookup is bank-conflict free -- and the LDS address of a lookup is
//     built by ONE v_perm_b32 (table byte, lane byte, table-select bit);
//   * the 64 stripe registers are folded by a 6-level wavefront butterfly:
//     register(l) = shift(register(l), stripe bytes * 2^k) ^ register(l+2^k),
//     where shift by 16*2^j bytes is 4 lookups in a GF(2) "multiply by
//     x^(8*16*2^j)" table (the carry-less combine of the reference's
//     CombineCRC, crc32c.cc:640-657, done with tables);
//   * unaligned starts: the first chunk's leading bytes are zeroed and the
//     initial register is pre-un-shifted (x^(-8h)) so it equals ~init at the
//     first real byte; ragged ends (< 16 bytes) are fed by the wave after the
//     fold.  So any offset/length/init is bit-exact.
//   * persistent grid: 1 workgroup of 16 waves per CU (LDS = 116 KiB), waves
//     stride over spans.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace wipdb {
namespace dev {

// ---------------------------------------------------------------------------
// LDS helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_u32(const uint8_t* lds, uint32_t addr) {
  return *reinterpret_cast<const uint32_t*>(lds + addr);
}

// LDS address of table entry (sel, byte k of x) for this lane: one v_perm.
// s0 = lane constant: byte0 = (lane&31)*4 (T1), byte1 = (lane&31)*4|0x80 (T0).
__device__ __forceinline__ uint32_t main_addr(uint32_t s0, uint32_t x,
                                              uint32_t sel) {
  return __builtin_amdgcn_perm(s0, x, sel);
}
constexpr uint32_t kSelT1B0 = 0x0c0c0004u;  // [s0.b0, x.b0, 0, 0] -> T1[x.b0]
constexpr uint32_t kSelT0B1 = 0x0c0c0105u;  // [s0.b1, x.b1, 0, 0] -> T0[x.b1]

// Feed one little-endian 32-bit word into register r (slicing-by-2 twice).
__device__ __forceinline__ uint32_t feed_word(const uint8_t* lds, uint32_t s0,
                                              uint32_t r, uint32_t w) {
  uint32_t x = r ^ w;
  uint32_t y = lds_u32(lds, main_addr(s0, x, kSelT1B0)) ^
               lds_u32(lds, main_addr(s0, x, kSelT0B1)) ^ (x >> 16);
  return lds_u32(lds, main_addr(s0, y, kSelT1B0)) ^
         lds_u32(lds, main_addr(s0, y, kSelT0B1)) ^ (y >> 16);
}

// Feed one byte (Sarwate step with this lane's T0 replica).
__device__ __forceinline__ uint32_t feed_byte(const uint8_t* lds, uint32_t s0,
                                              uint32_t r, uint32_t b) {
  uint32_t x = (r ^ b) & 0xffu;
  uint32_t addr = (x << 8) | ((s0 >> 8) & 0xffu);
  return lds_u32(lds, addr) ^ (r >> 8);
}

// r * x^(8 * 16 * 2^j) mod P: 4 lookups in shift table j.
__device__ __forceinline__ uint32_t shift_pow2(const uint8_t* lds, uint32_t r,
                                               uint32_t j) {
  const uint32_t base = kLdsShift + j * 4096u;
  return lds_u32(lds, base + ((r & 0xffu) << 2)) ^
         lds_u32(lds, base + 1024u + (((r >> 8) & 0xffu) << 2)) ^
         lds_u32(lds, base + 2048u + (((r >> 16) & 0xffu) << 2)) ^
         lds_u32(lds, base + 3072u + ((r >> 24) << 2));
}

// Un-feed h zero bytes (register that becomes r after h zero bytes).
__device__ __forceinline__ uint32_t unshift_bytes(const uint8_t* lds,
                                                  uint32_t s0, uint32_t r,
                                                  uint32_t h) {
  for (uint32_t i = 0; i < h; ++i) {
    uint32_t idx = lds_u32(lds, kLdsInvTop + ((r >> 24) << 2));
    uint32_t t0 = lds_u32(lds, (idx << 8) | ((s0 >> 8) & 0xffu));
    r = ((r ^ t0) << 8) | idx;
  }
  return r;
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

// ---------------------------------------------------------------------------
// One span segment (length <= kSegBytes) on one wavefront.
// Returns Extend(init, p, n) in every lane.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t segment_crc(const uint8_t* lds,
                                                uint32_t s0, uint32_t lane,
                                                const uint8_t* p, uint32_t n,
                                                uint32_t init) {
  const uint64_t start = reinterpret_cast<uint64_t>(p);
  const uint64_t end = start + n;
  const uint64_t a0 = start & ~uint64_t(15);
  const uint64_t e0 = end & ~uint64_t(15);
  uint32_t reg;  // register at max(e0, start)

  if (e0 > start) {
    // ---- main region [a0, e0): 16-byte chunks, c per lane ----
    const uint32_t cm = static_cast<uint32_t>((e0 - a0) >> 4);
    const uint32_t c = (cm + 63u) >> 6;
    const uint32_t pad = 64u * c - cm;
    const uint32_t h = static_cast<uint32_t>(start - a0);
    const uint32_t inj =
        (init == 0u) ? lds_u32(lds, kLdsHead0 + (h << 2))
                     : unshift_bytes(lds, s0, ~init, h);
    // leading-byte masks for chunk 0 (bytes [0, h) are not in the span)
    uint32_t m0 = h == 0 ? ~0u : (h >= 4 ? 0u : (~0u << (8 * h)));
    uint32_t m1 = h <= 4 ? ~0u : (h >= 8 ? 0u : (~0u << (8 * (h - 4))));
    uint32_t m2 = h <= 8 ? ~0u : (h >= 12 ? 0u : (~0u << (8 * (h - 8))));
    uint32_t m3 = h <= 12 ? ~0u : (~0u << (8 * (h - 12)));

    const int32_t q0 = static_cast<int32_t>(lane * c) - static_cast<int32_t>(pad);
    const u32x4* cp = reinterpret_cast<const u32x4*>(a0);
    uint32_t r = 0;
    for (uint32_t i = 0; i < c; i += 4) {
      u32x4 d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t q = q0 + static_cast<int32_t>(i) + j;
        d[j] = u32x4{0u, 0u, 0u, 0u};
        if (q >= 0 && i + j < c) d[j] = __builtin_nontemporal_load(cp + q);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t q = q0 + static_cast<int32_t>(i) + j;
        if (i + j < c) {
          u32x4 w = d[j];
          if (q == 0) {
            w.x &= m0; w.y &= m1; w.z &= m2; w.w &= m3;
            r = inj;
          }
          r = feed_word(lds, s0, r, w.x);
          r = feed_word(lds, s0, r, w.y);
          r = feed_word(lds, s0, r, w.z);
          r = feed_word(lds, s0, r, w.w);
        }
      }
    }
    // ---- wavefront butterfly: fold 64 stripe registers ----
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) {
      const uint32_t partner = __shfl_down(r, 1u << k, 64);
      if ((lane & ((2u << k) - 1u)) == 0u) {
        uint32_t v = r;
        for (uint32_t cb = c, b = 0; cb; cb >>= 1, ++b)
          if (cb & 1u) v = shift_pow2(lds, v, b + k);
        r = v ^ partner;
      }
    }
    reg = __builtin_amdgcn_readfirstlane(r);
  } else {
    reg = ~init;
  }

  // ---- ragged tail: bytes [max(e0, start), end) inside chunk [e0, e0+16) ----
  if (end > e0) {
    const uint32_t* tp = reinterpret_cast<const uint32_t*>(e0);
    const uint32_t o = start > e0 ? static_cast<uint32_t>(start - e0) : 0u;
    const uint32_t e = static_cast<uint32_t>(end - e0);
    uint32_t t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = (4u * j < e) ? tp[j] : 0u;
    uint32_t i = o;
    if (o == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (4u * j + 4u <= e) { reg = feed_word(lds, s0, reg, t[j]); i += 4; }
    }
    for (; i < e; ++i) {
      const uint32_t wd = i < 4 ? t[0] : (i < 8 ? t[1] : (i < 12 ? t[2] : t[3]));
      reg = feed_byte(lds, s0, reg, (wd >> (8 * (i & 3))) & 0xffu);
    }
  }
  return ~reg;
}

__device__ __forceinline__ uint32_t span_crc(const uint8_t* lds, uint32_t s0,
                                             uint32_t lane, const uint8_t* p,
                                             uint64_t n, uint32_t init) {
  uint32_t crc = init;
  while (n > kSegBytes) {
    crc = segment_crc(lds, s0, lane, p, kSegBytes, crc);
    p += kSegBytes;
    n -= kSegBytes;
  }
  return segment_crc(lds, s0, lane, p, static_cast<uint32_t>(n), crc);
}

// Copy the device tables into LDS: main tables replicated 32x, the rest
// linear.  Every thread of the workgroup takes part; ends with a barrier.
__device__ __forceinline__ void load_tables(uint8_t* lds,
                                            const DevTables* __restrict__ tab) {
  const uint32_t tid = threadIdx.x;
  const uint32_t nthr = blockDim.x;
  // main: entry e = b*64 + u*32 + lane ; 4 lanes per uint4 store
  for (uint32_t e4 = tid; e4 < 4096u; e4 += nthr) {
    const uint32_t e = e4 * 4u;
    const uint32_t b = e >> 6, u = (e >> 5) & 1u;
    const uint32_t v = u ? tab->t0[b] : tab->t1[b];
    *reinterpret_cast<uint4*>(lds + e * 4u) = make_uint4(v, v, v, v);
  }
  const uint4* src = reinterpret_cast<const uint4*>(tab->shift);
  uint4* dst = reinterpret_cast<uint4*>(lds + kLdsShift);
  for (uint32_t i = tid; i < kNumShift * 256u; i += nthr) dst[i] = src[i];
  uint32_t* inv = reinterpret_cast<uint32_t*>(lds + kLdsInvTop);
  for (uint32_t i = tid; i < 256u; i += nthr) inv[i] = tab->inv_top[i];
  uint32_t* hd = reinterpret_cast<uint32_t*>(lds + kLdsHead0);
  for (uint32_t i = tid; i < 16u; i += nthr) hd[i] = tab->head0[i];
  __syncthreads();
}

__device__ __forceinline__ uint32_t lane_const() {
  const uint32_t l4 = (threadIdx.x & 31u) * 4u;
  return l4 | ((l4 | 0x80u) << 8);
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// Descriptor batch: span i = base + offsets[i], lengths[i] bytes, inits[i].
__global__ __launch_bounds__(kThreads) void crc32c_spans_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags,
    const DevTables* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t s0 = lane_const();
  const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  for (uint64_t s = static_cast<uint64_t>(blockIdx.x) * kWaves + wave; s < count;
       s += nw) {
    const uint64_t off = offsets[s];
    const uint32_t n = lengths[s];
    const uint32_t init = inits ? inits[s] : 0u;
    uint32_t crc = span_crc(lds, s0, lane, base + off, n, init);
    if (flags & kFlagMask) crc = mask_crc(crc);
    if (lane == 0) out[s] = crc;
  }
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length,
    uint32_t init, uint32_t* __restrict__ out, uint64_t count, uint32_t flags,
    const DevTables* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t s0 = lane_const();
  const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  for (uint64_t s = static_cast<uint64_t>(blockIdx.x) * kWaves + wave; s < count;
       s += nw) {
    uint32_t crc = span_crc(lds, s0, lane, base + s * stride, length, init);
    if (flags & kFlagMask) crc = mask_crc(crc);
    if (lane == 0) out[s] = crc;
  }
}

// Read-side verify: block = base + off, n = handle size; crc over n+1 bytes
// compared with Unmask(LE32 at n+1) (kv/src/table/format.cc:91-99).
__global__ __launch_bounds__(kThreads) void crc32c_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status,
    uint64_t count, const DevTables* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t s0 = lane_const();
  const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  for (uint64_t s = static_cast<uint64_t>(blockIdx.x) * kWaves + wave; s < count;
       s += nw) {
    const uint8_t* blk = base + offsets[s];
    const uint32_t n = lengths[s];
    const uint32_t crc = span_crc(lds, s0, lane, blk, uint64_t(n) + 1u, 0u);
    if (lane == 0) {
      const uint8_t* t = blk + n + 1;
      const uint32_t stored = uint32_t(t[0]) | (uint32_t(t[1]) << 8) |
                              (uint32_t(t[2]) << 16) | (uint32_t(t[3]) << 24);
      const uint32_t rot = stored - 0xa282ead8u;
      status[s] = ((rot >> 17) | (rot << 15)) == crc ? 1 : 0;
    }
  }
}

// Read-stream ceiling: same loads as the strided CRC kernel, XOR-reduce
// only (diagnostic; the roofline's measured denominator).
__global__ __launch_bounds__(kThreads) void readstream_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length,
    uint32_t* __restrict__ out, uint64_t count) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint32_t chunks = length >> 4;
  for (uint64_t s = static_cast<uint64_t>(blockIdx.x) * kWaves + wave; s < count;
       s += nw) {
    const u32x4* cp = reinterpret_cast<const u32x4*>(base + s * stride);
    uint32_t acc = 0;
    for (uint32_t i = lane; i < chunks; i += 64) {
      u32x4 v = __builtin_nontemporal_load(cp + i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
    if (lane == 0) out[s] = acc;
  }
}

// Seeded test/bench data: 64-bit word k = splitmix64(seed + (k+1)*gamma)
// (tests/golden/common.py), so any block can be regenerated on the host.
__global__ __launch_bounds__(256) void fill_splitmix64_kernel(
    uint64_t* __restrict__ dst, uint64_t nwords, uint64_t first_word,
    uint64_t seed) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < nwords; i += step) {
    uint64_t z = seed + (first_word + i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[i] = z ^ (z >> 31);
  }
}

}  // namespace dev
}  // namespace wipdb
