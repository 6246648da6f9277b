// crc32c_kernels.hip -- hand-written CDNA4 (gfx950) kernels for batched
// CRC32C of WipDB table blocks.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// crc32c.cc:1225-1227) applied to every block span, as WriteRawBlock
// (kv/src/table/table_builder.cc:194-196) and ReadBlock
// (kv/src/table/format.cc:91-93) do one block at a time.
//
// Design (DESIGN.md "Kernels"):
//   * one span per wavefront.  The span's 16-byte chunks are split into
//     64*K contiguous stripes ("virtual lanes"); lane l runs K independent
//     CRC chains over K consecutive stripes, i.e. one contiguous run of
//     K*c' chunks (16-byte loads; every byte of every line the wave fetches
//     is used).  K chains per lane give the LDS-latency-bound byte scan the
//     instruction-level parallelism it needs.
//   * CRC arithmetic is table-driven from LDS (CDNA4 has no carry-less
//     multiply and this is a byte scan, not a contraction: no MFMA):
//     slicing-by-2 tables replicated 32x so lane l always reads bank l&31 --
//     every lookup is bank-conflict free -- and each lookup address is built
//     by ONE v_perm_b32 (table byte | lane byte | table-select bit).
//   * the 64*K stripe registers are folded by a GF(2) tree: first the K
//     chains inside a lane, then a 6-level wavefront butterfly,
//        reg(v) = shift(reg(v), stripe_bytes * 2^t) ^ reg(v + 2^t),
//     where shift by 16*2^j bytes is 4 lookups in a "multiply by
//     x^(8*16*2^j) mod P" table (the carry-less combine of the reference's
//     CombineCRC, crc32c.cc:640-657, done with tables).
//   * unaligned starts: the first chunk's leading bytes are zeroed and the
//     register injected there is pre-un-shifted (~init * x^(-8h)) so it
//     equals ~init at the first real byte; the ragged end (< 16 bytes) is
//     fed after the fold.  So any offset/length/init is bit-exact.
//   * latency hiding: persistent grid (1 workgroup of 16 waves per CU, LDS =
//     113 KiB), each wave walks its spans with a one-item software pipeline:
//     the next item's chunk loads are issued before the current item is
//     processed, and 64 span descriptors are fetched per vector load.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace wipdb {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(3))) const uint32_t l_u32;

// ---------------------------------------------------------------------------
// LDS helpers (dynamic LDS starts at address 0: no static __shared__ here)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_ld(uint32_t addr) {
  return *reinterpret_cast<l_u32*>(static_cast<uintptr_t>(addr));
}

constexpr uint32_t kSelT1B0 = 0x0c0c0004u;  // [s0.b0, x.b0, 0, 0] -> T1[x.b0]
constexpr uint32_t kSelT0B1 = 0x0c0c0105u;  // [s0.b1, x.b1, 0, 0] -> T0[x.b1]

// Feed one little-endian 32-bit word into register r (slicing-by-2 twice).
// s0 = lane constant: byte0 = (lane&31)*4 (T1), byte1 = (lane&31)*4|0x80 (T0).
__device__ __forceinline__ uint32_t feed_word(uint32_t s0, uint32_t r, uint32_t w) {
  const uint32_t x = r ^ w;
  const uint32_t y = lds_ld(__builtin_amdgcn_perm(s0, x, kSelT1B0)) ^
                     lds_ld(__builtin_amdgcn_perm(s0, x, kSelT0B1)) ^ (x >> 16);
  return lds_ld(__builtin_amdgcn_perm(s0, y, kSelT1B0)) ^
         lds_ld(__builtin_amdgcn_perm(s0, y, kSelT0B1)) ^ (y >> 16);
}

// One word step in "x form": x = register ^ word; returns the register after
// the word's 4 bytes XOR the next word (w_next = 0 at the end of a chain).
// Written so the compiler forms v_xor_b32_sdwa + v_xor3_b32 (8 VALU/word).
__device__ __forceinline__ uint32_t step_x(uint32_t s0, uint32_t x, uint32_t w_next) {
  const uint32_t y = lds_ld(__builtin_amdgcn_perm(s0, x, kSelT1B0)) ^
                     lds_ld(__builtin_amdgcn_perm(s0, x, kSelT0B1)) ^ (x >> 16);
  const uint32_t yw = (y >> 16) ^ w_next;
  return lds_ld(__builtin_amdgcn_perm(s0, y, kSelT1B0)) ^
         lds_ld(__builtin_amdgcn_perm(s0, y, kSelT0B1)) ^ yw;
}

// Feed one 16-byte chunk into K independent chains (interleaved word by word).
template <int K>
__device__ __forceinline__ void feed_chunks(uint32_t s0, uint32_t (&r)[K], const u32x4 (&d)[K]) {
  uint32_t x[K];
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = r[k] ^ d[k].x;
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = step_x(s0, x[k], d[k].y);
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = step_x(s0, x[k], d[k].z);
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = step_x(s0, x[k], d[k].w);
#pragma unroll
  for (int k = 0; k < K; ++k) r[k] = step_x(s0, x[k], 0u);
}

// DPP row shift-left: lane l receives lane l+n of its 16-lane row (0 past
// the row end).  Used for butterfly levels whose partners share a row.
template <int N>
__device__ __forceinline__ uint32_t row_shl(uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x100 | N, 0xF, 0xF, true));
}

// Feed one byte (Sarwate step with this lane's T0 replica).
__device__ __forceinline__ uint32_t feed_byte(uint32_t s0, uint32_t r, uint32_t b) {
  const uint32_t x = (r ^ b) & 0xffu;
  return lds_ld((x << 8) | ((s0 >> 8) & 0xffu)) ^ (r >> 8);
}

// r * x^(8 * 16 * 2^j) mod P: 4 lookups in shift table j.
__device__ __forceinline__ uint32_t shift_pow2(uint32_t r, uint32_t j) {
  const uint32_t base = kLdsShift + j * 4096u;
  return lds_ld(base + ((r & 0xffu) << 2)) ^
         lds_ld(base + 1024u + (((r >> 8) & 0xffu) << 2)) ^
         lds_ld(base + 2048u + (((r >> 16) & 0xffu) << 2)) ^
         lds_ld(base + 3072u + ((r >> 24) << 2));
}

// r * x^(8 * 16 * cp * 2^m): one table multiply per set bit of cp.
__device__ __forceinline__ uint32_t shift_chunks(uint32_t r, uint32_t cp, uint32_t m) {
  for (uint32_t b = 0; cp; cp >>= 1, ++b)
    if (cp & 1u) r = shift_pow2(r, b + m);
  return r;
}

// Un-feed h zero bytes (register that becomes r after h zero bytes).
__device__ __forceinline__ uint32_t unshift_bytes(uint32_t s0, uint32_t r, uint32_t h) {
  for (uint32_t i = 0; i < h; ++i) {
    const uint32_t idx = lds_ld(kLdsInvTop + ((r >> 24) << 2));
    const uint32_t t0 = lds_ld((idx << 8) | ((s0 >> 8) & 0xffu));
    r = ((r ^ t0) << 8) | idx;
  }
  return r;
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}

// ---------------------------------------------------------------------------
// Work items.  An item is one segment (<= kSegBytes) of one span; spans
// longer than a segment are chained (init of segment k+1 = crc of segment k).
// All fields are wave-uniform.
// ---------------------------------------------------------------------------
struct Item {
  uint64_t span;    // span index (>= count: no item)
  uint64_t start;   // first byte (absolute address)
  uint64_t rest;    // bytes of the span from `start` on (this + later segments)
  uint64_t a0;      // 16-aligned start of the main region
  uint32_t n;       // bytes in this segment
  uint32_t cp;      // chunks per chain (0: no main region)
  uint32_t pad;     // virtual chunks in front of the first real chunk
  uint32_t h;       // bytes of chunk 0 in front of `start`
};

template <int K>
__device__ __forceinline__ void item_geometry(Item& it) {
  it.n = it.rest > kSegBytes ? kSegBytes : static_cast<uint32_t>(it.rest);
  const uint64_t end = it.start + it.n;
  const uint64_t a0 = it.start & ~uint64_t(15);
  const uint64_t e0 = end & ~uint64_t(15);
  it.a0 = a0;
  it.h = static_cast<uint32_t>(it.start - a0);
  if (e0 > it.start) {
    const uint32_t cm = static_cast<uint32_t>((e0 - a0) >> 4);
    const uint32_t v = 64u * K;
    it.cp = (cm + v - 1u) / v;
    it.pad = v * it.cp - cm;
  } else {
    it.cp = 0;
    it.pad = 0;
  }
}

// Loads chunk group i of item `it` for this lane: chunk i of each of its K
// chains.  Virtual chunks in front of the span (q < 0) read chunk 0 instead
// (always mapped: it holds the span's first byte); the chains they feed are
// overwritten by the injection or zeroed before the fold, so their data
// never matters and the loads need no predicate.
template <int K>
__device__ __forceinline__ void load_group(const Item& it, uint32_t i, uint32_t lane,
                                           u32x4 (&d)[K]) {
  const int32_t q0 = static_cast<int32_t>(lane * K * it.cp + i) -
                     static_cast<int32_t>(it.pad);
  g_u32x4* cp = reinterpret_cast<g_u32x4*>(it.a0);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int32_t q = q0 + k * static_cast<int32_t>(it.cp);
    d[k] = __builtin_nontemporal_load(cp + (q > 0 ? q : 0));
  }
}

// ---------------------------------------------------------------------------
// Span sources: where item descriptors come from.  Descriptors are fetched
// 64 at a time by one vector load (lane j holds the wave's j-th next span)
// and broadcast with v_readlane, so they never sit on the LDS counter.
// ---------------------------------------------------------------------------
struct DescSource {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  const uint32_t* inits;
  uint64_t count;
  uint32_t extra;  // bytes added to every length (verify: +1 type byte)
  uint64_t cache_first;
  uint64_t c_off;
  uint32_t c_len, c_init;

  __device__ __forceinline__ void fetch(uint64_t first, uint64_t stride, uint32_t lane) {
    cache_first = first;
    const uint64_t s = first + lane * stride;
    c_off = 0;
    c_len = 0;
    c_init = 0;
    if (s < count) {
      c_off = __builtin_nontemporal_load(offsets + s);
      c_len = __builtin_nontemporal_load(lengths + s) + extra;
      c_init = inits ? __builtin_nontemporal_load(inits + s) : 0u;
    }
  }
  __device__ __forceinline__ void get(uint32_t j, uint64_t& start, uint64_t& len,
                                      uint32_t& init) const {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off), j);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off >> 32), j);
    start = reinterpret_cast<uint64_t>(base) + ((static_cast<uint64_t>(hi) << 32) | lo);
    len = __builtin_amdgcn_readlane(c_len, j);
    init = __builtin_amdgcn_readlane(c_init, j);
  }
  __device__ __forceinline__ void desc(uint64_t s, uint64_t stride, uint32_t lane,
                                       uint64_t& start, uint64_t& len, uint32_t& init) {
    uint64_t j = (s - cache_first) / stride;
    if (j >= 64) {
      fetch(s, stride, lane);
      j = 0;
    }
    get(static_cast<uint32_t>(j), start, len, init);
  }
};

struct StridedSource {
  const uint8_t* base;
  uint64_t stride_bytes;
  uint32_t length;
  uint32_t init;
  uint64_t count;
  __device__ __forceinline__ void desc(uint64_t s, uint64_t, uint32_t, uint64_t& start,
                                       uint64_t& len, uint32_t& ini) const {
    start = reinterpret_cast<uint64_t>(base) + s * stride_bytes;
    len = length;
    ini = init;
  }
};

// ---------------------------------------------------------------------------
// The wave loop.  out(span, crc, lane) is called once per span with the
// finished crc (uniform).
// ---------------------------------------------------------------------------
// Fold the 64*K stripe registers of a wave into the span register (uniform).
// r[k] of lane l covers virtual stripe l*K+k of cp chunks.  In-lane levels
// first, then the wavefront butterfly: DPP row shifts for partners 1..8
// lanes away, v_readlane for 16 and 32.  Shift tables of 16*2^j bytes.
template <int K>
__device__ __forceinline__ uint32_t fold_wave(uint32_t (&r)[K], uint32_t cp, uint32_t lane) {
  constexpr uint32_t kLogK = K == 1 ? 0 : (K == 2 ? 1 : (K == 4 ? 2 : 3));
#pragma unroll
  for (uint32_t m = 0, w = 1; w < K; ++m, w <<= 1) {
#pragma unroll
    for (uint32_t k = 0; k + w < K; k += 2 * w) r[k] = shift_chunks(r[k], cp, m) ^ r[k + w];
  }
  uint32_t v = r[0];
  uint32_t p = row_shl<1>(v);
  if ((lane & 1u) == 0u) v = shift_chunks(v, cp, kLogK + 0) ^ p;
  p = row_shl<2>(v);
  if ((lane & 3u) == 0u) v = shift_chunks(v, cp, kLogK + 1) ^ p;
  p = row_shl<4>(v);
  if ((lane & 7u) == 0u) v = shift_chunks(v, cp, kLogK + 2) ^ p;
  p = row_shl<8>(v);
  if ((lane & 15u) == 0u) v = shift_chunks(v, cp, kLogK + 3) ^ p;
  const uint32_t g16 = __builtin_amdgcn_readlane(v, 16);
  const uint32_t g48 = __builtin_amdgcn_readlane(v, 48);
  if ((lane & 31u) == 0u) v = shift_chunks(v, cp, kLogK + 4) ^ (lane ? g48 : g16);
  const uint32_t g0 = __builtin_amdgcn_readlane(v, 0);
  const uint32_t g32 = __builtin_amdgcn_readlane(v, 32);
  return uni(shift_chunks(g0, cp, kLogK + 5) ^ g32);
}

template <int K, typename Src, typename Out>
__device__ __forceinline__ void run_waves(Src& src, uint64_t first_span, uint64_t span_stride,
                                          Out out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t l4 = (threadIdx.x & 31u) * 4u;
  const uint32_t s0 = l4 | ((l4 | 0x80u) << 8);
  if (first_span >= src.count) return;
  Item it;
  uint32_t it_init;
  it.span = first_span;
  src.desc(it.span, span_stride, lane, it.start, it.rest, it_init);
  item_geometry<K>(it);

  u32x4 cur[K], nxt[K];
  if (it.cp) load_group<K>(it, 0, lane, cur);

  for (;;) {
    // next item (computed now so its first loads can be issued early)
    Item nx;
    uint32_t nx_init = 0;
    if (it.rest > it.n) {
      nx = it;
      nx.start = it.start + it.n;
      nx.rest = it.rest - it.n;
    } else {
      nx.span = it.span + span_stride;
      if (nx.span < src.count) src.desc(nx.span, span_stride, lane, nx.start, nx.rest, nx_init);
    }
    const bool nx_valid = nx.span < src.count;
    if (nx_valid) item_geometry<K>(nx);

    uint32_t reg;  // register after the main region (or ~init if none)
    const uint32_t cp = it.cp;
    const uint64_t end = it.start + it.n;
    if (cp && it.h == 0 && it.pad == 0 && (end & 15u) == 0) {
      // ---- fast path: aligned start, whole stripes, no ragged end ----
      // The register ~init enters at lane 0, chain 0, before any byte.
      uint32_t r[K];
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] = 0u;
      if (lane == 0) r[0] = ~it_init;
      for (uint32_t i = 0; i < cp; ++i) {
        if (i + 1 < cp) {
          load_group<K>(it, i + 1, lane, nxt);
        } else if (nx_valid && nx.cp) {
          load_group<K>(nx, 0, lane, nxt);
        }
        feed_chunks<K>(s0, r, cur);
#pragma unroll
        for (int k = 0; k < K; ++k) cur[k] = nxt[k];
      }
      reg = fold_wave<K>(r, cp, lane);
    } else if (cp) {
      // ---- general path: unaligned start, front padding, ragged end ----
      const uint32_t inj = (it_init == 0u) ? lds_ld(kLdsHead0 + (it.h << 2))
                                           : unshift_bytes(s0, ~it_init, it.h);
      const uint32_t h = it.h;
      const uint32_t m0 = h == 0 ? ~0u : (h >= 4 ? 0u : (~0u << (8 * h)));
      const uint32_t m1 = h <= 4 ? ~0u : (h >= 8 ? 0u : (~0u << (8 * (h - 4))));
      const uint32_t m2 = h <= 8 ? ~0u : (h >= 12 ? 0u : (~0u << (8 * (h - 8))));
      const uint32_t m3 = h <= 12 ? ~0u : (~0u << (8 * (h - 12)));
      // chunk 0 of the span sits at virtual chunk `pad`: lane l0, chain k0,
      // group i0 (all uniform)
      const uint32_t kcp = K * cp;
      const uint32_t l0 = it.pad / kcp;
      const uint32_t k0 = (it.pad - l0 * kcp) / cp;
      const uint32_t i0 = it.pad - l0 * kcp - k0 * cp;
      uint32_t r[K];
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] = 0u;

      for (uint32_t i = 0; i < cp; ++i) {
        // prefetch the next group (this item or the next one)
        if (i + 1 < cp) {
          load_group<K>(it, i + 1, lane, nxt);
        } else if (nx_valid && nx.cp) {
          load_group<K>(nx, 0, lane, nxt);
        }
        // chunk 0 of the span: mask its leading bytes, inject the register
        if (i == i0) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            if (static_cast<uint32_t>(k) == k0 && lane == l0) {
              cur[k].x &= m0;
              cur[k].y &= m1;
              cur[k].z &= m2;
              cur[k].w &= m3;
              r[k] = inj;
            }
          }
        }
        feed_chunks<K>(s0, r, cur);
#pragma unroll
        for (int k = 0; k < K; ++k) cur[k] = nxt[k];
      }
      // chains made only of virtual chunks (in front of the span) carry
      // garbage: they must be zero
      {
        const int32_t qlast = static_cast<int32_t>(lane * kcp + cp - 1u) -
                              static_cast<int32_t>(it.pad);
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (qlast + k * static_cast<int32_t>(cp) < 0) r[k] = 0u;
      }
      reg = fold_wave<K>(r, cp, lane);
    } else {
      reg = ~it_init;
      if (nx_valid && nx.cp) load_group<K>(nx, 0, lane, cur);
    }

    // ragged tail: bytes [max(e0, start), end) inside chunk [e0, e0+16)
    const uint64_t e0 = end & ~uint64_t(15);
    if (end > e0) {
      const uint32_t* tp = reinterpret_cast<const uint32_t*>(e0);
      const uint32_t o = it.start > e0 ? static_cast<uint32_t>(it.start - e0) : 0u;
      const uint32_t e = static_cast<uint32_t>(end - e0);
      uint32_t t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = (4u * j < e) ? tp[j] : 0u;
      uint32_t i = o;
      if (o == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (4u * j + 4u <= e) {
            reg = feed_word(s0, reg, t[j]);
            i += 4;
          }
      }
      for (; i < e; ++i) {
        const uint32_t wd = i < 4 ? t[0] : (i < 8 ? t[1] : (i < 12 ? t[2] : t[3]));
        reg = feed_byte(s0, reg, (wd >> (8 * (i & 3))) & 0xffu);
      }
    }
    const uint32_t crc = ~reg;

    if (it.rest > it.n) {
      nx_init = crc;  // next segment of the same span continues from here
    } else {
      out(it.span, crc, lane);
    }
    if (!nx_valid) break;
    it = nx;
    it_init = nx_init;
  }
}

// Copy the device tables into LDS: main tables replicated 32x, the rest
// linear.  Every thread of the workgroup takes part; ends with a barrier.
__device__ __forceinline__ void load_tables(uint8_t* lds, const DevTables* __restrict__ tab) {
  const uint32_t tid = threadIdx.x;
  const uint32_t nthr = blockDim.x;
  for (uint32_t e4 = tid; e4 < 4096u; e4 += nthr) {  // entry e = b*64 + u*32 + lane
    const uint32_t e = e4 * 4u;
    const uint32_t b = e >> 6, u = (e >> 5) & 1u;
    const uint32_t v = u ? tab->t0[b] : tab->t1[b];
    *reinterpret_cast<u32x4*>(lds + e * 4u) = u32x4{v, v, v, v};
  }
  const u32x4* src = reinterpret_cast<const u32x4*>(tab->shift);
  u32x4* dst = reinterpret_cast<u32x4*>(lds + kLdsShift);
  for (uint32_t i = tid; i < kNumShift * 256u; i += nthr) dst[i] = src[i];
  uint32_t* inv = reinterpret_cast<uint32_t*>(lds + kLdsInvTop);
  for (uint32_t i = tid; i < 256u; i += nthr) inv[i] = tab->inv_top[i];
  uint32_t* hd = reinterpret_cast<uint32_t*>(lds + kLdsHead0);
  for (uint32_t i = tid; i < 16u; i += nthr) hd[i] = tab->head0[i];
  __syncthreads();
}

__device__ __forceinline__ uint64_t wave_id() {
  return static_cast<uint64_t>(blockIdx.x) * kWaves + uni(threadIdx.x >> 6);
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
  DescSource src{base, offsets, lengths, inits, count, 0u, ~uint64_t(0) >> 1, 0, 0, 0};
  const bool msk = (flags & kFlagMask) != 0;
  run_waves<kChains>(src, wave_id(), static_cast<uint64_t>(gridDim.x) * kWaves,
                     [&](uint64_t s, uint32_t crc, uint32_t lane) {
                       if (lane == 0) out[s] = msk ? mask_crc(crc) : crc;
                     });
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags,
    const DevTables* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  StridedSource src{base, stride, length, init, count};
  const bool msk = (flags & kFlagMask) != 0;
  run_waves<kChains>(src, wave_id(), static_cast<uint64_t>(gridDim.x) * kWaves,
                     [&](uint64_t s, uint32_t crc, uint32_t lane) {
                       if (lane == 0) out[s] = msk ? mask_crc(crc) : crc;
                     });
}

// Read-side verify: block = base + off, n = handle size; crc over n+1 bytes
// compared with Unmask(LE32 at n+1) (kv/src/table/format.cc:91-99).
__global__ __launch_bounds__(kThreads) void crc32c_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status, uint64_t count,
    const DevTables* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  DescSource src{base, offsets, lengths, nullptr, count, 1u, ~uint64_t(0) >> 1, 0, 0, 0};
  run_waves<kChains>(src, wave_id(), static_cast<uint64_t>(gridDim.x) * kWaves,
                     [&](uint64_t s, uint32_t crc, uint32_t lane) {
                       if (lane == 0) {
                         const uint8_t* t = base + offsets[s] + lengths[s] + 1;
                         const uint32_t stored = uint32_t(t[0]) | (uint32_t(t[1]) << 8) |
                                                 (uint32_t(t[2]) << 16) |
                                                 (uint32_t(t[3]) << 24);
                         const uint32_t rot = stored - 0xa282ead8u;
                         status[s] = ((rot >> 17) | (rot << 15)) == crc ? 1 : 0;
                       }
                     });
}

// Read-stream ceiling: the same 16-byte nontemporal loads over fixed-size
// blocks, XOR-reduced (diagnostic; the roofline's measured denominator).
__global__ __launch_bounds__(kThreads) void readstream_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length,
    uint32_t* __restrict__ out, uint64_t count) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint32_t chunks = length >> 4;
  for (uint64_t s = wave_id(); s < count; s += nw) {
    g_u32x4* cp = reinterpret_cast<g_u32x4*>(reinterpret_cast<uintptr_t>(base + s * stride));
    uint32_t acc = 0;
    for (uint32_t i = lane; i < chunks; i += 64) {
      const u32x4 v = __builtin_nontemporal_load(cp + i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
    if (lane == 0) out[s] = acc;
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

}  // namespace dev
}  // namespace wipdb
