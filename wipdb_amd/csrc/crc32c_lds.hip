// crc32c_lds.hip -- hand-written CDNA4 (gfx950) kernels for batched CRC32C
// of WipDB table blocks, LDS-staged.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// kv/src/util/crc32c.cc:1225-1227) applied to every block span, as
// TableBuilder::WriteRawBlock (kv/src/table/table_builder.cc:194-196) and
// ReadBlock (kv/src/table/format.cc:91-93) do one block at a time; the
// reference's hot loop is crc32c_3way (crc32c.cc:667-1198).
//
// Design:
//   * persistent grid, one 16-wave workgroup per CU; the workgroup's waves
//     take spans from an LDS counter (static per-workgroup blocks of 16
//     spans, round robin over the grid, so the chip reads one compact window
//     of the batch at a time);
//   * a span is cut into segments of at most 256 chunks of its 16-byte grid
//     (4 KiB) plus a ragged tail (< 16 bytes, fed after the fold);
//   * a wave owns a 4 KiB LDS slot.  The next segment is DMA'd into it by
//     4 global_load_lds_dwordx4 (1 KiB each, nontemporal) as soon as the
//     current one has been read into registers, so one segment per wave is
//     always in flight while the wave computes -- no VGPR ring;
//   * lane l CRCs the 64-byte stripe [64 l, 64 l + 64) of the segment's
//     256-chunk window, the window END-aligned with the segment's last full
//     chunk (so every stripe is a whole number of 64 bytes from the end).
//     The DMA rotates the 4 chunks of each stripe by (stripe >> 2) & 3 via
//     the per-lane SOURCE address, so the stripe reads (ds_read_b128, 16
//     lanes per LDS cycle) hit 16 different 4-bank groups;
//   * slicing-by-4 from the 8-replica rotated tables (crc32c_lds.h): 4
//     v_perm + 4 ds_read_b32 + 2 v_bitop3 per word, conflict-free;
//   * fold: lane l's register is shifted by 64 (63 - l) bytes in two
//     per-lane table levels -- 64 (7 - l % 8) bytes, XOR over 8 lanes (DPP),
//     512 (7 - l / 8) bytes on the 8 block leaders, XOR (DPP + readlane).
//     This is the reference's CombineCRC (crc32c.cc:640-657) done with
//     tables: CDNA4 has no carry-less multiply;
//   * unaligned starts: chunks in front of the span are zeroed, the first h
//     bytes of its first chunk masked, and ~init * x^(-8h) is XORed into the
//     first word (the register is 0 there), so it equals ~init at the first
//     real byte.  Later segments of a span carry the register on.  Any
//     offset / length / init is bit-exact.
// Descriptors, tail chunks and stored trailers are scalar (SMEM) loads;
// every vector-memory instruction is a DMA or a result store, counted by
// hand (s_waitcnt vmcnt) -- see issue order in run().
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_lds.h"

namespace wipdb {
namespace lk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t l_u32;
typedef __attribute__((address_space(3))) uint32_t l_u32w;
typedef __attribute__((address_space(3))) const u32x4 l_u32x4;

__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {
  return *reinterpret_cast<l_u32*>(static_cast<uintptr_t>(a));
}
// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (static_cast<uint64_t>(uni(static_cast<uint32_t>(v >> 32))) << 32) |
         uni(static_cast<uint32_t>(v));
}
__device__ __forceinline__ uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
__device__ __forceinline__ uint32_t unmask_crc(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

// ---------------------------------------------------------------------------
// Per-lane table constants (crc32c_lds.h "Bank rule").
// ---------------------------------------------------------------------------
struct Lane {
  uint32_t sel[4];  // v_perm selector of lookup j: [K byte j, data byte t_j, 0, 0]
  uint32_t km;      // byte j: 32 t_j + 4 (l & 7)               (main tables)
  uint32_t k1;      // byte j: 128 + 4 (4 a + t_j), a = 7 - l % 8 (fold level 1)
  uint32_t k2;      // byte j: 8 (4 c + t_j), c = 7 - l / 8     (fold level 2, >> 1)
};

__device__ __forceinline__ Lane make_lane(uint32_t l) {
  Lane k;
  const uint32_t q = (l >> 3) & 3u, r = l & 7u, a = 7u - (l & 7u), c = 7u - (l >> 3);
  k.km = k.k1 = k.k2 = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t t = (j + q) & 3u;
    k.sel[j] = 0x0c0c0000u | (t << 8) | (4u + j);
    k.km |= (t * 32u + r * 4u) << (8 * j);
    k.k1 |= (128u + (a * 4u + t) * 4u) << (8 * j);
    k.k2 |= (8u * (c * 4u + t)) << (8 * j);
  }
  return k;
}

// One slicing-by-4 word step in "x form" (x = register ^ word): returns the
// register after the word's 4 bytes, XOR wn (the next word, 0 at the end).
__device__ __forceinline__ uint32_t step(const Lane& k, uint32_t x, uint32_t wn) {
  const uint32_t a0 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.km, x, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.km, x, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.km, x, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.km, x, k.sel[3]));
  return xor3(xor3(a0, a1, a2), a3, wn);
}

// r * x^(8 * 64 a) mod P (a = 7 - l % 8; a = 0: r itself)
__device__ __forceinline__ uint32_t fold_l1(const Lane& k, uint32_t l, uint32_t r) {
  const uint32_t a0 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1, r, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1, r, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1, r, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1, r, k.sel[3]));
  const uint32_t v = xor3(a0, a1, a2) ^ a3;
  return (l & 7u) == 7u ? r : v;
}

// r * x^(8 * 512 c) mod P (c = 7 - l / 8; c = 0: r itself)
__device__ __forceinline__ uint32_t fold_l2(const Lane& k, uint32_t l, uint32_t r) {
  const uint32_t a0 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[0]) >> 1));
  const uint32_t a1 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[1]) >> 1));
  const uint32_t a2 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[2]) >> 1));
  const uint32_t a3 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[3]) >> 1));
  const uint32_t v = xor3(a0, a1, a2) ^ a3;
  return (l >> 3) == 7u ? r : v;
}

// The segment register from the 64 lane registers: XOR over lanes of
// shift(r_l, 64 (63 - l)).  Uniform result.
__device__ __forceinline__ uint32_t fold(const Lane& k, uint32_t l, uint32_t r) {
  uint32_t v = fold_l1(k, l, r);
  v ^= dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v ^= dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v ^= dpp<0x104>(v);  // row_shl:4 -> lanes 8k hold their block of 8
  uint32_t w = 0;
  if ((l & 7u) == 0u) w = fold_l2(k, l, v);
  w ^= dpp<0x108>(w);  // row_shl:8 -> lanes 0, 16, 32, 48
  return __builtin_amdgcn_readlane(w, 0) ^ __builtin_amdgcn_readlane(w, 16) ^
         __builtin_amdgcn_readlane(w, 32) ^ __builtin_amdgcn_readlane(w, 48);
}

// Sarwate byte step with this lane's copy of T0 (main slot 3).
__device__ __forceinline__ uint32_t feed_byte(uint32_t l, uint32_t r, uint32_t b) {
  const uint32_t x = (r ^ b) & 0xffu;
  return lds_ld(kLdsMain + (x << 8) + 96u + 4u * (l & 7u)) ^ (r >> 8);
}

// Un-feed h zero bytes: the register that becomes r after h zero bytes.
__device__ __forceinline__ uint32_t unshift(uint32_t l, uint32_t r, uint32_t h) {
  for (uint32_t i = 0; i < h; ++i) {
    const uint32_t idx = lds_ld(MiscAddr(kMiscInvTop + (r >> 24)));
    const uint32_t t0 = lds_ld(kLdsMain + (idx << 8) + 96u + 4u * (l & 7u));
    r = ((r ^ t0) << 8) | idx;
  }
  return r;
}

// Feeds bytes [o, e) (e <= 16) of a 16-byte chunk t0..t3 into register r
// (uniform; whole words when the chunk starts the range).
__device__ __forceinline__ uint32_t feed_tail(const Lane& k, uint32_t l, uint32_t r, const u32x4& t,
                                              uint32_t o, uint32_t e) {
  uint32_t i = o;
  if (o == 0u) {
    if (e >= 4u) r = step(k, r ^ t.x, 0u), i = 4u;
    if (e >= 8u) r = step(k, r ^ t.y, 0u), i = 8u;
    if (e >= 12u) r = step(k, r ^ t.z, 0u), i = 12u;
  }
  for (; i < e; ++i) {
    const uint32_t wd = i < 4u ? t.x : (i < 8u ? t.y : (i < 12u ? t.z : t.w));
    r = feed_byte(l, r, (wd >> (8u * (i & 3u))) & 0xffu);
  }
  return uni(r);
}

// ---------------------------------------------------------------------------
// DMA.  The LDS destination of global_load_lds is M0 + 16 * lane (lane-
// linear); the source address is per lane (SGPR base + VGPR offset).
// ---------------------------------------------------------------------------
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
      : "memory");
}

__device__ __forceinline__ void dma1(uint64_t base, uint32_t dst, uint32_t off) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(dst), "s"(base)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
}

// Scalar (SMEM) loads of a uniform address, waited for in the same asm
// statement.  The data pointers of a batch are not kernel arguments the
// compiler can prove unclobbered, so plain C++ would emit vector loads --
// which would break the hand-counted vmcnt pipeline above.
__device__ __forceinline__ u32x4 sload4(uint64_t a) {
  u32x4 v;
  asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a) : "memory");
  return v;
}
__device__ __forceinline__ uint64_t sload2(uint64_t a) {
  uint64_t v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t sload1(uint64_t a) {
  uint32_t v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a) : "memory");
  return v;
}
// LE32 at byte sh / 8 of the 8 bytes v
__device__ __forceinline__ uint32_t funnel(uint64_t v, uint32_t sh) {
  return static_cast<uint32_t>(v >> sh);
}

// The table image (tables + misc words) into LDS [0, 96 KiB): wave w copies
// 6 KiB with 6 DMAs.  Ends with the workgroup barrier.
__device__ __forceinline__ void load_image(const uint8_t* image, uint32_t w, uint32_t l) {
  constexpr uint32_t per = kImageBytes / kWaves;  // 6 KiB
  const uint64_t src = reinterpret_cast<uint64_t>(image) + w * per;
#pragma unroll
  for (uint32_t q = 0; q < per / 1024u; ++q) dma1(src, w * per + 1024u * q, 1024u * q + 16u * l);
  wait_vm<0>();
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Span sources (all values uniform).
// ---------------------------------------------------------------------------
// Addresses are kept as byte offsets from the source's base pointer, so the
// scalar loads of tail chunks and trailers go through a pointer derived
// from a const __restrict__ kernel argument -- which is what lets the
// compiler use SMEM (s_load) for them instead of vector loads that would
// break the hand-counted vmcnt pipeline.
struct SpanD {
  uint64_t a;     // offset of the first byte from the source base
  uint32_t n;     // bytes
  uint32_t init;  // Extend's init_crc
};

// Descriptor batch: span i = base + offsets[i], lengths[i] (+ extra) bytes.
struct DescSrc {
  const uint8_t* base;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* init;
  uint64_t count;
  uint32_t extra;  // verify: +1 type byte
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    SpanD d;
    d.a = off[s];
    d.n = len[s] + extra;
    d.init = init ? init[s] : 0u;
    return d;
  }
};

// Fixed-size blocks at a fixed stride.
struct StridedSrc {
  const uint8_t* base;
  uint64_t stride;
  uint32_t length, init;
  uint64_t count;
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    return SpanD{s * stride, length, init};
  }
};

// ---------------------------------------------------------------------------
// Segments of a span (uniform).
// ---------------------------------------------------------------------------
constexpr uint32_t kSegValid = 1u, kSegFirst = 2u, kSegLast = 4u, kSegCut = 8u;

struct Seg {
  uint64_t a0;    // offset of the segment's first chunk (16-byte aligned address)
  uint32_t nc;    // full chunks (0..256)
  uint32_t h;     // first segment: bytes of the first chunk in front of the span
  uint32_t o, e;  // last segment: tail bytes [o, e) of the chunk at a0 + 16 nc
  uint32_t flags;
  uint32_t init;  // first segment: the span's init
  uint64_t id;    // span index
};

// A span being walked: grid base, full chunks, tail, segments.
struct Walk {
  uint64_t a0, id;
  uint32_t f, h, t, init, k, nseg;
  bool cut, valid;

  __device__ __forceinline__ void start(const uint8_t* base, const SpanD& d, uint64_t s,
                                        bool split_rem) {
    const uint64_t abs = reinterpret_cast<uint64_t>(base) + d.a;
    h = static_cast<uint32_t>(abs & 15u);
    a0 = d.a - h;
    const uint32_t hn = h + d.n;
    f = hn >> 4;
    t = d.n == 0u ? 0u : (hn & 15u);
    init = d.init;
    id = s;
    k = 0;
    cut = split_rem && SplitRemainder(abs, d.n) != 0u;
    nseg = cut ? 1u : (f == 0u ? 1u : (f + kSegChunks - 1u) / kSegChunks);
    valid = true;
  }
  __device__ __forceinline__ Seg next() {
    Seg g;
    const bool last = k + 1u == nseg;
    g.a0 = a0 + static_cast<uint64_t>(k) * (kSegChunks * 16u);
    const uint32_t left = f - k * kSegChunks;
    g.nc = left < kSegChunks ? left : kSegChunks;
    g.h = k == 0u ? h : 0u;
    // the tail: bytes [16 f, h + n) of the chunk after the last full one; a
    // span inside one chunk (f == 0) is all tail, from byte h
    // (t = hn & 15, which for f == 0 is the span's end in chunk 0)
    g.o = f == 0u ? h : 0u;
    g.e = (last && !cut) ? t : 0u;
    g.flags = kSegValid | (k == 0u ? kSegFirst : 0u) | (last ? kSegLast : 0u) | (cut ? kSegCut : 0u);
    g.init = init;
    g.id = id;
    if (last) valid = false;
    ++k;
    return g;
  }
};

// ---------------------------------------------------------------------------
// The wave loop.  Issue order of vector-memory instructions per wave:
//   DMA(seg i) ... result store(seg i-1) ... DMA(seg i+1) ...
// so waiting for seg i's DMA is vmcnt(1) when a store followed it, else 0.
// OUT: 0 = CRC (masked with kFlagMask), 1 = verify status byte.
// ---------------------------------------------------------------------------
template <int OUT, typename Src>
__device__ __forceinline__ void run(const Src& src, void* out, uint32_t* partial, uint32_t flags,
                                    const uint8_t* image) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  (void)lds;
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t w = uni(threadIdx.x >> 6);
  load_image(image, w, l);
  const Lane lk = make_lane(l);
  const uint32_t slot = kLdsSlots + w * kSlotBytes;
  // DMA load q, lane m: chunk 64q + cm of the 256-chunk window
  const uint32_t cm = 4u * (l >> 2) + (((l & 3u) - (l >> 4)) & 3u);
  // stripe read i of lane l: LDS position 4l + ((i + (l >> 2)) & 3)
  uint32_t rpos[4];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) rpos[i] = slot + 16u * (4u * l + ((i + (l >> 2)) & 3u));

  const bool skip_small = (flags & kFlagSkipSmall) != 0u;
  const bool split_rem = (flags & kFlagSplitRem) != 0u;
  const bool msk = (flags & kFlagMask) != 0u;
  const uint64_t count = src.count;
  const uint32_t nwg = gridDim.x, wg = blockIdx.x;
  l_u32w* unit_ctr = reinterpret_cast<l_u32w*>(static_cast<uintptr_t>(MiscAddr(kMiscUnit)));
  // the workgroup's unit u is span ((u / 16) * nwg + wg) * 16 + u % 16
  auto grab = [&]() -> uint64_t {
    uint32_t u = 0;
    if (l == 0u) u = __atomic_fetch_add(unit_ctr, 1u, __ATOMIC_RELAXED);
    u = uni(u);
    return (static_cast<uint64_t>(u >> 4) * nwg + wg) * 16u + (u & 15u);
  };
  // the next span of the wave (skipping small spans when asked)
  auto next_span = [&](Walk& wk) {
    for (;;) {
      const uint64_t s = grab();
      if (s >= count) {
        wk.valid = false;
        return;
      }
      const SpanD d = src.get(s);
      if (skip_small && d.n <= kSmallMax) continue;
      wk.start(src.base, d, s, split_rem);
      return;
    }
  };

  const uint64_t sbase = reinterpret_cast<uint64_t>(src.base);
  auto issue = [&](const Seg& g) {
    if (g.nc == kSegChunks) {
      dma4(sbase + g.a0, slot, 16u * cm, 16u * cm + 1024u, 16u * cm + 2048u, 16u * cm + 3072u);
    } else if (g.nc != 0u) {
      // chunks in front of the segment re-read its first chunk (zeroed later)
      const int32_t sub = static_cast<int32_t>(16u * (kSegChunks - g.nc));
      const int32_t b = static_cast<int32_t>(16u * cm) - sub;
      dma4(sbase + g.a0, slot, static_cast<uint32_t>(max(b, 0)), static_cast<uint32_t>(max(b + 1024, 0)),
           static_cast<uint32_t>(max(b + 2048, 0)), static_cast<uint32_t>(max(b + 3072, 0)));
    }
  };
  // scalar loads for the segment's end: its tail chunk and (verify) the
  // stored trailer, LE32 right after the span.  Synchronous (s_load + wait
  // in one asm statement): they are issued at the end of an iteration, when
  // the wave is about to wait for its next DMA anyway.
  auto load_end = [&](const Seg& g, u32x4& tail, uint32_t& stored) {
    tail = u32x4{0, 0, 0, 0};
    stored = 0;
    if (!(g.flags & kSegLast)) return;
    if (g.e != 0u) tail = sload4(sbase + g.a0 + 16u * g.nc);
    if (OUT == 1 && !(g.flags & kSegCut)) {
      const uint64_t ta = sbase + g.a0 + 16u * g.nc + g.e;  // trailer address
      const uint32_t sh = static_cast<uint32_t>(ta & 3u) * 8u;
      const uint64_t al = ta & ~uint64_t(3);
      // the second dword only when the trailer straddles it (never past
      // the 8-byte block holding the trailer's last byte)
      stored = sh ? funnel(sload2(al), sh) : sload1(al);
    }
  };

  Walk wk, pf;
  wk.valid = pf.valid = false;
  next_span(wk);
  if (!wk.valid) return;
  next_span(pf);
  Seg cur = wk.next();
  issue(cur);
  u32x4 tail;
  uint32_t stored;
  load_end(cur, tail, stored);
  uint32_t chain = 0;  // register carried between the segments of a span
  bool stored_prev = false;

  for (;;) {
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    u32x4 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(rpos[i]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is free again
    // the next segment: the rest of this span, or the prefetched span
    Seg nxt;
    nxt.flags = 0;
    bool took_pf = false;
    if (wk.valid) {
      nxt = wk.next();
    } else if (pf.valid) {
      wk = pf;
      took_pf = true;
      nxt = wk.next();
    }
    if (nxt.flags & kSegValid) issue(nxt);

    // ---- CRC of the current segment ----
    uint32_t R;
    if (cur.nc == 0u) {
      R = ~cur.init;  // a span inside one chunk: all of it is tail
    } else {
      uint32_t inj = chain;
      if (cur.flags & kSegFirst) {
        inj = cur.init == 0u ? lds_ld(MiscAddr(kMiscHead0 + cur.h)) : unshift(l, ~cur.init, cur.h);
        inj = uni(inj);
      }
      uint32_t W[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        W[4 * i] = d[i].x;
        W[4 * i + 1] = d[i].y;
        W[4 * i + 2] = d[i].z;
        W[4 * i + 3] = d[i].w;
      }
      if (cur.nc == kSegChunks && cur.h == 0u) {
        W[0] ^= l == 0u ? inj : 0u;
      } else {
        // chunk i of lane l is segment chunk 4l + i - (256 - nc): zero the
        // ones in front of the segment, mask the first h bytes of chunk 0
        // and put the register there
        const int32_t base = static_cast<int32_t>(kSegChunks - cur.nc);
        const uint32_t hh = cur.h;
        uint32_t hm[4];
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww)
          hm[ww] = hh >= 4u * ww + 4u ? 0u : (hh <= 4u * ww ? ~0u : (~0u << (8u * (hh - 4u * ww))));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int32_t ci = static_cast<int32_t>(4u * l) + i - base;
#pragma unroll
          for (int ww = 0; ww < 4; ++ww) {
            const uint32_t m = ci < 0 ? 0u : (ci == 0 ? hm[ww] : ~0u);
            W[4 * i + ww] &= m;
          }
          W[4 * i] ^= ci == 0 ? inj : 0u;
        }
      }
      uint32_t x = W[0];
#pragma unroll
      for (int i = 0; i < 15; ++i) x = step(lk, x, W[i + 1]);
      const uint32_t r = step(lk, x, 0u);
      R = fold(lk, l, r);
    }

    bool did_store = false;
    if (cur.flags & kSegLast) {
      if (cur.e > cur.o) R = feed_tail(lk, l, R, tail, cur.o, cur.e);
      const uint32_t crc = ~R;
      did_store = true;
      if (l == 0u) {
        if (cur.flags & kSegCut) {
          // partial CRC of a span the small-span path finishes
          if (OUT == 1) partial[cur.id] = crc;
          else static_cast<uint32_t*>(out)[cur.id] = crc;
        } else if (OUT == 1) {
          static_cast<uint8_t*>(out)[cur.id] = unmask_crc(stored) == crc ? 1u : 0u;
        } else {
          static_cast<uint32_t*>(out)[cur.id] = msk ? mask_crc(crc) : crc;
        }
      }
    } else {
      chain = R;
    }
    stored_prev = did_store;

    if (!(nxt.flags & kSegValid)) break;
    // refill the span prefetch and the next segment's scalar loads
    if (took_pf) next_span(pf);
    load_end(nxt, tail, stored);
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// Descriptor batch: out[i] = Extend(inits[i], base + offsets[i], lengths[i]).
__global__ __launch_bounds__(kThreads) void crc32c_lds_spans_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image) {
  const DescSrc src{base, offsets, lengths, inits, count, 0u};
  run<0>(src, out, nullptr, flags, image);
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_lds_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image) {
  const StridedSrc src{base, stride, length, init, count};
  run<0>(src, out, nullptr, flags & kFlagMask, image);
}

// Read-side verify (ReadBlock, kv/src/table/format.cc:91-99): block i =
// base + offsets[i], handle size n = lengths[i]; CRC over n + 1 bytes
// compared with Unmask(LE32 at n + 1).  With kFlagSkipSmall | kFlagSplitRem
// the small-span path takes blocks of at most kSmallMax bytes and finishes
// the cut ones from partial[i].
__global__ __launch_bounds__(kThreads) void crc32c_lds_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status, uint64_t count,
    uint32_t flags, uint32_t* __restrict__ partial, const uint8_t* __restrict__ image) {
  const DescSrc src{base, offsets, lengths, nullptr, count, 1u};
  run<1>(src, status, partial, flags & (kFlagSkipSmall | kFlagSplitRem), image);
}

}  // namespace lk
}  // namespace wipdb
