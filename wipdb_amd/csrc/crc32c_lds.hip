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

// G: spans per wave (groups of 64 / G lanes); the level-2 fold shifts the
// 8-lane block b of a group by 512 (blocks - 1 - b) bytes.
template <int G>
__device__ __forceinline__ Lane make_lane(uint32_t l) {
  Lane k;
  constexpr uint32_t LG = 64u / G;
  const uint32_t q = (l >> 3) & 3u, r = l & 7u, a = 7u - (l & 7u);
  const uint32_t c = (LG / 8u - 1u) - ((l % LG) >> 3);
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

// r * x^(8 * 512 c) mod P (c of make_lane; c = 0: r itself)
template <int G>
__device__ __forceinline__ uint32_t fold_l2(const Lane& k, uint32_t l, uint32_t r) {
  constexpr uint32_t LG = 64u / G;
  const uint32_t a0 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[0]) >> 1));
  const uint32_t a1 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[1]) >> 1));
  const uint32_t a2 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[2]) >> 1));
  const uint32_t a3 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(k.k2, r, k.sel[3]) >> 1));
  const uint32_t v = xor3(a0, a1, a2) ^ a3;
  return ((l % LG) >> 3) == LG / 8u - 1u ? r : v;
}

template <int G>
struct Folded {
  uint32_t v[G];
  __device__ __forceinline__ uint32_t operator[](int i) const { return v[i]; }
};

// The segment registers of the G groups from their lanes' registers: XOR
// over the group's lanes of shift(r_l, 64 (lanes - 1 - l % lanes)).  Uniform.
template <int G>
__device__ __forceinline__ Folded<G> fold(const Lane& k, uint32_t l, uint32_t r) {
  static_assert(G == 1 || G == 2 || G == 4, "groups of 64, 32 or 16 lanes");
  uint32_t v = fold_l1(k, l, r);
  v ^= dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v ^= dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v ^= dpp<0x104>(v);  // row_shl:4 -> lanes 8k hold their block of 8
  uint32_t w = 0;
  if ((l & 7u) == 0u) w = fold_l2<G>(k, l, v);
  w ^= dpp<0x108>(w);  // row_shl:8 -> lanes 16k hold their 16
  Folded<G> f;
  if constexpr (G == 1) {
    f.v[0] = __builtin_amdgcn_readlane(w, 0) ^ __builtin_amdgcn_readlane(w, 16) ^
             __builtin_amdgcn_readlane(w, 32) ^ __builtin_amdgcn_readlane(w, 48);
  } else if constexpr (G == 2) {
    f.v[0] = __builtin_amdgcn_readlane(w, 0) ^ __builtin_amdgcn_readlane(w, 16);
    f.v[1] = __builtin_amdgcn_readlane(w, 32) ^ __builtin_amdgcn_readlane(w, 48);
  } else {
#pragma unroll
    for (int g = 0; g < 4; ++g) f.v[g] = __builtin_amdgcn_readlane(w, 16 * g);
  }
  return f;
}

// The 16 words of a lane's stripe through the chain: the register after
// them (the lane's register before them is 0; the span's own register was
// XORed into its first word).
__device__ __forceinline__ uint32_t scan(const Lane& k, const uint32_t (&W)[16]) {
  uint32_t x = W[0];
#pragma unroll
  for (int i = 0; i < 15; ++i) x = step(k, x, W[i + 1]);
  return step(k, x, 0u);
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

// The same with per-lane o, e (each lane serves its group's span).
__device__ __forceinline__ uint32_t feed_tail_lanes(const Lane& k, uint32_t l, uint32_t r,
                                                    const u32x4& t, uint32_t o, uint32_t e) {
  const uint32_t tw[3] = {t.x, t.y, t.z};
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j) {
    const uint32_t x = step(k, r ^ tw[j], 0u);
    r = (o == 0u && e >= 4u * j + 4u) ? x : r;
  }
  const uint32_t b0 = o == 0u ? (e & ~3u) : o;
  for (uint32_t i = 0; i < 16u; ++i) {
    const uint32_t b = b0 + i;
    const bool p = b < e;
    if (__builtin_amdgcn_ballot_w64(p) == 0u) break;
    const uint32_t wd = b < 4u ? t.x : (b < 8u ? t.y : (b < 12u ? t.z : t.w));
    const uint32_t x = feed_byte(l, r, (wd >> (8u * (b & 3u))) & 0xffu);
    r = p ? x : r;
  }
  return r;
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

__device__ __forceinline__ void dma2(uint64_t base, uint32_t slot, uint32_t o0, uint32_t o1) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %4 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %4 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(o0), "v"(o1), "s"(slot), "s"(base)
      : "memory");
}

__device__ __forceinline__ void dma1nt(uint64_t base, uint32_t dst, uint32_t off) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3 nt\n\t"
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

// LE32 at any address (ReadBlock's trailer, kv/src/table/format.cc:91-93):
// the second dword only when the value straddles it, so nothing past the
// 8-byte block holding its last byte is read.
__device__ __forceinline__ uint32_t load_le32(uint64_t a) {
  const uint32_t sh = static_cast<uint32_t>(a & 3u) * 8u;
  const uint64_t al = a & ~uint64_t(3);
  return sh ? funnel(sload2(al), sh) : sload1(al);
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
// Span sources (all values uniform).  Addresses are byte offsets from the
// source's base pointer.
// ---------------------------------------------------------------------------
constexpr uint32_t kSpanCut = 1u;   // G = 1 list entry: stop after the first segment
constexpr uint32_t kSpanCont = 2u;  // G > 1 list entry: continue from the partial CRC

struct SpanD {
  uint64_t a;      // offset of the first byte from the source base
  uint32_t n;      // bytes
  uint32_t init;   // Extend's init_crc
  uint32_t flags;  // kSpanCut / kSpanCont
  uint64_t id;     // output slot
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
    d.flags = 0u;
    d.id = s;
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
    return SpanD{s * stride, length, init, 0u, s};
  }
};

// A size-class list written by crc32c_lds_partition_kernel (SpanList,
// crc32c_lds.h); its count is read from device memory at kernel start.
struct ListSrc {
  const uint8_t* base;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* init;
  const uint32_t* id;
  uint64_t count;
  // scalar loads (the list arrays are written by the partition kernel, so
  // the compiler cannot prove them read-only: plain loads would be vector)
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    const uint32_t w = sload1(reinterpret_cast<uint64_t>(id + s));
    return SpanD{sload2(reinterpret_cast<uint64_t>(off + s)),
                 sload1(reinterpret_cast<uint64_t>(len + s)),
                 sload1(reinterpret_cast<uint64_t>(init + s)),
                 ((w & kListCut) ? kSpanCut : 0u) | ((w & kListCont) ? kSpanCont : 0u),
                 w & kListIdMask};
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
  uint64_t id;    // output slot
};

// The chunk geometry of a span at absolute address abs: h bytes of its first
// chunk lie in front of it, f full chunks, t tail bytes (for f == 0, the
// span's end inside chunk 0; 0 for an empty span).
struct Geo {
  uint32_t h, f, t;
  __device__ __forceinline__ Geo(uint64_t abs, uint32_t n) {
    h = static_cast<uint32_t>(abs & 15u);
    const uint32_t hn = h + n;
    f = hn >> 4;
    t = n == 0u ? 0u : (hn & 15u);
  }
};

// A span being walked segment by segment (G = 1).
struct Walk {
  uint64_t a0, id;
  uint32_t f, h, t, init, k, nseg;
  bool cut, valid;

  __device__ __forceinline__ void start(const uint8_t* base, const SpanD& d) {
    const Geo g(reinterpret_cast<uint64_t>(base) + d.a, d.n);
    h = g.h;
    f = g.f;
    t = g.t;
    a0 = d.a - h;
    init = d.init;
    id = d.id;
    k = 0;
    cut = (d.flags & kSpanCut) != 0u;
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
    // the tail: bytes [0, t) of the chunk after the last full one; a span
    // inside one chunk (f == 0) is all tail, bytes [h, t)
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

// The register that must enter a span's first chunk (h bytes in front of
// the span): ~init * x^(-8h).  Uniform.
__device__ __forceinline__ uint32_t head_register(uint32_t l, uint32_t init, uint32_t h) {
  return uni(init == 0u ? lds_ld(MiscAddr(kMiscHead0 + h)) : unshift(l, ~init, h));
}

// Byte mask of word ww of a chunk whose first h bytes are not the span's.
__device__ __forceinline__ uint32_t head_mask(uint32_t h, uint32_t ww) {
  return h >= 4u * ww + 4u ? 0u : (h <= 4u * ww ? ~0u : (~0u << (8u * (h - 4u * ww))));
}

// ---------------------------------------------------------------------------
// Per-workgroup unit counter: unit u of workgroup wg is span
// ((u / 16) * grid + wg) * 16 + u % 16 -- blocks of 16 spans round robin
// over the grid, so the chip reads one compact window of the batch at a
// time, and within a workgroup whichever wave is free takes the next span.
// ---------------------------------------------------------------------------
template <uint32_t N>
__device__ __forceinline__ uint64_t grab_units(uint32_t l) {
  l_u32w* ctr = reinterpret_cast<l_u32w*>(static_cast<uintptr_t>(MiscAddr(kMiscUnit)));
  uint32_t u = 0;
  if (l == 0u) u = __atomic_fetch_add(ctr, N, __ATOMIC_RELAXED);
  u = uni(u);
  return (static_cast<uint64_t>(u >> 4) * gridDim.x + blockIdx.x) * 16u + (u & 15u);
}

// Lane-invariant pieces of the pipeline.
struct Pipe {
  uint32_t l, slot, cm;
  uint32_t rpos[4];
  __device__ __forceinline__ void init(uint32_t lane, uint32_t wave) {
    l = lane;
    slot = kLdsSlots + wave * kSlotBytes;
    // DMA load q, lane m: chunk 64q + cm of the 256-chunk window
    cm = 4u * (lane >> 2) + (((lane & 3u) - (lane >> 4)) & 3u);
    // stripe read i of lane l: LDS position 4l + ((i + (l >> 2)) & 3)
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) rpos[i] = slot + 16u * (4u * lane + ((i + (lane >> 2)) & 3u));
  }
  // The slot into 16 words: W[4i + j] = word j of stripe chunk i.
  __device__ __forceinline__ void read(uint32_t (&W)[16]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32x4 d = *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(rpos[i]));
      W[4 * i] = d.x;
      W[4 * i + 1] = d.y;
      W[4 * i + 2] = d.z;
      W[4 * i + 3] = d.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is free again
  }
  // DMA window instructions [q0, q0 + nq) of a window of `cap` chunks whose
  // last nc hold a segment at base: chunks in front of it re-read its first
  // chunk (zeroed later).
  template <uint32_t NQ>
  __device__ __forceinline__ void issue(uint64_t base, uint32_t q0, uint32_t cap, uint32_t nc) const {
    // window chunk 64 j + cm of the group (load q0 + j) is segment chunk
    // 64 j + cm - (cap - nc)
    const int32_t b = 16 * (static_cast<int32_t>(cm) - static_cast<int32_t>(cap - nc));
    const uint32_t o0 = static_cast<uint32_t>(max(b, 0));
    const uint32_t o1 = static_cast<uint32_t>(max(b + 1024, 0));
    if constexpr (NQ == 4) {
      dma4(base, slot, o0, o1, static_cast<uint32_t>(max(b + 2048, 0)),
           static_cast<uint32_t>(max(b + 3072, 0)));
    } else if constexpr (NQ == 2) {
      dma2(base, slot + 1024u * q0, o0, o1);
    } else {
      dma1nt(base, slot + 1024u * q0, o0);
    }
  }
};

// ---------------------------------------------------------------------------
// G = 1: one segment per wave iteration, spans of any length.  Issue order
// of vector-memory instructions per wave:
//   DMA(seg i) ... result store(seg i-1) ... DMA(seg i+1) ...
// so waiting for seg i's DMA is vmcnt(1) when a store followed it, else 0.
// OUT: 0 = CRC (masked with kFlagMask), 1 = verify status byte.
// ---------------------------------------------------------------------------
template <int OUT, typename Src>
__device__ __forceinline__ void run1(const Src& src, void* out, uint32_t* partial, uint32_t flags,
                                     const uint8_t* image) {
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t w = uni(threadIdx.x >> 6);
  const uint64_t count = src.count;
  if (static_cast<uint64_t>(blockIdx.x) * 16u >= count) return;  // no block of work
  load_image(image, w, l);
  const Lane lk = make_lane<1>(l);
  Pipe pp;
  pp.init(l, w);
  const bool msk = (flags & kFlagMask) != 0u;
  const uint64_t sbase = reinterpret_cast<uint64_t>(src.base);

  auto next_span = [&](Walk& wk) {
    const uint64_t s = grab_units<1>(l);
    if (s >= count) {
      wk.valid = false;
      return;
    }
    wk.start(src.base, src.get(s));
  };
  auto issue = [&](const Seg& g) {
    if (g.nc == kSegChunks) {
      dma4(sbase + g.a0, pp.slot, 16u * pp.cm, 16u * pp.cm + 1024u, 16u * pp.cm + 2048u,
           16u * pp.cm + 3072u);
    } else if (g.nc != 0u) {
      pp.issue<4>(sbase + g.a0, 0u, kSegChunks, g.nc);
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
    if (OUT == 1 && !(g.flags & kSegCut)) stored = load_le32(sbase + g.a0 + 16u * g.nc + g.e);
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
    uint32_t W[16];
    pp.read(W);
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
      const uint32_t inj = (cur.flags & kSegFirst) ? head_register(l, cur.init, cur.h) : chain;
      if (cur.nc == kSegChunks && cur.h == 0u) {
        W[0] ^= l == 0u ? inj : 0u;
      } else {
        // chunk i of lane l is segment chunk 4l + i - (256 - nc): zero the
        // ones in front of the segment, mask the first h bytes of chunk 0
        // and put the register there
        const int32_t base = static_cast<int32_t>(kSegChunks - cur.nc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int32_t ci = static_cast<int32_t>(4u * l) + i - base;
#pragma unroll
          for (uint32_t ww = 0; ww < 4; ++ww)
            W[4 * i + ww] &= ci < 0 ? 0u : (ci == 0 ? head_mask(cur.h, ww) : ~0u);
          W[4 * i] ^= ci == 0 ? inj : 0u;
        }
      }
      R = fold<1>(lk, l, scan(lk, W))[0];
    }

    bool did_store = false;
    if (cur.flags & kSegLast) {
      if (cur.e > cur.o) R = feed_tail(lk, l, R, tail, cur.o, cur.e);
      const uint32_t crc = ~R;
      did_store = true;
      if (l == 0u) {
        if (cur.flags & kSegCut) {
          // partial CRC of a span a size-class kernel finishes
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
// G = 2, 4: G spans per wave iteration, one per group of 64 / G lanes, each
// at most 256 / G chunks + a tail (a size-class list guarantees it).
// ---------------------------------------------------------------------------
template <int G>
struct GroupSpan {
  uint64_t a0;      // offset of the span's first chunk
  uint32_t nc;      // full chunks (<= 256 / G)
  uint32_t h, o, e; // head bytes, tail range
  uint32_t inj;     // register entering the first chunk
  uint32_t init;    // ~register for nc == 0 (all-tail spans)
  uint32_t id;
  bool valid, cont;
};

template <int G, int OUT>
__device__ __forceinline__ void run_g(const ListSrc& src, void* out, uint32_t* partial,
                                      uint32_t flags, const uint8_t* image) {
  constexpr uint32_t LG = 64u / G, CAP = kSegChunks / G;
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t w = uni(threadIdx.x >> 6);
  const uint64_t count = src.count;
  if (static_cast<uint64_t>(blockIdx.x) * 16u >= count) return;
  load_image(image, w, l);
  const Lane lk = make_lane<G>(l);
  Pipe pp;
  pp.init(l, w);
  const bool msk = (flags & kFlagMask) != 0u;
  const uint64_t sbase = reinterpret_cast<uint64_t>(src.base);
  const uint32_t gl = l % LG;
  const uint32_t* cont_src = OUT == 1 ? partial : static_cast<const uint32_t*>(out);

  typedef GroupSpan<G> GS;
  auto load = [&](GS (&gs)[G]) {
    const uint64_t s0 = grab_units<G>(l);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint64_t s = s0 + g;
      gs[g].valid = s < count;
      gs[g].nc = 0;
      gs[g].h = gs[g].o = gs[g].e = 0;
      gs[g].inj = gs[g].init = 0;
      gs[g].id = 0;
      gs[g].a0 = 0;
      gs[g].cont = false;
      if (!gs[g].valid) continue;
      const SpanD d = src.get(s);
      const Geo geo(sbase + d.a, d.n);
      gs[g].a0 = d.a - geo.h;
      gs[g].nc = geo.f;
      gs[g].h = geo.h;
      gs[g].o = geo.f == 0u ? geo.h : 0u;
      gs[g].e = geo.t;
      gs[g].id = static_cast<uint32_t>(d.id);
      gs[g].cont = (d.flags & kSpanCont) != 0u;
      // a continuation starts 16-aligned (h = 0) from the partial CRC
      gs[g].init = gs[g].cont ? sload1(reinterpret_cast<uint64_t>(cont_src + d.id)) : d.init;
    }
  };
  auto issue = [&](const GS (&gs)[G]) {
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (gs[g].valid && gs[g].nc != 0u) {
        if constexpr (G == 2) pp.issue<2>(sbase + gs[g].a0, 2u * g, CAP, gs[g].nc);
        else pp.issue<1>(sbase + gs[g].a0, static_cast<uint32_t>(g), CAP, gs[g].nc);
      }
  };
  auto load_end = [&](const GS (&gs)[G], u32x4 (&tail)[G], uint32_t (&stored)[G]) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      tail[g] = u32x4{0, 0, 0, 0};
      stored[g] = 0;
      if (!gs[g].valid) continue;
      if (gs[g].e != 0u) tail[g] = sload4(sbase + gs[g].a0 + 16u * gs[g].nc);
      if (OUT == 1) stored[g] = load_le32(sbase + gs[g].a0 + 16u * gs[g].nc + gs[g].e);
    }
  };
  // per-lane value of this lane's group: masked selects on per-group lane
  // masks (an opaque lane id keeps the compiler from turning the select
  // chain into an indexed scratch array -- scratch accesses would count in
  // vmcnt and break the hand-counted DMA waits)
  uint32_t lo = l;
  asm volatile("" : "+v"(lo));
  uint32_t gm[G];
#pragma unroll
  for (int g = 0; g < G; ++g) gm[g] = 0u - static_cast<uint32_t>(lo / LG == static_cast<uint32_t>(g));
  auto pick = [&](const uint32_t (&v)[G]) -> uint32_t {
    uint32_t r = v[0] & gm[0];
#pragma unroll
    for (int g = 1; g < G; ++g) r |= v[g] & gm[g];
    return r;
  };

  GS cur[G], nxt[G];
  load(cur);
  if (!cur[0].valid) return;
  issue(cur);
  u32x4 tail[G];
  uint32_t stored[G];
  load_end(cur, tail, stored);
  load(nxt);
  bool stored_prev = false;

  for (;;) {
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    uint32_t W[16];
    pp.read(W);
    if (nxt[0].valid) issue(nxt);

    // ---- the G spans of this iteration ----
    uint32_t inj_g[G], nc_g[G], h_g[G];
    bool fast = true;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      inj_g[g] = cur[g].valid ? head_register(l, cur[g].init, cur[g].h) : 0u;
      nc_g[g] = cur[g].valid ? cur[g].nc : 0u;
      h_g[g] = cur[g].h;
      fast = fast && nc_g[g] == CAP && h_g[g] == 0u;
    }
    const uint32_t inj = pick(inj_g);
    if (fast) {
      W[0] ^= gl == 0u ? inj : 0u;
    } else {
      const int32_t base = static_cast<int32_t>(CAP - pick(nc_g));
      const uint32_t hh = pick(h_g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t ci = static_cast<int32_t>(4u * gl) + i - base;
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww)
          W[4 * i + ww] &= ci < 0 ? 0u : (ci == 0 ? head_mask(hh, ww) : ~0u);
        W[4 * i] ^= ci == 0 ? inj : 0u;
      }
    }
    const auto Rg = fold<G>(lk, l, scan(lk, W));
    // registers after the main chunks; all-tail spans start from ~init
    uint32_t R[G], o_g[G], e_g[G];
    uint32_t tw[4][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      R[g] = cur[g].nc == 0u ? ~cur[g].init : Rg[g];
      o_g[g] = cur[g].o;
      e_g[g] = cur[g].valid ? cur[g].e : 0u;
      tw[0][g] = tail[g].x;
      tw[1][g] = tail[g].y;
      tw[2][g] = tail[g].z;
      tw[3][g] = tail[g].w;
    }
    // tails, all groups in the same instructions (lane l serves its group)
    uint32_t r = pick(R);
    {
      uint32_t need = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) need |= e_g[g];
      if (need != 0u) {
        const uint32_t o = pick(o_g), e = pick(e_g);
        const u32x4 t{pick(tw[0]), pick(tw[1]), pick(tw[2]), pick(tw[3])};
        r = feed_tail_lanes(lk, l, r, t, o, e);
      }
    }
    // results: the group leaders store
    const uint32_t val = ~r;
    bool valid_l = false;
    uint32_t ids[G], st[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      ids[g] = cur[g].id;
      st[g] = stored[g];
      valid_l = valid_l || (gm[g] != 0u && cur[g].valid);
    }
    const uint32_t myid = pick(ids);
    if (gl == 0u && valid_l) {
      if (OUT == 1) {
        static_cast<uint8_t*>(out)[myid] = unmask_crc(pick(st)) == val ? 1u : 0u;
      } else {
        static_cast<uint32_t*>(out)[myid] = msk ? mask_crc(val) : val;
      }
    }
    stored_prev = true;

    if (!nxt[0].valid) break;
#pragma unroll
    for (int g = 0; g < G; ++g) cur[g] = nxt[g];
    load_end(cur, tail, stored);
    load(nxt);
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
  run1<0>(src, out, nullptr, flags, image);
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_lds_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image) {
  const StridedSrc src{base, stride, length, init, count};
  run1<0>(src, out, nullptr, flags & kFlagMask, image);
}

// Read-side verify (ReadBlock, kv/src/table/format.cc:91-99): block i =
// base + offsets[i], handle size n = lengths[i]; CRC over n + 1 bytes
// compared with Unmask(LE32 at n + 1).
__global__ __launch_bounds__(kThreads) void crc32c_lds_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status, uint64_t count,
    const uint8_t* __restrict__ image) {
  const DescSrc src{base, offsets, lengths, nullptr, count, 1u};
  run1<1>(src, status, nullptr, 0u, image);
}

// A size-class list (HCRC_SPLIT_SMALL): G = 1 takes spans of more than
// 2 KiB (cut ones write their partial CRC), G = 2 / 4 the spans and
// remainders of at most 2 KiB / 1 KiB.  OUT: 0 = CRCs into out (u32), 1 =
// verify statuses into out (u8) with the cut blocks' partials in partial.
template <int G, int OUT>
__global__ __launch_bounds__(kThreads) void crc32c_lds_list_kernel(
    const uint8_t* __restrict__ base, SpanList list, void* out, uint32_t* partial, uint32_t flags,
    const uint8_t* __restrict__ image) {
  const uint32_t n = sload1(reinterpret_cast<uint64_t>(list.count));
  const ListSrc src{base, list.off, list.len, list.init, list.id, n};
  if constexpr (G == 1) run1<OUT>(src, out, partial, flags, image);
  else run_g<G, OUT>(src, out, partial, flags, image);
}
template __global__ void crc32c_lds_list_kernel<1, 0>(const uint8_t*, SpanList, void*, uint32_t*,
                                                      uint32_t, const uint8_t*);
template __global__ void crc32c_lds_list_kernel<2, 0>(const uint8_t*, SpanList, void*, uint32_t*,
                                                      uint32_t, const uint8_t*);
template __global__ void crc32c_lds_list_kernel<4, 0>(const uint8_t*, SpanList, void*, uint32_t*,
                                                      uint32_t, const uint8_t*);
template __global__ void crc32c_lds_list_kernel<1, 1>(const uint8_t*, SpanList, void*, uint32_t*,
                                                      uint32_t, const uint8_t*);
template __global__ void crc32c_lds_list_kernel<2, 1>(const uint8_t*, SpanList, void*, uint32_t*,
                                                      uint32_t, const uint8_t*);
template __global__ void crc32c_lds_list_kernel<4, 1>(const uint8_t*, SpanList, void*, uint32_t*,
                                                      uint32_t, const uint8_t*);

// ---------------------------------------------------------------------------
// Partition into size-class lists (HCRC_SPLIT_SMALL).  Workgroup w scans a
// contiguous range of the batch twice: counts per class, one global atomic
// per class to reserve its slices, then writes the entries (wave-ordered
// through a ballot prefix), so each list keeps the batch's memory order
// piecewise.
// ---------------------------------------------------------------------------
constexpr int kPartThreads = 256;

struct Classified {
  uint32_t cls;      // 1, 2 or 4
  bool cut;          // class 1: remainder entry too
  uint32_t rcls;     // the remainder's class
  uint64_t roff;     // remainder: offset of its first byte
  uint32_t rlen;
};

__device__ __forceinline__ Classified classify(const uint8_t* base, uint64_t off, uint32_t n) {
  Classified c;
  const uint32_t h = static_cast<uint32_t>((reinterpret_cast<uint64_t>(base) + off) & 15u);
  const uint32_t hn = h + n;
  const uint32_t f = hn >> 4;
  c.cls = f <= kClass4Chunks ? 4u : (f <= kClass2Chunks ? 2u : 1u);
  c.cut = f > kSegChunks && f - kSegChunks <= kClass2Chunks;
  c.rcls = 0;
  c.roff = 0;
  c.rlen = 0;
  if (c.cut) {
    const uint32_t first = kSegChunks * 16u - h;  // bytes of the first segment
    c.roff = off + first;
    c.rlen = n - first;
    c.rcls = (hn - kSegChunks * 16u) >> 4 <= kClass4Chunks ? 4u : 2u;
  }
  return c;
}

__device__ __forceinline__ void put(const SpanList& L, uint32_t pos, uint64_t off, uint32_t len,
                                    uint32_t init, uint32_t id) {
  L.off[pos] = off;
  L.len[pos] = len;
  L.init[pos] = init;
  L.id[pos] = id;
}

__global__ __launch_bounds__(kPartThreads) void crc32c_lds_partition_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits, uint64_t count,
    uint32_t extra, SpanList l1, SpanList l2, SpanList l4) {
  __shared__ uint32_t cnt[3], pos[3];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint64_t per = (count + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = per * blockIdx.x;
  const uint64_t hi = lo + per < count ? lo + per : count;
  if (tid < 3) cnt[tid] = 0;
  __syncthreads();
  auto slot = [](uint32_t cls) { return cls == 1u ? 0u : (cls == 2u ? 1u : 2u); };
  // pass 1: count
  uint32_t mine[3] = {0, 0, 0};
  for (uint64_t s = lo + tid; s < hi; s += kPartThreads) {
    const Classified c = classify(base, offsets[s], lengths[s] + extra);
    ++mine[slot(c.cls)];
    if (c.cut) ++mine[slot(c.rcls)];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (mine[k]) atomicAdd(&cnt[k], mine[k]);
  __syncthreads();
  if (tid == 0) {
    const SpanList* L[3] = {&l1, &l2, &l4};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pos[k] = cnt[k] ? atomicAdd(L[k]->count, cnt[k]) : 0u;
    }
  }
  __syncthreads();
  // pass 2: write, 64 spans per wave step, positions from a ballot prefix
  const SpanList* L[3] = {&l1, &l2, &l4};
  const uint64_t wbase = lo + (tid & ~63u);
  for (uint64_t s0 = wbase; s0 < hi; s0 += kPartThreads) {
    const uint64_t s = s0 + lane;
    const bool live = s < hi;
    Classified c{};
    uint64_t off = 0;
    uint32_t n = 0, ini = 0;
    if (live) {
      off = offsets[s];
      n = lengths[s] + extra;
      ini = inits ? inits[s] : 0u;
      c = classify(base, off, n);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t cls = k == 0 ? 1u : (k == 1 ? 2u : 4u);
      const bool a = live && c.cls == cls;
      const bool b = live && c.cut && c.rcls == cls;
      const uint64_t ma = __builtin_amdgcn_ballot_w64(a);
      const uint64_t mb = __builtin_amdgcn_ballot_w64(b);
      const uint32_t na = __builtin_popcountll(ma), nb = __builtin_popcountll(mb);
      if (na + nb == 0u) continue;
      uint32_t p0 = 0;
      if (lane == 0u) p0 = atomicAdd(&pos[k], na + nb);
      p0 = __builtin_amdgcn_readfirstlane(p0);
      const uint64_t below = (uint64_t(1) << lane) - 1u;
      if (a)
        put(*L[k], p0 + __builtin_popcountll(ma & below), off, n, ini,
            static_cast<uint32_t>(s) | (c.cut ? kListCut : 0u));
      if (b)
        put(*L[k], p0 + na + __builtin_popcountll(mb & below), c.roff, c.rlen, 0u,
            static_cast<uint32_t>(s) | kListCont);
    }
  }
}

}  // namespace lk
}  // namespace wipdb
