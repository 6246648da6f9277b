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
// Descriptors are scalar (SMEM) loads issued an iteration ahead; a span's
// tail chunk and stored trailer come in with its segment as one-lane DMAs
// into per-wave aux pieces.  Every vector-memory instruction is a DMA or a
// result store, counted by hand (s_waitcnt vmcnt) -- see the issue order in
// run_ea().
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32c_lds.h"
#include "crc32c_walk.h"

namespace wipdb {
namespace lk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t l_u32;
typedef __attribute__((address_space(3))) uint32_t l_u32w;
typedef __attribute__((address_space(3))) const u32x4 l_u32x4;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint8_t g_u8;

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
  uint32_t k1b;     // byte j: 128 + 4 (4 b + t_j), b = 3 - l % 4 (4-lane groups' level 1)
};

// G: spans per wave (groups of 64 / G lanes); the level-2 fold shifts the
// 8-lane block b of a group by 512 (blocks - 1 - b) bytes.
template <int G>
__device__ __forceinline__ Lane make_lane(uint32_t l) {
  Lane k;
  constexpr uint32_t LG = 64u / G;
  const uint32_t q = (l >> 3) & 3u, r = l & 7u, a = 7u - (l & 7u);
  const uint32_t c = (LG / 8u - 1u) - ((l % LG) >> 3);
  k.km = k.k1 = k.k2 = k.k1b = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t t = (j + q) & 3u;
    k.sel[j] = 0x0c0c0000u | (t << 8) | (4u + j);
    k.km |= (t * 32u + r * 4u) << (8 * j);
    k.k1 |= (128u + (a * 4u + t) * 4u) << (8 * j);
    k.k2 |= (8u * (c * 4u + t)) << (8 * j);
    k.k1b |= (128u + ((3u - (l & 3u)) * 4u + t) * 4u) << (8 * j);
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
      : "memory", "scc");
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
      : "memory", "scc");
}

__device__ __forceinline__ void dma1nt(uint64_t base, uint32_t dst, uint32_t off) {
  uint32_t keep;
  // (callers' values are uniform; say so, so they stay in SGPRs under a lane branch)
  dst = __builtin_amdgcn_readfirstlane(dst);
  base = uni64(base);
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

// One DMA with per-lane 64-bit source addresses (the lanes of one
// instruction may serve different spans).
__device__ __forceinline__ void dma1v(uint64_t addr, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(addr), "s"(dst)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
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
// source's base pointer.  Descriptor columns are const __restrict__ kernel
// arguments, so the compiler loads them with SMEM (asynchronously, waited
// for at first use).
// ---------------------------------------------------------------------------

// Descriptor batch: span i = base + offsets[i], lengths[i] (+ extra) bytes;
// kInit: an init column (else every init is 0 -- one pointer and one scalar
// load per span fewer for the batches that have none, e.g. WriteRawBlock's).
template <bool kInit>
struct DescSrc {
  const uint8_t* base;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* init;
  uint64_t count;
  uint32_t extra;  // verify: +1 type byte
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    return SpanD{off[s], len[s] + extra, kInit ? init[s] : 0u, static_cast<uint32_t>(s)};
  }
};

// Fixed-size blocks at a fixed stride.
struct StridedSrc {
  const uint8_t* base;
  uint64_t stride;
  uint32_t length, init;
  uint64_t count;
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    return SpanD{s * stride, length, init, static_cast<uint32_t>(s)};
  }
};

// A size-class list written by crc32c_lds_partition_kernel (SpanList).
struct ListSrc {
  const uint8_t* base;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* init;
  const uint32_t* id;
  uint64_t count;
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    return SpanD{off[s], len[s], init[s], id[s]};
  }
};

// ---------------------------------------------------------------------------
// Chunk geometry of the size-class lists' spans (run_g): a grid that starts
// at the span's first 16-byte-aligned chunk, with a ragged tail.
// ---------------------------------------------------------------------------
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

// The register that must enter a span's first chunk (h bytes in front of
// the span): ~init * x^(-8h).  Uniform.
__device__ __forceinline__ uint32_t head_register(uint32_t l, uint32_t init, uint32_t h) {
  return uni(init == 0u ? lds_ld(MiscAddr(kMiscHead0 + h)) : unshift(l, ~init, h));
}

// LE32 at byte e (< 16) of the 32 bytes lo || hi (a verify trailer).
__device__ __forceinline__ uint32_t le32_at(const u32x4& lo, const u32x4& hi, uint32_t e) {
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t a = w[0], b = w[1];
#pragma unroll
  for (uint32_t i = 1; i < 4; ++i) {
    if ((e >> 2) == i) {
      a = w[i];
      b = w[i + 1];
    }
  }
  const uint32_t sh = (e & 3u) * 8u;
  return sh ? (a >> sh) | (b << (32u - sh)) : a;
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

// One lane's DMA of a 16-byte chunk at base + off into an aux piece (the
// instruction runs with lane 0 alone: LDS destination M0 + 16 * 0).
__device__ __forceinline__ void dma_piece(uint32_t l, uint64_t base, uint32_t off, uint32_t dst) {
  if (l == 0u) dma1nt(base, dst, off);
}

// Lane-invariant pieces of the pipeline.
struct Pipe {
  uint32_t l, w, slot, cm;
  uint32_t rpos[4];
  __device__ __forceinline__ void init(uint32_t lane, uint32_t wave) {
    l = lane;
    w = wave;
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
  }
  __device__ __forceinline__ u32x4 piece(uint32_t k) const {
    return *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(AuxAddr(w, k)));
  }
  // aux piece k, k per lane
  __device__ __forceinline__ u32x4 piece_lane(uint32_t k) const {
    return *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(AuxAddr(w, k)));
  }
  // Every LDS read of the slot and the pieces has returned: the next DMA may
  // overwrite them.
  __device__ __forceinline__ void release() const {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // DMA window loads [q0, q0 + NQ) of a window of `cap` chunks whose last
  // nc hold a segment at base: chunks in front of it re-read its first chunk
  // (zeroed later).
  template <uint32_t NQ>
  __device__ __forceinline__ void issue(uint64_t base, uint32_t q0, uint32_t cap, uint32_t nc) const {
    // window chunk 64 j + cm of the group (load q0 + j) is segment chunk
    // 64 j + cm - (cap - nc)
    const int32_t b = 16 * (static_cast<int32_t>(cm) - static_cast<int32_t>(cap - nc));
    const uint32_t o0 = static_cast<uint32_t>(max(b, 0));
    const uint32_t o1 = static_cast<uint32_t>(max(b + 1024, 0));
    if constexpr (NQ == 4) {
      if (nc == cap)
        dma4(base, slot, 16u * cm, 16u * cm + 1024u, 16u * cm + 2048u, 16u * cm + 3072u);
      else
        dma4(base, slot, o0, o1, static_cast<uint32_t>(max(b + 2048, 0)),
             static_cast<uint32_t>(max(b + 3072, 0)));
    } else if constexpr (NQ == 2) {
      dma2(base, slot + 1024u * q0, o0, o1);
    } else {
      dma1nt(base, slot + 1024u * q0, o0);
    }
  }
  // A span's end chunks into aux pieces kAuxTail + g (its tail chunk) and
  // kAuxNext + g (the chunk after it, when a verify trailer at byte e
  // straddles the two).  tail: a ragged tail exists; trailer: verify.
  __device__ __forceinline__ void issue_end(uint64_t end_chunk, uint32_t g, bool tail, bool trailer,
                                            uint32_t e) const {
    if (tail || trailer) dma_piece(l, end_chunk, 0u, AuxAddr(w, kAuxTail + g));
    if (trailer && e > 12u) dma_piece(l, end_chunk, 16u, AuxAddr(w, kAuxNext + g));
  }
};

// ---------------------------------------------------------------------------
// The descriptor / strided / verify pipeline: the END-ALIGNED GRID
// (crc32c_walk.h: the grid, segments, pieces and their DMA sources).
// Main path: zero the window chunks in front of the segment (front, uniform)
// and put chunk 0 (window index front: lane front / 4, chunk front % 4) in
// its span form.
__device__ __forceinline__ void prepare_first(uint32_t (&W)[16], uint32_t l, uint32_t front,
                                              uint32_t hp, uint32_t ws, uint32_t inj) {
  if (front != 0u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool z = static_cast<int32_t>(4u * l) + i < static_cast<int32_t>(front);
#pragma unroll
      for (int w = 0; w < 4; ++w) W[4 * i + w] = z ? 0u : W[4 * i + w];
    }
  }
  const bool me = l == (front >> 2);
  // the chunk index is uniform: one static case
  auto apply = [&](auto I) {
    constexpr int i = decltype(I)::value;
    uint32_t c[4] = {W[4 * i], W[4 * i + 1], W[4 * i + 2], W[4 * i + 3]};
    fix_head(c, hp, ws, inj);
#pragma unroll
    for (int w = 0; w < 4; ++w) W[4 * i + w] = me ? c[w] : W[4 * i + w];
  };
  switch (front & 3u) {
    case 0: apply(std::integral_constant<int, 0>()); break;
    case 1: apply(std::integral_constant<int, 1>()); break;
    case 2: apply(std::integral_constant<int, 2>()); break;
    default: apply(std::integral_constant<int, 3>()); break;
  }
}

// Feeds the k (<= 3) low bytes of word tw into register r in one slicing
// step (tw = 0: r * x^(8k)).  Per lane.
__device__ __forceinline__ uint32_t tail_step(const Lane& lk, uint32_t r, uint32_t tw, uint32_t k) {
  const uint32_t x = (r ^ tw) << (8u * (4u - (k == 0u ? 4u : k)) & 31u);
  const uint32_t v = step(lk, k == 0u ? 0u : x, 0u) ^ (k == 0u ? r : (r >> (8u * k)));
  return v;
}

// The fold of 4-lane groups: lane l's register shifted by 64 (3 - l % 4)
// bytes (level-1 tables), XOR over the quad.  Valid in every lane.
__device__ __forceinline__ uint32_t fold4(const Lane& k, uint32_t l, uint32_t r) {
  const uint32_t a0 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1b, r, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1b, r, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1b, r, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + __builtin_amdgcn_perm(k.k1b, r, k.sel[3]));
  uint32_t v = (l & 3u) == 3u ? r : (xor3(a0, a1, a2) ^ a3);
  v ^= dpp<0xB1>(v);  // quad_perm [1,0,3,2]
  v ^= dpp<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}

// r * x^(8 * 512 c) mod P from the level-2 tables, for any lane (kc: the
// lane's selector constant for column c, make_l2c).
__device__ __forceinline__ uint32_t l2_shift(const Lane& k, uint32_t kc, uint32_t r) {
  const uint32_t a0 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(kc, r, k.sel[0]) >> 1));
  const uint32_t a1 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(kc, r, k.sel[1]) >> 1));
  const uint32_t a2 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(kc, r, k.sel[2]) >> 1));
  const uint32_t a3 = lds_ld(kLdsL2 + (__builtin_amdgcn_perm(kc, r, k.sel[3]) >> 1));
  return xor3(a0, a1, a2) ^ a3;
}
__device__ __forceinline__ uint32_t make_l2c(uint32_t l, uint32_t c) {
  const uint32_t q = (l >> 3) & 3u;
  uint32_t kc = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) kc |= (8u * (c * 4u + ((j + q) & 3u))) << (8 * j);
  return kc;
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(lane << 2),
                                                            static_cast<int>(v)));
}

struct PieceRing {
  uint32_t a_lo, a_hi, pw, inj, T, id;  // per lane: entry `lane`
  uint32_t head, count;                 // uniform
  __device__ __forceinline__ void push(uint32_t l, uint64_t c0, uint32_t w, uint32_t reg,
                                       uint32_t t, uint32_t sid) {
    const bool me = l == ((head + count) & 63u);
    a_lo = me ? static_cast<uint32_t>(c0) : a_lo;
    a_hi = me ? static_cast<uint32_t>(c0 >> 32) : a_hi;
    pw = me ? w : pw;
    inj = me ? reg : inj;
    T = me ? t : T;
    id = me ? sid : id;
    ++count;
  }
};

template <int OUT, typename Src>
__device__ __forceinline__ void run_ea(const Src& src, void* out, uint32_t flags,
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
  constexpr bool kVerify = OUT == 1;

  struct Pref {
    SpanD d;
    bool valid;
  };
  auto prefetch = [&](Pref& p) {
    const uint64_t s = grab_units<1>(l);
    p.valid = s < count;
    if (p.valid) p.d = src.get(s);
  };
  auto issue = [&](const SegE& g) {
    if (!(g.c.flags() & kENoBody)) {
      const uint64_t b = sbase + g.wb;
      const uint32_t o = 16u * pp.cm;
      if (g.src0 == 0u)
        dma4(b, pp.slot, o, o + 1024u, o + 2048u, o + 3072u);
      else
        dma4(b, pp.slot, SegChunkOffset(g, pp.cm), SegChunkOffset(g, pp.cm + 64u),
             SegChunkOffset(g, pp.cm + 128u), SegChunkOffset(g, pp.cm + 192u));
    }
    if (g.c.flags() & kEAux) dma_piece(l, sbase + g.ax, 0u, AuxAddr(w, kAuxTail));
  };
  PieceRing ring{0, 0, 0, 0, 0, 0, 0, 0};
  // a batch of the ring's next n (<= 16) pieces: their DMAs (16-chunk
  // windows END-aligned at each piece's last chunk).  Instruction q loads
  // pieces 4q .. 4q + 3, a quarter wave each, into slot KiB q: piece p's
  // window is slot bytes [256 p, 256 p + 256).
  auto issue_batch = [&](uint32_t h0, uint32_t n) {
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      if (4u * q >= n) break;
      const uint32_t p = 4u * q + (l >> 4);
      const uint32_t idx = (h0 + p) & 63u;
      const uint64_t c0 = (static_cast<uint64_t>(bperm(ring.a_hi, idx)) << 32) | bperm(ring.a_lo, idx);
      const uint32_t pw = bperm(ring.pw, idx);
      // lane m of the quarter loads window chunk cm mod 16 of its piece
      if (p < n) dma1v(sbase + c0 + PieceChunkOffset(pw, pp.cm & 15u), pp.slot + 1024u * q);
    }
  };

  WalkE wk;
  Pref pf;
  prefetch(pf);
  if (!pf.valid) return;
  wk.start(sbase, pf.d, kVerify);
  prefetch(pf);
  SegC cur;
  {
    const SegE g = wk.next();
    issue(g);
    cur = g.c;
  }
  uint32_t chain = 0;  // register carried between the segments of a span
  bool stored_prev = false;
  g_u32* const out32 = (g_u32*)(reinterpret_cast<uintptr_t>(out));
  g_u8* const out8 = (g_u8*)(reinterpret_cast<uintptr_t>(out));

  for (;;) {
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    uint32_t W[16];
    pp.read(W);
    u32x4 ax{0, 0, 0, 0};
    if (cur.flags() & kEAux) ax = pp.piece(kAuxTail);
    pp.release();
    // the next iteration: a batch of 8 pieces, the rest of this span, or
    // the prefetched span
    SegC nxt;
    nxt.g1 = 0;
    bool took_pf = false;
    const bool more = wk.valid || pf.valid;
    if (ring.count >= kBatch || (ring.count != 0u && !more)) {
      const uint32_t n = ring.count < kBatch ? ring.count : kBatch;
      nxt.g1 = kEValid | kEBatch;
      nxt.init = ring.head;
      nxt.id = n;
      issue_batch(ring.head, n);
      ring.head = (ring.head + n) & 63u;
      ring.count -= n;
    } else if (more) {
      bool fast = false;
      if (!wk.valid) {
        took_pf = true;
        uint64_t wb;
        fast = FastSeg(sbase, pf.d, kVerify, nxt, wb);
        if (fast) {
          // a simple span or a table block's main segment: one full window
          const uint32_t o = 16u * pp.cm;
          dma4(sbase + wb, pp.slot, o, o + 1024u, o + 2048u, o + 3072u);
        } else {
          wk.start(sbase, pf.d, kVerify);
        }
      }
      if (!fast) {
        const SegE g = wk.next();
        issue(g);
        nxt = g.c;
      }
    }

    bool did_store = false;
    if (cur.flags() & kEBatch) {
      // ---- a batch of front pieces, one per 4-lane group ----
      const uint32_t g = l >> 2, gl = l & 3u;
      const uint32_t idx = (cur.init + g) & 63u;
      const bool on = g < cur.id;
      const uint32_t pw = bperm(ring.pw, idx), inj = bperm(ring.inj, idx);
      const uint32_t T = bperm(ring.T, idx), sid = bperm(ring.id, idx);
      const int32_t front = static_cast<int32_t>(kPieceChunks - (on ? pw & 63u : 0u));
      const uint32_t hp = (pw >> 8) & 15u, ws = (pw >> 12) & 3u, k = (pw >> 14) & 3u;
      // window chunk 0 (the group leader's first chunk) is the span's aux
      // chunk: its tail word is the last word
      const uint32_t tw = W[3];
      // zero the chunks in front of the piece; its chunk 0 into span form
      uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t ci = static_cast<int32_t>(4u * gl) + i - front;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          c[q] = ci == 0 ? W[4 * i + q] : c[q];
          W[4 * i + q] = ci < 0 ? 0u : W[4 * i + q];
        }
      }
      fix_head(c, hp, ws, inj);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool h0 = static_cast<int32_t>(4u * gl) + i - front == 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) W[4 * i + q] = h0 ? c[q] : W[4 * i + q];
      }
      const uint32_t rp = fold4(lk, l, scan(lk, W));
      if (gl == 0u && on) {
        // register after piece || main = rp * x^(8 * 4096) ^ main register;
        // then the tail
        // (verify: T holds the residue, and there is no tail)
        const uint32_t sft = l2_shift(lk, make_l2c(l, 1u), l2_shift(lk, make_l2c(l, 7u), rp));
        if (kVerify) {
          out8[sid] = sft == T ? 1u : 0u;
        } else {
          const uint32_t v = tail_step(lk, sft ^ T, tw, k);
          out32[sid] = msk ? mask_crc(~v) : ~v;
        }
      }
      did_store = true;
    } else if (kVerify && (cur.flags() & kESimple)) {
      // ---- a simple verify span (the spans kernel measured faster through
      // the general segment code below): ~init enters at word 0, the stored
      // trailer is unmasked in place, a good block leaves the residue ----
      W[0] ^= l == 0u ? ~cur.init : 0u;
      uint32_t lo = W[14], hi = W[15];
      fix_trailer(lo, hi, cur.jv());
      W[14] = l == 63u ? lo : W[14];
      W[15] = l == 63u ? hi : W[15];
      const uint32_t R = fold<1>(lk, l, scan(lk, W))[0];
      if (l == 0u) {
        constexpr uint32_t kRes0 = verify_residue(0), kRes1 = verify_residue(1),
                           kRes2 = verify_residue(2), kRes3 = verify_residue(3);
        const uint32_t jv = cur.jv();
        const uint32_t res = jv == 0u ? kRes0 : (jv == 1u ? kRes1 : (jv == 2u ? kRes2 : kRes3));
        out8[cur.id] = R == res ? 1u : 0u;
      }
      did_store = true;
    } else {
      // ---- CRC of the current segment ----
      const uint32_t fl = cur.flags();
      uint32_t R;
      if (fl & kENoBody) {
        R = ~cur.init;
      } else {
        const uint32_t inj = (fl & kEFirst) ? head_register(l, cur.init, cur.hp())
                                            : ((fl & kEMain) ? 0u : chain);
        if ((cur.g1 & 0x1fff00u) == 0u) {  // front == 0, hp == 0
          W[0] ^= l == 0u ? inj : 0u;
        } else {
          prepare_first(W, l, cur.front(), cur.hp(), cur.ws(), inj);
        }
        if (kVerify && (fl & kELast)) {
          // the stored trailer, unmasked in place (lane 63, words 14-15)
          uint32_t lo = W[14], hi = W[15];
          fix_trailer(lo, hi, cur.jv());
          W[14] = l == 63u ? lo : W[14];
          W[15] = l == 63u ? hi : W[15];
        }
        R = fold<1>(lk, l, scan(lk, W))[0];
      }
      if (fl & kEAux) {
        const u32x4 a{uni(ax.x), uni(ax.y), uni(ax.z), uni(ax.w)};
        R = uni(tail_step(lk, R, le32_at(a, u32x4{0, 0, 0, 0}, cur.te()), cur.k()));
      }
      // verify: a good block leaves the residue
      constexpr uint32_t kRes0 = verify_residue(0), kRes1 = verify_residue(1),
                         kRes2 = verify_residue(2), kRes3 = verify_residue(3);
      const uint32_t jv = cur.jv();
      const uint32_t res = jv == 0u ? kRes0 : (jv == 1u ? kRes1 : (jv == 2u ? kRes2 : kRes3));
      if (fl & kEMain) {
        // the front piece goes to the ring with its head register; the span
        // (its tail) is finished there
        const uint32_t pw = cur.piece_word();
        const uint32_t hin = head_register(l, cur.init, cur.php());
        ring.push(l, cur.c0, pw, hin, kVerify ? R ^ res : R, cur.id);
      } else if (fl & kELast) {
        did_store = true;
        if (l == 0u) {
          if (kVerify) out8[cur.id] = R == res ? 1u : 0u;
          else out32[cur.id] = msk ? mask_crc(~R) : ~R;
        }
      } else {
        chain = R;
      }
    }
    stored_prev = did_store;

    if (!(nxt.g1 & kEValid)) {
      if (ring.count == 0u) break;
      // the last pieces, pushed by this iteration: their DMAs go out after
      // its store, so the next wait is for everything
      const uint32_t n = ring.count;
      nxt.g1 = kEValid | kEBatch;
      nxt.init = ring.head;
      nxt.id = n;
      issue_batch(ring.head, n);
      ring.head = (ring.head + n) & 63u;
      ring.count = 0;
      stored_prev = false;
    }
    if (took_pf) prefetch(pf);
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------
// G = 2, 4: G spans per wave iteration, one per group of 64 / G lanes, each
// at most 256 / G chunks + a tail (a size-class list guarantees it).
// ---------------------------------------------------------------------------
template <int G>
struct GroupSpan {
  uint64_t a0;  // offset of the span's first chunk
  // full chunks (<= 256 / G) | head bytes << 8 | tail range [o, e) << 12, 16 |
  // valid << 24 -- packed: the G-span loop is short of SGPRs
  uint32_t pk;
  uint32_t init;
  uint32_t id;
  __device__ __forceinline__ uint32_t nc() const { return pk & 0xffu; }
  __device__ __forceinline__ uint32_t h() const { return (pk >> 8) & 15u; }
  __device__ __forceinline__ uint32_t o() const { return (pk >> 12) & 15u; }
  __device__ __forceinline__ uint32_t e() const { return (pk >> 16) & 31u; }
  __device__ __forceinline__ bool valid() const { return (pk >> 24) != 0u; }
};

template <int G, int OUT>
__device__ __forceinline__ void run_g(const ListSrc& src, void* out, uint32_t flags,
                                      const uint8_t* image) {
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

  typedef GroupSpan<G> GS;
  // descriptors of the next G units (SMEM, waited for at first use)
  struct Pref {
    SpanD d[G];
    uint32_t nv;  // groups with a span (the first nv)
  };
  auto prefetch = [&](Pref& p) {
    const uint64_t s0 = grab_units<G>(l);
    p.nv = s0 >= count ? 0u : static_cast<uint32_t>(count - s0 < G ? count - s0 : G);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (static_cast<uint32_t>(g) < p.nv) p.d[g] = src.get(s0 + g);
  };
  auto take = [&](const Pref& p, GS (&gs)[G]) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      gs[g].pk = gs[g].init = gs[g].id = 0;
      gs[g].a0 = 0;
      if (static_cast<uint32_t>(g) >= p.nv) continue;
      const SpanD& d = p.d[g];
      const Geo geo(sbase + d.a, d.n);
      gs[g].a0 = d.a - geo.h;
      gs[g].pk = geo.f | (geo.h << 8) | ((geo.f == 0u ? geo.h : 0u) << 12) | (geo.t << 16) |
                 (1u << 24);
      gs[g].init = d.init;
      gs[g].id = static_cast<uint32_t>(d.id);
    }
  };
  auto issue = [&](const GS (&gs)[G]) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (!gs[g].valid()) continue;
      if (gs[g].nc() != 0u) {
        if constexpr (G == 2) pp.issue<2>(sbase + gs[g].a0, 2u * g, CAP, gs[g].nc());
        else pp.issue<1>(sbase + gs[g].a0, static_cast<uint32_t>(g), CAP, gs[g].nc());
      }
      pp.issue_end(sbase + gs[g].a0 + 16u * gs[g].nc(), static_cast<uint32_t>(g),
                   gs[g].e() > gs[g].o(), OUT == 1, gs[g].e());
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

  Pref pf;
  GS cur[G], nxt[G];
  prefetch(pf);
  if (pf.nv == 0u) return;
  take(pf, cur);
  prefetch(pf);
  issue(cur);
  bool stored_prev = false;

  for (;;) {
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    uint32_t W[16];
    pp.read(W);
    u32x4 tail[G], next[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      tail[g] = pp.piece(kAuxTail + g);
      next[g] = OUT == 1 ? pp.piece(kAuxNext + g) : u32x4{0, 0, 0, 0};
    }
    pp.release();
    const bool more = pf.nv != 0u;
    if (more) {
      take(pf, nxt);
      issue(nxt);
    }

    // ---- the G spans of this iteration ----
    uint32_t inj_g[G], nc_g[G], h_g[G];
    bool fast = true;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      inj_g[g] = cur[g].valid() ? head_register(l, cur[g].init, cur[g].h()) : 0u;
      nc_g[g] = cur[g].valid() ? cur[g].nc() : 0u;
      h_g[g] = cur[g].h();
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
    uint32_t R[G], o_g[G], e_g[G], tw[4][G], nw[4][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      R[g] = cur[g].nc() == 0u ? ~cur[g].init : Rg[g];
      o_g[g] = cur[g].o();
      e_g[g] = cur[g].valid() ? cur[g].e() : 0u;
      tw[0][g] = tail[g].x;
      tw[1][g] = tail[g].y;
      tw[2][g] = tail[g].z;
      tw[3][g] = tail[g].w;
      nw[0][g] = next[g].x;
      nw[1][g] = next[g].y;
      nw[2][g] = next[g].z;
      nw[3][g] = next[g].w;
    }
    // tails, all groups in the same instructions (lane l serves its group;
    // the aux pieces were read by every lane, so the words are uniform per
    // group already)
    uint32_t r = pick(R);
    const uint32_t o = pick(o_g), e = pick(e_g);
    const u32x4 t{pick(tw[0]), pick(tw[1]), pick(tw[2]), pick(tw[3])};
    {
      uint32_t need = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) need |= e_g[g];
      if (need != 0u) r = feed_tail_lanes(lk, l, r, t, o, e);
    }
    const uint32_t val = ~r;
    bool valid_l = false;
    uint32_t ids[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      ids[g] = cur[g].id;
      valid_l = valid_l || (gm[g] != 0u && cur[g].valid());
    }
    const uint32_t myid = pick(ids);
    if (gl == 0u && valid_l) {
      if (OUT == 1) {
        const u32x4 nx{pick(nw[0]), pick(nw[1]), pick(nw[2]), pick(nw[3])};
        static_cast<uint8_t*>(out)[myid] = unmask_crc(le32_at(t, nx, e)) == val ? 1u : 0u;
      } else {
        static_cast<uint32_t*>(out)[myid] = msk ? mask_crc(val) : val;
      }
    }
    stored_prev = true;

    if (!more) break;
#pragma unroll
    for (int g = 0; g < G; ++g) cur[g] = nxt[g];
    prefetch(pf);
  }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// Descriptor batch: out[i] = Extend(inits[i], base + offsets[i], lengths[i]);
// INIT = 0: no init column (all 0).
template <int INIT>
__global__ __launch_bounds__(kThreads) void crc32c_lds_spans_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image) {
  const DescSrc<INIT != 0> src{base, offsets, lengths, inits, count, 0u};
  run_ea<0>(src, out, flags, image);
}
template __global__ void crc32c_lds_spans_kernel<0>(const uint8_t*, const uint64_t*,
                                                    const uint32_t*, const uint32_t*, uint32_t*,
                                                    uint64_t, uint32_t, const uint8_t*);
template __global__ void crc32c_lds_spans_kernel<1>(const uint8_t*, const uint64_t*,
                                                    const uint32_t*, const uint32_t*, uint32_t*,
                                                    uint64_t, uint32_t, const uint8_t*);

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_lds_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image) {
  const StridedSrc src{base, stride, length, init, count};
  run_ea<0>(src, out, flags & kFlagMask, image);
}

// Read-side verify (ReadBlock, kv/src/table/format.cc:91-99): block i =
// base + offsets[i], handle size n = lengths[i]; CRC over n + 1 bytes
// compared with Unmask(LE32 at n + 1).
__global__ __launch_bounds__(kThreads) void crc32c_lds_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status, uint64_t count,
    const uint8_t* __restrict__ image) {
  const DescSrc<false> src{base, offsets, lengths, nullptr, count, 1u};
  run_ea<1>(src, status, 0u, image);
}

// A size-class list (HCRC_SPLIT_SMALL): G = 1 takes the spans of more than
// 128 chunks on the end-aligned pipeline (table blocks as main segment +
// front piece), G = 2 / 4 the spans of at most 128 / 64 chunks, several per
// wave iteration.  OUT: 0 = CRCs into out (u32, masked with kFlagMask),
// 1 = verify statuses into out (u8; the list lengths include the type byte).
template <int G, int OUT>
__global__ __launch_bounds__(kThreads) void crc32c_lds_list_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ init,
    const uint32_t* __restrict__ id, const uint32_t* __restrict__ count, void* out,
    uint32_t flags, const uint8_t* __restrict__ image) {
  const ListSrc src{base, off, len, init, id, *count};
  if constexpr (G == 1) run_ea<OUT>(src, out, flags, image);
  else run_g<G, OUT>(src, out, flags, image);
}
#define WIPDB_LIST_KERNEL(G, OUT)                                                          \
  template __global__ void crc32c_lds_list_kernel<G, OUT>(                                 \
      const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, const uint32_t*, \
      const uint32_t*, void*, uint32_t, const uint8_t*)
WIPDB_LIST_KERNEL(1, 0);
WIPDB_LIST_KERNEL(2, 0);
WIPDB_LIST_KERNEL(4, 0);
WIPDB_LIST_KERNEL(1, 1);
WIPDB_LIST_KERNEL(2, 1);
WIPDB_LIST_KERNEL(4, 1);
#undef WIPDB_LIST_KERNEL

// ---------------------------------------------------------------------------
// Partition into size-class lists (HCRC_SPLIT_SMALL).  Workgroup w scans a
// contiguous range of the batch twice: counts per class, one global atomic
// per class to reserve its slices, then writes the entries (wave-ordered
// through a ballot prefix), so each list keeps the batch's memory order
// piecewise.
// ---------------------------------------------------------------------------
constexpr int kPartThreads = 256;

// The class of a span of n bytes at address base + off: f = (a % 16 + n) / 16
// full chunks of its 16-byte grid; class 4: f <= 64, class 2: f <= 128,
// class 1: the rest.
__device__ __forceinline__ int class_slot(const uint8_t* base, uint64_t off, uint32_t n) {
  const uint32_t h = static_cast<uint32_t>((reinterpret_cast<uint64_t>(base) + off) & 15u);
  const uint32_t f = (h + n) >> 4;
  return f <= kClass4Chunks ? 2 : (f <= kClass2Chunks ? 1 : 0);
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
  // pass 1: count
  uint32_t mine[3] = {0, 0, 0};
  for (uint64_t s = lo + tid; s < hi; s += kPartThreads)
    ++mine[class_slot(base, offsets[s], lengths[s] + extra)];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (mine[k]) atomicAdd(&cnt[k], mine[k]);
  __syncthreads();
  if (tid == 0) {
    pos[0] = cnt[0] ? atomicAdd(l1.count, cnt[0]) : 0u;
    pos[1] = cnt[1] ? atomicAdd(l2.count, cnt[1]) : 0u;
    pos[2] = cnt[2] ? atomicAdd(l4.count, cnt[2]) : 0u;
  }
  __syncthreads();
  // pass 2: positions (ballot prefix per wave step of 64 spans), then writes
  const uint64_t wbase = lo + (tid & ~63u);
  const uint64_t below = (uint64_t(1) << lane) - 1u;
  for (uint64_t s0 = wbase; s0 < hi; s0 += kPartThreads) {
    const uint64_t s = s0 + lane;
    const bool live = s < hi;
    uint64_t off = 0;
    uint32_t n = 0, ini = 0;
    int cls = -1;
    if (live) {
      off = offsets[s];
      n = lengths[s] + extra;
      ini = inits ? inits[s] : 0u;
      cls = class_slot(base, off, n);
    }
    uint32_t pa = 0;  // this lane's entry position
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(cls == k);
      if (m == 0u) continue;
      uint32_t p0 = 0;
      if (lane == 0u) p0 = atomicAdd(&pos[k], static_cast<uint32_t>(__builtin_popcountll(m)));
      p0 = __builtin_amdgcn_readfirstlane(p0);
      if (cls == k) pa = p0 + __builtin_popcountll(m & below);
    }
    if (live) {
      const SpanList& L = cls == 0 ? l1 : (cls == 1 ? l2 : l4);
      L.off[pa] = off;
      L.len[pa] = n;
      L.init[pa] = ini;
      L.id[pa] = static_cast<uint32_t>(s);
    }
  }
}

}  // namespace lk
}  // namespace wipdb
