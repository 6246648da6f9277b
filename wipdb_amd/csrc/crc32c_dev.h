// crc32c_dev.h -- device helpers shared by the LDS-staged CRC32C kernels
// (crc32c_lds.hip: the lane-packed spans / strided / verify kernels;
// crc32c_list.hip: the size-class list kernels): the slicing-by-4 step on
// the rotated LDS tables, the two-level fold, the LDS DMA instructions, the
// per-workgroup unit counter and the slot pipeline.  DESIGN.md sections 3-4.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// kv/src/util/crc32c.cc:1225-1227); its hot loop is crc32c_3way
// (crc32c.cc:667-1198), whose CombineCRC (crc32c.cc:640-657) the fold
// tables restate (CDNA4 has no carry-less multiply).
#pragma once
#include <stdint.h>

#include <type_traits>

#include "crc32c_lds.h"
#include "crc32c_plan.h"
// the hardware primitives (DPP, ballot, LDS, DMA ...); tests/cpp/lk_emu.h
// supplies the same functions for the host SIMT emulation of the kernels
#if defined(WIPDB_LK_EMU)
#include "lk_emu.h"
#else
#include "crc32c_prim.h"
#endif

namespace wipdb {
namespace lk {

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
  const uint32_t a0 = lds_ld(kLdsMain + vperm(k.km, x, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + vperm(k.km, x, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + vperm(k.km, x, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + vperm(k.km, x, k.sel[3]));
  return xor3(xor3(a0, a1, a2), a3, wn);
}

// r * x^(8 * 64 a) mod P (a = 7 - l % 8; a = 0: r itself)
__device__ __forceinline__ uint32_t fold_l1(const Lane& k, uint32_t l, uint32_t r) {
  const uint32_t a0 = lds_ld(kLdsMain + vperm(k.k1, r, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + vperm(k.k1, r, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + vperm(k.k1, r, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + vperm(k.k1, r, k.sel[3]));
  const uint32_t v = xor3(a0, a1, a2) ^ a3;
  return (l & 7u) == 7u ? r : v;
}

// r * x^(8 * 512 c) mod P (c of make_lane; c = 0: r itself)
template <int G>
__device__ __forceinline__ uint32_t fold_l2(const Lane& k, uint32_t l, uint32_t r) {
  constexpr uint32_t LG = 64u / G;
  const uint32_t a0 = lds_ld(kLdsL2 + (vperm(k.k2, r, k.sel[0]) >> 1));
  const uint32_t a1 = lds_ld(kLdsL2 + (vperm(k.k2, r, k.sel[1]) >> 1));
  const uint32_t a2 = lds_ld(kLdsL2 + (vperm(k.k2, r, k.sel[2]) >> 1));
  const uint32_t a3 = lds_ld(kLdsL2 + (vperm(k.k2, r, k.sel[3]) >> 1));
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
    f.v[0] = rdlane(w, 0) ^ rdlane(w, 16) ^
             rdlane(w, 32) ^ rdlane(w, 48);
  } else if constexpr (G == 2) {
    f.v[0] = rdlane(w, 0) ^ rdlane(w, 16);
    f.v[1] = rdlane(w, 32) ^ rdlane(w, 48);
  } else {
#pragma unroll
    for (int g = 0; g < 4; ++g) f.v[g] = rdlane(w, 16 * g);
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
    if (ballot(p) == 0u) break;
    const uint32_t wd = b < 4u ? t.x : (b < 8u ? t.y : (b < 12u ? t.z : t.w));
    const uint32_t x = feed_byte(l, r, (wd >> (8u * (b & 3u))) & 0xffu);
    r = p ? x : r;
  }
  return r;
}

// The table image (tables + misc words) into LDS [0, 96 KiB): wave w copies
// 6 KiB with 6 DMAs.  Ends with the workgroup barrier.
__device__ __forceinline__ void load_image(const uint8_t* image, uint32_t w, uint32_t l) {
  constexpr uint32_t per = kImageBytes / kWaves;  // 6 KiB
  const uint64_t src = reinterpret_cast<uint64_t>(image) + w * per;
#pragma unroll
  for (uint32_t q = 0; q < per / 1024u; ++q) dma1(src, w * per + 1024u * q, 1024u * q + 16u * l);
  wait_vm<0>();
  wg_sync();
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
  const uint32_t* bounds;  // HCRC_BALANCE: workgroup ranges (else nullptr)
  __device__ __forceinline__ SpanD get(uint64_t s) const {
    return SpanD{off[s], len[s] + extra, kInit ? init[s] : 0u, static_cast<uint32_t>(s)};
  }
  // per lane (a desk of run_lp): vector loads, waited for at first use --
  // n is the length column as loaded (bytes(n) adds the type byte: no
  // arithmetic on a load still in flight)
  __device__ __forceinline__ void lane(uint64_t s, uint64_t& a, uint32_t& n, uint32_t& i) const {
    a = off[s];
    n = len[s];
    i = kInit ? init[s] : 0u;
  }
  __device__ __forceinline__ uint32_t bytes(uint32_t n) const { return n + extra; }
  // (a vector load: see vzero)
  __device__ __forceinline__ uint32_t init_of(uint64_t s) const {
    return kInit ? init[s + vzero()] : 0u;
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
  __device__ __forceinline__ void lane(uint64_t s, uint64_t& a, uint32_t& n, uint32_t& i) const {
    a = s * stride;
    n = length;
    i = init;
  }
  __device__ __forceinline__ uint32_t bytes(uint32_t n) const { return n; }
  __device__ __forceinline__ uint32_t init_of(uint64_t) const { return init; }
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
// The spans past the last whole round (count mod 16 grid) go round robin one
// at a time (unit u >= full: span u * grid + wg), so no workgroup holds more
// than one span beyond another's: blocks of 16 left up to 16 long spans on
// one workgroup while others had none (config 3's 32 / 64 KiB buckets:
// 15.04 / 7.52 blocks per workgroup, the launch paced by 16 / 8).
// ---------------------------------------------------------------------------
//
// HCRC_BALANCE: bounds (device, G + 1 entries, util::balance_bounds_kernel)
// give the workgroup the contiguous spans [bounds[g], bounds[g + 1]) instead,
// cut by weight, not count (lo = its first span; full = kBalanced).
constexpr uint32_t kBalanced = ~0u;
template <typename Src>
__device__ __forceinline__ const uint32_t* src_bounds(const Src&) { return nullptr; }
template <bool kInit>
__device__ __forceinline__ const uint32_t* src_bounds(const DescSrc<kInit>& s) { return s.bounds; }
struct WgUnits {
  uint32_t full;   // units in whole rounds (a multiple of 16); kBalanced: a range
  uint32_t count;  // the workgroup's units
  uint32_t lo;     // kBalanced: the first span of the range
};
__device__ __forceinline__ WgUnits wg_units(uint64_t count, const uint32_t* bounds) {
  const uint64_t G = group_count(), g = group_id();
  WgUnits u;
  if (bounds != nullptr) {
    u.lo = bounds[g];
    u.count = bounds[g + 1u] - u.lo;
    u.full = kBalanced;
    return u;
  }
  const uint64_t full = count / (16u * G) * 16u;
  const uint64_t rest = count - full * G;  // < 16 G
  u.full = static_cast<uint32_t>(full);
  u.count = static_cast<uint32_t>(full + (rest > g ? (rest - g - 1u) / G + 1u : 0u));
  u.lo = 0u;
  return u;
}
__device__ __forceinline__ uint64_t unit_span(uint32_t u, const WgUnits& w) {
  const uint64_t G = group_count(), g = group_id();
  if (w.full == kBalanced) return u < w.count ? static_cast<uint64_t>(w.lo) + u : ~0ull;
  return u < w.full ? (static_cast<uint64_t>(u >> 4) * G + g) * 16u + (u & 15u)
                    : static_cast<uint64_t>(u) * G + g;
}
// One unit (run_ea): its span (>= count once the workgroup's units are out).
__device__ __forceinline__ uint64_t grab_unit(uint32_t l, const WgUnits& w) {
  uint32_t u = 0;
  if (l == 0u) u = lds_add(MiscAddr(kMiscUnit), 1u);
  return unit_span(uni(u), w);
}
// N units at once (the size-class list kernels: N consecutive spans of one
// 16-span block, whole rounds only).
template <uint32_t N>
__device__ __forceinline__ uint64_t grab_units(uint32_t l) {
  uint32_t u = 0;
  if (l == 0u) u = lds_add(MiscAddr(kMiscUnit), N);
  u = uni(u);
  return (static_cast<uint64_t>(u >> 4) * group_count() + group_id()) * 16u + (u & 15u);
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
      const u32x4 d = lds_ld4(rpos[i]);
      W[4 * i] = d.x;
      W[4 * i + 1] = d.y;
      W[4 * i + 2] = d.z;
      W[4 * i + 3] = d.w;
    }
  }
  __device__ __forceinline__ u32x4 piece(uint32_t k) const {
    return lds_ld4(AuxAddr(w, k));
  }
  // aux piece k, k per lane
  __device__ __forceinline__ u32x4 piece_lane(uint32_t k) const {
    return lds_ld4(AuxAddr(w, k));
  }
  // Every LDS read of the slot and the pieces has returned: the next DMA may
  // overwrite them.
  __device__ __forceinline__ void release() const {
    lgkm_wait();
  }
  // DMA window loads [q0, q0 + NQ) of a window of `cap` chunks whose last
  // nc hold a segment at base: chunks in front of it re-read its first chunk
  // (zeroed later).
  template <uint32_t NQ>
  __device__ __forceinline__ void issue(uint64_t base, uint32_t q0, uint32_t cap, uint32_t nc) const {
    // window chunk 64 j + cm of the group (load q0 + j) is segment chunk
    // 64 j + cm - (cap - nc)
    const int32_t b = 16 * (static_cast<int32_t>(cm) - static_cast<int32_t>(cap - nc));
    const uint32_t o0 = static_cast<uint32_t>(b > 0 ? b : 0);
    const uint32_t o1 = static_cast<uint32_t>(b + 1024 > 0 ? b + 1024 : 0);
    if constexpr (NQ == 4) {
      if (nc == cap)
        dma4(base, slot, 16u * cm, 16u * cm + 1024u, 16u * cm + 2048u, 16u * cm + 3072u);
      else
        dma4(base, slot, o0, o1, static_cast<uint32_t>(b + 2048 > 0 ? b + 2048 : 0),
             static_cast<uint32_t>(b + 3072 > 0 ? b + 3072 : 0));
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
  const uint32_t a0 = lds_ld(kLdsMain + vperm(k.k1b, r, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + vperm(k.k1b, r, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + vperm(k.k1b, r, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + vperm(k.k1b, r, k.sel[3]));
  uint32_t v = (l & 3u) == 3u ? r : (xor3(a0, a1, a2) ^ a3);
  v ^= dpp<0xB1>(v);  // quad_perm [1,0,3,2]
  v ^= dpp<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}

// r * x^(8 * 512 c) mod P from the level-2 tables, for any lane (kc: the
// lane's selector constant for column c, make_l2c).
__device__ __forceinline__ uint32_t l2_shift(const Lane& k, uint32_t kc, uint32_t r) {
  const uint32_t a0 = lds_ld(kLdsL2 + (vperm(kc, r, k.sel[0]) >> 1));
  const uint32_t a1 = lds_ld(kLdsL2 + (vperm(kc, r, k.sel[1]) >> 1));
  const uint32_t a2 = lds_ld(kLdsL2 + (vperm(kc, r, k.sel[2]) >> 1));
  const uint32_t a3 = lds_ld(kLdsL2 + (vperm(kc, r, k.sel[3]) >> 1));
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
  return bperm_raw(v, lane);
}

}  // namespace lk
}  // namespace wipdb
