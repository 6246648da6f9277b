// crc32c_kernels.hip -- hand-written CDNA4 (gfx950) kernels for batched
// CRC32C of WipDB table blocks.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// crc32c.cc:1225-1227) applied to every block span, as WriteRawBlock
// (kv/src/table/table_builder.cc:194-196) and ReadBlock
// (kv/src/table/format.cc:91-93) do one block at a time.
//
// Design (DESIGN.md "Kernels"):
//   * one span per wavefront, cut into 4 KiB segments of its 16-byte chunk
//     grid.  A segment's 256 chunks are 64*K one-chunk stripes ("virtual
//     lanes"): lane l runs K = 4 independent CRC chains over chunks l,
//     64+l, 128+l, 192+l, so each 16-byte load instruction of the wave reads
//     one contiguous KiB (fully coalesced).  The K chains give the
//     LDS-latency-bound byte scan instruction-level parallelism.
//   * CRC arithmetic is table-driven from LDS (CDNA4 has no carry-less
//     multiply and this is a byte scan, not a contraction: no MFMA):
//     slicing-by-2 tables replicated 32x so lane l always reads bank l&31 --
//     every lookup is bank-conflict free -- and each lookup address is built
//     by ONE v_perm_b32 (table byte | lane byte | region byte).
//   * the 256 stripe registers are folded by a GF(2) tree: an in-lane Horner
//     step over the 4 chains (shift by 1 KiB), then a 6-level wavefront
//     butterfly (DPP row shifts, then v_readlane),
//        reg(v) = shift(reg(v), 16 * 2^t bytes) ^ reg(v + 2^t),
//     where shift by 16*2^j bytes is 4 lookups in a "multiply by
//     x^(8*16*2^j) mod P" table (the carry-less combine of the reference's
//     CombineCRC, crc32c.cc:640-657, done with tables).
//   * unaligned starts: the first chunk's leading bytes are zeroed and the
//     register injected there is pre-un-shifted (~init * x^(-8h)) so it
//     equals ~init at the first real byte; the ragged end (< 16 bytes) is
//     fed after the fold.  Segments of one span are chained through init.
//     So any offset/length/init is bit-exact.
//   * latency hiding: persistent grid (1 workgroup of 16 waves per CU), each
//     wave walks its spans' segments through a 3-slot register ring (two
//     segments of loads in flight while one is computed); 64 span
//     descriptors are fetched per vector load.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

#ifndef WIPDB_FOLD_SELECT
#define WIPDB_FOLD_SELECT 0
#endif
#ifndef WIPDB_OUTBUF
#define WIPDB_OUTBUF 1
#endif
#ifndef WIPDB_RING_SLOTS
#define WIPDB_RING_SLOTS 3
#endif

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

// s0 = lane constant: byte0 = (lane&31)*4 (T1), byte1 = (lane&31)*4|0x80
// (T0), byte2 = 0x01 (the 64 KiB region of the main tables).
constexpr uint32_t kSelT1B0 = 0x0c060004u;  // [s0.b0, x.b0, s0.b2, 0] -> T1[x.b0]
constexpr uint32_t kSelT0B1 = 0x0c060105u;  // [s0.b1, x.b1, s0.b2, 0] -> T0[x.b1]

// Feed one little-endian 32-bit word into register r (slicing-by-2 twice).
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
  return lds_ld(kLdsMain + ((x << 8) | ((s0 >> 8) & 0xffu))) ^ (r >> 8);
}

// r * x^(8 * 16 * 2^J) mod P: 4 lookups in shift table J.  The table base
// is a compile-time constant that lands in the ds_read offset field, so
// each address is one v_lshlrev_b32_sdwa (byte select).
template <uint32_t J>
__device__ __forceinline__ uint32_t shift_pow2_c(uint32_t r) {
  constexpr uint32_t base = kLdsShift + J * 4096u;
  static_assert(base + 4096u <= 65536u, "ds_read offset field is 16 bits");
  return lds_ld(base + ((r & 0xffu) << 2)) ^
         lds_ld(base + 1024u + (((r >> 8) & 0xffu) << 2)) ^
         lds_ld(base + 2048u + (((r >> 16) & 0xffu) << 2)) ^
         lds_ld(base + 3072u + ((r >> 24) << 2));
}

// Un-feed h zero bytes (register that becomes r after h zero bytes).
__device__ __forceinline__ uint32_t unshift_bytes(uint32_t s0, uint32_t r, uint32_t h) {
  for (uint32_t i = 0; i < h; ++i) {
    const uint32_t idx = lds_ld(kLdsInvTop + ((r >> 24) << 2));
    const uint32_t t0 = lds_ld(kLdsMain + ((idx << 8) | ((s0 >> 8) & 0xffu)));
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
// Segments.  A span is cut at 4 KiB boundaries of its 16-byte chunk grid:
// segment = [start, start+n) with n = min(rest, 4096 - (start & 15)), so its
// main region [start&~15, end&~15) holds at most 256 chunks = one chunk per
// chain (64 lanes x K=4).  Every fold therefore uses the compile-time tables
// of fold_wave_c2, and every segment is one load group.  Segments of one
// span are chained: init of segment k+1 = crc of segment k (Extend).
// All fields are wave-uniform.
// ---------------------------------------------------------------------------
constexpr uint32_t kSegChunks = 64u * kChains;  // 256 chunks = 4 KiB
constexpr uint32_t kSlotFirst = 1u, kSlotLast = 2u, kSlotValid = 4u;

// Segment geometry is kept in 32-bit offsets from the segment's 16-byte
// aligned base: hn = h + n where h = start & 15.  The main region is
// chunks [0, hn >> 4) of the base, the ragged tail is hn & 15 bytes after it.
// (Uniform 64-bit compares are VALU compares whose result must be moved to
// SCC; hipcc 7.2 mis-schedules that pattern next to another such compare, so
// the wave loop avoids them.)
struct Slot {
  uint64_t start;  // first byte (absolute address)
  uint32_t n;      // bytes in this segment
  uint32_t init;   // span init (first segment only)
  uint32_t flags;  // kSlotFirst | kSlotLast | kSlotValid
};

// Issues this lane's K = 4 chunk loads of segment s.  Virtual chunk
// v = 64*k + lane (chain k of this lane) holds chunk q = v - pad of the main
// region, so load k of the wave reads 64 consecutive chunks: one contiguous
// KiB per instruction, fully coalesced.  Virtual chunks in front (q < 0)
// read chunk 0 instead (always mapped: it holds the span's first byte); the
// chains they feed are overwritten by the injection or zeroed before the
// fold, so their data never matters.  Slots without a main region (or
// invalid slots) load the KiB at `dummy` so that EVERY slot issues exactly
// 4 vector loads: the ring stays regular.
//
// The issue is branch-free so hipcc's waitcnt pass sees the same 4 loads
// per slot on every path and can leave the ring's other slots in flight.
__device__ __forceinline__ void issue_seg(const Slot& s, uint32_t lane, const void* dummy,
                                          u32x4 (&d)[4]) {
  const uint32_t hn = static_cast<uint32_t>(s.start & 15u) + s.n;
  const bool live = (s.flags & kSlotValid) && hn >= 16u;
  const uint32_t pad = live ? kSegChunks - (hn >> 4) : 0u;
  const uint64_t base = live ? (s.start & ~uint64_t(15)) : reinterpret_cast<uint64_t>(dummy);
  const uint32_t step = live ? 64u : 0u;
  // chunk q_k = max(64k + lane - pad, 0), branch-free
  const uint32_t v0 = lane, v1 = lane + step, v2 = lane + 2u * step, v3 = lane + 3u * step;
  const uint32_t q0 = v0 > pad ? v0 - pad : 0u;
  const uint32_t q1 = v1 > pad ? v1 - pad : 0u;
  const uint32_t q2 = v2 > pad ? v2 - pad : 0u;
  const uint32_t q3 = v3 > pad ? v3 - pad : 0u;
  g_u32x4* g = reinterpret_cast<g_u32x4*>(base);
  d[0] = __builtin_nontemporal_load(g + q0);
  d[1] = __builtin_nontemporal_load(g + q1);
  d[2] = __builtin_nontemporal_load(g + q2);
  d[3] = __builtin_nontemporal_load(g + q3);
}

// The 16 bytes at a 16-byte aligned address `p` (uniform) through the
// scalar cache: the ragged tail of a segment.  The wait is inside the asm,
// so the vector-memory counter -- and the load ring -- is never drained.
__device__ __forceinline__ void tail_chunk(uint64_t p, uint32_t (&t)[4]) {
  typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
  u32x4s v;
  // early-clobber: the destination must not overlap the address registers
  asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(v) : "s"(p) : "memory");
  t[0] = v.x;
  t[1] = v.y;
  t[2] = v.z;
  t[3] = v.w;
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
  __device__ __forceinline__ void get(uint32_t j, uint64_t& start, uint32_t& len,
                                      uint32_t& init) const {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off), j);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off >> 32), j);
    start = reinterpret_cast<uint64_t>(base) + ((static_cast<uint64_t>(hi) << 32) | lo);
    len = __builtin_amdgcn_readlane(c_len, j);
    init = __builtin_amdgcn_readlane(c_init, j);
  }
  // Descriptor of span s, the wave's next span (spans are visited in order,
  // `stride` apart): the cache index advances by one, no division.
  uint32_t cj;
  __device__ __forceinline__ void desc(uint64_t s, uint64_t stride, uint32_t lane,
                                       uint64_t& start, uint32_t& len, uint32_t& init) {
    if (cj >= 64u) {
      fetch(s, stride, lane);
      cj = 0u;
    }
    get(cj, start, len, init);
    ++cj;
  }
};

struct StridedSource {
  const uint8_t* base;
  uint64_t stride_bytes;
  uint32_t length;
  uint32_t init;
  uint64_t count;
  __device__ __forceinline__ void desc(uint64_t s, uint64_t, uint32_t, uint64_t& start,
                                       uint32_t& len, uint32_t& ini) const {
    start = reinterpret_cast<uint64_t>(base) + s * stride_bytes;
    len = length;
    ini = init;
  }
};

// ---------------------------------------------------------------------------
// The wave loop.  out(span, crc, lane) is called once per span with the
// finished crc (uniform).
// ---------------------------------------------------------------------------
// Fold the 64*K one-chunk stripe registers of a wave into the segment
// register (uniform).  r[k] of lane l covers chunk 64k + l, i.e. sits
// (3-k)*1 KiB + (63-l)*16 bytes before the segment end.  In-lane Horner over
// k first (shift by 1 KiB), then the wavefront butterfly over lanes: DPP row
// shifts for partners 1..8 lanes away, v_readlane for 16 and 32.  All table
// indices are compile-time constants (shift by 16*2^J bytes).
template <int K>
__device__ __forceinline__ uint32_t fold_wave_c2(uint32_t (&r)[K], uint32_t lane) {
  static_assert(K == 4, "the fold is written for 4 chains per lane");
  uint32_t v = shift_pow2_c<6>(r[0]) ^ r[1];
  v = shift_pow2_c<6>(v) ^ r[2];
  v = shift_pow2_c<6>(v) ^ r[3];
#if WIPDB_FOLD_SELECT
  // every lane computes every level (no exec-mask regions); the partner
  // value is only kept where the level applies
  uint32_t p = row_shl<1>(v);
  uint32_t t = shift_pow2_c<0>(v) ^ p;
  v = (lane & 1u) == 0u ? t : v;
  p = row_shl<2>(v);
  t = shift_pow2_c<1>(v) ^ p;
  v = (lane & 3u) == 0u ? t : v;
  p = row_shl<4>(v);
  t = shift_pow2_c<2>(v) ^ p;
  v = (lane & 7u) == 0u ? t : v;
  p = row_shl<8>(v);
  t = shift_pow2_c<3>(v) ^ p;
  v = (lane & 15u) == 0u ? t : v;
  const uint32_t g16 = __builtin_amdgcn_readlane(v, 16);
  const uint32_t g48 = __builtin_amdgcn_readlane(v, 48);
  t = shift_pow2_c<4>(v) ^ (lane ? g48 : g16);
  v = (lane & 31u) == 0u ? t : v;
#else
  uint32_t p = row_shl<1>(v);
  if ((lane & 1u) == 0u) v = shift_pow2_c<0>(v) ^ p;
  p = row_shl<2>(v);
  if ((lane & 3u) == 0u) v = shift_pow2_c<1>(v) ^ p;
  p = row_shl<4>(v);
  if ((lane & 7u) == 0u) v = shift_pow2_c<2>(v) ^ p;
  p = row_shl<8>(v);
  if ((lane & 15u) == 0u) v = shift_pow2_c<3>(v) ^ p;
  const uint32_t g16 = __builtin_amdgcn_readlane(v, 16);
  const uint32_t g48 = __builtin_amdgcn_readlane(v, 48);
  if ((lane & 31u) == 0u) v = shift_pow2_c<4>(v) ^ (lane ? g48 : g16);
#endif
  const uint32_t g0 = __builtin_amdgcn_readlane(v, 0);
  const uint32_t g32 = __builtin_amdgcn_readlane(v, 32);
  return uni(shift_pow2_c<5>(g0) ^ g32);
}

// Walks the wave's spans (first_span, first_span + stride, ...) and emits
// their segments in order -- the load side of the pipeline.
template <typename Src>
struct SegCursor {
  uint64_t span, start, stride;
  uint32_t rest, init, first, left;  // left: spans not yet started, incl. this one

  __device__ __forceinline__ void begin(Src& src, uint64_t s, uint64_t str, uint32_t lane) {
    stride = str;
    span = s;
    left = static_cast<uint32_t>((src.count - s + str - 1) / str);  // s < count
    first = 1u;
    src.desc(s, stride, lane, start, rest, init);
  }
  __device__ __forceinline__ Slot next(Src& src, uint32_t lane) {
    // every field defined on every path: an undef field read by issue_seg
    // lets LLVM substitute another slot's value at the ring's merge points
    Slot sl{0, 0, 0, 0};
    if (left == 0u) return sl;
    const uint32_t room = 4096u - static_cast<uint32_t>(start & 15u);
    const bool last = rest <= room;
    const uint32_t n = last ? rest : room;
    sl.start = start;
    sl.n = n;
    sl.init = init;
    sl.flags = kSlotValid | (first ? kSlotFirst : 0u) | (last ? kSlotLast : 0u);
    if (last) {
      span += stride;
      first = 1u;
      --left;
      if (left != 0u) src.desc(span, stride, lane, start, rest, init);
    } else {
      start += n;
      rest -= n;
      first = 0u;
    }
    return sl;
  }
};

// Processes one segment whose chunks are in d (already waited for).
// Returns true when the segment completed its span; the span's crc is then
// in `crc`.  `chain` carries the crc from segment to segment of a span.
template <int K>
__device__ __forceinline__ bool process_seg(const Slot& s, u32x4 (&d)[K], uint32_t s0,
                                            uint32_t lane, uint32_t& chain, uint32_t& crc) {
  const uint32_t init = (s.flags & kSlotFirst) ? s.init : chain;
  const uint32_t h = static_cast<uint32_t>(s.start & 15u);
  const uint32_t hn = h + s.n;  // main region: chunks [0, hn >> 4) of a0
  const uint64_t a0 = s.start & ~uint64_t(15);
  uint32_t reg;  // register after the main region (or ~init if none)
  if (hn >= 16u) {
    const uint32_t pad = kSegChunks - (hn >> 4);
    uint32_t r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = 0u;
    if (hn == 4096u && h == 0u) {
      // fast path: a whole aligned 4 KiB segment; ~init enters at lane 0,
      // chain 0, before any byte
      if (lane == 0) r[0] = ~init;
      feed_chunks<K>(s0, r, d);
    } else {
      // general path: chunk 0 sits at virtual chunk `pad` (lane pad%64,
      // chain pad/64): mask its first h bytes and inject ~init * x^(-8h) there
      const uint32_t inj = (init == 0u) ? lds_ld(kLdsHead0 + (h << 2))
                                        : unshift_bytes(s0, ~init, h);
      const uint32_t m0 = h == 0 ? ~0u : (h >= 4 ? 0u : (~0u << (8 * h)));
      const uint32_t m1 = h <= 4 ? ~0u : (h >= 8 ? 0u : (~0u << (8 * (h - 4))));
      const uint32_t m2 = h <= 8 ? ~0u : (h >= 12 ? 0u : (~0u << (8 * (h - 8))));
      const uint32_t m3 = h <= 12 ? ~0u : (~0u << (8 * (h - 12)));
      const uint32_t l0 = pad & 63u, k0 = pad >> 6;
      u32x4 e[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        e[k] = d[k];
        if (static_cast<uint32_t>(k) == k0 && lane == l0) {
          e[k].x &= m0;
          e[k].y &= m1;
          e[k].z &= m2;
          e[k].w &= m3;
          r[k] = inj;
        }
      }
      feed_chunks<K>(s0, r, e);
      // chains of virtual chunks (in front of the span) carry garbage
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (lane + 64u * k < pad) r[k] = 0u;
    }
    reg = fold_wave_c2<K>(r, lane);
  } else {
    reg = ~init;
  }

  // ragged tail: bytes [o, e) of the chunk at a0 + (hn & ~15)
  const uint32_t e = hn & 15u;
  if (e != 0u) {
    const uint32_t o = hn < 16u ? h : 0u;
    const uint64_t e0 = a0 + (hn & ~15u);
    uint32_t t[4];
#ifdef WIPDB_TAIL_ASM
    tail_chunk(e0, t);  // the chunk holding `end` is mapped (it has span bytes)
#else
    {
      const uint32_t* tp = reinterpret_cast<const uint32_t*>(e0);
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = (4u * j < e) ? tp[j] : 0u;
    }
#endif
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
  const uint32_t c = ~reg;
  if (s.flags & kSlotLast) {
    crc = c;
    return true;
  }
  chain = c;
  return false;
}

// Per-wave output buffer: lane j holds the crc of the wave's (base + j)-th
// span; one vector store per 64 spans (flush(first_ordinal, crc_lane,
// nvalid) is called with all lanes active).
struct OutBuf {
  uint32_t v = 0;      // per lane
  uint32_t fill = 0;   // uniform: lanes filled
  uint64_t base = 0;   // uniform: wave-local ordinal of lane 0
};

// The wave loop: a register ring of WIPDB_RING_SLOTS slots (2 or 3).  While
// segment j is processed, the loads of the next 1 or 2 segments are in
// flight (4-8 KiB per wave, 64-128 KiB per CU, ahead of the compute).  Every
// step issues exactly 4 loads.
template <int K, typename Src, typename Flush>
__device__ __forceinline__ void run_waves(Src& src, uint64_t first_span, uint64_t span_stride,
                                          const void* dummy, Flush flush) {
  static_assert(K == 4, "the ring is written for 4 chunks per lane");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t l4 = (threadIdx.x & 31u) * 4u;
  const uint32_t s0 = l4 | ((l4 | 0x80u) << 8) | (1u << 16);
  if (first_span >= src.count) return;

  SegCursor<Src> cur;
  cur.begin(src, first_span, span_stride, lane);
  uint32_t chain = 0;
  OutBuf ob;

  auto finish = [&](const Slot& sl, u32x4 (&d)[4]) {
    uint32_t crc = 0;
    if (process_seg<K>(sl, d, s0, lane, chain, crc)) {
#if WIPDB_OUTBUF
      ob.v = (lane == ob.fill) ? crc : ob.v;
      if (++ob.fill == 64u) {
        flush(ob.base, ob.v, 64u);
        ob.base += 64u;
        ob.fill = 0u;
      }
#else
      flush(ob.base, crc, 1u);
      ob.base += 1u;
#endif
    }
  };

#if WIPDB_RING_SLOTS == 3
  u32x4 bA[4], bB[4], bC[4];
  Slot sA = cur.next(src, lane);
  issue_seg(sA, lane, dummy, bA);
  Slot sB = cur.next(src, lane);
  issue_seg(sB, lane, dummy, bB);
  for (;;) {
    Slot sC = cur.next(src, lane);
    issue_seg(sC, lane, dummy, bC);
    if (!(sA.flags & kSlotValid)) break;
    finish(sA, bA);

    sA = cur.next(src, lane);
    issue_seg(sA, lane, dummy, bA);
    if (!(sB.flags & kSlotValid)) break;
    finish(sB, bB);

    sB = cur.next(src, lane);
    issue_seg(sB, lane, dummy, bB);
    if (!(sC.flags & kSlotValid)) break;
    finish(sC, bC);
  }
#else
  // 2-slot ping-pong: one segment's loads in flight while one is computed
  u32x4 bA[4], bB[4];
  Slot sA = cur.next(src, lane);
  issue_seg(sA, lane, dummy, bA);
  for (;;) {
    Slot sB = cur.next(src, lane);
    issue_seg(sB, lane, dummy, bB);
    if (!(sA.flags & kSlotValid)) break;
    finish(sA, bA);

    sA = cur.next(src, lane);
    issue_seg(sA, lane, dummy, bA);
    if (!(sB.flags & kSlotValid)) break;
    finish(sB, bB);
  }
#endif
  if (ob.fill) flush(ob.base, ob.v, ob.fill);
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
    *reinterpret_cast<u32x4*>(lds + kLdsMain + e * 4u) = u32x4{v, v, v, v};
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
  DescSource src{base, offsets, lengths, inits, count, 0u, 0, 0, 0, 0, 64u};
  const bool msk = (flags & kFlagMask) != 0;
  const uint64_t first = wave_id();
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWaves;
  run_waves<kChains>(src, first, stride, tab, [&](uint64_t ord, uint32_t crc, uint32_t nvalid) {
    const uint32_t lane = threadIdx.x & 63u;
    if (lane < nvalid) out[first + (ord + lane) * stride] = msk ? mask_crc(crc) : crc;
  });
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride_bytes, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags,
    const DevTables* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  StridedSource src{base, stride_bytes, length, init, count};
  const bool msk = (flags & kFlagMask) != 0;
  const uint64_t first = wave_id();
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWaves;
  run_waves<kChains>(src, first, stride, tab, [&](uint64_t ord, uint32_t crc, uint32_t nvalid) {
    const uint32_t lane = threadIdx.x & 63u;
    if (lane < nvalid) out[first + (ord + lane) * stride] = msk ? mask_crc(crc) : crc;
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
  DescSource src{base, offsets, lengths, nullptr, count, 1u, 0, 0, 0, 0, 64u};
  const uint64_t first = wave_id();
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWaves;
  run_waves<kChains>(src, first, stride, tab, [&](uint64_t ord, uint32_t crc, uint32_t nvalid) {
    const uint32_t lane = threadIdx.x & 63u;
    if (lane < nvalid) {
      const uint64_t s = first + (ord + lane) * stride;
      const uint8_t* t = base + offsets[s] + lengths[s] + 1;
      const uint32_t stored = uint32_t(t[0]) | (uint32_t(t[1]) << 8) | (uint32_t(t[2]) << 16) |
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
