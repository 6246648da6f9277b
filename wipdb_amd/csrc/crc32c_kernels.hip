// crc32c_kernels.hip -- hand-written CDNA4 (gfx950) kernels for batched
// CRC32C of WipDB table blocks.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// crc32c.cc:1225-1227) applied to every block span, as WriteRawBlock
// (kv/src/table/table_builder.cc:194-196) and ReadBlock
// (kv/src/table/format.cc:91-93) do one block at a time.
//
// Design (DESIGN.md "Kernels"):
//   * a wave CRCs kGroups = 2 spans at once: lanes 0-31 one span, lanes
//     32-63 another, each group walking its own stream of spans.  A span is
//     cut into 4 KiB segments of its 16-byte chunk grid.  In a segment,
//     lane l of a group runs kChains = 8 independent CRC chains over chunks
//     l, 32+l, ..., 224+l, so each 16-byte load instruction of the wave
//     reads two contiguous 512 B runs (fully coalesced), and the 8 chains
//     give the LDS-latency-bound scan instruction-level parallelism.
//   * CRC arithmetic is table-driven from LDS (CDNA4 has no carry-less
//     multiply and this is a byte scan, not a contraction: no MFMA):
//     slicing-by-4 tables replicated 32x so lane l always reads bank l&31 --
//     every lookup is bank-conflict free -- and each lookup address is ONE
//     v_perm_b32 (table bits | data byte | lane byte); 160 KiB of LDS.
//   * the 256 stripe registers of a group fold by a GF(2) tree: an in-lane
//     Horner step over the 8 chains (shift by 512 B), then a 5-level
//     butterfly over the group's lanes (DPP row shifts, then v_readlane),
//        reg(v) = shift(reg(v), 16 * 2^t bytes) ^ reg(v + 2^t),
//     where shift by 16*2^j bytes is 4 lookups in a "multiply by
//     x^(8*16*2^j) mod P" table (the carry-less combine of the reference's
//     CombineCRC, crc32c.cc:640-657, done with tables).  Both groups fold in
//     the same instructions, so the fold costs half as much per span.
//   * unaligned starts: the first chunk's leading bytes are zeroed and the
//     register injected there is pre-un-shifted (~init * x^(-8h)) so it
//     equals ~init at the first real byte; the ragged end (< 16 bytes) is
//     fed after the fold.  Segments of one span are chained through init.
//     So any offset/length/init is bit-exact.
//   * latency hiding: persistent grid (1 workgroup of 16 waves per CU), each
//     wave walks its segment pairs through a register ring (the next
//     segments' loads are in flight while one is computed); up to 32 span
//     descriptors per group are fetched per vector load.
//   * load balance: a workgroup's 32 groups take its spans from an LDS work
//     counter in guided batches (WorkShare), so the waves the SIMD
//     arbitration favours take more spans and mixed sizes even out.
//   * the wave loop keeps segment geometry in 32-bit offsets and counts
//     spans down: uniform 64-bit compares become VALU compares moved to SCC,
//     which hipcc 7.2 mis-scheduled in this loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

// Build knobs (the defaults are the measured best; scripts/build_variant.sh
// builds the others for comparison):
//   WIPDB_CPC      16-byte chunks per chain (1 or 2)
//   WIPDB_NT       nontemporal data loads (1) or plain (0)
//   WIPDB_XCHG     C == 2 with coalesced loads + DPP pair exchange
//   WIPDB_SLOTS    register-ring depth (1, 2 or 3; 3 spills at K = 8)
//   WIPDB_ILP      chains interleaved per feed step
//   WIPDB_LOADONLY diagnostic: the loads and ring without the CRC work
//   WIPDB_NOFOLD   diagnostic: the scan without the cross-chain fold
//   WIPDB_NO_STORE diagnostic: the spans kernel's result stores compiled out
//   WIPDB_NO_TABLES, WIPDB_RS_UNROLL, WIPDB_RS_SPLIT: diagnostics for the
//                  load-only skeleton and the read-stream kernel
//                  (scripts/stream_probe.py)
#ifndef WIPDB_NT
#define WIPDB_NT 0
#endif
#ifndef WIPDB_LOADONLY
#define WIPDB_LOADONLY 0
#endif
#ifndef WIPDB_SLOTS
#define WIPDB_SLOTS 2
#endif
#ifndef WIPDB_ILP
#define WIPDB_ILP 8
#endif
#ifndef WIPDB_OPAQUE_LANE
#define WIPDB_OPAQUE_LANE 1
#endif
#ifndef WIPDB_XCHG
#define WIPDB_XCHG 0
#endif
#ifndef WIPDB_CPC
#define WIPDB_CPC 2
#endif
#ifndef WIPDB_NOFOLD
#define WIPDB_NOFOLD 0
#endif
#ifndef WIPDB_LEAN_ISSUE
#define WIPDB_LEAN_ISSUE 1
#endif
// WIPDB_LEAN_PAD: immediate-offset issue for segments with a short pad too
#ifndef WIPDB_LEAN_PAD
#define WIPDB_LEAN_PAD 1
#endif
// WIPDB_SHORT_PAD: a CRC path for segments whose span starts in chain 0
#ifndef WIPDB_SHORT_PAD
#define WIPDB_SHORT_PAD 1
#endif
// WIPDB_PAR_TAIL: both groups' ragged tails fed in the same instructions
#ifndef WIPDB_PAR_TAIL
#define WIPDB_PAR_TAIL 1
#endif
// WIPDB_DYN: the groups of a workgroup share its spans through an LDS work
// counter (guided batches) instead of walking fixed stride-apart lists
#ifndef WIPDB_DYN
#define WIPDB_DYN 1
#endif
// WIPDB_GPOOL: workgroups start with a static share and then take 32-span
// blocks from a grid-wide pool (global counter, LDS ring per workgroup), so
// the XCDs that the fabric serves faster take more of the batch
#ifndef WIPDB_GPOOL
#define WIPDB_GPOOL 1
#endif
#if WIPDB_GPOOL && !WIPDB_DYN
#error "WIPDB_GPOOL feeds the work-sharing cursor (WIPDB_DYN)"
#endif
#ifndef WIPDB_RS_UNROLL
#define WIPDB_RS_UNROLL 1
#endif
#ifndef WIPDB_RS_SPLIT
#define WIPDB_RS_SPLIT 0
#endif
#ifndef WIPDB_RS_SALU
#define WIPDB_RS_SALU 0
#endif
#ifndef WIPDB_NO_TABLES
#define WIPDB_NO_TABLES 0
#endif
// WIPDB_GUIDE: guided batch = what is left / (WIPDB_GUIDE * groups sharing);
// WIPDB_FRESH_EST: read the counter for that instead of the group's last grab
#ifndef WIPDB_GUIDE
#define WIPDB_GUIDE 2u
#endif
#ifndef WIPDB_FRESH_EST
#define WIPDB_FRESH_EST 1
#endif
// WIPDB_TIMELINE diagnostic: the spans kernel stamps the constant-rate wall
// clock per workgroup (entry, tables in LDS) and per wave (done) into
// g_timeline; hcrc_debug_timeline copies it out (scripts/timeline_probe.py)
#ifndef WIPDB_TIMELINE
#define WIPDB_TIMELINE 0
#endif
// WIPDB_TAIL_SELF: slots without a ragged tail load their own first chunk
// as the tail chunk instead of a device-wide dummy line
#ifndef WIPDB_TAIL_SELF
#define WIPDB_TAIL_SELF 0
#endif
#ifndef WIPDB_NO_STORE
#define WIPDB_NO_STORE 0
#endif



namespace wipdb {
namespace dev {

#if WIPDB_TIMELINE
constexpr int kTimelineWGs = 1024;
constexpr int kTimelineStride = 2 + kWaves;  // entry, tables, done per wave
__device__ uint64_t g_timeline[kTimelineWGs * kTimelineStride];
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(3))) const uint32_t l_u32;

constexpr int G = kGroupLanes;     // lanes per group (32)
constexpr int NL = kChunksPerLane; // 16-byte loads per lane per segment (8)
constexpr int C = WIPDB_CPC;       // consecutive chunks per chain
constexpr int K = NL / C;          // chains per lane
constexpr int S = kGroups;         // groups (spans) per wave (2)
// A ring slot holds the NL chunk loads plus the group's ragged-tail chunk
// (d[NL]), loaded with the slot so the tail never waits on memory.
constexpr int NLT = NL + 1;
constexpr uint32_t kLogC = C == 1 ? 0 : (C == 2 ? 1 : 2);
static_assert(G * NL == 256 && S * G == 64 && K * C == NL, "a group segment is 256 chunks");
static_assert(C == 1 || C == 2 || C == 4, "chunks per chain");
// WIPDB_XCHG (C == 2): loads stay fully coalesced (load i of lane gl reads
// chunk G*i + gl) and a DPP exchange between lane pairs gives each lane two
// consecutive chunks: even lane 2m of chain k owns chunks 64k + 2m, +1, odd
// lane 2m+1 owns chunks 64k + 32 + 2m, +1.
constexpr bool X = WIPDB_XCHG != 0;
static_assert(!X || C == 2, "the exchange pairs two chunks per chain");

// Virtual chunk (within the 256-chunk group segment) of chunk j of chain k
// of lane gl.
__device__ __forceinline__ uint32_t vchunk(uint32_t k, uint32_t gl, uint32_t j) {
  if (X) return 64u * k + 32u * (gl & 1u) + 2u * (gl >> 1) + j;
  return C * (gl + G * k) + j;
}

// ---------------------------------------------------------------------------
// LDS helpers (dynamic LDS starts at address 0: no static __shared__ here)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_ld(uint32_t addr) {
  return *reinterpret_cast<l_u32*>(static_cast<uintptr_t>(addr));
}

// s0 = lane constant: byte0 = (lane&31)*4, byte1 = (lane&31)*4 | 0x80,
// byte2 = 0x00, byte3 = 0x01.  Table t's entry for data byte p of x is at
// kLdsMain + perm(s0, x, sel(t, p)):
//   [s0.b(t&1), x.b(p), s0.b(2 + (t>>1)), 0].
__host__ __device__ constexpr uint32_t sel_tab(uint32_t t, uint32_t p) {
  return 0x0c000000u | ((6u + (t >> 1)) << 16) | (p << 8) | (4u + (t & 1u));
}

template <uint32_t T, uint32_t P>
__device__ __forceinline__ uint32_t look(uint32_t s0, uint32_t x) {
  return lds_ld(kLdsMain + __builtin_amdgcn_perm(s0, x, sel_tab(T, P)));
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One slicing-by-4 word step in "x form": x = register ^ word; returns the
// register after the word's 4 bytes XOR the next word (0 at a chain end):
// 4 v_perm_b32 + 4 ds_read_b32 + 2 v_bitop3_b32.
__device__ __forceinline__ uint32_t step4(uint32_t s0, uint32_t x, uint32_t w_next) {
  return xor3(xor3(look<3, 0>(s0, x), look<2, 1>(s0, x), look<1, 2>(s0, x)), look<0, 3>(s0, x),
              w_next);
}

__device__ __forceinline__ uint32_t feed_word(uint32_t s0, uint32_t r, uint32_t w) {
  return step4(s0, r ^ w, 0u);
}

// Feed the SUB-th chunk of every chain into it (chains interleaved by word,
// so their lookups are in flight together).  Chain k's chunks are
// d[k*C .. k*C + C).
// WIPDB_ILP chains at a time (fewer: fewer registers hold lookup results).
template <int SUB, int N>
__device__ __forceinline__ void feed_chunks(uint32_t s0, uint32_t (&r)[K], const u32x4 (&d)[N]) {
  static_assert(N >= NL, "a slot holds NL chunks");
  constexpr int I = WIPDB_ILP < K ? WIPDB_ILP : K;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += I) {
    uint32_t x[I];
#pragma unroll
    for (int i = 0; i < I; ++i) x[i] = r[k0 + i] ^ d[(k0 + i) * C + SUB].x;
#pragma unroll
    for (int i = 0; i < I; ++i) x[i] = step4(s0, x[i], d[(k0 + i) * C + SUB].y);
#pragma unroll
    for (int i = 0; i < I; ++i) x[i] = step4(s0, x[i], d[(k0 + i) * C + SUB].z);
#pragma unroll
    for (int i = 0; i < I; ++i) x[i] = step4(s0, x[i], d[(k0 + i) * C + SUB].w);
#pragma unroll
    for (int i = 0; i < I; ++i) r[k0 + i] = step4(s0, x[i], 0u);
  }
}

// Feed one byte (Sarwate step with this lane's T0 replica).
__device__ __forceinline__ uint32_t feed_byte(uint32_t s0, uint32_t r, uint32_t b) {
  const uint32_t x = (r ^ b) & 0xffu;
  return lds_ld(kLdsMain + ((x << 8) | (s0 & 0xffu))) ^ (r >> 8);
}

// DPP row shift-left: lane l receives lane l+n of its 16-lane row (0 past
// the row end).  Used for butterfly levels whose partners share a row.
template <int N>
__device__ __forceinline__ uint32_t row_shl(uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x100 | N, 0xF, 0xF, true));
}

template <int N>
__device__ __forceinline__ uint32_t row_shr(uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x110 | N, 0xF, 0xF, true));
}

// WIPDB_XCHG: loads 2k, 2k+1 hold chunks 64k + gl and 64k + 32 + gl; after
// the exchange lane 2m holds 64k + 2m, +1 and lane 2m+1 holds 64k + 32 + 2m,
// +1 (as d[2k], d[2k+1]).
// The select is done with a lane bit mask, not a conditional: a DPP read
// must execute with its source lanes active, and hipcc sinks a DPP operand
// of a per-lane ?: into an exec-masked branch (whose inactive source lanes
// then read as 0).
template <int NLx>
__device__ __forceinline__ void exchange_pairs(u32x4 (&d)[NLx], uint32_t gl) {
  const uint32_t m = 0u - (gl & 1u);  // all ones on odd lanes
#pragma unroll
  for (int k = 0; k < NLx / 2; ++k) {
    const u32x4 a = d[2 * k], b = d[2 * k + 1];
    u32x4 f, t;
    f.x = a.x ^ ((a.x ^ row_shr<1>(b.x)) & m);
    f.y = a.y ^ ((a.y ^ row_shr<1>(b.y)) & m);
    f.z = a.z ^ ((a.z ^ row_shr<1>(b.z)) & m);
    f.w = a.w ^ ((a.w ^ row_shr<1>(b.w)) & m);
    t.x = b.x ^ ((b.x ^ row_shl<1>(a.x)) & ~m);
    t.y = b.y ^ ((b.y ^ row_shl<1>(a.y)) & ~m);
    t.z = b.z ^ ((b.z ^ row_shl<1>(a.z)) & ~m);
    t.w = b.w ^ ((b.w ^ row_shl<1>(a.w)) & ~m);
    d[2 * k] = f;
    d[2 * k + 1] = t;
  }
}

// r * x^(8 * 16 * 2^J) mod P, XOR p: 4 lookups in shift table J.  The table
// base is a compile-time constant that lands in the ds_read offset field, so
// each address is one v_lshlrev_b32_sdwa (byte select).
template <uint32_t J>
__device__ __forceinline__ uint32_t shift_xor(uint32_t r, uint32_t p) {
  static_assert(J >= kLogC && J - kLogC < kLdsShiftTables, "shift table not kept in LDS");
  constexpr uint32_t base = kLdsShift + (J - kLogC) * 4096u;
  static_assert(base + 4096u <= 65536u, "ds_read offset field is 16 bits");
  return xor3(xor3(lds_ld(base + ((r & 0xffu) << 2)), lds_ld(base + 1024u + (((r >> 8) & 0xffu) << 2)),
                   lds_ld(base + 2048u + (((r >> 16) & 0xffu) << 2))),
              lds_ld(base + 3072u + ((r >> 24) << 2)), p);
}

// Un-feed h zero bytes (the register that becomes r after h zero bytes).
__device__ __forceinline__ uint32_t unshift_bytes(uint32_t s0, uint32_t r, uint32_t h) {
  for (uint32_t i = 0; i < h; ++i) {
    const uint32_t idx = lds_ld(kLdsInvTop + ((r >> 24) << 2));
    const uint32_t t0 = lds_ld(kLdsMain + ((idx << 8) | (s0 & 0xffu)));
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
// segment = [start, start+n) with n = rest if rest <= 4111 - (start & 15),
// else 4096 - (start & 15), so its main region holds at most 256 chunks and
// its ragged tail fewer than 16 bytes.
// Geometry is kept in 32-bit offsets from the 16-byte aligned base:
// hn = (start & 15) + n; the main region is chunks [0, hn >> 4), the ragged
// tail hn & 15 bytes after it.  All fields are uniform.
// ---------------------------------------------------------------------------
constexpr uint32_t kSegChunks = 256;
constexpr uint32_t kSlotFirst = 1u, kSlotLast = 2u, kSlotValid = 4u, kSlotPartial = 8u;

// Kept small: the ring holds several slots per group in SGPRs.
struct Slot {
  uint64_t start;  // first byte (absolute address)
  uint32_t init;   // span init (first segment only)
  uint32_t meta;   // bytes in this segment | flags << 16
  uint32_t ord;    // the group's span ordinal (output index = first + ord * stride)
  __device__ __forceinline__ uint32_t n() const { return meta & 0xffffu; }
  __device__ __forceinline__ uint32_t flags() const { return meta >> 16; }
};

// ---------------------------------------------------------------------------
// Span sources: where span descriptors come from.  Group g of wave w owns
// spans first_g, first_g + stride, ...  Descriptors are fetched G at a time
// by one vector load (lane g*G + j holds group g's j-th next span) and
// broadcast with v_readlane, so they never sit on the LDS counter.
// ---------------------------------------------------------------------------
struct DescSource {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  const uint32_t* inits;
  uint64_t count;
  uint32_t extra;  // bytes added to every length (verify: +1 type byte)
  bool trailer;    // verify: the init column carries the block's stored
                   // (masked) crc, read at fetch time; the CRC starts at 0
  uint64_t c_off;  // per lane
  uint32_t c_len, c_init;
  uint32_t c_span;  // WIPDB_GPOOL: the span index of the lane's entry
  uint32_t cj[S];  // next cache index per group (uniform)

  __device__ __forceinline__ void reset() {
    c_off = 0;
    c_len = 0;
    c_init = 0;
    c_span = 0;
#pragma unroll
    for (int g = 0; g < S; ++g) cj[g] = G;
  }
  __device__ __forceinline__ void fetch(int g, uint64_t first, uint64_t stride, uint32_t lane) {
    const uint64_t s = first + (lane & (G - 1)) * stride;
    if ((lane / G) == static_cast<uint32_t>(g) && s < count) {
      c_off = __builtin_nontemporal_load(offsets + s);
      c_len = __builtin_nontemporal_load(lengths + s) + extra;
      if (trailer) {
        // ReadBlock's trailer: LE32 at n + 1 (format.cc:91-93), any alignment
        const uint8_t* t = base + c_off + (c_len - extra) + 1;
        c_init = uint32_t(t[0]) | (uint32_t(t[1]) << 8) | (uint32_t(t[2]) << 16) |
                 (uint32_t(t[3]) << 24);
      } else {
        c_init = inits ? __builtin_nontemporal_load(inits + s) : 0u;
      }
    }
  }
  // Work sharing (WIPDB_DYN): group g grabbed units [ub, ub + nb) of its
  // workgroup's share; lane g*G + j loads the descriptor of unit ub + j.
  template <typename WS>
  __device__ __forceinline__ void fetch_units(int g, uint32_t ub, uint32_t nb, const WS& ws,
                                              uint32_t lane) {
    const uint32_t j = lane & (G - 1);
    if ((lane / G) == static_cast<uint32_t>(g) && j < nb) {
      const uint64_t sp = ws.span_of_lane(ub + j);
      c_span = static_cast<uint32_t>(sp);
      c_off = __builtin_nontemporal_load(offsets + sp);
      c_len = __builtin_nontemporal_load(lengths + sp) + extra;
      if (trailer) {
        const uint8_t* t = base + c_off + (c_len - extra) + 1;
        c_init = uint32_t(t[0]) | (uint32_t(t[1]) << 8) | (uint32_t(t[2]) << 16) |
                 (uint32_t(t[3]) << 24);
      } else {
        c_init = inits ? __builtin_nontemporal_load(inits + sp) : 0u;
      }
    }
  }
  // The span index of entry j of group g's batch (WIPDB_GPOOL).
  __device__ __forceinline__ uint32_t span_at(int g, uint32_t j) const {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(c_span, g * G + j));
  }
  // Entry j of group g's batch (uniform j).
  __device__ __forceinline__ void at(int g, uint32_t j, uint64_t, uint64_t& start, uint32_t& len,
                                     uint32_t& init) const {
    const uint32_t l = g * G + j;
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off >> 32), l);
    start = reinterpret_cast<uint64_t>(base) + ((static_cast<uint64_t>(hi) << 32) | lo);
    len = __builtin_amdgcn_readlane(c_len, l);
    init = __builtin_amdgcn_readlane(c_init, l);
  }
  // Descriptor of span s, group g's next span (spans are visited in order,
  // `stride` apart): the cache index advances by one, no division.
  __device__ __forceinline__ void desc(int g, uint64_t s, uint64_t stride, uint32_t lane,
                                       uint64_t& start, uint32_t& len, uint32_t& init) {
    if (cj[g] >= static_cast<uint32_t>(G)) {
      fetch(g, s, stride, lane);
      cj[g] = 0u;
    }
    const uint32_t j = g * G + cj[g];
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off), j);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(c_off >> 32), j);
    start = reinterpret_cast<uint64_t>(base) + ((static_cast<uint64_t>(hi) << 32) | lo);
    len = __builtin_amdgcn_readlane(c_len, j);
    init = __builtin_amdgcn_readlane(c_init, j);
    ++cj[g];
  }
};

struct StridedSource {
  const uint8_t* base;
  uint64_t stride_bytes;
  uint32_t length;
  uint32_t init;
  uint64_t count;
  static constexpr bool trailer = false;
  uint32_t c_span;  // WIPDB_GPOOL: per lane, the span index of the batch entry
  __device__ __forceinline__ void reset() { c_span = 0; }
  __device__ __forceinline__ uint32_t span_at(int g, uint32_t j) const {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(c_span, g * G + j));
  }
  __device__ __forceinline__ void desc(int, uint64_t s, uint64_t, uint32_t, uint64_t& start,
                                       uint32_t& len, uint32_t& ini) const {
    start = reinterpret_cast<uint64_t>(base) + s * stride_bytes;
    len = length;
    ini = init;
  }
  template <typename WS>
  __device__ __forceinline__ void fetch_units(int g, uint32_t ub, uint32_t nb, const WS& ws,
                                              uint32_t lane) {
#if WIPDB_GPOOL
    const uint32_t j = lane & (G - 1);
    if ((lane / G) == static_cast<uint32_t>(g) && j < nb)
      c_span = static_cast<uint32_t>(ws.span_of_lane(ub + j));
#else
    (void)g, (void)ub, (void)nb, (void)ws, (void)lane;
#endif
  }
  __device__ __forceinline__ void at(int, uint32_t, uint64_t s, uint64_t& start, uint32_t& len,
                                     uint32_t& ini) const {
    start = reinterpret_cast<uint64_t>(base) + s * stride_bytes;
    len = length;
    ini = init;
  }
};

// A workgroup's share of the batch: unit u is span (u / 32) * stride + wg0 +
// u % 32 -- the spans the static schedule gives the workgroup's 32 groups,
// round by round -- and its groups take units from an LDS counter in
// guided batches (half the per-group share of what is left, at most a
// descriptor load's 32, at least 1), so a group that the SIMD's arbitration
// serves faster simply takes more spans and all finish together.
#if WIPDB_GPOOL
// Grid-wide work pool (WIPDB_GPOOL).  The batch is cut into blocks of 32
// consecutive spans.  Workgroup w starts with its static share, blocks
// r * nwg + w for r < kStaticRounds (enough for each of its 32 groups'
// first batch), and then takes blocks from the pool -- one global counter,
// blocks kStaticRounds * nwg on -- into a ring in its LDS whenever fewer than
// kAhead fetched units are left; unit u of the workgroup is span
// ring[u / 32] * 32 + u % 32.  Its groups take units from the LDS counter in
// guided batches as before.  One global atomic per pool grab -- ~50 per
// microsecond for the whole chip at most, under the ~88 that one address
// sustains (scripts/atomic_probe.hip) -- lets every CU finish within about
// a span of the others, where static shares left the odd XCDs ~5 % behind.
// A unit's ring entry is read once, when its batch is fetched (the span
// index then rides in the descriptor cache, c_span): between a batch's
// first unit and the newest fetched unit lie at most the batch, what the
// other groups grab meanwhile (one batch each), kAhead and one pool grab --
// fewer than the kRing blocks after which an entry is recycled.  (Spans are
// 32-bit indices: count < 2^32 per launch.)
constexpr uint32_t kRing = 64;          // block indices in the LDS ring
constexpr uint32_t kStaticRounds = 32;  // a workgroup's static blocks
constexpr uint32_t kAhead = 64;         // fetched units kept ahead of the counter
constexpr uint32_t kMaxGrab = 4;        // blocks per pool grab
constexpr uint32_t kPoolArrive = 32;    // u32 index of the arrival count (own 128-B line)
static_assert(kRing * 32u > kSpansPerWG * G + G + kAhead + kMaxGrab * 32u,
              "a batch's ring entries outlive its fetch");
typedef __attribute__((address_space(3))) uint32_t l_u32w;
// LDS words: the unit counter, units fetched, refill lock, pool exhausted,
// this workgroup's view of the pool position; then the ring
__device__ __forceinline__ l_u32w* lw(uint32_t i) {
  return reinterpret_cast<l_u32w*>(static_cast<uintptr_t>(kLdsWork + 4u * i));
}
enum : uint32_t { kWCtr = 0, kWAvail = 1, kWLock = 2, kWDone = 3, kWPos = 4, kWRing = 8 };
static_assert(kLdsWork + 4u * (kWRing + kRing) <= kLdsMain, "pool state fits below the tables");

// An LDS word, read by every lane, as a scalar.
__device__ __forceinline__ uint32_t lds_word(uint32_t w) {
  return uni(static_cast<uint32_t>(
      __builtin_amdgcn_readfirstlane(static_cast<int>(__atomic_load_n(lw(w), __ATOMIC_ACQUIRE)))));
}
#endif

// A workgroup's share of the batch: unit u is span (u / 32) * stride + wg0 +
// u % 32 (or, with WIPDB_GPOOL, span ring[u / 32] * 32 + u % 32), and its
// groups take units from an LDS counter in guided batches.
struct WorkShare {
  uint64_t stride;  // spans per round of the grid (groups in the grid)
  uint64_t wg0;     // this workgroup's first span
  uint32_t units;   // units of this workgroup (WIPDB_GPOOL: unused)
#if WIPDB_GPOOL
  uint64_t count;
  uint32_t nblk, nwg, first_pool;
  uint32_t* pool;  // [0] the pool counter, [kPoolArrive] arrivals (release_pool)
#endif
  __device__ __forceinline__ uint64_t span_of(uint32_t u) const {
#if WIPDB_GPOOL
    return static_cast<uint64_t>(lds_word(kWRing + ((u >> 5) & (kRing - 1u)))) * 32u + (u & 31u);
#else
    return static_cast<uint64_t>(u >> 5) * stride + wg0 + (u & 31u);
#endif
  }
  // The same for a per-lane unit (descriptor fetch).
  __device__ __forceinline__ uint64_t span_of_lane(uint32_t u) const {
#if WIPDB_GPOOL
    return static_cast<uint64_t>(
               __atomic_load_n(lw(kWRing + ((u >> 5) & (kRing - 1u))), __ATOMIC_RELAXED)) *
               32u + (u & 31u);
#else
    return span_of(u);
#endif
  }
  __device__ __forceinline__ void init(uint64_t n, uint32_t* p) {
    stride = grid_groups();
    wg0 = static_cast<uint64_t>(blockIdx.x) * kSpansPerWG;
    units = 0u;
#if WIPDB_GPOOL
    // thread 0 sets up the LDS state; the caller's barrier publishes it.
    // The last block may be short: `avail` then stops at the batch's end.
    count = n;
    pool = p;
    nwg = gridDim.x;
    nblk = static_cast<uint32_t>((n + 31u) >> 5);
    first_pool = kStaticRounds * nwg;
    if (threadIdx.x == 0u) {
      uint32_t k = 0, av = 0;
      for (; k < kStaticRounds && k * nwg + blockIdx.x < nblk; ++k) {
        const uint32_t b = k * nwg + blockIdx.x;
        *lw(kWRing + k) = b;
        av = 32u * k + (b + 1u == nblk ? static_cast<uint32_t>(n - 32ull * b) : 32u);
      }
      *lw(kWCtr) = 0u;
      *lw(kWAvail) = av;
      *lw(kWLock) = 0u;
      *lw(kWDone) = first_pool < nblk ? 0u : 1u;
      *lw(kWPos) = 0u;
    }
#else
    (void)p;
    if (n > wg0) {
      const uint64_t r = n - wg0;
      const uint64_t full = r / stride;
      const uint64_t part = r - full * stride;
      units = static_cast<uint32_t>(full * kSpansPerWG + (part < kSpansPerWG ? part : kSpansPerWG));
    }
#endif
  }
#if WIPDB_GPOOL
  __device__ __forceinline__ uint32_t pool_left(uint32_t pos) const {
    return nblk > first_pool + pos ? nblk - first_pool - pos : 0u;
  }
  // Take blocks from the pool into the ring, unless another group is doing
  // so.  Uniform control flow: lane `ld` alone does the atomics and stores.
  __device__ __forceinline__ void refill(uint32_t lane, uint32_t ld) const {
    uint32_t busy = 1u;
    if (lane == ld) {
      uint32_t expect = 0u;
      busy = __atomic_compare_exchange_n(lw(kWLock), &expect, 1u, false, __ATOMIC_ACQUIRE,
                                         __ATOMIC_RELAXED)
                 ? 0u
                 : 1u;
    }
    if (uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(busy, ld))) != 0u) return;
    if (lds_word(kWDone) == 0u) {
      uint32_t nb = pool_left(lds_word(kWPos)) / (WIPDB_GUIDE * nwg);
      nb = nb < 1u ? 1u : (nb > kMaxGrab ? kMaxGrab : nb);
      uint32_t p = 0u;
      if (lane == ld)
        p = __hip_atomic_fetch_add(pool, nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      p = uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(p, ld)));
      const uint32_t b0 = first_pool + p;
      const uint32_t nv = b0 < nblk ? (nblk - b0 < nb ? nblk - b0 : nb) : 0u;
      const uint32_t av = lds_word(kWAvail);  // a multiple of 32 while blocks remain
      const uint32_t i = lane - ld;
      if (i < nv) *lw(kWRing + (((av >> 5) + i) & (kRing - 1u))) = b0 + i;
      // the batch's last block may be short
      const uint32_t add = nv == 0u ? 0u
                           : (b0 + nv == nblk ? 32u * (nv - 1u) + static_cast<uint32_t>(count - 32ull * (nblk - 1u))
                                              : 32u * nv);
      if (lane == ld) {
        __atomic_store_n(lw(kWPos), p + nb, __ATOMIC_RELAXED);
        __atomic_store_n(lw(kWAvail), av + add, __ATOMIC_RELEASE);
        if (nv < nb || b0 + nv == nblk) __atomic_store_n(lw(kWDone), 1u, __ATOMIC_RELEASE);
      }
    }
    if (lane == ld) __atomic_store_n(lw(kWLock), 0u, __ATOMIC_RELEASE);
  }
#endif
  static __device__ __forceinline__ uint64_t grid_groups() {
    return static_cast<uint64_t>(gridDim.x) * kSpansPerWG;
  }
};

// Walks one group's spans (first, first + stride, ...) and emits their
// segments in order -- the load side of the pipeline.
template <typename Src>
struct SegCursor {
  uint64_t start;
  uint32_t rest, init, first, left;  // left: spans not yet finished, incl. this one
  uint32_t ord;                      // ordinal of the current span
  uint32_t split;                    // kFlagSkipSmall | kFlagSplitRem
  bool skip;                         // kFlagSkipSmall: small spans are the small kernel's

  // With `skip`, step over spans of at most kSmallMax bytes (their ordinals
  // still count, so output slots stay put).
  __device__ __forceinline__ void skip_small(Src& src, int g, uint64_t s0, uint64_t stride,
                                            uint32_t lane) {
    while (skip && left != 0u && rest <= kSmallMax) {
      ++ord;
      --left;
      if (left != 0u) src.desc(g, s0 + static_cast<uint64_t>(ord) * stride, stride, lane, start,
                               rest, init);
    }
  }

  __device__ __forceinline__ void begin(Src& src, int g, uint64_t s, uint64_t stride,
                                       uint32_t lane, uint32_t split_flags) {
    // s < stride always, so this is ceil((count - s) / stride) or 0 -- no compare
    left = static_cast<uint32_t>((src.count + stride - 1 - s) / stride);
    first = 1u;
    ord = 0u;
    start = 0;
    rest = 0;
    init = 0;
    split = split_flags;
    skip = (split_flags & kFlagSkipSmall) != 0u;
    if (left != 0u) src.desc(g, s, stride, lane, start, rest, init);
    skip_small(src, g, s, stride, lane);
  }
  __device__ __forceinline__ Slot next(Src& src, int g, uint64_t s0, uint64_t stride,
                                       uint32_t lane) {
    // every field defined on every path (undef fields let LLVM substitute
    // another slot's value at the ring's merge points)
    Slot sl{0, 0, 0, 0};
    if (left == 0u) return sl;
    // a segment is at most 256 chunks of the 16-byte grid; when the rest of
    // the span fits that plus a ragged tail (< 16 bytes, fed after the
    // fold), it is the last segment -- so an unaligned 4 KiB block is one
    // segment, not 4096 - h bytes and an h-byte second one
    const uint32_t room = 4096u - static_cast<uint32_t>(start & 15u);
    const bool cut = first && (split & kFlagSplitRem) && SplitRemainder(start, rest) != 0u;
    const bool last = rest <= room + 15u || cut;
    const uint32_t n = rest <= room + 15u ? rest : room;
    sl.start = start;
    sl.init = init;
    sl.meta = n | ((kSlotValid | (first ? kSlotFirst : 0u) | (last ? kSlotLast : 0u) |
                    (cut ? kSlotPartial : 0u)) << 16);
    sl.ord = ord;
    if (last) {
      ++ord;
      first = 1u;
      --left;
      if (left != 0u) src.desc(g, s0 + static_cast<uint64_t>(ord) * stride, stride, lane, start,
                               rest, init);
      skip_small(src, g, s0, stride, lane);
    } else {
      start += n;
      rest -= n;
      first = 0u;
    }
    return sl;
  }
};

// The work-sharing cursor (WIPDB_DYN): like SegCursor, but the group's
// next span is the next unit of its grabbed batch, and an exhausted batch is
// replaced from the workgroup's LDS counter.  Slot.ord carries the unit.
template <typename Src>
struct DynCursor {
  uint64_t start;
  uint32_t rest, init, first, left;  // left: 1 while the group has a current span
  uint32_t u, ub, ue;                // current unit; grabbed batch [ub, ue)
  uint32_t split;                    // kFlagSkipSmall | kFlagSplitRem
#if WIPDB_GPOOL
  uint32_t span;                     // the current span (the ring entry may be recycled)
#endif
  bool skip;

  // Makes unit u (the next one) current, grabbing a batch when needed.
  __device__ __forceinline__ void load(Src& src, int g, const WorkShare& ws, uint32_t lane) {
    if (u >= ue) {
#if WIPDB_GPOOL
      const uint32_t ld = static_cast<uint32_t>(g * G);
      const uint32_t c = lds_word(kWCtr);
      const uint32_t av0 = lds_word(kWAvail);
      const uint32_t est =
          (av0 > c ? av0 - c : 0u) + ws.pool_left(lds_word(kWPos)) * 32u / ws.nwg;
#elif WIPDB_FRESH_EST
      // guided: a fraction of this group's share of what is left, read
      // from the counter just before the grab (other groups may take some
      // in between: the batch only comes out larger than the rule by what
      // they took)
      const uint32_t at = uni(static_cast<uint32_t>(
          __builtin_amdgcn_readfirstlane(static_cast<int>(lds_ld(kLdsWork)))));
      const uint32_t est = ws.units > at ? ws.units - at : 0u;
#else
      const uint32_t est = ws.units > ue ? ws.units - ue : 0u;
#endif
      uint32_t want = est / (WIPDB_GUIDE * kSpansPerWG);
      want = want < 1u ? 1u : (want > static_cast<uint32_t>(G) ? static_cast<uint32_t>(G) : want);
      uint32_t old = 0u;
      if (lane == static_cast<uint32_t>(g * G))
        old = __atomic_fetch_add(
            reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
                static_cast<uintptr_t>(kLdsWork)),
            want, __ATOMIC_RELAXED);
      old = uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(old, g * G)));
#if WIPDB_GPOOL
      // wait until the batch is fetched or the pool is empty, refilling
      // ahead (bounded: a refill is one global atomic away)
      const uint32_t end = old + want;
      uint32_t av = 0u;
      for (uint32_t it = 0; it < (1u << 22); ++it) {
        const uint32_t dn = lds_word(kWDone);
        av = lds_word(kWAvail);
        if (dn == 0u && av < end + kAhead) ws.refill(lane, ld);
        if (av >= end) break;
        if (dn != 0u) {
          av = lds_word(kWAvail);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const uint32_t lim = av < end ? av : end;
#else
      const uint32_t lim = old + want < ws.units ? old + want : ws.units;
#endif
      if (old >= lim) {
        left = 0u;
        ue = lim;
        return;
      }
      ub = old;
      ue = lim;
      u = ub;
      src.fetch_units(g, ub, ue - ub, ws, lane);
    }
    left = 1u;
#if WIPDB_GPOOL
    span = src.span_at(g, u - ub);
    src.at(g, u - ub, span, start, rest, init);
#else
    src.at(g, u - ub, ws.span_of(u), start, rest, init);
#endif
  }
  __device__ __forceinline__ void skip_small(Src& src, int g, const WorkShare& ws, uint32_t lane) {
    while (skip && left != 0u && rest <= kSmallMax) {
      ++u;
      load(src, g, ws, lane);
    }
  }
  __device__ __forceinline__ void begin(Src& src, int g, const WorkShare& ws, uint32_t lane,
                                       uint32_t split_flags) {
    first = 1u;
    start = 0;
    rest = 0;
    init = 0;
    u = ub = ue = 0u;
    left = 0u;
    split = split_flags;
    skip = (split_flags & kFlagSkipSmall) != 0u;
    load(src, g, ws, lane);
    skip_small(src, g, ws, lane);
  }
  __device__ __forceinline__ Slot next(Src& src, int g, const WorkShare& ws, uint32_t lane) {
    Slot sl{0, 0, 0, 0};
    if (left == 0u) return sl;
    const uint32_t room = 4096u - static_cast<uint32_t>(start & 15u);
    // HCRC_SPLIT_SMALL: a span whose rest after this first segment fits the
    // small kernel stops here (partial CRC, unmasked)
    const bool cut = first && (split & kFlagSplitRem) && SplitRemainder(start, rest) != 0u;
    const bool last = rest <= room + 15u || cut;
    const uint32_t n = rest <= room + 15u ? rest : room;
    sl.start = start;
    sl.init = init;
    sl.meta = n | ((kSlotValid | (first ? kSlotFirst : 0u) | (last ? kSlotLast : 0u) |
                    (cut ? kSlotPartial : 0u)) << 16);
#if WIPDB_GPOOL
    sl.ord = span;
#else
    sl.ord = u;
#endif
    if (last) {
      first = 1u;
      ++u;
      load(src, g, ws, lane);
      skip_small(src, g, ws, lane);
    } else {
      start += n;
      rest -= n;
      first = 0u;
    }
    return sl;
  }
};

// Per-lane select between the two groups' uniform values.
template <typename T>
__device__ __forceinline__ T gsel(bool hi, T v0, T v1) {
  return hi ? v1 : v0;
}

// Issues this lane's NL chunk loads of the segment pair.  Load i = k*C + j
// is chunk j of chain k: virtual chunk v = C*(G*k + gl) + j, which holds
// chunk q = v - pad of the group's main region; so load i of the wave reads
// the chunks C*G*k + j + {0, C, 2C, ...} of each group (C = 1: G
// consecutive chunks; C = 2: every other one, the next load the rest).
// Virtual chunks in front (q < 0) read chunk 0 instead (always mapped: it
// holds the span's first byte); the chains they feed are overwritten by the
// injection or zeroed before the fold.  A group without a main region (or
// an invalid one) loads the 4 KiB at `dummy`, so EVERY slot issues exactly
// NL vector loads and the ring stays regular.
__device__ __forceinline__ void issue_seg(const Slot (&s)[S], uint32_t lane, const void* dummy,
                                          u32x4 (&d)[NLT]) {
  // the ragged-tail chunk of each group's segment (the dummy if none): all
  // lanes of a group read the same 16 bytes
  uint64_t tail_g[S];
#pragma unroll
  for (int g = 0; g < S; ++g) {
    const uint32_t hn = static_cast<uint32_t>(s[g].start & 15u) + s[g].n();
#if WIPDB_TAIL_SELF
    // no ragged tail: read the segment's own first chunk (a line the slot
    // loads anyway) instead of one device-wide dummy line
    tail_g[g] = (s[g].flags() & kSlotValid)
                    ? (s[g].start & ~uint64_t(15)) + ((hn & 15u) ? (hn & ~15u) : 0u)
                    : reinterpret_cast<uint64_t>(dummy);
#else
    tail_g[g] = ((s[g].flags() & kSlotValid) && (hn & 15u))
                    ? (s[g].start & ~uint64_t(15)) + (hn & ~15u)
                    : reinterpret_cast<uint64_t>(dummy);
#endif
  }
  d[NL] = *reinterpret_cast<g_u32x4*>(gsel(lane >= static_cast<uint32_t>(G), tail_g[0], tail_g[1]));
  uint32_t pad_g[S];
  uint64_t base_g[S];
#pragma unroll
  for (int g = 0; g < S; ++g) {
    const uint32_t hn = static_cast<uint32_t>(s[g].start & 15u) + s[g].n();
    const bool live = (s[g].flags() & kSlotValid) && hn >= 16u;
    pad_g[g] = live ? kSegChunks - (hn >> 4) : 0u;
    base_g[g] = live ? (s[g].start & ~uint64_t(15)) : reinterpret_cast<uint64_t>(dummy);
  }
  // an opaque lane copy: the per-load chunk indices derived from it are
  // recomputed here (one VALU each) rather than hoisted out of the wave loop
  // into registers that the ring needs
  uint32_t ln = lane;
#if WIPDB_OPAQUE_LANE
  asm volatile("" : "+v"(ln));
#endif
  const bool hi = ln >= static_cast<uint32_t>(G);
  const uint32_t gl = ln & (G - 1);
  const uint32_t pad = gsel(hi, pad_g[0], pad_g[1]);
  g_u32x4* b = reinterpret_cast<g_u32x4*>(gsel(hi, base_g[0], base_g[1]));
#if WIPDB_LEAN_ISSUE
  if (!X && (pad_g[0] | pad_g[1]) == 0u) {
    // both groups' segments fill the whole chunk grid (the common case):
    // one lane address, the 8 loads at immediate offsets (C*G*k + j chunks)
    g_u32x4* bl = b + C * gl;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
#if WIPDB_NT
      d[i] = __builtin_nontemporal_load(bl + (C * G * (i / C) + i % C));
#else
      d[i] = bl[C * G * (i / C) + i % C];
#endif
    }
    return;
  }
  if (WIPDB_LEAN_PAD && !X && pad_g[0] < static_cast<uint32_t>(C * G) &&
      pad_g[1] < static_cast<uint32_t>(C * G)) {
    // a short pad (spans of 3 KiB+ -- a 4 KiB block minus its trailer):
    // only chain 0's loads can fall in front of the span, so chains 1.. load
    // at immediate offsets from one shifted lane address
    const int32_t sh = static_cast<int32_t>(C * gl) - static_cast<int32_t>(pad);
    g_u32x4* bl = b + sh;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      if (i < C) {
        const int32_t q = sh + i;
        d[i] = b[q > 0 ? q : 0];
      } else {
        d[i] = bl[C * G * (i / C) + i % C];
      }
    }
    return;
  }
#endif
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t v = X ? gl + G * i : vchunk(i / C, gl, i % C);
    const uint32_t q = v > pad ? v - pad : 0u;
#if WIPDB_NT
    d[i] = __builtin_nontemporal_load(b + q);
#else
    d[i] = b[q];
#endif
  }
}

// Fold the G*K chain registers of each group into the group's segment
// register.  Chain k of lane gl covers chunks C*(G*k + gl) .. +C-1, i.e.
// ends (K-1-k)*G*C*16 + (G-1-gl)*C*16 bytes before the segment end.
// In-lane Horner over k first (shift by G*C*16 bytes), then the butterfly
// over the group's lanes (shift by C*16*2^t): DPP row shifts for partners
// 1..8 lanes away, v_readlane for 16.  Returns the per-lane value; group
// g's result is in lane g*G.
__device__ __forceinline__ uint32_t fold_groups(uint32_t (&r)[K], uint32_t lane) {
  static_assert(G == 32, "the butterfly is written for 32-lane groups");
  constexpr uint32_t L = kLogC;
  uint32_t v = r[0];
#if WIPDB_NOFOLD
  // diagnostic: no GF(2) fold (wrong results)
#pragma unroll
  for (int k = 1; k < K; ++k) v ^= r[k];
  return v;
#endif
#pragma unroll
  for (int k = 1; k < K; ++k) v = shift_xor<5 + L>(v, r[k]);
  // with the exchange, lane bit 0 is chain-position bit 4 and lane bits
  // 1..4 are position bits 0..3: the partner distance of each level follows
  constexpr uint32_t J0 = X ? 4 + L : 0 + L, J1 = X ? 0 + L : 1 + L, J2 = X ? 1 + L : 2 + L;
  constexpr uint32_t J3 = X ? 2 + L : 3 + L, J4 = X ? 3 + L : 4 + L;
  uint32_t p = row_shl<1>(v);
  if ((lane & 1u) == 0u) v = shift_xor<J0>(v, p);
  p = row_shl<2>(v);
  if ((lane & 3u) == 0u) v = shift_xor<J1>(v, p);
  p = row_shl<4>(v);
  if ((lane & 7u) == 0u) v = shift_xor<J2>(v, p);
  p = row_shl<8>(v);
  if ((lane & 15u) == 0u) v = shift_xor<J3>(v, p);
  const uint32_t g16 = __builtin_amdgcn_readlane(v, 16);
  const uint32_t g48 = __builtin_amdgcn_readlane(v, 48);
  if ((lane & 31u) == 0u) v = shift_xor<J4>(v, lane ? g48 : g16);
  return v;
}

// Feeds bytes [o, e) of a 16-byte chunk held as words t0..t3.
__device__ __forceinline__ uint32_t feed_tail_words(uint32_t s0, uint32_t reg, uint32_t t0,
                                                    uint32_t t1, uint32_t t2, uint32_t t3,
                                                    uint32_t o, uint32_t e) {
  uint32_t i = o;
  if (o == 0) {
    if (e >= 4u) reg = feed_word(s0, reg, t0), i = 4u;
    if (e >= 8u) reg = feed_word(s0, reg, t1), i = 8u;
    if (e >= 12u) reg = feed_word(s0, reg, t2), i = 12u;
  }
  for (; i < e; ++i) {
    const uint32_t wd = i < 4 ? t0 : (i < 8 ? t1 : (i < 12 ? t2 : t3));
    reg = feed_byte(s0, reg, (wd >> (8 * (i & 3))) & 0xffu);
  }
  return reg;
}

// The same for the chunk at e0 in memory (only the words that hold bytes
// below e are read).
__device__ __forceinline__ uint32_t feed_tail(uint32_t s0, uint32_t reg, uint64_t e0, uint32_t o,
                                              uint32_t e) {
  const uint32_t* tp = reinterpret_cast<const uint32_t*>(e0);
  const uint32_t t0 = tp[0];
  const uint32_t t1 = e > 4u ? tp[1] : 0u;
  const uint32_t t2 = e > 8u ? tp[2] : 0u;
  const uint32_t t3 = e > 12u ? tp[3] : 0u;
  return feed_tail_words(s0, reg, t0, t1, t2, t3, o, e);
}

// Processes one segment pair whose chunks are in d (already waited for).
// For each group: `chain` carries the crc from segment to segment of a
// span; when the segment completes its span, crc[g] is the span's crc and
// done[g] is set.
__device__ __forceinline__ void process_seg(const Slot (&s)[S], u32x4 (&d)[NLT], uint32_t s0,
                                            uint32_t lane, uint32_t (&chain)[S],
                                            uint32_t (&crc)[S], bool (&done)[S], bool trailer) {
  const bool hi = lane >= static_cast<uint32_t>(G);
  const uint32_t gl = lane & (G - 1);
  uint32_t init[S], h[S], hn[S];
  bool main_g[S], fast = true, any_main = false, short_pad = !X, any_h = false;
#pragma unroll
  for (int g = 0; g < S; ++g) {
    init[g] = (s[g].flags() & kSlotFirst) ? (trailer ? 0u : s[g].init) : chain[g];
    h[g] = static_cast<uint32_t>(s[g].start & 15u);
    hn[g] = h[g] + s[g].n();
    main_g[g] = (s[g].flags() & kSlotValid) && hn[g] >= 16u;
    fast = fast && main_g[g] && h[g] == 0u && hn[g] == 4096u;
    // the span's first chunk falls in chain 0 (pad < C*G chunks)
    short_pad = short_pad && main_g[g] && (hn[g] >> 4) > kSegChunks - C * G;
    any_h = any_h || h[g] != 0u;
    any_main = any_main || main_g[g];
  }
  uint32_t reg[S];
#pragma unroll
  for (int g = 0; g < S; ++g) reg[g] = ~init[g];
#if WIPDB_LOADONLY
  // diagnostic: the same loads and ring, no CRC work (wrong results)
  if (any_main) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) x ^= d[i].x ^ d[i].y ^ d[i].z ^ d[i].w;
    x = __builtin_amdgcn_readlane(x, 0) ^ __builtin_amdgcn_readlane(x, 32);
#pragma unroll
    for (int g = 0; g < S; ++g)
      if (main_g[g]) reg[g] = x;
  }
  if (false) {
#else
  if (any_main) {
#endif
    uint32_t r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = 0u;
    if (X) exchange_pairs(d, gl);
    if (fast) {
      // every group holds a whole aligned 4 KiB segment: ~init enters at
      // the group's lane 0, chain 0, before any byte
      if (gl == 0) r[0] = gsel(hi, ~init[0], ~init[1]);
      feed_chunks<0>(s0, r, d);
      if constexpr (C > 1) feed_chunks<1>(s0, r, d);
      if constexpr (C > 2) feed_chunks<2>(s0, r, d);
      if constexpr (C > 3) feed_chunks<3>(s0, r, d);
    } else if (WIPDB_SHORT_PAD && short_pad) {
      // both groups' spans start in chain 0 (segments of 3 KiB+, e.g. a 4 KiB
      // block minus its trailer): the general path below with k0 = 0 known,
      // so only loads 0..C-1 of lane l0 can need the head mask, only chain 0
      // takes the injection, and only chain 0 of the lanes in front of l0 is
      // all virtual
      uint32_t pad_g[S], inj_g[S], m_g[S][4];
#pragma unroll
      for (int g = 0; g < S; ++g) {
        pad_g[g] = kSegChunks - (hn[g] >> 4);
        const uint32_t hh = h[g];
        inj_g[g] = (init[g] == 0u) ? lds_ld(kLdsHead0 + (hh << 2)) : unshift_bytes(s0, ~init[g], hh);
        m_g[g][0] = hh == 0 ? ~0u : (hh >= 4 ? 0u : (~0u << (8 * hh)));
        m_g[g][1] = hh <= 4 ? ~0u : (hh >= 8 ? 0u : (~0u << (8 * (hh - 4))));
        m_g[g][2] = hh <= 8 ? ~0u : (hh >= 12 ? 0u : (~0u << (8 * (hh - 8))));
        m_g[g][3] = hh <= 12 ? ~0u : (~0u << (8 * (hh - 12)));
      }
      const uint32_t pad = gsel(hi, pad_g[0], pad_g[1]);
      const uint32_t inj = gsel(hi, inj_g[0], inj_g[1]);
      const uint32_t l0 = pad / C, j0 = pad % C;
      const bool at0 = gl == l0;
      if (any_h) {
        const uint32_t m0 = gsel(hi, m_g[0][0], m_g[1][0]), m1 = gsel(hi, m_g[0][1], m_g[1][1]);
        const uint32_t m2 = gsel(hi, m_g[0][2], m_g[1][2]), m3 = gsel(hi, m_g[0][3], m_g[1][3]);
#pragma unroll
        for (int j = 0; j < C; ++j) {
          const bool mj = at0 && j0 == static_cast<uint32_t>(j);
          d[j].x &= mj ? m0 : ~0u;
          d[j].y &= mj ? m1 : ~0u;
          d[j].z &= mj ? m2 : ~0u;
          d[j].w &= mj ? m3 : ~0u;
        }
      }
      if (at0 && j0 == 0u) r[0] = inj;
      feed_chunks<0>(s0, r, d);
      if constexpr (C > 1) {
        if (at0 && j0 == 1u) r[0] = inj;
        feed_chunks<1>(s0, r, d);
      }
      if constexpr (C > 2) {
        if (at0 && j0 == 2u) r[0] = inj;
        feed_chunks<2>(s0, r, d);
      }
      if constexpr (C > 3) {
        if (at0 && j0 == 3u) r[0] = inj;
        feed_chunks<3>(s0, r, d);
      }
      if (gl < l0) r[0] = 0u;
    } else {
      // general path: chunk 0 of a group sits at its virtual chunk `pad`
      // (chain k0 = pad / (G*C), lane l0, sub-chunk j0): mask its first h
      // bytes and inject ~init * x^(-8h) into the chain just before it.  A
      // group without a main region gets pad = 256: all its chains are
      // zeroed.
      uint32_t pad_g[S], inj_g[S], m_g[S][4];
#pragma unroll
      for (int g = 0; g < S; ++g) {
        pad_g[g] = main_g[g] ? kSegChunks - (hn[g] >> 4) : kSegChunks;
        const uint32_t hh = h[g];
        inj_g[g] = 0u;
        if (main_g[g])
          inj_g[g] = (init[g] == 0u) ? lds_ld(kLdsHead0 + (hh << 2))
                                     : unshift_bytes(s0, ~init[g], hh);
        m_g[g][0] = hh == 0 ? ~0u : (hh >= 4 ? 0u : (~0u << (8 * hh)));
        m_g[g][1] = hh <= 4 ? ~0u : (hh >= 8 ? 0u : (~0u << (8 * (hh - 4))));
        m_g[g][2] = hh <= 8 ? ~0u : (hh >= 12 ? 0u : (~0u << (8 * (hh - 8))));
        m_g[g][3] = hh <= 12 ? ~0u : (~0u << (8 * (hh - 12)));
      }
      const uint32_t pad = gsel(hi, pad_g[0], pad_g[1]);
      const uint32_t inj = gsel(hi, inj_g[0], inj_g[1]);
      const uint32_t k0 = pad / (G * C), rem = pad % (G * C);
      const uint32_t l0 = X ? ((rem & 31u) & ~1u) + (rem >> 5) : rem / C;
      const uint32_t j0 = rem % C;
      const bool at0 = gl == l0;
      const uint32_t m0 = gsel(hi, m_g[0][0], m_g[1][0]), m1 = gsel(hi, m_g[0][1], m_g[1][1]);
      const uint32_t m2 = gsel(hi, m_g[0][2], m_g[1][2]), m3 = gsel(hi, m_g[0][3], m_g[1][3]);
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        if (at0 && static_cast<uint32_t>(i) == k0 * C + j0) {
          d[i].x &= m0;
          d[i].y &= m1;
          d[i].z &= m2;
          d[i].w &= m3;
        }
      }
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (at0 && static_cast<uint32_t>(k) == k0 && j0 == 0u) r[k] = inj;
      feed_chunks<0>(s0, r, d);
      // a chain whose first chunks are virtual: the register enters before
      // its first real chunk j0
      auto inject = [&](uint32_t j) {
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (at0 && static_cast<uint32_t>(k) == k0 && j0 == j) r[k] = inj;
      };
      if constexpr (C > 1) {
        inject(1u);
        feed_chunks<1>(s0, r, d);
      }
      if constexpr (C > 2) {
        inject(2u);
        feed_chunks<2>(s0, r, d);
      }
      if constexpr (C > 3) {
        inject(3u);
        feed_chunks<3>(s0, r, d);
      }
      // chains made only of virtual chunks (in front of the span) carry
      // garbage
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (vchunk(k, gl, C - 1) < pad) r[k] = 0u;
    }
    const uint32_t v = fold_groups(r, lane);
#pragma unroll
    for (int g = 0; g < S; ++g)
      if (main_g[g]) reg[g] = __builtin_amdgcn_readlane(v, g * G);
  }
  // ragged tails: bytes [o, e) of the chunk at a0 + (hn & ~15).  The tail
  // chunk came with the slot (d[NL], the same in a group's lanes), so the
  // lanes of each group feed their group's tail: both tails in the same
  // instructions
  uint32_t e_g[S], o_g[S];
  bool any_tail = false;
#pragma unroll
  for (int g = 0; g < S; ++g) {
    e_g[g] = (s[g].flags() & kSlotValid) ? (hn[g] & 15u) : 0u;
    o_g[g] = hn[g] < 16u ? h[g] : 0u;
    any_tail = any_tail || e_g[g] != 0u;
  }
#if WIPDB_PAR_TAIL
  if (any_tail) {
    const uint32_t rt = feed_tail_words(s0, gsel(hi, reg[0], reg[1]), d[NL].x, d[NL].y, d[NL].z,
                                        d[NL].w, gsel(hi, o_g[0], o_g[1]), gsel(hi, e_g[0], e_g[1]));
#pragma unroll
    for (int g = 0; g < S; ++g)
      if (e_g[g] != 0u) reg[g] = uni(static_cast<uint32_t>(__builtin_amdgcn_readlane(rt, g * G)));
  }
#else
#pragma unroll
  for (int g = 0; g < S; ++g) {
    if (e_g[g] != 0u) {
      const uint32_t t0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(d[NL].x, g * G));
      const uint32_t t1 = static_cast<uint32_t>(__builtin_amdgcn_readlane(d[NL].y, g * G));
      const uint32_t t2 = static_cast<uint32_t>(__builtin_amdgcn_readlane(d[NL].z, g * G));
      const uint32_t t3 = static_cast<uint32_t>(__builtin_amdgcn_readlane(d[NL].w, g * G));
      reg[g] = uni(feed_tail_words(s0, reg[g], t0, t1, t2, t3, o_g[g], e_g[g]));
    }
  }
  (void)any_tail;
#endif
#pragma unroll
  for (int g = 0; g < S; ++g) {
    const uint32_t c = ~reg[g];
    done[g] = (s[g].flags() & kSlotLast) != 0u;
    crc[g] = c;
    if (!done[g]) chain[g] = c;
  }
}

// The wave loop over segment pairs (one segment per group).  emit(span,
// crc, g) is called for every finished span, with all lanes active (span
// and crc uniform).
template <typename Src, typename Emit>
__device__ __forceinline__ void run_waves(Src& src, uint64_t wave, uint64_t waves,
                                          const void* dummy, uint32_t split, uint32_t* work,
                                          Emit emit) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t l4 = (threadIdx.x & 31u) * 4u;
  const uint32_t s0 = l4 | ((l4 | 0x80u) << 8) | (1u << 24);
  [[maybe_unused]] const uint64_t stride = waves * S;

  src.reset();
#if WIPDB_DYN
  WorkShare ws;
  ws.init(src.count, work);
#if WIPDB_GPOOL
  __syncthreads();
  auto span_of = [&](int, uint32_t ord) { return static_cast<uint64_t>(ord); };
#else
  auto span_of = [&](int, uint32_t ord) { return ws.span_of(ord); };
#endif
  DynCursor<Src> cur[S];
#else
  SegCursor<Src> cur[S];
  auto span_of = [&](int g, uint32_t ord) {
    return wave * S + g + static_cast<uint64_t>(ord) * stride;
  };
#endif
  uint32_t chain[S];
  uint32_t live = 0;  // groups with spans left (checked once: all zero -> return)
#pragma unroll
  for (int g = 0; g < S; ++g) {
#if WIPDB_DYN
    cur[g].begin(src, g, ws, lane, split);
#else
    cur[g].begin(src, g, wave * S + g, stride, lane, split);
#endif
    chain[g] = 0;
    live |= cur[g].left;
  }
  if (live == 0u) return;

  auto next = [&](Slot (&sl)[S]) {
#pragma unroll
    for (int g = 0; g < S; ++g)
#if WIPDB_DYN
      sl[g] = cur[g].next(src, g, ws, lane);
#else
      sl[g] = cur[g].next(src, g, wave * S + g, stride, lane);
#endif
  };
  auto valid = [](const Slot (&sl)[S]) {
    uint32_t f = 0;
#pragma unroll
    for (int g = 0; g < S; ++g) f |= sl[g].meta;
    return (f & (kSlotValid << 16)) != 0u;
  };
  auto finish = [&](const Slot (&sl)[S], u32x4 (&d)[NLT]) {
    uint32_t crc[S];
    bool done[S];
    // an opaque copy of the lane id: the lane predicates derived from it
    // are recomputed per segment (one v_cmp each) instead of being hoisted
    // into SGPR pairs that the register allocator then spills
    uint32_t ln = lane;
#if WIPDB_OPAQUE_LANE
    asm volatile("" : "+v"(ln));
#endif
    process_seg(sl, d, s0, ln, chain, crc, done, src.trailer);
#pragma unroll
    for (int g = 0; g < S; ++g)
      if (done[g])
        emit(span_of(g, sl[g].ord), crc[g], g, sl[g].init,
             (sl[g].flags() & kSlotPartial) != 0u);
  };

#if WIPDB_SLOTS == 1
  // One slot: issue a segment pair's loads, wait for all of them, compute
  // (nothing of this wave in flight while it computes).
  Slot sA[S];
  u32x4 bA[NLT];
  for (;;) {
    next(sA);
    if (!valid(sA)) break;
    issue_seg(sA, lane, dummy, bA);
    finish(sA, bA);
  }
#elif WIPDB_SLOTS == 3
  // Three slots: while one pair is processed the next two pairs' loads are
  // in flight.
  Slot sA[S], sB[S], sC[S];
  u32x4 bA[NLT], bB[NLT], bC[NLT];
  next(sA);
  issue_seg(sA, lane, dummy, bA);
  next(sB);
  issue_seg(sB, lane, dummy, bB);
  for (;;) {
    next(sC);
    issue_seg(sC, lane, dummy, bC);
    if (!valid(sA)) break;
    finish(sA, bA);

    next(sA);
    issue_seg(sA, lane, dummy, bA);
    if (!valid(sB)) break;
    finish(sB, bB);

    next(sB);
    issue_seg(sB, lane, dummy, bB);
    if (!valid(sC)) break;
    finish(sC, bC);
  }
#else
  // Two slots: while one pair is processed the other's loads are in flight.
  Slot sA[S], sB[S];
  u32x4 bA[NLT], bB[NLT];
  next(sA);
  issue_seg(sA, lane, dummy, bA);
  for (;;) {
    next(sB);
    issue_seg(sB, lane, dummy, bB);
    if (!valid(sA)) break;
    finish(sA, bA);

    next(sA);
    issue_seg(sA, lane, dummy, bA);
    if (!valid(sB)) break;
    finish(sB, bB);
  }
#endif
}

// Copy the device tables into LDS: main tables replicated 32x, the rest
// linear.  Every thread of the workgroup takes part; ends with a barrier.
__device__ __forceinline__ void load_tables(uint8_t* lds, const DevTables* __restrict__ tab) {
#if WIPDB_NO_TABLES  // diagnostic (load-only builds): skip the table copy
  if (threadIdx.x == 0u) *reinterpret_cast<uint32_t*>(lds + kLdsWork) = 0u;
  __syncthreads();
  return;
#endif
  const uint32_t tid = threadIdx.x;
  const uint32_t nthr = blockDim.x;
  // main: 4 tables x 256 bytes x 32 replicas; 4 consecutive replicas per store
  for (uint32_t e4 = tid; e4 < 8192u; e4 += nthr) {
    const uint32_t rep4 = e4 & 7u;          // replicas 4*rep4 .. 4*rep4+3
    const uint32_t b = (e4 >> 3) & 255u;
    const uint32_t t = e4 >> 11;            // 0..3
    const uint32_t v = tab->t[t][b];
    const uint32_t addr = kLdsMain + (t >> 1) * 65536u + b * 256u + (t & 1u) * 128u + rep4 * 16u;
    *reinterpret_cast<u32x4*>(lds + addr) = u32x4{v, v, v, v};
  }
  const u32x4* src = reinterpret_cast<const u32x4*>(tab->shift[kLogC]);
  u32x4* dst = reinterpret_cast<u32x4*>(lds + kLdsShift);
  for (uint32_t i = tid; i < kLdsShiftTables * 256u; i += nthr) dst[i] = src[i];
  uint32_t* inv = reinterpret_cast<uint32_t*>(lds + kLdsInvTop);
  for (uint32_t i = tid; i < 256u; i += nthr) inv[i] = tab->inv_top[i];
  uint32_t* hd = reinterpret_cast<uint32_t*>(lds + kLdsHead0);
  for (uint32_t i = tid; i < 16u; i += nthr) hd[i] = tab->head0[i];
  if (tid == 0u) *reinterpret_cast<uint32_t*>(lds + kLdsWork) = 0u;
  __syncthreads();
}

__device__ __forceinline__ uint64_t wave_id() {
  return static_cast<uint64_t>(blockIdx.x) * kWaves + uni(threadIdx.x >> 6);
}

__device__ __forceinline__ uint64_t grid_waves() {
  return static_cast<uint64_t>(gridDim.x) * kWaves;
}

// End of a kernel that took blocks from the pool `work`: once all of a
// workgroup's waves are done it checks in, and the last workgroup to check
// in zeroes the pool counter and the arrival count, so the buffer is ready
// for its next launch (hcrc_api.cc WorkPool).
__device__ __forceinline__ void release_pool(uint32_t* work) {
#if WIPDB_GPOOL
  __syncthreads();
  if (threadIdx.x == 0u) {
    uint32_t* arrived = work + kPoolArrive;
    const uint32_t n =
        __hip_atomic_fetch_add(arrived, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (n + 1u == gridDim.x) {
      __hip_atomic_store(work, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(arrived, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#else
  (void)work;
#endif
}

// Stores one value per finished span: lane g*G writes group g's result.
__device__ __forceinline__ bool group_leader(int g) {
  return (threadIdx.x & 63u) == static_cast<uint32_t>(g * G);
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// Descriptor batch: span i = base + offsets[i], lengths[i] bytes, inits[i].
__global__ __launch_bounds__(kThreads) void crc32c_spans_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags,
    const DevTables* __restrict__ tab, uint32_t* __restrict__ work) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
#if WIPDB_TIMELINE
  const uint64_t t_entry = wall_clock64();
#endif
  load_tables(lds, tab);
#if WIPDB_TIMELINE
  uint64_t* tl = g_timeline + static_cast<uint64_t>(blockIdx.x) * kTimelineStride;
  const bool stamp = blockIdx.x < static_cast<uint32_t>(kTimelineWGs) && (threadIdx.x & 63u) == 0u;
  if (stamp && threadIdx.x == 0u) {
    tl[0] = t_entry;
    tl[1] = wall_clock64();
  }
#endif
  DescSource src{base, offsets, lengths, inits, count, 0u, false, 0, 0, 0, 0, {0, 0}};
  const bool msk = (flags & kFlagMask) != 0;
  run_waves(src, wave_id(), grid_waves(), tab, flags & (kFlagSkipSmall | kFlagSplitRem), work,
            [&](uint64_t span, uint32_t crc, int g, uint32_t, bool partial) {
    // a partial CRC (remainder left to the small kernel) stays unmasked
#if WIPDB_NO_STORE  // diagnostic: what the scattered 4-byte result stores cost (wrong results)
    if (group_leader(g) && crc == 0x9E3779B9u) out[span] = crc;
#else
    if (group_leader(g)) out[span] = msk && !partial ? mask_crc(crc) : crc;
#endif
  });
#if WIPDB_TIMELINE
  if (stamp) tl[2 + (threadIdx.x >> 6)] = wall_clock64();
#endif
  release_pool(work);
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride_bytes, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags,
    const DevTables* __restrict__ tab, uint32_t* __restrict__ work) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  StridedSource src{base, stride_bytes, length, init, count, 0u};
  const bool msk = (flags & kFlagMask) != 0;
  run_waves(src, wave_id(), grid_waves(), tab, 0u, work,
            [&](uint64_t span, uint32_t crc, int g, uint32_t, bool) {
    if (group_leader(g)) out[span] = msk ? mask_crc(crc) : crc;
  });
  release_pool(work);
}

// Read-side verify: block = base + off, n = handle size; crc over n+1 bytes
// compared with Unmask(LE32 at n+1) (kv/src/table/format.cc:91-99).
// With HCRC_SPLIT_SMALL (flags kFlagSkipSmall | kFlagSplitRem) blocks of at
// most kSmallMax bytes are left to the small kernel, and a block that just
// overruns a segment stops after it, its partial CRC going to partial[s]
// for the small kernel to continue (and to verify).
__global__ __launch_bounds__(kThreads) void crc32c_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status, uint64_t count,
    const DevTables* __restrict__ tab, uint32_t* __restrict__ work, uint32_t flags,
    uint32_t* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_tables(lds, tab);
  // the stored trailer crc rides in the descriptor cache (fetched with the
  // offsets, 32 spans at a time), so emitting a status needs no load
  DescSource src{base, offsets, lengths, nullptr, count, 1u, true, 0, 0, 0, 0, {0, 0}};
  run_waves(src, wave_id(), grid_waves(), tab, flags & (kFlagSkipSmall | kFlagSplitRem), work,
            [&](uint64_t s, uint32_t crc, int g, uint32_t stored, bool cut) {
              if (group_leader(g)) {
                if (cut) {
                  partial[s] = crc;
                } else {
                  const uint32_t rot = stored - 0xa282ead8u;
                  status[s] = ((rot >> 17) | (rot << 15)) == crc ? 1 : 0;
                }
              }
            });
  release_pool(work);
}

#include "crc32c_small.inc"

// Read-stream ceiling: the same 16-byte nontemporal loads over fixed-size
// blocks, XOR-reduced (diagnostic; the roofline's measured denominator).
__global__ __launch_bounds__(kThreads) void readstream_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length,
    uint32_t* __restrict__ out, uint64_t count) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint32_t chunks = length >> 4;
#if WIPDB_RS_SPLIT
  // diagnostic: a half-wave per block, like the CRC kernels' lane groups
  // (32 lanes x WIPDB_RS_UNROLL loads in flight)
  for (uint64_t s2 = wave_id(); 2 * s2 < count; s2 += nw) {
    const uint64_t s = 2 * s2 + (lane >> 5);
    uint32_t acc = 0;
    if (s < count) {
      g_u32x4* cp = reinterpret_cast<g_u32x4*>(reinterpret_cast<uintptr_t>(base + s * stride));
      uint32_t i = lane & 31u;
      for (; i + 32u * (WIPDB_RS_UNROLL - 1) < chunks; i += 32u * WIPDB_RS_UNROLL) {
        u32x4 v[WIPDB_RS_UNROLL];
#pragma unroll
        for (int k = 0; k < WIPDB_RS_UNROLL; ++k) v[k] = __builtin_nontemporal_load(cp + i + 32u * k);
#pragma unroll
        for (int k = 0; k < WIPDB_RS_UNROLL; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      }
    }
#if WIPDB_RS_SALU
    // diagnostic: the CRC skeleton's scalar work per slot, as dependent SALU ops
    {
      uint32_t x = static_cast<uint32_t>(s2);
#pragma unroll
      for (int k = 0; k < WIPDB_RS_SALU; ++k) asm volatile("s_add_u32 %0, %0, 1" : "+s"(x));
      acc ^= x & 0x80000000u;
    }
#endif
#pragma unroll
    for (int k = 16; k >= 1; k >>= 1) acc ^= __shfl_xor(acc, k, 64);
    if ((lane & 31u) == 0u && s < count) out[s] = acc;
  }
  return;
#endif
  for (uint64_t s = wave_id(); s < count; s += nw) {
    g_u32x4* cp = reinterpret_cast<g_u32x4*>(reinterpret_cast<uintptr_t>(base + s * stride));
    uint32_t acc = 0;
#if WIPDB_RS_UNROLL > 1
    // diagnostic: more loads in flight per wave
    uint32_t i = lane;
    for (; i + 64u * (WIPDB_RS_UNROLL - 1) < chunks; i += 64u * WIPDB_RS_UNROLL) {
      u32x4 v[WIPDB_RS_UNROLL];
#pragma unroll
      for (int k = 0; k < WIPDB_RS_UNROLL; ++k) v[k] = __builtin_nontemporal_load(cp + i + 64u * k);
#pragma unroll
      for (int k = 0; k < WIPDB_RS_UNROLL; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < chunks; i += 64) {
      const u32x4 v = __builtin_nontemporal_load(cp + i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
#else
    for (uint32_t i = lane; i < chunks; i += 64) {
      const u32x4 v = __builtin_nontemporal_load(cp + i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
#endif
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

#if WIPDB_TIMELINE
// Diagnostic (variant builds only): copy the last spans launch's stamps.
extern "C" int hcrc_debug_timeline(uint64_t* dst, size_t n) {
  const size_t cap = static_cast<size_t>(wipdb::dev::kTimelineWGs) * wipdb::dev::kTimelineStride;
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(wipdb::dev::g_timeline), n * 8) == hipSuccess
             ? static_cast<int>(n) : -1;
}
#endif
