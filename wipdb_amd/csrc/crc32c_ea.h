// crc32c_ea.h -- run_ea, the END-ALIGNED pipeline (round 2's spans kernel):
// one span at a time per wave (a unit per LDS atomic, its descriptor through
// scalar loads), its segments END-aligned at its last chunk, the first one
// partial, table blocks as a main segment + a front piece of <= 16 chunks
// batched 16 per iteration (crc32c_walk.h).  Used by the class-1 list kernel
// (crc32c_list.hip: HCRC_SPLIT_SMALL's long class, HCRC_SPLIT_LONG's parts)
// and by the spans / verify / strided kernels for batches whose sampled spans
// all suit it (crc32c_lds.hip pick_pipeline: aligned 4 KiB blocks, table
// blocks, ReadBlock's 4 KiB blocks, spans of >= 16 KiB).  DESIGN.md section 4.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// kv/src/util/crc32c.cc:1225-1227) applied per block span, as
// TableBuilder::WriteRawBlock (kv/src/table/table_builder.cc:194-196) and
// ReadBlock (kv/src/table/format.cc:91-93) do.
#pragma once
#include <stdint.h>

#include <type_traits>

#include "crc32c_dev.h"
#include "crc32c_walk.h"

#ifndef LP_T  // (the profiling build's markers, crc32c_lds.hip)
#define LP_T(x)
#define LP_ACC(k, v)
#endif

namespace wipdb {
namespace lk {

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
  const uint32_t l = lane_tid() & 63u;
  const uint32_t w = uni(lane_tid() >> 6);
  const uint64_t count = src.count;
  const WgUnits units = wg_units(count, src_bounds(src));
  if (units.count == 0u) return;  // no unit of work
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
    const uint64_t s = grab_unit(l, units);
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
#ifdef WIPDB_PROF_ON
  // profiling build: 0 wait, 1 landed -> next DMA out, 2 compute, 4 pages, 7 life
  uint64_t prof[kProfN] = {};
  LP_T(t_start);
#endif
  uint32_t chain = 0;  // register carried between the segments of a span
  bool stored_prev = false;
  g_u32* const out32 = (g_u32*)(reinterpret_cast<uintptr_t>(out));
  g_u8* const out8 = (g_u8*)(reinterpret_cast<uintptr_t>(out));

  for (;;) {
    LP_T(e0);
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    LP_T(e1);
    LP_ACC(0, e1 - e0);
    LP_ACC(4, 1);
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

    LP_T(e2);
    LP_ACC(1, e2 - e1);
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
#ifdef WIPDB_PROF_ON
    LP_T(e3);
    LP_ACC(2, e3 - e2);
#endif

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
#ifdef WIPDB_PROF_ON
  LP_T(t_end);
  prof[7] = t_end - t_start;
  if (l == 0u) {
    const uint32_t slot = (group_id() * static_cast<uint32_t>(kWaves) + w) & 4095u;
    for (int k = 0; k < kProfN; ++k)
      atomicAdd(&g_lp_prof[slot * kProfN + k], static_cast<unsigned long long>(prof[k]));
  }
#endif
}

}  // namespace lk
}  // namespace wipdb
