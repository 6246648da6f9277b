// crc32c_ps.h -- run_ps, the STREAM-TILED pipeline for SST-packed batches
// (HCRC_PACKED).  DESIGN.md section 4 "Packed batches".
//
// A packed batch is what TableBuilder::WriteRawBlock leaves in a write buffer
// (kv/src/table/table_builder.cc:183-202: contents + type byte, then the
// 4-byte trailer, then the next block), what a WAL block holds, and config 3:
// spans sorted by offset, not overlapping, with gaps of less than 4 KiB.  Such
// a batch is one byte stream, and run_ps reads it as one: the covering range
// is cut into 4 KiB pages ("windows", page-aligned in the address space), and
// a wave iteration DMAs one window into its LDS slot exactly like an aligned
// 4 KiB block (global_load_lds_dwordx4, fully coalesced, no per-lane source
// exchange) and lane l checksums stripe [64 l, 64 l + 64) of it.
//
// Span boundaries are made harmless in the window itself, before the lanes
// read it: the lanes of the wave's desk (one span each) zero the gap bytes
// in front of their span (trailers, other spans' bytes), mask the bytes in
// front of its first byte and XOR its head register ~init * x^(-8 h) into its
// first word (ds_* on the slot), and hand the lane of the stripe that holds
// its last stream word the cut's position (v_writelane, no LDS).  A span of n bytes at A is its STREAM words [A & ~3,
// E4 = (A + n) & ~3) plus a tail of k = (A + n) & 3 bytes, which the desk lane
// loads from memory and feeds at the end (one slicing step).  A lane's scan
// over its 16 words then only has to cut once: at the stripe's span end (at
// most one -- stream spans are >= 64 bytes), where it keeps the register F
// and starts again from 0.  Per window:
//
//   O_l   the register at the end of stripe l (the span open there, or 0),
//   IN_L  for a cut lane L: the register entering stripe L of its span =
//         XOR over the lanes l of its segment (from the previous cut lane to
//         L - 1) of O_l * x^(8 * 64 (L - 1 - l)) -- each lane shifts its O
//         by whole stripes (the two fold-table levels, shift64) and one wave
//         prefix XOR gives every segment (the reference's CombineCRC identity,
//         kv/src/util/crc32c.cc:640-657, at stripe granularity),
//   carry the register of the span still open at the window's end, XORed
//         into word 0 of the next window by lane 0.
//
// The register at a span's end is IN * x^(32 t) ^ F (t = its words in the cut
// stripe) -- a per-span shift of 1 .. 16 words, deferred to the desk's end,
// when all its lanes run it at once (one 16-step pass per 64 spans), then
// the tail step, ~, Mask and the store.  Spans of fewer than 64 bytes (and
// empty ones) are not in the stream: their bytes are zeroed as gap and the
// desk lane computes them from memory (rare: a table's metaindex block).
//
// Work: the pre-pass (ps_index_kernel; the host does it for host batches)
// checks the batch (sorted, no overlap, gaps < 4 KiB, at most 62 spans
// starting in any 4 KiB) and cuts the covering range into C equal byte
// chunks, first[c] = the first span starting in chunk c.  Workgroup g takes
// chunks [g C / G, (g + 1) C / G) -- equal bytes, whatever the sizes -- and
// its waves take them one at a time; a chunk is its spans, whole (the range
// a wave reads ends at its last span's end).  A batch that fails the check
// runs the lane-packed pipeline (run_lp) instead: HCRC_PACKED is a promise the
// kernel verifies, never a way to a wrong CRC.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// crc32c.cc:1225-1227) per block span, as WriteRawBlock
// (kv/src/table/table_builder.cc:194-196) applies it.
#pragma once
#include <stdint.h>

#include "crc32c_dev.h"

namespace wipdb {
namespace lk {

constexpr uint32_t kPsDesk = 64;        // spans per desk (one per lane)
constexpr uint32_t kPsMinStream = 96;   // spans shorter than this are computed off the stream
                                        // (a stream span's stream part is then >= 64 bytes)
constexpr uint32_t kPsMaxGap = 4096;    // a larger gap could leave a page of no span's bytes
constexpr uint32_t kPsDense = 62;       // spans i, i + 62 start >= 4 KiB apart

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// the inclusive max over lanes 0 .. l (values >= 0; lanes without a DPP
// source read 0)
__device__ __forceinline__ uint32_t scan_max(uint32_t v) {
  v = umax(v, dpp<0x111>(v));
  v = umax(v, dpp<0x112>(v));
  v = umax(v, dpp<0x114>(v));
  v = umax(v, dpp<0x118>(v));
  v = umax(v, bcast15(v));
  return umax(v, bcast31(v));
}

// The LDS address of window byte p (< 4096) in a wave slot: the window DMA
// (Pipe::cm) puts window chunk 64 q + cm(m) at slot + 1024 q + 16 m, so the
// lanes' stripe reads are conflict-free; m = cm^-1(c).
__device__ __forceinline__ uint32_t ps_lds_addr(uint32_t slot, uint32_t p) {
  const uint32_t C = p >> 4, c = C & 63u;
  const uint32_t m = (c & ~3u) | (((c & 3u) + (c >> 4)) & 3u);
  return slot + ((C >> 6) << 10) + (m << 4) + (p & 15u);
}

// The low b bytes of a word kept (b = 0..4).
__device__ __forceinline__ uint32_t low_bytes(uint32_t b) {
  return b >= 4u ? ~0u : ((1u << (8u * b)) - 1u);
}

// ---------------------------------------------------------------------------
// The pre-pass: check the batch, cut its covering range into C chunks.
// Thread i handles span i (grid-stride); meta[0] is ORed, first[] written
// where the chunk index steps.  first has C + 1 entries, first[C] = n.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ps_index(const uint8_t* base, const uint64_t* off,
                                         const uint32_t* len, uint64_t n, uint32_t C,
                                         uint32_t* first, uint32_t* meta, uint64_t tid,
                                         uint64_t nthreads) {
  if (n == 0) return;
  const uint64_t lo = off[0];
  const uint64_t hi = off[n - 1] + len[n - 1];
  const uint64_t range = hi > lo ? hi - lo : 1u;
  uint64_t cb = (range + C - 1u) / C;
  cb = (cb + 4095u) & ~uint64_t(4095);
  if (cb < 4096u) cb = 4096u;
  if (tid == 0) {
    meta[1] = static_cast<uint32_t>(cb);
    meta[2] = static_cast<uint32_t>(cb >> 32);
    meta[3] = static_cast<uint32_t>(lo);
    meta[4] = static_cast<uint32_t>(lo >> 32);
  }
  uint32_t bad = 0;
  for (uint64_t i = tid; i < n; i += nthreads) {
    const uint64_t a = off[i];
    uint64_t c = a >= lo ? (a - lo) / cb : 0u;
    if (a < lo || c >= C) {
      bad |= kPsBad;
      c = C - 1u;
    }
    uint64_t cp = 0;  // chunks (cp, c] start at span i
    if (i == 0) {
      cp = 0;
      first[0] = 0;
    } else {
      const uint64_t ap = off[i - 1], bp = ap + len[i - 1];
      if (a < bp || a - bp >= kPsMaxGap) bad |= kPsBad;
      cp = ap >= lo ? (ap - lo) / cb : 0u;
      if (cp > c) cp = c;
    }
    for (uint64_t k = cp + 1u; k <= c; ++k) first[k] = static_cast<uint32_t>(i);
    if (i + kPsDense < n && off[i + kPsDense] - a < 4096u) bad |= kPsBadDense;
    if (i + kPsDense < n && off[i + kPsDense] < a) bad |= kPsBad;
    if (i == n - 1)
      for (uint64_t k = c + 1u; k <= C; ++k) first[k] = static_cast<uint32_t>(n);
  }
  (void)base;
  if (bad) global_or(meta, bad);
}

// ---------------------------------------------------------------------------
// run_ps.  Src: DescSrc (offsets, lengths, inits).
// ---------------------------------------------------------------------------
template <typename Src>
__device__ __forceinline__ void run_ps(const Src& src, void* out, uint32_t flags,
                                       const uint8_t* image, const uint32_t* __restrict__ first,
                                       uint32_t C, unsigned int* fault) {
  const uint32_t l = lane_tid() & 63u;
  const uint32_t w = uni(lane_tid() >> 6);
  const uint32_t G = group_count(), g = group_id();
  const bool rr = (flags & kFlagPsRR) != 0u;
  const uint32_t c_lo = rr ? 0u : static_cast<uint32_t>(static_cast<uint64_t>(C) * g / G);
  const uint32_t c_hi = rr ? (C > g ? (C - g + G - 1u) / G : 0u)
                           : static_cast<uint32_t>(static_cast<uint64_t>(C) * (g + 1u) / G);
  if (c_lo >= c_hi) return;
  load_image(image, w, l);
  const Lane lk = make_lane<1>(l);
  Pipe pp;
  pp.init(l, w);
  const bool msk = (flags & kFlagMask) != 0u;
  const uint64_t sbase = reinterpret_cast<uint64_t>(src.base);
  g_u32* const out32 = (g_u32*)(reinterpret_cast<uintptr_t>(out));
  // per-lane selector bases of shift64
  uint32_t k1b = 0, k2b = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t t = (j + ((l >> 3) & 3u)) & 3u;
    k1b |= (128u + 4u * t) << (8 * j);
    k2b |= (8u * t) << (8 * j);
  }
  const uint32_t dma_o = 16u * pp.cm;

  // ---- desk state (lane j: span d0 + j), relative to the chunk's W0 ----
  // A stream span [a, b) is its stream words [a & ~3, E16 = b & ~15) and a
  // tail of k16 = b - E16 < 16 bytes (loaded from memory with the desk): its
  // last stream word is the last of a 16-byte chunk, so the scan can only
  // have to cut after word 3, 7, 11 or 15 of a stripe.
  uint32_t a32 = 0, b32 = 0;      // span [a32, b32)
  uint32_t hw = 0;                // its head word: bytes before A zeroed, ~init * x^(-8 h) XORed in
  uint32_t pe = 0;                // E16 of the previous stream span: its pre-gap is [pe, hd)
  u32x4 tt{0, 0, 0, 0};           // the tail chunk [E16, E16 + 16) from memory
  uint32_t in_r = 0, f_r = 0;     // IN and F at its cut
  uint32_t hwin = 0, cwin = 0;    // the pages (relative indices) of its head word and its cut
  uint32_t ha = 0, cs = 0, cv = 0;  // LDS address of the head word; cut stripe, tc | lane << 8
  uint32_t st = 0;                // bit 0: a stream span; bit 1: it has a pre-gap
  uint32_t id = 0;
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
  // profiling build: 0 wait, 1 landed -> next DMA out, 2 compute, 3 desk
  // loads, 4 pages, 5 pages with a cut, 6 chunk starts, 7 life, 8 finish,
  // 9 chunks
  uint64_t prof[kProfN] = {};
  LP_T(t_start);
#endif

  for (;;) {
    // ---- the next chunk of the workgroup ----
    uint32_t cc = 0;
    if (l == 0u) cc = lds_add(MiscAddr(kMiscUnit), 1u);
    cc = uni(cc) + c_lo;
    if (cc >= c_hi) break;
    if (rr) cc = cc * G + g;
    const uint32_t s_lo = uni(first[cc]), s_hi = uni(first[cc + 1u]);
    if (s_lo >= s_hi) continue;
    LP_ACC(9, 1);
    const uint64_t a_first = sbase + src.off[s_lo];
    const uint64_t b_last = sbase + src.off[s_hi - 1u] + src.len[s_hi - 1u];
    const uint64_t W0 = a_first & ~uint64_t(4095);
    const uint32_t wend = static_cast<uint32_t>(((b_last + 4095u) & ~uint64_t(4095)) - W0);
    // the first window's DMA right away (the desk loads go out behind it)
    dma4(W0, pp.slot, dma_o, dma_o + 1024u, dma_o + 2048u, dma_o + 3072u);
    uint32_t d0 = s_lo, dn = 0;
    uint32_t pe_carry = 0;  // E16 of the last stream span before the desk
    uint32_t pe_end = 0;    // E16 of the chunk's last stream span (its last desk)
    bool last_desk = false;
    uint32_t carry = 0;
    uint32_t wr = 0;

    // the deferred end of the stream spans of the desk whose cut is done
    // (lanes in `done`): R = IN * x^(32 t) ^ F (t = 4 tc words), the tail's
    // k16 bytes, ~, Mask, store
    auto finish = [&](uint64_t done) {
      const bool me = ((done >> l) & 1u) != 0u;
      const uint32_t t = 4u * (cv & 7u);
      uint32_t r = in_r;
      for (uint32_t i = 0; i < 16u; ++i) {
        const bool go = me && i < t;
        if (ballot(go) == 0u) break;
        const uint32_t x = step(lk, r, 0u);
        r = go ? x : r;
      }
      r ^= f_r;
      const uint32_t k16 = b32 & 15u, kw = k16 >> 2;
      const uint32_t t0 = step(lk, r ^ tt.x, 0u);
      r = kw >= 1u ? t0 : r;
      const uint32_t t1 = step(lk, r ^ tt.y, 0u);
      r = kw >= 2u ? t1 : r;
      const uint32_t t2 = step(lk, r ^ tt.z, 0u);
      r = kw >= 3u ? t2 : r;
      const uint32_t twd = kw == 0u ? tt.x : (kw == 1u ? tt.y : (kw == 2u ? tt.z : tt.w));
      r = tail_step(lk, r, twd, k16 & 3u);
      const uint32_t crc = ~r;
      if (me) out32[id] = msk ? mask_crc(crc) : crc;
    };

    for (;;) {
      // ---- a desk: spans [d0, d0 + dn); short / empty spans answered here ----
      LP_T(dk0);
      dn = umin(kPsDesk, s_hi - d0);
      last_desk = d0 + dn == s_hi;
      {
        const bool v = l < dn;
        uint64_t a = 0;
        uint32_t n = 0, iv = 0;
        if (v) src.lane(d0 + l, a, n, iv);
        wait_vm<0>();
        loads_landed(a);
        loads_landed(n);
        loads_landed(iv);
        a32 = v ? static_cast<uint32_t>(sbase + a - W0) : wend;
        b32 = v ? a32 + n : wend;
        id = d0 + l;
        const bool stream = v && n >= kPsMinStream;
        const uint32_t e16 = b32 & ~15u, hd = a32 & ~3u;
        // the previous stream span's E16 (exclusive max over the lanes before)
        const uint32_t incl = scan_max(stream ? e16 : 0u);
        const uint32_t pb = bperm(incl, l == 0u ? 0u : l - 1u);  // (every lane: a wave op)
        pe = umax(l == 0u ? 0u : pb, pe_carry);
        if (last_desk) pe_end = umax(pe_carry, rdlane(incl, 63));
        const uint32_t inj = head_register_lane(l, stream ? iv : 0u, a32 - hd);
        st = (stream ? 1u : 0u) | (stream && pe < hd ? 2u : 0u);
        in_r = f_r = 0;
        // the page events: head word, cut (the last stream chunk's stripe)
        const uint32_t lc = e16 - 16u;
        hwin = stream ? hd >> 12 : ~0u;
        cwin = stream ? lc >> 12 : ~0u;
        ha = ps_lds_addr(pp.slot, hd & 4095u);
        cs = (lc & 4095u) >> 6;
        cv = (((lc & 63u) >> 4) + 1u) | (l << 8);
        // head word and tail chunk from memory (each in the span's pages)
        hw = 0;
        if (stream) hw = *reinterpret_cast<const uint32_t*>(W0 + hd);
        hw = (hw & ~low_bytes(a32 - hd)) ^ inj;
        tt = u32x4{0, 0, 0, 0};
        if (stream && (b32 & 15u) != 0u) tt = *reinterpret_cast<const u32x4*>(W0 + e16);
        // spans off the stream: empty ones (crc = init) and short ones,
        // byte by byte from aligned memory words
        const bool small = v && !stream;
        if (ballot(small) != 0u) {
          uint32_t r = ~iv;
          if (small && n != 0u) {
            uint32_t wd = 0;
            for (uint32_t p = a32; p < b32; ++p) {
              if (p == a32 || (p & 3u) == 0u) wd = *reinterpret_cast<const uint32_t*>(W0 + (p & ~3u));
              r = feed_byte(l, r, (wd >> (8u * (p & 3u))) & 0xffu);
            }
          }
          const uint32_t crc = ~r;
          if (small) out32[id] = msk ? mask_crc(crc) : crc;
        }
      }
      // the windows this desk covers: up to the one where its last span
      // starts (the next span may start there)
      const uint32_t wstop =
          last_desk ? wend : umin(wend, uni(rdlane(a32, dn - 1u)) & ~4095u);
      LP_T(dk1);
      LP_ACC(3, dk1 - dk0);
      const bool sstream = (st & 1u) != 0u;
      for (; wr < wstop; wr += 4096u) {
        // ---- the page's fix-ups, planned before it lands ----
        const uint32_t wi = wr >> 12, wrel_end = wr + 4096u;
        const bool head = hwin == wi;
        const bool cut = cwin == wi;
        const bool gap = (st & 2u) != 0u && pe < wrel_end && (a32 & ~3u) > wr;
        const bool gaps = ballot(gap) != 0u;
        const bool post = last_desk && pe_end < wrel_end;
        // the cuts to their stripes' lanes (tc: after chunk tc, 0 = none)
        uint32_t tc = 0;
        for (uint64_t cm = ballot(cut); cm != 0u; cm &= cm - 1u) {
          const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(cm));
          tc = wrlane(tc, rdlane(cv, j) & 7u, rdlane(cs, j));
        }
        LP_T(w0);
        wait_vm<0>();
        LP_T(w1);
        LP_ACC(0, w1 - w0);
        LP_ACC(4, 1);
        loads_landed(hw);
        loads_landed(tt);
        // the page has landed: this wave issues ahead of the others' compute
        // until its next DMA is out (as run_lp does)
        if constexpr (kPrio != 0) lk_prio<kPrio>();
        if (gaps) {
          // each lane the first 8 words of its gap (trailers, tails: a few
          // words), the wave together the rest of longer ones (a chunk's
          // first page in front of its first span)
          const uint32_t z0 = umax(pe, wr);
          const uint32_t z1 = umin(a32 & ~3u, wrel_end);
          for (uint32_t p = z0;; p += 4u) {
            const bool go = gap && p < z1;
            if (ballot(go) == 0u || p >= z0 + 32u) break;
            if (go) lds_st(ps_lds_addr(pp.slot, p - wr), 0u);
          }
          uint64_t big = ballot(gap && z1 > z0 + 32u);
          while (big != 0u) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(big));
            big &= big - 1u;
            const uint32_t b = rdlane(z1, j);
            for (uint32_t p = rdlane(z0, j) + 32u + 4u * l; p < b; p += 256u)
              lds_st(ps_lds_addr(pp.slot, p - wr), 0u);
          }
        }
        if (post) {
          for (uint32_t p = umax(pe_end, wr) + 4u * l; p < wrel_end; p += 256u)
            lds_st(ps_lds_addr(pp.slot, p - wr), 0u);
        }
        if (head) lds_st(ha, hw);
        lds_order();  // the fix-ups, then the lanes' reads of the page
        uint32_t W[16];
        pp.read(W);
        pp.release();
        // ---- the next page's DMA ----
        if (wrel_end < wend) dma4(W0 + wrel_end, pp.slot, dma_o, dma_o + 1024u, dma_o + 2048u, dma_o + 3072u);
        if constexpr (kPrio != 0) lk_prio<0>();
        LP_T(w2);
        LP_ACC(1, w2 - w1);
        // ---- the scan ----
        W[0] ^= l == 0u ? carry : 0u;
        const uint64_t cutm = ballot(tc != 0u);
        const bool at_end = cutm == (uint64_t(1) << 63) && rdlane(tc, 63) == 4u;
        if (cutm == 0u || at_end) {
          // no span ends in this page (long spans' middles): the plain scan
          // and the whole-page fold carry the open span on; or the one that
          // ends does so at the page's end (aligned blocks): the fold is its
          // register, and nothing is carried
          const uint32_t r = fold<1>(lk, l, scan(lk, W))[0];
          carry = at_end ? 0u : r;
          if (at_end && cut) {
            in_r = r;
            f_r = 0;
            cv &= ~7u;  // (no words after IN)
          }
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
          LP_T(w3);
          LP_ACC(2, w3 - w2);
#endif
          continue;
        }
        uint32_t x = W[0], fr = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t a0 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[0]));
          const uint32_t a1 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[1]));
          const uint32_t a2 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[2]));
          const uint32_t a3 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[3]));
          uint32_t y = xor3(a0, a1, a2) ^ a3;  // the register after word i
          if ((i & 3) == 3) {  // a chunk's end: the cut may be here
            const bool c = tc == static_cast<uint32_t>((i >> 2) + 1);
            fr = c ? y : fr;
            y = c ? 0u : y;
          }
          x = i < 15 ? y ^ W[i + 1 < 16 ? i + 1 : 15] : y;
        }
        const uint32_t o_r = x;  // the register at the stripe's end (0 after a cut at word 15)
        // ---- the page's segments ----
        const uint64_t above = l == 63u ? 0u : (cutm >> (l + 1u)) << (l + 1u);
        const uint32_t nxt = above ? static_cast<uint32_t>(__builtin_ctzll(above)) : 64u;
        const uint32_t v = shift64(lk, k1b, k2b, o_r, nxt - 1u - l);
        const uint32_t qx = scan_xor(v);
        const uint64_t below = cutm & ((uint64_t(1) << l) - 1u);
        const uint32_t prv = below ? 63u - static_cast<uint32_t>(__builtin_clzll(below)) : 0u;
        const uint32_t q1 = bperm(qx, l == 0u ? 0u : l - 1u);
        const uint32_t q2 = bperm(qx, prv == 0u ? 0u : prv - 1u);
        const uint32_t in_l = (l == 0u ? 0u : q1) ^ (prv == 0u ? 0u : q2);
        {  // the carry: the last segment, to the page's end
          const uint32_t plast = 63u - static_cast<uint32_t>(__builtin_clzll(cutm));
          const uint32_t q63 = rdlane(qx, 63);
          const uint32_t qp = plast == 0u ? 0u : rdlane(qx, plast - 1u);
          carry = q63 ^ qp;
        }
        {  // desk lanes whose span was cut here take IN and F from the cut stripe
          const uint32_t sl = cut ? cs : l;
          const uint32_t gi = bperm(in_l, sl), gf = bperm(fr, sl);
          if (cut) {
            in_r = gi;
            f_r = gf;
          }
        }
        LP_ACC(5, 1);
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
        LP_T(w3);
        LP_ACC(2, w3 - w2);
#endif
      }
      if (wr >= wend) break;
      // ---- the next desk: the spans done are a prefix (ordered spans): a
      // stream span once its cut is behind the page, any other once its
      // bytes are (answered at its desk's load) ----
      const bool done = l < dn && (sstream ? (b32 & ~15u) <= wr : b32 <= wr);
      const uint32_t ngone = static_cast<uint32_t>(__builtin_popcountll(ballot(done)));
      LP_T(f0);
      finish(ballot(done && sstream));
      LP_T(f1);
      LP_ACC(8, f1 - f0);
      pe_carry = umax(pe_carry, rdlane(scan_max(done && sstream ? (b32 & ~15u) : 0u), 63));
      if (ngone == 0u) {  // (cannot happen in a checked batch: at most 63 spans meet a page)
        report_fault(fault, kFaultPsDesk);
        return;
      }
      d0 += ngone;
    }
    // ---- the chunk's end: every stream span of its last desk ----
    LP_T(f0);
    finish(ballot(l < dn && (st & 1u) != 0u));
    LP_T(f1);
    LP_ACC(8, f1 - f0);
  }
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
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
