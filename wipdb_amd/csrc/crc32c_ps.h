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
// first word (ds_* on the slot), and mark the stripe that holds its last word
// in a per-wave table.  A span of n bytes at A is its STREAM words [A & ~3,
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
constexpr uint32_t kPsMinStream = 64;   // spans shorter than this are computed off the stream
constexpr uint32_t kPsMaxGap = 4096;    // a larger gap could leave a page of no span's bytes
constexpr uint32_t kPsDense = 62;       // spans i, i + 62 start >= 4 KiB apart

// The per-wave cut table: 64 words (stripe s: 0, or (te | owner desk lane <<
// 8), te = 1 .. 16 the words up to and including the span's last stream
// word) in the a = 0 column of the wave's 16 main rows (the aux pieces of
// the other pipelines).
__device__ __forceinline__ uint32_t PsCutAddr(uint32_t w, uint32_t s) {
  return AuxAddr(w, s >> 2) + 4u * (s & 3u);
}

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
  const uint32_t c_lo = static_cast<uint32_t>(static_cast<uint64_t>(C) * g / G);
  const uint32_t c_hi = static_cast<uint32_t>(static_cast<uint64_t>(C) * (g + 1u) / G);
  if (c_lo >= c_hi) return;
  load_image(image, w, l);
  lds_st_sync(PsCutAddr(w, l), 0u);  // (the image load left the aux column zero; to be sure)
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
  const uint32_t cut_addr = PsCutAddr(w, l);

  // ---- desk state (lane j: span d0 + j) ----
  // relative addresses: byte offsets from the chunk's first window W0
  uint32_t a32 = 0, b32 = 0;   // span [a32, b32)
  uint32_t hw = 0;             // the head word as the stream needs it: bytes before A zeroed,
                               // the head register ~init * x^(-8 h) XORed in
  uint32_t pe = 0;             // E4 of the previous stream span (start of this one's pre-gap)
  uint32_t tw = 0;             // tail word (bytes [E4, E4 + 4) of memory)
  uint32_t in_r = 0, f_r = 0;  // IN and F at the span's cut
  uint32_t tk = 0;             // t (words in the cut stripe) | k << 8 | stream << 12 | cut seen << 13
  uint32_t id = 0;
  uint32_t dn = 0;             // uniform: spans in the desk

  for (;;) {
    // ---- the next chunk of the workgroup ----
    uint32_t cc = 0;
    if (l == 0u) cc = lds_add(MiscAddr(kMiscUnit), 1u);
    cc = uni(cc) + c_lo;
    if (cc >= c_hi) break;
    const uint32_t s_lo = uni(first[cc]), s_hi = uni(first[cc + 1u]);
    if (s_lo >= s_hi) continue;
    const uint64_t a_first = sbase + src.off[s_lo];
    const uint64_t b_last = sbase + src.off[s_hi - 1u] + src.len[s_hi - 1u];
    const uint64_t W0 = a_first & ~uint64_t(4095);
    const uint32_t wend = static_cast<uint32_t>(((b_last + 4095u) & ~uint64_t(4095)) - W0);
    // the first window's DMA right away (the desk loads go out behind it)
    {
      const uint32_t o = 16u * pp.cm;
      dma4(W0, pp.slot, o, o + 1024u, o + 2048u, o + 3072u);
    }
    uint32_t d0 = s_lo;
    uint32_t pe_carry = 0;  // E4 of the last stream span before the desk
    uint32_t pe_end = 0;    // E4 of the chunk's last stream span (valid once its desk is in)
    bool last_desk = false;
    uint32_t carry = 0;

    // loads one desk at d0 and prepares its lanes (short / empty spans are
    // answered here); called with nothing pending but the window DMA
    auto load_desk = [&]() {
      dn = umin(kPsDesk, s_hi - d0);
      last_desk = d0 + dn == s_hi;
      const bool v = l < dn;
      uint64_t a = 0;
      uint32_t n = 0, iv = 0;
      if (v) src.lane(d0 + l, a, n, iv);
      wait_vm<0>();
      loads_landed(a);
      loads_landed(n);
      loads_landed(iv);
      const uint64_t A = sbase + a;
      a32 = v ? static_cast<uint32_t>(A - W0) : wend;
      b32 = v ? a32 + n : wend;
      id = d0 + l;
      const bool stream = v && n >= kPsMinStream;
      const uint32_t e4 = b32 & ~3u, hd = a32 & ~3u;
      // the previous stream span's E4 (exclusive max over the lanes before)
      const uint32_t incl = scan_max(stream ? e4 : 0u);
      const uint32_t pb = bperm(incl, l == 0u ? 0u : l - 1u);  // (every lane: a wave op)
      const uint32_t before = l == 0u ? 0u : pb;
      pe = umax(before, pe_carry);
      if (last_desk) pe_end = umax(pe_carry, rdlane(incl, 63));
      const uint32_t inj = head_register_lane(l, stream ? iv : 0u, a32 - hd);
      tk = (stream ? 1u << 12 : 0u) | ((b32 & 3u) << 8);
      in_r = f_r = 0;
      // tail word: the aligned word holding bytes [E4, B) (in the span's page)
      tw = 0;
      if (stream && (b32 & 3u) != 0u) {
        tw = *reinterpret_cast<const uint32_t*>(W0 + e4);
      }
      // the head word from memory too (so the page's fix-up is one write)
      hw = 0;
      if (stream) hw = *reinterpret_cast<const uint32_t*>(W0 + hd);
      hw = (hw & ~low_bytes(a32 - hd)) ^ inj;
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
    };
    load_desk();

    // the deferred end of every stream span of the desk whose cut is done
    // (lanes in `done`): R = IN * x^(32 t) ^ F, the tail, ~, Mask, store
    auto finish = [&](uint64_t done) {
      const bool me = ((done >> l) & 1u) != 0u;
      const uint32_t t = tk & 31u;
      uint32_t r = in_r;
      for (uint32_t i = 0; i < 16u; ++i) {
        const bool go = me && i < t;
        if (ballot(go) == 0u) break;
        const uint32_t x = step(lk, r, 0u);
        r = go ? x : r;
      }
      r ^= f_r;
      r = tail_step(lk, r, tw, (tk >> 8) & 3u);
      const uint32_t crc = ~r;
      if (me) out32[id] = msk ? mask_crc(crc) : crc;
    };

    for (uint32_t wr = 0; wr < wend; wr += 4096u) {
      // ---- a new desk when the window may hold spans past this one ----
      if (!last_desk && uni(rdlane(a32, dn - 1u)) < wr + 4096u) {
        // the desk's spans that are done: a stream span once its cut is
        // behind the window (its tail word is in a register), any other
        // once its bytes are (answered at its desk's load) -- a prefix, the
        // spans being ordered
        const bool st = l < dn && ((tk >> 12) & 1u) != 0u;
        const bool done = l < dn && (st ? (b32 & ~3u) <= wr : b32 <= wr);
        const uint32_t ngone = static_cast<uint32_t>(__builtin_popcountll(ballot(done)));
        finish(ballot(done && st));
        pe_carry = umax(pe_carry, rdlane(scan_max(done && st ? (b32 & ~3u) : 0u), 63));
        if (ngone == 0u) {  // (cannot happen in a checked batch: at most 63 spans meet a window)
          report_fault(fault, kFaultPsDesk);
          return;
        }
        d0 += ngone;
        load_desk();
      }
      // ---- the window's fix-ups, planned before it lands (the stretch from
      // its arrival to the next DMA's issue is kept to the LDS work) ----
      const uint32_t wrel_end = wr + 4096u;
      const bool stream = l < dn && ((tk >> 12) & 1u) != 0u;
      const uint32_t e4 = b32 & ~3u, hd = a32 & ~3u;
      // pre-gap [pe, hd) of the span (trailers, other spans' bytes)
      uint32_t z0 = umax(pe, wr), z1 = umin(hd, wrel_end);
      if (!stream) z0 = z1 = 0;
      const bool gaps = ballot(z0 < z1) != 0u;
      // after the chunk's last stream span: zeroed by every lane
      const uint32_t p0 = last_desk ? umax(pe_end, wr) : wrel_end;
      // head word: bytes before A masked, the head register injected
      const bool head = stream && hd >= wr && hd < wrel_end;
      const uint32_t head_a = ps_lds_addr(pp.slot, (hd - wr) & 4095u);
      // cut: the stripe of the last stream word
      const bool cut = stream && e4 > wr && e4 <= wrel_end;
      const uint32_t cq = (e4 - 4u - wr) >> 2;
      const uint32_t cut_a = PsCutAddr(w, (cq >> 4) & 63u);
      wait_vm<0>();
      loads_landed(tw);
      loads_landed(hw);
      // the window has landed: this wave issues ahead of the others' compute
      // until its next DMA is out (as run_lp / run_ea do)
      if constexpr (kPrio != 0) lk_prio<kPrio>();
      if (gaps) {
        for (;;) {
          const bool more = z0 < z1;
          if (more) lds_st(ps_lds_addr(pp.slot, z0 - wr), 0u);
          z0 += 4u;
          if (ballot(z0 < z1) == 0u) break;
        }
      }
      for (uint32_t p = p0 + 4u * l; p < wrel_end; p += 256u) lds_st(ps_lds_addr(pp.slot, p - wr), 0u);
      if (head) lds_st(head_a, hw);
      if (cut) lds_st(cut_a, ((cq & 15u) + 1u) | (l << 8));
      lds_order();  // the fix-ups, then the lanes' reads of the window and the table
      const uint32_t ce = lds_ld(cut_addr);
      uint32_t W[16];
      pp.read(W);
      pp.release();
      // ---- the next window's DMA ----
      if (wrel_end < wend) {
        const uint32_t o = 16u * pp.cm;
        dma4(W0 + wrel_end, pp.slot, o, o + 1024u, o + 2048u, o + 3072u);
      }
      if constexpr (kPrio != 0) lk_prio<0>();
      lds_st(cut_addr, 0u);  // (read above; the next window's marks come after)
      // ---- the scan ----
      const uint32_t te = ce & 31u;
      W[0] ^= l == 0u ? carry : 0u;
      const uint64_t cutm = ballot(te != 0u);
      if (cutm == 0u) {
        // no span ends in this window (long spans' middles): the plain scan
        // and the whole-window fold carry the open span on
        carry = fold<1>(lk, l, scan(lk, W))[0];
        continue;
      }
      // cut once at te
      uint32_t x = W[0], fr = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t a0 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[0]));
        const uint32_t a1 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[1]));
        const uint32_t a2 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[2]));
        const uint32_t a3 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[3]));
        const uint32_t y = xor3(a0, a1, a2) ^ a3;  // register after word i
        const bool cut = te == static_cast<uint32_t>(i + 1);
        fr = cut ? y : fr;
        const uint32_t keep = cut ? 0u : y;
        x = i < 15 ? keep ^ W[i + 1 < 16 ? i + 1 : 15] : keep;
      }
      const uint32_t o_r = x;  // the register at the stripe's end (0 after a cut at word 15)
      // ---- the window's segments ----
      const uint64_t above = l == 63u ? 0u : (cutm >> (l + 1u)) << (l + 1u);
      const uint32_t nxt = above ? static_cast<uint32_t>(__builtin_ctzll(above)) : 64u;
      const uint32_t v = shift64(lk, k1b, k2b, o_r, nxt - 1u - l);
      const uint32_t qx = scan_xor(v);
      const uint64_t below = cutm & ((uint64_t(1) << l) - 1u);
      const uint32_t prv = below ? 63u - static_cast<uint32_t>(__builtin_clzll(below)) : ~0u;
      const uint32_t q1 = bperm(qx, l == 0u ? 0u : l - 1u);
      const uint32_t q2 = bperm(qx, prv == ~0u || prv == 0u ? 0u : prv - 1u);
      const uint32_t in_l = (l == 0u ? 0u : q1) ^ (prv == ~0u || prv == 0u ? 0u : q2);
      // carry: the last segment, to the window's end
      {
        const uint32_t plast = 63u - static_cast<uint32_t>(__builtin_clzll(cutm));
        const uint32_t q63 = rdlane(qx, 63);
        const uint32_t qp = plast == 0u ? 0u : rdlane(qx, plast - 1u);
        carry = q63 ^ qp;
      }
      // ---- desk lanes whose span was cut here take IN and F ----
      {
        const bool mine = cut;
        const uint32_t q = cq;
        const uint32_t src_l = mine ? q >> 4 : l;
        const uint32_t gi = bperm(in_l, src_l), gf = bperm(fr, src_l);
        if (mine) {
          in_r = gi;
          f_r = gf;
          tk = (tk & ~31u) | ((q & 15u) + 1u) | (1u << 13);
        }
      }
    }
    // ---- the chunk's end: every stream span of the last desk ----
    finish(ballot(l < dn && ((tk >> 12) & 1u) != 0u));
  }
}

}  // namespace lk
}  // namespace wipdb
