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
// A stream span [a, b) (>= 96 bytes) is its STREAM CHUNKS [H16 = a & ~15,
// E16 = b & ~15) -- 16-byte chunks of the page -- plus a tail of b - E16 < 16
// bytes, which the desk lane loads from memory and feeds at the end.  Its
// boundaries become two events of the scan, both at chunk boundaries:
//
//   RESET  the desk lane rewrites the span's head chunk in the page (bytes
//          before a zeroed, ~init * x^(-8 (a - H16)) XORed into its first
//          word: one ds_write_b128), and the lane of the stripe holding it
//          starts that chunk from register 0;
//   CUT    the lane of the stripe holding the span's last chunk keeps the
//          register after it (F) and goes on from 0.
//
// Bytes between a cut and the next reset -- trailers, short spans, a chunk's
// front -- are never zeroed: what they leave in the registers reaches no
// segment.  The desk hands each page's events to their stripes' lanes before
// the page lands (v_writelane for one or two; else the OR of the event
// stripes, each lane's rank among them (mbcnt) and one ds_bpermute from the
// desk's stream spans in rank order, laid out once per desk by ds_permute).
// Per page:
//
//   O_l   the register at the end of stripe l (from its reset, or from 0
//         after a cut),
//   IN_L  for a cut lane L: the register entering stripe L of its span =
//         XOR over the lanes l from its reset stripe R (or the page's start)
//         to L - 1 of O_l * x^(8 * 64 (L - 1 - l)) -- each lane shifts its O
//         by whole stripes to the next cut (the two fold-table levels,
//         shift64) and one wave prefix XOR q gives IN_L = q[L-1] ^ q[R-1]
//         (the reference's CombineCRC identity, kv/src/util/crc32c.cc:640-657,
//         at stripe granularity),
//   carry the register of the span open at the page's end (from the last
//         reset), XORed into word 0 of the next page by lane 0.
//
// A page with no event but a reset at its start and a cut at its end (long
// spans' middles, aligned blocks) takes the plain scan and the whole-page
// fold.  The register at a span's end is IN * x^(32 t) ^ F (t = its words in
// the cut stripe) -- a per-span shift of 4 .. 16 words, deferred to the
// desk's end, when all its lanes run it at once, then the tail, ~, Mask and
// the store.  Spans of fewer than 96 bytes (and empty ones) are not in the
// stream: the desk lane computes them from memory (rare: a table's
// metaindex block).
//
// Work: the pre-pass (ps_index_kernel) checks the batch (sorted, no overlap,
// gaps < 4 KiB, at most 62 spans starting in any 4 KiB, no run of 8 spans
// under 96 bytes nor 32 among 64 -- WAL records, which run_lp does faster)
// and cuts the covering range into C equal byte chunks, first[c] = the first
// span starting in chunk c: one chunk per wave (C = 16 per workgroup); a chunk is its
// spans, whole.  The SIMDs issue oldest-first, which on equal shares makes a
// wave's speed its age (the last wave of a SIMD up to 15 % behind the first):
// every 4 pages a wave compares its pages with its workgroup's and takes a
// priority by how many are ahead.  A batch that fails the check runs the
// default pipelines instead: HCRC_PACKED is a promise the kernel verifies,
// never a way to a wrong CRC.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// crc32c.cc:1225-1227) per block span, as WriteRawBlock
// (kv/src/table/table_builder.cc:194-196) applies it.
#pragma once
#include <stdint.h>

#include "crc32c_dev.h"

namespace wipdb {
namespace lk {

#ifndef WIPDB_PS_PRIO
#define WIPDB_PS_PRIO 3
#endif
constexpr int kPsPrio = WIPDB_PS_PRIO;  // wave priority from a page's landing to its next DMA
constexpr uint32_t kPsDesk = 64;        // spans per desk (one per lane)
constexpr uint32_t kPsMinStream = 96;   // spans shorter than this are computed off the stream
                                        // (a stream span's stream part is then >= 64 bytes)
constexpr uint32_t kPsMaxGap = 4096;    // a larger gap could leave a page of no span's bytes
constexpr uint32_t kPsDense = 62;       // spans i, i + 62 start >= 4 KiB apart
constexpr uint32_t kPsShortRun = 8;     // this many short spans in a row: not for run_ps
constexpr uint32_t kPsDenseBytes = 1600;  // a desk of spans shorter on average plans a page ahead

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

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
// Thread i handles span i (grid-stride, a wave's 64 spans consecutive);
// first[] written where the chunk index steps (first has C + 1 entries,
// first[C] = n).  The verdict word meta[0] is tagged with the launch's
// epoch (its stream's count of packed launches): thread 0 raises it to
// epoch << 4, a workgroup that finds the batch broken to epoch << 4 |
// kPsBad* (and its waves stop there), so it needs no clearing between
// launches (a stale word is an older epoch, lower).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ps_index(const uint8_t* base, const uint64_t* off,
                                         const uint32_t* len, uint64_t n, uint32_t C,
                                         uint32_t* first, uint32_t* meta, uint64_t tid,
                                         uint64_t nthreads, uint32_t epoch) {
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
  // the chunk of address a: (a - lo) / cb in 32 bits (cb is whole pages;
  // the page index of any address of a device buffer fits, one that does
  // not is past the range: C, broken).  (Cheaper than the 64-bit division;
  // the pass's time did not move, profiles/r05ar_wal_kernels.txt r05as.)
  const uint32_t cbp = static_cast<uint32_t>(cb >> 12);
  auto chunk_of = [lo, cbp, C](uint64_t a) -> uint64_t {
    if (a < lo) return 0u;
    const uint64_t v = (a - lo) >> 12;
    return (v >> 32) ? uint64_t(C) : uint64_t(static_cast<uint32_t>(v) / cbp);
  };
  // a wave takes 64 consecutive spans a step, kPsIndexSteps steps an
  // iteration with all their loads issued first (the pass is latency-bound:
  // 21 -> 16 us on 3.5 Mi spans, 71 -> 42 us on 21 Mi); the trip count
  // is wave-uniform, so the ballots below see every lane.  Chunks of 16 TiB
  // and more (no device holds such a batch) would not divide in 32 bits:
  // broken.
  constexpr uint32_t U = kPsIndexSteps;
  uint32_t bad = (cb >> 44) ? kPsBad : 0u;
  for (uint64_t w0 = tid & ~uint64_t(63); w0 < n; w0 += U * nthreads) {
    uint64_t A[U], AP[U], AD[U];
    uint32_t LP[U], L[U];
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) {
      const uint64_t i = w0 + j * nthreads + (tid & 63u);
      A[j] = AP[j] = AD[j] = 0;
      LP[j] = L[j] = 0;
      if (i < n) {
        A[j] = off[i];
        L[j] = len[i];
        if (i > 0) {
          AP[j] = off[i - 1];
          LP[j] = len[i - 1];
        }
        if (i + kPsDense < n) AD[j] = off[i + kPsDense];
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) {
      const uint64_t i = w0 + j * nthreads + (tid & 63u);
      bool shrt = false;
      if (i < n) {
        const uint64_t a = A[j];
        uint64_t c = chunk_of(a);
        if (a < lo || c >= C) {
          bad |= kPsBad;
          c = C - 1u;
        }
        uint64_t cp = 0;  // chunks (cp, c] start at span i
        if (i == 0) {
          first[0] = 0;
        } else {
          const uint64_t ap = AP[j], bp = ap + LP[j];
          if (a < bp || a - bp >= kPsMaxGap) bad |= kPsBad;
          cp = chunk_of(ap);
          if (cp > c) cp = c;
        }
        for (uint64_t k = cp + 1u; k <= c; ++k) first[k] = static_cast<uint32_t>(i);
        // run_ps keeps a chunk's positions in 32 bits from the page of its
        // first span (W0 >= the chunk's start - 4095): a span starting in the
        // chunk ends before W0 + cb + 4096 + len, rounded up to a page -- it
        // must stay below 2^32 (a span of ~4 GiB not on the
        // chunk's first page would wrap)
        if (cb + L[j] + 8192u >= (uint64_t(1) << 32)) bad |= kPsBad;
        if (i + kPsDense < n && AD[j] - a < 4096u) bad |= kPsBadDense;
        if (i + kPsDense < n && AD[j] < a) bad |= kPsBad;
        if (i == n - 1)
          for (uint64_t k = c + 1u; k <= C; ++k) first[k] = static_cast<uint32_t>(n);
        shrt = L[j] < kPsMinStream;
      }
      // a run of kPsShortRun short spans among the step's 64 (bit b of m:
      // spans b..b+7 all short; a run across two steps may go unseen -- the
      // verdict is a speed choice, every pipeline computes short spans
      // exactly).  One ballot, no loads: a per-span look-ahead loop cost
      // 150 us on 20 Mi spans (profiles/r05ar_wal_kernels.txt).
      static_assert(kPsShortRun == 8, "the run test below is three shift-ANDs");
      uint64_t m = ballot(shrt);
      // (or half the step's spans short: WAL records of 64..127 B rarely
      // make a run of 8, and the look stops at the first step)
      if (__builtin_popcountll(m) >= 32) bad |= kPsBadShort;
      m &= m >> 1;
      m &= m >> 2;
      m &= m >> 4;
      if (m) bad |= kPsBadShort;
    }
    if (ballot(bad != 0u)) break;  // (broken: first[] goes unread, the verdict is raised below)
  }
  (void)base;
  // one atomic per workgroup: a broken batch of tiny spans has every thread
  // of the grid find it so, and same-word device atomics serialize (~11 ns
  // each: 512 Ki of them took 6 ms, 8 Ki 98 us -- profiles/r05ao_wal_ab.log,
  // r05ar_wal_kernels.txt).  The waves' ORs (ballot per bit) meet in LDS words
  // 0..15 (the kernel's 64 bytes), thread 0 raises the verdict.
  uint32_t w = 0;
  for (uint32_t b = 1u; b <= (kPsBad | kPsBadDense | kPsBadShort); b <<= 1)
    if (ballot((bad & b) != 0u)) w |= b;
  const uint32_t t = lane_tid();
  if ((t & 63u) == 0u) lds_st_sync((t >> 6) * 4u, w);
  wg_sync();
  if (t == 0) {
    for (uint32_t k = 1; k < kPsIndexThreads / 64u; ++k) w |= lds_ld_sync(k * 4u);
    if (w != 0u || tid == 0) global_max(meta, (epoch << 4) | w);
  }
}

// A page's events to the lanes of their stripes: the lanes with `ev`
// (consecutive: the desk's stream spans in rank order, below) each hand
// `val` (nonzero) to lane `stripe` (distinct, increasing with the lane);
// the others get 0.  The OR of the event stripes (DPP), each stripe lane's
// rank among them (mbcnt) and one ds_bpermute: no branch, so the page loop
// runs it for the next page inside this page's scan (a latency chain beside
// another).
// The same for pages of few events (desks of long spans): v_writelane for one
// or two, the general form for more -- cheaper per page, but a branch, so
// it runs in the page's own turn, not inside the previous page's scan.
__device__ __forceinline__ uint32_t ps_deliver(uint32_t l, bool ev, uint32_t stripe, uint32_t val);
__device__ __forceinline__ uint32_t ps_deliver_few(uint32_t l, bool ev, uint32_t stripe, uint32_t val) {
  const uint64_t m = ballot(ev);
  if (m == 0u) return 0u;
  if (__builtin_popcountll(m) <= 2) {
    uint32_t r = 0;
    for (uint64_t e = m; e != 0u; e &= e - 1u) {
      const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(e));
      r = wrlane(r, rdlane(val, j), rdlane(stripe, j));
    }
    return r;
  }
  return ps_deliver(l, ev, stripe, val);
}
__device__ __forceinline__ uint32_t ps_deliver(uint32_t l, bool ev, uint32_t stripe, uint32_t val) {
  const uint64_t m = ballot(ev);
  const uint32_t lo = scan_or(ev && stripe < 32u ? 1u << stripe : 0u);
  const uint32_t hi = scan_or(ev && stripe >= 32u ? 1u << (stripe - 32u) : 0u);
  const uint32_t k = mbcnt_hi(hi, mbcnt_lo(lo, 0u));  // event stripes below the lane
  const uint32_t j = (m != 0u ? static_cast<uint32_t>(__builtin_ctzll(m)) : 0u) + k;
  const uint32_t v = bperm(val, j & 63u);
  const bool mine = ((l < 32u ? lo >> l : hi >> (l - 32u)) & 1u) != 0u;
  return mine ? v : 0u;
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
  // the wave's progress word (pages done), read by the others (below)
  const uint32_t prog_addr = MiscAddr(kMiscPsProgress + w);
  lds_st_sync(prog_addr, 0u);
  load_image(image, w, l);  // (its barrier: every progress word is 0 before any is read)
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
  // A stream span [a, b) is its stream chunks [H16 = a & ~15, E16 = b & ~15)
  // and a tail of k16 = b - E16 < 16 bytes (loaded from memory with the
  // desk).  Its head chunk is rewritten in the page (bytes before a zeroed,
  // ~init * x^(-8 (a - H16)) XORed in) and the scan of the stripe holding it
  // starts that chunk from register 0 (a RESET); the stripe holding its last
  // chunk keeps the register after it (F) and starts again from 0 (a CUT).
  // Bytes between a cut and the next reset (trailers, short spans, a chunk's
  // front) are never zeroed: what they leave in the registers no segment uses.
  uint32_t a32 = 0, b32 = 0;      // span [a32, b32)
  uint32_t hb = 0, inj = 0;       // its head chunk's leading bytes before a, the head register
  u32x4 tt{0, 0, 0, 0};           // its tail chunk [E16, E16 + 16)
  uint32_t in_r = 0, f_r = 0;     // IN and F at its cut
  uint32_t hwin = 0, cwin = 0;    // the pages (relative indices) of its head chunk and its cut
  uint32_t twin = ~0u;            // the page its tail chunk is read from in LDS (~0: none)
  uint32_t ha = 0, ta = 0;        // the LDS addresses of its head and tail chunks in the slot
  uint32_t cs = 0;                // cut stripe
  uint32_t cv = 0;                // tc: the cut after stripe chunk tc - 1 (1..4)
  // the page events of the desk's stream spans in rank order (lane r: the
  // r-th stream span; then the others): page << 12 | stripe << 3 | value,
  // value = tc for a cut, reset boundary + 1 for a head; ~0 for none
  uint32_t cev = ~0u, hev = ~0u;
  bool sstream = false;           // a stream span
  uint32_t id = 0;
  uint32_t pages = 0;   // pages done (all chunks)
  uint32_t behind = 0;  // the wave's priority outside a page's landing: waves ahead of it / 4
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
  // profiling build: 0 wait, 1 landed -> next DMA out, 2 compute, 3 desk
  // loads, 4 pages, 5 pages with a cut, 6 plan, 7 life, 8 finish,
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
    const uint32_t s_lo = uni(first[cc]), s_hi = uni(first[cc + 1u]);
    if (s_lo >= s_hi) continue;
    LP_ACC(9, 1);
    const uint64_t a_first = sbase + src.off[s_lo];
    const uint64_t b_last = sbase + src.off[s_hi - 1u] + src.len[s_hi - 1u];
    const uint64_t W0 = a_first & ~uint64_t(4095);
    const uint32_t wend = static_cast<uint32_t>(((b_last + 4095u) & ~uint64_t(4095)) - W0);
    // the first window's DMA right away (the desk loads go out behind it;
    // none when the chunk is empty spans at a page-aligned end)
    if (wend != 0u) dma4(W0, pp.slot, dma_o, dma_o + 1024u, dma_o + 2048u, dma_o + 3072u);
    uint32_t d0 = s_lo, dn = 0;
    bool last_desk = false;
    uint32_t carry = 0;
    uint32_t wr = 0;
    // a desk's descriptors, loaded ahead: the first desk's here (behind the
    // first page's DMA), each next one's before the previous desk's
    // deferred span ends run
    uint64_t nx_a = 0;
    uint32_t nx_n = 0, nx_iv = 0;
    auto load_desc = [&]() {
      if (l < umin(kPsDesk, s_hi - d0)) src.lane(d0 + l, nx_a, nx_n, nx_iv);
    };
    load_desc();

    // the deferred end of the stream spans of the desk whose cut is done
    // (lanes in `done`): R = IN * x^(32 t) ^ F (t = 4 tc words), the tail's
    // k16 bytes, ~, Mask, store
    auto finish = [&](uint64_t done) {
      const bool me = ((done >> l) & 1u) != 0u;
      const uint32_t t = 4u * cv;
      uint32_t r = in_r;
      for (uint32_t i = 0; i < 16u; ++i) {
        const bool go = me && i < t;
        if (ballot(go) == 0u) break;
        const uint32_t x = step(lk, r, 0u);
        r = go ? x : r;
      }
      r ^= f_r;
      const uint32_t k16 = b32 & 15u, kw = k16 >> 2;
      if (ballot(me && kw >= 1u) != 0u) {
        const uint32_t t0 = step(lk, r ^ tt.x, 0u);
        r = kw >= 1u ? t0 : r;
      }
      if (ballot(me && kw >= 2u) != 0u) {
        const uint32_t t1 = step(lk, r ^ tt.y, 0u);
        r = kw >= 2u ? t1 : r;
      }
      if (ballot(me && kw >= 3u) != 0u) {
        const uint32_t t2 = step(lk, r ^ tt.z, 0u);
        r = kw >= 3u ? t2 : r;
      }
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
        wait_vm<0>();
        loads_landed(nx_a);
        loads_landed(nx_n);
        loads_landed(nx_iv);
        const uint64_t a = v ? nx_a : 0u;
        const uint32_t n = v ? nx_n : 0u, iv = v ? nx_iv : 0u;
        a32 = v ? static_cast<uint32_t>(sbase + a - W0) : wend;
        b32 = v ? a32 + n : wend;
        id = d0 + l;
        const bool stream = v && n >= kPsMinStream;
        sstream = stream;
        const uint32_t e16 = b32 & ~15u, h16 = a32 & ~15u;
        hb = a32 - h16;
        inj = head_register_lane(l, stream ? iv : 0u, hb);
        in_r = f_r = 0;
        // the page events: head chunk (a reset), last chunk (a cut)
        const uint32_t lc = e16 - 16u;
        hwin = stream ? h16 >> 12 : ~0u;
        cwin = stream ? lc >> 12 : ~0u;
        ha = ps_lds_addr(pp.slot, h16 & 4095u);
        cs = (lc & 4095u) >> 6;
        cv = ((lc & 63u) >> 4) + 1u;
        {
          const uint64_t sm = ballot(stream);
          const uint32_t nst = static_cast<uint32_t>(__builtin_popcountll(sm));
          const uint32_t rk = stream ? mbcnt_hi(static_cast<uint32_t>(sm >> 32), mbcnt_lo(static_cast<uint32_t>(sm), 0u))
                                     : nst + mbcnt_hi(static_cast<uint32_t>(~sm >> 32), mbcnt_lo(static_cast<uint32_t>(~sm), 0u));
          cev = fperm(stream ? (lc >> 12) << 12 | cs << 3 | cv : ~0u, rk);
          hev = fperm(stream ? (h16 >> 12) << 12 | ((h16 & 4095u) >> 6) << 3 | (((h16 & 63u) >> 4) + 1u) : ~0u, rk);
        }
        // head and tail chunks: read from the page in LDS when it lands
        // (below), not from memory -- a desk's global loads of them were a
        // round trip on every desk and 128-byte lines beside the page stream
        // (the packed 512 B bucket read 1.23 x its bytes, profiles/
        // r06g_traffic.json).  A tail chunk that starts a page belongs to a
        // span finished before that page lands: that one comes from memory.
        ta = ps_lds_addr(pp.slot, e16 & 4095u);
        const bool tail = stream && (b32 & 15u) != 0u;
        twin = tail && (e16 & 4095u) != 0u ? e16 >> 12 : ~0u;
        tt = u32x4{0, 0, 0, 0};
        if (tail && (e16 & 4095u) == 0u) tt = *reinterpret_cast<const u32x4*>(W0 + e16);
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
      // a page's events to their stripes' lanes (rz: reset before chunk
      // rz - 1, 0 = none; tc: cut after chunk tc - 1, 0 = none).  A desk of
      // short spans (many events a page) plans each next page inside the
      // page before (the branch-free form, its latency beside the scan's);
      // one of long spans plans each page in its own turn (v_writelane)
      const bool dense =
          uni(rdlane(b32, dn - 1u)) - uni(rdlane(a32, 0u)) < dn * kPsDenseBytes;
      auto page_loop = [&](auto kDense) {
      constexpr bool D = decltype(kDense)::value;
      auto plan = [&](uint32_t wi, uint32_t& tcp, uint32_t& rzp) {
        if constexpr (D) {
          tcp = ps_deliver(l, cev != ~0u && (cev >> 12) == wi, (cev >> 3) & 63u, cev & 7u);
          rzp = ps_deliver(l, hev != ~0u && (hev >> 12) == wi, (hev >> 3) & 63u, hev & 7u);
        } else {
          tcp = ps_deliver_few(l, cev != ~0u && (cev >> 12) == wi, (cev >> 3) & 63u, cev & 7u);
          rzp = ps_deliver_few(l, hev != ~0u && (hev >> 12) == wi, (hev >> 3) & 63u, hev & 7u);
        }
      };
      uint32_t tc_n = 0, rz_n = 0;
      if constexpr (D) plan(wr >> 12, tc_n, rz_n);
      for (; wr < wstop; wr += 4096u, ++pages) {
        // ---- the page's events (a dense desk planned them a page ahead) ----
        LP_T(p0);
        const uint32_t wi = wr >> 12;
        const bool head = hwin == wi;
        const bool cut = cwin == wi;
        if constexpr (!D) plan(wi, tc_n, rz_n);
        const uint32_t tc = tc_n, rz = rz_n;
        LP_T(w0);
        LP_ACC(6, w0 - p0);
        wait_vm<0>();
        LP_T(w1);
        LP_ACC(0, w1 - w0);
        LP_ACC(4, 1);
        // the page has landed: this wave issues ahead of the others' compute
        // until its next DMA is out (as run_lp does)
        if constexpr (kPsPrio != 0) lk_prio<kPsPrio>();
        // the tail chunks in this page (as DMA'd: read before any head is
        // rewritten -- a span's tail chunk may be the next one's head chunk),
        // then the head chunks in their stream form: the bytes before a
        // zeroed, the head register XORed into its first word
        const bool tl = twin == wi;
        if (ballot(head || tl) != 0u) {
          u32x4 hc{0, 0, 0, 0}, tv{0, 0, 0, 0};
          if (head) hc = lds_ld4(ha);
          if (tl) tv = lds_ld4(ta);
          lgkm_wait();
          if (tl) tt = tv;
          if (head) {
            hc.x = (hb >= 4u ? 0u : hc.x & ~low_bytes(hb)) ^ inj;
            hc.y = hb >= 8u ? 0u : (hb <= 4u ? hc.y : hc.y & ~low_bytes(hb - 4u));
            hc.z = hb >= 12u ? 0u : (hb <= 8u ? hc.z : hc.z & ~low_bytes(hb - 8u));
            hc.w = hb <= 12u ? hc.w : hc.w & ~low_bytes(hb - 12u);
            lds_st4(ha, hc);
          }
        }
        lds_order();  // the head chunks, then the lanes' reads of the page
        uint32_t W[16];
        pp.read(W);
        pp.release();
        // ---- the next page's DMA ----
        if (wr + 4096u < wend) dma4(W0 + wr + 4096u, pp.slot, dma_o, dma_o + 1024u, dma_o + 2048u, dma_o + 3072u);
        if constexpr (kPsPrio != 0) {
          if (behind == 0u) lk_prio<0>();
          else if (behind == 1u) lk_prio<1>();
          else if (behind == 2u) lk_prio<2>();
          else lk_prio<3>();
        }
        LP_T(w2);
        LP_ACC(1, w2 - w1);
        // ---- progress: every 4 pages the wave compares its pages with its
        // workgroup's other waves and takes a priority by how many are ahead
        // (the SIMDs' oldest-first issue otherwise makes a wave's speed its
        // age: up to 15 % between the first and the last wave of a SIMD on
        // equal byte shares) ----
        if ((pages & 3u) == 3u) {
          if (l == 0u) lds_st_sync(prog_addr, pages);
          const uint32_t pv = l < static_cast<uint32_t>(kWaves) ? lds_ld_sync(MiscAddr(kMiscPsProgress + l)) : 0u;
          const uint32_t ahead = static_cast<uint32_t>(
              __builtin_popcountll(ballot(l < static_cast<uint32_t>(kWaves) && pv > pages)));
          behind = umin(3u, ahead * 4u / static_cast<uint32_t>(kWaves));
        }
        // ---- the scan ----
        const uint64_t cutm = ballot(tc != 0u), resm = ballot(rz != 0u);
        // lane 0's register enters from the previous page unless a span
        // starts at the page (a reset before its chunk 0)
        const bool r0 = (resm & 1u) != 0u && rdlane(rz, 0) == 1u;
        W[0] ^= l == 0u && !r0 ? carry : 0u;
        const bool at_end = cutm == (uint64_t(1) << 63) && rdlane(tc, 63) == 4u;
        if ((cutm == 0u || at_end) && (resm == 0u || (resm == 1u && r0))) {
          // no span ends in this page but at its end (aligned blocks) and
          // none starts but at its start: the plain scan and the whole-page
          // fold give the open span's register at the page's end
          if constexpr (D) plan(wi + 1u, tc_n, rz_n);
          const uint32_t r = fold<1>(lk, l, scan(lk, W))[0];
          carry = at_end ? 0u : r;
          if (at_end && cut) {
            in_r = r;
            f_r = 0;
            cv = 0;  // (no words after IN)
          }
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
          LP_T(w3);
          LP_ACC(2, w3 - w2);
#endif
          continue;
        }
        if constexpr (D) plan(wi + 1u, tc_n, rz_n);
        uint32_t x = W[0], fr = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t a0 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[0]));
          const uint32_t a1 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[1]));
          const uint32_t a2 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[2]));
          const uint32_t a3 = lds_ld(kLdsMain + vperm(lk.km, x, lk.sel[3]));
          uint32_t y = xor3(a0, a1, a2) ^ a3;  // the register after word i
          if ((i & 3) == 3) {  // a chunk's end: a cut, a reset may be here
            const bool c = tc == static_cast<uint32_t>((i >> 2) + 1);
            fr = c ? y : fr;
            y = c || rz == static_cast<uint32_t>((i >> 2) + 2) ? 0u : y;
          }
          x = i < 15 ? y ^ W[i + 1 < 16 ? i + 1 : 15] : y;
        }
        // (a reset before chunk 0 of lanes > 0: their register from the
        // previous stripes is left out below, as the segment starts there)
        const uint32_t o_r = x;  // the register at the stripe's end
        // ---- the page's segments: a span's register enters its cut stripe
        // L from the stripes since its reset stripe R (or the page's start):
        // IN_L = XOR over l in [R, L) of O_l * x^(8 * 64 (L - 1 - l)) ----
        const uint64_t above = l == 63u ? 0u : (cutm >> (l + 1u)) << (l + 1u);
        const uint32_t nxt = above ? static_cast<uint32_t>(__builtin_ctzll(above)) : 64u;
        const uint32_t v = shift64(lk, k1b, k2b, o_r, nxt - 1u - l);
        const uint32_t qx = scan_xor(v);
        {  // desk lanes whose span was cut here (stripe L = cs, reset stripe
           // R): IN = q[L - 1] ^ q[R - 1], F from stripe L -- one exchange
          const uint64_t below = resm & ((uint64_t(1) << cs) - 1u);
          const uint32_t R = below ? 63u - static_cast<uint32_t>(__builtin_clzll(below)) : 0u;
          const uint32_t g1 = bperm(qx, cut && cs != 0u ? cs - 1u : l);
          const uint32_t g2 = bperm(qx, cut && R != 0u ? R - 1u : l);
          const uint32_t gf = bperm(fr, cut ? cs : l);
          if (cut) {
            in_r = (cs == 0u ? 0u : g1) ^ (R == 0u ? 0u : g2);
            f_r = gf;
          }
        }
        {  // the carry: the span open at the page's end, from its reset
           // stripe (a cut after the last reset: no span is open)
          const uint32_t plast = resm ? 63u - static_cast<uint32_t>(__builtin_clzll(resm)) : 0u;
          const uint32_t q63 = rdlane(qx, 63);
          const uint32_t qp = plast == 0u ? 0u : rdlane(qx, plast - 1u);
          carry = q63 ^ qp;
        }
        LP_ACC(5, 1);
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
        LP_T(w3);
        LP_ACC(2, w3 - w2);
#endif
      }
      };
      if (dense) page_loop(std::true_type{});
      else page_loop(std::false_type{});
      if (wr >= wend) break;
      // ---- the next desk: the spans done are a prefix (ordered spans): a
      // stream span once its cut is behind the page, any other once its
      // bytes are (answered at its desk's load) ----
      const bool done = l < dn && (sstream ? (b32 & ~15u) <= wr : b32 <= wr);
      const uint32_t ngone = static_cast<uint32_t>(__builtin_popcountll(ballot(done)));
      if (ngone == 0u) {  // (cannot happen in a checked batch: at most 63 spans meet a page)
        report_fault(fault, kFaultPsDesk);
        return;
      }
      d0 += ngone;
      load_desc();  // the next desk's descriptors, behind the deferred ends
      LP_T(f0);
      finish(ballot(done && sstream));
      LP_T(f1);
      LP_ACC(8, f1 - f0);
    }
    // ---- the chunk's end: every stream span of its last desk ----
    LP_T(f0);
    finish(ballot(l < dn && sstream));
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
