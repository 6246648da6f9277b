// crc32c_lds.hip -- hand-written CDNA4 (gfx950) kernels for batched CRC32C
// of WipDB table blocks, LDS-staged and lane-packed.
//
// Reference function: kv::crc32c::Extend (kv/src/util/crc32c.h:24,
// kv/src/util/crc32c.cc:1225-1227) applied to every block span, as
// TableBuilder::WriteRawBlock (kv/src/table/table_builder.cc:194-196) and
// ReadBlock (kv/src/table/format.cc:91-93) do one block at a time; the
// reference's hot loop is crc32c_3way (crc32c.cc:667-1198), which runs every
// length through one loop at one per-byte rate.  So does this kernel: one
// launch for any mix of sizes.
//
//   * persistent grid, one 16-wave workgroup per CU; a wave owns a 4 KiB LDS
//     slot that the next iteration's bytes are DMA'd into (4 x
//     global_load_lds_dwordx4, nontemporal) while it computes the current
//     one, and lane l CRCs the 64-byte stripe [64 l, 64 l + 64) of it
//     (slicing-by-4 on the rotated LDS tables, crc32c_dev.h);
//   * spans come in DESKS of 32 (one LDS atomic on the workgroup's unit
//     counter, the descriptors vector-loaded a desk ahead, one span per
//     lane), planned per lane (crc32c_plan.h): m full 4 KiB segments from
//     the start of the span's grid, then a back piece of the remaining
//     chunks (a span under 4 KiB is all piece);
//   * a span with segments goes to the WORKGROUP's long-span queue (LDS), so
//     the 16 waves share long spans one at a time (no wave is left holding a
//     desk of them); a wave takes one, runs its segments on consecutive
//     iterations chained by the register, and pushes its back piece;
//   * pieces queue in the wave's PIECE RING (one entry per lane: source,
//     piece word, entering register, output slot).  One iteration
//     checksums as many pieces as fit in its 64 lanes, each on ceil(chunks /
//     4) lanes -- the batch DMA takes every lane's source from the lane that
//     owns the stripe (ds_bpermute), the registers are folded per piece by a
//     per-lane shift of 64 (lanes after it) bytes and a segmented XOR scan,
//     and each piece's leader lane finishes its span (tail step, output).
//     A 512-byte span costs 9 lanes, not a 4 KiB window;
//   * every vector-memory instruction is a DMA, a desk descriptor load (issued
//     before the DMA it rides with) or an output store, and the loop-top wait
//     is counted by hand (vmcnt(1) when a store followed the DMA).
#include <stdint.h>

#include "crc32c_dev.h"

#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
// Profiling build only: per wave, the cycles of each part of a pipeline's
// loop (s_memtime) and its iteration counts, summed over launches
// (scripts/debug/lp_prof.py, ps_prof.py).
namespace wipdb {
namespace lk {
constexpr int kProfN = 16;  // accumulators per wave
__device__ unsigned long long g_lp_prof[4096 * kProfN];
}  // namespace lk
}  // namespace wipdb
#define WIPDB_PROF_ON 1
#define LP_T(x) const uint64_t x = __builtin_amdgcn_s_memtime()
#define LP_ACC(k, v) (prof[k] += (v))
#endif

#include "crc32c_ea.h"

namespace wipdb {
namespace lk {

// ---------------------------------------------------------------------------
// Spans per desk (lanes 0 .. kDesk - 1 hold a desk; masks are 32 bits)
constexpr uint32_t kDesk = 32;
// Desk size after a desk that held spans with segments (8: 0.650 ms on the
// headline vs 0.658 with 16, 0.664 with 32, 0.669 with 4, 0.714 with 2 --
// profiles/r03u_long_desk_ab.log, r03v_long_desk_small_ab.log)
#ifndef WIPDB_LP_LONG_DESK
#define WIPDB_LP_LONG_DESK 8
#endif
constexpr uint32_t kLongDesk = WIPDB_LP_LONG_DESK;
// Spans of this many segments or more are queued for the workgroup as soon
// as their desk is sorted (8: config 3's Zipf mix +2 % over 4, same session,
// profiles/r03w_eager_ab.log)
#ifndef WIPDB_LP_EAGER_SEGS
#define WIPDB_LP_EAGER_SEGS 8
#endif
constexpr uint32_t kEagerSegs = WIPDB_LP_EAGER_SEGS;
// Wave priority from a slot's arrival to the next DMA's issue (0: off): the
// wave whose bytes just landed gets its next 4 KiB in flight ahead of the
// other waves' compute (3: headline 0.6450 -> 0.6415 ms, short buckets +1 %,
// same session, profiles/r03y_prio_ab.log)
#ifndef WIPDB_LP_PRIO
#define WIPDB_LP_PRIO 3
#endif
constexpr int kPrio = WIPDB_LP_PRIO;
// (Variants measured and dropped, same-session A/B under profiles/: each lane
// DMA-ing its own stripe instead of the exchanged segment layout, -3..-12 %
// on short buckets, r03g_ab.log; the batch DMA through the caches, within
// noise, r03z_bnt_hiu_ab.log; exchanging the stripes' high address words only
// when they differ, within noise, same log; the per-lane selects as ?:
// chains, which hipcc lowered into exec-masked branches, short buckets -7 %,
// r03v2_vsel_ab.log; wave scans joined through readlane instead of DPP row
// broadcasts, -0.5..1 %, r03v4_bcast_ab.log; the wave OR by row broadcasts,
// mixed, r03v5_bcast_or_ab.log.)

// Bound of the long-span queue's spins (a popper waiting for its record's
// producer, a producer waiting for a slot to be freed): never reached while
// the workgroup's waves run (each wait is for a wave that writes next); if it
// is, the launch reports a fault (kFault*) instead of computing a wrong CRC.
// The host emulation sets a small bound to exercise that path.
#ifndef WIPDB_LP_SPIN
#define WIPDB_LP_SPIN (1u << 22)
#endif

// ---------------------------------------------------------------------------
// Wave scans (row-local DPP steps, rows joined by DPP row broadcasts)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t scan_add(uint32_t v) {
  v += dpp<0x111>(v);  // row_shr:1 (lanes without a source read 0)
  v += dpp<0x112>(v);  // row_shr:2
  v += dpp<0x114>(v);  // row_shr:4
  v += dpp<0x118>(v);  // row_shr:8
  v += bcast15(v);     // rows 1, 3 += lane 15 of the row before
  return v + bcast31(v);  // rows 2, 3 += lane 31
}
__device__ __forceinline__ uint32_t scan_xor(uint32_t v) {
  v ^= dpp<0x111>(v);
  v ^= dpp<0x112>(v);
  v ^= dpp<0x114>(v);
  v ^= dpp<0x118>(v);
  v ^= bcast15(v);
  return v ^ bcast31(v);
}
__device__ __forceinline__ uint32_t scan_or(uint32_t v) {  // the OR of the wave (uniform)
  v |= dpp<0x111>(v);
  v |= dpp<0x112>(v);
  v |= dpp<0x114>(v);
  v |= dpp<0x118>(v);
  return rdlane(v, 15) | rdlane(v, 31) |
         rdlane(v, 47) | rdlane(v, 63);
}

// r * x^(8 * 64 d) mod P for a per-lane d in [0, 63]: level-1 tables (64 a
// bytes, a = d % 8) then level-2 tables (512 c bytes, c = d / 8).  k1b / k2b:
// the lane's selector bases (bytes 128 + 4 t_j / 8 t_j, crc32c_lds.h).
__device__ __forceinline__ uint32_t shift64(const Lane& k, uint32_t k1b, uint32_t k2b, uint32_t r,
                                            uint32_t d) {
  const uint32_t a = d & 7u, c = (d >> 3) & 7u;
  const uint32_t k1 = k1b + a * 0x10101010u;
  const uint32_t a0 = lds_ld(kLdsMain + vperm(k1, r, k.sel[0]));
  const uint32_t a1 = lds_ld(kLdsMain + vperm(k1, r, k.sel[1]));
  const uint32_t a2 = lds_ld(kLdsMain + vperm(k1, r, k.sel[2]));
  const uint32_t a3 = lds_ld(kLdsMain + vperm(k1, r, k.sel[3]));
  const uint32_t v = a != 0u ? (xor3(a0, a1, a2) ^ a3) : r;
  const uint32_t k2 = k2b + c * 0x20202020u;
  const uint32_t b0 = lds_ld(kLdsL2 + (vperm(k2, v, k.sel[0]) >> 1));
  const uint32_t b1 = lds_ld(kLdsL2 + (vperm(k2, v, k.sel[1]) >> 1));
  const uint32_t b2 = lds_ld(kLdsL2 + (vperm(k2, v, k.sel[2]) >> 1));
  const uint32_t b3 = lds_ld(kLdsL2 + (vperm(k2, v, k.sel[3]) >> 1));
  return c != 0u ? (xor3(b0, b1, b2) ^ b3) : v;
}

// ~init * x^(-8 h) per lane (head_register is the uniform form).
__device__ __forceinline__ uint32_t head_register_lane(uint32_t l, uint32_t init, uint32_t h) {
  const uint32_t h0 = lds_ld(MiscAddr(kMiscHead0 + h));
  uint32_t r = ~init;
  if (ballot(init != 0u) != 0u) {
    for (uint32_t i = 0; i < 15u; ++i) {  // un-feed up to 15 zero bytes, lanes masked
      const uint32_t idx = lds_ld(MiscAddr(kMiscInvTop + (r >> 24)));
      const uint32_t t0 = lds_ld(kLdsMain + (idx << 8) + 96u + 4u * (l & 7u));
      const uint32_t u = ((r ^ t0) << 8) | idx;
      r = i < h ? u : r;
    }
  }
  return init == 0u ? h0 : r;
}

// verify_residue(jv) for a run-time jv (the constants, selected: the
// constexpr function itself would run its bit loop per span)
__device__ __forceinline__ uint32_t residue_of(uint32_t jv) {
  constexpr uint32_t kRes0 = verify_residue(0), kRes1 = verify_residue(1),
                     kRes2 = verify_residue(2), kRes3 = verify_residue(3);
  return jv == 0u ? kRes0 : (jv == 1u ? kRes1 : (jv == 2u ? kRes2 : kRes3));
}

// Word e / 4 .. of the 16 bytes c0..c3 at byte e (per lane; e + 4 may pass
// byte 16 -- only the low k <= 3 bytes of a tail word are used), with the
// selects on ballot masks (all lanes call it; hipcc turned ?: chains into
// exec-masked branches)
__device__ __forceinline__ uint32_t word_at_v(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t e) {
  const uint32_t q = e >> 2;
  const uint64_t q1 = ballot(q == 1u), q2 = ballot(q == 2u), q3 = ballot(q == 3u);
  const uint32_t lo = vsel(q3, c3, vsel(q2, c2, vsel(q1, c1, c0)));
  const uint32_t hi = vsel(q3, 0u, vsel(q2, c3, vsel(q1, c2, c1)));
  return alignbit(hi, lo, 8u * (e & 3u));
}
// fix_head (crc32c_plan.h) with the selects on ballot masks and the head
// masks by a 64-bit shift (all lanes call it; per-lane hp, ws, inj)
__device__ __forceinline__ void fix_head_v(uint32_t (&c)[4], uint32_t hp, uint32_t ws, uint32_t inj) {
  const uint64_t w1 = ballot(ws == 1u), w2 = ballot(ws == 2u), w3 = ballot(ws == 3u);
  uint32_t d[4];
  d[3] = vsel(w3, c[0], vsel(w2, c[1], vsel(w1, c[2], c[3])));
  d[2] = vsel(w3, 0u, vsel(w2, c[0], vsel(w1, c[1], c[2])));
  d[1] = vsel(w3 | w2, 0u, vsel(w1, c[0], c[1]));
  d[0] = vsel(w3 | w2 | w1, 0u, c[0]);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int32_t t0 = static_cast<int32_t>(hp) - 4 * w;
    const uint32_t t = static_cast<uint32_t>(t0 < 0 ? 0 : (t0 > 4 ? 4 : t0));
    c[w] = d[w] & static_cast<uint32_t>(0xffffffffull << (8u * t));
  }
  c[0] ^= inj;
}

// MakeStripe (crc32c_plan.h) with its select on a ballot mask (all lanes
// call it)
__device__ __forceinline__ Stripe make_stripe_v(PW pw, uint32_t j) {
  const int32_t f = static_cast<int32_t>(pw.front()) - 4 * static_cast<int32_t>(j);
  const uint32_t fr = f <= 0 ? 0u : static_cast<uint32_t>(f);
  const uint32_t real0 = (f >= 0 && f < 4 && pw.r() != 0u) ? 1u : 0u;
  Stripe st;
  st.s = -16 * static_cast<int64_t>(f);
  const uint32_t src = vsel(ballot(pw.x() != 0u), 16u * pw.r() - pw.te(), 4u * pw.ws());
  const uint32_t dif = src + 16u * static_cast<uint32_t>(f);
  st.info = fr | (real0 << 3) | (pw.ws() << 4) | (fr ? dif << 6 : 0u);
  return st;
}

// A segment iteration (uniform).
constexpr uint32_t kSFirst = 1u, kSLast = 2u, kSPush = 4u, kSAux = 8u;
struct SegW {
  uint32_t fl;
  uint32_t hw;    // hp | ws << 4 | k << 6 | jv << 8
  uint32_t init, id;
  uint32_t pw;    // kSPush: the back piece's word
  uint64_t p0;    // kSPush: its first chunk (offset from the source base)
};
// What an iteration computes.
constexpr uint32_t kWNone = 0u, kWSeg = 1u, kWBatch = 2u;

#if !defined(WIPDB_LK_EMU)
// A launch that saw a fault (kFault*) sets its own fault word: a word of the
// context's pinned fault table, one per synchronous lane and one per caller
// stream (hcrc_api.cc), so a fault is reported to the caller whose launch it
// was.  The pointer is a kernel argument that run_lp parks in LDS right after
// the table image (kMiscFaultWord) and reads back only on the way out: no
// register stays live for it through the loop.  A plain store of 1, system
// scope (the word is in host memory the host reads after the stream).
__device__ __forceinline__ void report_fault(unsigned int* word, uint32_t) {
  if ((lane_tid() & 63u) == 0u) __hip_atomic_store(word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif


template <int OUT, typename Src>
__device__ __forceinline__ void run_lp(const Src& src, void* out, uint32_t flags,
                                       const uint8_t* image, unsigned int* fault) {
  constexpr bool kV = OUT == 1;
  const uint32_t l = lane_tid() & 63u;
  const uint32_t w = uni(lane_tid() >> 6);
  const uint64_t count = src.count;
  const WgUnits units = wg_units(count, src_bounds(src));
  if (units.count == 0u) return;  // no unit of work
  load_image(image, w, l);
  {  // (every lane of every wave: the same value; each wave reads back its own)
    const uint64_t fw = reinterpret_cast<uint64_t>(fault);
    lds_st_sync(MiscAddr(kMiscFaultWord), static_cast<uint32_t>(fw));
    lds_st_sync(MiscAddr(kMiscFaultWord + 1u), static_cast<uint32_t>(fw >> 32));
  }
  const Lane lk = make_lane<1>(l);
  Pipe pp;
  pp.init(l, w);
  const bool msk = (flags & kFlagMask) != 0u;
  const uint64_t sbase = reinterpret_cast<uint64_t>(src.base);
  g_u32* const out32 = (g_u32*)(reinterpret_cast<uintptr_t>(out));
  g_u8* const out8 = (g_u8*)(reinterpret_cast<uintptr_t>(out));

  // per-lane selector bases of the batch fold (shift64) and the batch DMA's
  // stripe / chunk of this lane in each of its 4 instructions
  uint32_t k1b = 0, k2b = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t t = (j + ((l >> 3) & 3u)) & 3u;
    k1b |= (128u + 4u * t) << (8 * j);
    k2b |= (8u * t) << (8 * j);
  }
  const uint32_t dsl = l >> 2;                          // stripe lane 16 q + dsl
  const uint32_t dci = ((l & 3u) - (l >> 4)) & 3u;      // chunk of that stripe

  // ---- the piece ring: entry q in lane q ----
  uint32_t rp_lo = 0, rp_hi = 0, rpw = 0, rinj = 0, rid = 0;
  uint32_t rcnt = 0, rlanes = 0;
  // ---- the desk (lanes 0 .. kDesk - 1) and the next desk, loading ----
  uint64_t da = 0, na = 0;
  uint32_t dn = 0, di = 0, nn = 0, ni = 0;
  uint32_t dpl = 0, dpw = 0;  // the desk's plan and piece words
  uint32_t npl = 0, npw = 0;  // the next desk's (sort_desk)
  uint32_t dbase = 0, nbase = 0;  // first unit of the desk (span_of: its span)
  uint32_t dtotal = 0;        // the desk's long spans still counted in the held count
  uint32_t dshort = 0;        // desk lanes whose short span is not in the ring yet
  uint32_t dlong = 0;         // desk lanes whose long span this wave has not taken
  uint32_t nlive = 0;         // next desk: lanes holding a span
  uint32_t nshort = 0, nlong = 0;  // next desk: its short / long spans (once sorted)
  uint32_t nstate = 0;        // next desk: 0 none, 1 loads issued, 2 loads waited for
  bool nsorted = false;       // next desk: sorted (empty spans answered)
  bool exhausted = false;
  bool wide = true;           // the last sorted desk was all short spans: full desks
  // ---- the long span being run (taken from the desk or the queue) ----
  // (c0 = a - hp, plan word, piece word: crc32c_plan.h PackPL)
  uint64_t lc0 = 0;
  uint32_t lpl = 0, lpw = 0;
  uint32_t lt = 0, linit = 0, lid = 0;
  bool lvalid = false;
  // ---- the iterations: current and next ----
  // kind (2) | a batch's lanes (7) << 2 | its split piece's first lane
  // (7; 64: none) << 9
  uint32_t ck = kWNone, nk = kWNone;
  SegW cs{}, ns{};
  uint32_t cb_pw = 0, cb_inj = 0, cb_id = 0, cb_j = 0;  // batch, per lane
  uint32_t nb_pw = 0, nb_inj = 0, nb_id = 0, nb_j = 0;
  uint32_t carry = 0, carry_tw = 0;   // the split piece's register over its first lanes, tail word
  uint32_t chain = 0;

  // The workgroup's units (crc32c_dev.h wg_units): blocks of 16 spans round
  // robin over the grid, so the chip reads one compact window of the batch
  // at a time, then the spans past the last whole round one at a time; ug =
  // its unit count.
  auto span_of = [&](uint32_t un) -> uint64_t { return unit_span(un, units); };
  const uint32_t ug = units.count;
  // A desk: one unit-counter add, the descriptors loaded (lanes 0 .. size -
  // 1; waited for at first use).  kDesk units while the workgroup has
  // plenty left, then 16 and 8 (the waves' last desks end close together).
  auto grab_desk = [&]() {
    uint32_t u = 0, size = kDesk;
    if (l == 0u) {
      const uint32_t seen = lds_ld_sync(MiscAddr(kMiscUnit));
      const uint32_t rem = seen < ug ? ug - seen : 0u;
      size = rem >= 32u * kDesk ? kDesk : (rem >= 16u * kDesk ? kDesk / 2u : kDesk / 4u);
      // half desks after a desk that held spans with segments (they take a
      // wave iteration each: a full desk is a long stretch of one wave's work)
      if (!wide && size > kLongDesk) size = kLongDesk;
      u = lds_add(MiscAddr(kMiscUnit), size);
    }
    u = uni(u);
    size = uni(size);
    nbase = u;
    if (u >= ug) {
      exhausted = true;
      nstate = 0;
      return;
    }
    const uint32_t un = u + l;
    const bool v = l < size && un < ug;
    nlive = static_cast<uint32_t>(ballot(v));
    if (v) src.lane(span_of(un), na, nn, ni);
    if (l == 0u) lds_add(MiscAddr(kMiscDesks), 1u);
    nstate = 1;
    nsorted = false;
  };

  // The long-span queue (workgroup, LDS): a wave's own long spans go there
  // only when another wave has run out of work (share).  pop: claim the head
  // record by CAS while head < tail, read it once its producer has written
  // it, free it.
  auto pop = [&]() {
    uint32_t got = 0, idx = 0;
    if (l == 0u) {
      uint32_t h = lds_ld_sync(MiscAddr(kMiscQHead));
      for (int tries = 0; tries < 64; ++tries) {
        const uint32_t t = lds_ld_sync(MiscAddr(kMiscQTail));
        if (static_cast<int32_t>(t - h) <= 0) break;
        const uint32_t old = lds_cas(MiscAddr(kMiscQHead), h, h + 1u);
        if (old == h) {
          got = 1;
          idx = h;
          break;
        }
        h = old;
      }
    }
    if (uni(got) == 0u) return;
    idx = uni(idx);
    const uint32_t ra = QRecAddr(idx);
    uint32_t r3 = 0;
#pragma nounroll
    for (uint32_t spin = 0; spin < WIPDB_LP_SPIN; ++spin) {  // its producer writes it next
      r3 = uni(queue_marker(lds_ld_sync(ra + 12u), idx));
      if (r3 != 0u) break;
      lk_sleep();
    }
    compiler_barrier();  // the record after its marker
    const uint32_t r0 = uni(lds_ld_sync(ra)), r1 = uni(lds_ld_sync(ra + 4u)),
                   r2 = uni(lds_ld_sync(ra + 8u)),
                   ri = uni(lds_ld_sync(MiscAddr(kMiscQInit + (idx & (kQSlots - 1u)))));
    lgkm_wait();  // read before the slot is freed
    if (l == 0u) {
      if (r3 != 0u) {
        lds_st_sync(ra + 12u, 0u);
        lds_add(MiscAddr(kMiscQRes), 0xffffffffu);
      } else {
        // never written within the bound (no schedule of the workgroup's
        // waves gets here: its producer reserved the slot and writes it
        // next) -- the span is lost, so the launch reports it; the record
        // stays claimed and unfreed, so no later push overwrites a slot its
        // producer may still fill
        lds_st_sync(MiscAddr(kMiscFault), kFaultQueuePop);
      }
    }
    if (r3 == 0u) return;
    const uint64_t a = (static_cast<uint64_t>(r1) << 32) | r0;
    lid = r3 - 1u;
    linit = ri;
    const Plan p = MakePlan(a, static_cast<uint32_t>(sbase + a), r2, kV);
    lpl = PackPL(p);
    lpw = p.pw;
    lc0 = p.c0;
    lt = 0;
    lvalid = true;
  };
  // The long spans of desk lanes m (a, bytes b, init iv, span base + lane)
  // into the queue, if it has room for them all (reserved in the QRes
  // count, so a push never waits on a slot no wave will free); `held` of the
  // workgroup's held count leave it once queued.  Returns whether queued.
  auto queue_longs = [&](uint32_t m, uint64_t a, uint32_t b, uint32_t iv, uint32_t base,
                         uint32_t held) -> bool {
    const bool lng = l < kDesk && ((m >> (l & (kDesk - 1u))) & 1u) != 0u;  // (a shift by >= 32 is mod 32)
    const uint32_t k = static_cast<uint32_t>(__builtin_popcount(m));
    uint32_t rs = 0;
    if (l == 0u) rs = lds_add(MiscAddr(kMiscQRes), k);
    rs = uni(rs);
    if (rs + k > kQSlots) {
      if (l == 0u) lds_add(MiscAddr(kMiscQRes), 0u - k);
      return false;
    }
    uint32_t q = 0;
    if (l == 0u) q = lds_add(MiscAddr(kMiscQTail), k);
    q = uni(q);
    const uint32_t qk = q + mbcnt_lo(m, 0u);
    const uint32_t ra = QRecAddr(qk);
    // a slot is reused only once its last record has been read (queue
    // records are popped by the waves that asked for work: this rarely waits)
    bool busy = false;
#pragma nounroll
    for (uint32_t spin = 0; spin < WIPDB_LP_SPIN; ++spin) {
      busy = lng && lds_ld_sync(ra + 12u) != 0u;
      if (ballot(busy) == 0u) break;
      lk_sleep();
    }
    // a slot still not freed within the bound is never overwritten: its span
    // is lost, and the popper that takes slot qk next finds the OLD record
    // there (its marker still set) and runs that span a second time -- a
    // duplicate as well as a loss.  Both are covered by the fault: the launch
    // says so (kFaultQueueSlot, the launch's fault word), and its outputs are
    // not to be used (HCRC_ERR_KERNEL)
    if (busy) lds_st_sync(MiscAddr(kMiscFault), kFaultQueueSlot);
    if (lng && !busy) {
      lds_st_sync(ra, static_cast<uint32_t>(a));
      lds_st_sync(ra + 4u, static_cast<uint32_t>(a >> 32));
      lds_st_sync(ra + 8u, b);
      lds_st_sync(MiscAddr(kMiscQInit + (qk & (kQSlots - 1u))), iv);
    }
    lgkm_wait();  // the record before its marker
    if (lng && !busy) lds_st_sync(ra + 12u, static_cast<uint32_t>(span_of(base + l)) + 1u);
    if (l == 0u && held != 0u) lds_add(MiscAddr(kMiscHeld), 0u - held);  // (after the records: in order)
    return true;
  };

  // The next desk, once its descriptors are in: its empty spans answered,
  // its short and long spans sorted into lane masks (the long ones held by
  // this wave, counted in the workgroup's held count before the desk leaves
  // the in-flight count).
  auto sort_desk = [&]() {
    const bool live = l < kDesk && ((nlive >> (l & (kDesk - 1u))) & 1u) != 0u;
    const uint64_t s = span_of(nbase + l);
    const Plan p = MakePlan(na, static_cast<uint32_t>(sbase + na), src.bytes(nn), kV);
    const bool empty = live && p.empty;
    if (!kV && empty) out32[s] = msk ? mask_crc(ni) : ni;
    npl = PackPL(p);
    npw = p.pw;
    nshort = static_cast<uint32_t>(ballot(live && !p.empty && p.m == 0u));
    nlong = static_cast<uint32_t>(ballot(live && !p.empty && p.m != 0u));
    wide = nlong == 0u;
    // spans of kEagerSegs segments or more go to the queue right away (if it
    // has room): the workgroup's waves take them one at a time, as they
    // become free -- a desk of long spans is not left on one wave
    const uint32_t big = static_cast<uint32_t>(ballot(live && !p.empty && p.m >= kEagerSegs));
    if (big != 0u && queue_longs(big, na, src.bytes(nn), ni, nbase, 0u)) nlong &= ~big;
    if (l == 0u) {
      if (nlong != 0u) lds_add(MiscAddr(kMiscHeld), static_cast<uint32_t>(__builtin_popcount(nlong)));
      lds_add(MiscAddr(kMiscDesks), 0xffffffffu);
    }
    nsorted = true;
  };
  // Waves out of work (the idle count): this wave's held long spans, of the
  // desk and of the sorted next desk, into the queue.
  // (the desk's long spans leave the held count all at once: those it has
  // taken and those it queues now)
  auto share = [&]() {
    if (dlong != 0u && queue_longs(dlong, da, dn, di, dbase, dtotal)) {
      dlong = 0;
      dtotal = 0;
    }
    if (nstate == 2u && nsorted && nlong != 0u &&
        queue_longs(nlong, na, src.bytes(nn), ni, nbase, static_cast<uint32_t>(__builtin_popcount(nlong))))
      nlong = 0;
  };
  // The desk's next own long span becomes the one being run; the desk's
  // long spans leave the held count when the last is taken.
  auto take_own = [&]() {
    const uint32_t k = static_cast<uint32_t>(__builtin_ctz(dlong));
    const uint32_t pl = rdlane(dpl, k);
    lc0 = ((static_cast<uint64_t>(rdlane(static_cast<uint32_t>(da >> 32), k)) << 32) |
           rdlane(static_cast<uint32_t>(da), k)) - PL_hp(pl);
    lpl = pl;
    lpw = rdlane(dpw, k);
    linit = rdlane(di, k);
    lid = static_cast<uint32_t>(span_of(dbase + k));
    lt = 0;
    lvalid = true;
    dlong &= dlong - 1u;
    if (dlong == 0u) {
      if (l == 0u) lds_add(MiscAddr(kMiscHeld), 0u - dtotal);
      dtotal = 0;
    }
  };
  // The next desk becomes the desk.
  auto switch_desk = [&]() {
    if (!nsorted) sort_desk();
    dpl = npl;
    dpw = npw;
    da = na;
    dn = src.bytes(nn);
    di = ni;
    dbase = nbase;
    dshort = nshort;
    dlong = nlong;
    dtotal = static_cast<uint32_t>(__builtin_popcount(nlong));
    nlong = 0;
    nstate = 0;
  };

  // The desk's short spans into the ring, as many as it has room for.
  auto push_shorts = [&]() {
    const uint32_t room = 64u - rcnt;
    const uint32_t c = static_cast<uint32_t>(__builtin_popcount(dshort));
    const uint32_t take = c < room ? c : room;
    // desk lane l: its piece (valid in the short lanes: the whole span, m = 0)
    const uint32_t hp = PL_hp(dpl);
    const uint64_t p0 = da - hp;
    const uint32_t inj = head_register_lane(l, di, hp);
    const uint32_t rank = mbcnt_lo(dshort, 0u);
    const bool tk = l < kDesk && ((dshort >> (l & (kDesk - 1u))) & 1u) != 0u && rank < take;
    const uint32_t tmask = static_cast<uint32_t>(ballot(tk));
    const uint32_t nl_sum = scan_add(tk ? PW{dpw}.nl() : 0u);
    // ring lane q in [rcnt, rcnt + take) pulls the (q - rcnt)-th short lane
    const uint32_t kq = l - rcnt;
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = kDesk / 2u; st != 0u; st >>= 1) {  // (pos + st <= 31)
      const uint32_t below = dshort & ((1u << (pos + st)) - 1u);
      pos = static_cast<uint32_t>(__builtin_popcount(below)) <= kq ? pos + st : pos;
    }
    const bool me = l >= rcnt && kq < take;
    const uint32_t v_lo = bperm(static_cast<uint32_t>(p0), pos);
    const uint32_t v_hi = bperm(static_cast<uint32_t>(p0 >> 32), pos);
    const uint32_t v_pw = bperm(dpw, pos), v_inj = bperm(inj, pos);
    const uint32_t v_id = static_cast<uint32_t>(span_of(dbase + pos));
    rp_lo = me ? v_lo : rp_lo;
    rp_hi = me ? v_hi : rp_hi;
    rpw = me ? v_pw : rpw;
    rinj = me ? v_inj : rinj;
    rid = me ? v_id : rid;
    rcnt += take;
    rlanes += rdlane(nl_sum, 63);
    dshort &= ~tmask;
  };

  // ---- decide: issue the next iteration's DMA ----
  auto issue_seg = [&]() {
    const uint32_t m = PL_m(lpl);
    const uint64_t p0 = lc0 + 4096u * static_cast<uint64_t>(m);  // the back piece / span grid end
    const uint64_t wb = sbase + lc0 + 4096u * static_cast<uint64_t>(lt);
    const uint32_t o = 16u * pp.cm;
    const uint32_t s0 = lt == 0u ? 4u * PL_ws(lpl) : 0u;
    dma4(wb, pp.slot, o > s0 ? o : s0, o + 1024u, o + 2048u, o + 3072u);
    const bool last = lt + 1u == m;
    const bool aux = last && PL_aux(lpl) != 0u;
    ns.fl = (lt == 0u ? kSFirst : 0u) | (last ? kSLast : 0u) |
            (last && lpw != 0u ? kSPush : 0u) | (aux ? kSAux : 0u);
    // (seg_aux: no piece, so the grid ends at c0 + 4096 m; the aux chunk is
    // the 16 bytes ending at E4 + 4)
    if (aux) dma_piece(l, sbase + p0 - 12u, 0u, SegAuxAddr(w));
    ns.hw = PL_hw(lpl);
    ns.init = linit;
    ns.id = lid;
    ns.pw = lpw;
    ns.p0 = p0;
    nk = kWSeg;
    ++lt;
    if (last) lvalid = false;
  };
  // A batch: the ring's first pieces, each on its remaining lanes, in order;
  // the batch fills all 64 lanes -- a piece that does not fit is split, its
  // first lanes now and the rest (a continuation, its register carried) at
  // the head of the next batch.
  auto issue_batch = [&]() {
    const PW rw{rpw};
    const uint32_t rem = l < rcnt ? rw.rem() : 0u;
    const uint32_t incl = scan_add(rem);
    const bool tk = l < rcnt && incl <= 64u;
    const uint32_t n = static_cast<uint32_t>(__builtin_popcountll(ballot(tk)));  // >= 1
    const uint32_t usedf = rdlane(incl, n - 1u);
    const bool part = usedf < 64u && n < rcnt;  // entry n is split
    const uint32_t used = part ? 64u : usedf;
    const uint32_t st = incl - rem;
    // start lanes of the taken pieces, and each lane's piece
    const bool sb = tk || (part && l == n);
    const uint32_t smlo = scan_or(sb && st < 32u ? 1u << (st & 31u) : 0u);
    const uint32_t smhi = scan_or(sb && st >= 32u ? 1u << (st & 31u) : 0u);
    const uint32_t le = mbcnt_hi(smhi, mbcnt_lo(smlo, 0u)) +
                        (((l < 32u ? smlo : smhi) >> (l & 31u)) & 1u);
    const uint32_t e = le - 1u;
    const bool live = l < used;
    const uint32_t b_lo = bperm(rp_lo, e), b_hi = bperm(rp_hi, e);
    const uint32_t b_pw = bperm(rpw, e), b_inj = bperm(rinj, e), b_id = bperm(rid, e);
    const uint32_t b_st = bperm(st, e);
    const PW pw{live ? b_pw : 0u};
    const uint32_t j = live ? pw.j0() + (l - b_st) : 0u;  // the lane's stripe of its piece
    const Stripe sp = make_stripe_v(pw, j);
    const uint64_t S = sbase + ((static_cast<uint64_t>(b_hi) << 32) | b_lo) +
                       static_cast<uint64_t>(sp.s);
    const uint32_t s_lo = static_cast<uint32_t>(S), s_hi = static_cast<uint32_t>(S >> 32);
    // instruction q: lane m loads chunk dci of stripe 16 q + dsl (the
    // segment DMA's layout), its address from the lane that owns the stripe
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t sl = 16u * q + dsl;
      const uint32_t x_lo = bperm(s_lo, sl), x_hi = bperm(s_hi, sl), x_in = bperm(sp.info, sl);
      // StripeChunkSrc(x_in, dci) on ballot masks
      const uint32_t fr = x_in & 7u;
      const uint64_t lt = ballot(dci < fr), eq = ballot(dci == fr && (x_in & 8u) != 0u);
      const uint32_t off = vsel(lt, x_in >> 6, 16u * dci + vsel(eq, (x_in >> 2) & 12u, 0u));
      const uint64_t a = ((static_cast<uint64_t>(x_hi) << 32) | x_lo) + off;
      if (sl < used) dma1v(a, pp.slot + 1024u * q);
    }
    nb_pw = pw.v;
    nb_inj = b_inj;
    nb_id = b_id;
    nb_j = j;
    nk = kWBatch | (used << 2) | ((part ? usedf : 64u) << 9);
    // the ring drops its first n entries; a split one stays at its head
    rp_lo = bperm(rp_lo, l + n);
    rp_hi = bperm(rp_hi, l + n);
    rpw = bperm(rpw, l + n);
    rinj = bperm(rinj, l + n);
    rid = bperm(rid, l + n);
    if (part && l == 0u) rpw = PW{rpw}.advanced(64u - usedf);
    rcnt -= n;
    rlanes -= used;
  };
  // Chooses and issues the next iteration (nkind = kWNone: no work left).
  auto decide = [&]() {
    nk = kWNone;
    for (int guard = 0; guard < 64; ++guard) {
      if (rcnt != 0u && (rlanes >= 64u || rcnt == 64u)) break;  // a full batch
      if (lvalid) {
        issue_seg();
        return;
      }
      if (dshort != 0u) {
        push_shorts();
        continue;
      }
      if (dlong != 0u) {
        take_own();
        continue;
      }
      pop();  // long spans another wave shared
      if (lvalid) continue;
      if (nstate != 0u) {
        // (stalls on the desk's loads if they were issued just now)
        switch_desk();
        continue;
      }
      if (rcnt != 0u) break;  // the ring's last pieces
      if (!exhausted) {
        grab_desk();  // (a stall: nothing else to do)
        loads_landed(na);
        loads_landed(nn);
        loads_landed(ni);
        continue;
      }
      // out of work: counted idle, so that the waves holding long spans
      // share them, take what they queue until none is held and no desk is
      // in flight (bounded)
      if (l == 0u) lds_add(MiscAddr(kMiscIdle), 1u);
      bool again = false;
#pragma nounroll
      for (uint32_t spin = 0; spin < (1u << 16); ++spin) {
        pop();
        if (lvalid) {
          again = true;
          break;
        }
        const uint32_t held = uni(lds_ld_sync(MiscAddr(kMiscHeld)));
        const uint32_t desks = uni(lds_ld_sync(MiscAddr(kMiscDesks)));
        lgkm_wait();  // (both read before the queue is looked at again)
        if (held == 0u && desks == 0u) {
          pop();
          again = lvalid;
          break;
        }
        lk_sleep();
      }
      if (l == 0u) lds_add(MiscAddr(kMiscIdle), 0xffffffffu);
      if (!again) break;
    }
    if (rcnt != 0u) issue_batch();
  };

  // One full 4 KiB segment of a long span (the iteration described by c,
  // its 64 stripes in W): chained, pushed to the ring (a back piece follows)
  // or finished (stored: returns true).
  auto seg_compute = [&](const SegW& c, uint32_t (&W)[16], const u32x4& ax) -> bool {
      // ---- one full 4 KiB segment of a long span ----
      const uint32_t hp = c.hw & 15u, ws = (c.hw >> 4) & 3u;
      {
        // lane 0's first chunk: the head (masked, shifted, the head register
        // injected) or the chain register -- computed aside, selected in
        // (one register assignment of W whichever branch ran)
        uint32_t h4[4] = {W[0], W[1], W[2], W[3]};
        if (c.fl & kSFirst) {
          // (no head bytes and init 0 -- aligned blocks, WriteRawBlock's
          // spans: ~0, no table read in front of the scan)
          const uint32_t inj = (c.init | hp) == 0u ? ~0u : head_register(l, c.init, hp);
          if ((hp | ws) == 0u) h4[0] ^= inj;
          else fix_head(h4, hp, ws, inj);
        } else {
          h4[0] ^= chain;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) W[i] = l == 0u ? h4[i] : W[i];
      }
      if (kV && (c.fl & kSLast) && !(c.fl & kSPush)) {
        uint32_t lo = W[14], hi = W[15];
        fix_trailer(lo, hi, (c.hw >> 8) & 3u);
        W[14] = l == 63u ? lo : W[14];
        W[15] = l == 63u ? hi : W[15];
      }
      uint32_t R = fold<1>(lk, l, scan(lk, W))[0];
      if (!(c.fl & kSLast)) {
        chain = R;
        return false;
      }
      if (c.fl & kSPush) {
        // the back piece enters the ring with the segments' register
        const bool me = l == rcnt;
        rp_lo = me ? static_cast<uint32_t>(c.p0) : rp_lo;
        rp_hi = me ? static_cast<uint32_t>(c.p0 >> 32) : rp_hi;
        rpw = me ? c.pw : rpw;
        rinj = me ? R : rinj;
        rid = me ? c.id : rid;
        ++rcnt;
        rlanes += PW{c.pw}.nl();
        return false;
      }
      {
        if (c.fl & kSAux) {
          const uint32_t tw = uni(ax.w);  // the aux chunk ends at E4 + 4
          R = uni(tail_step(lk, R, tw, (c.hw >> 6) & 3u));
        }
        if (l == 0u) {
          if (kV) out8[c.id] = R == residue_of((c.hw >> 8) & 3u) ? 1u : 0u;
          else out32[c.id] = msk ? mask_crc(~R) : ~R;
        }
      }
      return true;
  };

  // The loop: wait for this iteration's bytes, read them, issue the next
  // iteration's DMA (decide), compute this one.  An iteration that ends the
  // work may have pushed the last pieces: the loop then decides once more
  // without an iteration in hand (that DMA goes out after its store, so the
  // next wait is for everything).  One call site of decide: the kernel's
  // code stays small.
  bool have = false, stored_prev = false;
#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
  uint64_t prof[kProfN] = {};
  LP_T(t_start);
#endif
  for (;;) {
    // ---- segments back to back: the long span in hand, then the desk's
    // own spans with segments (aligned 4 KiB blocks, table blocks' main
    // segments, verify blocks, long spans) -- a loop of its own, with only
    // what they need live.  Entered with a segment issued, left with one
    // issued (the general loop below takes it): when a batch is due, the
    // desk has no span with segments left, or another wave is idle while
    // this one holds long spans (the general loop shares them). ----
    if (have && (nk & 3u) == kWSeg) {
      bool fidle = false;
#pragma nounroll
      for (;;) {
        LP_T(s0);
        // the desk is out of spans with segments: a span queued for the
        // workgroup, else the next desk if it is in, sorted, and holds only
        // spans with segments
        if (!lvalid && dlong == 0u) pop();
        if (!lvalid && dlong == 0u && dshort == 0u && nstate == 2u && nsorted && nshort == 0u &&
            nlong != 0u && !fidle)
          switch_desk();
        if (!lvalid && (dlong == 0u || fidle)) break;
        if (rcnt >= 62u || rlanes + ((ns.fl & kSPush) ? PW{ns.pw}.nl() : 0u) >= 64u) break;  // a batch is due
        LP_T(s1);
        if (stored_prev) wait_vm<1>();
        else wait_vm<0>();
        LP_T(s2);
        if constexpr (kPrio != 0) lk_prio<kPrio>();
        if (nstate == 1u) {
          // the desk loads are older than the DMA just waited for: the
          // compiler's own wait for them goes here, once per desk (not on
          // every iteration, where it would also wait for the last store)
          nstate = 2u;
          loads_landed(na);
          loads_landed(nn);
          loads_landed(ni);
        }
        const SegW c = ns;
        const uint32_t idle_w = lds_ld_sync(MiscAddr(kMiscIdle));
        uint32_t W[16];
        pp.read(W);
        u32x4 fax{0, 0, 0, 0};
        if (c.fl & kSAux) fax = lds_ld4(SegAuxAddr(w));
        pp.release();
        // the next desk sorted once its loads are in (before this
        // iteration's DMA: any wait the compiler adds for them is free here)
        if (nstate == 2u && !nsorted) sort_desk();
        // the desk after the next: its loads go out BEFORE this iteration's
        // DMA, so the wait for that DMA covers them (and the store issued
        // after it may stay in flight)
        if (nstate == 0u && !exhausted) grab_desk();
        if (!lvalid) take_own();
        LP_T(s3);
        issue_seg();
        if constexpr (kPrio != 0) lk_prio<0>();
        LP_T(s4);
        stored_prev = seg_compute(c, W, fax);
        fidle = uni(idle_w) != 0u;
        LP_T(s5);
        LP_ACC(8, s1 - s0);   // checks (pop, switch_desk, exits)
        LP_ACC(9, s2 - s1);   // wait for the slot
        LP_ACC(10, s3 - s2);  // read, sort / grab / take
        LP_ACC(11, s4 - s3);  // issue the next DMA
        LP_ACC(12, s5 - s4);  // compute
        LP_ACC(13, 1u);
      }
    }
    LP_T(t0);
    uint32_t W[16];
    uint32_t idle = 0;  // waves of the workgroup out of work
    u32x4 ax{0, 0, 0, 0};
    if (have) {
      if (stored_prev) wait_vm<1>();
      else wait_vm<0>();
      if constexpr (kPrio != 0) lk_prio<kPrio>();
      if (nstate == 1u) {  // the next desk's loads are in (see the segment loop)
        nstate = 2u;
        loads_landed(na);
        loads_landed(nn);
        loads_landed(ni);
      }
      ck = nk;
      cs = ns;
      cb_pw = nb_pw;
      cb_inj = nb_inj;
      cb_id = nb_id;
      cb_j = nb_j;
      const uint32_t idle_w = lds_ld_sync(MiscAddr(kMiscIdle));  // (rides with the slot's reads)
      pp.read(W);
      if ((ck & 3u) == kWSeg && (cs.fl & kSAux)) ax = lds_ld4(SegAuxAddr(w));
      pp.release();
      idle = uni(idle_w);
    } else {
      ck = kWNone;
    }
    const uint32_t ckind = ck & 3u;
    // the next desk sorted once its loads are in (before the next DMA)
    if (nstate == 2u && !nsorted) sort_desk();
    // the next desk's descriptor loads go out before the next DMA (decide):
    // the wait for that DMA covers them, the store after it may stay in
    // flight (decide stalls on them only when the desk in hand runs dry)
    if (nstate == 0u && !exhausted) grab_desk();
    LP_T(t1);
    decide();
    if constexpr (kPrio != 0) lk_prio<0>();
    LP_T(t2);

    bool did_store = false;
    if (ckind == kWSeg) {
      did_store = seg_compute(cs, W, ax);
    } else if (ckind == kWBatch) {
      // ---- a batch of pieces, each on its own lanes ----
      const uint32_t cused = (ck >> 2) & 127u, csplit = ck >> 9;
      const bool live = l < cused;
      const PW pw{cb_pw};
      const uint32_t j = cb_j, nl = pw.nl(), r = pw.r();
      const int32_t f = static_cast<int32_t>(pw.front()) - 4 * static_cast<int32_t>(j);
      // lane 0 of a piece with a tail: its chunk 0 is the aux chunk
      const uint32_t tw = word_at_v(W[0], W[1], W[2], W[3], pw.te());
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool z = !live || i < f;
#pragma unroll
        for (int q = 0; q < 4; ++q) W[4 * i + q] = z ? 0u : W[4 * i + q];
      }
      // the piece's first real chunk (chunk f of the lane with 0 <= f < 4)
      if (ballot(live && r != 0u && f >= 0 && f < 4) != 0u) {
        const bool has = live && r != 0u && f >= 0 && f < 4;
        uint32_t c[4];
        const uint64_t f1 = ballot(f == 1), f2 = ballot(f == 2), f3 = ballot(f == 3);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          c[q] = vsel(f3, W[12 + q], vsel(f2, W[8 + q], vsel(f1, W[4 + q], W[q])));
        fix_head_v(c, pw.hp(), pw.ws(), cb_inj);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint64_t hi = ballot(has && f == i);
#pragma unroll
          for (int q = 0; q < 4; ++q) W[4 * i + q] = vsel(hi, c[q], W[4 * i + q]);
        }
      }
      if (kV) {
        uint32_t lo = W[14], hi = W[15];
        fix_trailer(lo, hi, pw.jv());
        const bool lastl = live && j + 1u == nl;
        W[14] = lastl ? lo : W[14];
        W[15] = lastl ? hi : W[15];
      }
      const uint32_t R = scan(lk, W);
      const uint32_t d = live ? nl - 1u - j : 0u;  // lanes of the piece after this one
      const uint32_t v = shift64(lk, k1b, k2b, R, d);
      const uint32_t xs = scan_xor(v);
      // the piece's lanes in this batch end at lane l + min(d, 63 - l): the
      // XOR over them, at its first lane here (j == j0)
      const uint32_t last = l + (d < 63u - l ? d : 63u - l);
      uint32_t G = bperm(xs, last) ^ xs ^ v;
      const bool leader = live && j == pw.j0();
      const bool done = d <= 63u - l;  // (at the leader) the piece ends in this batch
      // a continuation finishes with the register carried from its first
      // lanes (and their tail word); a split piece leaves its own for the next
      const uint32_t c_new = csplit < 64u ? rdlane(G, csplit) : 0u;
      const uint32_t t_new = csplit < 64u ? rdlane(tw, csplit) : 0u;
      G ^= pw.cont() ? carry : 0u;
      const uint32_t twv = pw.cont() ? carry_tw : tw;
      G ^= r == 0u ? cb_inj : 0u;
      carry = c_new;
      carry_tw = t_new;
      const bool fin = leader && done;
      if (kV) {
        if (fin) out8[cb_id] = G == residue_of(pw.jv()) ? 1u : 0u;
      } else {
        const uint32_t Gt = tail_step(lk, G, twv, pw.k());
        G = pw.x() ? Gt : G;
        if (fin) out32[cb_id] = msk ? mask_crc(~G) : ~G;
      }
      did_store = true;
    }
    stored_prev = did_store;
    LP_T(t3);
    if (have) {
      // while the DMA flies: share the long spans this wave holds when
      // another wave is out of work
      if (idle != 0u && (dlong | nlong) != 0u) share();
    }
    LP_T(t4);
    LP_ACC(0, t1 - t0);
    LP_ACC(1, t2 - t1);
    LP_ACC(2, t3 - t2);
    LP_ACC(3, t4 - t3);
    LP_ACC(4, ckind == kWSeg ? 1u : 0u);
    LP_ACC(5, ckind == kWBatch ? 1u : 0u);
    LP_ACC(6, ckind == kWNone ? 1u : 0u);
    if ((nk & 3u) == kWNone) {
      // (decide gives up after 64 steps -- e.g. desks of empty spans -- with
      // work left: decide again)
      const bool left = nstate != 0u || !exhausted || dshort != 0u || rcnt != 0u || lvalid;
      if (!have && !left) break;
      have = false;
      continue;
    }
    have = true;
  }
  // a queue wait that ran out of its bound (kFault*, kept in LDS) is
  // reported when the wave leaves: the wave that saw it leaves after it (a
  // global write inside the queue's code made hipcc lose track of the uniform
  // values there; a register for it cost SGPR spills)
  {
    const uint32_t f = uni(lds_ld_sync(MiscAddr(kMiscFault)));
    if (f != 0u) {
      const uint64_t fw = (static_cast<uint64_t>(uni(lds_ld_sync(MiscAddr(kMiscFaultWord + 1u)))) << 32) |
                          uni(lds_ld_sync(MiscAddr(kMiscFaultWord)));
      report_fault(reinterpret_cast<unsigned int*>(fw), f);
    }
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

// run_ps, the stream-tiled pipeline of packed batches (HCRC_PACKED)
#include "crc32c_ps.h"

namespace wipdb {
namespace lk {

// ---------------------------------------------------------------------------
// The pipeline of a launch.  run_lp packs short spans (3.3-3.7 TiB/s on the
// 512 B .. 2 KiB buckets, where run_ea gives each span a whole iteration:
// 0.75-3 TiB/s) and wins on 4-8 KiB SST-packed spans; run_ea -- round 2's
// lean one-span-per-iteration loop -- is 2-6 % faster on aligned 4 KiB
// blocks, table blocks (4 KiB + a front of <= 16 chunks), ReadBlock's 4 KiB
// blocks and spans of >= 16 KiB (same-session A/Bs).
// Every wave of every workgroup samples the same 64 spans spread over the
// batch (one vector load per lane) and takes run_ea only when all of them
// suit it, so a workgroup's waves always agree (the two pipelines use the
// LDS aux column differently) and a mixed batch stays on run_lp.  The choice
// changes speed only: both compute every span exactly.
// ---------------------------------------------------------------------------
// kLong: the chunks from which a span counts as long (16 KiB; the packed
// kernel and its pre-pass: 32 KiB -- spans of 16..32 KiB run faster
// streamed, 5941-5947 vs 5535-5558 GiB/s on config 3's 16 KiB bucket, while
// 32 KiB ones do not, 5835-5844 vs 5977-5985, same session,
// profiles/r06q_pick_ab.log)
template <bool kV, uint32_t kLong = 4u * kSegChunks, typename Src>
__device__ __forceinline__ bool pick_ea(const Src& src) {
  const uint32_t l = lane_tid() & 63u;
  const uint64_t count = src.count;
  const uint64_t s = (count * l) >> 6;  // (count < 2^31: no overflow)
  uint64_t a = 0;
  uint32_t n = 0, init = 0;
  src.lane(s, a, n, init);
  const Plan p = MakePlan(a, static_cast<uint32_t>(reinterpret_cast<uint64_t>(src.base) + a),
                          src.bytes(n), kV);
  // one segment + a front of <= 16 chunks (run_ea's batched pieces), or a
  // span of >= 16 KiB
  const bool ok = p.empty || (p.C >= kSegChunks && p.C <= kSegChunks + 16u) || p.C >= kLong;
  return pipeline_marker(ballot(!ok) == 0u);
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
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image,
    const uint32_t* __restrict__ bounds, unsigned int* fault) {
  const DescSrc<INIT != 0> src{base, offsets, lengths, inits, count, 0u, bounds};
  if (pick_ea<false>(src)) run_ea<0>(src, out, flags, image);
  else run_lp<0>(src, out, flags, image, fault);
}
template __global__ void crc32c_lds_spans_kernel<0>(const uint8_t*, const uint64_t*,
                                                    const uint32_t*, const uint32_t*, uint32_t*,
                                                    uint64_t, uint32_t, const uint8_t*,
                                                    const uint32_t*, unsigned int*);
template __global__ void crc32c_lds_spans_kernel<1>(const uint8_t*, const uint64_t*,
                                                    const uint32_t*, const uint32_t*, uint32_t*,
                                                    uint64_t, uint32_t, const uint8_t*,
                                                    const uint32_t*, unsigned int*);

// the packed kernel's (and its pre-pass's) long-span bound for run_ea
constexpr uint32_t kPsLongChunks = 8u * kSegChunks;

// Packed batch (HCRC_PACKED, crc32c_ps.h): run_ea when the batch suits it
// (pick_ea: aligned 4 KiB blocks, table blocks, spans of >= 16 KiB -- where it
// is 4-7 % faster than run_ps, profiles/r05v_ab.log), else run_ps when the
// pre-pass found the batch packed (meta[0] == epoch << 4: this launch's
// verdict, nothing broken), else the lane-packed pipeline -- a broken
// promise (or a verdict that is not this launch's) costs speed, never a
// CRC.  first / C: the chunk index.
template <int INIT>
__global__ __launch_bounds__(kThreads) void crc32c_lds_packed_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image,
    const uint32_t* __restrict__ first, const uint32_t* __restrict__ meta, uint32_t C,
    uint32_t epoch, unsigned int* fault, unsigned int* hint) {
  const DescSrc<INIT != 0> src{base, offsets, lengths, inits, count, 0u, nullptr};
  // the pre-pass's verdict back to the host (hcrc_api.cc PsScratch::h_hint:
  // a repeated batch that suits run_ea or is not packed skips the pass next
  // time); a plain system-scope store, as the fault words
  if (hint != nullptr && group_id() == 0u && lane_tid() == 0u) {
#if !defined(WIPDB_LK_EMU)
    __hip_atomic_store(hint, meta[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
    *hint = meta[0];
#endif
  }
  if ((flags & kFlagPsOnly) == 0u && pick_ea<false, kPsLongChunks>(src))
    run_ea<0>(src, out, flags & kFlagMask, image);
  else if (meta[0] != epoch << 4) run_lp<0>(src, out, flags & kFlagMask, image, fault);
  else run_ps(src, out, flags, image, first, C, fault);
}
template __global__ void crc32c_lds_packed_kernel<0>(const uint8_t*, const uint64_t*,
                                                     const uint32_t*, const uint32_t*, uint32_t*,
                                                     uint64_t, uint32_t, const uint8_t*,
                                                     const uint32_t*, const uint32_t*, uint32_t,
                                                     uint32_t, unsigned int*, unsigned int*);
template __global__ void crc32c_lds_packed_kernel<1>(const uint8_t*, const uint64_t*,
                                                     const uint32_t*, const uint32_t*, uint32_t*,
                                                     uint64_t, uint32_t, const uint8_t*,
                                                     const uint32_t*, const uint32_t*, uint32_t,
                                                     uint32_t, unsigned int*, unsigned int*);

// The packed batch's pre-pass (crc32c_ps.h ps_index); epoch: the launch's
// tag of the verdict word (1 .. 2^28 - 1, the host's per-stream count).
// kPsIndexThreads threads a workgroup, kPsIndexLds bytes of LDS.  A batch
// that suits run_ea (the packed kernel's own pick_ea, the same 64 sampled
// spans) is not checked or indexed at all: the packed kernel takes run_ea
// before it reads either, so the pass stops after its sample (aligned
// blocks, table blocks, spans of >= 16 KiB: the flag then costs one short
// launch, not a pass over the descriptors -- VERDICT r5 weak item 6).
__global__ __launch_bounds__(kPsIndexThreads) void crc32c_ps_index_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint64_t count, uint32_t C, uint32_t* __restrict__ first,
    uint32_t* __restrict__ meta, uint32_t epoch, uint32_t flags) {
  if ((flags & kFlagPsOnly) == 0u) {
    const DescSrc<false> src{base, offsets, lengths, nullptr, count, 0u, nullptr};
    if (pick_ea<false, kPsLongChunks>(src)) {
      if (group_id() == 0u && lane_tid() == 0u) global_max(meta, (epoch << 4) | kPsEa);
      return;
    }
  }
  const uint64_t nt = static_cast<uint64_t>(group_count()) * kPsIndexThreads;
  const uint64_t tid = static_cast<uint64_t>(group_id()) * kPsIndexThreads + lane_tid();
  ps_index(nullptr, offsets, lengths, count, C, first, meta, tid, nt, epoch);
}

// Fixed-size blocks at a fixed stride.
__global__ __launch_bounds__(kThreads) void crc32c_lds_strided_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t length, uint32_t init,
    uint32_t* __restrict__ out, uint64_t count, uint32_t flags, const uint8_t* __restrict__ image,
    unsigned int* fault) {
  const StridedSrc src{base, stride, length, init, count};
  if ((flags & kFlagPsOnly) == 0u && pick_ea<false>(src)) run_ea<0>(src, out, flags & kFlagMask, image);
  else run_lp<0>(src, out, flags & kFlagMask, image, fault);
}

// Read-side verify (ReadBlock, kv/src/table/format.cc:91-99): block i =
// base + offsets[i], handle size n = lengths[i]; CRC over n + 1 bytes
// compared with Unmask(LE32 at n + 1).
__global__ __launch_bounds__(kThreads) void crc32c_lds_verify_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint8_t* __restrict__ status, uint64_t count,
    const uint8_t* __restrict__ image, unsigned int* fault) {
  const DescSrc<false> src{base, offsets, lengths, nullptr, count, 1u, nullptr};
  if (pick_ea<true>(src)) run_ea<1>(src, status, 0u, image);
  else run_lp<1>(src, status, 0u, image, fault);
}

#if !defined(WIPDB_LK_EMU)
// The memory side of run_ea alone -- the roofline's same-box ceiling
// (hcrc_dma_ceiling_async).  Everything run_ea does with
// memory on fixed-size 4 KiB blocks, nothing else: the 96 KiB table image
// into LDS, the same unit deal (wg_units / grab_unit), the same four
// 1 KiB global_load_lds_dwordx4 per block into the wave's slot (pp.cm's
// rotated chunk order), the next block's DMA issued right after the slot is
// read, the same slot reads, and 4 bytes stored per block. No CRC: the word
// stored for block b is the XOR of its first 64 bytes (lane 0's stripe).
// length must be 4096 (the host checks).
__global__ __launch_bounds__(kThreads) void crc32c_dma_ceiling_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t* __restrict__ out, uint64_t count,
    const uint8_t* __restrict__ image) {
  const uint32_t l = lane_tid() & 63u;
  const uint32_t w = uni(lane_tid() >> 6);
  const WgUnits units = wg_units(count, nullptr);
  if (units.count == 0u) return;
  load_image(image, w, l);
  Pipe pp;
  pp.init(l, w);
  const uint64_t sbase = reinterpret_cast<uint64_t>(base);
  const uint32_t o = 16u * pp.cm;
  uint64_t s = grab_unit(l, units);
  if (s >= count) return;
  dma4(sbase + s * stride, pp.slot, o, o + 1024u, o + 2048u, o + 3072u);
  uint64_t nx = grab_unit(l, units);
  g_u32* const out32 = (g_u32*)(reinterpret_cast<uintptr_t>(out));
  bool stored_prev = false;
  for (;;) {
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    uint32_t W[16];
    pp.read(W);
    pp.release();
    const uint64_t cur = s;
    s = nx;
    if (s < count) {
      dma4(sbase + s * stride, pp.slot, o, o + 1024u, o + 2048u, o + 3072u);
      nx = grab_unit(l, units);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= W[i];
    if (l == 0u) out32[cur] = acc;
    stored_prev = true;
    if (s >= count) break;
  }
}
#endif

}  // namespace lk
}  // namespace wipdb

#if !defined(WIPDB_LK_EMU)
// Sets a launch's fault word as a faulting wave does (the test build's
// WIPDB_HCRC_FORCE_FAULT launches it after each lane-packed launch).
__global__ void crc32c_lds_fault_probe_kernel(unsigned int* fault) {
  if (threadIdx.x == 0) wipdb::lk::report_fault(fault, wipdb::lk::kFaultQueuePop);
}
#endif

#if defined(WIPDB_LP_PROF) && !defined(WIPDB_LK_EMU)
// Profiling build only: copies (and with reset != 0 zeroes) g_lp_prof.
extern "C" __attribute__((visibility("default"))) int hcrc_debug_lp_prof(void* host, uint64_t bytes,
                                                                          int reset) {
  if (bytes > sizeof(unsigned long long) * 4096 * wipdb::lk::kProfN) return -1;
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(wipdb::lk::g_lp_prof), bytes) != hipSuccess)
    return -2;
  if (reset) {
    static unsigned long long zero[4096 * wipdb::lk::kProfN];
    if (hipMemcpyToSymbol(HIP_SYMBOL(wipdb::lk::g_lp_prof), zero, sizeof(zero)) != hipSuccess)
      return -3;
  }
  return 0;
}
#endif
