// crc32c_list.hip -- the size-class list kernels (HCRC_SPLIT_SMALL) and the
// class-1 list kernel of the long-span split (HCRC_SPLIT_LONG): a partition
// pass sorts a batch into lists, each list runs one kernel.  These predate
// the lane-packed spans kernel (crc32c_lds.hip), which handles every span
// size in one launch; they stay as the opt-in flag paths of the C-ABI.
//
//   * run_ea: the end-aligned pipeline -- a span's segments END-aligned at
//     its last chunk, the first one partial (window chunks in front of it
//     zeroed), table blocks as a main segment + a front piece batched 16 per
//     iteration in 4-lane groups (crc32c_walk.h);
//   * run_g: G = 2 / 4 spans of at most 128 / 64 chunks per wave iteration,
//     one per group of 64 / G lanes, a start-aligned grid with ragged tails.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32c_dev.h"
#include "crc32c_walk.h"

namespace wipdb {
namespace lk {

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
