// crc32c_walk.h -- the span geometry of the LDS-staged CRC32C kernels
// (crc32c_lds.hip): the end-aligned chunk grid, its segments and front
// pieces, and the byte ranges every DMA of a span reads.  Host + device: the
// kernels use it, and tests/cpp/test_walk.cc runs the same code on the host
// -- every DMA source of every lane checked against the span's pages, and
// the kernel's arithmetic replayed with a byte-serial CRC -- so a geometry
// change is checked before it reaches a GPU.  DESIGN.md section 4.
#pragma once
#include <stdint.h>

#include "crc32c_lds.h"
#include "crc32c_plan.h"

namespace wipdb {
namespace lk {

// ---------------------------------------------------------------------------
// The descriptor / strided / verify pipeline: the END-ALIGNED GRID.
//
// A span of n bytes at s ends at E = s + n; E4 = E rounded down to a 4-byte
// boundary (of the address).  The k = E - E4 <= 3 trailing bytes are the
// span's tail; the body [s, E4) is cut into C = ceil((E4 - s) / 16) chunks
// whose grid ENDS at E4: chunk j = [E4 - 16 (C - j), +16), so every chunk
// starts on a 4-byte boundary (global_load_lds_dwordx4 at dword alignment
// costs ~2 % over 16-byte alignment; at byte alignment 30-40 %,
// scripts/probes/dma_align_probe.hip, scripts/probe_shapes.py) and only
// chunk 0 is partial: hp = 16 C - (E4 - s) of its leading bytes are not the
// span's and are masked -- or, when reading them could cross into the page
// below s, chunk 0 is read from s rounded down to 4 and shifted right by whole
// words before the mask.  The tail is ONE slicing step:
//   reg' = T-step((reg ^ tail word) << 8 (4 - k)) ^ (reg >> 8 k),
// with the tail word in 16 bytes read with the last segment.  A verify span
// has no tail: its grid runs on over the 4-byte stored trailer to the next
// 4-byte boundary, and the trailer is checked through the CRC residue
// (fix_trailer).  Nothing outside [s, E) (+ the trailer of a verify span) is
// read, except within the 4-byte words holding s and E.
//
// Segments are 256-chunk windows END-aligned at their last chunk: the first
// covers chunks [0, C - 256 (m - 1)), the m - 1 others 256 each, chained by
// the register.  A span of 257..271 chunks (a table block: 4 KiB + its last
// entry + the type byte) is instead ONE full main segment -- its last 256
// chunks, from a zero register -- plus a front piece of its first 1..15
// chunks, which joins the wave's piece ring: entry k in lane k of six
// VGPRs.  Once 16 are pending (or the wave runs out of segments), one
// iteration CRCs them all, a piece per 4-lane group (a 16-chunk window each,
// four per DMA instruction with per-lane addresses), folded within the group
// (level 1 + DPP), and finishes each span by linearity:
//   register = piece register * x^(8 * 4096) ^ main register, then the tail.
// ---------------------------------------------------------------------------
constexpr uint32_t kEValid = 1u, kEFirst = 2u, kELast = 4u, kEMain = 8u, kEBatch = 16u,
                   kENoBody = 32u, kEAux = 64u, kESimple = 128u;
constexpr uint32_t kPieceChunks = 16;  // a piece window: 4 lanes x 4 chunks
constexpr uint32_t kPieceMax = 15;     // piece chunks: window chunk 0 stays free for the aux chunk
constexpr uint32_t kBatch = 16;        // pieces per batch iteration

// A segment as issued (DMA sources) and as computed (the packed SegC, the
// only part kept live across the iteration: SGPRs are the kernel's scarce
// resource).
//   g1: flags (8) | front (9) << 8 | hp (4) << 17 | ws (2) << 21 | k (2) << 23 |
//       te (4) << 25
//   g2: jv (2) | main: the front piece's chunks (5) << 4 | its hp (4) << 9 |
//       its ws (2) << 13
struct SegC {
  uint32_t g1, g2;
  uint32_t init;  // first segment / main: the span's init (batch: ring head)
  uint32_t id;    // output slot (batch: the number of pieces)
  uint64_t c0;    // main: offset of the span's chunk 0 (the piece's)
  WIPDB_LK_HD inline uint32_t flags() const { return g1 & 0xffu; }
  WIPDB_LK_HD inline uint32_t front() const { return (g1 >> 8) & 0x1ffu; }
  WIPDB_LK_HD inline uint32_t hp() const { return (g1 >> 17) & 15u; }
  WIPDB_LK_HD inline uint32_t ws() const { return (g1 >> 21) & 3u; }
  WIPDB_LK_HD inline uint32_t k() const { return (g1 >> 23) & 3u; }
  WIPDB_LK_HD inline uint32_t te() const { return (g1 >> 25) & 15u; }
  WIPDB_LK_HD inline uint32_t jv() const { return g2 & 3u; }  // verify: grid bytes past the trailer
  WIPDB_LK_HD inline uint32_t r() const { return (g2 >> 4) & 31u; }
  WIPDB_LK_HD inline uint32_t php() const { return (g2 >> 9) & 15u; }
  WIPDB_LK_HD inline uint32_t pws() const { return (g2 >> 13) & 3u; }
  // the ring word of a main segment's front piece
  WIPDB_LK_HD inline uint32_t piece_word() const { return r() | (php() << 8) | (pws() << 12) | (k() << 14); }
};
struct SegE {
  SegC c;
  uint64_t wb;    // offset (from the source base) of window chunk 0
  uint64_t ax;    // last: offset of the 16 bytes holding the tail word
  uint32_t src0;  // DMA offset (from wb) of the span's chunk 0, also read by the in-front lanes
};

// The two common span shapes without the walk (scalar work per span is the
// kernels' scarce resource):
//   * a SIMPLE span, one whole 256-chunk window: a 4-byte aligned start and a
//     body (+ the verify trailer) of exactly 4096 bytes -- hp = ws = k = 0,
//     no piece, no aux chunk (the aligned 4 KiB block; ReadBlock on a
//     4091-byte block).  g1 = kEValid | kEFirst | kELast | kESimple;
//   * a TABLE BLOCK, 257..271 chunks: one full main segment + a front piece.
// Fills the segment (and its window base wb) exactly as WalkE::start + next
// would -- tests/cpp/test_walk.cc checks it -- except for the kESimple flag
// and a main segment's te (unused there: its tail rides with the piece).
// Returns false for any other shape: the walk takes it.
WIPDB_LK_HD inline bool FastSeg(uint64_t sbase, const SpanD& d, bool verify, SegC& c, uint64_t& wb) {
  const uint32_t n = d.n;
  const uint32_t s_lo = static_cast<uint32_t>(sbase) + static_cast<uint32_t>(d.a);
  uint32_t k, nb, jv;
  if (verify) {
    jv = (0u - (s_lo + n + 4u)) & 3u;
    k = 0;
    nb = n + 4u + jv;
  } else {
    jv = 0;
    const uint32_t e3 = (s_lo + n) & 3u;
    k = e3 < n ? e3 : n;
    nb = n - k;
  }
  const uint32_t C = (nb + 15u) >> 4;
  const uint32_t hp = (C << 4) - nb;
  c.init = d.init;
  c.id = static_cast<uint32_t>(d.id);
  if (C == kSegChunks && (hp | k) == 0u) {
    c.g1 = kEValid | kEFirst | kELast | kESimple;
    c.g2 = jv;
    c.c0 = d.a;
    wb = d.a;
    return true;
  }
  if (C - (kSegChunks + 1u) >= kPieceMax) return false;  // not 257..271
  const uint32_t pg = s_lo & 4095u;
  const uint32_t ws = pg < hp ? (hp - (pg & 3u)) >> 2 : 0u;
  const uint32_t nc0 = C - kSegChunks;
  c.c0 = d.a - hp;
  wb = c.c0 + 16u * nc0;
  c.g1 = kEValid | kELast | kEMain | (k << 23);
  c.g2 = jv | (nc0 << 4) | (hp << 9) | (ws << 13);
  return true;
}

struct WalkE {
  uint64_t c0;
  uint32_t axd;   // the aux chunk at c0 + (int32) axd
  uint32_t id, init;
  // hp | ws << 4 | k << 6 | te << 8 | jv << 12 | piece << 16 | no body << 17 |
  // nc0 << 18 (chunks of the first segment; piece: the piece's)
  uint32_t geo;
  uint32_t j, nseg;
  bool valid;

  // sbase: the source base address; verify: the span is followed by a
  // 4-byte trailer, which the grid takes in.  Scalar work per span is the
  // kernels' scarce resource (one scalar unit per CU serves 16 waves): the
  // rare parts -- the aux chunk, a head read late, pieces, several segments
  // -- sit behind uniform branches.
  WIPDB_LK_HD inline void start(uint64_t sbase, const SpanD& d, bool verify) {
    const uint32_t n = d.n;
    const uint32_t s_lo = static_cast<uint32_t>(sbase) + static_cast<uint32_t>(d.a);
    uint32_t k, nb, jv = 0;
    if (verify) {
      // the grid takes the stored trailer and ends at the first 4-byte
      // boundary at or after it: jv <= 3 bytes past it, in its last word
      const uint32_t e_lo = s_lo + n + 4u;
      jv = (0u - e_lo) & 3u;
      k = 0;
      nb = n + 4u + jv;
    } else {
      const uint32_t e3 = (s_lo + n) & 3u;
      k = e3 < n ? e3 : n;  // tail bytes
      nb = n - k;           // body bytes [s, E4)
    }
    const uint32_t C = (nb + 15u) >> 4;
    const uint32_t hp = (C << 4) - nb;
    c0 = d.a - hp;
    init = d.init;
    id = static_cast<uint32_t>(d.id);
    j = 0;
    valid = true;
    geo = hp | (k << 6) | (jv << 12);
    const uint32_t pg = s_lo & 4095u;
    // reading hp bytes in front of s would leave its page: read chunk 0 from
    // s rounded down to 4, i.e. ws = (hp - s % 4) / 4 words late
    if (pg < hp) geo |= ((hp - (pg & 3u)) >> 2) << 4;
    uint32_t nc0;
    if (C <= kSegChunks) {
      nseg = 1;
      nc0 = C;
      if (C == 0u) geo |= 1u << 17;
    } else if (C <= kSegChunks + kPieceMax) {
      nseg = 1;
      nc0 = C - kSegChunks;
      geo |= 1u << 16;
    } else {
      nseg = (C + kSegChunks - 1u) / kSegChunks;
      nc0 = C - kSegChunks * (nseg - 1u);
    }
    geo |= nc0 << 18;
    if (k != 0u) {
      // the aux chunk: 16 bytes ending at the 4-byte word that holds the
      // span's last byte -- or, when they would start in the page below a
      // short span, from s rounded down to 4
      const uint32_t e_lo = s_lo + n;
      const uint32_t a_lo = ((e_lo + 3u) & ~3u) - 16u;  // 16 <= n + 3: a_lo may precede s
      const uint32_t before = s_lo - a_lo;              // bytes in front of s (mod 2^32)
      const uint32_t a_fix = (before <= 16u && before > pg) ? (s_lo & ~3u) : a_lo;
      axd = (a_fix - s_lo) + hp;  // from c0 = s - hp
      geo |= ((e_lo - k - a_fix) & 15u) << 8;
    } else {
      axd = 0;
    }
  }
  WIPDB_LK_HD inline SegE next() {
    SegE g;
    const bool last = j + 1u == nseg;
    const uint32_t hp = geo & 15u, ws = (geo >> 4) & 3u, k = (geo >> 6) & 3u;
    const uint32_t nc0 = geo >> 18;
    uint32_t fl = kEValid | (last ? kELast : 0u);
    // (a piece span's tail word comes with its piece, PieceChunkOffset)
    if (last && k != 0u && !(geo & (1u << 16))) fl |= kEAux;
    g.c.init = init;
    g.c.id = id;
    g.c.c0 = c0;
    g.c.g2 = (geo >> 12) & 3u;
    g.ax = c0 + static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(axd)));
    g.src0 = 0;
    uint32_t front = 0, h = 0, w = 0;
    if (geo & (3u << 16)) {
      if (geo & (1u << 17)) {
        fl |= kEFirst | kENoBody;
        g.wb = 0;
      } else {
        fl |= kEMain;
        g.wb = c0 + 16u * nc0;
        g.c.g2 |= (nc0 << 4) | (hp << 9) | (ws << 13);
      }
    } else {
      // the segment's last chunk, and its window's first
      g.wb = c0 + 16u * (nc0 + kSegChunks * j) - 16u * kSegChunks;
      if (j == 0u) {
        fl |= kEFirst;
        front = kSegChunks - nc0;
        h = hp;
        w = ws;
        g.src0 = 16u * front + 4u * ws;
      }
    }
    g.c.g1 = fl | (front << 8) | (h << 17) | (w << 21) | (k << 23) | (((geo >> 8) & 15u) << 25);
    if (last) valid = false;
    ++j;
    return g;
  }
};

// The DMA source of window chunk t (0..255) of a segment, as a byte offset
// from sbase + g.wb: the in-front chunks re-read chunk 0's source.
WIPDB_LK_HD inline uint32_t SegChunkOffset(const SegE& g, uint32_t t) {
  const uint32_t o = 16u * t;
  return o > g.src0 ? o : g.src0;
}

// The DMA source of window chunk t (0..15) of a front piece with ring word
// pw (chunks | hp << 8 | ws << 12 | k << 14), from sbase + its c0.
// Window chunk 0 (always in front of a piece of <= kPieceMax chunks) instead
// reads the span's aux chunk when it has a tail: the 16 bytes ending at the
// 4-byte word holding its last byte, i.e. at offset 16 (C - 1) + 4 from
// chunk 0, C = 256 + piece chunks; the tail word is its last word.  (A
// verify span has no tail: its grid holds the trailer, WalkE::start.)
WIPDB_LK_HD inline uint32_t PieceChunkOffset(uint32_t pw, uint32_t t) {
  if (t == 0u && (pw & (3u << 14)) != 0u) return 16u * (kSegChunks + (pw & 63u)) - 12u;
  const int32_t front = static_cast<int32_t>(kPieceChunks - (pw & 63u));
  const int32_t s0 = static_cast<int32_t>(4u * ((pw >> 12) & 3u));
  const int32_t b = 16 * (static_cast<int32_t>(t) - front);
  return static_cast<uint32_t>(b > s0 ? b : s0);
}

}  // namespace lk
}  // namespace wipdb
