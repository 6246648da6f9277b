// crc32c_plan.h -- span plans of the lane-packed CRC32C kernels
// (crc32c_lds.hip, run_lp): how a span is cut into full 4 KiB segments and a
// lane-packed back piece, and the byte ranges every DMA of it reads.  Host +
// device: the kernels use it, and tests/cpp/test_plan.cc runs the same code
// on the host -- every DMA source checked against the span's pages, and the
// kernel's arithmetic replayed with a byte-serial CRC -- before a geometry
// change reaches a GPU.  DESIGN.md section 4.
//
// The grid.  A span of n bytes at s ends at E = s + n; E4 = E rounded down
// to a 4-byte address boundary.  The k = E - E4 <= 3 trailing bytes are the
// span's tail; the body [s, E4) is cut into C = ceil((E4 - s) / 16) chunks
// whose grid ENDS at E4: chunk j = [E4 - 16 (C - j), +16).  Every chunk
// starts on a 4-byte boundary (global_load_lds_dwordx4 at dword alignment
// costs ~2 % over 16-byte alignment, at byte alignment 30-40 %), and only
// chunk 0 is partial: its hp = 16 C - (E4 - s) leading bytes are not the
// span's and are masked -- or, when reading them could cross into the page
// below s, chunk 0 is read ws words late (from s rounded down to 4) and
// shifted.  A verify span (ReadBlock: contents + type byte, then the 4-byte
// stored crc) has no tail: its grid runs on over the trailer to the next
// 4-byte boundary (jv <= 3 bytes past it) and the trailer is checked through
// the CRC residue (fix_trailer / verify_residue).
//
// The plan.  m = C / 256 full segments FROM THE START of the grid (segment t
// = chunks [256 t, 256 t + 256), one wave iteration each, chained by the
// register; segment 0 carries the head), then a BACK PIECE of r = C mod 256
// chunks (a span of fewer than 256 chunks is all piece, head included).  A
// piece does not get a 4 KiB window of its own: pieces queue in the wave's
// piece ring and one wave iteration checksums as many of them as fit in its
// 64 lanes -- a piece takes nl = ceil((r + x) / 4) lanes, x = 1 when it needs
// its aux chunk (the 16 bytes holding its tail word) -- each lane a 64-byte
// stripe of the piece's window, END-aligned at the piece's last chunk.  The
// front = 4 nl - r window chunks in front of the piece are zeroed (window
// chunk 0 holds the aux chunk when x), the piece's register is folded over
// its lanes (shift by 64 (nl - 1 - j) bytes, then a segmented XOR), and its
// leader lane finishes the span: one slicing step for the tail, the output.
// A back piece enters with the register of the segments before it (its
// "inj"), a whole-span piece with the head register ~init * x^(-8 hp).
#pragma once
#include <stdint.h>

#include "crc32c_lds.h"

namespace wipdb {
namespace lk {

// A span as a source hands it out (all values uniform).
struct SpanD {
  uint64_t a;      // offset of the first byte from the source base
  uint32_t n;      // bytes
  uint32_t init;   // Extend's init_crc
  uint32_t id;     // output slot (launches hold < 2^31 spans)
};

// Byte mask of word ww of chunk 0: its first h bytes are not the span's.
WIPDB_LK_HD inline uint32_t head_mask(uint32_t h, uint32_t ww) {
  return h >= 4u * ww + 4u ? 0u : (h <= 4u * ww ? ~0u : (~0u << (8u * (h - 4u * ww))));
}

// ---- piece word: the packed geometry of a piece (ring entry) ----
//   r (8) | x << 8 | hp (4) << 9 | ws (2) << 13 | te (4) << 15 | k (2) << 19 |
//   jv (2) << 21 | cont << 23 | j0 (6) << 24
// r: the piece's chunks; x: the aux chunk is read (the span has a tail);
// hp / ws: head bytes masked / words read late (a whole-span piece only);
// te: the byte of the aux chunk where the tail word starts (the aux chunk
// is the 16 bytes at E4 - te); k: tail bytes; jv: verify grid bytes past
// the trailer.  The piece's first real chunk is at p0 = E4 - 16 r.  cont /
// j0: the kernel split the piece over two batch iterations and lanes
// [j0, nl) of it are still to come (the register of lanes [0, j0) is carried).
constexpr uint32_t kPWCont = 1u << 23;
struct PW {
  uint32_t v;
  WIPDB_LK_HD inline uint32_t r() const { return v & 0xffu; }
  WIPDB_LK_HD inline uint32_t x() const { return (v >> 8) & 1u; }
  WIPDB_LK_HD inline uint32_t hp() const { return (v >> 9) & 15u; }
  WIPDB_LK_HD inline uint32_t ws() const { return (v >> 13) & 3u; }
  WIPDB_LK_HD inline uint32_t te() const { return (v >> 15) & 15u; }
  WIPDB_LK_HD inline uint32_t k() const { return (v >> 19) & 3u; }
  WIPDB_LK_HD inline uint32_t jv() const { return (v >> 21) & 3u; }
  WIPDB_LK_HD inline bool cont() const { return (v & kPWCont) != 0u; }
  WIPDB_LK_HD inline uint32_t j0() const { return (v >> 24) & 63u; }
  // lanes of the piece, and its window chunks in front of it
  WIPDB_LK_HD inline uint32_t nl() const { return (r() + x() + 3u) >> 2; }
  WIPDB_LK_HD inline uint32_t front() const { return 4u * nl() - r(); }
  // lanes still to come, and the word once `taken` more of them were batched
  WIPDB_LK_HD inline uint32_t rem() const { return nl() - j0(); }
  WIPDB_LK_HD inline uint32_t advanced(uint32_t taken) const {
    return (v & ~(63u << 24)) | kPWCont | ((j0() + taken) << 24);
  }
};
WIPDB_LK_HD inline uint32_t PackPW(uint32_t r, uint32_t x, uint32_t hp, uint32_t ws, uint32_t te,
                                   uint32_t k, uint32_t jv) {
  return r | (x << 8) | (hp << 9) | (ws << 13) | (te << 15) | (k << 19) | (jv << 21);
}

// The plan of one span.
struct Plan {
  uint64_t c0;    // offset (from the source base) of grid chunk 0 (= s - hp)
  uint64_t p0;    // offset of the piece's first chunk (c0 + 4096 m = E4 - 16 r)
  uint32_t C;     // body chunks
  uint32_t m;     // full segments
  uint32_t hp, ws, k, jv;
  uint32_t pw;    // the piece word (0: no piece)
  uint32_t seg_aux;  // m > 0, no piece, a tail: the last segment reads the aux chunk at c0 + 16 C - 12
  bool empty;     // a CRC span of 0 bytes: out = init, nothing read
};

// s_lo: the low 32 bits of the span's absolute address (sbase + a).
WIPDB_LK_HD inline Plan MakePlan(uint64_t a, uint32_t s_lo, uint32_t n, bool verify) {
  Plan p;
  uint32_t k, nb, jv = 0;
  if (verify) {
    // the grid takes the stored trailer and ends at the first 4-byte
    // boundary at or after it: jv <= 3 bytes past it, in its last word
    jv = (0u - (s_lo + n + 4u)) & 3u;
    k = 0;
    nb = n + 4u + jv;
  } else {
    const uint32_t e3 = (s_lo + n) & 3u;
    k = e3 < n ? e3 : n;  // tail bytes
    nb = n - k;           // body bytes [s, E4)
  }
  const uint32_t C = (nb + 15u) >> 4;
  const uint32_t hp = (C << 4) - nb;
  const uint32_t pg = s_lo & 4095u;
  // reading hp bytes in front of s would leave its page: read chunk 0 from
  // s rounded down to 4, i.e. ws = (hp - s % 4) / 4 words late
  const uint32_t ws = pg < hp ? (hp - (pg & 3u)) >> 2 : 0u;
  p.c0 = a - hp;
  p.C = C;
  p.m = C >> 8;
  p.hp = hp;
  p.ws = ws;
  p.k = k;
  p.jv = jv;
  p.empty = !verify && n == 0u;
  p.seg_aux = 0;
  const uint32_t r = C & 255u;
  p.p0 = p.c0 + 4096u * static_cast<uint64_t>(p.m);
  p.pw = 0;
  if (p.m != 0u && r == 0u) {
    p.seg_aux = k != 0u ? 1u : 0u;  // aux chunk: c0 + 16 C - 12 (16 bytes ending at E4 + 4)
    return p;
  }
  if (p.empty) return p;
  // the piece: the whole span (m = 0, head included) or the chunks after
  // the segments (no head).  x: its aux chunk, the 16 bytes ending at the
  // 4-byte word that holds the span's last byte -- or, when those would
  // start in the page below a short span, from s rounded down to 4 (a span
  // of < 12 body bytes).  E4 = s + nb: the tail word starts te bytes into
  // the aux chunk (a span inside one word has E4 = s, unaligned, and r = 0).
  const uint32_t x = k != 0u ? 1u : 0u;
  uint32_t te = 0;
  if (x) {
    const uint32_t e_lo = s_lo + n;
    const uint32_t a_lo = ((e_lo + 3u) & ~3u) - 16u;  // may precede s (short spans)
    const uint32_t before = s_lo - a_lo;              // bytes in front of s (mod 2^32)
    const uint32_t a_fix = (before <= 16u && before > pg) ? (s_lo & ~3u) : a_lo;
    te = (e_lo - k - a_fix) & 15u;
  }
  const bool whole = p.m == 0u;
  p.pw = PackPW(r, x, whole ? hp : 0u, whole ? ws : 0u, te, k, jv);
  return p;
}

// ---- plan word: what a wave needs of a span with segments besides its
// address (c0 = a - hp) and piece word, packed so a desk lane hands it over
// in one readlane:  hp (4) | ws (2) << 4 | k (2) << 6 | jv (2) << 8 |
// seg_aux << 10 | m << 11  (the low 10 bits are a segment's `hw`).
WIPDB_LK_HD inline uint32_t PackPL(const Plan& p) {
  return p.hp | (p.ws << 4) | (p.k << 6) | (p.jv << 8) | (p.seg_aux << 10) | (p.m << 11);
}
WIPDB_LK_HD inline uint32_t PL_hp(uint32_t pl) { return pl & 15u; }
WIPDB_LK_HD inline uint32_t PL_ws(uint32_t pl) { return (pl >> 4) & 3u; }
WIPDB_LK_HD inline uint32_t PL_hw(uint32_t pl) { return pl & 1023u; }
WIPDB_LK_HD inline uint32_t PL_aux(uint32_t pl) { return (pl >> 10) & 1u; }
WIPDB_LK_HD inline uint32_t PL_m(uint32_t pl) { return pl >> 11; }

// ---- the batch window of a piece (lanes j = 0 .. nl - 1 of its group) ----
// Window chunk w (0 .. 4 nl - 1) of the piece with first real chunk at p0:
// w > front reads p0 + 16 (w - front); w == front, its first real chunk,
// reads p0 + 4 ws (ws words late: fix_head shifts it back); the in-front
// chunks (zeroed later) read the aux chunk p0 + 16 r - te when x -- window
// chunk 0 is always in front then, and its words are where lane 0 finds
// the tail word -- else p0 + 4 ws.  Returned as a byte offset from p0.
WIPDB_LK_HD inline int64_t PieceChunkSrc(PW pw, uint32_t w) {
  const uint32_t front = pw.front();
  if (w > front) return 16 * static_cast<int64_t>(w - front);
  if (w < front && pw.x()) return 16 * static_cast<int64_t>(pw.r()) - static_cast<int64_t>(pw.te());
  return 4 * static_cast<int64_t>(pw.ws());
}

// The per-lane stripe descriptor the batch DMA hands between lanes: S = the
// source of window chunk 4 j were the window linear, p0 + 16 (4 j - front),
// and info = fr (3) | real0 << 3 | ws (2) << 4 | dIF << 6: fr = the
// stripe's in-front chunks (lane 0's only, <= 4), real0: its chunk fr is the
// piece's first real chunk (read ws words late), dIF = the in-front chunks'
// source relative to S.
struct Stripe {
  int64_t s;  // relative to p0
  uint32_t info;
};
WIPDB_LK_HD inline Stripe MakeStripe(PW pw, uint32_t j) {
  const int32_t f = static_cast<int32_t>(pw.front()) - 4 * static_cast<int32_t>(j);
  const uint32_t fr = f <= 0 ? 0u : static_cast<uint32_t>(f);
  const uint32_t real0 = (f >= 0 && f < 4 && pw.r() != 0u) ? 1u : 0u;
  Stripe st;
  st.s = -16 * static_cast<int64_t>(f);
  const int64_t dif = (pw.x() ? 16 * static_cast<int64_t>(pw.r()) - static_cast<int64_t>(pw.te())
                              : 4 * static_cast<int64_t>(pw.ws())) - st.s;
  st.info = fr | (real0 << 3) | (pw.ws() << 4) | (fr ? static_cast<uint32_t>(dif) << 6 : 0u);
  return st;
}
// The source of chunk i (0..3) of a stripe, relative to its S.
WIPDB_LK_HD inline int64_t StripeChunkSrc(uint32_t info, uint32_t i) {
  const uint32_t fr = info & 7u;
  if (i < fr) return static_cast<int64_t>(info >> 6);
  return 16 * static_cast<int64_t>(i) + ((i == fr && (info & 8u)) ? 4 * ((info >> 4) & 3u) : 0u);
}

// ---- verify: the CRC residue ----
// A verify span's grid ends jv <= 3 bytes past its stored trailer, so the
// last 8 bytes of its last segment or piece -- words 14 and 15 of the last
// lane -- hold the trailer at byte 4 - jv.  fix_trailer unmasks it in place
// and zeroes the jv bytes after it; the register after the block ||
// Unmask(trailer) || jv zero bytes is then the constant verify_residue(jv)
// exactly when the trailer matches (feeding a word w: r -> zero-feed(r ^ w,
// 4), and r ^ crc = ~0 for the register r = ~crc of the block; zero-feeds
// are bijections), so no lane needs the trailer as a value.
WIPDB_LK_HD constexpr uint32_t verify_residue(uint32_t jv) {
  uint32_t r = ~0u;
  for (uint32_t i = 0; i < 8u * (4u + jv); ++i) r = (r >> 1) ^ (0x82f63b78u & (0u - (r & 1u)));
  return r;
}
WIPDB_LK_HD inline void fix_trailer(uint32_t& lo, uint32_t& hi, uint32_t jv) {
  const uint64_t x = static_cast<uint64_t>(lo) | (static_cast<uint64_t>(hi) << 32);
  const uint32_t sh = 8u * (4u - jv);  // 8 .. 32
  const uint32_t r = static_cast<uint32_t>(x >> sh) - 0xa282ead8u;
  const uint32_t c = (r >> 17) | (r << 15);
  const uint64_t y = (x & ((uint64_t(1) << sh) - 1u)) | (static_cast<uint64_t>(c) << sh);
  lo = static_cast<uint32_t>(y);
  hi = static_cast<uint32_t>(y >> 32);
}

// Chunk 0 of a span into its span form: read ws words late (shift right by
// ws words), its hp leading bytes masked, the register inj entering at its
// first byte.  Per lane.
WIPDB_LK_HD inline void fix_head(uint32_t (&c)[4], uint32_t hp, uint32_t ws, uint32_t inj) {
  uint32_t d[4];
  d[3] = ws == 0u ? c[3] : (ws == 1u ? c[2] : (ws == 2u ? c[1] : c[0]));
  d[2] = ws == 0u ? c[2] : (ws == 1u ? c[1] : (ws == 2u ? c[0] : 0u));
  d[1] = ws == 0u ? c[1] : (ws == 1u ? c[0] : 0u);
  d[0] = ws == 0u ? c[0] : 0u;
  for (uint32_t w = 0; w < 4; ++w) c[w] = d[w] & head_mask(hp, w);
  c[0] ^= inj;
}

}  // namespace lk
}  // namespace wipdb
