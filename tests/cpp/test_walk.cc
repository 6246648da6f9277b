// tests/cpp/test_walk.cc -- host check of the LDS kernels' span geometry
// (wipdb_amd/csrc/crc32c_walk.h), before any of it reaches a GPU:
//
//   * every DMA source the kernel computes for a span (each window chunk of
//     each segment, each chunk of a front piece, the aux chunk with the tail
//     word / verify trailer) lies in a page that holds a byte of the span (or
//     of its trailer) -- so no geometry can fault on memory the caller did
//     not hand over;
//   * replaying the kernel's arithmetic with those exact sources -- window
//     registers from zero, zeroed in-front chunks, chunk 0 shifted / masked
//     with the head register injected, the chain register of later segments,
//     the one-step tail, the front piece finished by linearity -- with a
//     byte-serial CRC gives Extend(init, span) for every shape, and verify
//     accepts a good trailer and rejects a flipped byte;
//   * FastSeg (the kernels' walk-free path for simple spans and table
//     blocks) yields the same first segment as the walk wherever it applies.
//
// The GPU-only parts (LDS table layout, lane rotation, the fold) are covered
// by the -m gpu parity tests.  Build: g++ -O2 -std=c++17 -I wipdb_amd/csrc.
// Exit 0 = pass.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <set>
#include <vector>

#include "crc32c_walk.h"

using namespace wipdb::lk;

namespace {

wipdb::gf2::Tables T;

uint32_t Feed(uint32_t r, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) r = T.t[0][(r ^ p[i]) & 0xffu] ^ (r >> 8);
  return r;
}
uint32_t FeedZeros(uint32_t r, size_t n) {
  for (size_t i = 0; i < n; ++i) r = T.t[0][r & 0xffu] ^ (r >> 8);
  return r;
}
// the register that becomes ~init after h zero bytes (the kernel's head_register)
uint32_t HeadRegister(uint32_t init, uint32_t h) {
  uint32_t r = ~init;
  for (uint32_t i = 0; i < h; ++i) {
    const uint8_t idx = T.inv_top[r >> 24];
    r = ((r ^ T.t[0][idx]) << 8) | idx;
  }
  return r;
}
uint32_t Mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
uint32_t Unmask(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}
uint32_t Le32(const uint8_t* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

int g_fail = 0, g_cases = 0, g_fast = 0;

struct Case {
  // memory: [kBase, kBase + buf.size()) of absolute addresses
  static constexpr uint64_t kBase = uint64_t(1) << 32;
  std::vector<uint8_t>& buf;
  uint64_t sbase, s_abs;
  uint32_t n, init;
  bool verify;
  std::set<uint64_t> pages;  // pages the span (+ trailer) touches
  bool bad_read = false;

  const uint8_t* Read(uint64_t addr, uint32_t len) {
    for (uint64_t a = addr; a < addr + len; a += 1)
      if (!pages.count(a >> 12)) {
        if (!bad_read)
          fprintf(stderr, "  read [%#llx, +%u) leaves the span's pages (s %#llx n %u v %d)\n",
                  (unsigned long long)addr, len, (unsigned long long)s_abs, n, verify);
        bad_read = true;
        break;
      }
    return &buf[addr - kBase];
  }

  // FastSeg, where it applies, is the walk's one and only segment (bar the
  // kESimple flag and a main segment's unused te).
  void CheckFast(const SpanD& d, WalkE wk) {
    SegC fc;
    uint64_t fwb = 0;
    if (!FastSeg(sbase, d, verify, fc, fwb)) return;
    ++g_fast;
    const SegE g0 = wk.next();
    const uint32_t ign = (fc.flags() & kEMain) ? (15u << 25) : 0u;
    const bool same = !wk.valid && ((fc.g1 & ~kESimple) & ~ign) == (g0.c.g1 & ~ign) &&
                      fc.g2 == g0.c.g2 && fc.init == g0.c.init && fc.id == g0.c.id &&
                      fc.c0 == g0.c.c0 && fwb == g0.wb && g0.src0 == 0u &&
                      !(g0.c.flags() & kEAux) &&
                      ((fc.flags() & kESimple) != 0u) == ((g0.c.flags() & kEMain) == 0u);
    if (!same) {
      if (g_fail < 20)
        fprintf(stderr, "fast s %#llx n %u v %d: g1 %x/%x g2 %x/%x wb %llx/%llx\n",
                (unsigned long long)s_abs, n, verify, fc.g1, g0.c.g1, fc.g2, g0.c.g2,
                (unsigned long long)fwb, (unsigned long long)g0.wb);
      ++g_fail;
    }
  }

  // Returns the kernel's result: the CRC (verify: 1 = good block).
  uint32_t Run() {
    const uint64_t end = s_abs + n + (verify ? 4u : 0u);
    for (uint64_t a = s_abs; a < end; ++a) pages.insert(a >> 12);
    SpanD d{s_abs - sbase, n, init, 7u};
    WalkE wk;
    wk.start(sbase, d, verify);
    CheckFast(d, wk);
    uint32_t chain = 0, result = 0;
    for (;;) {
      const SegE g = wk.next();
      const uint32_t fl = g.c.flags();
      uint32_t R = 0;
      if (fl & kENoBody) {
        R = ~init;
      } else {
        uint8_t win[4096];
        for (uint32_t t = 0; t < kSegChunks; ++t)
          memcpy(win + 16 * t, Read(sbase + g.wb + SegChunkOffset(g, t), 16), 16);
        const uint32_t inj = (fl & kEFirst) ? HeadRegister(init, g.c.hp()) : ((fl & kEMain) ? 0u : chain);
        const uint32_t front = g.c.front();
        if (front == 0u && g.c.hp() == 0u) {
          uint32_t w0 = Le32(win) ^ inj;
          memcpy(win, &w0, 4);
        } else {
          memset(win, 0, 16 * front);
          uint32_t c[4];
          memcpy(c, win + 16 * front, 16);
          fix_head(c, g.c.hp(), g.c.ws(), inj);
          memcpy(win + 16 * front, c, 16);
        }
        if (verify && (fl & kELast)) {
          // lane 63's words 14, 15: the trailer unmasked in place
          uint32_t lo, hi;
          memcpy(&lo, win + 4088, 4);
          memcpy(&hi, win + 4092, 4);
          fix_trailer(lo, hi, g.c.jv());
          memcpy(win + 4088, &lo, 4);
          memcpy(win + 4092, &hi, 4);
        }
        R = Feed(0u, win, sizeof(win));
      }
      if ((fl & kEAux) && (verify || !g.c.k())) {
        fprintf(stderr, "  aux chunk without a tail\n");
        ++g_fail;
      }
      if (fl & kEAux) {
        const uint8_t* a = Read(sbase + g.ax, 16);
        if (g.c.te() + g.c.k() > 16u) {
          fprintf(stderr, "  tail word outside the aux chunk\n");
          ++g_fail;
        }
        R = Feed(R, a + g.c.te(), g.c.k());
      }
      const uint32_t residue = verify ? verify_residue(g.c.jv()) : 0u;
      if (fl & kEMain) {
        const uint32_t hp = g.c.php(), r = g.c.r();
        const uint32_t pw = g.c.piece_word();
        if ((fl & kEAux) || r > kPieceMax) {
          fprintf(stderr, "  piece span with an aux chunk in its main segment / too long\n");
          ++g_fail;
        }
        uint8_t pwin[256];
        for (uint32_t t = 0; t < kPieceChunks; ++t) {
          const uint64_t at = sbase + g.c.c0 + PieceChunkOffset(pw, t);
          if (t == 0u && (at & 3u)) {
            fprintf(stderr, "  piece aux chunk not dword aligned\n");
            ++g_fail;
          }
          memcpy(pwin + 16 * t, Read(at, 16), 16);
        }
        // window chunk 0: the aux chunk, its last word the tail word
        const uint32_t tw = Le32(pwin + 12);
        if (verify && g.c.k()) {
          fprintf(stderr, "  verify piece with a tail\n");
          ++g_fail;
        }
        const uint32_t front = kPieceChunks - r;
        memset(pwin, 0, 16 * front);
        uint32_t c[4];
        memcpy(c, pwin + 16 * front, 16);
        fix_head(c, hp, g.c.pws(), HeadRegister(init, hp));
        memcpy(pwin + 16 * front, c, 16);
        const uint32_t rp = Feed(0u, pwin, sizeof(pwin));
        // the kernel's ring holds T = R ^ residue; the register after
        // piece || main is rp * x^(8 * 4096) ^ R
        const uint32_t T = R ^ residue;
        uint32_t v = FeedZeros(rp, 4096u) ^ T;
        uint8_t t4[4];
        memcpy(t4, &tw, 4);
        v = Feed(v, t4, g.c.k());  // the tail
        result = verify ? (v == 0u) : ~v;
        break;
      } else if (fl & kELast) {
        result = verify ? (R == residue) : ~R;
        break;
      }
      chain = R;
    }
    return result;
  }
};

void Check(std::vector<uint8_t>& buf, uint64_t sbase, uint64_t s_abs, uint32_t n, uint32_t init) {
  const uint8_t* p = &buf[s_abs - Case::kBase];
  const uint32_t want = ~Feed(~init, p, n);
  {
    Case c{buf, sbase, s_abs, n, init, false};
    const uint32_t got = c.Run();
    ++g_cases;
    if (got != want || c.bad_read) {
      if (getenv("WALK_VERBOSE")) {
        SpanD d{s_abs - sbase, n, init, 7u};
        WalkE wk;
        wk.start(sbase, d, false);
        fprintf(stderr, "F geo %x nseg %u nc0 %u pg %u\n", wk.geo, wk.nseg, wk.geo >> 18, unsigned(s_abs & 4095));
      }
      if (g_fail < 20)
        fprintf(stderr, "crc  s %#llx n %u init %#x: got %08x want %08x\n",
                (unsigned long long)s_abs, n, init, got, want);
      ++g_fail;
    }
  }
  // verify: a trailer after the span (init 0: ReadBlock's Value), good and bad
  if (init == 0u) {
    uint8_t save[4];
    uint8_t* q = &buf[s_abs - Case::kBase + n];
    memcpy(save, q, 4);
    const uint32_t m = Mask(want);
    memcpy(q, &m, 4);
    Case good{buf, sbase, s_abs, n, 0u, true};
    const uint32_t ok = good.Run();
    uint32_t bad_ok = 0;
    bool bad_read = false;
    if (n > 0) {
      buf[s_abs - Case::kBase + n / 2] ^= 0x10;
      Case bad{buf, sbase, s_abs, n, 0u, true};
      bad_ok = bad.Run();
      bad_read = bad.bad_read;
      buf[s_abs - Case::kBase + n / 2] ^= 0x10;
    }
    memcpy(q, save, 4);
    ++g_cases;
    if (ok != 1u || bad_ok != 0u || good.bad_read || bad_read) {
      if (g_fail < 20)
        fprintf(stderr, "verify s %#llx n %u: good %u bad %u\n", (unsigned long long)s_abs, n, ok,
                bad_ok);
      ++g_fail;
    }
  }
}

}  // namespace

int main() {
  wipdb::gf2::BuildTables(&T);
  std::vector<uint8_t> buf(3u << 20);
  uint64_t x = 0x243F6A8885A308D3ull;
  for (auto& b : buf) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = static_cast<uint8_t>(x);
  }
  const uint64_t B = Case::kBase;
  // span starts: page starts and ends (the head and trailer edge cases), and
  // every 16-byte alignment
  std::vector<uint64_t> starts;
  for (uint64_t pg : {uint64_t(1) << 12, uint64_t(5) << 12}) {
    for (uint32_t o = 0; o < 20; ++o) starts.push_back(B + pg + o);
    for (uint32_t o = 1; o <= 20; ++o) starts.push_back(B + pg - o);
    starts.push_back(B + pg + 1000);
    starts.push_back(B + pg + 2051);
  }
  std::vector<uint32_t> lens;
  for (uint32_t n = 0; n <= 300; ++n) lens.push_back(n);
  for (uint32_t n = 3960; n <= 4240; ++n) lens.push_back(n);  // 4 KiB blocks, table blocks, pieces
  for (uint32_t n : {4300u, 4352u, 4353u, 4400u, 4500u, 4608u, 4609u, 5000u, 8191u, 8192u, 8193u,
                     8195u, 8200u, 8300u, 12288u, 12290u, 16384u, 20000u, 65536u, 65539u, 65636u})
    lens.push_back(n);
  uint64_t seed = 1;
  for (uint64_t s : starts)
    for (uint32_t n : lens) {
      seed = seed * 6364136223846793005ull + 1442695040888963407ull;
      const uint32_t init = (seed >> 40) % 3 == 0 ? static_cast<uint32_t>(seed >> 8) : 0u;
      // source base: the span's page, or far below it
      const uint64_t sbase = (seed >> 33) & 1 ? (s & ~uint64_t(4095)) : B;
      Check(buf, sbase, s, n, init);
    }
  printf("%s: %d cases (%d on the fast path), %d failures\n", g_fail ? "FAIL" : "PASS", g_cases,
         g_fast, g_fail);
  return g_fail || g_fast < 1000 ? 1 : 0;
}
