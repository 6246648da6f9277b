// tests/cpp/test_plan.cc -- host check of the lane-packed kernels' span plans
// (wipdb_amd/csrc/crc32c_plan.h), before any of it reaches a GPU:
//
//   * every DMA source the kernel computes for a span -- each window chunk of
//     each full segment (chunk 0 of segment 0 read ws words late), the
//     segment aux chunk, and each chunk of each lane's stripe of the back
//     piece as the batch DMA derives it from the lane's Stripe (S, info) --
//     lies in a page that holds a byte of the span (or of its trailer), is
//     4-byte aligned, and agrees with PieceChunkSrc;
//   * replaying the kernel's arithmetic with those exact sources --
//     segments from the start, chained by the register, the head register
//     injected into segment 0's chunk 0; the back piece's window END-aligned,
//     in-front chunks zeroed, its first real chunk in span form with the
//     segments' register (or the head register) injected, each lane's
//     64-byte stripe from a zero register shifted by 64 (nl - 1 - j) bytes
//     and XORed, the tail word from lane 0's aux chunk in one step -- with a
//     byte-serial CRC gives Extend(init, span) for every shape, and verify
//     accepts a good trailer and rejects a flipped byte.
//
// The GPU-only parts (LDS tables, lane rotation, the fold's tables, the
// segmented scan) are covered by the -m gpu parity tests.
// Build: g++ -O2 -std=c++17 -I wipdb_amd/csrc.  Exit 0 = pass.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <set>
#include <vector>

#include "crc32c_plan.h"

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
uint32_t HeadRegister(uint32_t init, uint32_t h) {
  uint32_t r = ~init;
  for (uint32_t i = 0; i < h; ++i) {
    const uint8_t idx = T.inv_top[r >> 24];
    r = ((r ^ T.t[0][idx]) << 8) | idx;
  }
  return r;
}
uint32_t Mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

int g_fail = 0, g_cases = 0, g_pieces = 0, g_segs = 0;
uint32_t g_max_nl = 0;

struct Case {
  static constexpr uint64_t kBase = uint64_t(1) << 32;
  std::vector<uint8_t>& buf;
  uint64_t sbase, s_abs;
  uint32_t n, init;
  bool verify;
  std::set<uint64_t> pages;
  bool bad_read = false;

  const uint8_t* Read(uint64_t addr, uint32_t len) {
    if (addr & 3u) {
      if (!bad_read) fprintf(stderr, "  DMA source %#llx not dword aligned\n", (unsigned long long)addr);
      bad_read = true;
    }
    for (uint64_t a = addr; a < addr + len; ++a)
      if (!pages.count(a >> 12)) {
        if (!bad_read)
          fprintf(stderr, "  read [%#llx, +%u) leaves the span's pages (s %#llx n %u v %d)\n",
                  (unsigned long long)addr, len, (unsigned long long)s_abs, n, verify);
        bad_read = true;
        break;
      }
    return &buf[addr - kBase];
  }

  // the kernel's result: the CRC (verify: 1 = good block)
  uint32_t Run() {
    const uint64_t end = s_abs + n + (verify ? 4u : 0u);
    for (uint64_t a = s_abs; a < end; ++a) pages.insert(a >> 12);
    const uint64_t a = s_abs - sbase;
    const Plan p = MakePlan(a, static_cast<uint32_t>(s_abs), n, verify);
    if (p.empty) return init;
    const uint32_t residue = verify ? verify_residue(p.jv) : 0u;
    // ---- full segments, from the start ----
    uint32_t R = 0;
    for (uint32_t t = 0; t < p.m; ++t) {
      ++g_segs;
      uint8_t win[4096];
      const uint64_t wb = sbase + p.c0 + 4096u * uint64_t(t);
      for (uint32_t c = 0; c < 256; ++c) {
        // the segment DMA: lane 0's chunk 0 of segment 0 is read ws words late
        const uint32_t o = (t == 0u && c == 0u) ? 4u * p.ws : 16u * c;
        memcpy(win + 16 * c, Read(wb + o, 16), 16);
      }
      if (t == 0u) {
        uint32_t c4[4];
        memcpy(c4, win, 16);
        fix_head(c4, p.hp, p.ws, HeadRegister(init, p.hp));
        memcpy(win, c4, 16);
      } else {
        uint32_t w0;
        memcpy(&w0, win, 4);
        w0 ^= R;
        memcpy(win, &w0, 4);
      }
      const bool last = t + 1u == p.m;
      if (verify && last && p.pw == 0u) {
        uint32_t lo, hi;
        memcpy(&lo, win + 4088, 4);
        memcpy(&hi, win + 4092, 4);
        fix_trailer(lo, hi, p.jv);
        memcpy(win + 4088, &lo, 4);
        memcpy(win + 4092, &hi, 4);
      }
      R = Feed(0u, win, sizeof(win));
    }
    if (p.pw == 0u) {
      if (p.m == 0u) {
        fprintf(stderr, "  no segment and no piece\n");
        ++g_fail;
      }
      if (p.seg_aux) {
        const uint8_t* ax = Read(sbase + p.c0 + 16u * uint64_t(p.C) - 12u, 16);
        R = Feed(R, ax + 12, p.k);
      } else if (p.k && !verify) {
        fprintf(stderr, "  a tail but no aux chunk\n");
        ++g_fail;
      }
      return verify ? (R == residue) : ~R;
    }
    // ---- the back piece (or the whole span) on nl lanes ----
    ++g_pieces;
    const PW pw{p.pw};
    const uint32_t nl = pw.nl(), front = pw.front(), r = pw.r();
    if (nl == 0u || nl > 64u || r != (p.C & 255u) || (p.m != 0u && (pw.hp() || pw.ws()))) {
      fprintf(stderr, "  bad piece word %#x (nl %u, C %u, m %u)\n", p.pw, nl, p.C, p.m);
      ++g_fail;
      return 0;
    }
    if (nl > g_max_nl) g_max_nl = nl;
    if (verify && pw.x()) {
      fprintf(stderr, "  verify piece with a tail\n");
      ++g_fail;
    }
    const uint32_t inj = p.m == 0u ? HeadRegister(init, p.hp) : R;
    std::vector<uint8_t> win(64u * nl);
    for (uint32_t j = 0; j < nl; ++j) {
      const Stripe st = MakeStripe(pw, j);
      for (uint32_t i = 0; i < 4; ++i) {
        const int64_t rel = st.s + StripeChunkSrc(st.info, i);
        if (rel != PieceChunkSrc(pw, 4 * j + i)) {
          fprintf(stderr, "  stripe %u chunk %u: %lld vs %lld\n", j, i, (long long)rel,
                  (long long)PieceChunkSrc(pw, 4 * j + i));
          ++g_fail;
        }
        memcpy(&win[64 * j + 16 * i], Read(sbase + p.p0 + rel, 16), 16);
      }
    }
    // lane 0: the tail word from its chunk 0 (the aux chunk)
    uint8_t tw[4] = {0, 0, 0, 0};
    if (pw.x()) {
      if (pw.te() + pw.k() > 16u || front == 0u) {
        fprintf(stderr, "  tail word outside the aux chunk / aux chunk not in front\n");
        ++g_fail;
      }
      for (uint32_t b = 0; b < pw.k(); ++b) tw[b] = win[pw.te() + b];
    }
    memset(win.data(), 0, 16u * front);
    if (r != 0u) {
      uint32_t c4[4];
      memcpy(c4, &win[16u * front], 16);
      fix_head(c4, pw.hp(), pw.ws(), inj);
      memcpy(&win[16u * front], c4, 16);
    }
    if (verify) {
      uint32_t lo, hi;
      uint8_t* q = &win[64u * nl - 8u];
      memcpy(&lo, q, 4);
      memcpy(&hi, q + 4, 4);
      fix_trailer(lo, hi, pw.jv());
      memcpy(q, &lo, 4);
      memcpy(q + 4, &hi, 4);
    }
    uint32_t G = 0;
    for (uint32_t j = 0; j < nl; ++j) G ^= FeedZeros(Feed(0u, &win[64 * j], 64), 64u * (nl - 1u - j));
    if (r == 0u) G ^= inj;
    if (pw.x()) G = Feed(G, tw, pw.k());
    return verify ? (G == residue) : ~G;
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
      if (g_fail < 20)
        fprintf(stderr, "crc  s %#llx n %u init %#x: got %08x want %08x\n",
                (unsigned long long)s_abs, n, init, got, want);
      ++g_fail;
    }
  }
  if (init == 0u) {  // ReadBlock: a trailer after the span, good and bad
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
  std::vector<uint64_t> starts;
  for (uint64_t pg : {uint64_t(1) << 12, uint64_t(5) << 12}) {
    for (uint32_t o = 0; o < 20; ++o) starts.push_back(B + pg + o);
    for (uint32_t o = 1; o <= 20; ++o) starts.push_back(B + pg - o);
    starts.push_back(B + pg + 1000);
    starts.push_back(B + pg + 2051);
  }
  std::vector<uint32_t> lens;
  for (uint32_t n = 0; n <= 300; ++n) lens.push_back(n);
  for (uint32_t n : {500u, 511u, 512u, 513u, 575u, 1000u, 1023u, 1024u, 1025u, 1151u, 2047u, 2048u,
                     2049u, 2303u, 3000u})
    lens.push_back(n);
  for (uint32_t n = 3960; n <= 4240; ++n) lens.push_back(n);  // 4 KiB blocks, table blocks
  for (uint32_t n : {4300u, 4352u, 4353u, 4400u, 4500u, 4608u, 4609u, 5000u, 8191u, 8192u, 8193u,
                     8195u, 8200u, 8300u, 9216u, 12288u, 12290u, 16384u, 20000u, 65536u, 65539u,
                     65636u, 73727u})
    lens.push_back(n);
  uint64_t seed = 1;
  for (uint64_t s : starts)
    for (uint32_t n : lens) {
      seed = seed * 6364136223846793005ull + 1442695040888963407ull;
      const uint32_t init = (seed >> 40) % 3 == 0 ? static_cast<uint32_t>(seed >> 8) : 0u;
      const uint64_t sbase = (seed >> 33) & 1 ? (s & ~uint64_t(4095)) : B;
      Check(buf, sbase, s, n, init);
    }
  printf("%s: %d cases, %d pieces (max %u lanes), %d segments, %d failures\n",
         g_fail ? "FAIL" : "PASS", g_cases, g_pieces, g_max_nl, g_segs, g_fail);
  return g_fail || g_max_nl != 64u ? 1 : 0;
}
