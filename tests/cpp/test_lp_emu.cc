// tests/cpp/test_lp_emu.cc -- the lane-packed spans / verify / strided
// kernels (wipdb_amd/csrc/crc32c_lds.hip, their own source) run on the host
// under the SIMT emulation of tests/cpp/lk_emu.h, against a byte-serial
// CRC32C: every span shape (short spans packed many per iteration, table
// blocks as a segment + back piece, long spans shared through the
// workgroup's queue, empty spans, inits, masked output), ReadBlock's verify
// with good and corrupted trailers, and every DMA source inside the test's
// buffer.  Catches control-flow and indexing errors of the kernel loop (the
// desk, the ring, the queue, the batch packing) before a GPU run.
// The queue's timeout path is forced once (a hidden record marker and a small
// spin bound): the launch must report the fault.
// Build: clang++ -std=c++17 -O1 -pthread -I wipdb_amd/csrc -I tests/cpp.
// Usage: test_lp_emu [--pipe=ea|lp] [case ...]; exit 0 = pass.
#define WIPDB_LK_EMU 1
// the queue's spin bound, set per case (run-time in the emulation)
#define WIPDB_LP_SPIN (::wipdb::lk::emu::g_spin.load())
#include "crc32c_lds.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

using namespace wipdb::lk;

namespace {

wipdb::gf2::Tables T;
std::vector<uint32_t> g_image(kImageBytes / 4);

uint32_t Extend(uint32_t init, const uint8_t* p, size_t n) {
  uint32_t r = ~init;
  for (size_t i = 0; i < n; ++i) r = T.t[0][(r ^ p[i]) & 0xffu] ^ (r >> 8);
  return ~r;
}

int g_fail = 0;
// the pipeline the next launches must choose (1 run_ea, 2 run_lp, 0 any)
uint32_t g_want_pipe = 0;

// DMA sources must lie in the pages of the buffer (the kernel's guarantee:
// nothing outside the pages that hold bytes of a span is read)
void SetRange(const std::vector<uint8_t>& buf) {
  const uint64_t lo = reinterpret_cast<uint64_t>(buf.data());
  emu::g_src_lo = lo & ~uint64_t(4095);
  emu::g_src_hi = (lo + buf.size() + 4095) & ~uint64_t(4095);
}

uint32_t Grid(size_t count, uint32_t cus) {
  const size_t need = (count + 15) / 16;
  return static_cast<uint32_t>(need < cus ? (need ? need : 1) : cus);
}

void Report(const char* name, const std::vector<uint32_t>& got, const std::vector<uint32_t>& want,
            const std::vector<uint64_t>& offs, const std::vector<uint32_t>& lens) {
  size_t bad = 0;
  for (size_t i = 0; i < want.size(); ++i) {
    if (got[i] != want[i]) {
      if (bad < 6)
        fprintf(stderr, "  %s: span %zu off %llu len %u: got %08x want %08x\n", name, i,
                (unsigned long long)offs[i], lens[i], got[i], want[i]);
      ++bad;
    }
  }
  const uint64_t bs = emu::g_bad_src.exchange(0);
  if (bs) fprintf(stderr, "  %s: DMA source %#llx outside the buffer\n", name, (unsigned long long)(bs & ~1ull));
  const uint32_t fb = emu::g_faults.exchange(0);
  if (fb) fprintf(stderr, "  %s: the launch reported fault bits %#x\n", name, fb);
  const uint32_t pipes = emu::g_pipes.exchange(0);
  const bool pipe_bad =
      pipes == 3u || (g_want_pipe != 0u && emu::g_force_pipe.load() < 0 && pipes != g_want_pipe);
  if (pipe_bad) fprintf(stderr, "  %s: pipelines %#x, want %#x\n", name, pipes, g_want_pipe);
  const bool fail = bad || bs || fb || pipe_bad;
  printf("%-34s %6zu spans  %s %s (%zu bad)\n", name, want.size(), pipes == 1u ? "ea" : "lp",
         fail ? "FAIL" : "ok", bad);
  if (fail) ++g_fail;
}

// HCRC_BALANCE's workgroup ranges, restated on the host
// (util::balance_bounds_kernel): bounds[g] = #{i : excl(i) < g T / G},
// weight = length + 64.  g_balance: RunSpans passes them to the kernel.
bool g_balance = false;
std::vector<uint32_t> BalanceBounds(const std::vector<uint32_t>& lens, uint32_t G) {
  uint64_t T = 0;
  for (uint32_t n : lens) T += n + 64u;
  std::vector<uint32_t> b(G + 1, 0);
  b[G] = static_cast<uint32_t>(lens.size());
  for (uint32_t g = 1; g < G; ++g) {
    const uint64_t target = (T / G) * g + (T % G) * g / G;
    uint64_t e = 0;
    uint32_t c = 0;
    for (uint32_t n : lens) {
      if (e >= target) break;
      ++c;
      e += n + 64u;
    }
    b[g] = c;
  }
  return b;
}

// CRC batch through crc32c_lds_spans_kernel
void RunSpans(const char* name, std::vector<uint8_t>& buf, const std::vector<uint64_t>& offs,
              const std::vector<uint32_t>& lens, const std::vector<uint32_t>* inits, bool mask,
              uint32_t cus) {
  const size_t n = offs.size();
  const std::vector<uint32_t> bounds =
      g_balance ? BalanceBounds(lens, Grid(n, cus)) : std::vector<uint32_t>();
  const uint32_t* bd = g_balance ? bounds.data() : nullptr;
  std::vector<uint32_t> want(n), got(n, 0x5A5A5A5Au);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t c = Extend(inits ? (*inits)[i] : 0u, buf.data() + offs[i], lens[i]);
    want[i] = mask ? wipdb::gf2::Mask(c) : c;
  }
  SetRange(buf);
  const uint8_t* img = reinterpret_cast<const uint8_t*>(g_image.data());
  emu::launch(Grid(n, cus), [&] {
    if (inits)
      crc32c_lds_spans_kernel<1>(buf.data(), offs.data(), lens.data(), inits->data(), got.data(), n,
                                 mask ? kFlagMask : 0u, img, bd);
    else
      crc32c_lds_spans_kernel<0>(buf.data(), offs.data(), lens.data(), nullptr, got.data(), n,
                                 mask ? kFlagMask : 0u, img, bd);
  });
  Report(name, got, want, offs, lens);
}

// ReadBlock verify: spans of n bytes (contents + type) followed by a masked
// trailer; every 7th block corrupted
void RunVerify(const char* name, std::vector<uint8_t>& buf, const std::vector<uint64_t>& offs,
               const std::vector<uint32_t>& lens, uint32_t cus) {
  const size_t n = offs.size();
  std::vector<uint32_t> want(n), hl(n);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t m = wipdb::gf2::Mask(Extend(0u, buf.data() + offs[i], lens[i]));
    memcpy(buf.data() + offs[i] + lens[i], &m, 4);
    want[i] = 1;
    if (i % 7 == 3) {
      buf[offs[i] + (i % 5 == 0 ? lens[i] + 2 : lens[i] / 2)] ^= 0x40;  // data or trailer
      want[i] = 0;
    }
    hl[i] = lens[i] - 1;  // handle size (the type byte is the +1)
  }
  std::vector<uint8_t> st(n, 0x5A);
  SetRange(buf);
  const uint8_t* img = reinterpret_cast<const uint8_t*>(g_image.data());
  emu::launch(Grid(n, cus), [&] {
    crc32c_lds_verify_kernel(buf.data(), offs.data(), hl.data(), st.data(), n, img);
  });
  std::vector<uint32_t> got(st.begin(), st.end());
  Report(name, got, want, offs, lens);
  for (size_t i = 0; i < n; ++i)  // undo the corruption
    if (i % 7 == 3) buf[offs[i] + (i % 5 == 0 ? lens[i] + 2 : lens[i] / 2)] ^= 0x40;
}

void RunStrided(const char* name, std::vector<uint8_t>& buf, uint64_t stride, uint32_t len,
                uint32_t init, size_t n, uint32_t cus, bool mask = false) {
  std::vector<uint64_t> offs(n);
  std::vector<uint32_t> lens(n, len), want(n), got(n, 0x5A5A5A5Au);
  for (size_t i = 0; i < n; ++i) {
    offs[i] = i * stride;
    want[i] = Extend(init, buf.data() + offs[i], len);
    if (mask) want[i] = wipdb::gf2::Mask(want[i]);
  }
  SetRange(buf);
  const uint8_t* img = reinterpret_cast<const uint8_t*>(g_image.data());
  emu::launch(Grid(n, cus), [&] {
    crc32c_lds_strided_kernel(buf.data(), stride, len, init, got.data(), n, mask ? kFlagMask : 0u,
                              img);
  });
  Report(name, got, want, offs, lens);
}

std::vector<uint64_t> Packed(const std::vector<uint32_t>& lens, uint64_t start, uint32_t gap) {
  std::vector<uint64_t> o(lens.size());
  uint64_t cur = start;
  for (size_t i = 0; i < lens.size(); ++i) {
    o[i] = cur;
    cur += lens[i] + gap;
  }
  return o;
}

bool Want(int argc, char** argv, const char* name) {
  bool any = false;
  for (int i = 1; i < argc; ++i) {
    if (argv[i][0] == '-') continue;
    any = true;
    if (strstr(name, argv[i])) return true;
  }
  return !any;
}

}  // namespace

int main(int argc, char** argv) {
  // --pipe=ea / --pipe=lp: every launch takes that pipeline (both must be
  // exact on every shape; the choice only changes speed)
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--pipe=ea")) emu::g_force_pipe = 1;
    if (!strcmp(argv[i], "--pipe=lp")) emu::g_force_pipe = 0;
  }
  wipdb::gf2::BuildTables(&T);
  BuildLdsImage(g_image.data());
  std::mt19937_64 rng(7);
  std::vector<uint8_t> buf(24u << 20);
  for (auto& b : buf) b = static_cast<uint8_t>(rng());
  auto lens_of = [&](size_t n, uint32_t lo, uint32_t hi) {
    std::vector<uint32_t> v(n);
    for (auto& x : v) x = lo + static_cast<uint32_t>(rng() % (hi - lo + 1));
    return v;
  };
  auto inits_of = [&](size_t n) {
    std::vector<uint32_t> v(n);
    for (size_t i = 0; i < n; ++i) v[i] = i % 3 ? static_cast<uint32_t>(rng()) : 0u;
    return v;
  };
  if (Want(argc, argv, "one short")) RunSpans("one short", buf, {64}, {100}, nullptr, false, 1);
  if (Want(argc, argv, "one 4096")) RunSpans("one 4096", buf, {4096}, {4096}, nullptr, false, 1);
  if (Want(argc, argv, "one 5000")) RunSpans("one 5000", buf, {4099}, {5000}, nullptr, false, 1);
  if (Want(argc, argv, "17 short")) {
    std::vector<uint64_t> o;
    for (int i = 0; i < 17; ++i) o.push_back(128u * i);
    RunSpans("17 short", buf, o, std::vector<uint32_t>(17, 100), nullptr, false, 1);
  }
  if (Want(argc, argv, "tiny 0..40")) {
    std::vector<uint32_t> l;
    std::vector<uint64_t> o;
    for (uint32_t n = 0; n <= 40; ++n)
      for (uint32_t a = 0; a < 8; ++a) {
        l.push_back(n);
        o.push_back(4096u * 3 - 20 + a + 64u * n);
      }
    auto in = inits_of(l.size());
    RunSpans("tiny 0..40 (inits)", buf, o, l, &in, false, 2);
  }
  if (Want(argc, argv, "short 0..300")) {
    auto l = lens_of(3000, 0, 300);
    auto in = inits_of(l.size());
    RunSpans("short 0..300 packed (inits)", buf, Packed(l, 5, 3), l, &in, false, 3);
  }
  if (Want(argc, argv, "512 bucket")) {
    auto l = lens_of(3000, 512, 576);
    RunSpans("512 bucket packed", buf, Packed(l, 3, 5), l, nullptr, true, 4);
  }
  if (Want(argc, argv, "1-2 KiB buckets")) {  // pieces of 16..58 lanes: most split over two batches
    auto l = lens_of(1500, 1024, 1152);
    RunSpans("1 KiB bucket packed", buf, Packed(l, 1, 5), l, nullptr, false, 3);
    auto l2 = lens_of(1500, 2048, 3700);
    auto in = inits_of(l2.size());
    RunSpans("2-3.6 KiB packed (inits)", buf, Packed(l2, 6, 5), l2, &in, true, 3);
  }
  if (Want(argc, argv, "aligned 4 KiB")) {
    std::vector<uint64_t> o;
    for (int i = 0; i < 2000; ++i) o.push_back(4096u * i);
    g_want_pipe = 1;
    RunSpans("aligned 4 KiB", buf, o, std::vector<uint32_t>(2000, 4096), nullptr, false, 3);
    g_want_pipe = 0;
  }
  if (Want(argc, argv, "table blocks")) {
    auto l = lens_of(2000, 4097, 4225);
    g_want_pipe = 1;
    RunSpans("table blocks", buf, Packed(l, 0, 4), l, nullptr, true, 3);
    g_want_pipe = 0;
  }
  if (Want(argc, argv, "near 4 KiB")) {
    auto l = lens_of(2000, 3960, 4240);
    auto in = inits_of(l.size());
    RunSpans("near 4 KiB (inits)", buf, Packed(l, 1, 7), l, &in, false, 3);
  }
  if (Want(argc, argv, "small pieces")) {
    // m segments + 0 .. 36 chunks: segments with back pieces of every
    // small size (table blocks, ReadBlock's 4 KiB + type + trailer), odd
    // offsets, inits
    std::vector<uint32_t> l;
    for (uint32_t m = 1; m <= 3; ++m)
      for (uint32_t f = 0; f <= 36; ++f)
        for (uint32_t d = 0; d < 4; ++d) l.push_back(4096u * m + 16u * f - 2u + d);
    auto in = inits_of(l.size());
    RunSpans("segments + small pieces (inits)", buf, Packed(l, 3, 5), l, &in, true, 2);
    RunVerify("verify segments + small pieces", buf, Packed(l, 1, 4), l, 2);
  }
  if (Want(argc, argv, "long")) {
    auto l = lens_of(300, 8000, 70000);
    g_want_pipe = 2;
    RunSpans("long 8..70 KiB", buf, Packed(l, 2, 5), l, nullptr, false, 2);
    auto l2 = lens_of(120, 32768, 200000);
    auto in2 = inits_of(l2.size());
    g_want_pipe = 1;
    RunSpans("long 32..200 KiB (inits)", buf, Packed(l2, 5, 3), l2, &in2, true, 2);
    g_want_pipe = 0;
  }
  // the shapes of run_lp's long-span queue: its spans are all >= 16 KiB,
  // which the launch-level choice gives run_ea, so run_lp is forced (unless
  // the command line forces a pipeline)
  const bool force_lp = emu::g_force_pipe.load() < 0;
  if (force_lp) emu::g_force_pipe = 0;
  if (Want(argc, argv, "shared long")) {  // one wave's desks of long spans, the others idle: shared
    auto l = lens_of(16, 20000, 70000);
    auto in = inits_of(l.size());
    RunSpans("shared long: one desk (inits)", buf, Packed(l, 3, 5), l, &in, false, 1);
    auto l2 = lens_of(40, 8000, 300000);
    auto in2 = inits_of(l2.size());
    RunSpans("shared long: 40 (inits)", buf, Packed(l2, 1, 5), l2, &in2, true, 2);
  }
  if (Want(argc, argv, "queue full")) {  // one workgroup, more long spans than queue slots
    auto l = lens_of(700, 16384, 24000);
    auto in = inits_of(l.size());
    RunSpans("queue full: 700 long (inits)", buf, Packed(l, 7, 5), l, &in, false, 1);
  }
  if (Want(argc, argv, "queue timeout")) {
    // record 0's marker hidden, a bound of 64 spins: its popper times out.
    // The launch must end (no hang), say so in its error word (kFaultQueuePop;
    // slot 0 then stays claimed, so record 256's producer reports
    // kFaultQueueSlot rather than overwrite it), and every span it did not
    // lose must still be right.
    auto l = lens_of(700, 16384, 24000);
    const auto o = Packed(l, 7, 5);
    std::vector<uint32_t> want(l.size()), got(l.size(), 0x5A5A5A5Au);
    for (size_t i = 0; i < l.size(); ++i) want[i] = Extend(0u, buf.data() + o[i], l[i]);
    SetRange(buf);
    emu::g_spin = 64;
    emu::g_hide_marker = 0;
    emu::g_pipes = 0;
    const uint8_t* img = reinterpret_cast<const uint8_t*>(g_image.data());
    emu::launch(1, [&] {
      crc32c_lds_spans_kernel<0>(buf.data(), o.data(), l.data(), nullptr, got.data(), l.size(), 0u,
                                 img, nullptr);
    });
    emu::g_spin = 1u << 22;
    emu::g_hide_marker = ~0u;
    size_t lost = 0;
    for (size_t i = 0; i < l.size(); ++i) lost += got[i] != want[i];
    const uint32_t fb = emu::g_faults.exchange(0);
    const bool ok = (fb & kFaultQueuePop) != 0 && lost >= 1 && lost <= 4 &&
                    emu::g_bad_src.exchange(0) == 0;
    printf("%-34s %6zu spans  %s (fault bits %#x, %zu lost)\n", "queue timeout: fault reported",
           l.size(), ok ? "ok" : "FAIL", fb, lost);
    if (!ok) ++g_fail;
  }
  if (force_lp) emu::g_force_pipe = -1;
  if (Want(argc, argv, "zipf mix")) {
    const uint32_t B[] = {512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
    std::vector<uint32_t> l;
    for (int i = 0; i < 1500; ++i) {
      const double u = (rng() >> 11) * (1.0 / 9007199254740992.0);
      int k = 0;
      double c = 0, z = 0;
      for (int j = 0; j < 8; ++j) z += 1.0 / (j + 1);
      for (; k < 7; ++k) {
        c += 1.0 / (k + 1) / z;
        if (u < c) break;
      }
      l.push_back(B[k] + static_cast<uint32_t>(rng() % (B[k] / 8 + 1)));
    }
    g_want_pipe = 2;
    RunSpans("zipf mix", buf, Packed(l, 3, 5), l, nullptr, false, 4);
    // HCRC_BALANCE: contiguous byte-balanced workgroup ranges, both pipelines
    g_balance = true;
    RunSpans("zipf mix balanced", buf, Packed(l, 3, 5), l, nullptr, false, 4);
    g_want_pipe = 0;
    {
      std::vector<uint32_t> in(l.size());
      for (auto& x : in) x = static_cast<uint32_t>(rng());
      RunSpans("zipf mix balanced (inits, mask)", buf, Packed(l, 6, 5), l, &in, true, 3);
    }
    auto l4 = lens_of(1200, 4096, 4096);
    std::vector<uint64_t> o4(l4.size());
    for (size_t i = 0; i < o4.size(); ++i) o4[i] = i * 4096;
    RunSpans("aligned 4 KiB balanced", buf, o4, l4, nullptr, false, 3);
    g_balance = false;
  }
  if (Want(argc, argv, "verify")) {
    auto l = lens_of(1500, 1, 5000);
    RunVerify("verify mixed", buf, Packed(l, 9, 4), l, 3);
    auto l2 = lens_of(1000, 4096, 4225);
    g_want_pipe = 1;
    RunVerify("verify table blocks", buf, Packed(l2, 0, 4), l2, 3);
    // long blocks (run_ea), good and corrupted
    auto l3 = lens_of(150, 32768, 120000);
    RunVerify("verify long 32..120 KiB", buf, Packed(l3, 6, 3), l3, 2);
    g_want_pipe = 0;
  }
  if (Want(argc, argv, "strided")) {
    g_want_pipe = 1;
    RunStrided("strided 4096", buf, 4096, 4096, 0, 1500, 3);
    g_want_pipe = 0;
    RunStrided("strided 700 / 513 (init)", buf, 700, 513, 0x12345678u, 1500, 2);
    RunStrided("strided 4096 masked", buf, 4096, 4096, 0, 255, 2, true);
    RunStrided("strided 4101 / 4097 masked (init)", buf, 4101, 4097, 0x12345678u, 255, 2, true);
    RunStrided("strided 4096 / 100 masked (init)", buf, 4096, 100, 7, 255, 2, true);
  }
  printf("%s: %d failing cases\n", g_fail ? "FAIL" : "PASS", g_fail);
  return g_fail ? 1 : 0;
}
