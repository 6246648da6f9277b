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
// Build: clang++ -std=c++20 -O1 -pthread -I wipdb_amd/csrc -I tests/cpp.
// Usage: test_lp_emu [--pipe=ea|lp] [case ...]; exit 0 = pass.
#define WIPDB_LK_EMU 1
// the queue's spin bound, set per case (run-time in the emulation)
#define WIPDB_LP_SPIN (::wipdb::lk::emu::g_spin.load())
#include "crc32c_lds.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
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
// the launches' fault word (every launch must leave it 0, except the forced
// queue timeout, which must set it)
unsigned int g_fault_word = 0;
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
  const uint32_t fb = emu::g_faults.exchange(0) | (__atomic_exchange_n(&g_fault_word, 0u, __ATOMIC_SEQ_CST) ? 0x80000000u : 0u);
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
                                 mask ? kFlagMask : 0u, img, bd, &g_fault_word);
    else
      crc32c_lds_spans_kernel<0>(buf.data(), offs.data(), lens.data(), nullptr, got.data(), n,
                                 mask ? kFlagMask : 0u, img, bd, &g_fault_word);
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
    crc32c_lds_verify_kernel(buf.data(), offs.data(), hl.data(), st.data(), n, img, &g_fault_word);
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
                              img, &g_fault_word);
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

// A buffer of exactly `bytes` bytes whose last byte is followed by a PROT_NONE
// page (and whose first page is preceded by one): a read of the emulated
// kernel past the end of the data, a descriptor column or the output faults
// the test process.  Untouched pages cost no memory (MAP_NORESERVE), so a
// 2 GiB data buffer of which one workgroup's 8 MiB is written is cheap.
template <class T>
struct Guarded {
  uint8_t* map = nullptr;
  size_t maplen = 0;
  T* p = nullptr;
  size_t n = 0;
  explicit Guarded(size_t count) : n(count) {
    const size_t pg = 4096, bytes = count * sizeof(T), body = (bytes + pg - 1) / pg * pg;
    maplen = body + 2 * pg;
    void* m = mmap(nullptr, maplen, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                   -1, 0);
    if (m == MAP_FAILED) abort();
    map = static_cast<uint8_t*>(m);
    mprotect(map, pg, PROT_NONE);
    mprotect(map + pg + body, pg, PROT_NONE);
    p = reinterpret_cast<T*>(map + pg + body - bytes);
  }
  ~Guarded() { munmap(map, maplen); }
  Guarded(const Guarded&) = delete;
  Guarded& operator=(const Guarded&) = delete;
  T& operator[](size_t i) { return p[i]; }
};

// An exact-fit launch (verdict r4 item 1): spans whose last one ends at the
// last byte of the data buffer, every column exactly `n` entries, each
// followed by a guard page; the DMA range is the data's own pages.  Runs the
// workgroups `blocks` of a `grid` launch (the last workgroup holds the last
// span under both deals) and checks their spans.  verify: ReadBlock spans
// (lens = handle sizes; the +1 type byte and the trailer are in the data).
void RunExact(const char* name, Guarded<uint8_t>& data, const std::vector<uint64_t>& offs_v,
              const std::vector<uint32_t>& lens_v, bool verify, bool balance, uint32_t grid,
              const std::vector<uint32_t>& blocks) {
  const size_t n = offs_v.size();
  Guarded<uint64_t> off(n);
  Guarded<uint32_t> len(n);
  for (size_t i = 0; i < n; ++i) off[i] = offs_v[i], len[i] = lens_v[i];
  // the spans the chosen workgroups own (both deals of crc32c_dev.h wg_units)
  std::vector<uint32_t> bounds;
  if (balance) {
    std::vector<uint32_t> w(lens_v);
    if (verify)
      for (auto& x : w) x += 1u;
    bounds = BalanceBounds(w, grid);
  }
  std::vector<uint8_t> mine(n, 0);
  for (uint32_t g : blocks) {
    if (balance) {
      for (uint32_t s = bounds[g]; s < bounds[g + 1]; ++s) mine[s] = 1;
    } else {
      const uint64_t full = n / (16u * grid) * 16u;
      for (uint64_t u = 0; u < full; ++u) mine[((u >> 4) * grid + g) * 16u + (u & 15u)] = 1;
      for (uint64_t u = full; u * grid + g < n; ++u) mine[u * grid + g] = 1;
    }
  }
  std::vector<uint32_t> want(n, 0x5A5A5A5Au);
  size_t owned = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!mine[i]) continue;
    ++owned;
    const uint32_t c = Extend(0u, data.p + offs_v[i], lens_v[i] + (verify ? 1u : 0u));
    if (verify) {
      uint32_t m;
      memcpy(&m, data.p + offs_v[i] + lens_v[i] + 1u, 4);
      want[i] = m == wipdb::gf2::Mask(c) ? 1u : 0u;
    } else {
      want[i] = c;
    }
  }
  const uint64_t lo = reinterpret_cast<uint64_t>(data.p);
  emu::g_src_lo = lo & ~uint64_t(4095);
  emu::g_src_hi = lo + data.n;  // the data ends at a page boundary
  const uint8_t* img = reinterpret_cast<const uint8_t*>(g_image.data());
  std::vector<uint32_t> got(n, 0x5A5A5A5Au);
  if (verify) {
    Guarded<uint8_t> st(n);
    for (size_t i = 0; i < n; ++i) st[i] = 0x5A;
    emu::launch_blocks(grid, blocks, [&] {
      crc32c_lds_verify_kernel(data.p, off.p, len.p, st.p, n, img, &g_fault_word);
    });
    for (size_t i = 0; i < n; ++i) got[i] = st[i] == 0x5A ? 0x5A5A5A5Au : st[i];
    (void)balance;  // the verify entry point has no balanced deal
  } else {
    Guarded<uint32_t> out(n);
    for (size_t i = 0; i < n; ++i) out[i] = 0x5A5A5A5Au;
    emu::launch_blocks(grid, blocks, [&] {
      crc32c_lds_spans_kernel<0>(data.p, off.p, len.p, nullptr, out.p, n, 0u, img,
                                 balance ? bounds.data() : nullptr, &g_fault_word);
    });
    for (size_t i = 0; i < n; ++i) got[i] = out[i];
  }
  char label[96];
  snprintf(label, sizeof label, "%s (%zu owned)", name, owned);
  Report(label, got, want, offs_v, lens_v);
}

// HCRC_PACKED: the pre-pass (crc32c_ps_index_kernel) then the packed kernel
// (run_ps, or run_lp when the pre-pass finds the batch not packed), on
// `data` (any buffer; the DMA range is its pages).  C: chunks of the launch
// (0: 32 per workgroup, as the host picks).  want_packed: what the pre-pass
// must decide.
// the packed launches' flags beyond the mask: kFlagPsOnly keeps them on run_ps
// where the kernel would hand a batch that suits it to run_ea
uint32_t g_packed_flags = kFlagPsOnly;

void RunPacked(const char* name, const uint8_t* data0, size_t data_n, const std::vector<uint64_t>& offs,
               const std::vector<uint32_t>& lens, const std::vector<uint32_t>* inits, bool mask,
               uint32_t cus, uint32_t C, bool want_packed) {
  // the data on whole pages of its own, at the same page offset (the kernel
  // may read any byte of a page that holds a span byte; ASan builds of this
  // test see a heap buffer's page neighbours as foreign)
  const size_t pofs = reinterpret_cast<uintptr_t>(data0) & 4095u;
  const size_t pbytes = (pofs + data_n + 4095u) & ~size_t(4095);
  void* pm = nullptr;
  if (posix_memalign(&pm, 4096, pbytes) != 0) abort();
  memcpy(static_cast<uint8_t*>(pm) + pofs, data0, data_n);
  struct Free { void* p; ~Free() { free(p); } } free_pm{pm};
  const uint8_t* data = static_cast<const uint8_t*>(pm) + pofs;
  const size_t n = offs.size();
  const uint32_t grid = Grid(n, cus);
  if (C == 0) C = 32u * grid;
  std::vector<uint32_t> want(n), got(n, 0x5A5A5A5Au);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t c = Extend(inits ? (*inits)[i] : 0u, data + offs[i], lens[i]);
    want[i] = mask ? wipdb::gf2::Mask(c) : c;
  }
  // the verdict word as a stream's earlier launches left it (an older
  // epoch's tag, broken): the pre-pass must raise it to this launch's
  constexpr uint32_t kEpoch = 7;
  std::vector<uint32_t> first(C + 1, 0xFFFFFFFFu), meta(kPsMetaWords, 0u);
  meta[0] = (kEpoch - 1) << 4 | kPsBad;
  static_assert(kThreads == kPsIndexThreads, "emu::launch runs kThreads lanes a workgroup");
  const uint32_t pgrid = static_cast<uint32_t>(std::min<size_t>((n + kPsIndexThreads - 1) / kPsIndexThreads, 8));
  emu::launch(pgrid ? pgrid : 1, [&] {
    crc32c_ps_index_kernel(data, offs.data(), lens.data(), n, C, first.data(), meta.data(), kEpoch,
                           g_packed_flags);
  });
  // this launch's verdict, nothing broken; kPsEa: the batch suits run_ea,
  // which the packed kernel takes without the index (none was written)
  const bool ea_only = meta[0] == (kEpoch << 4 | kPsEa);
  const bool packed = meta[0] == kEpoch << 4 || ea_only;
  if (packed && !ea_only)
    for (uint32_t c = 0; c <= C; ++c)
      if (first[c] > n || (c && first[c] < first[c - 1])) {
        fprintf(stderr, "  %s: first[%u] = %u\n", name, c, first[c]);
        ++g_fail;
        return;
      }
  const uint64_t lo = reinterpret_cast<uint64_t>(data);
  emu::g_src_lo = lo & ~uint64_t(4095);
  emu::g_src_hi = (lo + data_n + 4095) & ~uint64_t(4095);
  const uint8_t* img = reinterpret_cast<const uint8_t*>(g_image.data());
  emu::g_pipes.exchange(0);
  emu::launch(grid, [&] {
    if (inits)
      crc32c_lds_packed_kernel<1>(data, offs.data(), lens.data(), inits->data(), got.data(), n,
                                  (mask ? kFlagMask : 0u) | g_packed_flags, img, first.data(), meta.data(), C,
                                  kEpoch, &g_fault_word, nullptr);
    else
      crc32c_lds_packed_kernel<0>(data, offs.data(), lens.data(), nullptr, got.data(), n,
                                  (mask ? kFlagMask : 0u) | g_packed_flags, img, first.data(), meta.data(), C,
                                  kEpoch, &g_fault_word, nullptr);
  });
  char label[96];
  const int pipes = emu::g_pipes.load();
  snprintf(label, sizeof label, "%s [%s]", name,
           !packed ? "fallback" : ((pipes & 1) != 0 ? "ea" : "ps"));
  if (packed != want_packed) {
    fprintf(stderr, "  %s: the pre-pass says %s (meta %#x)\n", name, packed ? "packed" : "not packed",
            meta[0]);
    ++g_fail;
  }
  emu::g_pipes.exchange(0);
  Report(label, got, want, offs, lens);
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
  if (Want(argc, argv, "front pieces")) {
    // pieces of every size 1..15 chunks (spans 4097..4336 B: both piece
    // rings of run_ea, 8- and 16-chunk windows, interleaved), with inits
    auto l = lens_of(3000, 4097, 4336);
    auto in = inits_of(l.size());
    g_want_pipe = 1;
    RunSpans("front pieces 1..15 chunks", buf, Packed(l, 3, 4), l, &in, false, 3);
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
                                 img, nullptr, &g_fault_word);
    });
    emu::g_spin = 1u << 22;
    emu::g_hide_marker = ~0u;
    size_t lost = 0;
    for (size_t i = 0; i < l.size(); ++i) lost += got[i] != want[i];
    const uint32_t fb = emu::g_faults.exchange(0);
    const bool word = __atomic_exchange_n(&g_fault_word, 0u, __ATOMIC_SEQ_CST) != 0u;
    const bool ok = (fb & kFaultQueuePop) != 0 && word && lost >= 1 && lost <= 4 &&
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
  {
    // Every buffer ends at a guard page: data, descriptor columns, outputs.
    auto fill = [](Guarded<uint8_t>& d, uint64_t seed) {
      uint64_t x = seed;
      for (size_t i = 0; i + 8 <= d.n; i += 8) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(d.p + i, &z, 8);
      }
    };
    if (Want(argc, argv, "exact fit 2 GiB")) {
      // the r04an shape: 512 Ki aligned 4 KiB blocks filling exactly 2 GiB,
      // a 256-workgroup launch, its first and last workgroups, both deals
      const size_t n = size_t(1) << 19;
      Guarded<uint8_t> d(n * 4096);
      fill(d, 11);
      std::vector<uint64_t> o(n);
      for (size_t i = 0; i < n; ++i) o[i] = 4096u * i;
      const std::vector<uint32_t> l(n, 4096u);
      RunExact("exact fit 2 GiB 4 KiB, round robin", d, o, l, false, false, 256, {0, 255});
      RunExact("exact fit 2 GiB 4 KiB, balanced", d, o, l, false, true, 256, {0, 255});
    }
    if (Want(argc, argv, "exact fit verify 4 KiB")) {
      // ReadBlock's 4 KiB blocks (4091 + type + trailer), the last trailer
      // at the end; every 5th block corrupted
      const size_t n = 16384;
      Guarded<uint8_t> d(n * 4096);
      fill(d, 12);
      std::vector<uint64_t> o(n);
      for (size_t i = 0; i < n; ++i) {
        o[i] = 4096u * i;
        uint32_t m = wipdb::gf2::Mask(Extend(0u, d.p + o[i], 4092));
        if (i % 5 == 4) m ^= 1u << (i % 32);
        memcpy(d.p + o[i] + 4092, &m, 4);
      }
      RunExact("exact fit verify 4 KiB", d, o, std::vector<uint32_t>(n, 4091u), true, false, 256,
               {0, 255});
    }
    auto packed_exact = [&](const char* name, uint32_t lo, uint32_t hi, uint32_t gap, size_t n,
                            bool verify) {
      auto l = lens_of(n, lo, hi);
      const auto o = Packed(l, 0, gap + (verify ? 5u : 0u));
      const size_t end = o.back() + l.back() + (verify ? 5u : 0u);
      Guarded<uint8_t> d(end);
      fill(d, lo + hi);
      if (verify) {
        for (size_t i = 0; i < n; ++i) {
          uint32_t m = wipdb::gf2::Mask(Extend(0u, d.p + o[i], l[i] + 1u));
          if (i % 7 == 6) m ^= 0x100u;
          memcpy(d.p + o[i] + l[i] + 1u, &m, 4);
        }
      }
      const uint32_t grid = Grid(n, 3);
      std::vector<uint32_t> all(grid);
      for (uint32_t g = 0; g < grid; ++g) all[g] = g;
      std::string s = std::string(name) + ", round robin";
      RunExact(s.c_str(), d, o, l, verify, false, grid, all);
      if (!verify) {
        s = std::string(name) + ", balanced";
        RunExact(s.c_str(), d, o, l, false, true, grid, all);
      }
    };
    if (Want(argc, argv, "exact fit packed")) {
      packed_exact("exact fit packed table blocks", 4097, 4225, 4, 600, false);
      packed_exact("exact fit packed verify table blocks", 4096, 4224, 0, 600, true);
      packed_exact("exact fit packed 512 B..2 KiB", 512, 2200, 5, 1200, false);
      packed_exact("exact fit packed verify 300..5000", 300, 5000, 0, 600, true);
      packed_exact("exact fit packed 16..64 KiB", 16384, 65536, 5, 120, false);
    }
  }
  if (Want(argc, argv, "packed tiny")) {  // single spans and pairs, one window or two
    RunPacked("packed tiny one 4096", buf.data(), buf.size(), {0}, {4096}, nullptr, false, 1, 0, true);
    RunPacked("packed tiny one 2000", buf.data(), buf.size(), {0}, {2000}, nullptr, false, 1, 0, true);
    RunPacked("packed tiny one 2000 at 8", buf.data(), buf.size(), {8}, {2000}, nullptr, false, 1, 0, true);
    RunPacked("packed tiny one 2001 at 9", buf.data(), buf.size(), {9}, {2001}, nullptr, false, 1, 0, true);
    RunPacked("packed tiny two", buf.data(), buf.size(), {0, 2005}, {2000, 1500}, nullptr, false, 1, 0, true);
    RunPacked("packed tiny one 8192", buf.data(), buf.size(), {0}, {8192}, nullptr, false, 1, 0, true);
    RunPacked("packed tiny one 6000 at 3", buf.data(), buf.size(), {3}, {6000}, nullptr, false, 1, 0, true);
  }
  if (Want(argc, argv, "packed batches")) {
    // HCRC_PACKED batches (crc32c_ps.h): SST-packed shapes on run_ps, and
    // batches the pre-pass must refuse (the lane-packed fallback)
    auto gaps = [&](const std::vector<uint32_t>& l, uint64_t start, uint32_t glo, uint32_t ghi) {
      std::vector<uint64_t> o(l.size());
      uint64_t cur = start;
      for (size_t i = 0; i < l.size(); ++i) {
        o[i] = cur;
        cur += l[i] + glo + static_cast<uint32_t>(rng() % (ghi - glo + 1));
      }
      return o;
    };
    {
      auto l = lens_of(1000, 512, 2200);
      RunPacked("packed 512 B..2 KiB", buf.data(), buf.size(), Packed(l, 3, 5), l, nullptr, false, 3, 0,
                true);
      auto in = inits_of(l.size());
      RunPacked("packed 512 B..2 KiB (inits, mask)", buf.data(), buf.size(), Packed(l, 6, 5), l, &in,
                true, 2, 0, true);
    }
    {
      // two spans a page at most: the desks' two-event hand-off
      auto l = lens_of(700, 1600, 2600);
      RunPacked("packed 1.6..2.6 KiB", buf.data(), buf.size(), Packed(l, 9, 4), l, nullptr, false, 3, 0,
                true);
    }
    {
      auto l = lens_of(500, 4097, 4225);
      RunPacked("packed table blocks", buf.data(), buf.size(), Packed(l, 0, 4), l, nullptr, true, 3, 0,
                true);
      g_packed_flags = 0;  // the kernel's own choice: run_ea
      RunPacked("packed table blocks, dispatched", buf.data(), buf.size(), Packed(l, 0, 4), l, nullptr,
                true, 3, 0, true);
      g_packed_flags = kFlagPsOnly;
    }
    {
      std::vector<uint64_t> o;
      for (int i = 0; i < 600; ++i) o.push_back(4096u * i);
      RunPacked("packed aligned 4 KiB", buf.data(), buf.size(), o, std::vector<uint32_t>(600, 4096),
                nullptr, false, 3, 0, true);
    }
    {
      const uint32_t B[] = {512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
      std::vector<uint32_t> l;
      uint64_t tot = 0;
      while (tot < (6u << 20)) {
        const uint32_t b = B[rng() % 8 < 5 ? rng() % 4 : 4 + rng() % 4];
        l.push_back(b + static_cast<uint32_t>(rng() % (b / 8 + 1)));
        tot += l.back() + 5;
      }
      auto in = inits_of(l.size());
      RunPacked("packed mix 512 B..72 KiB (inits)", buf.data(), buf.size(), Packed(l, 1, 5), l, &in,
                false, 4, 0, true);
      RunPacked("packed mix, 4 KiB chunks", buf.data(), buf.size(), Packed(l, 7, 5), l, nullptr, true,
                3, 1500, true);
    }
    {
      // short and empty spans among the stream ones, ragged gaps 0..300,
      // spans of exactly 64 / 65 bytes, words shared across a 0..3-byte gap
      std::vector<uint32_t> l;
      for (int i = 0; i < 1000; ++i) {
        const uint32_t r = static_cast<uint32_t>(rng() % 20);
        l.push_back(r == 0 ? 0u : r == 1 ? 1u + static_cast<uint32_t>(rng() % 63)
                   : r == 2 ? 64u : r == 3 ? 65u : 64u + static_cast<uint32_t>(rng() % 3000));
      }
      auto in = inits_of(l.size());
      RunPacked("packed shorts, empties, 64 B, gaps 0..300", buf.data(), buf.size(), gaps(l, 5, 0, 300),
                l, &in, true, 3, 0, true);
      RunPacked("packed tight gaps 0..3", buf.data(), buf.size(), gaps(l, 2, 0, 3), l, nullptr, false, 3,
                0, true);
      RunPacked("packed gaps up to 4095, small chunks", buf.data(), buf.size(), gaps(l, 9, 0, 4095),
                  l, &in, false, 2, 300, true);
    }
    {
      // exact fit: the last span's last byte is the buffer's last byte
      auto l = lens_of(600, 700, 5000);
      const auto o = Packed(l, 0, 4);
      Guarded<uint8_t> d(o.back() + l.back());
      for (size_t i = 0; i < d.n; ++i) d[i] = static_cast<uint8_t>(rng());
      RunPacked("packed exact fit", d.p, d.n, o, l, nullptr, true, 3, 0, true);
    }
    {
      // not packed: the fallback computes them all the same
      auto l = lens_of(800, 300, 3000);
      auto o = Packed(l, 3, 5);
      std::swap(o[100], o[101]);
      std::swap(l[100], l[101]);
      RunPacked("not packed: unsorted", buf.data(), buf.size(), o, l, nullptr, false, 3, 0, false);
      auto o2 = Packed(l, 3, 5);
      o2[500] -= 10;  // overlaps the span before
      RunPacked("not packed: overlap", buf.data(), buf.size(), o2, l, nullptr, false, 3, 0, false);
      auto o3 = Packed(l, 3, 5);
      for (size_t i = 400; i < o3.size(); ++i) o3[i] += 5000;  // a gap of 5 KiB
      RunPacked("not packed: a 5 KiB gap", buf.data(), buf.size(), o3, l, nullptr, false, 3, 0, false);
      // WAL-like records behind 7-byte headers: runs of spans under the
      // stream minimum (sparse enough to pass the density check)
      auto l5 = lens_of(1500, 40, 95);
      RunPacked("not packed: runs of short spans", buf.data(), buf.size(), Packed(l5, 7, 7), l5, nullptr,
                false, 3, 0, false);
      auto l4 = lens_of(1200, 5, 60);
      RunPacked("not packed: dense short spans", buf.data(), buf.size(), Packed(l4, 1, 7), l4, nullptr,
                false, 3, 0, false);
    }
  }
  printf("%s: %d failing cases\n", g_fail ? "FAIL" : "PASS", g_fail);
  return g_fail ? 1 : 0;
}
