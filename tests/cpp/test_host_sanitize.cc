// tests/cpp/test_host_sanitize.cc -- the library's host code under
// AddressSanitizer + UndefinedBehaviorSanitizer (the reference
// carries UBSan annotations on exactly this code, kv/src/util/crc32c.cc:
// 609-615, 660-666).  Built by `make -C wipdb_amd/csrc sanitize` (every
// source of the library compiled with -fsanitize=address,undefined for the
// host; device code is not instrumented) and run by
// tests/test_abi.py::test_host_code_under_sanitizers on the CPU:
//
//   * the host CRC path (hcrc_cpu_extend / hcrc_cpu_batch, SSE4.2 3-stream
//     and its heads / tails) against a byte-serial CRC at every length and
//     alignment around its stream boundaries, and the reference KATs;
//   * the table layer in its host modes: builds (bytewise and internal keys,
//     bloom, tiny blocks, mid-table buffer flushes), VerifyTables, ReadBlock
//     and CompactionInput over every single-bit corruption of a table's
//     first bytes, its index and footer, and truncations;
//   * the WAL writer and recovery reader over damaged images;
//   * the C-ABI's argument checks and the device entry points with no device.
//
// Exit 0 = pass (a sanitizer report aborts with a non-zero status).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "hip_crc32c_batch.h"
#include "wipdb/log.h"
#include "wipdb/table.h"
#include "wipdb_sst.h"

namespace {

int g_fail = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c);      \
      ++g_fail;                                                                  \
    }                                                                            \
  } while (0)

uint32_t Table0[256];
void InitTable() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82f63b78u & (0u - (c & 1u)));
    Table0[i] = c;
  }
}
uint32_t Sarwate(uint32_t init, const uint8_t* p, size_t n) {
  uint32_t r = ~init;
  for (size_t i = 0; i < n; ++i) r = Table0[(r ^ p[i]) & 0xffu] ^ (r >> 8);
  return ~r;
}

uint64_t g_x = 0x9E3779B97F4A7C15ull;
uint64_t Rnd() {
  g_x ^= g_x << 13;
  g_x ^= g_x >> 7;
  g_x ^= g_x << 17;
  return g_x;
}

void CpuCrc() {
  // exact-size heap buffers so any over-read is an ASan report
  const uint8_t kat[] = "123456789";
  CHECK(hcrc_cpu_extend(0, kat, 9) == 0xE3069283u);
  CHECK(hcrc_cpu_extend_portable(0, kat, 9) == 0xE3069283u);
  for (size_t n = 0; n < 2100; n += (n < 600 ? 1 : 37)) {
    for (size_t a = 0; a < 16; a += (n < 300 ? 1 : 5)) {
      uint8_t* buf = static_cast<uint8_t*>(malloc(a + n + 1));
      for (size_t i = 0; i < a + n; ++i) buf[i] = static_cast<uint8_t>(Rnd());
      const uint32_t init = static_cast<uint32_t>(Rnd());
      CHECK(hcrc_cpu_extend(init, buf + a, n) == Sarwate(init, buf + a, n));
      // the portable slicing-by-8 fallback on the same exact-size buffer
      CHECK(hcrc_cpu_extend_portable(init, buf + a, n) == Sarwate(init, buf + a, n));
      free(buf);
    }
  }
  for (size_t n : {size_t(65535), size_t(65536), size_t(65537), size_t(200003)}) {
    std::vector<uint8_t> v(n);
    for (auto& b : v) b = static_cast<uint8_t>(Rnd());
    CHECK(hcrc_cpu_extend(7, v.data(), n) == Sarwate(7, v.data(), n));
    CHECK(hcrc_cpu_extend_portable(7, v.data(), n) == Sarwate(7, v.data(), n));
  }
  // batch, 4 threads, inits and masks
  std::vector<uint8_t> base(1 << 20);
  for (auto& b : base) b = static_cast<uint8_t>(Rnd());
  const size_t cnt = 3000;
  std::vector<uint64_t> off(cnt);
  std::vector<uint32_t> len(cnt), ini(cnt), out(cnt);
  for (size_t i = 0; i < cnt; ++i) {
    len[i] = static_cast<uint32_t>(Rnd() % 9000);
    off[i] = Rnd() % (base.size() - len[i]);
    ini[i] = static_cast<uint32_t>(Rnd());
  }
  CHECK(hcrc_cpu_batch(base.data(), off.data(), len.data(), ini.data(), out.data(), cnt,
                       HCRC_MASK_OUTPUT, 4) == HCRC_OK);
  for (size_t i = 0; i < cnt; ++i)
    CHECK(out[i] == hcrc_mask(Sarwate(ini[i], base.data() + off[i], len[i])));
}

std::vector<std::pair<std::string, std::string>> Entries(size_t n, bool internal) {
  std::vector<std::pair<std::string, std::string>> kv;
  uint64_t user = 0, seq = uint64_t(1) << 40;
  for (size_t i = 0; i < n; ++i) {
    user += 1 + Rnd() % 1000;
    char k[40];
    snprintf(k, sizeof(k), "key%012llu", static_cast<unsigned long long>(user));
    std::string key(k);
    if (internal) {
      seq -= 1 + Rnd() % 7;
      const uint64_t tag = (seq << 8) | 1u;
      for (int b = 0; b < 8; ++b) key.push_back(static_cast<char>(tag >> (8 * b)));
    }
    std::string val(Rnd() % 300, 'v');
    for (auto& c : val) c = static_cast<char>(32 + Rnd() % 95);
    kv.emplace_back(std::move(key), std::move(val));
  }
  return kv;
}

std::string Build(const std::vector<std::pair<std::string, std::string>>& kv,
                  wipdb::table::TableOptions o) {
  wipdb::table::StringSink sink;
  wipdb::table::TableBuilder tb(o, &sink);
  for (const auto& e : kv) tb.Add(e.first, e.second);
  CHECK(tb.Finish().ok());
  return sink.contents;
}

void Tables() {
  using namespace wipdb::table;
  for (CrcMode mode : {CrcMode::kInline, CrcMode::kBatchCpu}) {
    for (int internal = 0; internal < 2; ++internal) {
      TableOptions o;
      o.crc_mode = mode;
      o.block_size = internal ? 256 : 4096;
      o.block_restart_interval = internal ? 2 : 16;
      o.bloom_bits_per_key = 10;
      o.max_buffer_size = 8192;  // buffer flushes mid-table
      if (internal) o = InternalKeyTableOptions(o);
      const auto kv = Entries(internal ? 900 : 2500, internal != 0);
      const std::string img = Build(kv, o);
      // clean: verify, read back through the compaction input
      std::vector<BlockCheck> blocks;
      CHECK(VerifyTable(img.data(), img.size(), 10, mode, 0, &blocks).ok());
      CompactionInput::Options co;
      co.comparator = internal ? InternalBytewiseComparator() : BytewiseComparator();
      co.crc_mode = mode;
      co.prefetch_blocks = 3;
      {
        const char* im = img.data();
        const size_t sz = img.size();
        CompactionInput it(&im, &sz, 1, co);
        size_t k = 0;
        for (it.SeekToFirst(); it.Valid(); it.Next(), ++k)
          CHECK(k < kv.size() && it.key() == kv[k].first && it.value() == kv[k].second);
        CHECK(k == kv.size() && it.status().ok());
      }
      // damage: single bits over the first 600 bytes, the last 300 (index,
      // meta-index, footer), and truncations; every reader must stay in bounds
      std::vector<size_t> where;
      for (size_t p = 0; p < 600 && p < img.size(); p += 3) where.push_back(p);
      for (size_t p = img.size() > 300 ? img.size() - 300 : 0; p < img.size(); ++p)
        where.push_back(p);
      for (size_t p : where) {
        std::string bad = img;
        bad[p] ^= static_cast<char>(1u << (Rnd() % 8));
        char* exact = static_cast<char*>(malloc(bad.size()));
        memcpy(exact, bad.data(), bad.size());
        const char* im = exact;
        const size_t sz = bad.size();
        std::vector<wipdb::Status> st;
        (void)VerifyTables(&im, &sz, 1, 10, mode, 0, &st);
        CompactionInput it(&im, &sz, 1, co);
        for (it.SeekToFirst(); it.Valid(); it.Next()) (void)it.key();
        (void)it.status();
        std::string_view c;
        for (const auto& b : blocks) (void)ReadBlock(exact, sz, b.offset, b.size, true, &c);
        free(exact);
      }
      for (size_t cut = 0; cut < img.size(); cut += 1 + img.size() / 97) {
        char* exact = static_cast<char*>(malloc(cut + 1));
        memcpy(exact, img.data(), cut);
        const char* im = exact;
        const size_t sz = cut;
        std::vector<wipdb::Status> st;
        CHECK(!VerifyTables(&im, &sz, 1, 10, mode, 0, &st).ok());
        CompactionInput it(&im, &sz, 1, co);
        for (it.SeekToFirst(); it.Valid(); it.Next()) (void)it.value();
        free(exact);
      }
    }
  }
}

void Logs() {
  using namespace wipdb;
  std::vector<std::string> recs;
  for (int i = 0; i < 3000; ++i) recs.emplace_back(Rnd() % (i % 97 == 0 ? 70000 : 500), 'r');
  for (auto& r : recs)
    for (auto& c : r) c = static_cast<char>(Rnd());
  std::vector<std::string_view> views(recs.begin(), recs.end());
  for (int recycle = 0; recycle < 2; ++recycle) {
    std::string img;
    CHECK(log::WriteLog(views, recycle != 0, 9, table::CrcMode::kBatchCpu, 0, &img).ok());
    for (int t = 0; t < 60; ++t) {
      std::string bad = img;
      if (t % 3 == 0) bad.resize(Rnd() % bad.size());
      else bad[Rnd() % bad.size()] ^= 0x20;
      char* exact = static_cast<char*>(malloc(bad.size() + 1));
      memcpy(exact, bad.data(), bad.size());
      const char* im = exact;
      const size_t sz = bad.size();
      std::vector<std::vector<log::Record>> res;
      std::vector<std::vector<log::Drop>> drops;
      (void)log::ReadLogs(&im, &sz, 1, table::CrcMode::kBatchCpu, 0, &res, &drops);
      free(exact);
    }
  }
}

void CAbi() {
  uint32_t out = 0;
  uint64_t off = 0;
  uint32_t len = 1;
  const char b = 'x';
  CHECK(hcrc_batch(nullptr, &b, &off, &len, nullptr, &out, 1, 0) == HCRC_ERR_INVALID);
  hcrc_ctx* ctx = nullptr;
  const int rc = hcrc_ctx_create(0, &ctx);
  if (rc == HCRC_OK) {
    CHECK(hcrc_batch(ctx, &b, &off, &len, nullptr, &out, 1, 0x40) == HCRC_ERR_INVALID);
    hcrc_ctx_destroy(ctx);
  } else {
    CHECK(rc == HCRC_ERR_NO_DEVICE && ctx == nullptr);
  }
  CHECK(hcrc_ctx_create(100000, &ctx) == HCRC_ERR_NO_DEVICE);
  CHECK(wsst_build_tables_ex(1, nullptr, nullptr, nullptr, nullptr, nullptr, 4096, 16, 0, 1, 0, 0,
                             0, nullptr, 0, nullptr, nullptr, nullptr) == WSST_ERR_INVALID);
  uint64_t ne = 0;
  CHECK(wsst_merge_tables(nullptr, nullptr, 0, 7, 1, 4, 1, 0, nullptr, 0, nullptr, nullptr, 0,
                          nullptr, 0, &ne, nullptr) == WSST_ERR_INVALID);
}

}  // namespace

int main() {
  InitTable();
  CpuCrc();
  Tables();
  Logs();
  CAbi();
  printf("%s (%d failures)\n", g_fail ? "FAIL" : "PASS", g_fail);
  return g_fail ? 1 : 0;
}
