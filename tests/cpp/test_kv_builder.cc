// tests/cpp/test_kv_builder.cc -- the reference-side integration of the
// batched table builder, compiled against the reference's
// headers and linked with the reference's table code (oracle/_ref/
// libref_table.so, compiled from /root/reference/kv/src) and this library.
//
// It plays the patched BuildTableKV (kv/src/db/builder.cc:18-109) and a
// compaction with several outputs (DoCompactionWork) under the DB's options
// (InternalKeyComparator + InternalFilterPolicy, kv/src/db/db_impl.cc:141-144):
//   * an internal-key stream (user keys with several versions, puts and
//     deletions) goes through kv::TableBuilder and through
//     wipdb::table::TableBuilder behind kvcompat::WritableFileWriterSink --
//     both over a kv::WritableFileWriter -- and the files must be equal;
//   * a compaction's outputs are finished with ONE FinishTables batch and
//     each must equal kv::TableBuilder's file;
//   * every file is opened with kv::Table::Open(paranoid_checks) under the
//     DB's options and iterated with verify_checksums, and must return the
//     stream's keys and values.
//
// Usage: test_kv_builder <crc_mode 0..3>   (exit 0 = pass)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "db/dbformat.h"
#include "kv/comparator.h"
#include "kv/env.h"
#include "kv/filter_policy.h"
#include "kv/iterator.h"
#include "kv/options.h"
#include "kv/table.h"
#include "kv/table_builder.h"
#include "util/file_reader_writer.h"
#include "wipdb_compat/kv_table_sink.h"

namespace {

int g_fail = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                     \
    }                                                               \
  } while (0)

class MemWritable : public kv::WritableFile {
 public:
  std::string data;
  kv::Status Append(const kv::Slice& s) override {
    data.append(s.data(), s.size());
    return kv::Status::OK();
  }
  // BuildTableKV opens its writer with is_pwrite = true (builder.cc:41)
  kv::Status PositionedAppend(const kv::Slice& s, uint64_t offset) override {
    if (data.size() < offset + s.size()) data.resize(offset + s.size());
    memcpy(&data[offset], s.data(), s.size());
    return kv::Status::OK();
  }
  kv::Status Close() override { return kv::Status::OK(); }
  kv::Status Flush() override { return kv::Status::OK(); }
  kv::Status Sync() override { return kv::Status::OK(); }
};

class MemRandom : public kv::RandomAccessFile {
 public:
  const std::string& d;
  explicit MemRandom(const std::string& s) : d(s) {}
  kv::Status Read(uint64_t off, size_t len, kv::Slice* result, char* scratch) const override {
    if (off >= d.size()) {
      *result = kv::Slice(scratch, 0);
      return kv::Status::OK();
    }
    const size_t m = off + len > d.size() ? d.size() - off : len;
    memcpy(scratch, d.data() + off, m);
    *result = kv::Slice(scratch, m);
    return kv::Status::OK();
  }
};

struct Entry {
  std::string key, value;
};

// Deterministic internal-key stream: user keys "user%012llu" with 1..3
// versions (sequence descending), 10 % deletions, 16..300-byte values.
std::vector<Entry> Stream(size_t n_users, uint64_t seed) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&x]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  std::vector<Entry> out;
  uint64_t seq = uint64_t(1) << 40, user = 0;
  for (size_t u = 0; u < n_users; ++u) {
    user += 1 + rnd() % 5000;
    char uk[32];
    snprintf(uk, sizeof(uk), "user%012llu", static_cast<unsigned long long>(user));
    const int versions = 1 + static_cast<int>(rnd() % 3);
    for (int v = 0; v < versions; ++v) {
      seq -= 1 + rnd() % 100;
      const bool del = rnd() % 10 == 0;
      Entry e;
      e.key = uk;
      kv::PutFixed64(&e.key, (seq << 8) | (del ? kv::kTypeDeletion : kv::kTypeValue));
      if (!del) {
        const size_t vl = 16 + rnd() % 285;
        for (size_t i = 0; i < vl; ++i) e.value.push_back(static_cast<char>(32 + rnd() % 95));
      }
      out.push_back(std::move(e));
    }
  }
  return out;
}

struct DbOptions {
  const kv::FilterPolicy* bloom = kv::NewBloomFilterPolicy(10);
  kv::InternalKeyComparator icmp{kv::BytewiseComparator()};
  kv::InternalFilterPolicy ipolicy{bloom};
  kv::Options opt;
  kv::EnvOptions eo;
  DbOptions() {
    opt.comparator = &icmp;
    opt.filter_policy = &ipolicy;
    opt.paranoid_checks = true;
  }
  ~DbOptions() { delete bloom; }
};

std::string RefBuild(const DbOptions& d, const std::vector<Entry>& es, size_t lo, size_t hi) {
  MemWritable* f = new MemWritable;
  std::string out;
  {
    kv::WritableFileWriter w(f, "ref.sst", d.eo, true);
    kv::TableBuilder tb(d.opt, &w);
    for (size_t i = lo; i < hi; ++i) tb.Add(es[i].key, es[i].value);
    CHECK(tb.Finish().ok());
    CHECK(w.Flush().ok());
    out = f->data;
  }
  return out;
}

// The stream's entries [lo, hi) back through kv::Table under the DB's options.
void CheckReadsBack(const DbOptions& d, const std::string& img, const std::vector<Entry>& es,
                    size_t lo, size_t hi) {
  MemRandom f(img);
  kv::Table* t = nullptr;
  kv::Status s = kv::Table::Open(d.opt, &f, img.size(), &t);
  CHECK(s.ok());
  if (!s.ok()) return;
  kv::ReadOptions ro;
  ro.verify_checksums = true;
  std::unique_ptr<kv::Iterator> it(t->NewIterator(ro));
  size_t i = lo;
  for (it->SeekToFirst(); it->Valid() && i < hi; it->Next(), ++i) {
    CHECK(it->key().ToString() == es[i].key);
    CHECK(it->value().ToString() == es[i].value);
  }
  CHECK(!it->Valid() && i == hi);
  CHECK(it->status().ok());
  // a seek through the shortened index separators lands on each block's keys
  for (size_t k = lo; k < hi; k += 97) {
    it->Seek(es[k].key);
    CHECK(it->Valid() && it->key().ToString() == es[k].key);
  }
  it.reset();
  delete t;
}

}  // namespace

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 1;
  if (mode < 0 || mode > 3) return 2;
  DbOptions d;
  const std::vector<Entry> es = Stream(30000, 7);

  // flush: one table (BuildTableKV)
  {
    MemWritable* f = new MemWritable;
    std::string got;
    {
      kv::WritableFileWriter w(f, "wip.sst", d.eo, true);
      wipdb::kvcompat::WritableFileWriterSink sink(&w);
      wipdb::table::TableBuilder tb(
          wipdb::kvcompat::TableOptionsFrom(d.opt, d.eo, 10, static_cast<wipdb::table::CrcMode>(mode)),
          &sink);
      for (const Entry& e : es) tb.Add(e.key, e.value);
      const wipdb::Status s = tb.Finish();
      if (!s.ok()) fprintf(stderr, "Finish: %s\n", s.ToString().c_str());
      CHECK(s.ok());
      CHECK(tb.BatchedBlocks() > 0 || mode == 0);
      CHECK(w.Flush().ok());
      got = f->data;
    }
    const std::string want = RefBuild(d, es, 0, es.size());
    CHECK(got == want);
    CheckReadsBack(d, got, es, 0, es.size());
    printf("flush: %zu entries, %zu bytes, %s\n", es.size(), got.size(),
           got == want ? "identical" : "DIFFERENT");
  }

  // compaction: 6 outputs finished in one batch
  {
    const size_t per = es.size() / 6;
    std::vector<MemWritable*> files;
    std::vector<std::unique_ptr<kv::WritableFileWriter>> writers;
    std::vector<std::unique_ptr<wipdb::kvcompat::WritableFileWriterSink>> sinks;
    std::vector<std::unique_ptr<wipdb::table::TableBuilder>> tbs;
    std::vector<wipdb::table::TableBuilder*> raw;
    const auto to = wipdb::kvcompat::TableOptionsFrom(d.opt, d.eo, 10,
                                                      static_cast<wipdb::table::CrcMode>(mode));
    for (size_t k = 0; k < 6; ++k) {
      files.push_back(new MemWritable);
      writers.emplace_back(new kv::WritableFileWriter(files.back(), "out.sst", d.eo, true));
      sinks.emplace_back(new wipdb::kvcompat::WritableFileWriterSink(writers.back().get()));
      tbs.emplace_back(new wipdb::table::TableBuilder(to, sinks.back().get()));
      raw.push_back(tbs.back().get());
      const size_t lo = k * per, hi = k == 5 ? es.size() : lo + per;
      for (size_t i = lo; i < hi; ++i) tbs.back()->Add(es[i].key, es[i].value);
    }
    CHECK(wipdb::table::FinishTables(raw.data(), raw.size()).ok());
    int same = 0;
    for (size_t k = 0; k < 6; ++k) {
      CHECK(writers[k]->Flush().ok());
      const size_t lo = k * per, hi = k == 5 ? es.size() : lo + per;
      const std::string want = RefBuild(d, es, lo, hi);
      same += files[k]->data == want;
      CHECK(files[k]->data == want);
      CheckReadsBack(d, files[k]->data, es, lo, hi);
    }
    printf("compaction: 6 outputs, %d identical\n", same);
    tbs.clear();
    sinks.clear();
    writers.clear();  // ~WritableFileWriter owns and deletes its file
  }
  printf("%s (%d failures)\n", g_fail ? "FAIL" : "PASS", g_fail);
  return g_fail ? 1 : 0;
}
