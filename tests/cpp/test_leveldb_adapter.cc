// tests/cpp/test_leveldb_adapter.cc -- the leveldb/table adapter
// (include/wipdb_compat/leveldb_table_sink.h) on leveldb's real types: built
// by oracle/Makefile against leveldb's headers and leveldb's table code
// compiled in place (libref_leveldb.so: BytewiseComparator,
// InternalKeyComparator, the built-in bloom filter), so the GPU box runs it
// prebuilt:
//
//   * Instantiate() type-checks the adapter on leveldb::WritableFile,
//     leveldb::Options and leveldb::RandomAccessFile (compiled, never run);
//   * main() writes one table through WritableFileSink + TableOptionsFrom
//     (a leveldb::Options with leveldb's own comparator and filter policy),
//     reads it back through ReadImage and VerifyTable, and writes the bytes
//     out for tests/test_table.py to compare with leveldb's own
//     TableBuilder (and to have leveldb's Table::Open + ReadBlock verify).
//
// Usage: test_leveldb_adapter <entries.bin> <out.sst> <block_size> <restart>
//                             <bloom_bits> <internal 0|1> <crc_mode 0..3>
// entries.bin: u32 count, then (u32 klen, key, u32 vlen, value) per entry.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "db/dbformat.h"  // leveldb::InternalKeyComparator, InternalFilterPolicy
#include "wipdb_compat/leveldb_table_sink.h"

namespace {

// (compiled against the real leveldb types; not called)
__attribute__((used)) void Instantiate(leveldb::WritableFile* f, const leveldb::Options* o,
                                       const leveldb::RandomAccessFile* r, std::string* img) {
  wipdb::leveldbcompat::WritableFileSink<> sink(f);
  wipdb::table::TableBuilder tb(
      wipdb::leveldbcompat::TableOptionsFrom(*o, 10, wipdb::table::CrcMode::kBatchAuto), &sink);
  (void)wipdb::leveldbcompat::SupportedOptions(*o);
  (void)wipdb::leveldbcompat::ReadImage(r, 100, img);
}

// leveldb::WritableFile's Append / Flush, in memory
struct MemFile {
  std::string data;
  int flushes = 0;
  leveldb::Status Append(const leveldb::Slice& s) {
    data.append(s.data(), s.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Flush() {
    ++flushes;
    return leveldb::Status::OK();
  }
};
// leveldb::RandomAccessFile's Read, short reads of at most 1 MiB
struct MemRandom {
  const std::string* d;
  leveldb::Status Read(uint64_t off, size_t n, leveldb::Slice* result, char* scratch) const {
    const size_t m = std::min<size_t>(std::min<size_t>(n, 1u << 20), d->size() - off);
    memcpy(scratch, d->data() + off, m);
    *result = leveldb::Slice(scratch, m);
    return leveldb::Status::OK();
  }
};
// a filter policy the adapter must refuse (not the built-in bloom filter)
struct PrefixPolicy : leveldb::FilterPolicy {
  const char* Name() const override { return "my.PrefixFilter"; }
  void CreateFilter(const leveldb::Slice*, int, std::string*) const override {}
  bool KeyMayMatch(const leveldb::Slice&, const leveldb::Slice&) const override { return true; }
};

}  // namespace

int main(int argc, char** argv) {
  if (argc != 8) {
    fprintf(stderr, "usage: %s entries.bin out.sst block_size restart bloom internal crc_mode\n",
            argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::string in;
  char b[1 << 16];
  size_t r;
  while ((r = fread(b, 1, sizeof(b), f)) > 0) in.append(b, r);
  fclose(f);
  size_t pos = 0;
  auto u32 = [&]() {
    uint32_t v;
    memcpy(&v, in.data() + pos, 4);
    pos += 4;
    return v;
  };
  const uint32_t n = u32();
  const int bloom = atoi(argv[5]);
  const leveldb::FilterPolicy* bloomp = bloom ? leveldb::NewBloomFilterPolicy(bloom) : nullptr;
  const leveldb::InternalKeyComparator icmp(leveldb::BytewiseComparator());
  const leveldb::InternalFilterPolicy ipol(bloomp);
  const bool internal = atoi(argv[6]) != 0;
  leveldb::Options o;  // what a leveldb DB / table user passes
  o.block_size = static_cast<size_t>(atol(argv[3]));
  o.block_restart_interval = atoi(argv[4]);
  o.compression = leveldb::kNoCompression;
  o.comparator = internal ? static_cast<const leveldb::Comparator*>(&icmp)
                          : leveldb::BytewiseComparator();
  o.filter_policy = bloomp ? (internal ? static_cast<const leveldb::FilterPolicy*>(&ipol) : bloomp)
                           : nullptr;
  const auto mode = static_cast<wipdb::table::CrcMode>(atoi(argv[7]));
  if (!wipdb::leveldbcompat::SupportedOptions(o)) return 3;
  // options the adapter must refuse: compression, a filter policy other than
  // the built-in bloom filter (any comparator is served: its own separators)
  leveldb::Options bad = o;
  bad.compression = leveldb::kSnappyCompression;
  if (wipdb::leveldbcompat::SupportedOptions(bad)) return 3;
  static const PrefixPolicy custom;
  bad = o;
  bad.filter_policy = &custom;
  if (wipdb::leveldbcompat::SupportedOptions(bad)) return 3;
  bad = o;
  bad.comparator = nullptr;  // (leveldb's default: bytewise)
  if (!wipdb::leveldbcompat::SupportedOptions(bad)) return 3;

  MemFile file;
  wipdb::leveldbcompat::WritableFileSink<MemFile> sink(&file);
  // (the comparator wrapper owned by the caller on odd entry counts, from the
  // adapter's cache on even ones: the same bytes either way)
  std::unique_ptr<wipdb::table::Comparator> own;
  wipdb::table::TableBuilder tb(
      wipdb::leveldbcompat::TableOptionsFrom(o, bloom, mode, -1, (n & 1) ? &own : nullptr), &sink);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t kl = u32();
    std::string k = in.substr(pos, kl);
    pos += kl;
    const uint32_t vl = u32();
    std::string v = in.substr(pos, vl);
    pos += vl;
    tb.Add(k, v);
  }
  wipdb::Status s = tb.Finish();
  if (!s.ok()) {
    fprintf(stderr, "Finish: %s\n", s.ToString().c_str());
    return 1;
  }
  if (file.flushes == 0 || tb.FileSize() != file.data.size()) {
    fprintf(stderr, "sink: %d flushes, %zu bytes, builder says %llu\n", file.flushes,
            file.data.size(), (unsigned long long)tb.FileSize());
    return 1;
  }
  // read it back the leveldb way and verify every block in batches
  std::string img;
  MemRandom rf{&file.data};
  s = wipdb::leveldbcompat::ReadImage(&rf, file.data.size(), &img);
  if (!s.ok() || img != file.data) {
    fprintf(stderr, "ReadImage: %s\n", s.ToString().c_str());
    return 1;
  }
  std::vector<wipdb::table::BlockCheck> blocks;
  s = wipdb::table::VerifyTable(img.data(), img.size(), bloom, mode, -1, &blocks);
  if (!s.ok()) {
    fprintf(stderr, "VerifyTable: %s\n", s.ToString().c_str());
    return 1;
  }
  FILE* g = fopen(argv[2], "wb");
  if (!g || fwrite(file.data.data(), 1, file.data.size(), g) != file.data.size()) return 2;
  fclose(g);
  printf("wrote %zu bytes, %llu entries, %zu blocks verified, %llu batched\n", file.data.size(),
         (unsigned long long)tb.NumEntries(), blocks.size(),
         (unsigned long long)tb.BatchedBlocks());
  return 0;
}
