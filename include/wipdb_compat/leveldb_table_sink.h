// include/wipdb_compat/leveldb_table_sink.h -- the leveldb/table side of the
// batched block checksums (SURVEY.md 8f-1 / 8f-2 for the reference's second
// table stack, /root/reference/leveldb).  Compiled with leveldb's public
// headers (leveldb/include) on the include path, it lets the code that runs
// leveldb::TableBuilder (leveldb/table/table_builder.cc) and ReadBlock
// (leveldb/table/format.cc:66-143) use wipdb::table instead:
//
//   * write side -- table_builder.cc:185-187 computes crc32c::Value(contents)
//     + Extend(type byte) inline in WriteRawBlock for every block.  Here
//     wipdb::table::TableBuilder writes the same bytes and computes the
//     CRCs of all buffered blocks in one batch (MI355X or host):
//
//       wipdb::leveldbcompat::WritableFileSink<> sink(file);   // leveldb::WritableFile*
//       wipdb::table::TableBuilder tb(
//           wipdb::leveldbcompat::TableOptionsFrom(options, /*bloom_bits=*/10,
//                                                  wipdb::table::CrcMode::kBatchAuto), &sink);
//       ... tb.Add(key, value) ...; tb.Finish(); file->Sync(); file->Close();
//
//   * read side -- format.cc:91-92 checks Unmask(stored) == Value(data, n+1)
//     one block at a time.  ReadImage pulls a table through a
//     leveldb::RandomAccessFile, and wipdb::table::VerifyTables /
//     CompactionInput check every block of many tables in batches.
//
// The on-disk framing is the same as kv's (the 5-byte block trailer, the
// 48-byte footer, kTableMagicNumber 0xdb4775248b80fb57).  The index keys are
// leveldb's: the builder shortens them with the leveldb::Options comparator
// itself (ComparatorFrom wraps it), so tests/cpp/test_leveldb_adapter.cc's
// tables equal, byte for byte, what leveldb's own TableBuilder writes for the
// same entries and options (leveldb compiled in place, oracle/Makefile
// LDB_SO; tests/test_table.py), and leveldb's Table::Open + ReadBlock accept
// them.
//
// Link requirement: the adapter calls leveldb::BytewiseComparator() (the
// default comparator, not inline), so a program using this header links
// libleveldb -- a leveldb deployment does anyway; otherwise only inline
// members of leveldb's headers are used.
// SupportedOptions says whether a leveldb::Options can be served (no
// compression -- WipDB's benchmarks run without it, kv_bench.cc:984 -- and
// no filter or the built-in bloom filter); call it first.
#pragma once
#include <string.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <type_traits>

#include "leveldb/comparator.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/options.h"
#include "leveldb/slice.h"
#include "leveldb/status.h"
#include "wipdb/table.h"

namespace wipdb {
namespace leveldbcompat {

// TableSink over a leveldb::WritableFile (or anything with the same Append
// and Flush): each buffer the builder hands over is appended, then flushed,
// as leveldb::TableBuilder::Flush does after every data block
// (table_builder.cc:130-133).
template <class File = leveldb::WritableFile>
class WritableFileSink : public table::TableSink {
 public:
  explicit WritableFileSink(File* f) : f_(f) {}
  Status Append(const char* data, size_t n) override {
    leveldb::Status s = f_->Append(leveldb::Slice(data, n));
    if (s.ok()) s = f_->Flush();
    if (s.ok()) return Status::OK();
    return Status::IOError(s.IsIOError() ? "leveldb WritableFile: IO error"
                                         : "leveldb WritableFile: append failed");
  }

 private:
  File* f_;
};

// wipdb::table's comparator interface over a leveldb::Comparator (or
// anything with its Name / Compare / FindShortestSeparator /
// FindShortSuccessor): the builder's index keys are then leveldb's own
// (leveldb/table/table_builder.cc:106-107, 199-200 call the same two
// functions), whatever the comparator -- bytewise, InternalKeyComparator
// (db/dbformat.cc), or a user's.
template <class Cmp = leveldb::Comparator>
class ComparatorFrom : public table::Comparator {
 public:
  explicit ComparatorFrom(const Cmp* c) : c_(c) {}
  const char* Name() const override { return c_->Name(); }
  int Compare(std::string_view a, std::string_view b) const override {
    return c_->Compare(leveldb::Slice(a.data(), a.size()), leveldb::Slice(b.data(), b.size()));
  }
  void FindShortestSeparator(std::string* start, std::string_view limit) const override {
    c_->FindShortestSeparator(start, leveldb::Slice(limit.data(), limit.size()));
  }
  void FindShortSuccessor(std::string* key) const override { c_->FindShortSuccessor(key); }

 private:
  const Cmp* c_;
};

// One wrapper per leveldb comparator, kept by address until
// ReleaseComparator(c) (leveldb::BytewiseComparator() is a singleton; a DB's
// InternalKeyComparator lives as long as the DB: call ReleaseComparator when
// the DB closes, or let the caller own the wrapper -- TableOptionsFrom's
// `owner` argument -- so that no cache entry is made at all).  Keyed by
// address, not name: two InternalKeyComparators share a name but may wrap
// different user comparators.
template <class Cmp>
inline std::map<const Cmp*, std::unique_ptr<ComparatorFrom<Cmp>>>& WrapperCache(std::mutex** mu) {
  static std::mutex m;
  static auto* cache = new std::map<const Cmp*, std::unique_ptr<ComparatorFrom<Cmp>>>;
  *mu = &m;
  return *cache;
}
template <class Cmp>
inline const table::Comparator* WrapComparator(const Cmp* c) {
  std::mutex* mu;
  auto& m = WrapperCache<Cmp>(&mu);
  std::lock_guard<std::mutex> lk(*mu);
  auto& w = m[c];
  if (!w) w.reset(new ComparatorFrom<Cmp>(c));
  return w.get();
}
// Drops c's cached wrapper (its TableOptions must no longer be in use).
template <class Cmp>
inline void ReleaseComparator(const Cmp* c) {
  std::mutex* mu;
  auto& m = WrapperCache<Cmp>(&mu);
  std::lock_guard<std::mutex> lk(*mu);
  m.erase(c);
}

// Whether wipdb::table can write what leveldb::TableBuilder would for these
// options.  Anything else must stay on leveldb::TableBuilder, since
// TableOptionsFrom would write a different (valid-looking) table:
//   * no compression (the builder stores blocks raw);
//   * no filter policy, or one named "leveldb.BuiltinBloomFilter2"
//     (leveldb/util/bloom.cc; the InternalFilterPolicy wrapping it reports the
//     same name, dbformat.cc:101-103): the meta entry "filter.<Name>" and the
//     filter bytes are the built-in bloom filter's.
// Any comparator is served: its own separators shorten the index keys.  A
// comparator named "leveldb.InternalKeyComparator" means internal keys (the
// bloom filter hashes the user key, as InternalFilterPolicy does); the second
// argument is DEPRECATED: kept for source compatibility and ignored.
template <class Opts = leveldb::Options>
inline bool SupportedOptions(const Opts& o, bool /*internal_user_bytewise: deprecated*/ = false) {
  if (o.compression != leveldb::kNoCompression) return false;
  if (o.filter_policy && strcmp(o.filter_policy->Name(), "leveldb.BuiltinBloomFilter2") != 0)
    return false;
  return true;
}

// The table options a leveldb::Options stands for (only for options
// SupportedOptions accepts).  leveldb::FilterPolicy does not expose its bits
// per key, so the caller passes what it gave NewBloomFilterPolicy (0 = no
// filter policy).  A null comparator is leveldb's default,
// leveldb::BytewiseComparator().  owner (nullable): the comparator wrapper
// is created into *owner, which must outlive the options; without it the
// wrapper comes from WrapComparator's cache.
template <class Opts = leveldb::Options>
inline table::TableOptions TableOptionsFrom(const Opts& o, int bloom_bits, table::CrcMode mode,
                                            int device = -1,
                                            std::unique_ptr<table::Comparator>* owner = nullptr) {
  table::TableOptions t;
  t.block_size = o.block_size;
  t.block_restart_interval = o.block_restart_interval;
  t.bloom_bits_per_key = o.filter_policy ? bloom_bits : 0;
  t.crc_mode = mode;
  t.device = device;
  const auto* c = o.comparator ? o.comparator : leveldb::BytewiseComparator();
  if (strcmp(c->Name(), "leveldb.InternalKeyComparator") == 0)
    t = table::InternalKeyTableOptions(t);  // (user-key bloom filter)
  if (owner) {
    owner->reset(new ComparatorFrom<std::remove_cv_t<std::remove_pointer_t<decltype(c)>>>(c));
    t.comparator = owner->get();
  } else {
    t.comparator = WrapComparator(c);
  }
  return t;
}

// A whole table through a leveldb::RandomAccessFile (Read(offset, n,
// &result, scratch), env.h), for VerifyTables / CompactionInput.
template <class File = leveldb::RandomAccessFile>
inline Status ReadImage(const File* f, uint64_t size, std::string* image) {
  image->resize(size);
  uint64_t off = 0;
  while (off < size) {
    const size_t want = size - off < (uint64_t(1) << 26) ? size_t(size - off) : size_t(1) << 26;
    leveldb::Slice got;
    leveldb::Status s = f->Read(off, want, &got, &(*image)[off]);
    if (!s.ok()) return Status::IOError("leveldb RandomAccessFile: read failed");
    if (got.size() == 0) return Status::Corruption("truncated block read");
    if (got.data() != &(*image)[off]) memmove(&(*image)[off], got.data(), got.size());
    off += got.size();
  }
  return Status::OK();
}

}  // namespace leveldbcompat
}  // namespace wipdb
