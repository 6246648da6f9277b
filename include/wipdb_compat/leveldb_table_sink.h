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
// 48-byte footer, kTableMagicNumber 0xdb4775248b80fb57): tests/cpp/
// test_leveldb_adapter.cc writes tables through this adapter and the file
// must equal the bytes the reference's kv::TableBuilder writes for the same
// entries and options.  leveldb's OWN TableBuilder is not compiled here (its
// port layer needs the CMake-generated port/port_config.h), so the
// leveldb-side byte identity is parity-unpinned beyond that kv equivalence.
//
// Only inline members of leveldb's headers are used, so including this file
// links against no leveldb library.  SupportedOptions says whether a
// leveldb::Options can be served (no compression -- WipDB's benchmarks run
// without it, kv_bench.cc:984 -- a bytewise or internal-over-bytewise
// comparator, no filter or the built-in bloom filter); call it first.
#pragma once
#include <string.h>

#include <string>

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

// Whether wipdb::table can write what leveldb::TableBuilder would for these
// options.  Anything else must stay on leveldb::TableBuilder, since
// TableOptionsFrom would write a different (valid-looking) table:
//   * no compression (the builder stores blocks raw);
//   * comparator "leveldb.BytewiseComparator" (leveldb's default), or
//     "leveldb.InternalKeyComparator" (leveldb/db/dbformat.cc:46-48) over a
//     bytewise user comparator -- the wrapped comparator is not visible
//     through leveldb's public headers, so the caller confirms it
//     (internal_user_bytewise); index separators and successors are computed
//     bytewise on the (user) key, any other order would misplace lookups;
//   * no filter policy, or one named "leveldb.BuiltinBloomFilter2"
//     (leveldb/util/bloom.cc; the InternalFilterPolicy wrapping it reports the
//     same name, dbformat.cc:101-103): the meta entry "filter.<Name>" and the
//     filter bytes are the built-in bloom filter's.
template <class Opts = leveldb::Options>
inline bool SupportedOptions(const Opts& o, bool internal_user_bytewise = false) {
  if (o.compression != leveldb::kNoCompression) return false;
  const char* cmp = o.comparator ? o.comparator->Name() : "leveldb.BytewiseComparator";
  if (strcmp(cmp, "leveldb.InternalKeyComparator") == 0) {
    if (!internal_user_bytewise) return false;
  } else if (strcmp(cmp, "leveldb.BytewiseComparator") != 0) {
    return false;
  }
  if (o.filter_policy && strcmp(o.filter_policy->Name(), "leveldb.BuiltinBloomFilter2") != 0)
    return false;
  return true;
}

// The table options a leveldb::Options stands for (only for options
// SupportedOptions accepts).  leveldb::FilterPolicy
// does not expose its bits per key, so the caller passes what it gave
// NewBloomFilterPolicy (0 = no filter policy).  A comparator named
// "leveldb.InternalKeyComparator" (leveldb/db/dbformat.cc) selects internal
// keys and the InternalFilterPolicy's user-key hashing, as in kv.
template <class Opts = leveldb::Options>
inline table::TableOptions TableOptionsFrom(const Opts& o, int bloom_bits, table::CrcMode mode,
                                            int device = -1) {
  table::TableOptions t;
  t.block_size = o.block_size;
  t.block_restart_interval = o.block_restart_interval;
  t.bloom_bits_per_key = o.filter_policy ? bloom_bits : 0;
  t.crc_mode = mode;
  t.device = device;
  if (o.comparator && strcmp(o.comparator->Name(), "leveldb.InternalKeyComparator") == 0)
    t = table::InternalKeyTableOptions(t);
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
