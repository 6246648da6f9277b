// oracle/ref_leveldb_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" driver over leveldb's own table code, compiled in place from
// /root/reference/leveldb (oracle/Makefile, targets libref_leveldb.so and
// libref_leveldb_dropin.so), the second reference call site of the CRC path:
//   leveldb::TableBuilder        leveldb/table/table_builder.cc:185-187
//                                (WriteRawBlock: crc32c::Value + Extend +
//                                Mask into the block trailer)
//   leveldb::Table::Open, ReadBlock  leveldb/table/table.cc, format.cc:91-92
//                                (Unmask(trailer) vs Value(data, n + 1))
//   leveldb::NewBloomFilterPolicy, InternalKeyComparator,
//   InternalFilterPolicy         leveldb/util/bloom.cc, db/dbformat.cc
// leveldb's port layer is configured from the command line only, with the
// macros port/port_config.h.in:8-31 leaves to it (LEVELDB_HAS_PORT_CONFIG_H=0,
// port/port_stdcxx.h:11-23); no header is written.
// It writes tables into memory so tests/test_table.py can byte-compare the
// leveldb adapter (include/wipdb_compat/leveldb_table_sink.h) with leveldb's
// own builder, and reads images back with verify_checksums to compare
// statuses.  Only tests/ may load this library.
#include <stdint.h>
#include <string.h>

#include <string>

#include "db/dbformat.h"
#include "leveldb/comparator.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "leveldb/table_builder.h"
#include "table/format.h"
#include "util/crc32c.h"

namespace {

class MemWritable : public leveldb::WritableFile {
 public:
  std::string data;
  leveldb::Status Append(const leveldb::Slice& s) override {
    data.append(s.data(), s.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Close() override { return leveldb::Status::OK(); }
  leveldb::Status Flush() override { return leveldb::Status::OK(); }
  leveldb::Status Sync() override { return leveldb::Status::OK(); }
};

class MemRandom : public leveldb::RandomAccessFile {
 public:
  const char* p;
  size_t n;
  MemRandom(const char* p_, size_t n_) : p(p_), n(n_) {}
  leveldb::Status Read(uint64_t off, size_t len, leveldb::Slice* result,
                       char* scratch) const override {
    if (off >= n) {
      *result = leveldb::Slice(scratch, 0);
      return leveldb::Status::OK();
    }
    size_t m = len;
    if (off + m > n) m = n - off;
    memcpy(scratch, p + off, m);
    *result = leveldb::Slice(scratch, m);
    return leveldb::Status::OK();
  }
};

// 0 OK, 1 other corruption, 2 "block checksum mismatch", 3 other error (the
// codes of oracle/ref_table_shim.cc)
int StatusCode(const leveldb::Status& s) {
  if (s.ok()) return 0;
  if (s.IsCorruption()) {
    return s.ToString().find("block checksum mismatch") != std::string::npos ? 2 : 1;
  }
  return 3;
}

}  // namespace

extern "C" {

// leveldb::crc32c::Value of n bytes (the KAT: "123456789" -> 0xe3069283)
uint32_t ldb_crc32c_value(const char* data, size_t n) { return leveldb::crc32c::Value(data, n); }

// One table from n sorted (key, value) pairs with leveldb's TableBuilder, no
// compression; bloom_bits <= 0: no filter; internal != 0: the DB's options
// (InternalKeyComparator(BytewiseComparator) + InternalFilterPolicy,
// leveldb/db/db_impl.cc SanitizeOptions).  Returns the table size (at most
// cap bytes copied to out), or -1 on a builder error.
long ldb_build_table_ex(const char* keys, const uint32_t* key_lens, const char* vals,
                        const uint32_t* val_lens, size_t n, int block_size,
                        int restart_interval, int bloom_bits, int internal, char* out,
                        size_t cap) {
  leveldb::Options opt;
  opt.block_size = static_cast<size_t>(block_size);
  opt.block_restart_interval = restart_interval;
  opt.compression = leveldb::kNoCompression;
  const leveldb::FilterPolicy* fp =
      bloom_bits > 0 ? leveldb::NewBloomFilterPolicy(bloom_bits) : nullptr;
  leveldb::InternalKeyComparator icmp(leveldb::BytewiseComparator());
  leveldb::InternalFilterPolicy ipolicy(fp);
  opt.filter_policy = fp;
  if (internal) {
    opt.comparator = &icmp;
    opt.filter_policy = fp ? &ipolicy : nullptr;
  }
  MemWritable f;
  long rc = -1;
  {
    leveldb::TableBuilder tb(opt, &f);
    size_t ko = 0, vo = 0;
    for (size_t i = 0; i < n; ++i) {
      tb.Add(leveldb::Slice(keys + ko, key_lens[i]), leveldb::Slice(vals + vo, val_lens[i]));
      ko += key_lens[i];
      vo += val_lens[i];
    }
    leveldb::Status s = tb.Finish();
    if (s.ok()) {
      rc = static_cast<long>(f.data.size());
      memcpy(out, f.data.data(), f.data.size() < cap ? f.data.size() : cap);
    }
  }
  delete fp;
  return rc;
}

// Table::Open (paranoid_checks) + a full iteration with verify_checksums:
// the status code; *blocks is unused (0), kept for the kv shim's signature.
int ldb_verify_table(const char* data, size_t n, int bloom_bits, int internal, size_t* blocks) {
  leveldb::Options opt;
  opt.paranoid_checks = true;
  const leveldb::FilterPolicy* fp =
      bloom_bits > 0 ? leveldb::NewBloomFilterPolicy(bloom_bits) : nullptr;
  leveldb::InternalKeyComparator icmp(leveldb::BytewiseComparator());
  leveldb::InternalFilterPolicy ipolicy(fp);
  opt.filter_policy = fp;
  if (internal) {
    opt.comparator = &icmp;
    opt.filter_policy = fp ? &ipolicy : nullptr;
  }
  MemRandom f(data, n);
  leveldb::Table* t = nullptr;
  leveldb::Status s = leveldb::Table::Open(opt, &f, n, &t);
  *blocks = 0;
  int rc = StatusCode(s);
  if (s.ok()) {
    leveldb::ReadOptions ro;
    ro.verify_checksums = true;
    ro.fill_cache = false;
    leveldb::Iterator* it = t->NewIterator(ro);
    for (it->SeekToFirst(); it->Valid(); it->Next()) {
    }
    rc = StatusCode(it->status());
    delete it;
    delete t;
  }
  delete fp;
  return rc;
}

// leveldb::ReadBlock(verify_checksums) on one handle of an image.
int ldb_read_block(const char* data, size_t n, uint64_t offset, uint64_t size) {
  MemRandom f(data, n);
  leveldb::ReadOptions ro;
  ro.verify_checksums = true;
  leveldb::BlockHandle h;
  h.set_offset(offset);
  h.set_size(size);
  leveldb::BlockContents c;
  leveldb::Status s = leveldb::ReadBlock(&f, ro, h, &c);
  if (s.ok() && c.heap_allocated) delete[] c.data.data();
  return StatusCode(s);
}

}  // extern "C"
