// oracle/ref_table_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" driver over the reference's own table code, compiled in place
// from /root/reference/kv/src (oracle/Makefile, target libref_table.so):
//   kv::TableBuilder           kv/src/table/table_builder.cc:66-271
//   kv::Table::Open / ReadBlock kv/src/table/table.cc:37-82, format.cc:66-143
//   kv::NewBloomFilterPolicy   kv/src/table/bloom.cc:88-90
//   kv::InternalKeyComparator, kv::InternalFilterPolicy  kv/src/db/dbformat.cc:45-136
//     (the options WipDB's DB builds every SST with, db_impl.cc:141-144)
// It writes SSTs into memory (an in-memory kv::WritableFile behind the
// reference's WritableFileWriter) so the tests can byte-compare the batched
// table builder's output with the reference's, and it reads them back
// through Table::Open + ReadBlock(verify_checksums) to check that the
// reference accepts (or rejects) what the batched path produced.
// Only tests/ may load this library; nothing in the product links it.
#include <stdint.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "db/dbformat.h"
#include "kv/comparator.h"
#include "kv/env.h"
#include "kv/filter_policy.h"
#include "kv/options.h"
#include "kv/table.h"
#include "kv/table_builder.h"
#include "table/format.h"
#include "table/merger.h"
#include "util/file_reader_writer.h"

namespace {

class MemWritable : public kv::WritableFile {
 public:
  std::string data;
  kv::Status Append(const kv::Slice& s) override {
    data.append(s.data(), s.size());
    return kv::Status::OK();
  }
  kv::Status Close() override { return kv::Status::OK(); }
  kv::Status Flush() override { return kv::Status::OK(); }
  kv::Status Sync() override { return kv::Status::OK(); }
};

class MemRandom : public kv::RandomAccessFile {
 public:
  const char* p;
  size_t n;
  MemRandom(const char* p_, size_t n_) : p(p_), n(n_) {}
  kv::Status Read(uint64_t off, size_t len, kv::Slice* result, char* scratch) const override {
    // pread semantics of PosixRandomAccessFile: past the end reads 0 bytes
    if (off >= n) {
      *result = kv::Slice(scratch, 0);
      return kv::Status::OK();
    }
    size_t m = len;
    if (off + m > n) m = n - off;
    memcpy(scratch, p + off, m);
    *result = kv::Slice(scratch, m);
    return kv::Status::OK();
  }
};

int StatusCode(const kv::Status& s) {
  if (s.ok()) return 0;
  if (s.IsCorruption()) {
    const std::string m = s.ToString();
    if (m.find("block checksum mismatch") != std::string::npos) return 2;
    return 1;
  }
  return 3;
}

}  // namespace

extern "C" {

// Builds one table from n sorted (key, value) pairs (concatenated blobs +
// lengths) with the reference TableBuilder.  bloom_bits <= 0: no filter.
// internal != 0: the DB's options -- InternalKeyComparator(BytewiseComparator)
// and InternalFilterPolicy around the bloom policy (SanitizeOptions,
// kv/src/db/db_impl.cc:104-111).  Writes at most cap bytes of the table to
// out; returns the table size, or -1 on a builder error.
long ref_build_table_ex(const char* keys, const uint32_t* key_lens, const char* vals,
                        const uint32_t* val_lens, size_t n, int block_size,
                        int restart_interval, int bloom_bits, int internal, char* out,
                        size_t cap) {
  kv::Options opt;
  opt.block_size = static_cast<size_t>(block_size);
  opt.block_restart_interval = restart_interval;
  const kv::FilterPolicy* fp = bloom_bits > 0 ? kv::NewBloomFilterPolicy(bloom_bits) : nullptr;
  kv::InternalKeyComparator icmp(kv::BytewiseComparator());
  kv::InternalFilterPolicy ipolicy(fp);
  opt.filter_policy = fp;
  if (internal) {
    opt.comparator = &icmp;
    opt.filter_policy = fp ? &ipolicy : nullptr;
  }
  MemWritable* mf = new MemWritable;
  long rc = -1;
  {
    kv::EnvOptions eo;
    kv::WritableFileWriter w(mf, "mem.sst", eo, false);
    kv::TableBuilder tb(opt, &w);
    size_t ko = 0, vo = 0;
    for (size_t i = 0; i < n; ++i) {
      tb.Add(kv::Slice(keys + ko, key_lens[i]), kv::Slice(vals + vo, val_lens[i]));
      ko += key_lens[i];
      vo += val_lens[i];
    }
    kv::Status s = tb.Finish();
    if (s.ok()) s = w.Flush();
    if (s.ok()) {
      rc = static_cast<long>(mf->data.size());
      memcpy(out, mf->data.data(), mf->data.size() < cap ? mf->data.size() : cap);
    }
  }  // ~WritableFileWriter closes (and owns) the file
  delete fp;
  return rc;
}

long ref_build_table(const char* keys, const uint32_t* key_lens, const char* vals,
                     const uint32_t* val_lens, size_t n, int block_size,
                     int restart_interval, int bloom_bits, char* out, size_t cap) {
  return ref_build_table_ex(keys, key_lens, vals, val_lens, n, block_size, restart_interval,
                            bloom_bits, 0, out, cap);
}

// kv::InternalKeyComparator(BytewiseComparator) on two keys: <0, 0, >0.
int ref_internal_compare(const char* a, size_t an, const char* b, size_t bn) {
  kv::InternalKeyComparator icmp(kv::BytewiseComparator());
  return icmp.Compare(kv::Slice(a, an), kv::Slice(b, bn));
}

// Bloom KeyMayMatch of the table's filter for `key` through the reference's
// Table::InternalGet path is not exposed; instead this returns the filter
// policy's verdict on a filter blob (InternalFilterPolicy when internal).
int ref_filter_may_match(const char* filter, size_t fn, const char* key, size_t kn,
                         int bloom_bits, int internal) {
  const kv::FilterPolicy* fp = kv::NewBloomFilterPolicy(bloom_bits);
  kv::InternalFilterPolicy ipolicy(fp);
  const kv::FilterPolicy* use = internal ? static_cast<const kv::FilterPolicy*>(&ipolicy) : fp;
  const int r = use->KeyMayMatch(kv::Slice(key, kn), kv::Slice(filter, fn)) ? 1 : 0;
  delete fp;
  return r;
}

// Opens a table image with Table::Open (paranoid_checks: the index block is
// read with verify_checksums) and reads every data block named by the index
// with ReadBlock(verify_checksums = true).  Returns 0 = all OK, 1 = other
// corruption, 2 = "block checksum mismatch", 3 = other error; *blocks gets
// the number of data blocks read before the first failure.
int ref_verify_table(const char* data, size_t n, int bloom_bits, size_t* blocks) {
  kv::Options opt;
  opt.paranoid_checks = true;
  const kv::FilterPolicy* fp = bloom_bits > 0 ? kv::NewBloomFilterPolicy(bloom_bits) : nullptr;
  opt.filter_policy = fp;
  MemRandom f(data, n);
  kv::Table* t = nullptr;
  kv::Status s = kv::Table::Open(opt, &f, n, &t);
  *blocks = 0;
  int rc = StatusCode(s);
  if (s.ok()) {
    kv::ReadOptions ro;
    ro.verify_checksums = true;
    kv::Iterator* it = t->NewIterator(ro);
    for (it->SeekToFirst(); it->Valid(); it->Next()) {
    }
    rc = StatusCode(it->status());
    delete it;
    delete t;
  }
  delete fp;
  return rc;
}

// MakeInputIteratorKV (kv/src/db/version_set.cc:1348-1373) over n table
// images: Table::Open with paranoid_checks = verify (TableCache::FindTable),
// an error iterator for a table that fails to open, NewIterator with
// verify_checksums = verify and fill_cache = false, NewMergingIterator under
// InternalKeyComparator(Bytewise) (internal) or BytewiseComparator.  Writes
// the merged entries like wsst_merge_tables; returns the status code
// (-2 when a capacity is exceeded).
int ref_merge_tables(const char* const* imgs, const size_t* sizes, size_t n, int internal,
                     int verify, char* kout, size_t kcap, uint32_t* klens, char* vout,
                     size_t vcap, uint32_t* vlens, size_t max_entries, size_t* nentries) {
  kv::InternalKeyComparator icmp(kv::BytewiseComparator());
  const kv::Comparator* cmp = internal ? static_cast<const kv::Comparator*>(&icmp)
                                       : kv::BytewiseComparator();
  kv::Options opt;
  opt.comparator = cmp;
  opt.paranoid_checks = verify != 0;
  kv::ReadOptions ro;
  ro.verify_checksums = verify != 0;
  ro.fill_cache = false;
  std::vector<std::unique_ptr<MemRandom>> files;
  std::vector<kv::Table*> tables;
  std::vector<kv::Iterator*> list;
  for (size_t i = 0; i < n; ++i) {
    files.emplace_back(new MemRandom(imgs[i], sizes[i]));
    kv::Table* t = nullptr;
    kv::Status s = kv::Table::Open(opt, files.back().get(), sizes[i], &t);
    if (s.ok()) {
      tables.push_back(t);
      list.push_back(t->NewIterator(ro));
    } else {
      list.push_back(kv::NewErrorIterator(s));
    }
  }
  kv::Iterator* it = kv::NewMergingIterator(cmp, list.data(), static_cast<int>(list.size()));
  size_t k = 0, ko = 0, vo = 0;
  int rc = 0;
  for (it->SeekToFirst(); it->Valid(); it->Next(), ++k) {
    const kv::Slice key = it->key(), val = it->value();
    if (k >= max_entries || ko + key.size() > kcap || vo + val.size() > vcap) {
      rc = -2;
      break;
    }
    memcpy(kout + ko, key.data(), key.size());
    memcpy(vout + vo, val.data(), val.size());
    klens[k] = static_cast<uint32_t>(key.size());
    vlens[k] = static_cast<uint32_t>(val.size());
    ko += key.size();
    vo += val.size();
  }
  *nentries = k;
  if (rc == 0) rc = StatusCode(it->status());
  delete it;
  for (kv::Table* t : tables) delete t;
  return rc;
}

// ReadBlock(verify_checksums) on one handle of a table image: 0 OK,
// 1 other corruption, 2 checksum mismatch, 3 other error.
int ref_read_block(const char* data, size_t n, uint64_t offset, uint64_t size) {
  MemRandom f(data, n);
  kv::ReadOptions ro;
  ro.verify_checksums = true;
  kv::BlockHandle h;
  h.set_offset(offset);
  h.set_size(size);
  kv::BlockContents c;
  kv::Status s = kv::ReadBlock(&f, ro, h, &c);
  if (s.ok() && c.heap_allocated) delete[] c.data.data();
  return StatusCode(s);
}

}  // extern "C"
