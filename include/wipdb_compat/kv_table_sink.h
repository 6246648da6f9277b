// include/wipdb_compat/kv_table_sink.h -- the reference-side adapter of the
// batched table builder.  Compiled INSIDE the reference
// tree (its kv/src and kv/src/include on the include path, ahead of this
// directory), it lets BuildTableKV (kv/src/db/builder.cc:18-109) and the
// compaction output path write through wipdb::table::TableBuilder instead of
// kv::TableBuilder, with the same WritableFileWriter, the same options and
// byte-identical files:
//
//   kv::WritableFileWriter w(file, fname, env_options, true);
//   wipdb::kvcompat::WritableFileWriterSink sink(&w);
//   wipdb::table::TableBuilder tb(wipdb::kvcompat::TableOptionsFrom(
//       options, env_options, /*bloom_bits=*/10, wipdb::table::CrcMode::kBatchAuto), &sink);
//   ... tb.Add(key, value) ...; tb.Finish(); w.Sync(false); w.Close();
//
// INTEGRATION.md section 3 shows the whole patch; tests/cpp/test_kv_builder.cc
// builds it against the compiled reference and byte-compares.
#pragma once
#include <string.h>

#include "kv/options.h"
#include "kv/status.h"
#include "util/file_reader_writer.h"
#include "wipdb/table.h"

namespace wipdb {
namespace kvcompat {

// TableSink over kv::WritableFileWriter::Append (kv/src/util/file_reader_writer.cc:30-98):
// the builder hands over whole buffers (at most max_buffer_size bytes, or the
// rest at Finish), the writer buffers / writes them as it did for
// kv::TableBuilder.
class WritableFileWriterSink : public table::TableSink {
 public:
  explicit WritableFileWriterSink(kv::WritableFileWriter* w) : w_(w) {}
  Status Append(const char* data, size_t n) override {
    const kv::Status s = w_->Append(kv::Slice(data, n));
    return s.ok() ? Status::OK() : Status::IOError(s.ToString());
  }

 private:
  kv::WritableFileWriter* w_;
};

// The table options a kv::Options (as SanitizeOptions leaves it,
// kv/src/db/db_impl.cc:104-111) stands for.  kv::FilterPolicy does not expose
// its bits per key, so the caller passes what it gave NewBloomFilterPolicy
// (0 = no filter policy).  An InternalKeyComparator selects internal keys
// and the InternalFilterPolicy's user-key hashing.
inline table::TableOptions TableOptionsFrom(const kv::Options& o, const kv::EnvOptions& eo,
                                            int bloom_bits, table::CrcMode mode,
                                            int device = 0) {
  table::TableOptions t;
  t.block_size = o.block_size;
  t.block_restart_interval = o.block_restart_interval;
  t.bloom_bits_per_key = o.filter_policy ? bloom_bits : 0;
  t.max_buffer_size = eo.writable_file_max_buffer_size;
  t.crc_mode = mode;
  t.device = device;
  if (o.comparator && strcmp(o.comparator->Name(), "leveldb.InternalKeyComparator") == 0)
    t = table::InternalKeyTableOptions(t);
  return t;
}

}  // namespace kvcompat
}  // namespace wipdb
