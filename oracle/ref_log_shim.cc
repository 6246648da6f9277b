// oracle/ref_log_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" driver over the reference's WAL code, compiled in place from
// /root/reference/kv/src (oracle/Makefile, into libref_table.so):
//   kv::log::Writer::AddRecord    kv/src/db/log_writer.cc:38-154
//   kv::log::Reader::ReadRecord   kv/src/db/log_reader.cc:62-279
// so the tests can byte-compare the batched log writer with the reference's
// and check that the batched recovery reader returns the same records and
// the same corruption reports for clean and damaged log images.
#include <stdint.h>
#include <string.h>

#include <memory>
#include <string>

#include "db/log_reader.h"
#include "db/log_writer.h"
#include "kv/env.h"
#include "util/file_reader_writer.h"

namespace {

class MemWritable : public kv::WritableFile {
 public:
  std::string* data;
  explicit MemWritable(std::string* d) : data(d) {}
  kv::Status Append(const kv::Slice& s) override {
    data->append(s.data(), s.size());
    return kv::Status::OK();
  }
  kv::Status Close() override { return kv::Status::OK(); }
  kv::Status Flush() override { return kv::Status::OK(); }
  kv::Status Sync() override { return kv::Status::OK(); }
};

class MemSequential : public kv::SequentialFile {
 public:
  const char* p;
  size_t n, pos = 0;
  MemSequential(const char* p_, size_t n_) : p(p_), n(n_) {}
  kv::Status Read(size_t len, kv::Slice* result, char* scratch) override {
    const size_t m = pos + len <= n ? len : n - pos;
    memcpy(scratch, p + pos, m);
    pos += m;
    *result = kv::Slice(scratch, m);
    return kv::Status::OK();
  }
  kv::Status Skip(uint64_t k) override {
    pos = pos + k <= n ? pos + k : n;
    return kv::Status::OK();
  }
};

class Collect : public kv::log::Reader::Reporter {
 public:
  uint64_t* bytes;
  char* reasons;
  size_t cap, n = 0;
  Collect(uint64_t* b, char* r, size_t c) : bytes(b), reasons(r), cap(c) {}
  void Corruption(size_t nbytes, const kv::Status& s) override {
    if (n < cap) {
      bytes[n] = nbytes;
      std::string m = s.ToString();
      strncpy(reasons + 64 * n, m.c_str(), 63);
      reasons[64 * n + 63] = 0;
    }
    ++n;
  }
};

}  // namespace

extern "C" {

// AddRecord for n records (concatenated + lengths) into a fresh log; returns
// the image size (or -1), copying at most cap bytes to out.
long ref_log_write(const char* recs, const uint32_t* lens, size_t n, int recycle,
                   uint64_t log_number, char* out, size_t cap) {
  std::string data;
  long rc = -1;
  {
    kv::EnvOptions eo;
    std::unique_ptr<kv::WritableFileWriter> w(
        new kv::WritableFileWriter(new MemWritable(&data), "mem.log", eo, false));
    kv::log::Writer lw(std::move(w), log_number, recycle != 0, false);
    size_t o = 0;
    kv::Status s;
    for (size_t i = 0; i < n && s.ok(); ++i) {
      s = lw.AddRecord(kv::Slice(recs + o, lens[i]));
      o += lens[i];
    }
    if (s.ok()) rc = 0;
  }
  if (rc == 0) {
    rc = static_cast<long>(data.size());
    memcpy(out, data.data(), data.size() < cap ? data.size() : cap);
  }
  return rc;
}

// Reader(checksum, initial_offset 0) over a log image: every record
// (bytes into rec_out, lengths, LastRecordOffset) and every Corruption()
// report (dropped bytes, "Corruption: <reason>" in 64-byte slots).
int ref_log_read(const char* img, size_t n, int checksum, char* rec_out, size_t rec_cap,
                 uint32_t* rec_lens, uint64_t* rec_offsets, size_t max_recs, size_t* nrecs,
                 uint64_t* drop_bytes, char* drop_reasons, size_t max_drops, size_t* ndrops) {
  MemSequential f(img, n);
  Collect rep(drop_bytes, drop_reasons, max_drops);
  kv::log::Reader r(&f, &rep, checksum != 0, 0);
  kv::Slice rec;
  std::string scratch;
  size_t k = 0, used = 0;
  int rc = 0;
  while (r.ReadRecord(&rec, &scratch)) {
    if (k < max_recs && used + rec.size() <= rec_cap) {
      memcpy(rec_out + used, rec.data(), rec.size());
      rec_lens[k] = static_cast<uint32_t>(rec.size());
      rec_offsets[k] = r.LastRecordOffset();
      used += rec.size();
    } else {
      rc = -2;
    }
    ++k;
  }
  *nrecs = k;
  *ndrops = rep.n;
  return rc;
}

}  // extern "C"
