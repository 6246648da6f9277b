// include/wipdb/table.h -- SST writing and verification with batched block
// checksums.
//
// TableBuilder mirrors kv::TableBuilder (kv/src/include/kv/table_builder.h,
// kv/src/table/table_builder.cc) and writes the identical bytes, but its
// WriteRawBlock (table_builder.cc:183-202) no longer computes the trailer
// CRC inline: it appends a placeholder trailer, records the span
// (contents || type byte), and the CRCs of all pending blocks are computed
// in ONE batch -- on the MI355X through the C-ABI (hcrc_batch), or on the
// host -- and patched in right before the bytes leave the builder's buffer
// (at most TableOptions::max_buffer_size, the WritableFileWriter buffer of
// kv/src/include/kv/env.h:85, and at Finish).  FinishTables() finishes many
// builders (one compaction's outputs) with a single batch.
//
// VerifyTable / VerifyTables are Table::Open(paranoid_checks) + a full
// iteration with ReadOptions::verify_checksums (kv/src/table/table.cc:37-82,
// format.cc:66-143), as batches: all index blocks in one batch, then every
// data block of every table in one batch.  The status is the one the
// reference reports for the same image; per-block results are returned too.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <string_view>
#include <vector>

#include "wipdb/status.h"

namespace wipdb {
namespace table {

// Where block checksums are computed.
enum class CrcMode {
  kInline = 0,     // per block, host CPU, at WriteRawBlock (the reference's schedule)
  kBatchCpu = 1,   // deferred and batched, host CPU
  kBatchGpu = 2,   // deferred and batched on the MI355X; a device error is a Status
  kBatchAuto = 3,  // deferred and batched; MI355X when usable, else host
};

// The table-side methods of kv::Comparator (kv/src/include/kv/comparator.h:
// 18-70): the builder shortens index keys with them.
class Comparator {
 public:
  virtual ~Comparator() = default;
  virtual const char* Name() const = 0;
  virtual int Compare(std::string_view a, std::string_view b) const = 0;
  // If *start < limit, changes *start to a short key in [start, limit).
  virtual void FindShortestSeparator(std::string* start, std::string_view limit) const = 0;
  // Changes *key to a short key >= *key.
  virtual void FindShortSuccessor(std::string* key) const = 0;
};

// kv::BytewiseComparator() (kv/src/util/comparator.cc:22-96).
const Comparator* BytewiseComparator();

// kv::InternalKeyComparator (kv/src/db/dbformat.cc:45-120): keys are
// user_key || fixed64(sequence << 8 | type); order is user key ascending
// (by `user`), then sequence descending.  A shortened user key gets the tag
// (kMaxSequenceNumber, kValueTypeForSeek).  This is the comparator WipDB's
// flush and compaction build every SST with (SanitizeOptions,
// kv/src/db/db_impl.cc:104-111,141-144).
class InternalKeyComparator : public Comparator {
 public:
  explicit InternalKeyComparator(const Comparator* user) : user_(user) {}
  const char* Name() const override;
  int Compare(std::string_view a, std::string_view b) const override;
  void FindShortestSeparator(std::string* start, std::string_view limit) const override;
  void FindShortSuccessor(std::string* key) const override;
  const Comparator* user_comparator() const { return user_; }

 private:
  const Comparator* user_;
};

// InternalKeyComparator(BytewiseComparator()), process-lifetime.
const Comparator* InternalBytewiseComparator();

// Which bytes of a key the bloom filter hashes.
enum class FilterKeys {
  kWholeKey = 0,  // NewBloomFilterPolicy used directly (kv::Options default)
  kUserKey = 1,   // InternalFilterPolicy: ExtractUserKey(key), the 8-byte tag
                  // stripped (kv/src/db/dbformat.cc:122-136)
};

struct TableOptions {
  size_t block_size = 4096;          // kv/src/util/options.cc:22
  int block_restart_interval = 16;   // options.cc:23
  int bloom_bits_per_key = 0;        // 0: no filter policy; else NewBloomFilterPolicy(bits)
  size_t max_buffer_size = 4u << 20; // EnvOptions::writable_file_max_buffer_size (env.h:85)
  CrcMode crc_mode = CrcMode::kBatchAuto;
  int device = -1;                   // HIP device for the batched modes; -1: WIPDB_CRC_DEVICES, else 0
                                     // (wipdb::crc32c::kDeviceFromEnv)
  const Comparator* comparator = nullptr;  // nullptr: BytewiseComparator()
  FilterKeys filter_keys = FilterKeys::kWholeKey;
  // kBatchGpu / kBatchAuto: the write buffer is pinned host memory (pooled),
  // so block CRC batches read it zero-copy instead of through staging
  bool pinned_buffers = true;
};

// The options WipDB's DB hands its TableBuilders (BuildTableKV,
// kv/src/db/builder.cc:46, and compaction outputs): internal keys over the
// bytewise user comparator, the bloom filter wrapped in InternalFilterPolicy.
TableOptions InternalKeyTableOptions(TableOptions base);

// Destination of a table's bytes (the WritableFileWriter role).
class TableSink {
 public:
  virtual ~TableSink() = default;
  virtual Status Append(const char* data, size_t n) = 0;
};

class StringSink : public TableSink {
 public:
  Status Append(const char* data, size_t n) override {
    contents.append(data, n);
    return Status::OK();
  }
  std::string contents;
};

class TableBuilder {
 public:
  TableBuilder(const TableOptions& options, TableSink* sink);
  ~TableBuilder();
  TableBuilder(const TableBuilder&) = delete;
  TableBuilder& operator=(const TableBuilder&) = delete;

  // REQUIRES: key > every key added before (in options.comparator's order).
  void Add(std::string_view key, std::string_view value);
  void Flush();
  Status Finish();
  void Abandon();
  Status status() const;
  uint64_t NumEntries() const;
  uint64_t FileSize() const;
  // Blocks whose CRC was computed in a batch (deferred modes).
  uint64_t BatchedBlocks() const;

 private:
  friend Status FinishTables(TableBuilder* const* builders, size_t n);
  struct Rep;
  Rep* rep_;
};

// Finish() for n builders sharing one TableOptions::crc_mode, with the CRCs
// of all their still-buffered blocks computed in ONE batch.  Returns the
// first non-OK status; every builder is finished either way.
Status FinishTables(TableBuilder* const* builders, size_t n);

// ---- verification ----
enum class BlockKind : uint8_t { kData = 0, kIndex = 1, kMetaIndex = 2, kFilter = 3 };

struct BlockCheck {
  uint64_t offset;
  uint64_t size;   // handle size (contents, without the 5-byte trailer)
  BlockKind kind;
  bool ok;         // trailer present and Unmask(stored) == crc32c(contents || type)
};

// ReadBlock(verify_checksums) over an in-memory table image (format.cc:66-143):
// OK, "truncated block read", "block checksum mismatch", "bad block type",
// "corrupted compressed block contents".  *contents views the block.
Status ReadBlock(const char* image, size_t image_size, uint64_t offset, uint64_t size,
                 bool verify_checksums, std::string_view* contents);

// Table::Open(paranoid_checks = true) + iterating every data block with
// verify_checksums = true; meta-index and filter blocks are verified too but,
// as in Table::ReadMeta (table.cc:84-138), their failures do not fail the
// table.  blocks (optional) receives every block checked, in file order of
// discovery.  bloom_bits_per_key > 0 reads the filter named by the policy.
Status VerifyTable(const char* image, size_t image_size, int bloom_bits_per_key, CrcMode mode,
                   int device, std::vector<BlockCheck>* blocks);

// The same for many tables at once: one batch for the index blocks, one for
// every other block.  statuses[i] is table i's status.
Status VerifyTables(const char* const* images, const size_t* sizes, size_t n,
                    int bloom_bits_per_key, CrcMode mode, int device,
                    std::vector<Status>* statuses);

// ---- the compaction input path ----
//
// VersionSet::MakeInputIteratorKV (kv/src/db/version_set.cc:1348-1373): a
// merging iterator (table/merger.cc, ties to the lower input) over the input
// tables' two-level iterators (Table::NewIterator, table.cc:164-229), with
// ReadOptions::verify_checksums = paranoid_checks.  The reference reads and
// checks one data block at a time in Table::BlockReader; this reader checks
// the next `prefetch_blocks` blocks of EVERY input in one CRC batch (on the
// MI355X in the batched modes) whenever the merge reaches an unchecked
// block.  Same entries, same order, same status: an input whose Open fails
// contributes nothing; a block that fails (checksum, short read, bad type,
// bad handle) is skipped and its error kept; status() is the first input's
// (in input order) first error, an index-block error first
// (TwoLevelIterator::status).
class CompactionInput {
 public:
  struct Options {
    const Comparator* comparator = nullptr;  // nullptr: InternalBytewiseComparator()
    bool verify_checksums = true;            // Options::paranoid_checks
    size_t prefetch_blocks = 64;             // per input and CRC batch
    CrcMode crc_mode = CrcMode::kBatchAuto;
    int device = -1;  // -1: WIPDB_CRC_DEVICES, else 0 (crc32c::kDeviceFromEnv)
  };
  // The images must outlive the reader (an mmap'd file, or pinned memory for
  // zero-copy batches).
  CompactionInput(const char* const* images, const size_t* sizes, size_t n, const Options& o);
  ~CompactionInput();
  CompactionInput(const CompactionInput&) = delete;
  CompactionInput& operator=(const CompactionInput&) = delete;

  void SeekToFirst();
  bool Valid() const;
  void Next();
  std::string_view key() const;    // REQUIRES: Valid()
  std::string_view value() const;  // REQUIRES: Valid()
  Status status() const;
  uint64_t CrcBatches() const;     // CRC batches issued (index blocks included)
  uint64_t BlocksChecked() const;  // block CRCs computed

 private:
  struct Rep;
  Rep* rep_;
};

}  // namespace table
}  // namespace wipdb
