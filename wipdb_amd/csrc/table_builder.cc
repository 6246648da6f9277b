// table_builder.cc -- wipdb::table::TableBuilder: kv::TableBuilder's table
// (kv/src/table/table_builder.cc) with the block-trailer CRCs computed in
// batches, and the span-batch helper of span_crc.h.
#include "../../include/wipdb/table.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <new>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/hip_crc32c_batch.h"
#include "../../include/wipdb/crc32c.h"
#include "span_crc.h"
#include "sst_format.h"

namespace wipdb {
namespace cpu {
uint32_t Extend(uint32_t init_crc, const void* data, size_t n);
}  // namespace cpu

namespace spancrc {

Status Compute(const char* const* ptrs, const uint32_t* lens, size_t n, bool mask,
               table::CrcMode mode, int device, uint32_t* out) {
  if (n == 0) return Status::OK();
  if (mode == table::CrcMode::kInline || mode == table::CrcMode::kBatchCpu) {
    for (size_t i = 0; i < n; ++i) {
      const uint32_t c = cpu::Extend(0, ptrs[i], lens[i]);
      out[i] = mask ? kv::crc32c::Mask(c) : c;
    }
    return Status::OK();
  }
  // The batch entry takes one base and 64-bit offsets: base = lowest span.
  const char* base = *std::min_element(ptrs, ptrs + n);
  std::vector<uint64_t> offs(n);
  for (size_t i = 0; i < n; ++i) offs[i] = static_cast<uint64_t>(ptrs[i] - base);
  const auto policy = mode == table::CrcMode::kBatchGpu ? crc32c::BatchPolicy::kGpuOnly
                                                        : crc32c::BatchPolicy::kAuto;
  const int rc = crc32c::ExtendBatch(base, offs.data(), lens, nullptr, out, n, mask, policy,
                                     device);
  if (rc != HCRC_OK) return Status::IOError(std::string("hcrc batch: ") + hcrc_strerror(rc));
  return Status::OK();
}

}  // namespace spancrc

namespace table {

using sst::Handle;

namespace {

class Bytewise : public Comparator {
 public:
  const char* Name() const override { return "leveldb.BytewiseComparator"; }
  int Compare(std::string_view a, std::string_view b) const override { return a.compare(b); }
  void FindShortestSeparator(std::string* start, std::string_view limit) const override {
    sst::ShortestSeparator(start, limit);
  }
  void FindShortSuccessor(std::string* key) const override { sst::ShortSuccessor(key); }
};

// dbformat.h:74-75, 68: the tag a shortened internal key gets
constexpr uint64_t kMaxSequenceNumber = (uint64_t(1) << 56) - 1;
constexpr uint64_t kValueTypeForSeek = 1;  // kTypeValue

void PutFixed64(std::string* d, uint64_t v) {
  sst::PutFixed32(d, static_cast<uint32_t>(v));
  sst::PutFixed32(d, static_cast<uint32_t>(v >> 32));
}
uint64_t DecodeFixed64(const char* p) {
  return uint64_t(sst::DecodeFixed32(p)) | (uint64_t(sst::DecodeFixed32(p + 4)) << 32);
}
// ExtractUserKey (dbformat.h:96-99); keys shorter than the tag are kept
// whole (the reference asserts size >= 8)
std::string_view UserKey(std::string_view k) { return k.size() >= 8 ? k.substr(0, k.size() - 8) : k; }

}  // namespace

const Comparator* BytewiseComparator() {
  static const Bytewise* c = new Bytewise;
  return c;
}

const char* InternalKeyComparator::Name() const { return "leveldb.InternalKeyComparator"; }

int InternalKeyComparator::Compare(std::string_view a, std::string_view b) const {
  int r = user_->Compare(UserKey(a), UserKey(b));
  if (r == 0 && a.size() >= 8 && b.size() >= 8) {
    const uint64_t an = DecodeFixed64(a.data() + a.size() - 8);
    const uint64_t bn = DecodeFixed64(b.data() + b.size() - 8);
    r = an > bn ? -1 : (an < bn ? 1 : 0);  // larger sequence first
  }
  return r;
}

void InternalKeyComparator::FindShortestSeparator(std::string* start, std::string_view limit) const {
  const std::string_view us = UserKey(*start);
  std::string tmp(us);
  user_->FindShortestSeparator(&tmp, UserKey(limit));
  if (tmp.size() < us.size() && user_->Compare(us, tmp) < 0) {
    PutFixed64(&tmp, (kMaxSequenceNumber << 8) | kValueTypeForSeek);
    start->swap(tmp);
  }
}

void InternalKeyComparator::FindShortSuccessor(std::string* key) const {
  const std::string_view uk = UserKey(*key);
  std::string tmp(uk);
  user_->FindShortSuccessor(&tmp);
  if (tmp.size() < uk.size() && user_->Compare(uk, tmp) < 0) {
    PutFixed64(&tmp, (kMaxSequenceNumber << 8) | kValueTypeForSeek);
    key->swap(tmp);
  }
}

const Comparator* InternalBytewiseComparator() {
  static const InternalKeyComparator* c = new InternalKeyComparator(BytewiseComparator());
  return c;
}

TableOptions InternalKeyTableOptions(TableOptions base) {
  base.comparator = InternalBytewiseComparator();
  base.filter_keys = FilterKeys::kUserKey;
  return base;
}

namespace {

// Pinned host buffers (hcrc_host_alloc) recycled process-wide: pinning is
// slow (milliseconds per MiB), table builders are many and short-lived.
class PinnedPool {
 public:
  static PinnedPool& Get() {
    static PinnedPool* p = new PinnedPool;
    return *p;
  }
  // A buffer of at least `bytes` (capacity in *cap), or nullptr when
  // pinned memory is unavailable (no device).
  char* Take(size_t bytes, size_t* cap) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = free_.lower_bound(bytes);
      if (it != free_.end() && it->first <= 2 * bytes) {
        char* p = it->second;
        *cap = it->first;
        held_ -= it->first;
        free_.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    if (hcrc_host_alloc(bytes, &p) != HCRC_OK) return nullptr;
    *cap = bytes;
    return static_cast<char*>(p);
  }
  void Give(char* p, size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (held_ + cap <= kMaxHeld) {
        free_.emplace(cap, p);
        held_ += cap;
        return;
      }
    }
    (void)hcrc_host_free(p);
  }

 private:
  static constexpr size_t kMaxHeld = size_t(1) << 30;
  std::mutex mu_;
  std::multimap<size_t, char*> free_;
  size_t held_ = 0;
};

// The builder's write buffer: pinned in the MI355X modes (so the batch of its
// block spans -- one builder's, or all of FinishTables' -- runs zero-copy,
// hcrc_host_alloc), plain heap memory otherwise or when pinning fails.
class HostBuf {
 public:
  HostBuf(bool pinned, size_t reserve) : pinned_(pinned) { Reserve(reserve); }
  ~HostBuf() { Release(); }
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  void append(const char* p, size_t n) {
    Reserve(size_ + n);
    memcpy(data_ + size_, p, n);
    size_ += n;
  }
  void append(const std::string& s) { append(s.data(), s.size()); }
  char* data() { return data_; }
  const char* data() const { return data_; }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  void clear() { size_ = 0; }
  char& operator[](size_t i) { return data_[i]; }

 private:
  void Reserve(size_t need) {
    if (need <= cap_) return;
    const size_t want = std::max(need, cap_ + cap_ / 2);
    size_t cap = 0;
    char* p = pinned_ ? PinnedPool::Get().Take(want, &cap) : nullptr;
    const bool pinned = p != nullptr;
    pinned_ = pinned;  // no pinned memory (no device): stop asking
    if (!p) {
      p = static_cast<char*>(malloc(want));
      if (!p) throw std::bad_alloc();
      cap = want;
    }
    if (size_) memcpy(p, data_, size_);
    Release();
    data_ = p;
    cap_ = cap;
    held_pinned_ = pinned;
  }
  void Release() {
    if (!data_) return;
    if (held_pinned_) PinnedPool::Get().Give(data_, cap_);
    else free(data_);
    data_ = nullptr;
    cap_ = 0;
  }
  bool pinned_;
  bool held_pinned_ = false;
  char* data_ = nullptr;
  size_t size_ = 0, cap_ = 0;
};

}  // namespace

struct TableBuilder::Rep {
  TableOptions opt;
  const Comparator* cmp;
  TableSink* sink;
  uint64_t offset = 0;  // file offset of the next byte
  Status status;
  sst::BlockBuilder data_block;
  sst::BlockBuilder index_block;
  std::string last_key;
  uint64_t num_entries = 0;
  bool closed = false;
  std::unique_ptr<sst::FilterBuilder> filter;
  bool pending_index_entry = false;
  Handle pending_handle;
  // bytes not yet handed to the sink
  HostBuf buf;
  // blocks in buf whose trailer CRC is still to be computed:
  // (position of the contents in buf, contents size + 1 type byte)
  std::vector<std::pair<size_t, uint32_t>> pending;
  uint64_t batched_blocks = 0;

  Rep(const TableOptions& o, TableSink* s)
      : opt(o),
        cmp(o.comparator ? o.comparator : BytewiseComparator()),
        sink(s),
        data_block(o.block_restart_interval),
        index_block(1),
        buf(o.pinned_buffers &&
                (o.crc_mode == CrcMode::kBatchGpu || o.crc_mode == CrcMode::kBatchAuto),
            o.max_buffer_size + (64u << 10)) {
    if (o.bloom_bits_per_key > 0) {
      filter.reset(new sst::FilterBuilder(o.bloom_bits_per_key));
      filter->StartBlock(0);
    }
  }

  bool deferred() const { return opt.crc_mode != CrcMode::kInline; }

  // kv TableBuilder::WriteRawBlock, with the CRC deferred in batched modes.
  void WriteRawBlock(std::string_view contents, int type, Handle* h) {
    h->offset = offset;
    h->size = contents.size();
    const size_t pos = buf.size();
    buf.append(contents.data(), contents.size());
    char trailer[sst::kBlockTrailerSize] = {static_cast<char>(type), 0, 0, 0, 0};
    if (!deferred()) {
      uint32_t crc = cpu::Extend(0, contents.data(), contents.size());
      crc = cpu::Extend(crc, trailer, 1);
      sst::EncodeFixed32(trailer + 1, kv::crc32c::Mask(crc));
    } else {
      pending.emplace_back(pos, static_cast<uint32_t>(contents.size() + 1));
    }
    buf.append(trailer, sizeof(trailer));
    offset += contents.size() + sst::kBlockTrailerSize;
    if (buf.size() >= opt.max_buffer_size) FlushBuffer();
  }

  void WriteBlock(sst::BlockBuilder* b, Handle* h) {
    // Compression is not built into this library: a snappy-less reference
    // build stores every block uncompressed with type 0 as well
    // (table_builder.cc:137-151, port_posix.h:194-205).
    WriteRawBlock(b->Finish(), sst::kNoCompression, h);
    b->Reset();
  }

  // Patches the trailers of pending blocks from crcs and hands buf over.
  void Drain(const uint32_t* crcs) {
    for (size_t i = 0; i < pending.size(); ++i)
      sst::EncodeFixed32(&buf[pending[i].first + pending[i].second], crcs[i]);
    batched_blocks += pending.size();
    pending.clear();
    if (status.ok() && !buf.empty()) status = sink->Append(buf.data(), buf.size());
    buf.clear();
  }

  void CollectSpans(std::vector<const char*>* p, std::vector<uint32_t>* l) const {
    for (const auto& s : pending) {
      p->push_back(buf.data() + s.first);
      l->push_back(s.second);
    }
  }

  void FlushBuffer() {
    std::vector<const char*> p;
    std::vector<uint32_t> l;
    CollectSpans(&p, &l);
    std::vector<uint32_t> crc(p.size());
    Status s = spancrc::Compute(p.data(), l.data(), p.size(), true, opt.crc_mode, opt.device,
                                crc.data());
    if (!s.ok()) {
      if (status.ok()) status = s;
      pending.clear();
      buf.clear();
      return;
    }
    Drain(crc.data());
  }

  void Flush() {
    if (!status.ok() || data_block.empty()) return;
    WriteBlock(&data_block, &pending_handle);
    if (status.ok()) pending_index_entry = true;
    if (filter) filter->StartBlock(offset);
  }

  // kv TableBuilder::Finish without the final buffer hand-over.
  void FinishBody() {
    Flush();
    closed = true;
    Handle filter_h, meta_h, index_h;
    if (status.ok() && filter) WriteRawBlock(filter->Finish(), sst::kNoCompression, &filter_h);
    if (status.ok()) {
      sst::BlockBuilder meta(opt.block_restart_interval);
      if (filter) {
        std::string enc;
        filter_h.EncodeTo(&enc);
        meta.Add(std::string("filter.") + sst::Bloom::Name(), enc);
      }
      WriteBlock(&meta, &meta_h);
    }
    if (status.ok()) {
      if (pending_index_entry) {
        cmp->FindShortSuccessor(&last_key);
        std::string enc;
        pending_handle.EncodeTo(&enc);
        index_block.Add(last_key, enc);
        pending_index_entry = false;
      }
      WriteBlock(&index_block, &index_h);
    }
    if (status.ok()) {
      std::string footer;
      sst::EncodeFooter(meta_h, index_h, &footer);
      buf.append(footer);
      offset += footer.size();
    }
  }
};

TableBuilder::TableBuilder(const TableOptions& options, TableSink* sink)
    : rep_(new Rep(options, sink)) {}

TableBuilder::~TableBuilder() { delete rep_; }

void TableBuilder::Add(std::string_view key, std::string_view value) {
  Rep* r = rep_;
  if (r->closed || !r->status.ok()) return;
  if (r->pending_index_entry) {
    r->cmp->FindShortestSeparator(&r->last_key, key);
    std::string enc;
    r->pending_handle.EncodeTo(&enc);
    r->index_block.Add(r->last_key, enc);
    r->pending_index_entry = false;
  }
  if (r->filter) r->filter->AddKey(r->opt.filter_keys == FilterKeys::kUserKey ? UserKey(key) : key);
  r->last_key.assign(key.data(), key.size());
  ++r->num_entries;
  r->data_block.Add(key, value);
  if (r->data_block.SizeEstimate() >= r->opt.block_size) r->Flush();
}

void TableBuilder::Flush() {
  if (!rep_->closed) rep_->Flush();
}

Status TableBuilder::Finish() {
  Rep* r = rep_;
  if (r->closed) return Status::InvalidArgument("table already finished or abandoned");
  r->FinishBody();
  if (r->status.ok()) r->FlushBuffer();
  return r->status;
}

void TableBuilder::Abandon() {
  Rep* r = rep_;
  if (r->closed) return;
  r->closed = true;
  // what was appended stays in the file, as with kv's WritableFileWriter
  if (r->status.ok()) r->FlushBuffer();
}

Status TableBuilder::status() const { return rep_->status; }
uint64_t TableBuilder::NumEntries() const { return rep_->num_entries; }
uint64_t TableBuilder::FileSize() const { return rep_->offset; }
uint64_t TableBuilder::BatchedBlocks() const { return rep_->batched_blocks; }

Status FinishTables(TableBuilder* const* builders, size_t n) {
  if (n == 0) return Status::OK();
  const CrcMode mode = builders[0]->rep_->opt.crc_mode;
  const int device = builders[0]->rep_->opt.device;
  for (size_t i = 0; i < n; ++i)
    if (builders[i]->rep_->opt.crc_mode != mode || builders[i]->rep_->opt.device != device)
      return Status::InvalidArgument("FinishTables: builders differ in crc_mode/device");
  std::vector<const char*> p;
  std::vector<uint32_t> l;
  std::vector<size_t> first(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    TableBuilder::Rep* r = builders[i]->rep_;
    if (!r->closed) r->FinishBody();
    first[i] = p.size();
    if (r->status.ok()) r->CollectSpans(&p, &l);
  }
  first[n] = p.size();
  std::vector<uint32_t> crc(p.size());
  Status s = spancrc::Compute(p.data(), l.data(), p.size(), true, mode, device, crc.data());
  Status result;
  for (size_t i = 0; i < n; ++i) {
    TableBuilder::Rep* r = builders[i]->rep_;
    if (!s.ok() && r->status.ok()) r->status = s;
    if (r->status.ok()) {
      r->Drain(crc.data() + first[i]);
    } else {
      r->pending.clear();
      r->buf.clear();
    }
    if (result.ok() && !r->status.ok()) result = r->status;
  }
  return result;
}

}  // namespace table
}  // namespace wipdb
