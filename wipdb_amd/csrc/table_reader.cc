// table_reader.cc -- batched block-checksum verification of table images
// (SURVEY.md 8f-2): kv::ReadBlock (kv/src/table/format.cc:66-143) and
// Table::Open / ReadMeta / ReadFilter with paranoid_checks plus a full
// verified iteration (kv/src/table/table.cc:37-138), with every block CRC of
// a stage computed in one batch (span_crc.h); and the compaction input path
// (CompactionInput: MakeInputIteratorKV, kv/src/db/version_set.cc:1348-1373)
// with its data blocks checked ahead of the merge, many per batch.
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/wipdb/crc32c.h"
#include "../../include/wipdb/table.h"
#include "span_crc.h"
#include "sst_format.h"

namespace wipdb {
namespace table {

namespace {

using sst::Handle;

// Bounds of a block read (format.cc:73-84): n + 5 bytes must be there.
bool InBounds(size_t image_size, const Handle& h) {
  return h.offset <= image_size && h.size <= image_size &&
         h.size + sst::kBlockTrailerSize <= image_size - h.offset;
}

// After the CRC: the type byte decides (format.cc:101-140).  Snappy is not
// built in, so type 1 fails like a snappy-less reference build.
Status TypeStatus(const char* image, const Handle& h) {
  const int type = static_cast<uint8_t>(image[h.offset + h.size]);
  if (type == sst::kNoCompression) return Status::OK();
  if (type == sst::kSnappyCompression)
    return Status::Corruption("corrupted compressed block contents");
  return Status::Corruption("bad block type");
}

uint32_t StoredCrc(const char* image, const Handle& h) {
  return kv::crc32c::Unmask(sst::DecodeFixed32(image + h.offset + h.size + 1));
}

// Entries of a block (kv/src/table/block.cc): the values, in order.  Fails
// like Block's constructor / iterator ("bad block contents", "bad entry in
// block").
template <class Sink>
Status ForEachEntry(std::string_view b, std::string* key, Sink&& sink) {
  if (b.size() < 4) return Status::Corruption("bad block contents");
  const uint32_t nrest = sst::DecodeFixed32(b.data() + b.size() - 4);
  if (nrest > (b.size() - 4) / 4) return Status::Corruption("bad block contents");
  if (nrest == 0) return Status::OK();  // an empty iterator (block.cc:261-262)
  const size_t limit_off = b.size() - (1 + size_t(nrest)) * 4;
  // SeekToFirst: the first entry is at restart point 0 (block.cc SeekToRestartPoint)
  const char* p = b.data() + sst::DecodeFixed32(b.data() + limit_off);
  const char* limit = b.data() + limit_off;
  key->clear();
  while (p < limit) {
    uint32_t shared, non_shared, vlen;
    p = sst::GetVarint32(p, limit, &shared);
    if (p) p = sst::GetVarint32(p, limit, &non_shared);
    if (p) p = sst::GetVarint32(p, limit, &vlen);
    if (!p || static_cast<size_t>(limit - p) < size_t(non_shared) + vlen || shared > key->size())
      return Status::Corruption("bad entry in block");
    key->resize(shared);
    key->append(p, non_shared);
    sink(*key, std::string_view(p + non_shared, vlen));
    p += non_shared + vlen;
  }
  return Status::OK();
}
Status BlockValues(std::string_view b, std::vector<std::pair<std::string, std::string_view>>* kv) {
  std::string key;
  return ForEachEntry(b, &key, [kv](const std::string& k, std::string_view v) { kv->emplace_back(k, v); });
}

struct TableJob {
  const char* img;
  size_t size;
  Status st;
  Handle meta, index;
  std::vector<Handle> data;
  bool has_filter = false;
  Handle filter;
  std::vector<BlockCheck> checks;
};

// One batch over (table, handle) pairs already bounds-checked: ok[i].
Status CheckBatch(const std::vector<TableJob*>& t, const std::vector<Handle>& h, CrcMode mode,
                  int device, std::vector<bool>* ok) {
  std::vector<const char*> p(h.size());
  std::vector<uint32_t> l(h.size()), crc(h.size());
  for (size_t i = 0; i < h.size(); ++i) {
    p[i] = t[i]->img + h[i].offset;
    l[i] = static_cast<uint32_t>(h[i].size + 1);
  }
  Status s = spancrc::Compute(p.data(), l.data(), h.size(), false, mode, device, crc.data());
  if (!s.ok()) return s;
  ok->resize(h.size());
  for (size_t i = 0; i < h.size(); ++i) (*ok)[i] = crc[i] == StoredCrc(t[i]->img, h[i]);
  return Status::OK();
}

Status VerifyJobs(std::vector<TableJob>& jobs, int bloom_bits, CrcMode mode, int device) {
  // 1. footers (format.cc:34-62, table.cc:44-59)
  std::vector<TableJob*> bt;
  std::vector<Handle> bh;
  std::vector<BlockKind> bk;
  for (TableJob& j : jobs) {
    if (j.size < sst::kFooterLength) {
      j.st = Status::Corruption("file is too short to be an sstable");
      continue;
    }
    const char* f = j.img + j.size - sst::kFooterLength;
    const uint64_t magic = uint64_t(sst::DecodeFixed32(f + sst::kFooterLength - 8)) |
                           (uint64_t(sst::DecodeFixed32(f + sst::kFooterLength - 4)) << 32);
    if (magic != sst::kTableMagicNumber) {
      j.st = Status::Corruption("not an sstable (bad magic number)");
      continue;
    }
    std::string_view in(f, sst::kFooterLength);
    if (!j.meta.DecodeFrom(&in) || !j.index.DecodeFrom(&in)) {
      j.st = Status::Corruption("bad block handle");
      continue;
    }
    // the index block gates Open; the meta-index is read only with a policy
    if (!InBounds(j.size, j.index)) {
      j.st = Status::Corruption("truncated block read");
      j.checks.push_back({j.index.offset, j.index.size, BlockKind::kIndex, false});
      continue;
    }
    bt.push_back(&j);
    bh.push_back(j.index);
    bk.push_back(BlockKind::kIndex);
    if (bloom_bits > 0) {
      if (InBounds(j.size, j.meta)) {
        bt.push_back(&j);
        bh.push_back(j.meta);
        bk.push_back(BlockKind::kMetaIndex);
      } else {
        j.checks.push_back({j.meta.offset, j.meta.size, BlockKind::kMetaIndex, false});
      }
    }
  }
  // 2. one batch: every index (and meta-index) block
  std::vector<bool> ok;
  Status s = CheckBatch(bt, bh, mode, device, &ok);
  if (!s.ok()) return s;
  for (size_t i = 0; i < bt.size(); ++i) {
    TableJob& j = *bt[i];
    j.checks.push_back({bh[i].offset, bh[i].size, bk[i], static_cast<bool>(ok[i])});
    Status bs = ok[i] ? TypeStatus(j.img, bh[i]) : Status::Corruption("block checksum mismatch");
    std::vector<std::pair<std::string, std::string_view>> ents;
    if (bk[i] == BlockKind::kIndex) {
      if (!bs.ok()) {
        j.st = bs;
        continue;
      }
      // 3. the index's values are the data block handles (two_level_iterator)
      Status ps = BlockValues(std::string_view(j.img + bh[i].offset, bh[i].size), &ents);
      for (auto& e : ents) {
        if (!ps.ok()) break;
        Handle h;
        std::string_view v = e.second;
        if (!h.DecodeFrom(&v)) ps = Status::Corruption("bad block handle");
        else j.data.push_back(h);
      }
      if (!ps.ok()) j.st = ps;
    } else if (bs.ok()) {
      // meta-index: "filter.<policy name>" -> filter handle (table.cc:84-113)
      if (BlockValues(std::string_view(j.img + bh[i].offset, bh[i].size), &ents).ok()) {
        const std::string want = std::string("filter.") + sst::Bloom::Name();
        for (auto& e : ents) {
          if (e.first != want) continue;
          std::string_view v = e.second;
          j.has_filter = j.filter.DecodeFrom(&v);
        }
      }
    }
  }
  // 4. one batch: every data block (and filter) of every table
  bt.clear();
  bh.clear();
  bk.clear();
  for (TableJob& j : jobs) {
    if (!j.st.ok()) continue;  // Open failed: nothing is iterated
    if (j.has_filter) {
      if (InBounds(j.size, j.filter)) {
        bt.push_back(&j);
        bh.push_back(j.filter);
        bk.push_back(BlockKind::kFilter);
      } else {
        j.checks.push_back({j.filter.offset, j.filter.size, BlockKind::kFilter, false});
      }
    }
    for (const Handle& h : j.data) {  // short reads are reported in index order below
      bt.push_back(&j);
      bh.push_back(h);
      bk.push_back(BlockKind::kData);
    }
  }
  // out-of-bounds handles are kept out of the CRC batch
  std::vector<TableJob*> ct;
  std::vector<Handle> ch;
  std::vector<size_t> at(bh.size(), SIZE_MAX);
  for (size_t i = 0; i < bh.size(); ++i) {
    if (!InBounds(bt[i]->size, bh[i])) continue;
    at[i] = ch.size();
    ct.push_back(bt[i]);
    ch.push_back(bh[i]);
  }
  s = CheckBatch(ct, ch, mode, device, &ok);
  if (!s.ok()) return s;
  for (size_t i = 0; i < bh.size(); ++i) {
    TableJob& j = *bt[i];
    const bool in = at[i] != SIZE_MAX;
    const bool good = in && ok[at[i]];
    j.checks.push_back({bh[i].offset, bh[i].size, bk[i], good});
    if (bk[i] != BlockKind::kData || !j.st.ok()) continue;
    // the first failing data block in index order sets the table's status
    if (!in) j.st = Status::Corruption("truncated block read");
    else if (!good) j.st = Status::Corruption("block checksum mismatch");
    else j.st = TypeStatus(j.img, bh[i]);
  }
  return Status::OK();
}

}  // namespace

Status ReadBlock(const char* image, size_t image_size, uint64_t offset, uint64_t size,
                 bool verify_checksums, std::string_view* contents) {
  Handle h;
  h.offset = offset;
  h.size = size;
  if (!InBounds(image_size, h)) return Status::Corruption("truncated block read");
  if (verify_checksums) {
    const uint32_t actual = kv::crc32c::Value(image + offset, size + 1);
    if (actual != StoredCrc(image, h)) return Status::Corruption("block checksum mismatch");
  }
  Status s = TypeStatus(image, h);
  if (s.ok() && contents) *contents = std::string_view(image + offset, size);
  return s;
}

Status VerifyTable(const char* image, size_t image_size, int bloom_bits_per_key, CrcMode mode,
                   int device, std::vector<BlockCheck>* blocks) {
  std::vector<TableJob> jobs(1);
  jobs[0].img = image;
  jobs[0].size = image_size;
  Status s = VerifyJobs(jobs, bloom_bits_per_key, mode, device);
  if (!s.ok()) return s;
  if (blocks) *blocks = std::move(jobs[0].checks);
  return jobs[0].st;
}

Status VerifyTables(const char* const* images, const size_t* sizes, size_t n,
                    int bloom_bits_per_key, CrcMode mode, int device,
                    std::vector<Status>* statuses) {
  std::vector<TableJob> jobs(n);
  for (size_t i = 0; i < n; ++i) {
    jobs[i].img = images[i];
    jobs[i].size = sizes[i];
  }
  Status s = VerifyJobs(jobs, bloom_bits_per_key, mode, device);
  if (!s.ok()) return s;
  Status first;
  if (statuses) statuses->clear();
  for (TableJob& j : jobs) {
    if (statuses) statuses->push_back(j.st);
    if (first.ok() && !j.st.ok()) first = j.st;
  }
  return first;
}

// ---------------------------------------------------------------------------
// CompactionInput
// ---------------------------------------------------------------------------
namespace {

// A block iterator's entries (kv/src/table/block.cc): decoded up to the end
// or the first bad entry ("bad entry in block", the entries before it are
// still returned), "bad block contents" for a block whose restart array
// does not fit.
Status BlockEntries(std::string_view b, std::vector<std::pair<std::string, std::string_view>>* kv) {
  kv->clear();
  return BlockValues(b, kv);
}

// Per-block state of the checks ahead of the merge.
enum : uint8_t { kUnchecked = 0, kGood = 1, kBadCrc = 2, kShort = 3 };

}  // namespace

struct CompactionInput::Rep {
  struct In {
    const char* img;
    size_t size;
    Status open;                 // Table::Open's status
    Status index;                // the index iterator's (bad entry in the index block)
    Status saved;                // TwoLevelIterator::status_: the first block error
    std::vector<Handle> blocks;  // data block handles, index order
    std::vector<Status> bad_handle;  // per block: "bad block handle" (value undecodable)
    std::vector<uint8_t> chk;    // per block: kUnchecked / kGood / kBadCrc / kShort
    size_t next_check = 0;       // first block not yet sent to a CRC batch
    size_t bi = 0;               // current block
    // the current block's entries: keys back to back in `arena`, values
    // viewing the image
    struct Ent {
      uint32_t ko, kl;
      const char* v;
      size_t vl;
    };
    std::string arena, scratch;
    std::vector<Ent> ents;
    size_t ei = 0;
    bool valid = false;
    std::string_view key() const { return {arena.data() + ents[ei].ko, ents[ei].kl}; }
    std::string_view value() const { return {ents[ei].v, ents[ei].vl}; }
    void Save(const Status& s) {
      if (saved.ok() && !s.ok()) saved = s;
    }
    Status status() const {
      if (!open.ok()) return open;
      if (!index.ok()) return index;
      return saved;
    }
  };
  Options opt;
  const Comparator* cmp;
  std::vector<In> in;
  uint64_t batches = 0, checked = 0;
  Status fatal;  // a device error of a CRC batch (kBatchGpu)
  // merge: a binary min-heap of the valid inputs by current key (ties: the
  // lower input first, merger.cc's order); the top is the current entry and
  // Next() re-sifts it in place
  std::vector<size_t> heap;
  size_t cur = SIZE_MAX;
  bool Before(size_t a, size_t b) const {
    const int c = cmp->Compare(in[a].key(), in[b].key());
    return c < 0 || (c == 0 && a < b);
  }
  void SiftDown(size_t pos) {
    const size_t n = heap.size();
    const size_t item = heap[pos];
    for (;;) {
      size_t c = 2 * pos + 1;
      if (c >= n) break;
      if (c + 1 < n && Before(heap[c + 1], heap[c])) ++c;
      if (!Before(heap[c], item)) break;
      heap[pos] = heap[c];
      pos = c;
    }
    heap[pos] = item;
  }
  void SiftUp(size_t pos) {
    const size_t item = heap[pos];
    while (pos > 0) {
      const size_t p = (pos - 1) / 2;
      if (!Before(item, heap[p])) break;
      heap[pos] = heap[p];
      pos = p;
    }
    heap[pos] = item;
  }

  void Open() {
    // Table::Open(paranoid_checks) of every input: one batch of index blocks
    std::vector<TableJob> jobs(in.size());
    std::vector<TableJob*> bt;
    std::vector<Handle> bh;
    for (size_t i = 0; i < in.size(); ++i) {
      TableJob& j = jobs[i];
      j.img = in[i].img;
      j.size = in[i].size;
      if (j.size < sst::kFooterLength) {
        in[i].open = Status::Corruption("file is too short to be an sstable");
        continue;
      }
      const char* f = j.img + j.size - sst::kFooterLength;
      const uint64_t magic = uint64_t(sst::DecodeFixed32(f + sst::kFooterLength - 8)) |
                             (uint64_t(sst::DecodeFixed32(f + sst::kFooterLength - 4)) << 32);
      std::string_view fin(f, sst::kFooterLength);
      if (magic != sst::kTableMagicNumber) {
        in[i].open = Status::Corruption("not an sstable (bad magic number)");
      } else if (!j.meta.DecodeFrom(&fin) || !j.index.DecodeFrom(&fin)) {
        in[i].open = Status::Corruption("bad block handle");
      } else if (!InBounds(j.size, j.index)) {
        in[i].open = Status::Corruption("truncated block read");
      } else {
        bt.push_back(&j);
        bh.push_back(j.index);
      }
    }
    std::vector<bool> ok;
    if (opt.verify_checksums && !bt.empty()) {
      fatal = CheckBatch(bt, bh, opt.crc_mode, opt.device, &ok);
      if (!fatal.ok()) return;
      ++batches;
      checked += bt.size();
    }
    for (size_t k = 0; k < bt.size(); ++k) {
      In& x = in[static_cast<size_t>(bt[k] - jobs.data())];
      const Handle& h = bh[k];
      if (opt.verify_checksums && !ok[k]) {
        x.open = Status::Corruption("block checksum mismatch");
        continue;
      }
      x.open = TypeStatus(x.img, h);
      if (!x.open.ok()) continue;
      // the index iterator: handles up to a bad entry (the index's status)
      std::vector<std::pair<std::string, std::string_view>> ents;
      x.index = BlockEntries(std::string_view(x.img + h.offset, h.size), &ents);
      for (auto& e : ents) {
        Handle bhd;
        std::string_view v = e.second;
        const bool good = bhd.DecodeFrom(&v);
        x.blocks.push_back(good ? bhd : Handle());
        x.bad_handle.push_back(good ? Status::OK() : Status::Corruption("bad block handle"));
      }
      x.chk.assign(x.blocks.size(), kUnchecked);
    }
  }

  // One CRC batch: the next prefetch_blocks unchecked blocks of every input
  // that still has some (the merge drains the inputs at similar rates).
  void CheckAhead() {
    std::vector<TableJob> jobs;
    std::vector<std::pair<size_t, size_t>> who;  // (input, block)
    std::vector<TableJob*> bt;
    std::vector<Handle> bh;
    jobs.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
      In& x = in[i];
      if (!x.open.ok()) continue;
      jobs.push_back(TableJob{});
      jobs.back().img = x.img;
      jobs.back().size = x.size;
      const size_t end = std::min(x.blocks.size(), x.next_check + opt.prefetch_blocks);
      for (size_t b = x.next_check; b < end; ++b) {
        if (!x.bad_handle[b].ok()) continue;
        if (!InBounds(x.size, x.blocks[b])) {
          x.chk[b] = kShort;
          continue;
        }
        who.emplace_back(i, b);
        bt.push_back(&jobs.back());
        bh.push_back(x.blocks[b]);
      }
      x.next_check = end;
    }
    if (bh.empty()) return;
    std::vector<bool> ok;
    fatal = CheckBatch(bt, bh, opt.crc_mode, opt.device, &ok);
    if (!fatal.ok()) return;
    ++batches;
    checked += bh.size();
    for (size_t k = 0; k < who.size(); ++k)
      in[who[k].first].chk[who[k].second] = ok[k] ? kGood : kBadCrc;
  }

  // Table::BlockReader + the two-level iterator's skip of empty or failed
  // blocks: position input x on block b or a later one with an entry.
  void Load(In& x, size_t b) {
    for (; b < x.blocks.size(); ++b) {
      x.bi = b;
      x.ents.clear();
      x.arena.clear();
      x.ei = 0;
      if (!x.bad_handle[b].ok()) {
        x.Save(x.bad_handle[b]);
        continue;
      }
      const Handle& h = x.blocks[b];
      if (!InBounds(x.size, h)) {
        x.Save(Status::Corruption("truncated block read"));
        continue;
      }
      if (opt.verify_checksums) {
        if (x.chk[b] == kUnchecked) CheckAhead();
        if (!fatal.ok()) break;
        if (x.chk[b] == kBadCrc) {
          x.Save(Status::Corruption("block checksum mismatch"));
          continue;
        }
      }
      const Status ts = TypeStatus(x.img, h);
      if (!ts.ok()) {
        x.Save(ts);
        continue;
      }
      x.Save(ForEachEntry(std::string_view(x.img + h.offset, h.size), &x.scratch,
                          [&x](const std::string& k, std::string_view v) {
                            x.ents.push_back(In::Ent{static_cast<uint32_t>(x.arena.size()),
                                                     static_cast<uint32_t>(k.size()), v.data(),
                                                     v.size()});
                            x.arena.append(k);
                          }));
      if (!x.ents.empty()) {
        x.valid = true;
        return;
      }
    }
    x.valid = false;
  }

  void Step(size_t i) {
    In& x = in[i];
    if (++x.ei < x.ents.size()) return;
    Load(x, x.bi + 1);
  }

  void Pick() {
    cur = SIZE_MAX;
    if (!fatal.ok() || heap.empty()) return;
    cur = heap[0];
  }
};

CompactionInput::CompactionInput(const char* const* images, const size_t* sizes, size_t n,
                                 const Options& o)
    : rep_(new Rep) {
  rep_->opt = o;
  if (rep_->opt.prefetch_blocks == 0) rep_->opt.prefetch_blocks = 1;
  rep_->cmp = o.comparator ? o.comparator : InternalBytewiseComparator();
  rep_->in.resize(n);
  for (size_t i = 0; i < n; ++i) {
    rep_->in[i].img = images[i];
    rep_->in[i].size = sizes[i];
  }
  rep_->Open();
}

CompactionInput::~CompactionInput() { delete rep_; }

void CompactionInput::SeekToFirst() {
  Rep* r = rep_;
  r->heap.clear();
  for (auto& x : r->in) {
    x.saved = Status::OK();
    x.valid = false;
  }
  if (!r->fatal.ok()) return;
  for (size_t i = 0; i < r->in.size(); ++i) {
    Rep::In& x = r->in[i];
    if (!x.open.ok()) continue;
    r->Load(x, 0);
    if (x.valid) {
      r->heap.push_back(i);
      r->SiftUp(r->heap.size() - 1);
    }
  }
  r->Pick();
}

bool CompactionInput::Valid() const { return rep_->cur != SIZE_MAX; }

void CompactionInput::Next() {
  Rep* r = rep_;
  const size_t i = r->cur;  // == heap[0]
  r->Step(i);
  if (!r->in[i].valid) {
    r->heap[0] = r->heap.back();
    r->heap.pop_back();
  }
  if (!r->heap.empty()) r->SiftDown(0);
  r->Pick();
}

std::string_view CompactionInput::key() const {
  return rep_->in[rep_->cur].key();
}

std::string_view CompactionInput::value() const {
  return rep_->in[rep_->cur].value();
}

Status CompactionInput::status() const {
  if (!rep_->fatal.ok()) return rep_->fatal;
  for (const auto& x : rep_->in)
    if (!x.status().ok()) return x.status();
  return Status::OK();
}

uint64_t CompactionInput::CrcBatches() const { return rep_->batches; }
uint64_t CompactionInput::BlocksChecked() const { return rep_->checked; }

}  // namespace table
}  // namespace wipdb
