// table_reader.cc -- batched block-checksum verification of table images
// (SURVEY.md 8f-2): kv::ReadBlock (kv/src/table/format.cc:66-143) and
// Table::Open / ReadMeta / ReadFilter with paranoid_checks plus a full
// verified iteration (kv/src/table/table.cc:37-138), with every block CRC of
// a stage computed in one batch (span_crc.h).
#include <stdint.h>

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
Status BlockValues(std::string_view b, std::vector<std::pair<std::string, std::string_view>>* kv) {
  if (b.size() < 4) return Status::Corruption("bad block contents");
  const uint32_t nrest = sst::DecodeFixed32(b.data() + b.size() - 4);
  if (nrest > (b.size() - 4) / 4) return Status::Corruption("bad block contents");
  const size_t limit_off = b.size() - (1 + size_t(nrest)) * 4;
  const char* p = b.data();
  const char* limit = b.data() + limit_off;
  std::string key;
  while (p < limit) {
    uint32_t shared, non_shared, vlen;
    p = sst::GetVarint32(p, limit, &shared);
    if (p) p = sst::GetVarint32(p, limit, &non_shared);
    if (p) p = sst::GetVarint32(p, limit, &vlen);
    if (!p || static_cast<size_t>(limit - p) < size_t(non_shared) + vlen || shared > key.size())
      return Status::Corruption("bad entry in block");
    key.resize(shared);
    key.append(p, non_shared);
    kv->emplace_back(key, std::string_view(p + non_shared, vlen));
    p += non_shared + vlen;
  }
  return Status::OK();
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

}  // namespace table
}  // namespace wipdb
