// log_batch.cc -- the write-ahead log with batched record CRCs (SURVEY.md
// 8f-3): kv::log::Writer::AddRecord (kv/src/db/log_writer.cc:38-154) laid
// out for many records with one CRC batch, and kv::log::Reader::ReadRecord
// (kv/src/db/log_reader.cc:62-279) over whole images with the CRC of every
// physical record computed in one batch before the reader's state machine
// is replayed.
#include "../../include/wipdb/log.h"

#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "../../include/wipdb/crc32c.h"
#include "span_crc.h"
#include "sst_format.h"

namespace wipdb {
namespace log {

namespace {

// kv/src/db/log_format.h
enum : unsigned {
  kZeroType = 0, kFullType = 1, kFirstType = 2, kMiddleType = 3, kLastType = 4,
  kRecyclableFullType = 5, kRecyclableFirstType = 6, kRecyclableMiddleType = 7,
  kRecyclableLastType = 8,
  kMaxRecordType = kRecyclableLastType,
  kEof = kMaxRecordType + 1,        // the reader's internal codes
  kBadRecord = kMaxRecordType + 2,  // (log_reader.h)
};

struct Span {
  uint64_t hdr;   // absolute header offset
  uint32_t crc;   // crc32c of header[6, 7 + length)
};

// Every physical record the reader could visit, block by block: it reads a
// block, walks headers while they fit, and after a failure moves on to the
// next block -- so its path through a block is a prefix of this walk.
// Each header's position depends on the previous one's length, so the walk
// is a chain of dependent loads: it prefetches the image 2 KiB ahead to keep
// that chain out of DRAM latency.  visit(header, span length).
template <class Visit>
void Walk(const char* img, size_t n, size_t from, size_t to, Visit&& visit) {
  for (size_t b = from; b < to; b += kBlockSize) {
    const size_t end = std::min(n, b + kBlockSize);
    size_t p = b, pf = b;
    while (end - p >= kHeaderSize) {
      for (; pf < p + 2048 && pf < end; pf += 64) __builtin_prefetch(img + pf);
      const uint32_t length = uint32_t(uint8_t(img[p + 4])) | (uint32_t(uint8_t(img[p + 5])) << 8);
      const unsigned type = static_cast<unsigned>(static_cast<signed char>(img[p + 6]));
      if (kHeaderSize + length > end - p) break;
      if (type == kZeroType && length == 0) break;
      visit(p, length + 1);
      p += kHeaderSize + length;
    }
  }
}

// kv::log::Reader (checksum, initial offset 0) over one image.  The record
// CRCs come precomputed (spans, in Walk order: one batch for every log), or
// -- host schedules, where a second pass over a large image would run from
// DRAM -- per record as the reader reaches it (window 0, the reference's
// schedule) or in batches of `window` blocks just ahead of it.
class Replay {
 public:
  Replay(const char* img, size_t n, const std::vector<Span>* spans)
      : img_(img), n_(n), spans_(spans) {}
  Replay(const char* img, size_t n, size_t window) : img_(img), n_(n), window_(window) {
    spans_ = &own_;
    direct_ = window == 0;
  }

  // emit(offset, data, size) per record; a record of one fragment is handed
  // over in place, a fragmented one from the scratch buffer
  template <class Emit>
  void Run(Emit&& emit, std::vector<Drop>* drops) {
    drops_ = drops;
    std::string scratch;
    uint64_t last_record_offset = 0;
    for (;;) {
      scratch.clear();
      bool in_frag = false, whole = false;
      uint64_t prospective = 0;
      for (;;) {
        const unsigned type = ReadPhysical();
        const uint64_t phys = end_ - size() - kHeaderSize - frag_len_;
        bool done = false, got = false;
        switch (type) {
          case kFullType:
            if (in_frag && !scratch.empty()) Report(scratch.size(), "partial record without end(1)");
            prospective = phys;
            last_record_offset = prospective;
            done = got = whole = true;
            break;
          case kFirstType:
            if (in_frag && !scratch.empty()) Report(scratch.size(), "partial record without end(2)");
            prospective = phys;
            scratch.assign(img_ + frag_, frag_len_);
            in_frag = true;
            break;
          case kMiddleType:
            if (!in_frag) Report(frag_len_, "missing start of fragmented record(1)");
            else scratch.append(img_ + frag_, frag_len_);
            break;
          case kLastType:
            if (!in_frag) {
              Report(frag_len_, "missing start of fragmented record(2)");
            } else {
              scratch.append(img_ + frag_, frag_len_);
              last_record_offset = prospective;
              done = got = true;
            }
            break;
          case kEof:
            if (in_frag) scratch.clear();
            done = true;
            break;
          case kBadRecord:
            if (in_frag) {
              Report(scratch.size(), "error in middle of record");
              in_frag = false;
              scratch.clear();
            }
            break;
          default: {
            char buf[40];
            snprintf(buf, sizeof(buf), "unknown record type %u", type);
            Report(frag_len_ + (in_frag ? scratch.size() : 0), buf);
            in_frag = false;
            scratch.clear();
            break;
          }
        }
        if (done) {
          if (!got) return;
          if (whole) emit(last_record_offset, img_ + frag_, frag_len_);
          else emit(last_record_offset, scratch.data(), scratch.size());
          break;
        }
      }
    }
  }

 private:
  size_t size() const { return buf_end_ - buf_; }

  void Report(uint64_t bytes, const char* reason) {
    drops_->push_back({bytes, std::string("Corruption: ") + reason});
  }

  // Reader::ReadPhysicalRecord; the fragment is (frag_, frag_len_) and keeps
  // its previous value on kEof / kBadRecord, as the reference's Slice does.
  unsigned ReadPhysical() {
    for (;;) {
      if (size() < kHeaderSize) {
        if (!eof_) {
          buf_ = end_;
          buf_end_ = std::min<uint64_t>(n_, end_ + kBlockSize);
          end_ = buf_end_;
          if (size() < kBlockSize) eof_ = true;
          continue;
        }
        buf_ = buf_end_;
        return kEof;
      }
      const char* h = img_ + buf_;
      const uint32_t length = uint32_t(uint8_t(h[4])) | (uint32_t(uint8_t(h[5])) << 8);
      const unsigned type = static_cast<unsigned>(static_cast<signed char>(h[6]));
      if (kHeaderSize + length > size()) {
        const size_t drop = size();
        buf_ = buf_end_;
        if (!eof_) {
          Report(drop, "bad record length");
          return kBadRecord;
        }
        return kEof;
      }
      if (type == kZeroType && length == 0) {
        buf_ = buf_end_;
        return kBadRecord;
      }
      const uint32_t expected = kv::crc32c::Unmask(sst::DecodeFixed32(h));
      uint32_t actual;
      if (direct_) {
        actual = kv::crc32c::Value(h + 6, 1 + length);
      } else {
        if (window_ != 0 && buf_ >= win_end_) Refill();
        const std::vector<Span>& sp = *spans_;
        while (k_ < sp.size() && sp[k_].hdr < buf_) ++k_;
        // the reader's path through a block is a prefix of Walk's, so the
        // span is there; computing it here is only a guard
        actual = (k_ < sp.size() && sp[k_].hdr == buf_) ? sp[k_].crc
                                                        : kv::crc32c::Value(h + 6, 1 + length);
      }
      if (actual != expected) {
        const size_t drop = size();
        buf_ = buf_end_;
        Report(drop, "checksum mismatch");
        return kBadRecord;
      }
      frag_ = buf_ + kHeaderSize;
      frag_len_ = length;
      buf_ += kHeaderSize + length;
      return type;
    }
  }

  // the spans of the `window_` blocks from the one holding buf_ (host CRCs)
  void Refill() {
    const size_t from = buf_ / kBlockSize * kBlockSize;
    const size_t to = std::min<size_t>(n_, from + window_ * kBlockSize);
    own_.clear();
    Walk(img_, n_, from, to, [this](uint64_t h, uint32_t l) {
      own_.push_back({h, kv::crc32c::Value(img_ + h + 6, l)});
    });
    k_ = 0;
    win_end_ = to;
  }

  const char* img_;
  size_t n_;
  const std::vector<Span>* spans_ = nullptr;
  std::vector<Span> own_;
  size_t window_ = 0, win_end_ = 0;
  bool direct_ = false;
  size_t k_ = 0;
  uint64_t buf_ = 0, buf_end_ = 0;  // the unread part of the current block
  uint64_t end_ = 0;                // end_of_buffer_offset_
  bool eof_ = false;
  uint64_t frag_ = 0;
  size_t frag_len_ = 0;
  std::vector<Drop>* drops_ = nullptr;
};

}  // namespace

namespace {

// AddRecord's layout of the records (log_writer.cc:35-106): returns the image
// size; with dst, writes the image there (CRC fields zero) and records every
// header's position and CRC span length (type [+ log number] + payload).
size_t Layout(const std::vector<std::string_view>& records, bool recycle, uint64_t log_number,
              char* dst, std::vector<uint64_t>* at, std::vector<uint32_t>* span) {
  const size_t hsize = recycle ? kRecyclableHeaderSize : kHeaderSize;
  size_t pos = 0, block_offset = 0;
  for (std::string_view rec : records) {
    const char* ptr = rec.data();
    size_t left = rec.size();
    bool begin = true;
    do {
      const size_t leftover = kBlockSize - block_offset;
      if (leftover < hsize) {
        if (dst) memset(dst + pos, 0, leftover);
        pos += leftover;
        block_offset = 0;
      }
      const size_t avail = kBlockSize - block_offset - hsize;
      const size_t frag = left < avail ? left : avail;
      const bool end = left == frag;
      if (dst) {
        unsigned t = begin && end ? kFullType : (begin ? kFirstType : (end ? kLastType : kMiddleType));
        if (recycle) t += kRecyclableFullType - kFullType;
        char h[kRecyclableHeaderSize] = {0, 0, 0, 0, char(frag & 0xff), char(frag >> 8), char(t)};
        if (recycle) sst::EncodeFixed32(h + 7, static_cast<uint32_t>(log_number));
        at->push_back(pos);
        span->push_back(static_cast<uint32_t>(hsize - 6 + frag));
        memcpy(dst + pos, h, hsize);
        memcpy(dst + pos + hsize, ptr, frag);
      }
      pos += hsize + frag;
      block_offset += hsize + frag;
      ptr += frag;
      left -= frag;
      begin = false;
    } while (left > 0);
  }
  return pos;
}

// The image laid out at dst (Layout's size), every header CRC in one batch.
Status LayoutAndCrc(const std::vector<std::string_view>& records, bool recycle,
                    uint64_t log_number, table::CrcMode mode, int device, char* dst) {
  std::vector<uint64_t> at;
  std::vector<uint32_t> span;
  at.reserve(records.size() + 16);
  span.reserve(records.size() + 16);
  Layout(records, recycle, log_number, dst, &at, &span);
  std::vector<const char*> p(at.size());
  for (size_t i = 0; i < at.size(); ++i) p[i] = dst + at[i] + 6;
  std::vector<uint32_t> crc(at.size());
  Status s = spancrc::Compute(p.data(), span.data(), p.size(), true, mode, device, crc.data());
  if (!s.ok()) return s;
  for (size_t i = 0; i < at.size(); ++i) sst::EncodeFixed32(dst + at[i], crc[i]);
  return Status::OK();
}

}  // namespace

Status WriteLog(const std::vector<std::string_view>& records, bool recycle, uint64_t log_number,
                table::CrcMode mode, int device, std::string* out) {
  const size_t base = out->size();
  out->resize(base + Layout(records, recycle, log_number, nullptr, nullptr, nullptr));
  Status s = LayoutAndCrc(records, recycle, log_number, mode, device, &(*out)[base]);
  if (!s.ok()) out->resize(base);
  return s;
}

Status WriteLogTo(const std::vector<std::string_view>& records, bool recycle, uint64_t log_number,
                  table::CrcMode mode, int device, char* out, size_t cap, size_t* size) {
  *size = Layout(records, recycle, log_number, nullptr, nullptr, nullptr);
  if (*size > cap) return Status::InvalidArgument("log image larger than the output buffer");
  return LayoutAndCrc(records, recycle, log_number, mode, device, out);
}

Status ReadLogsEach(const char* const* images, const size_t* sizes, size_t nlogs,
                    table::CrcMode mode, int device, RecordFn fn, void* ctx,
                    std::vector<std::vector<Drop>>* drops) {
  drops->assign(nlogs, {});
  if (mode == table::CrcMode::kInline || mode == table::CrcMode::kBatchCpu) {
    // host CRCs: per record, or 64 blocks (2 MiB) at a time, cache-resident
    const size_t window = mode == table::CrcMode::kInline ? 0 : 64;
    for (size_t i = 0; i < nlogs; ++i)
      Replay(images[i], sizes[i], window)
          .Run([&](uint64_t off, const char* d, size_t n) { fn(ctx, i, off, d, n); }, &(*drops)[i]);
    return Status::OK();
  }
  std::vector<std::vector<uint64_t>> hdr(nlogs);
  std::vector<const char*> p;
  std::vector<uint32_t> len;
  for (size_t i = 0; i < nlogs; ++i) {
    Walk(images[i], sizes[i], 0, sizes[i], [&](uint64_t h, uint32_t l) {
      hdr[i].push_back(h);
      p.push_back(images[i] + h + 6);
      len.push_back(l);
    });
  }
  std::vector<uint32_t> crc(p.size());
  Status s = spancrc::Compute(p.data(), len.data(), p.size(), false, mode, device, crc.data());
  if (!s.ok()) return s;
  size_t k = 0;
  for (size_t i = 0; i < nlogs; ++i) {
    std::vector<Span> spans(hdr[i].size());
    for (size_t j = 0; j < spans.size(); ++j) spans[j] = {hdr[i][j], crc[k++]};
    Replay(images[i], sizes[i], &spans)
        .Run([&](uint64_t off, const char* d, size_t n) { fn(ctx, i, off, d, n); }, &(*drops)[i]);
  }
  return Status::OK();
}

Status ReadLogs(const char* const* images, const size_t* sizes, size_t nlogs,
                table::CrcMode mode, int device, std::vector<std::vector<Record>>* records,
                std::vector<std::vector<Drop>>* drops) {
  records->assign(nlogs, {});
  return ReadLogsEach(
      images, sizes, nlogs, mode, device,
      [](void* c, size_t log, uint64_t off, const char* d, size_t n) {
        (*static_cast<std::vector<std::vector<Record>>*>(c))[log].push_back({off, std::string(d, n)});
      },
      records, drops);
}

Status ReadLog(const char* image, size_t n, table::CrcMode mode, int device,
               std::vector<Record>* records, std::vector<Drop>* drops) {
  std::vector<std::vector<Record>> r;
  std::vector<std::vector<Drop>> d;
  Status s = ReadLogs(&image, &n, 1, mode, device, &r, &d);
  if (!s.ok()) return s;
  *records = std::move(r[0]);
  *drops = std::move(d[0]);
  return Status::OK();
}

}  // namespace log
}  // namespace wipdb
