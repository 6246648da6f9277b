// sst_format.h -- WipDB's on-disk table format, restated for the batched
// table builder / verifier (table_builder.cc, table_reader.cc).  Internal
// header (host C++ only).
//
// The format is the reference's, byte for byte:
//   block      = entries, restart array (fixed32 each), restart count
//                (kv/src/table/block_builder.cc:36-107); an entry is
//                varint32 shared | non_shared | value_len, key delta, value
//   trailer    = type byte + fixed32 Mask(crc32c(contents || type))
//                (kv/src/table/table_builder.cc:183-202, format.h:84)
//   handle     = varint64 offset, varint64 size (format.cc:15-32)
//   footer     = metaindex handle, index handle, zero pad to 40 bytes,
//                fixed64 magic 0xdb4775248b80fb57 (format.cc:34-62, h:80)
//   filter     = per-2KiB bloom filters, offset array, array offset,
//                base lg 11 (kv/src/table/filter_block.cc:15-98); bloom
//                "leveldb.BuiltinBloomFilter2", k = bits*0.69 in [1, 30]
//                (kv/src/table/bloom.cc:19-62), hash = kv::Hash(.., 0xbc9f1d34)
//                (kv/src/util/hash.cc:16-48, hash.h:17-19)
//   index keys = BytewiseComparator FindShortestSeparator /
//                FindShortSuccessor (kv/src/util/comparator.cc:31-96)
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <string_view>
#include <vector>

namespace wipdb {
namespace sst {

constexpr size_t kBlockTrailerSize = 5;
constexpr uint64_t kTableMagicNumber = 0xdb4775248b80fb57ull;
constexpr size_t kMaxHandleLength = 20;
constexpr size_t kFooterLength = 2 * kMaxHandleLength + 8;
constexpr int kNoCompression = 0;
constexpr int kSnappyCompression = 1;

// ---- little-endian coding (kv/src/util/coding.h) ----
inline void PutFixed32(std::string* d, uint32_t v) {
  char b[4] = {char(v), char(v >> 8), char(v >> 16), char(v >> 24)};
  d->append(b, 4);
}
inline void EncodeFixed32(char* p, uint32_t v) {
  p[0] = char(v); p[1] = char(v >> 8); p[2] = char(v >> 16); p[3] = char(v >> 24);
}
inline uint32_t DecodeFixed32(const char* p) {
  const uint8_t* u = reinterpret_cast<const uint8_t*>(p);
  return uint32_t(u[0]) | (uint32_t(u[1]) << 8) | (uint32_t(u[2]) << 16) |
         (uint32_t(u[3]) << 24);
}
inline void PutVarint64(std::string* d, uint64_t v) {
  while (v >= 0x80) {
    d->push_back(char(v | 0x80));
    v >>= 7;
  }
  d->push_back(char(v));
}
inline void PutVarint32(std::string* d, uint32_t v) { PutVarint64(d, v); }
// Returns the byte after the varint, or nullptr when [p, limit) holds no
// complete one of at most `maxbytes` bytes.
inline const char* GetVarint(const char* p, const char* limit, uint64_t* v, int maxbytes) {
  uint64_t r = 0;
  for (int shift = 0, i = 0; i < maxbytes && p < limit; ++i, shift += 7) {
    const uint64_t b = static_cast<uint8_t>(*p++);
    r |= (b & 0x7f) << shift;
    if (b < 0x80) {
      *v = r;
      return p;
    }
  }
  return nullptr;
}
inline const char* GetVarint32(const char* p, const char* limit, uint32_t* v) {
  uint64_t w = 0;
  p = GetVarint(p, limit, &w, 5);
  if (p) *v = static_cast<uint32_t>(w);
  return p;
}

// ---- block handle / footer (kv/src/table/format.h) ----
struct Handle {
  uint64_t offset = ~uint64_t(0);
  uint64_t size = ~uint64_t(0);
  void EncodeTo(std::string* d) const {
    PutVarint64(d, offset);
    PutVarint64(d, size);
  }
  // Consumes a handle from the front of *in; false = "bad block handle".
  bool DecodeFrom(std::string_view* in) {
    const char* p = in->data();
    const char* lim = p + in->size();
    p = GetVarint(p, lim, &offset, 10);
    if (p) p = GetVarint(p, lim, &size, 10);
    if (!p) return false;
    in->remove_prefix(static_cast<size_t>(p - in->data()));
    return true;
  }
};

inline void EncodeFooter(const Handle& metaindex, const Handle& index, std::string* d) {
  const size_t start = d->size();
  metaindex.EncodeTo(d);
  index.EncodeTo(d);
  d->resize(start + 2 * kMaxHandleLength);
  PutFixed32(d, static_cast<uint32_t>(kTableMagicNumber & 0xffffffffu));
  PutFixed32(d, static_cast<uint32_t>(kTableMagicNumber >> 32));
}

// ---- hash, bloom, comparator ----
inline uint32_t Hash(const char* data, size_t n, uint32_t seed) {
  const uint32_t m = 0xc6a4a793u;
  uint32_t h = seed ^ static_cast<uint32_t>(n * m);
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    h += DecodeFixed32(data + i);
    h *= m;
    h ^= h >> 16;
  }
  const size_t rest = n - i;
  if (rest) {
    const uint8_t* u = reinterpret_cast<const uint8_t*>(data + i);
    if (rest == 3) h += uint32_t(u[2]) << 16;
    if (rest >= 2) h += uint32_t(u[1]) << 8;
    h += u[0];
    h *= m;
    h ^= h >> 24;
  }
  return h;
}

inline uint32_t BloomHash(std::string_view key) { return Hash(key.data(), key.size(), 0xbc9f1d34u); }

struct Bloom {
  size_t bits_per_key;
  size_t k;
  explicit Bloom(int bits) : bits_per_key(static_cast<size_t>(bits)) {
    size_t kk = static_cast<size_t>(bits * 0.69);
    k = kk < 1 ? 1 : (kk > 30 ? 30 : kk);
  }
  static const char* Name() { return "leveldb.BuiltinBloomFilter2"; }
  void CreateFilter(const std::vector<std::string_view>& keys, std::string* dst) const {
    size_t bits = keys.size() * bits_per_key;
    if (bits < 64) bits = 64;
    const size_t bytes = (bits + 7) / 8;
    bits = bytes * 8;
    const size_t at = dst->size();
    dst->resize(at + bytes, 0);
    dst->push_back(static_cast<char>(k));
    char* a = &(*dst)[at];
    for (std::string_view key : keys) {
      uint32_t h = BloomHash(key);
      const uint32_t delta = (h >> 17) | (h << 15);
      for (size_t j = 0; j < k; ++j) {
        const uint32_t pos = static_cast<uint32_t>(h % bits);
        a[pos / 8] |= static_cast<char>(1 << (pos % 8));
        h += delta;
      }
    }
  }
};

// BytewiseComparator::FindShortestSeparator (the variant that skips past a
// +1 overflow to the first non-0xff byte, kv/src/util/comparator.cc:31-80).
inline void ShortestSeparator(std::string* start, std::string_view limit) {
  const size_t min_len = start->size() < limit.size() ? start->size() : limit.size();
  size_t i = 0;
  while (i < min_len && (*start)[i] == limit[i]) ++i;
  if (i >= min_len) return;  // one is a prefix of the other
  const uint8_t sb = static_cast<uint8_t>((*start)[i]);
  const uint8_t lb = static_cast<uint8_t>(limit[i]);
  if (sb >= lb) return;
  if (i < limit.size() - 1 || sb + 1 < lb) {
    (*start)[i] = static_cast<char>(sb + 1);
    start->resize(i + 1);
    return;
  }
  for (++i; i < start->size(); ++i) {
    if (static_cast<uint8_t>((*start)[i]) < 0xff) {
      (*start)[i] = static_cast<char>(static_cast<uint8_t>((*start)[i]) + 1);
      start->resize(i + 1);
      return;
    }
  }
}

inline void ShortSuccessor(std::string* key) {
  for (size_t i = 0; i < key->size(); ++i) {
    const uint8_t b = static_cast<uint8_t>((*key)[i]);
    if (b != 0xff) {
      (*key)[i] = static_cast<char>(b + 1);
      key->resize(i + 1);
      return;
    }
  }
}

// ---- block builder (restart-point prefix compression) ----
class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval) : interval_(restart_interval) { restarts_.push_back(0); }
  void Reset() {
    buf_.clear();
    restarts_.assign(1, 0);
    counter_ = 0;
    last_.clear();
  }
  bool empty() const { return buf_.empty(); }
  size_t SizeEstimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  void Add(std::string_view key, std::string_view value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      const size_t m = last_.size() < key.size() ? last_.size() : key.size();
      while (shared < m && last_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back(static_cast<uint32_t>(buf_.size()));
      counter_ = 0;
    }
    const size_t non_shared = key.size() - shared;
    PutVarint32(&buf_, static_cast<uint32_t>(shared));
    PutVarint32(&buf_, static_cast<uint32_t>(non_shared));
    PutVarint32(&buf_, static_cast<uint32_t>(value.size()));
    buf_.append(key.data() + shared, non_shared);
    buf_.append(value.data(), value.size());
    last_.assign(key.data(), key.size());
    ++counter_;
  }
  // Appends the restart array; the contents stay valid until Reset().
  std::string_view Finish() {
    for (uint32_t r : restarts_) PutFixed32(&buf_, r);
    PutFixed32(&buf_, static_cast<uint32_t>(restarts_.size()));
    return buf_;
  }
  void set_interval(int v) { interval_ = v; }

 private:
  int interval_;
  std::string buf_;
  std::vector<uint32_t> restarts_;
  int counter_ = 0;
  std::string last_;
};

// ---- filter block builder (one bloom filter per 2 KiB of file offset) ----
class FilterBuilder {
 public:
  explicit FilterBuilder(int bits) : bloom_(bits) {}
  void StartBlock(uint64_t block_offset) {
    const uint64_t idx = block_offset >> kBaseLg;
    while (idx > offsets_.size()) Generate();
  }
  void AddKey(std::string_view k) {
    starts_.push_back(keys_.size());
    keys_.append(k.data(), k.size());
  }
  std::string_view Finish() {
    if (!starts_.empty()) Generate();
    const uint32_t array_off = static_cast<uint32_t>(result_.size());
    for (uint32_t o : offsets_) PutFixed32(&result_, o);
    PutFixed32(&result_, array_off);
    result_.push_back(static_cast<char>(kBaseLg));
    return result_;
  }
  const Bloom& bloom() const { return bloom_; }

 private:
  static constexpr int kBaseLg = 11;
  void Generate() {
    offsets_.push_back(static_cast<uint32_t>(result_.size()));
    if (starts_.empty()) return;
    std::vector<std::string_view> ks;
    ks.reserve(starts_.size());
    for (size_t i = 0; i < starts_.size(); ++i) {
      const size_t end = i + 1 < starts_.size() ? starts_[i + 1] : keys_.size();
      ks.emplace_back(keys_.data() + starts_[i], end - starts_[i]);
    }
    bloom_.CreateFilter(ks, &result_);
    keys_.clear();
    starts_.clear();
  }
  Bloom bloom_;
  std::string keys_;
  std::vector<size_t> starts_;
  std::string result_;
  std::vector<uint32_t> offsets_;
};

}  // namespace sst
}  // namespace wipdb
