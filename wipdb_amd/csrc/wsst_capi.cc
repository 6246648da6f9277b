// wsst_capi.cc -- the C-ABI of include/wipdb_sst.h over the C++ table layer.
#include "../../include/wipdb_sst.h"

#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/wipdb/log.h"
#include "../../include/wipdb/table.h"

namespace {

using wipdb::Status;
using wipdb::table::CrcMode;

int Code(const Status& s) {
  if (s.ok()) return WSST_OK;
  if (s.code() == Status::kIOError && s.message().rfind("hcrc", 0) == 0) return WSST_ERR_DEVICE;
  if (s.IsCorruption())
    return s.message().find("checksum mismatch") != std::string::npos ? WSST_CRC_MISMATCH
                                                                      : WSST_CORRUPTION;
  return WSST_OTHER;
}

bool ModeOf(int m, CrcMode* out) {
  if (m < WSST_CRC_INLINE || m > WSST_CRC_BATCH_AUTO) return false;
  *out = static_cast<CrcMode>(m);
  return true;
}

}  // namespace

extern "C" {

int wsst_build_tables(size_t ntables, const size_t* entries, const char* keys,
                      const uint32_t* key_lens, const char* vals, const uint32_t* val_lens,
                      int block_size, int restart_interval, int bloom_bits,
                      size_t max_buffer_size, int crc_mode, int device, char* out,
                      size_t cap, uint64_t* out_offsets, uint64_t* sizes,
                      uint64_t* batched_blocks) {
  return wsst_build_tables_ex(ntables, entries, keys, key_lens, vals, val_lens, block_size,
                              restart_interval, bloom_bits, max_buffer_size, crc_mode, device,
                              WSST_KEYS_BYTEWISE, out, cap, out_offsets, sizes, batched_blocks);
}

int wsst_build_tables_ex(size_t ntables, const size_t* entries, const char* keys,
                         const uint32_t* key_lens, const char* vals, const uint32_t* val_lens,
                         int block_size, int restart_interval, int bloom_bits,
                         size_t max_buffer_size, int crc_mode, int device, int key_format,
                         char* out, size_t cap, uint64_t* out_offsets, uint64_t* sizes,
                         uint64_t* batched_blocks) {
  CrcMode mode;
  if (!ModeOf(crc_mode, &mode) || !entries || !out || !out_offsets || !sizes ||
      block_size <= 0 || restart_interval <= 0 || max_buffer_size == 0 ||
      (key_format != WSST_KEYS_BYTEWISE && key_format != WSST_KEYS_INTERNAL))
    return WSST_ERR_INVALID;
  wipdb::table::TableOptions opt;
  opt.block_size = static_cast<size_t>(block_size);
  opt.block_restart_interval = restart_interval;
  opt.bloom_bits_per_key = bloom_bits;
  opt.max_buffer_size = max_buffer_size;
  opt.crc_mode = mode;
  opt.device = device;
  if (key_format == WSST_KEYS_INTERNAL) opt = wipdb::table::InternalKeyTableOptions(opt);
  std::vector<std::unique_ptr<wipdb::table::StringSink>> sinks(ntables);
  std::vector<std::unique_ptr<wipdb::table::TableBuilder>> tbs(ntables);
  std::vector<wipdb::table::TableBuilder*> raw(ntables);
  size_t ko = 0, vo = 0, e = 0;
  for (size_t t = 0; t < ntables; ++t) {
    sinks[t].reset(new wipdb::table::StringSink);
    tbs[t].reset(new wipdb::table::TableBuilder(opt, sinks[t].get()));
    raw[t] = tbs[t].get();
    for (size_t i = 0; i < entries[t]; ++i, ++e) {
      tbs[t]->Add(std::string_view(keys + ko, key_lens[e]),
                  std::string_view(vals + vo, val_lens[e]));
      ko += key_lens[e];
      vo += val_lens[e];
    }
  }
  const Status s = wipdb::table::FinishTables(raw.data(), ntables);
  uint64_t total = 0, batched = 0;
  for (size_t t = 0; t < ntables; ++t) {
    out_offsets[t] = total;
    sizes[t] = sinks[t]->contents.size();
    if (total + sizes[t] > cap) return WSST_ERR_TOO_SMALL;
    memcpy(out + total, sinks[t]->contents.data(), sizes[t]);
    total += sizes[t];
    batched += tbs[t]->BatchedBlocks();
  }
  if (batched_blocks) *batched_blocks = batched;
  return Code(s);
}

int wsst_merge_tables(const char* const* images, const size_t* sizes, size_t n, int key_format,
                      int verify, size_t prefetch_blocks, int crc_mode, int device,
                      char* key_out, size_t key_cap, uint32_t* key_lens, char* val_out,
                      size_t val_cap, uint32_t* val_lens, size_t max_entries,
                      uint64_t* nentries, uint64_t* crc_batches) {
  CrcMode mode;
  if (!ModeOf(crc_mode, &mode) || (n && (!images || !sizes)) || !nentries ||
      (key_format != WSST_KEYS_BYTEWISE && key_format != WSST_KEYS_INTERNAL))
    return WSST_ERR_INVALID;
  wipdb::table::CompactionInput::Options o;
  o.comparator = key_format == WSST_KEYS_INTERNAL ? wipdb::table::InternalBytewiseComparator()
                                                  : wipdb::table::BytewiseComparator();
  o.verify_checksums = verify != 0;
  o.prefetch_blocks = prefetch_blocks;
  o.crc_mode = mode;
  o.device = device;
  wipdb::table::CompactionInput it(images, sizes, n, o);
  size_t k = 0, ko = 0, vo = 0;
  for (it.SeekToFirst(); it.Valid(); it.Next(), ++k) {
    const std::string_view key = it.key(), val = it.value();
    if (k >= max_entries || ko + key.size() > key_cap || vo + val.size() > val_cap)
      return WSST_ERR_TOO_SMALL;
    memcpy(key_out + ko, key.data(), key.size());
    memcpy(val_out + vo, val.data(), val.size());
    key_lens[k] = static_cast<uint32_t>(key.size());
    val_lens[k] = static_cast<uint32_t>(val.size());
    ko += key.size();
    vo += val.size();
  }
  *nentries = k;
  if (crc_batches) *crc_batches = it.CrcBatches();
  return Code(it.status());
}

int wsst_read_block(const char* image, size_t n, uint64_t offset, uint64_t size) {
  if (!image) return WSST_ERR_INVALID;
  return Code(wipdb::table::ReadBlock(image, n, offset, size, true, nullptr));
}

int wsst_verify_tables(const char* const* images, const size_t* sizes, size_t n,
                       int bloom_bits, int crc_mode, int device, int* codes,
                       uint64_t* blocks_checked, uint64_t* bad_blocks) {
  CrcMode mode;
  if (!ModeOf(crc_mode, &mode) || (n && (!images || !sizes))) return WSST_ERR_INVALID;
  uint64_t checked = 0, bad = 0;
  int first = WSST_OK;
  if (!blocks_checked && !bad_blocks) {
    std::vector<Status> st;
    const Status s = wipdb::table::VerifyTables(images, sizes, n, bloom_bits, mode, device, &st);
    if (s.code() == Status::kIOError && st.empty()) return Code(s);
    for (size_t i = 0; i < st.size(); ++i) {
      if (codes) codes[i] = Code(st[i]);
      if (first == WSST_OK) first = Code(st[i]);
    }
    return first;
  }
  // per-block accounting: one table at a time (still one batch per stage)
  for (size_t i = 0; i < n; ++i) {
    std::vector<wipdb::table::BlockCheck> b;
    const Status s =
        wipdb::table::VerifyTable(images[i], sizes[i], bloom_bits, mode, device, &b);
    const int c = Code(s);
    if (c == WSST_ERR_DEVICE) return c;
    if (codes) codes[i] = c;
    if (first == WSST_OK) first = c;
    checked += b.size();
    for (const auto& x : b) bad += x.ok ? 0 : 1;
  }
  if (blocks_checked) *blocks_checked = checked;
  if (bad_blocks) *bad_blocks = bad;
  return first;
}

int wsst_log_write(const char* records, const uint32_t* lens, size_t n, int recycle,
                   uint64_t log_number, int crc_mode, int device, char* out, size_t cap,
                   uint64_t* out_size) {
  CrcMode mode;
  if (!ModeOf(crc_mode, &mode) || !out || !out_size || (n && (!records || !lens)))
    return WSST_ERR_INVALID;
  std::vector<std::string_view> recs(n);
  size_t o = 0;
  for (size_t i = 0; i < n; ++i) {
    recs[i] = std::string_view(records + o, lens[i]);
    o += lens[i];
  }
  size_t size = 0;
  const Status s =
      wipdb::log::WriteLogTo(recs, recycle != 0, log_number, mode, device, out, cap, &size);
  *out_size = size;
  if (size > cap) return WSST_ERR_TOO_SMALL;
  return s.ok() ? WSST_OK : Code(s);
}

int wsst_log_read(const char* const* images, const size_t* sizes, size_t nlogs, int crc_mode,
                  int device, char* rec_out, size_t rec_cap, uint32_t* rec_lens,
                  uint64_t* rec_offsets, size_t max_recs, uint64_t* nrecs,
                  uint64_t* drop_bytes, char* drop_reasons, size_t max_drops,
                  uint64_t* ndrops) {
  CrcMode mode;
  if (!ModeOf(crc_mode, &mode) || (nlogs && (!images || !sizes || !nrecs || !ndrops)))
    return WSST_ERR_INVALID;
  struct Out {
    char* rec_out;
    size_t rec_cap, max_recs, r = 0, used = 0;
    uint32_t* rec_lens;
    uint64_t* rec_offsets;
    uint64_t* nrecs;
    bool full = false;
  } o{rec_out, rec_cap, max_recs, 0, 0, rec_lens, rec_offsets, nrecs};
  for (size_t i = 0; i < nlogs; ++i) nrecs[i] = 0;
  std::vector<std::vector<wipdb::log::Drop>> drops;
  const Status s = wipdb::log::ReadLogsEach(
      images, sizes, nlogs, mode, device,
      [](void* c, size_t log, uint64_t off, const char* d, size_t n) {
        Out& o = *static_cast<Out*>(c);
        ++o.nrecs[log];
        if (o.full || o.r >= o.max_recs || o.used + n > o.rec_cap || !o.rec_out || !o.rec_lens ||
            !o.rec_offsets) {
          o.full = true;
          return;
        }
        memcpy(o.rec_out + o.used, d, n);
        o.rec_lens[o.r] = static_cast<uint32_t>(n);
        o.rec_offsets[o.r] = off;
        o.used += n;
        ++o.r;
      },
      &o, &drops);
  if (!s.ok()) return Code(s);
  int rc = o.full ? WSST_ERR_TOO_SMALL : WSST_OK;
  size_t d = 0;
  for (size_t i = 0; i < nlogs; ++i) {
    ndrops[i] = drops[i].size();
    for (const auto& x : drops[i]) {
      if (d >= max_drops || !drop_bytes || !drop_reasons) {
        rc = WSST_ERR_TOO_SMALL;
        break;
      }
      drop_bytes[d] = x.bytes;
      strncpy(drop_reasons + 64 * d, x.reason.c_str(), 63);
      drop_reasons[64 * d + 63] = 0;
      ++d;
    }
  }
  return rc;
}

}  // extern "C"
