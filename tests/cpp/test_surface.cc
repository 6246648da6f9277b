// tests/cpp/test_surface.cc -- the drop-in C++ surface, compiled the way
// WipDB's callers would compile against it (include/wipdb/crc32c.h) and
// linked against libhip_crc32c_batch.so.  Restates the reference tests
// rocksdb/util/crc32c_test.cc:66-138 and leveldb/util/crc32c_test.cc:13-66
// for both namespaces, then exercises ExtendBatch.
//
// Usage: test_surface [mode]   (exit 0 = pass; modes in main)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hip_crc32c_batch.h"
#include "util/crc32c.h"  // include/wipdb_compat: the path kv/leveldb/rocksdb sources use

static int g_fail = 0;
#define CHECK_EQ(a, b)                                                       \
  do {                                                                       \
    unsigned long long a_ = (unsigned long long)(a), b_ = (unsigned long long)(b); \
    if (a_ != b_) {                                                          \
      fprintf(stderr, "%s:%d: %s = %llx != %s = %llx\n", __FILE__, __LINE__, \
              #a, a_, #b, b_);                                               \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

template <uint32_t (*ExtendFn)(uint32_t, const char*, size_t),
          uint32_t (*MaskFn)(uint32_t), uint32_t (*UnmaskFn)(uint32_t)>
static void StandardResults() {
  char buf[32];
  memset(buf, 0, sizeof(buf));
  CHECK_EQ(ExtendFn(0, buf, sizeof(buf)), 0x8a9136aaU);
  memset(buf, 0xff, sizeof(buf));
  CHECK_EQ(ExtendFn(0, buf, sizeof(buf)), 0x62a8ab43U);
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(i);
  CHECK_EQ(ExtendFn(0, buf, sizeof(buf)), 0x46dd794eU);
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(31 - i);
  CHECK_EQ(ExtendFn(0, buf, sizeof(buf)), 0x113fdb5cU);
  unsigned char data[48] = {0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                            0x14, 0, 0, 0, 0, 0, 0x04, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18,
                            0x28, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0, 0, 0, 0, 0, 0};
  CHECK_EQ(ExtendFn(0, reinterpret_cast<char*>(data), sizeof(data)), 0xd9963a56U);
  CHECK_EQ(ExtendFn(0, "TestCRCBuffer", 13), 0xdcbc59faU);
  // Values / Extend / Mask
  if (ExtendFn(0, "a", 1) == ExtendFn(0, "foo", 3)) ++g_fail;
  CHECK_EQ(ExtendFn(0, "hello world", 11), ExtendFn(ExtendFn(0, "hello ", 6), "world", 5));
  uint32_t crc = ExtendFn(0, "foo", 3);
  if (crc == MaskFn(crc) || crc == MaskFn(MaskFn(crc))) ++g_fail;
  CHECK_EQ(UnmaskFn(MaskFn(crc)), crc);
  CHECK_EQ(UnmaskFn(UnmaskFn(MaskFn(MaskFn(crc)))), crc);
}

static uint32_t KvExtend(uint32_t c, const char* d, size_t n) { return kv::crc32c::Extend(c, d, n); }
static uint32_t KvMask(uint32_t c) { return kv::crc32c::Mask(c); }
static uint32_t KvUnmask(uint32_t c) { return kv::crc32c::Unmask(c); }
static uint32_t LdbExtend(uint32_t c, const char* d, size_t n) { return leveldb::crc32c::Extend(c, d, n); }
static uint32_t LdbMask(uint32_t c) { return leveldb::crc32c::Mask(c); }
static uint32_t LdbUnmask(uint32_t c) { return leveldb::crc32c::Unmask(c); }
static uint32_t RdbExtend(uint32_t c, const char* d, size_t n) { return rocksdb::crc32c::Extend(c, d, n); }
static uint32_t RdbMask(uint32_t c) { return rocksdb::crc32c::Mask(c); }
static uint32_t RdbUnmask(uint32_t c) { return rocksdb::crc32c::Unmask(c); }

int main(int argc, char** argv) {
  // argv[1]: 0 = no device, 1 = a device, 2 = a device + WIPDB_CRC_MODE=cpu,
  // 3 = a device + WIPDB_CRC_DEVICES=0,0, 4 = a device, linked against the
  // test build with WIPDB_HCRC_FORCE_FAULT=1 (every kernel reports a fault)
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const bool expect_gpu = mode != 0;
  StandardResults<KvExtend, KvMask, KvUnmask>();
  StandardResults<LdbExtend, LdbMask, LdbUnmask>();
  StandardResults<RdbExtend, RdbMask, RdbUnmask>();
  CHECK_EQ(rocksdb::crc32c::IsFastCrc32Supported() == kv::crc32c::IsFastCrc32Supported(), 1);
  CHECK_EQ(kv::crc32c::Value("hello", 5), leveldb::crc32c::Value("hello", 5));
  CHECK_EQ(kv::crc32c::kMaskDelta, 0xa282ead8u);

  // A WriteRawBlock-shaped batch: ~4 KiB blocks + type byte, SST packing.
  std::vector<char> file(1 << 20);
  uint64_t x = 88172645463325252ull;
  for (auto& c : file) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    c = static_cast<char>(x);
  }
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  uint64_t cur = 0;
  while (cur + 4300 < file.size()) {
    uint32_t n = 4097 + static_cast<uint32_t>(cur % 129);
    off.push_back(cur);
    len.push_back(n);
    cur += n + 4;
  }
  std::vector<uint32_t> want(off.size()), got(off.size());
  for (size_t i = 0; i < off.size(); ++i)
    want[i] = kv::crc32c::Mask(kv::crc32c::Value(file.data() + off[i], len[i]));
  using wipdb::crc32c::BatchPolicy;
  CHECK_EQ(wipdb::crc32c::ExtendBatch(file.data(), off.data(), len.data(), nullptr,
                                      got.data(), off.size(), true, BatchPolicy::kCpuOnly),
           0);
  for (size_t i = 0; i < off.size(); ++i) CHECK_EQ(got[i], want[i]);
  std::fill(got.begin(), got.end(), 0u);
  CHECK_EQ(wipdb::crc32c::ExtendBatch(file.data(), off.data(), len.data(), nullptr,
                                      got.data(), off.size(), true, BatchPolicy::kAuto),
           0);
  for (size_t i = 0; i < off.size(); ++i) CHECK_EQ(got[i], want[i]);
  auto st = wipdb::crc32c::GetBatchStats();
  if (mode == 4) {
    // the kernel reported a fault: kAuto computed the batch on the host
    // (outputs right, checked above), kGpuOnly returns HCRC_ERR_KERNEL
    CHECK_EQ(st.cpu_batches, 2);
    CHECK_EQ(st.gpu_batches, 0);
    CHECK_EQ(st.last_error, HCRC_ERR_KERNEL);
    CHECK_EQ(wipdb::crc32c::ExtendBatch(file.data(), off.data(), len.data(), nullptr,
                                        got.data(), off.size(), true, BatchPolicy::kGpuOnly),
             HCRC_ERR_KERNEL);
  } else if (mode == 2) {
    // GPU present, WIPDB_CRC_MODE=cpu: kAuto stays on the host, kGpuOnly
    // still reaches the device
    CHECK_EQ(st.cpu_batches, 2);
    CHECK_EQ(st.gpu_batches, 0);
    std::fill(got.begin(), got.end(), 0u);
    CHECK_EQ(wipdb::crc32c::ExtendBatch(file.data(), off.data(), len.data(), nullptr,
                                        got.data(), off.size(), true, BatchPolicy::kGpuOnly),
             0);
    for (size_t i = 0; i < off.size(); ++i) CHECK_EQ(got[i], want[i]);
    CHECK_EQ(wipdb::crc32c::GetBatchStats().gpu_batches, 1);
  } else if (mode == 3) {
    // GPU present, WIPDB_CRC_DEVICES lists device 0 twice: a batch of
    // >= 8192 spans is sharded over the list (hcrc_batch_multi)
    CHECK_EQ(st.gpu_batches, 1);
    std::vector<uint64_t> o2;
    std::vector<uint32_t> l2, w2, g2;
    for (int r = 0; r < 40; ++r)
      for (size_t i = 0; i < off.size(); ++i) {
        o2.push_back(off[i]);
        l2.push_back(len[i]);
        w2.push_back(want[i]);
      }
    g2.assign(o2.size(), 0u);
    CHECK_EQ(wipdb::crc32c::ExtendBatch(file.data(), o2.data(), l2.data(), nullptr, g2.data(),
                                        o2.size(), true, BatchPolicy::kGpuOnly),
             0);
    for (size_t i = 0; i < o2.size(); ++i) CHECK_EQ(g2[i], w2[i]);
  } else if (expect_gpu) {
    CHECK_EQ(st.gpu_batches, 1);
    std::fill(got.begin(), got.end(), 0u);
    CHECK_EQ(wipdb::crc32c::ExtendBatch(file.data(), off.data(), len.data(), nullptr,
                                        got.data(), off.size(), true, BatchPolicy::kGpuOnly),
             0);
    for (size_t i = 0; i < off.size(); ++i) CHECK_EQ(got[i], want[i]);
  } else {
    // no device: kAuto stays infallible on the host, kGpuOnly reports it
    CHECK_EQ(st.cpu_batches, 2);
    int rc = wipdb::crc32c::ExtendBatch(file.data(), off.data(), len.data(), nullptr,
                                        got.data(), off.size(), true, BatchPolicy::kGpuOnly);
    if (rc == 0) ++g_fail;
  }
  printf("%s (%zu blocks, gpu=%d)\n", g_fail ? "FAIL" : "PASS", off.size(), (int)expect_gpu);
  return g_fail ? 1 : 0;
}
