// include/wipdb/crc32c.h -- the C++ CRC32C surface WipDB's callers compile
// against, unchanged from the reference, plus the batch extension.
//
// Drop-in for:
//   kv/src/util/crc32c.h:15-50      namespace kv::crc32c
//     (IsFastCrc32Supported :19, Extend :24, Value :27-29, kMaskDelta :31,
//      Mask :38-41, Unmask :44-47)
//   leveldb/util/crc32c.h:11-41     namespace leveldb::crc32c
//     (Extend :17, Value :20-22, kMaskDelta :24, Mask :29-32, Unmask :35-38)
//   pebblesdb/src/util/crc32c.h:11-41 the same leveldb::crc32c (one symbol
//     serves both trees)
//   rocksdb/util/crc32c.h:14-41     namespace rocksdb::crc32c
//     (IsFastCrc32Supported :16, Extend :21, Value :23-25, kMaskDelta :27,
//      Mask :32-35, Unmask :38-41) -- the comparison stores of SURVEY 8f-4
//
// Extend/Value keep their reference meaning and stay infallible (host CPU
// path, crc32c_cpu.cc).  ExtendBatch is new: it hands a whole batch of block
// spans to the MI355X engine (include/hip_crc32c_batch.h) and, under the
// kAuto policy only, computes on the CPU when no device is usable -- the
// reference's callers never see an error, as with Extend.  Under kGpuOnly
// the HCRC_ERR_* code is returned instead.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace wipdb {
namespace crc32c {

enum class BatchPolicy { kAuto = 0, kGpuOnly = 1, kCpuOnly = 2 };

// The device argument's default: the devices listed in WIPDB_CRC_DEVICES
// (below), else device 0.
constexpr int kDeviceFromEnv = -1;

struct BatchStats {
  uint64_t gpu_batches = 0;
  uint64_t cpu_batches = 0;  // kAuto batches that ran on the host
  int last_error = 0;        // last HCRC_ERR_* seen under kAuto
};

// out[i] = Extend(inits ? inits[i] : 0, base + offsets[i], lengths[i]),
// Mask()-ed when mask is true.  Host memory.  Returns 0 or an HCRC_ERR_*
// code (only possible under kGpuOnly).
//
// Runtime selection without recompiling the caller (read once per process):
//   WIPDB_CRC_MODE=auto|gpu|cpu   what kAuto means: the size threshold
//                                  below (default), every batch on the GPU
//                                  (still falling back to the host if no
//                                  device works), or every batch on the host
//   WIPDB_CRC_MIN_GPU_BATCH=N     kAuto's threshold (default 64 spans)
//   WIPDB_CRC_DEVICES=0,1,...     devices for device == kDeviceFromEnv:
//                                  calls are spread round robin over them, and
//                                  a batch of >= 8192 spans is sharded over
//                                  all of them by bytes (hcrc_batch_multi)
int ExtendBatch(const char* base, const uint64_t* offsets,
                const uint32_t* lengths, const uint32_t* inits, uint32_t* out,
                size_t count, bool mask,
                BatchPolicy policy = BatchPolicy::kAuto,
                int device = kDeviceFromEnv);

// Below this many spans kAuto stays on the CPU (a launch costs more);
// overrides WIPDB_CRC_MIN_GPU_BATCH.
void SetMinGpuBatch(size_t spans);
BatchStats GetBatchStats();

}  // namespace crc32c
}  // namespace wipdb

namespace kv {
namespace crc32c {

extern std::string IsFastCrc32Supported();
extern uint32_t Extend(uint32_t init_crc, const char* data, size_t n);
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8ul;
inline uint32_t Mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + kMaskDelta;
}
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace crc32c
}  // namespace kv

namespace leveldb {
namespace crc32c {

uint32_t Extend(uint32_t init_crc, const char* data, size_t n);
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8ul;
inline uint32_t Mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + kMaskDelta;
}
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace crc32c
}  // namespace leveldb

namespace rocksdb {
namespace crc32c {

extern std::string IsFastCrc32Supported();
extern uint32_t Extend(uint32_t init_crc, const char* data, size_t n);
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8ul;
inline uint32_t Mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + kMaskDelta;
}
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace crc32c
}  // namespace rocksdb
