// crc32c_api.cc -- the C++ surface of include/wipdb/crc32c.h and the CPU
// entry points of the C-ABI.
//
// kv::crc32c::Extend replaces kv/src/util/crc32c.cc:1225-1227 (and its
// cpuid dispatch :1202-1224, here done lazily inside crc32c_cpu.cc, so there
// is no static-initialisation-order hazard when Extend is called from
// another translation unit's static constructor).  leveldb::crc32c::Extend
// replaces leveldb/util/crc32c.cc:275-380 (and pebblesdb/src/util/crc32c.cc,
// the same symbol); rocksdb::crc32c::Extend / IsFastCrc32Supported replace
// rocksdb/util/crc32c.cc's.
#include <stdint.h>

#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hip_crc32c_batch.h"
#include "../../include/wipdb/crc32c.h"
#include "gf2_crc32c.h"

namespace wipdb {
namespace cpu {
uint32_t Extend(uint32_t init_crc, const void* data, size_t n);
uint32_t ExtendPortable(uint32_t init_crc, const void* data, size_t n);
bool IsAccelerated();
void Batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
           const uint32_t* inits, uint32_t* out, size_t count, bool mask,
           int threads);
}  // namespace cpu
}  // namespace wipdb

namespace kv {
namespace crc32c {

std::string IsFastCrc32Supported() {
  // Same strings as the reference (kv/src/util/crc32c.cc:467-492).
  return wipdb::cpu::IsAccelerated() ? "Supported on x86" : "Not supported on x86";
}

uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return wipdb::cpu::Extend(init_crc, data, n);
}

}  // namespace crc32c
}  // namespace kv

namespace leveldb {
namespace crc32c {
uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return wipdb::cpu::Extend(init_crc, data, n);
}
}  // namespace crc32c
}  // namespace leveldb

namespace rocksdb {
namespace crc32c {
std::string IsFastCrc32Supported() {
  // rocksdb/util/crc32c.cc's wording for the SSE4.2 build
  return wipdb::cpu::IsAccelerated() ? "Supported on x86" : "Not supported on x86";
}
uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return wipdb::cpu::Extend(init_crc, data, n);
}
}  // namespace crc32c
}  // namespace rocksdb

namespace wipdb {
namespace crc32c {

namespace {
constexpr size_t kDefaultMinGpuBatch = 64;
constexpr size_t kMultiMinSpans = 8192;  // a listed-devices batch this big is sharded
constexpr size_t kUnset = ~size_t(0);
std::atomic<size_t> g_min_gpu_batch{kUnset};  // SetMinGpuBatch, else the env / default
std::atomic<uint64_t> g_gpu_batches{0}, g_cpu_batches{0};
std::atomic<int> g_last_error{0};
std::atomic<uint32_t> g_round_robin{0};
std::mutex g_mu;
int g_ctx_rc[64] = {0};  // a device's first failure, kept

// WIPDB_CRC_* (include/wipdb/crc32c.h), read once.
struct EnvConfig {
  enum Mode { kAuto, kGpu, kCpu } mode = kAuto;
  size_t min_batch = kDefaultMinGpuBatch;
  std::vector<int> devices;
};
const EnvConfig& Env() {
  static const EnvConfig cfg = [] {
    EnvConfig c;
    if (const char* m = getenv("WIPDB_CRC_MODE")) {
      const std::string v(m);
      if (v == "gpu") c.mode = EnvConfig::kGpu;
      else if (v == "cpu") c.mode = EnvConfig::kCpu;
    }
    if (const char* n = getenv("WIPDB_CRC_MIN_GPU_BATCH")) {
      char* end = nullptr;
      const unsigned long long v = strtoull(n, &end, 10);
      if (end != n && *end == '\0') c.min_batch = static_cast<size_t>(v);
    }
    if (const char* d = getenv("WIPDB_CRC_DEVICES")) {
      const char* p = d;
      while (*p) {
        char* end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p) break;  // not a number: ignore the rest
        if (v >= 0 && v < 64) c.devices.push_back(static_cast<int>(v));
        p = *end == ',' ? end + 1 : end;
      }
    }
    return c;
  }();
  return cfg;
}

// The process-wide context of a device (hcrc_ctx_shared: created on first
// use, it lives until the process ends -- hcrc_ctx_destroy refuses it), shared
// with hcrc_batch_multi; a device whose context could not be created is not
// retried.
int CtxFor(int device, hcrc_ctx** out) {
  if (device < 0 || device >= 64) return HCRC_ERR_NO_DEVICE;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx_rc[device] != HCRC_OK) return g_ctx_rc[device];
  }
  const int rc = hcrc_ctx_shared(device, out);
  if (rc != HCRC_OK) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_ctx_rc[device] = rc;
  }
  return rc;
}

int GpuBatch(const char* base, const uint64_t* offsets, const uint32_t* lengths,
             const uint32_t* inits, uint32_t* out, size_t count, int flags, int device) {
  const EnvConfig& env = Env();
  if (device == kDeviceFromEnv) {
    const size_t nd = env.devices.size();
    if (nd > 1 && count >= kMultiMinSpans)
      return hcrc_batch_multi(env.devices.data(), static_cast<int>(nd), base, offsets, lengths,
                              inits, out, count, flags);
    device = nd ? env.devices[g_round_robin.fetch_add(1) % nd] : 0;
  }
  hcrc_ctx* ctx = nullptr;
  int rc = CtxFor(device, &ctx);
  if (rc == HCRC_OK) rc = hcrc_batch(ctx, base, offsets, lengths, inits, out, count, flags);
  return rc;
}
}  // namespace

int ExtendBatch(const char* base, const uint64_t* offsets, const uint32_t* lengths,
                const uint32_t* inits, uint32_t* out, size_t count, bool mask,
                BatchPolicy policy, int device) {
  const int flags = mask ? HCRC_MASK_OUTPUT : 0;
  const EnvConfig& env = Env();
  size_t min_batch = g_min_gpu_batch.load();
  if (min_batch == kUnset) min_batch = env.min_batch;
  if (policy == BatchPolicy::kAuto) {
    if (env.mode == EnvConfig::kCpu) policy = BatchPolicy::kCpuOnly;
    else if (env.mode == EnvConfig::kGpu) min_batch = 0;
  }
  if (policy != BatchPolicy::kCpuOnly &&
      (policy == BatchPolicy::kGpuOnly || count >= min_batch)) {
    const int rc = GpuBatch(base, offsets, lengths, inits, out, count, flags, device);
    if (rc == HCRC_OK) {
      ++g_gpu_batches;
      return HCRC_OK;
    }
    if (policy == BatchPolicy::kGpuOnly) return rc;
    g_last_error = rc;  // kAuto: stay infallible, like Extend
  }
  wipdb::cpu::Batch(reinterpret_cast<const uint8_t*>(base), offsets, lengths, inits,
                    out, count, mask, 1);
  ++g_cpu_batches;
  return HCRC_OK;
}

void SetMinGpuBatch(size_t spans) { g_min_gpu_batch = spans; }

BatchStats GetBatchStats() {
  BatchStats s;
  s.gpu_batches = g_gpu_batches.load();
  s.cpu_batches = g_cpu_batches.load();
  s.last_error = g_last_error.load();
  return s;
}

}  // namespace crc32c
}  // namespace wipdb

extern "C" {

uint32_t hcrc_cpu_extend(uint32_t init_crc, const void* data, size_t n) {
  return wipdb::cpu::Extend(init_crc, data, n);
}

uint32_t hcrc_cpu_extend_portable(uint32_t init_crc, const void* data, size_t n) {
  return wipdb::cpu::ExtendPortable(init_crc, data, n);
}

int hcrc_cpu_batch(const void* base, const uint64_t* offsets,
                   const uint32_t* lengths, const uint32_t* init_crcs,
                   uint32_t* out_crcs, size_t count, int flags, int threads) {
  if (count && (!base || !offsets || !lengths || !out_crcs)) return HCRC_ERR_INVALID;
  if (flags & HCRC_DEVICE_PTRS) return HCRC_ERR_INVALID;
  wipdb::cpu::Batch(static_cast<const uint8_t*>(base), offsets, lengths, init_crcs,
                    out_crcs, count, (flags & HCRC_MASK_OUTPUT) != 0, threads);
  return HCRC_OK;
}

int hcrc_cpu_is_accelerated(void) { return wipdb::cpu::IsAccelerated() ? 1 : 0; }

uint32_t hcrc_mask(uint32_t crc) { return wipdb::gf2::Mask(crc); }
uint32_t hcrc_unmask(uint32_t masked_crc) { return wipdb::gf2::Unmask(masked_crc); }

}  // extern "C"
