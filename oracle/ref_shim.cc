// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY (see oracle/crc32c_oracle.c).
//
// A C-ABI shim around the REFERENCE kv::crc32c (kv/src/util/crc32c.h:24,
// kv/src/util/crc32c.cc:1225-1227), compiled from the reference's own
// sources where they lie under /root/reference by oracle/Makefile into
// oracle/_ref/libref_crc32c.so.  Nothing from the reference is copied into
// this repository: this file only includes the reference header through -I.
//
// Used (a) by tests/ to pin oracle/crc32c_oracle.c and to regenerate
// tests/golden/, and (b) by bench.py's cpu_baseline leg as the reference
// CPU throughput (cpu_baseline.kind = "reference").
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <thread>
#include <vector>

#include "util/crc32c.h"  // /root/reference/kv/src/util/crc32c.h

extern "C" {

uint32_t ref_crc32c_extend(uint32_t init_crc, const char* data, size_t n) {
  return kv::crc32c::Extend(init_crc, data, n);
}

uint32_t ref_crc32c_value(const char* data, size_t n) {
  return kv::crc32c::Value(data, n);
}

uint32_t ref_mask(uint32_t crc) { return kv::crc32c::Mask(crc); }
uint32_t ref_unmask(uint32_t m) { return kv::crc32c::Unmask(m); }

// 1 if the reference picked an SSE4.2 path ("Supported on x86").
int ref_is_fast(void) {
  return kv::crc32c::IsFastCrc32Supported().rfind("Supported", 0) == 0;
}

// Batch loop over the reference Extend, statically partitioned over
// `threads` std::threads (threads <= 1: caller's thread).  This is what
// WriteRawBlock does per block (kv/src/table/table_builder.cc:194-196) but
// over a whole array, so the CPU baseline can be timed beside the GPU.
void ref_crc32c_batch(const char* base, const uint64_t* offsets,
                      const uint32_t* lengths, const uint32_t* inits,
                      uint32_t* out, size_t count, int mask, int threads) {
  auto run = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      uint32_t c = kv::crc32c::Extend(inits ? inits[i] : 0u, base + offsets[i],
                                      lengths[i]);
      out[i] = mask ? kv::crc32c::Mask(c) : c;
    }
  };
  if (threads <= 1 || count < 2) {
    run(0, count);
    return;
  }
  std::vector<std::thread> pool;
  size_t per = (count + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    size_t lo = per * t, hi = lo + per < count ? lo + per : count;
    if (lo >= hi) break;
    pool.emplace_back(run, lo, hi);
  }
  for (auto& th : pool) th.join();
}

}  // extern "C"
