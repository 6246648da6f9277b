// hcrc_api.cc -- host side of the hip_crc32c_batch C-ABI
// (include/hip_crc32c_batch.h): contexts, table upload, launches, pinned
// staging for host-resident batches, multi-GPU sharding.
//
// The kernels are in crc32c_kernels.hip; the CPU path in crc32c_cpu.cc.
// No entry point here falls back to the CPU: every HIP failure is returned
// as an HCRC_ERR_* code (DESIGN.md "Errors").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/hip_crc32c_batch.h"
#include "crc32c_device.h"
#include "crc32c_lds.h"
#include "gf2_crc32c.h"

namespace wipdb {
namespace cpu {
uint32_t Extend(uint32_t init_crc, const void* data, size_t n);
bool IsAccelerated();
void Batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
           const uint32_t* inits, uint32_t* out, size_t count, bool mask,
           int threads);
}  // namespace cpu
namespace dev {
__global__ void crc32c_spans_kernel(const uint8_t*, const uint64_t*,
                                    const uint32_t*, const uint32_t*, uint32_t*,
                                    uint64_t, uint32_t, const DevTables*, uint32_t*);
__global__ void crc32c_strided_kernel(const uint8_t*, uint64_t, uint32_t,
                                      uint32_t, uint32_t*, uint64_t, uint32_t,
                                      const DevTables*, uint32_t*);
__global__ void crc32c_verify_kernel(const uint8_t*, const uint64_t*,
                                     const uint32_t*, uint8_t*, uint64_t,
                                     const DevTables*, uint32_t*, uint32_t, uint32_t*);
__global__ void readstream_kernel(const uint8_t*, uint64_t, uint32_t, uint32_t*,
                                  uint64_t);
__global__ void fill_splitmix64_kernel(uint64_t*, uint64_t, uint64_t, uint64_t);
__global__ void crc32c_partition_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                        const uint32_t*, uint64_t, SmallList, uint32_t,
                                        SmallList);
// instantiated for 8-lane (257..1024 B) and 2-lane (<= 256 B) subgroups
template <int SGT>
__global__ void crc32c_small_kernel(const uint8_t*, SmallList, uint32_t*, uint32_t,
                                    const DevTables*, uint8_t*);
}  // namespace dev
namespace lk {
__global__ void crc32c_lds_spans_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                        const uint32_t*, uint32_t*, uint64_t, uint32_t,
                                        const uint8_t*);
__global__ void crc32c_lds_strided_kernel(const uint8_t*, uint64_t, uint32_t, uint32_t,
                                          uint32_t*, uint64_t, uint32_t, const uint8_t*);
__global__ void crc32c_lds_verify_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                         uint8_t*, uint64_t, uint32_t, uint32_t*,
                                         const uint8_t*);
}  // namespace lk
}  // namespace wipdb

using wipdb::dev::DevTables;

namespace {

constexpr size_t kSlotBytes = size_t(64) << 20;  // pinned staging per slot
constexpr size_t kSlotSpans = size_t(1) << 18;   // descriptors per slot

struct Slot {
  uint8_t* h_data = nullptr;  // pinned
  uint64_t* h_off = nullptr;  // pinned
  uint32_t* h_len = nullptr;
  uint32_t* h_init = nullptr;
  uint32_t* h_out = nullptr;
  uint8_t* d_data = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint32_t* d_init = nullptr;
  uint32_t* d_out = nullptr;
  size_t cap_bytes = 0;
  hipEvent_t done = nullptr;
  // results still to be copied out to the caller once `done` fires
  uint32_t* user_out = nullptr;
  size_t n_out = 0;
};

}  // namespace

// A launch's work-pool counters (crc32c_kernels.hip WorkShare, WIPDB_GPOOL):
// the pool counter and the arrival count, 128 bytes apart.  The kernel's
// last workgroup zeroes them, so a buffer is ready again once `ev`
// (recorded after its launch) has completed.
struct PoolBuf {
  uint32_t* p = nullptr;
  hipEvent_t ev = nullptr;
};

struct hcrc_ctx {
  std::vector<PoolBuf> pools;  // under mu
  // stream-ordered scratch (small-span lists) comes from a private pool that
  // keeps its memory mapped between calls (release threshold: never)
  hipMemPool_t scratch_pool = nullptr;
  int device = -1;
  hipStream_t stream = nullptr;
  DevTables* d_tab = nullptr;      // small-span kernel tables
  uint8_t* d_image = nullptr;       // LDS image of the LDS-staged kernels (crc32c_lds.h)
  int num_cu = 0;
  std::mutex mu;
  Slot slots[2];
  bool slots_ready = false;
};

namespace {

#define HCRC_CHECK(expr)                                  \
  do {                                                    \
    hipError_t e_ = (expr);                               \
    if (e_ != hipSuccess) {                               \
      return e_ == hipErrorOutOfMemory ? HCRC_ERR_NO_MEMORY \
                                       : HCRC_ERR_HIP;    \
    }                                                     \
  } while (0)

const wipdb::gf2::Tables& HostTables() {
  static const wipdb::gf2::Tables* t = [] {
    auto* x = new wipdb::gf2::Tables;
    wipdb::gf2::BuildTables(x);
    return x;
  }();
  return *t;
}

void BuildDevTables(DevTables* dt) {
  const auto& T = HostTables();
  memcpy(dt->t, T.t, sizeof(dt->t));  // slicing-by-4: T.t[0..3]
  for (uint32_t j = 0; j < wipdb::dev::kNumShift; ++j)
    wipdb::gf2::BuildShiftTable(uint64_t(16) << j, dt->shift[j]);
  for (int i = 0; i < 256; ++i) dt->inv_top[i] = T.inv_top[i];
  memcpy(dt->head0, T.head0, sizeof(dt->head0));
}

// WIPDB_GRID_CAP (diagnostic build knob): at most this many workgroups, i.e.
// CUs, for the spans kernels (the package-power experiments)
#ifndef WIPDB_GRID_CAP
#define WIPDB_GRID_CAP 0
#endif
int LaunchGrid(hcrc_ctx* ctx, size_t count) {
  size_t need = (count + wipdb::dev::kSpansPerWG - 1) / wipdb::dev::kSpansPerWG;
  size_t g = std::min<size_t>(need, size_t(ctx->num_cu));
  if (WIPDB_GRID_CAP > 0) g = std::min<size_t>(g, size_t(WIPDB_GRID_CAP));
  return static_cast<int>(std::max<size_t>(g, 1));
}

// A pool buffer no launch is using (caller holds ctx->mu); Release records
// the launch that uses it.  Buffers are zeroed once at allocation, and every
// launch leaves its buffer zeroed (release_pool), so reuse needs no memset.
struct WorkPool {
  hcrc_ctx* ctx = nullptr;
  size_t idx = 0;
  uint32_t* p = nullptr;
  int Acquire(hcrc_ctx* c, hipStream_t st) {
    ctx = c;
    for (idx = 0; idx < ctx->pools.size(); ++idx)
      if (hipEventQuery(ctx->pools[idx].ev) == hipSuccess) break;
    if (idx == ctx->pools.size()) {
      PoolBuf b;
      HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&b.p), 256));
      if (hipMemsetAsync(b.p, 0, 256, st) != hipSuccess ||
          hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipFree(b.p);
        return HCRC_ERR_HIP;
      }
      ctx->pools.push_back(b);
    }
    p = ctx->pools[idx].p;
    return HCRC_OK;
  }
  int Release(hipStream_t st) {
    if (!p) return HCRC_OK;
    p = nullptr;
    return hipEventRecord(ctx->pools[idx].ev, st) == hipSuccess ? HCRC_OK : HCRC_ERR_HIP;
  }
};

// partition kernel workgroups per CU: enough waves to hide the descriptor
// loads' latency (2 per CU: 187 us for 1 M spans, 16: ~50 us)
#ifndef WIPDB_PART_WG
#define WIPDB_PART_WG 16
#endif

// The kernels keep span indices in 32 bits: larger batches go in pieces.
constexpr size_t kMaxLaunchSpans = size_t(1) << 31;

// LDS-staged kernels: one workgroup per CU, but no more than the batch's
// 16-span blocks (a workgroup's units are blocks w, w + grid, ...).
int LdsGrid(hcrc_ctx* ctx, size_t count) {
  const size_t need = (count + 15) / 16;
  return static_cast<int>(std::max<size_t>(std::min<size_t>(need, size_t(ctx->num_cu)), 1));
}

int LaunchSpansKernel(hcrc_ctx* ctx, const void* base, const uint64_t* off,
                      const uint32_t* len, const uint32_t* init, uint32_t* out,
                      size_t count, uint32_t kflags, hipStream_t st) {
  for (size_t pos = 0; pos < count; pos += kMaxLaunchSpans) {
    const size_t n = std::min(count - pos, kMaxLaunchSpans);
    hipLaunchKernelGGL(wipdb::lk::crc32c_lds_spans_kernel, dim3(LdsGrid(ctx, n)),
                       dim3(wipdb::lk::kThreads), wipdb::lk::kLdsBytes, st,
                       static_cast<const uint8_t*>(base), off + pos, len + pos,
                       init ? init + pos : nullptr, out + pos, static_cast<uint64_t>(n), kflags,
                       ctx->d_image);
    if (hipGetLastError() != hipSuccess) return HCRC_ERR_LAUNCH;
  }
  return HCRC_OK;
}

// Two small-span lists (8-lane and 2-lane subgroups) carved out of one
// scratch block of n * 40 + 64 bytes; returns their two counters.
uint32_t* CarveSmallLists(uint8_t* scratch, size_t n, wipdb::dev::SmallList* sl,
                          wipdb::dev::SmallList* tl) {
  wipdb::dev::SmallList* l[2] = {sl, tl};
  uint8_t* p = scratch;
  for (auto* x : l) {
    x->off = reinterpret_cast<uint64_t*>(p);
    x->len = reinterpret_cast<uint32_t*>(p + n * 8);
    x->init = x->len + n;
    x->id = x->init + n;
    p += n * 20;
  }
  uint32_t* counts = reinterpret_cast<uint32_t*>(p);
  sl->count = counts;
  tl->count = counts + 1;
  return counts;
}

// The small-span kernel over both lists (each launch exits at once when its
// list is empty).
int LaunchSmall(hcrc_ctx* ctx, const uint8_t* base, const wipdb::dev::SmallList& sl,
                const wipdb::dev::SmallList& tl, uint32_t* out, uint32_t flags, uint8_t* status,
                hipStream_t st) {
  hipLaunchKernelGGL((wipdb::dev::crc32c_small_kernel<8>), dim3(ctx->num_cu),
                     dim3(wipdb::dev::kThreads), wipdb::dev::kLdsBytes, st, base, sl, out, flags,
                     ctx->d_tab, status);
  hipLaunchKernelGGL((wipdb::dev::crc32c_small_kernel<2>), dim3(ctx->num_cu),
                     dim3(wipdb::dev::kThreads), wipdb::dev::kLdsBytes, st, base, tl, out, flags,
                     ctx->d_tab, status);
  return hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH;
}

// HCRC_SPLIT_SMALL: the spans of at most kSmallMax bytes are compacted by
// the partition kernel and checksummed 8 per wave slot by the small kernel;
// the spans kernel skips them.  Everything is ordered on `st`, the scratch
// is stream-ordered (hipMallocFromPoolAsync / hipFreeAsync), so concurrent calls on
// different streams never share it.
int LaunchSplit(hcrc_ctx* ctx, const void* base, const uint64_t* off, const uint32_t* len,
                const uint32_t* init, uint32_t* out, size_t count, uint32_t mask,
                hipStream_t st) {
  const size_t n = count;
  uint8_t* scratch = nullptr;
  HCRC_CHECK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&scratch), n * 40 + 64,
                                    ctx->scratch_pool, st));
  wipdb::dev::SmallList sl, tl;
  uint32_t* counts = CarveSmallLists(scratch, n, &sl, &tl);
  int rc = HCRC_OK;
  if (hipMemsetAsync(counts, 0, 8, st) != hipSuccess) rc = HCRC_ERR_HIP;
  if (rc == HCRC_OK) {
    const int pgrid = static_cast<int>(std::min<size_t>((n + 255) / 256, size_t(ctx->num_cu) * WIPDB_PART_WG));
    hipLaunchKernelGGL(wipdb::dev::crc32c_partition_kernel, dim3(pgrid), dim3(256), 0, st,
                       static_cast<const uint8_t*>(base), off, len, init,
                       static_cast<uint64_t>(n), sl, 0u, tl);
    rc = hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH;
  }
  // the spans kernel first: it leaves the partial CRCs of the spans it cuts
  // (kFlagSplitRem) in out, which the small kernel then continues
  if (rc == HCRC_OK)
    rc = LaunchSpansKernel(ctx, base, off, len, init, out, count,
                           mask | wipdb::dev::kFlagSkipSmall | wipdb::dev::kFlagSplitRem, st);
  if (rc == HCRC_OK)
    rc = LaunchSmall(ctx, static_cast<const uint8_t*>(base), sl, tl, out, mask, nullptr, st);
  if (hipFreeAsync(scratch, st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
  return rc;
}

// split: HCRC_SPLIT_SMALL requested (device batches) or chosen for a host
// piece with enough small spans.
int LaunchSpans(hcrc_ctx* ctx, const void* base, const uint64_t* off,
                const uint32_t* len, const uint32_t* init, uint32_t* out,
                size_t count, int flags, hipStream_t st) {
  if (count == 0) return HCRC_OK;
  const uint32_t mask = static_cast<uint32_t>(flags & HCRC_MASK_OUTPUT);
  if ((flags & HCRC_SPLIT_SMALL) && count < (size_t(1) << 31))
    return LaunchSplit(ctx, base, off, len, init, out, count, mask, st);
  return LaunchSpansKernel(ctx, base, off, len, init, out, count, mask, st);
}

// Host pieces: split when enough spans are small, or just over a segment
// (a table block of 4 KiB + its last entry: the remainder goes to the small
// kernel), for the small kernel to pay for its two extra launches.
#ifndef WIPDB_AUTO_SPLIT_MIN
#define WIPDB_AUTO_SPLIT_MIN 256
#endif
constexpr size_t kAutoSplitMin = WIPDB_AUTO_SPLIT_MIN;

int AutoSplit(const uint32_t* lengths, size_t n) {
  size_t small = 0;
  for (size_t i = 0; i < n && small < kAutoSplitMin; ++i) {
    const uint32_t l = lengths[i];
    small += l <= wipdb::dev::kSmallMax || (l > 4096u + 15u && l <= 4096u + wipdb::dev::kSmallMax);
  }
  return small >= kAutoSplitMin ? HCRC_SPLIT_SMALL : 0;
}

// Async entry points take the caller's stream; NULL is the HIP default
// (null) stream, as everywhere in HIP (torch's default stream is NULL too).
// The context's own stream is available through hcrc_ctx_stream().
hipStream_t StreamOf(hcrc_ctx* ctx, void* stream) {
  (void)ctx;
  return static_cast<hipStream_t>(stream);
}

int EnsureSlots(hcrc_ctx* ctx) {
  if (ctx->slots_ready) return HCRC_OK;
  for (Slot& s : ctx->slots) {
    HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_data), kSlotBytes));
    HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_off), kSlotSpans * 8));
    HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_len), kSlotSpans * 4));
    HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_init), kSlotSpans * 4));
    HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_out), kSlotSpans * 4));
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_data), kSlotBytes));
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_off), kSlotSpans * 8));
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_len), kSlotSpans * 4));
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_init), kSlotSpans * 4));
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_out), kSlotSpans * 4));
    HCRC_CHECK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    s.cap_bytes = kSlotBytes;
  }
  ctx->slots_ready = true;
  return HCRC_OK;
}

int GrowSlot(Slot& s, size_t bytes) {
  if (bytes <= s.cap_bytes) return HCRC_OK;
  HCRC_CHECK(hipHostFree(s.h_data));
  HCRC_CHECK(hipFree(s.d_data));
  s.h_data = nullptr;
  s.d_data = nullptr;
  HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_data), bytes));
  HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_data), bytes));
  s.cap_bytes = bytes;
  return HCRC_OK;
}

// Wait for a slot's previous piece and hand its results to the caller.
int DrainSlot(Slot& s) {
  if (!s.user_out) return HCRC_OK;
  HCRC_CHECK(hipEventSynchronize(s.done));
  memcpy(s.user_out, s.h_out, s.n_out * 4);
  s.user_out = nullptr;
  s.n_out = 0;
  return HCRC_OK;
}

// Copy spans [lo, hi) into the slot's pinned buffer, keeping each span's
// address mod 16 (so aligned blocks stay on the aligned fast path).
void PackSpans(Slot& s, const uint8_t* base, const uint64_t* offsets,
               const uint32_t* lengths, const uint32_t* inits, size_t lo,
               size_t hi, size_t* used_bytes) {
  size_t cur = 0;
  for (size_t i = lo; i < hi; ++i) {
    const uint8_t* src = base + offsets[i];
    cur = ((cur + 15) & ~size_t(15)) + (reinterpret_cast<uintptr_t>(src) & 15);
    s.h_off[i - lo] = cur;
    s.h_len[i - lo] = lengths[i];
    s.h_init[i - lo] = inits ? inits[i] : 0u;
    cur += lengths[i];
  }
  *used_bytes = cur;
  // the byte copy itself, split over a few threads for big pieces
  const size_t n = hi - lo;
  auto copy = [&](size_t a, size_t b) {
    for (size_t i = a; i < b; ++i)
      memcpy(s.h_data + s.h_off[i], base + offsets[lo + i], s.h_len[i]);
  };
  if (cur < (size_t(8) << 20) || n < 64) {
    copy(0, n);
  } else {
    const int nt = 8;
    std::vector<std::thread> pool;
    const size_t per = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
      size_t a = per * t, b = std::min(n, a + per);
      if (a >= b) break;
      pool.emplace_back(copy, a, b);
    }
    for (auto& th : pool) th.join();
  }
}

size_t PackedBytes(const uint64_t* offsets, const uint32_t* lengths,
                   const uint8_t* base, size_t i) {
  (void)offsets;
  (void)base;
  return size_t(lengths[i]) + 32;
}

// Device-visible address of host memory that is pinned (hcrc_host_alloc,
// hipHostMalloc) or registered (hcrc_host_register, hipHostRegister) over
// the whole span range [lo, hi); nullptr for pageable memory.
const uint8_t* MappedDevicePtr(const uint8_t* lo, const uint8_t* hi) {
  auto map = [](const uint8_t* p) -> const uint8_t* {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
      (void)hipGetLastError();  // pageable memory: not an error for us
      return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return static_cast<const uint8_t*>(a.devicePointer) +
           (p - static_cast<const uint8_t*>(a.hostPointer));
  };
  const uint8_t* dlo = map(lo);
  if (!dlo || hi <= lo) return dlo;
  const uint8_t* dhi = map(hi - 1);  // the same allocation must cover the end
  return (dhi && dhi - dlo == (hi - 1) - lo) ? dlo : nullptr;
}

// Zero-copy: the kernel reads the spans straight out of mapped host memory
// over PCIe (no staging copy, no device buffer); only the descriptors and
// the results cross through the slots.  ~1.6x the staged path's rate.
int BatchZeroCopy(hcrc_ctx* ctx, const uint8_t* dev_base, const uint64_t* offsets,
                  const uint32_t* lengths, const uint32_t* inits, uint32_t* out,
                  size_t count, int flags) {
  size_t i = 0;
  int k = 0;
  while (i < count) {
    Slot& s = ctx->slots[k];
    int rc = DrainSlot(s);
    if (rc) return rc;
    const size_t n = std::min(count - i, kSlotSpans);
    memcpy(s.h_off, offsets + i, n * 8);
    memcpy(s.h_len, lengths + i, n * 4);
    if (inits) memcpy(s.h_init, inits + i, n * 4);
    else memset(s.h_init, 0, n * 4);
    HCRC_CHECK(hipMemcpyAsync(s.d_off, s.h_off, n * 8, hipMemcpyHostToDevice, ctx->stream));
    HCRC_CHECK(hipMemcpyAsync(s.d_len, s.h_len, n * 4, hipMemcpyHostToDevice, ctx->stream));
    HCRC_CHECK(hipMemcpyAsync(s.d_init, s.h_init, n * 4, hipMemcpyHostToDevice, ctx->stream));
    rc = LaunchSpans(ctx, dev_base, s.d_off, s.d_len, s.d_init, s.d_out, n,
                     flags | AutoSplit(lengths + i, n), ctx->stream);
    if (rc) return rc;
    HCRC_CHECK(hipMemcpyAsync(s.h_out, s.d_out, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HCRC_CHECK(hipEventRecord(s.done, ctx->stream));
    s.user_out = out + i;
    s.n_out = n;
    i += n;
    k ^= 1;
  }
  for (Slot& s : ctx->slots) {
    int rc = DrainSlot(s);
    if (rc) return rc;
  }
  return HCRC_OK;
}

int BatchHost(hcrc_ctx* ctx, const uint8_t* base, const uint64_t* offsets,
              const uint32_t* lengths, const uint32_t* inits, uint32_t* out,
              size_t count, int flags) {
  int rc = EnsureSlots(ctx);
  if (rc) return rc;
  {
    uint64_t lo = ~uint64_t(0), hi = 0;
    for (size_t i = 0; i < count; ++i) {
      lo = std::min(lo, offsets[i]);
      hi = std::max(hi, offsets[i] + lengths[i]);
    }
    const uint8_t* dev = MappedDevicePtr(base + lo, base + hi);
    if (dev) return BatchZeroCopy(ctx, dev - lo, offsets, lengths, inits, out, count, flags);
  }
  size_t i = 0;
  int k = 0;
  while (i < count) {
    Slot& s = ctx->slots[k];
    rc = DrainSlot(s);
    if (rc) return rc;
    // piece = spans [i, j) fitting the slot
    size_t bytes = 0, j = i;
    while (j < count && j - i < kSlotSpans) {
      size_t b = PackedBytes(offsets, lengths, base, j);
      if (j > i && bytes + b > s.cap_bytes) break;
      bytes += b;
      ++j;
    }
    rc = GrowSlot(s, bytes);
    if (rc) return rc;
    size_t used = 0;
    PackSpans(s, base, offsets, lengths, inits, i, j, &used);
    const size_t n = j - i;
    HCRC_CHECK(hipMemcpyAsync(s.d_data, s.h_data, used, hipMemcpyHostToDevice,
                              ctx->stream));
    HCRC_CHECK(hipMemcpyAsync(s.d_off, s.h_off, n * 8, hipMemcpyHostToDevice,
                              ctx->stream));
    HCRC_CHECK(hipMemcpyAsync(s.d_len, s.h_len, n * 4, hipMemcpyHostToDevice,
                              ctx->stream));
    HCRC_CHECK(hipMemcpyAsync(s.d_init, s.h_init, n * 4, hipMemcpyHostToDevice,
                              ctx->stream));
    rc = LaunchSpans(ctx, s.d_data, s.d_off, s.d_len, s.d_init, s.d_out, n,
                     flags | AutoSplit(lengths + i, n), ctx->stream);
    if (rc) return rc;
    HCRC_CHECK(hipMemcpyAsync(s.h_out, s.d_out, n * 4, hipMemcpyDeviceToHost,
                              ctx->stream));
    HCRC_CHECK(hipEventRecord(s.done, ctx->stream));
    s.user_out = out + i;
    s.n_out = n;
    i = j;
    k ^= 1;
  }
  for (Slot& s : ctx->slots) {
    rc = DrainSlot(s);
    if (rc) return rc;
  }
  return HCRC_OK;
}

std::mutex g_ctx_mu;
std::map<int, hcrc_ctx*>& SharedCtxs() {
  static auto* m = new std::map<int, hcrc_ctx*>;
  return *m;
}

int SharedCtx(int device, hcrc_ctx** out) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto& m = SharedCtxs();
  auto it = m.find(device);
  if (it != m.end()) {
    *out = it->second;
    return HCRC_OK;
  }
  int rc = hcrc_ctx_create(device, out);
  if (rc) return rc;
  m[device] = *out;
  return HCRC_OK;
}

}  // namespace

extern "C" {

int hcrc_abi_version(void) { return HCRC_ABI_VERSION; }

int hcrc_device_count(int* count) {
  if (!count) return HCRC_ERR_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    *count = 0;
    return HCRC_ERR_NO_DEVICE;
  }
  *count = n;
  return HCRC_OK;
}

const char* hcrc_strerror(int code) {
  switch (code) {
    case HCRC_OK: return "ok";
    case HCRC_ERR_INVALID: return "invalid argument";
    case HCRC_ERR_NO_DEVICE: return "no HIP device";
    case HCRC_ERR_NO_MEMORY: return "out of memory";
    case HCRC_ERR_HIP: return "HIP runtime error";
    case HCRC_ERR_LAUNCH: return "kernel launch failed";
    case HCRC_ERR_MISMATCH: return "checksum mismatch";
    default: return "unknown error";
  }
}

int hcrc_ctx_create(int device, hcrc_ctx** out_ctx) {
  if (!out_ctx) return HCRC_ERR_INVALID;
  *out_ctx = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
    return HCRC_ERR_NO_DEVICE;
  std::unique_ptr<hcrc_ctx> ctx(new hcrc_ctx);
  ctx->device = device;
  HCRC_CHECK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HCRC_CHECK(hipGetDeviceProperties(&prop, device));
  ctx->num_cu = prop.multiProcessorCount;
  HCRC_CHECK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  {
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    HCRC_CHECK(hipMemPoolCreate(&ctx->scratch_pool, &props));
    uint64_t keep = ~uint64_t(0);
    HCRC_CHECK(hipMemPoolSetAttribute(ctx->scratch_pool, hipMemPoolAttrReleaseThreshold, &keep));
  }
  const unsigned lds = wipdb::dev::kLdsBytes;
  static_assert(wipdb::lk::kLdsBytes == wipdb::dev::kLdsBytes, "both kernel families use 160 KiB");
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::lk::crc32c_lds_spans_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::lk::crc32c_lds_strided_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::lk::crc32c_lds_verify_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::dev::crc32c_spans_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::dev::crc32c_strided_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::dev::crc32c_verify_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::dev::crc32c_small_kernel<8>),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::dev::crc32c_small_kernel<2>),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  HCRC_CHECK(hipFuncSetAttribute(
      reinterpret_cast<const void*>(wipdb::dev::readstream_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  std::unique_ptr<DevTables> ht(new DevTables);
  BuildDevTables(ht.get());
  HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx->d_tab), sizeof(DevTables)));
  HCRC_CHECK(hipMemcpy(ctx->d_tab, ht.get(), sizeof(DevTables),
                       hipMemcpyHostToDevice));
  {
    std::vector<uint32_t> img(wipdb::lk::kImageBytes / 4);
    wipdb::lk::BuildLdsImage(img.data());
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx->d_image), wipdb::lk::kImageBytes));
    HCRC_CHECK(hipMemcpy(ctx->d_image, img.data(), wipdb::lk::kImageBytes, hipMemcpyHostToDevice));
  }
  *out_ctx = ctx.release();
  return HCRC_OK;
}

int hcrc_ctx_destroy(hcrc_ctx* ctx) {
  if (!ctx) return HCRC_ERR_INVALID;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto& m = SharedCtxs();
    auto it = m.find(ctx->device);
    if (it != m.end() && it->second == ctx) m.erase(it);
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (Slot& s : ctx->slots) {
    if (s.h_data) (void)hipHostFree(s.h_data);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_len) (void)hipHostFree(s.h_len);
    if (s.h_init) (void)hipHostFree(s.h_init);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_data) (void)hipFree(s.d_data);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_len) (void)hipFree(s.d_len);
    if (s.d_init) (void)hipFree(s.d_init);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  for (PoolBuf& b : ctx->pools) {
    if (b.ev) {
      (void)hipEventSynchronize(b.ev);
      (void)hipEventDestroy(b.ev);
    }
    (void)hipFree(b.p);
  }
  if (ctx->d_tab) (void)hipFree(ctx->d_tab);
  if (ctx->d_image) (void)hipFree(ctx->d_image);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->scratch_pool) {
    (void)hipDeviceSynchronize();
    (void)hipMemPoolDestroy(ctx->scratch_pool);
  }
  delete ctx;
  return HCRC_OK;
}

void* hcrc_ctx_stream(hcrc_ctx* ctx) { return ctx ? ctx->stream : nullptr; }
int hcrc_ctx_device(hcrc_ctx* ctx) { return ctx ? ctx->device : -1; }

int hcrc_batch(hcrc_ctx* ctx, const void* base, const uint64_t* offsets,
               const uint32_t* lengths, const uint32_t* init_crcs,
               uint32_t* out_crcs, size_t count, int flags) {
  if (!ctx || (count && (!base || !offsets || !lengths || !out_crcs)))
    return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_DEVICE_PTRS | HCRC_MASK_OUTPUT | HCRC_SPLIT_SMALL)) return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HCRC_CHECK(hipSetDevice(ctx->device));
  if (flags & HCRC_DEVICE_PTRS) {
    // default stream: ordered after whatever the caller enqueued there
    int rc = LaunchSpans(ctx, base, offsets, lengths, init_crcs, out_crcs, count,
                         flags, nullptr);
    if (rc) return rc;
    HCRC_CHECK(hipStreamSynchronize(nullptr));
    return HCRC_OK;
  }
  return BatchHost(ctx, static_cast<const uint8_t*>(base), offsets, lengths,
                   init_crcs, out_crcs, count, flags);
}

int hcrc_batch_async(hcrc_ctx* ctx, const void* d_base, const uint64_t* d_offsets,
                     const uint32_t* d_lengths, const uint32_t* d_init_crcs,
                     uint32_t* d_out_crcs, size_t count, int flags,
                     void* stream) {
  if (!ctx || !(flags & HCRC_DEVICE_PTRS)) return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_DEVICE_PTRS | HCRC_MASK_OUTPUT | HCRC_SPLIT_SMALL)) return HCRC_ERR_INVALID;
  if (count && (!d_base || !d_offsets || !d_lengths || !d_out_crcs))
    return HCRC_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HCRC_CHECK(hipSetDevice(ctx->device));
  return LaunchSpans(ctx, d_base, d_offsets, d_lengths, d_init_crcs, d_out_crcs,
                     count, flags, StreamOf(ctx, stream));
}

int hcrc_batch_strided_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride,
                             uint32_t length, uint32_t init_crc,
                             uint32_t* d_out_crcs, size_t count, int flags,
                             void* stream) {
  if (!ctx || !(flags & HCRC_DEVICE_PTRS)) return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_DEVICE_PTRS | HCRC_MASK_OUTPUT)) return HCRC_ERR_INVALID;
  if (count && (!d_base || !d_out_crcs)) return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HCRC_CHECK(hipSetDevice(ctx->device));
  const hipStream_t st = StreamOf(ctx, stream);
  for (size_t pos = 0; pos < count; pos += kMaxLaunchSpans) {
    const size_t n = std::min(count - pos, kMaxLaunchSpans);
    hipLaunchKernelGGL(wipdb::lk::crc32c_lds_strided_kernel, dim3(LdsGrid(ctx, n)),
                       dim3(wipdb::lk::kThreads), wipdb::lk::kLdsBytes, st,
                       static_cast<const uint8_t*>(d_base) + pos * stride, stride, length,
                       init_crc, d_out_crcs + pos, static_cast<uint64_t>(n),
                       static_cast<uint32_t>(flags & HCRC_MASK_OUTPUT), ctx->d_image);
    if (hipGetLastError() != hipSuccess) return HCRC_ERR_LAUNCH;
  }
  return HCRC_OK;
}

namespace {
// One verify launch (count < 2^31); with split, blocks of at most kSmallMax
// bytes and the remainders of blocks that just overrun a segment go to the
// small kernel, the cut blocks' partial CRCs passing through `partial`.
int LaunchVerify(hcrc_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                 uint8_t* status, size_t n, bool split, hipStream_t st) {
  uint8_t* scratch = nullptr;
  wipdb::dev::SmallList sl{}, tl{};
  uint32_t* partial = nullptr;
  uint32_t kflags = 0;
  int rc = HCRC_OK;
  if (split) {
    HCRC_CHECK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&scratch), n * 44 + 64,
                                      ctx->scratch_pool, st));
    partial = reinterpret_cast<uint32_t*>(scratch);
    uint32_t* counts = CarveSmallLists(scratch + n * 4, n, &sl, &tl);
    kflags = wipdb::dev::kFlagSkipSmall | wipdb::dev::kFlagSplitRem;
    if (hipMemsetAsync(counts, 0, 8, st) != hipSuccess) rc = HCRC_ERR_HIP;
    if (rc == HCRC_OK) {
      const int pgrid =
          static_cast<int>(std::min<size_t>((n + 255) / 256, size_t(ctx->num_cu) * WIPDB_PART_WG));
      hipLaunchKernelGGL(wipdb::dev::crc32c_partition_kernel, dim3(pgrid), dim3(256), 0, st,
                         base, off, len, nullptr, static_cast<uint64_t>(n), sl, 1u, tl);
      rc = hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH;
    }
  }
  if (rc == HCRC_OK) {
    hipLaunchKernelGGL(wipdb::lk::crc32c_lds_verify_kernel, dim3(LdsGrid(ctx, n)),
                       dim3(wipdb::lk::kThreads), wipdb::lk::kLdsBytes, st, base, off, len,
                       status, static_cast<uint64_t>(n), kflags, partial, ctx->d_image);
    rc = hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH;
  }
  if (split && rc == HCRC_OK)
    rc = LaunchSmall(ctx, base, sl, tl, partial, wipdb::dev::kFlagVerify, status, st);
  if (scratch && hipFreeAsync(scratch, st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
  return rc;
}
}  // namespace

int hcrc_verify_async_ex(hcrc_ctx* ctx, const void* d_base, const uint64_t* d_offsets,
                         const uint32_t* d_lengths, uint8_t* d_status, size_t count, int flags,
                         void* stream) {
  if (!ctx) return HCRC_ERR_INVALID;
  if (flags & ~HCRC_SPLIT_SMALL) return HCRC_ERR_INVALID;
  if (count && (!d_base || !d_offsets || !d_lengths || !d_status))
    return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HCRC_CHECK(hipSetDevice(ctx->device));
  const hipStream_t st = StreamOf(ctx, stream);
  for (size_t pos = 0; pos < count; pos += kMaxLaunchSpans) {
    const size_t n = std::min(count - pos, kMaxLaunchSpans);
    const int rc = LaunchVerify(ctx, static_cast<const uint8_t*>(d_base), d_offsets + pos,
                                d_lengths + pos, d_status + pos, n,
                                (flags & HCRC_SPLIT_SMALL) != 0, st);
    if (rc != HCRC_OK) return rc;
  }
  return HCRC_OK;
}

int hcrc_verify_async(hcrc_ctx* ctx, const void* d_base, const uint64_t* d_offsets,
                      const uint32_t* d_lengths, uint8_t* d_status, size_t count,
                      void* stream) {
  return hcrc_verify_async_ex(ctx, d_base, d_offsets, d_lengths, d_status, count, 0, stream);
}

int hcrc_readstream_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride,
                          uint32_t length, uint32_t* d_out, size_t count,
                          void* stream) {
  if (!ctx || (count && (!d_base || !d_out)) || (length & 15))
    return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HCRC_CHECK(hipSetDevice(ctx->device));
  // same geometry as the CRC kernels, no LDS tables
#ifndef WIPDB_RS_LDS
#define WIPDB_RS_LDS 0
#endif
  hipLaunchKernelGGL(wipdb::dev::readstream_kernel, dim3(LaunchGrid(ctx, count)),
                     dim3(wipdb::dev::kThreads), WIPDB_RS_LDS ? wipdb::dev::kLdsBytes : 0,
                     StreamOf(ctx, stream),
                     static_cast<const uint8_t*>(d_base), stride, length, d_out,
                     static_cast<uint64_t>(count));
  return hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH;
}

int hcrc_fill_splitmix64_async(hcrc_ctx* ctx, void* d_dst, uint64_t nbytes,
                               uint64_t seed, uint64_t first_word, void* stream) {
  if (!ctx || (nbytes && !d_dst) || (nbytes & 7) ||
      (reinterpret_cast<uintptr_t>(d_dst) & 7))
    return HCRC_ERR_INVALID;
  if (nbytes == 0) return HCRC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HCRC_CHECK(hipSetDevice(ctx->device));
  const uint64_t nwords = nbytes / 8;
  const int grid = static_cast<int>(std::min<uint64_t>((nwords + 255) / 256,
                                                       uint64_t(ctx->num_cu) * 16));
  hipLaunchKernelGGL(wipdb::dev::fill_splitmix64_kernel, dim3(grid), dim3(256), 0,
                     StreamOf(ctx, stream), static_cast<uint64_t*>(d_dst), nwords,
                     first_word, seed);
  return hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH;
}

int hcrc_sync(hcrc_ctx* ctx, void* stream) {
  if (!ctx) return HCRC_ERR_INVALID;
  HCRC_CHECK(hipSetDevice(ctx->device));
  HCRC_CHECK(hipStreamSynchronize(StreamOf(ctx, stream)));
  return HCRC_OK;
}

int hcrc_batch_multi(const int* devices, int ndev, const void* base,
                     const uint64_t* offsets, const uint32_t* lengths,
                     const uint32_t* init_crcs, uint32_t* out_crcs, size_t count,
                     int flags) {
  if (!devices || ndev <= 0 || (flags & HCRC_DEVICE_PTRS)) return HCRC_ERR_INVALID;
  if (count && (!base || !offsets || !lengths || !out_crcs))
    return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  // byte-balanced contiguous shards
  uint64_t total = 0;
  for (size_t i = 0; i < count; ++i) total += lengths[i] + 64;
  std::vector<size_t> cut(ndev + 1, count);
  cut[0] = 0;
  uint64_t acc = 0;
  int d = 1;
  for (size_t i = 0; i < count && d < ndev; ++i) {
    acc += lengths[i] + 64;
    while (d < ndev && acc >= total * d / ndev) cut[d++] = i + 1;
  }
  std::vector<int> rcs(ndev, HCRC_OK);
  std::vector<std::thread> pool;
  for (int k = 0; k < ndev; ++k) {
    const size_t lo = cut[k], hi = cut[k + 1];
    if (lo >= hi) continue;
    pool.emplace_back([&, k, lo, hi] {
      hcrc_ctx* ctx = nullptr;
      int rc = SharedCtx(devices[k], &ctx);
      if (rc == HCRC_OK)
        rc = hcrc_batch(ctx, base, offsets + lo, lengths + lo,
                        init_crcs ? init_crcs + lo : nullptr, out_crcs + lo,
                        hi - lo, flags & HCRC_MASK_OUTPUT);
      rcs[k] = rc;
    });
  }
  for (auto& th : pool) th.join();
  for (int rc : rcs)
    if (rc) return rc;
  return HCRC_OK;
}

int hcrc_host_alloc(size_t bytes, void** out_ptr) {
  if (!out_ptr) return HCRC_ERR_INVALID;
  // portable + mapped: every device of a multi-GPU batch reads it zero-copy
  HCRC_CHECK(hipHostMalloc(out_ptr, bytes, hipHostMallocPortable | hipHostMallocMapped));
  return HCRC_OK;
}

int hcrc_host_free(void* ptr) {
  HCRC_CHECK(hipHostFree(ptr));
  return HCRC_OK;
}

int hcrc_host_register(void* ptr, size_t bytes) {
  if (!ptr || !bytes) return HCRC_ERR_INVALID;
  HCRC_CHECK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  return HCRC_OK;
}

int hcrc_host_unregister(void* ptr) {
  if (!ptr) return HCRC_ERR_INVALID;
  HCRC_CHECK(hipHostUnregister(ptr));
  return HCRC_OK;
}

}  // extern "C"
