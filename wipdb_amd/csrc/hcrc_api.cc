// hcrc_api.cc -- host side of the hip_crc32c_batch C-ABI
// (include/hip_crc32c_batch.h): contexts, the LDS image upload, launches,
// size-class splitting, pinned staging for host-resident batches, zero-copy
// for registered host memory, multi-GPU sharding.
//
// The kernels are in crc32c_lds.hip (+ crc32c_util.hip); the CPU path in
// crc32c_cpu.cc.  No entry point here falls back to the CPU: every HIP
// failure is returned as an HCRC_ERR_* code (DESIGN.md "Errors").
//
// Threading (flush, compaction and split threads call the engine
// concurrently, kv/tests/db/kv_bench.cc:2041-2043): the async entry points
// take no lock at all -- they only enqueue on the caller's stream; a
// synchronous call leases a "lane" (its own stream and pinned staging
// slots) for its duration, so concurrent callers of one context run on
// different streams at the same time.  Every entry point restores the
// caller's current HIP device before it returns.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/hip_crc32c_batch.h"
#include "crc32c_lds.h"

namespace wipdb {
namespace lk {
template <int INIT>
__global__ void crc32c_lds_spans_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                        const uint32_t*, uint32_t*, uint64_t, uint32_t,
                                        const uint8_t*, const uint32_t*, unsigned int*);
__global__ void crc32c_lds_strided_kernel(const uint8_t*, uint64_t, uint32_t, uint32_t,
                                          uint32_t*, uint64_t, uint32_t, const uint8_t*,
                                          unsigned int*);
__global__ void crc32c_lds_verify_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                         uint8_t*, uint64_t, const uint8_t*, unsigned int*);
template <int INIT>
__global__ void crc32c_lds_packed_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                         const uint32_t*, uint32_t*, uint64_t, uint32_t,
                                         const uint8_t*, const uint32_t*, const uint32_t*, uint32_t,
                                         uint32_t, unsigned int*, unsigned int*);
__global__ void crc32c_ps_index_kernel(const uint8_t*, const uint64_t*, const uint32_t*, uint64_t,
                                       uint32_t, uint32_t*, uint32_t*, uint32_t, uint32_t);
__global__ void crc32c_dma_ceiling_kernel(const uint8_t*, uint64_t, uint32_t*, uint64_t,
                                          const uint8_t*);
template <int G, int OUT>
__global__ void crc32c_lds_list_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                       const uint32_t*, const uint32_t*, const uint32_t*, void*,
                                       uint32_t, const uint8_t*);
__global__ void crc32c_lds_partition_kernel(const uint8_t*, const uint64_t*, const uint32_t*,
                                            const uint32_t*, uint64_t, uint32_t, SpanList,
                                            SpanList, SpanList);
}  // namespace lk
namespace util {
__global__ void readstream_kernel(const uint8_t*, uint64_t, uint32_t, uint32_t*, uint64_t);
__global__ void fill_splitmix64_kernel(uint64_t*, uint64_t, uint64_t, uint64_t);
__global__ void check_spans_kernel(const uint64_t*, const uint32_t*, uint64_t, uint64_t, uint32_t,
                                   unsigned long long*);
__global__ void split_expand_kernel(const uint64_t*, const uint32_t*, const uint32_t*, uint64_t,
                                    uint32_t, uint32_t, uint32_t, uint64_t*, uint32_t*, uint32_t*,
                                    uint32_t*, uint32_t*, uint32_t*, uint32_t*);
__global__ void balance_sums_kernel(const uint32_t*, uint64_t, uint32_t, uint64_t*);
__global__ void balance_bounds_kernel(const uint32_t*, uint64_t, uint32_t, const uint64_t*, uint32_t,
                                      uint32_t, uint32_t*);
__global__ void split_copy_kernel(const uint32_t*, const uint32_t*, uint32_t*, uint64_t, uint32_t);
__global__ void split_combine_kernel(const uint32_t*, const uint32_t*, const uint32_t*,
                                     const uint32_t*, const uint32_t*, uint32_t*, uint64_t, uint32_t,
                                     uint32_t, uint32_t);
}  // namespace util
}  // namespace wipdb

__global__ void crc32c_lds_fault_probe_kernel(unsigned int*);

namespace lk = wipdb::lk;

namespace {

#define HCRC_CHECK(expr)                                    \
  do {                                                      \
    hipError_t e_ = (expr);                                 \
    if (e_ != hipSuccess) {                                 \
      return e_ == hipErrorOutOfMemory ? HCRC_ERR_NO_MEMORY \
                                       : HCRC_ERR_HIP;      \
    }                                                       \
  } while (0)

// Makes `device` current and restores the caller's device on scope exit, so
// a library call never leaves a WipDB flush thread or a torch process on
// another GPU.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    ok_ = prev_ == device || hipSetDevice(device) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev_ >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev_) (void)hipSetDevice(prev_);
  }
  bool ok() const { return ok_; }

 private:
  int prev_ = -1;
  bool ok_ = false;
};

#define HCRC_DEVICE(ctx)          \
  DeviceGuard dg_((ctx)->device); \
  if (!dg_.ok()) return HCRC_ERR_HIP

constexpr size_t kStageBytes = size_t(32) << 20;  // pinned staging per slot
constexpr size_t kStageSpans = size_t(1) << 17;   // descriptors per slot
constexpr int kMaxLanes = 8;                      // concurrent synchronous calls per context
// Fault words of the lane-packed kernels (crc32c_lds.hip report_fault): one
// per launch owner -- word k (1 .. kMaxLanes) for synchronous lane k, then
// one per caller stream of the *_async entry points (kStreamFaultWords; past
// that, streams share word 0).
constexpr uint32_t kStreamFaultWords = 1024;
constexpr uint32_t kFaultWords = 1 + kMaxLanes + kStreamFaultWords;
// HCRC_PACKED chunks per workgroup (one per wave, progress-balanced;
// WIPDB_PS_CHUNKS: tuning runs) and the largest grid a host-built index serves
constexpr int kPsChunksPerGroup = 16;
constexpr uint32_t kPsMaxHostChunks = 16u * 1024u;
constexpr size_t kPsHostWords = lk::kPsMetaWords + kPsMaxHostChunks + 1;

// One piece of a host batch in flight: pinned host buffers and their device
// mirrors.  A piece's descriptors -- offsets, lengths, inits and a
// host-built HCRC_PACKED index (meta words + first[]) -- share one block
// (Layout) and cross in one copy (SendDesc): each small copy costs
// ~10 us of a one-SST call.
constexpr size_t kDescBytes = kStageSpans * 16 + 3 * 256 + kPsHostWords * 4;
struct Slot {
  uint8_t* h_data = nullptr;  // pinned
  uint8_t* h_desc = nullptr;  // pinned, kDescBytes
  uint32_t* h_out = nullptr;  // pinned
  uint8_t* d_data = nullptr;
  uint8_t* d_desc = nullptr;
  uint32_t* d_out = nullptr;
  // device views of h_desc / h_out: a small zero-copy piece's kernel reads
  // its descriptors and writes its results there (no copy either way)
  uint8_t* hd_desc = nullptr;
  uint32_t* hd_out = nullptr;
  // the current piece's views of the descriptor blocks (Layout)
  uint64_t* h_off = nullptr;
  uint32_t* h_len = nullptr;
  uint32_t* h_init = nullptr;
  uint32_t* h_ps = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint32_t* d_init = nullptr;
  uint32_t* d_ps = nullptr;
  size_t len_at = 0, init_at = 0, ps_at = 0;
  size_t cap_bytes = 0;
  hipEvent_t done = nullptr;
  // the copy engine's pieces of pinned batches (BatchZeroCopy): a device
  // buffer of kDmaBytes and the event of its copy, made on first use
  uint8_t* d_copy = nullptr;
  hipEvent_t copied = nullptr;
  // results still to be copied out to the caller once `done` fires
  uint32_t* user_out = nullptr;
  size_t n_out = 0;

  void Free() {
    if (h_data) (void)hipHostFree(h_data);
    if (h_desc) (void)hipHostFree(h_desc);
    if (h_out) (void)hipHostFree(h_out);
    if (d_data) (void)hipFree(d_data);
    if (d_desc) (void)hipFree(d_desc);
    if (d_out) (void)hipFree(d_out);
    if (done) (void)hipEventDestroy(done);
    if (d_copy) (void)hipFree(d_copy);
    if (copied) (void)hipEventDestroy(copied);
    *this = Slot();
  }
  // All buffers, or none (a partial failure frees what it got).
  int Alloc() {
    hipError_t e = hipSuccess;
    auto host = [&](void** p, size_t n) {
      if (e == hipSuccess) e = hipHostMalloc(p, n);
    };
    auto dev = [&](void** p, size_t n) {
      if (e == hipSuccess) e = hipMalloc(p, n);
    };
    host(reinterpret_cast<void**>(&h_data), kStageBytes);
    host(reinterpret_cast<void**>(&h_desc), kDescBytes);
    host(reinterpret_cast<void**>(&h_out), kStageSpans * 4);
    dev(reinterpret_cast<void**>(&d_data), kStageBytes);
    dev(reinterpret_cast<void**>(&d_desc), kDescBytes);
    dev(reinterpret_cast<void**>(&d_out), kStageSpans * 4);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&hd_desc), h_desc, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&hd_out), h_out, 0);
    if (e != hipSuccess) {
      Free();
      return e == hipErrorOutOfMemory ? HCRC_ERR_NO_MEMORY : HCRC_ERR_HIP;
    }
    cap_bytes = kStageBytes;
    return HCRC_OK;
  }
  // The descriptor views for a piece of n (<= kStageSpans) spans: offsets,
  // lengths, inits, the index, each 256-byte aligned.
  void Layout(size_t n) {
    auto up = [](size_t b) { return (b + 255) & ~size_t(255); };
    len_at = up(n * 8);
    init_at = len_at + up(n * 4);
    ps_at = init_at + up(n * 4);
    h_off = reinterpret_cast<uint64_t*>(h_desc);
    h_len = reinterpret_cast<uint32_t*>(h_desc + len_at);
    h_init = reinterpret_cast<uint32_t*>(h_desc + init_at);
    h_ps = reinterpret_cast<uint32_t*>(h_desc + ps_at);
    d_off = reinterpret_cast<uint64_t*>(d_desc);
    d_len = reinterpret_cast<uint32_t*>(d_desc + len_at);
    d_init = reinterpret_cast<uint32_t*>(d_desc + init_at);
    d_ps = reinterpret_cast<uint32_t*>(d_desc + ps_at);
  }
  // The same views with the device side on h_desc itself (a small
  // zero-copy piece: the kernel reads the descriptors over PCIe).
  void DirectLayout(size_t n) {
    Layout(n);
    d_off = reinterpret_cast<uint64_t*>(hd_desc);
    d_len = reinterpret_cast<uint32_t*>(hd_desc + len_at);
    d_init = reinterpret_cast<uint32_t*>(hd_desc + init_at);
    d_ps = reinterpret_cast<uint32_t*>(hd_desc + ps_at);
  }
  // One copy of the piece's descriptors (+ inits, + ps_words of index).
  hipError_t SendDesc(size_t n, bool inits, size_t ps_words, hipStream_t st) {
    const size_t bytes = ps_words ? ps_at + ps_words * 4 : (inits ? init_at : len_at) + n * 4;
    return hipMemcpyAsync(d_desc, h_desc, bytes, hipMemcpyHostToDevice, st);
  }
  // A data buffer of at least `bytes` (one span larger than the slot): the
  // new buffers are allocated before the old ones are released, so a
  // failure leaves the slot as it was.
  int Grow(size_t bytes) {
    if (bytes <= cap_bytes) return HCRC_OK;
    uint8_t *h = nullptr, *d = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&h), bytes) != hipSuccess) return HCRC_ERR_NO_MEMORY;
    if (hipMalloc(reinterpret_cast<void**>(&d), bytes) != hipSuccess) {
      (void)hipHostFree(h);
      return HCRC_ERR_NO_MEMORY;
    }
    (void)hipHostFree(h_data);
    (void)hipFree(d_data);
    h_data = h;
    d_data = d;
    cap_bytes = bytes;
    return HCRC_OK;
  }
  // Wait for the piece in flight and hand its results to the caller.
  int Drain() {
    if (!user_out) return HCRC_OK;
    HCRC_CHECK(hipEventSynchronize(done));
    memcpy(user_out, h_out, n_out * 4);
    user_out = nullptr;
    n_out = 0;
    return HCRC_OK;
  }
};

// The resources of one synchronous call: a stream and two staging slots
// (one piece is copied and computed while the next is packed).
struct Lane {
  hipStream_t stream = nullptr;
  hipStream_t copy = nullptr;  // the copy engine's pieces (BatchZeroCopy), made on first use
  Slot slots[2];
  bool slots_ready = false;
  int index = 0;  // 1 .. kMaxLanes: its fault word (hcrc_ctx::fault_words[index])
};

// Host ranges pinned (hcrc_host_alloc) or registered (hcrc_host_register)
// through this library, by start address.
struct HostRange {
  size_t bytes;
  uint8_t* dev;  // device-visible address of the first byte
};
std::mutex g_host_mu;
std::map<uintptr_t, HostRange>& HostRanges() {
  static auto* m = new std::map<uintptr_t, HostRange>;
  return *m;
}

// The device-side base for a host batch whose every span lies inside a range
// pinned or registered through this library (zero-copy), or nullptr (some
// span is in pageable memory, or straddles two ranges: the batch is staged).
// Each span is looked up -- the ranges are sorted by start and a batch's
// spans usually walk them in order, so the last hit is tried first.  Spans in
// one range translate through its device address; spans over several
// ranges need every range identity-mapped (device address == host address,
// what ROCm gives pinned and registered memory under unified addressing).
const uint8_t* MappedSpans(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                           size_t n) {
  std::lock_guard<std::mutex> lk(g_host_mu);
  auto& m = HostRanges();
  if (m.empty() || n == 0) return nullptr;
  auto hit = m.end();
  bool several = false, identity = true;
  for (size_t i = 0; i < n; ++i) {
    const uintptr_t lo = reinterpret_cast<uintptr_t>(base + offsets[i]);
    const uintptr_t hi = lo + lengths[i];
    if (hit == m.end() || lo < hit->first || hi > hit->first + hit->second.bytes) {
      auto it = m.upper_bound(lo);
      if (it == m.begin()) return nullptr;
      --it;
      if (hi > it->first + it->second.bytes) return nullptr;
      if (hit != m.end() && it != hit) several = true;
      hit = it;
      identity = identity && reinterpret_cast<uintptr_t>(hit->second.dev) == hit->first;
    }
  }
  if (several) return identity ? base : nullptr;
  return hit->second.dev - (hit->first - reinterpret_cast<uintptr_t>(base));
}

// The pinned or registered range holding host address a: [*lo, *hi), or false.
bool PinnedRangeOf(uintptr_t a, uintptr_t* lo, uintptr_t* hi) {
  std::lock_guard<std::mutex> lk(g_host_mu);
  auto& m = HostRanges();
  auto it = m.upper_bound(a);
  if (it == m.begin()) return false;
  --it;
  if (a >= it->first + it->second.bytes) return false;
  *lo = it->first;
  *hi = it->first + it->second.bytes;
  return true;
}

}  // namespace

struct hcrc_ctx {
  int device = -1;
  int num_cu = 0;
  hipStream_t stream = nullptr;  // the context's own stream (hcrc_ctx_stream)
  uint8_t* d_image = nullptr;    // LDS image of the kernels (crc32c_lds.h)
  // stream-ordered scratch (size-class lists) from a private pool that keeps
  // its memory mapped between calls (release threshold: never)
  hipMemPool_t scratch_pool = nullptr;
  // fault words of the lane-packed kernels (kFaultWords, pinned coherent
  // host memory the kernels write with a system-scope store; d_: its device
  // view): a launch that saw a fault (crc32c_lds.h kFault*) sets its owner's
  // word, so the fault is reported to that owner only -- a synchronous
  // call's lane, or the caller stream of an async launch (stream_words,
  // assigned on first use; hcrc_sync / hcrc_ctx_check read and clear them)
  unsigned int* fault_words = nullptr;
  unsigned int* d_fault_words = nullptr;
  std::mutex faults_mu;
  std::map<hipStream_t, uint32_t> stream_words;
  uint32_t stream_words_next = 0;        // words handed out so far (of kStreamFaultWords)
  std::vector<uint32_t> free_stream_words;  // returned by hcrc_stream_forget
  // HCRC_PACKED's pre-pass output per stream (meta words + the chunk index),
  // kept across launches: the verdict word is tagged with the stream's
  // launch count, so nothing is cleared or allocated per call
  struct PsScratch {
    uint32_t* d = nullptr;
    uint32_t epoch = 0;
    std::mutex mu;  // a launch pair (pre-pass, kernel) is enqueued whole
    // The verdict of the stream's last pre-pass, as its packed kernel left it
    // (a pinned word the kernel stores with system scope: epoch << 4 | the
    // kPsBad* / kPsEa bits), and the batch it was for: the next launch of
    // the SAME batch (base, columns, count) whose verdict came back "suits
    // run_ea" or "not packed" skips the pre-pass and runs the spans kernel,
    // which samples and chooses by itself -- so a repeated batch pays the
    // pre-pass once, and a wrong hint (the caller rewrote the columns in
    // place) costs speed, never a CRC.  Re-checked every kHintRecheck skips.
    uint32_t* h_hint = nullptr;  // pinned, coherent
    uint32_t* d_hint = nullptr;  // its device view
    const void* key_base = nullptr;
    const void* key_off = nullptr;
    const void* key_len = nullptr;
    size_t key_n = 0;
    uint32_t key_epoch = 0;
    uint32_t skips = 0;
  };
  std::mutex ps_mu;
  std::map<hipStream_t, std::unique_ptr<PsScratch>> ps_scratch;
  // lanes of synchronous calls
  std::mutex lanes_mu;
  std::condition_variable lanes_cv;
  std::vector<Lane*> free_lanes;
  std::vector<std::unique_ptr<Lane>> lanes;
  // Releases what the context holds: hcrc_ctx_destroy, and every error
  // return of hcrc_ctx_create after a partial construction.
  ~hcrc_ctx();
};

namespace {

// A lane for the duration of one synchronous call.
class LaneLease {
 public:
  explicit LaneLease(hcrc_ctx* ctx) : ctx_(ctx) {
    std::unique_lock<std::mutex> lk(ctx->lanes_mu);
    for (;;) {
      if (!ctx->free_lanes.empty()) {
        lane_ = ctx->free_lanes.back();
        ctx->free_lanes.pop_back();
        return;
      }
      if (static_cast<int>(ctx->lanes.size()) < kMaxLanes) {
        ctx->lanes.emplace_back(new Lane);
        lane_ = ctx->lanes.back().get();
        lane_->index = static_cast<int>(ctx->lanes.size());
        return;
      }
      ctx->lanes_cv.wait(lk);
    }
  }
  ~LaneLease() {
    // An error return mid-batch can leave a slot with a piece in flight and
    // the caller's output pointer recorded: wait for the stream and forget
    // those pointers, so the next lessee's Drain() never writes into a
    // buffer the failed call's caller (or BatchHostLong's temporary) owned.
    bool pending = false;
    for (const Slot& s : lane_->slots) pending = pending || s.user_out != nullptr;
    if (pending) {
      if (lane_->stream) (void)hipStreamSynchronize(lane_->stream);
      if (lane_->copy) (void)hipStreamSynchronize(lane_->copy);
      for (Slot& s : lane_->slots) {
        s.user_out = nullptr;
        s.n_out = 0;
      }
    }
    {
      std::lock_guard<std::mutex> lk(ctx_->lanes_mu);
      ctx_->free_lanes.push_back(lane_);
    }
    ctx_->lanes_cv.notify_one();
  }
  LaneLease(const LaneLease&) = delete;
  LaneLease& operator=(const LaneLease&) = delete;
  // The lane's stream, created on first use (on the context's device).
  int Stream() {
    if (!lane_->stream) HCRC_CHECK(hipStreamCreateWithFlags(&lane_->stream, hipStreamNonBlocking));
    return HCRC_OK;
  }
  // The lane's fault word, cleared before the call's launches (the lane's
  // earlier launches are complete: its calls are synchronous).
  int FaultsBefore() {
    __atomic_store_n(ctx_->fault_words + lane_->index, 0u, __ATOMIC_SEQ_CST);
    return HCRC_OK;
  }
  // The device view of the lane's fault word (the kernels' argument).
  unsigned int* FaultWord() const { return ctx_->d_fault_words + lane_->index; }
  // After the call's launches: waits for the stream, then HCRC_ERR_KERNEL if
  // one of them left a span uncomputed, else HCRC_OK.
  int CheckFaults() {
    HCRC_CHECK(hipStreamSynchronize(lane_->stream));
    return __atomic_load_n(ctx_->fault_words + lane_->index, __ATOMIC_SEQ_CST) ? HCRC_ERR_KERNEL
                                                                                : HCRC_OK;
  }
  // Stream and staging slots.
  int Staging() {
    int rc = Stream();
    if (rc) return rc;
    if (lane_->slots_ready) return HCRC_OK;
    for (Slot& s : lane_->slots)
      if (!s.cap_bytes && (rc = s.Alloc()) != HCRC_OK) return rc;
    lane_->slots_ready = true;
    return HCRC_OK;
  }
  Lane* operator->() const { return lane_; }
  Lane* get() const { return lane_; }

 private:
  hcrc_ctx* ctx_;
  Lane* lane_ = nullptr;
};

// The kernels keep span indices in 32 bits; size-class lists in 30.
constexpr size_t kMaxLaunchSpans = size_t(1) << 31;

// LDS-staged kernels: one workgroup per CU, but no more than the batch's
// 16-span blocks (a workgroup's units are blocks w, w + grid, ...).
int LdsGrid(hcrc_ctx* ctx, size_t count) {
  const size_t need = (count + 15) / 16;
  return static_cast<int>(std::max<size_t>(std::min<size_t>(need, size_t(ctx->num_cu)), 1));
}

int Launched() { return hipGetLastError() == hipSuccess ? HCRC_OK : HCRC_ERR_LAUNCH; }

// Size classes of a batch (HCRC_SPLIT_SMALL, crc32c_lds.h): a partition pass
// writes three lists, then the class-1, class-2 and class-4 kernels run in
// stream order.  Stream-ordered scratch, so concurrent calls on different
// streams never share it.  out_kind 0: CRCs (masked when `mask`)
// into u32 out; 1: verify statuses into u8 out.
int LaunchClasses(hcrc_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                  const uint32_t* init, void* out, size_t n, int out_kind, bool mask,
                  hipStream_t st) {
  // scratch: 3 lists of n entries -- the u64 offset columns first (8-byte
  // aligned), then the u32 columns (len, init, id), the 3 counters
  const size_t bytes = n * (3 * 8 + 3 * 12) + 16;
  uint8_t* scratch = nullptr;
  HCRC_CHECK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&scratch), bytes, ctx->scratch_pool,
                                    st));
  lk::SpanList L[3];
  uint8_t* p = scratch;
  for (auto& l : L) {
    l.off = reinterpret_cast<uint64_t*>(p);
    p += n * 8;
  }
  for (auto& l : L) {
    l.len = reinterpret_cast<uint32_t*>(p);
    l.init = l.len + n;
    l.id = l.init + n;
    p += n * 12;
  }
  uint32_t* counts = reinterpret_cast<uint32_t*>(p);
  for (int k = 0; k < 3; ++k) L[k].count = counts + k;

  int rc = hipMemsetAsync(counts, 0, 16, st) == hipSuccess ? HCRC_OK : HCRC_ERR_HIP;
  if (rc == HCRC_OK) {
    const size_t pgrid = std::min<size_t>((n + 255) / 256, size_t(ctx->num_cu) * 4);
    hipLaunchKernelGGL(lk::crc32c_lds_partition_kernel, dim3(std::max<size_t>(pgrid, 1)),
                       dim3(256), 0, st, base, off, len, init, static_cast<uint64_t>(n),
                       out_kind ? 1u : 0u, L[0], L[1], L[2]);
    rc = Launched();
  }
  const uint32_t kf = mask ? lk::kFlagMask : 0u;
  const dim3 grid(ctx->num_cu), blk(lk::kThreads);
  auto launch = [&](auto kernel, const lk::SpanList& l) {
    hipLaunchKernelGGL(kernel, grid, blk, lk::kLdsBytes, st, base,
                       static_cast<const uint64_t*>(l.off), static_cast<const uint32_t*>(l.len),
                       static_cast<const uint32_t*>(l.init), static_cast<const uint32_t*>(l.id),
                       static_cast<const uint32_t*>(l.count), out, kf,
                       static_cast<const uint8_t*>(ctx->d_image));
  };
  if (rc == HCRC_OK) {
    if (out_kind) {
      launch(lk::crc32c_lds_list_kernel<1, 1>, L[0]);
      launch(lk::crc32c_lds_list_kernel<2, 1>, L[1]);
      launch(lk::crc32c_lds_list_kernel<4, 1>, L[2]);
    } else {
      launch(lk::crc32c_lds_list_kernel<1, 0>, L[0]);
      launch(lk::crc32c_lds_list_kernel<2, 0>, L[1]);
      launch(lk::crc32c_lds_list_kernel<4, 0>, L[2]);
    }
    rc = Launched();
  }
  if (hipFreeAsync(scratch, st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
  return rc;
}

// Long spans of a device batch (HCRC_SPLIT_LONG, crc32c_util.hip): spans of
// at least kDevLongSpan bytes run as kDevPartBytes parts on many waves.  An
// expand pass writes the list (every other span once, the long ones' parts;
// a pool of `cap` part slots, past which spans stay whole), the class-1 list
// kernel computes it into a scratch array, then the unsplit results are
// copied out and each split span's parts combined by one wave.
constexpr uint32_t kDevPartBytes = 16u << 10;
constexpr uint32_t kDevLongSpan = 128u << 10;
constexpr size_t kDevPartCap = size_t(1) << 20;
constexpr size_t kDevPartCapMin = size_t(1) << 16;  // 1 GiB of long spans in any batch

int LaunchLong(hcrc_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len,
               const uint32_t* init, uint32_t* out, size_t n, bool mask, hipStream_t st) {
  const size_t cap = std::min(kDevPartCap, std::max(kDevPartCapMin, 16 * n));
  const size_t E = n + cap;  // list entries / scratch results
  const size_t bytes = E * 8 + E * 16 + n * 8 + 16;
  uint8_t* scratch = nullptr;
  HCRC_CHECK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&scratch), bytes, ctx->scratch_pool,
                                    st));
  uint64_t* l_off = reinterpret_cast<uint64_t*>(scratch);
  uint32_t* l_len = reinterpret_cast<uint32_t*>(scratch + E * 8);
  uint32_t* l_init = l_len + E;
  uint32_t* l_id = l_init + E;
  uint32_t* tmp = l_id + E;
  uint32_t* first = tmp + E;
  uint32_t* split_idx = first + n;
  uint32_t* counters = split_idx + n;
  int rc = hipMemsetAsync(counters, 0, 16, st) == hipSuccess ? HCRC_OK : HCRC_ERR_HIP;
  if (rc == HCRC_OK) {
    const int g = static_cast<int>(std::min<size_t>((n + 255) / 256, size_t(ctx->num_cu) * 8));
    hipLaunchKernelGGL(wipdb::util::split_expand_kernel, dim3(std::max(g, 1)), dim3(256), 0, st,
                       off, len, init, static_cast<uint64_t>(n), kDevPartBytes, kDevLongSpan,
                       static_cast<uint32_t>(cap), l_off, l_len, l_init, l_id, first, split_idx,
                       counters);
    auto* const list1 = lk::crc32c_lds_list_kernel<1, 0>;
    hipLaunchKernelGGL(list1, dim3(ctx->num_cu), dim3(lk::kThreads),
                       lk::kLdsBytes, st, base, static_cast<const uint64_t*>(l_off),
                       static_cast<const uint32_t*>(l_len), static_cast<const uint32_t*>(l_init),
                       static_cast<const uint32_t*>(l_id), static_cast<const uint32_t*>(counters),
                       static_cast<void*>(tmp), 0u, static_cast<const uint8_t*>(ctx->d_image));
    hipLaunchKernelGGL(wipdb::util::split_copy_kernel, dim3(std::max(g, 1)), dim3(256), 0, st,
                       static_cast<const uint32_t*>(tmp), static_cast<const uint32_t*>(first), out,
                       static_cast<uint64_t>(n), mask ? 1u : 0u);
    hipLaunchKernelGGL(wipdb::util::split_combine_kernel, dim3(ctx->num_cu * 4), dim3(256), 0, st,
                       len, static_cast<const uint32_t*>(first),
                       static_cast<const uint32_t*>(split_idx),
                       static_cast<const uint32_t*>(counters), static_cast<const uint32_t*>(tmp),
                       out, static_cast<uint64_t>(n), kDevPartBytes,
                       wipdb::gf2::XPow8N(kDevPartBytes), mask ? 1u : 0u);
    rc = Launched();
  }
  if (hipFreeAsync(scratch, st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
  return rc;
}

// A device batch of at most this many spans takes the long-span split by
// itself: its lengths are unknown on the host, and with so few spans one
// long span is the whole job -- run whole, a span's segments are chained on
// one wave (a lone 1 MiB span: 0.4 ms), split they run on the whole chip
// (0.07 ms).  Larger batches keep every wave busy with spans of their own
// (the spans kernel shares long spans over a workgroup's waves).  A host
// piece's lengths are known: it takes the split only when one of its spans
// is long enough to be cut (AutoLongHost).
constexpr size_t kAutoLongSpans = 16;
// HCRC_PACKED launches of fewer spans run the default path (LaunchSpans)
constexpr size_t kPackedMinSpans = size_t(1) << 15;
// streams with a packed scratch of their own (~16 KiB each); further streams'
// packed batches take the default path
constexpr size_t kPsStreams = 1024;
// a repeated batch skips the pre-pass on its last verdict at most this many
// times in a row, then is checked again (a buffer freed and reallocated at
// the same address with new contents is re-judged)
constexpr uint32_t kHintRecheck = 64;
enum class AutoLong { kNo, kDevice };

#ifdef WIPDB_HCRC_TEST_HOOKS
// Test build only (make testlib, tests/test_gpu_parity.py): with
// WIPDB_HCRC_FORCE_FAULT=1 every lane-packed launch reports a fault (its
// error word set after it, as the kernel would) -- the HCRC_ERR_KERNEL paths.
// hcrc_test_force_fault(on) overrides it from then on (per-stream tests).
std::atomic<int> g_force_fault{-1};
// the last packed launch's pre-pass words (meta[0]: 0 = streamed, else the
// kPsBad* bits of the fallback; meta[1..2]: chunk bytes)
uint32_t g_test_ps_meta[lk::kPsMetaWords];
// pieces of pinned batches copied by the copy engine / run zero-copy
std::atomic<uint64_t> g_test_dma_pieces{0}, g_test_zc_pieces{0};
bool ForcedFault() {
  int f = g_force_fault.load();
  if (f < 0) {
    const char* e = getenv("WIPDB_HCRC_FORCE_FAULT");
    int want = e && *e == '1' ? 1 : 0, expect = -1;
    g_force_fault.compare_exchange_strong(expect, want);
    f = g_force_fault.load();
  }
  return f == 1;
}
#endif

// A lane-packed launch is done: with the test build's forced fault, a fault
// is counted after it, as a faulting launch would count it.
int LaunchedLp(hipStream_t st, unsigned int* fault) {
  int rc = Launched();
#ifdef WIPDB_HCRC_TEST_HOOKS
  if (rc == HCRC_OK && ForcedFault()) {
    hipLaunchKernelGGL(crc32c_lds_fault_probe_kernel, dim3(1), dim3(64), 0, st, fault);
    rc = Launched();
  }
#else
  (void)st;
  (void)fault;
#endif
  return rc;
}

// The fault word of async launches on `st` (assigned on first use; word 0,
// shared, once kStreamFaultWords streams have one).  Device view.
unsigned int* StreamFaultWord(hcrc_ctx* ctx, hipStream_t st) {
  std::lock_guard<std::mutex> lk(ctx->faults_mu);
  auto it = ctx->stream_words.find(st);
  if (it != ctx->stream_words.end()) return ctx->d_fault_words + it->second;
  uint32_t k;
  if (!ctx->free_stream_words.empty()) {  // (a forgotten stream's word, cleared then)
    k = ctx->free_stream_words.back();
    ctx->free_stream_words.pop_back();
  } else if (ctx->stream_words_next < kStreamFaultWords) {
    k = 1u + kMaxLanes + ctx->stream_words_next++;
  } else {
    return ctx->d_fault_words;
  }
  ctx->stream_words.emplace(st, k);
  return ctx->d_fault_words + k;
}

// The stream's HCRC_PACKED scratch (words 32-bit words, cleared once),
// created on the stream's first packed launch; nullptr past kPsStreams
// streams or out of memory.
hcrc_ctx::PsScratch* PsScratchFor(hcrc_ctx* ctx, hipStream_t st, size_t words) {
  std::lock_guard<std::mutex> lk(ctx->ps_mu);
  auto it = ctx->ps_scratch.find(st);
  if (it != ctx->ps_scratch.end()) return it->second.get();
  if (ctx->ps_scratch.size() >= kPsStreams) return nullptr;
  auto ps = std::make_unique<hcrc_ctx::PsScratch>();
  if (hipHostMalloc(reinterpret_cast<void**>(&ps->h_hint), 4,
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return nullptr;
  *ps->h_hint = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&ps->d_hint), ps->h_hint, 0) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&ps->d), words * 4) != hipSuccess) {
    (void)hipHostFree(ps->h_hint);
    return nullptr;
  }
  // the verdict words only, ordered on the caller's stream ahead of its first
  // pre-pass (first[] is written by every pre-pass before it is read)
  if (hipMemsetAsync(ps->d, 0, lk::kPsMetaWords * 4, st) != hipSuccess) {
    (void)hipFree(ps->d);
    (void)hipHostFree(ps->h_hint);
    return nullptr;
  }
  hcrc_ctx::PsScratch* raw = ps.get();
  ctx->ps_scratch.emplace(st, std::move(ps));
  return raw;
}

// Descriptor batch on device memory, enqueued on st.  auto_long: kDevice for
// the device entry points (a batch of <= kAutoLongSpans spans splits its long
// spans by itself); host pieces decide on the host (AutoLongHost).
// A chunk index the host built for a piece it staged or checked
// (HostPsIndex): device words [meta (kPsMetaWords) | first[C + 1]], verdict
// tagged with epoch 1.
struct HostIndex {
  const uint32_t* d_ps;
  uint32_t C;
};

int PsChunksPerGroup() {
  static const int v = [] {
    const char* e = getenv("WIPDB_PS_CHUNKS");  // (tuning: chunks per workgroup)
    const int c = e ? atoi(e) : 0;
    return c >= 1 && c <= 1024 ? c : kPsChunksPerGroup;
  }();
  return v;
}
bool PsOnly() {
  static const bool v = getenv("WIPDB_PS_ONLY") && atoi(getenv("WIPDB_PS_ONLY")) != 0;
  return v;
}

int LaunchSpans(hcrc_ctx* ctx, const void* base, const uint64_t* off, const uint32_t* len,
                const uint32_t* init, uint32_t* out, size_t count, int flags, hipStream_t st,
                AutoLong auto_long, unsigned int* fault, const HostIndex* hidx = nullptr) {
  const bool mask = (flags & HCRC_MASK_OUTPUT) != 0;
  const bool split_long = (flags & HCRC_SPLIT_LONG) != 0 ||
                          (auto_long == AutoLong::kDevice && (flags & HCRC_SPLIT_SMALL) == 0 &&
                           count <= kAutoLongSpans);
  const bool split = !split_long && (flags & HCRC_SPLIT_SMALL) != 0;
  const size_t piece_max = split_long ? size_t(lk::kMaxListSpans) - kDevPartCap
                           : split    ? size_t(lk::kMaxListSpans)
                                      : kMaxLaunchSpans;
  for (size_t pos = 0; pos < count; pos += piece_max) {
    const size_t n = std::min(count - pos, piece_max);
    int rc;
    if (split_long) {
      rc = LaunchLong(ctx, static_cast<const uint8_t*>(base), off + pos, len + pos,
                      init ? init + pos : nullptr, out + pos, n, mask, st);
    } else if (split) {
      rc = LaunchClasses(ctx, static_cast<const uint8_t*>(base), off + pos, len + pos,
                         init ? init + pos : nullptr, out + pos, n, 0, mask, st);
    } else {
      const int grid = LdsGrid(ctx, n);
      // (HCRC_PACKED on fewer than kPackedMinSpans spans: the default path --
      // the pre-pass's launches cost ~10 us a call, more than the stream
      // saves on batches below ~128 MiB, profiles/r05ae_latency*.log)
      static const size_t packed_min = [] {
        const char* e = getenv("WIPDB_PS_MIN_SPANS");
        return e && *e ? static_cast<size_t>(atol(e)) : kPackedMinSpans;
      }();
      const int chunks_per_group = PsChunksPerGroup();
      const bool ps_only = PsOnly();
      if (hidx && count <= kMaxLaunchSpans &&
          hidx->C == static_cast<uint32_t>(chunks_per_group * grid)) {
        // a piece whose index the host built (HostPsIndex): no pre-pass, no
        // floor -- the packed kernel's own pick_ea still takes run_ea where
        // it suits the piece
        hipLaunchKernelGGL(init ? lk::crc32c_lds_packed_kernel<1> : lk::crc32c_lds_packed_kernel<0>,
                           dim3(grid), dim3(lk::kThreads), lk::kLdsBytes, st,
                           static_cast<const uint8_t*>(base), off, len, init, out,
                           static_cast<uint64_t>(n),
                           (mask ? lk::kFlagMask : 0u) | (ps_only ? lk::kFlagPsOnly : 0u),
                           ctx->d_image, hidx->d_ps + lk::kPsMetaWords, hidx->d_ps, hidx->C, 1u,
                           fault, static_cast<unsigned int*>(nullptr));
        rc = LaunchedLp(st, fault);
        if (rc) return rc;
        continue;
      }
      // the stream's pre-pass scratch (none: past kPsStreams streams or out
      // of memory -- the batch takes the default path)
      // (hipStreamPerThread is another queue on every host thread: a scratch
      // keyed by it would be shared between queues, so its batches take the
      // default path -- ADVICE r5)
      // Device batches of >= packed_min spans take the packed sequence --
      // flagged (HCRC_PACKED) or not: the pre-pass checks the promise, and a
      // batch that breaks it, or suits run_ea, runs the default pipelines
      // inside the packed kernel.  A repeated batch whose last verdict was
      // one of those skips the pre-pass (PsScratch::h_hint) and runs the
      // spans kernel below.
      // (no flag: launches of >= auto_min spans; WIPDB_PS_AUTO_MIN_SPANS for
      // tests and A/Bs, 0 = never)
      static const size_t auto_min = [] {
        const char* e = getenv("WIPDB_PS_AUTO_MIN_SPANS");
        return e && *e ? static_cast<size_t>(atol(e)) : kPackedMinSpans;
      }();
      const bool want_ps =
          (flags & HCRC_PACKED) ? n >= packed_min
                                : auto_long == AutoLong::kDevice && (flags & HCRC_BALANCE) == 0 &&
                                      auto_min != 0 && n >= auto_min;
      hcrc_ctx::PsScratch* ps =
          want_ps && st != hipStreamPerThread
              ? PsScratchFor(ctx, st, size_t(chunks_per_group) * ctx->num_cu + 1 + lk::kPsMetaWords)
              : nullptr;
      std::unique_lock<std::mutex> psl;
      if (ps) {
        psl = std::unique_lock<std::mutex>(ps->mu);
        const bool same = ps->key_base == base && ps->key_off == off + pos &&
                          ps->key_len == len + pos && ps->key_n == n;
        const uint32_t h = __atomic_load_n(ps->h_hint, __ATOMIC_ACQUIRE);
        if (same && (h >> 4) == ps->key_epoch && (h & 15u) != 0u && !ps_only &&
            ps->skips < kHintRecheck) {
          ++ps->skips;  // (the last verdict of this batch: run_ea or not packed)
          ps = nullptr;
          psl.unlock();
        }
      }
      if (ps) {
        // HCRC_PACKED: the pre-pass checks the batch and cuts its covering
        // range into C equal byte chunks (first[c]); the packed kernel then
        // streams it (crc32c_ps.h), or runs the default pipeline when the
        // pre-pass found the batch not packed
        // (tests, A/Bs, ps_only: the stream-tiled pipeline even where run_ea suits the batch)
        const uint32_t C = static_cast<uint32_t>(chunks_per_group * grid);
        if (++ps->epoch >= (1u << 28)) {  // (the tag's range: start over from a cleared word)
          HCRC_CHECK(hipMemsetAsync(ps->d, 0, lk::kPsMetaWords * 4, st));
          ps->epoch = 1;
        }
        ps->key_base = base;
        ps->key_off = off + pos;
        ps->key_len = len + pos;
        ps->key_n = n;
        ps->key_epoch = ps->epoch;
        ps->skips = 0;
        uint32_t* meta = ps->d;
        uint32_t* first = meta + lk::kPsMetaWords;
        const int pgrid = static_cast<int>(std::max<size_t>(
            1, std::min<size_t>((n + lk::kPsIndexThreads - 1) / lk::kPsIndexThreads,
                                size_t(ctx->num_cu) * 2)));
        hipLaunchKernelGGL(lk::crc32c_ps_index_kernel, dim3(pgrid), dim3(lk::kPsIndexThreads),
                           lk::kPsIndexLds, st, static_cast<const uint8_t*>(base), off + pos,
                           len + pos, static_cast<uint64_t>(n), C, first, meta, ps->epoch,
                           ps_only ? lk::kFlagPsOnly : 0u);
#ifdef WIPDB_HCRC_TEST_HOOKS
        // (test build: the pre-pass's verdict and chunk size, for the tests
        // that check which pipeline a packed batch took; word 0 as the
        // kernel reads it: 0 = this launch's and packed, else its bits)
        HCRC_CHECK(hipMemcpyAsync(g_test_ps_meta, meta, sizeof(g_test_ps_meta),
                                  hipMemcpyDeviceToHost, st));
        HCRC_CHECK(hipStreamSynchronize(st));
        g_test_ps_meta[0] = (g_test_ps_meta[0] >> 4) == ps->epoch ? (g_test_ps_meta[0] & 15u) : ~0u;
        g_test_ps_meta[7] = 0u;
#endif
        hipLaunchKernelGGL(init ? lk::crc32c_lds_packed_kernel<1> : lk::crc32c_lds_packed_kernel<0>,
                           dim3(grid), dim3(lk::kThreads), lk::kLdsBytes, st,
                           static_cast<const uint8_t*>(base), off + pos, len + pos,
                           init ? init + pos : nullptr, out + pos, static_cast<uint64_t>(n),
                           (mask ? lk::kFlagMask : 0u) |
                               (ps_only ? lk::kFlagPsOnly : 0u),
                           ctx->d_image, first, meta, C, ps->epoch, fault,
                           reinterpret_cast<unsigned int*>(ps->d_hint));
        rc = LaunchedLp(st, fault);
        if (rc) return rc;
        continue;
      }
      // HCRC_BALANCE: byte-balanced contiguous workgroup ranges, two small
      // passes over the length column first (only worth it where the spans'
      // sizes vary: the static deal is exact for equal spans)
      const bool bal = (flags & HCRC_BALANCE) != 0 && n >= size_t(64) * grid && grid > 1;
      uint8_t* scratch = nullptr;
      const uint32_t* bounds = nullptr;
      if (bal) {
        const size_t C = std::max<size_t>(1024, (n + 4095) / 4096 + 255) / 256 * 256;
        const uint32_t nb = static_cast<uint32_t>((n + C - 1) / C);
        const size_t bytes = size_t(nb) * 8 + (size_t(grid) + 1) * 4;
        HCRC_CHECK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&scratch), bytes,
                                          ctx->scratch_pool, st));
        uint64_t* sums = reinterpret_cast<uint64_t*>(scratch);
        uint32_t* bd = reinterpret_cast<uint32_t*>(scratch + size_t(nb) * 8);
        hipLaunchKernelGGL(wipdb::util::balance_sums_kernel, dim3(nb), dim3(256), 0, st,
                           len + pos, static_cast<uint64_t>(n), static_cast<uint32_t>(C), sums);
        hipLaunchKernelGGL(wipdb::util::balance_bounds_kernel, dim3(grid - 1), dim3(256), 0, st,
                           len + pos, static_cast<uint64_t>(n), static_cast<uint32_t>(C), sums,
                           nb, static_cast<uint32_t>(grid), bd);
        bounds = bd;
      }
      hipLaunchKernelGGL(init ? lk::crc32c_lds_spans_kernel<1> : lk::crc32c_lds_spans_kernel<0>,
                         dim3(grid), dim3(lk::kThreads),
                         lk::kLdsBytes, st, static_cast<const uint8_t*>(base), off + pos,
                         len + pos, init ? init + pos : nullptr, out + pos,
                         static_cast<uint64_t>(n), mask ? lk::kFlagMask : 0u, ctx->d_image,
                         bounds, fault);
      rc = LaunchedLp(st, fault);
      if (scratch && hipFreeAsync(scratch, st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
    }
    if (rc) return rc;
  }
  return HCRC_OK;
}

// HCRC_PACKED's pre-pass restated for a piece the host holds
// (crc32c_ps.h ps_index: the same promise, the same chunk index): spans
// sorted, not overlapping, gaps < 4 KiB, no 63 starts within 4 KiB, no
// position of a chunk past 2^32 from its first page, and not WAL-like (a run
// of 8 spans under the stream minimum, or 32 of them, among an aligned group
// of 64).  Writes meta words [0] = 1 << 4 (epoch 1; | kPsBad* bits when the
// promise is broken), [1..2] chunk bytes, [3..4] the first span's offset, and
// first[0 .. C] after them.  Returns the kPsBad* bits (0: packed).  On the
// host a piece costs O(n) over descriptors it already touched -- no pre-pass
// launch and no floor.
uint32_t HostPsIndex(const uint64_t* off, const uint32_t* len, size_t n, uint32_t C, uint32_t* ps) {
  uint32_t* meta = ps;
  uint32_t* first = ps + lk::kPsMetaWords;
  for (uint32_t k = 0; k < lk::kPsMetaWords; ++k) meta[k] = 0;
  if (n == 0 || C == 0) return lk::kPsBad;
  const uint64_t lo = off[0], hi = off[n - 1] + len[n - 1];
  const uint64_t range = hi > lo ? hi - lo : 1u;
  uint64_t cb = (range + C - 1u) / C;
  cb = (cb + 4095u) & ~uint64_t(4095);
  if (cb < 4096u) cb = 4096u;
  uint32_t bad = (cb >> 44) ? lk::kPsBad : 0u;
  auto chunk_of = [lo, cb, C](uint64_t a) -> uint64_t {
    if (a < lo) return 0u;
    const uint64_t c = (a - lo) / cb;
    return c < C ? c : uint64_t(C);
  };
  first[0] = 0;
  uint64_t prev_c = 0;
  uint64_t shorts = 0;  // bit j: span 64 g + j of the group is short
  for (size_t i = 0; i < n && bad == 0u; ++i) {
    const uint64_t a = off[i];
    uint64_t c = chunk_of(a);
    if (a < lo || c >= C) {
      bad |= lk::kPsBad;
      break;
    }
    if (i > 0) {
      const uint64_t bp = off[i - 1] + len[i - 1];
      if (a < bp || a - bp >= 4096u) bad |= lk::kPsBad;
    }
    for (uint64_t k = prev_c + 1u; k <= c && i > 0; ++k) first[k] = static_cast<uint32_t>(i);
    prev_c = c;
    if (cb + len[i] + 8192u >= (uint64_t(1) << 32)) bad |= lk::kPsBad;
    if (i + 62 < n) {
      if (off[i + 62] < a) bad |= lk::kPsBad;
      else if (off[i + 62] - a < 4096u) bad |= lk::kPsBadDense;
    }
    if (len[i] < 96u) shorts |= uint64_t(1) << (i & 63u);
    if ((i & 63u) == 63u || i + 1 == n) {
      uint64_t m = shorts;
      if (__builtin_popcountll(m) >= 32) bad |= lk::kPsBadShort;
      m &= m >> 1;
      m &= m >> 2;
      m &= m >> 4;
      if (m) bad |= lk::kPsBadShort;
      shorts = 0;
    }
  }
  if (bad == 0u)
    for (uint64_t k = prev_c + 1u; k <= C; ++k) first[k] = static_cast<uint32_t>(n);
  meta[0] = (1u << 4) | bad;
  meta[1] = static_cast<uint32_t>(cb);
  meta[2] = static_cast<uint32_t>(cb >> 32);
  meta[3] = static_cast<uint32_t>(lo);
  meta[4] = static_cast<uint32_t>(lo >> 32);
  return bad;
}

// Host pieces of at least this many spans take a host-built index when the
// promise holds (WIPDB_PS_MIN_SPANS overrides, as for device batches)
constexpr size_t kHostPackedMinSpans = 4096;
size_t HostPackedMinSpans() {
  static const size_t v = [] {
    const char* e = getenv("WIPDB_PS_MIN_SPANS");
    return e && *e ? static_cast<size_t>(atol(e)) : kHostPackedMinSpans;
  }();
  return v;
}

// The piece's index into the slot's descriptor block (it crosses with the
// descriptors, Slot::SendDesc) when the piece may take the packed kernel: no
// size-class / long-span flag, enough spans, and the promise holds.  Returns
// the index to launch with, or nullptr.
const HostIndex* SlotHostIndex(hcrc_ctx* ctx, Slot& s, const uint64_t* h_off, const uint32_t* h_len,
                               size_t n, int flags, HostIndex* keep) {
  if (flags & (HCRC_SPLIT_SMALL | HCRC_SPLIT_LONG | HCRC_BALANCE)) return nullptr;
  if (n < HostPackedMinSpans() || n <= kAutoLongSpans) return nullptr;
  const uint32_t C = static_cast<uint32_t>(PsChunksPerGroup() * LdsGrid(ctx, n));
  if (C > kPsMaxHostChunks) return nullptr;
  if (HostPsIndex(h_off, h_len, n, C, s.h_ps) != 0u) return nullptr;
#ifdef WIPDB_HCRC_TEST_HOOKS
  for (uint32_t k = 0; k < lk::kPsMetaWords; ++k) g_test_ps_meta[k] = s.h_ps[k];
  g_test_ps_meta[0] = s.h_ps[0] & 15u;
  g_test_ps_meta[7] = 0x484F5354u;  // ("HOST": the index was built on the host)
#endif
  keep->d_ps = s.d_ps;
  keep->C = C;
  return keep;
}

// A host piece of at most kAutoLongSpans spans with one of >= kDevLongSpan
// bytes: the long-span split, as a device batch of that size would take.
// (Spans of >= 256 KiB were already cut into parts on the host,
// BatchHostLong.)  Other pieces pay for no split.
int AutoLongHost(const uint32_t* lengths, size_t n) {
  if (n > kAutoLongSpans) return 0;
  for (size_t i = 0; i < n; ++i)
    if (lengths[i] >= kDevLongSpan) return HCRC_SPLIT_LONG;
  return 0;
}

// Whether a host piece goes through the size classes (HCRC_SPLIT_SMALL) by
// itself: no longer.  Round 2 chose them for pieces of >= 256 short spans;
// on round 3's lane-packed kernel they lose everywhere (same session,
// profiles/r04c_autosplit_ab.log: WAL records, meta blocks, 512 B and 1 KiB
// spans, 4 and 32 MiB batches -- device-resident 2-2.7x slower, zero-copy up
// to 17 % slower, staged within 4 % either way), so the default kernel runs
// every host piece; the classes stay an opt-in flag.
int AutoSplit(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, size_t n) {
  (void)base;
  (void)offsets;
  (void)lengths;
  (void)n;
#ifdef WIPDB_HCRC_TEST_HOOKS
  // the A/B of the choice (scripts/autosplit_ab.py): "1" forces the classes
  if (const char* e = getenv("WIPDB_HCRC_AUTOSPLIT"))
    if (*e == '1') return HCRC_SPLIT_SMALL;
#endif
  return 0;
}

// Persistent helper threads for the pageable -> pinned staging copy (the
// bound of host batches from pageable memory): spawning threads per piece
// cost a visible share of each 32 MiB piece.  One Run at a time uses the
// pool; a concurrent caller (another lane) copies on its own thread instead.
// Never destroyed (no exit-order hazard with other static destructors).
class CopyPool {
 public:
  static CopyPool& Get() {
    static CopyPool* p = new CopyPool;
    return *p;
  }
  // fn(a, b) over [0, n) in parts, the caller running one of them
  void Run(size_t n, const std::function<void(size_t, size_t)>& fn) {
    if (g_forked_child.load(std::memory_order_relaxed)) {  // no helpers after fork()
      fn(0, n);
      return;
    }
    std::unique_lock<std::mutex> run(run_mu_, std::try_to_lock);
    if (!run.owns_lock() || workers_.empty()) {
      fn(0, n);
      return;
    }
    const size_t parts = workers_.size() + 1, per = (n + parts - 1) / parts;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      per_ = per;
      pending_ = workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    fn(0, std::min(n, per));
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  static std::atomic<bool> g_forked_child;
  CopyPool() {
    // a forked child inherits neither the helper threads nor consistent locks
    pthread_atfork(nullptr, nullptr, [] { g_forked_child.store(true); });
    const unsigned hw = std::thread::hardware_concurrency();
    unsigned nt = std::min(7u, hw > 1 ? hw - 1 : 0u);
    // (WIPDB_COPY_THREADS: the helpers' count for A/Bs, at most 31)
    if (const char* e = getenv("WIPDB_COPY_THREADS"))
      if (*e) nt = std::min(31u, static_cast<unsigned>(atoi(e)));
    for (unsigned t = 0; t < nt; ++t) workers_.emplace_back([this, t] { Loop(t + 1); });
    for (auto& w : workers_) w.detach();
  }
  void Loop(size_t part) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(size_t, size_t)>* fn;
      size_t a, b;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        fn = fn_;
        a = std::min(n_, per_ * part);
        b = std::min(n_, a + per_);
      }
      if (a < b) (*fn)(a, b);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(size_t, size_t)>* fn_ = nullptr;
  size_t n_ = 0, per_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};
std::atomic<bool> CopyPool::g_forked_child{false};

// Test hook (fault injection; the test build only, make testlib,
// tests/test_gpu_parity.py): with WIPDB_HCRC_FAIL_PIECE=k in the
// environment, the first host batch that reaches its k-th piece fails there
// with HCRC_ERR_LAUNCH while the previous piece is still in flight -- the
// error path LaneLease must clean up.  Fires once per process.  The product
// library has no hook: the environment cannot change what it does.
bool InjectedPieceFault(size_t piece) {
#ifdef WIPDB_HCRC_TEST_HOOKS
  static const long at = [] {
    const char* e = getenv("WIPDB_HCRC_FAIL_PIECE");
    return e && *e ? atol(e) : -1L;
  }();
  static std::atomic<bool> fired{false};
  return at >= 0 && piece == static_cast<size_t>(at) && !fired.exchange(true);
#else
  (void)piece;
  return false;
#endif
}

// Copy spans [lo, hi) into a slot's pinned buffer, keeping each span's
// address mod 16 (so aligned blocks stay on the aligned fast path and the
// size classes are the caller's).
void PackSpans(Slot& s, const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
               const uint32_t* inits, size_t lo, size_t hi, size_t* used_bytes) {
  size_t cur = 0;
  for (size_t i = lo; i < hi; ++i) {
    const uint8_t* src = base + offsets[i];
    cur = ((cur + 15) & ~size_t(15)) + (reinterpret_cast<uintptr_t>(src) & 15);
    s.h_off[i - lo] = cur;
    s.h_len[i - lo] = lengths[i];
    if (inits) s.h_init[i - lo] = inits[i];
    cur += lengths[i];
  }
  *used_bytes = cur;
  // the byte copy itself, split over the copy pool for big pieces
  const size_t n = hi - lo;
  auto copy = [&](size_t a, size_t b) {
    for (size_t i = a; i < b; ++i) memcpy(s.h_data + s.h_off[i], base + offsets[lo + i], s.h_len[i]);
  };
  if (cur < (size_t(4) << 20) || n < 64) copy(0, n);
  else CopyPool::Get().Run(n, copy);
}

// Whether pinned batches copy their dense pieces with the copy engine
// (WIPDB_HOST_DMA=0: every piece zero-copy; A/Bs only)
bool HostDma() {
  static const bool v = [] {
    const char* e = getenv("WIPDB_HOST_DMA");
    return !(e && *e && atoi(e) == 0);
  }();
  return v;
}

// The copy engine's pieces: at most kDmaBytes of covering range (a slot's
// d_copy), at least kDmaMinBytes -- a smaller batch returns sooner zero-copy
// (one ~2 MiB SST a call: 73 us p50 zero-copy, 83 us copied); the last
// piece of a batch after a copied one has no floor
constexpr size_t kDmaBytes = size_t(128) << 20;
constexpr size_t kDmaMinBytes = size_t(8) << 20;
// zero-copy pieces of at most this many spans skip the descriptor and result
// copies (Slot::DirectLayout)
constexpr size_t kDirectSpans = 4096;

// A dense piece of a pinned batch for the copy engine: spans [i, j) in
// address order inside ONE pinned range whose covering bytes fit cap bytes
// (at the source address mod 256), hold at most an eighth + 64 KiB more than
// the spans and at least kDmaMinBytes, unless it ends the batch after a
// copied piece (tail); [*a, *b) is the range to copy.  Returns j, or i when
// the piece starting at i is not such a piece (it runs zero-copy).
size_t DensePiece(const uint8_t* host_base, const uint64_t* offsets, const uint32_t* lengths,
                  size_t i, size_t count, size_t cap, bool tail, uintptr_t* a, uintptr_t* b) {
  const uintptr_t first = reinterpret_cast<uintptr_t>(host_base + offsets[i]);
  uintptr_t rlo, rhi;
  if (!PinnedRangeOf(first, &rlo, &rhi)) return i;
  const uintptr_t lim = std::min(rhi, first - (first & 255u) + cap);
  uintptr_t hi = first, prev = first;
  uint64_t bytes = 0;
  size_t j = i;
  while (j < count && j - i < kStageSpans) {
    const uintptr_t lo = reinterpret_cast<uintptr_t>(host_base + offsets[j]);
    const uintptr_t end = lo + lengths[j];
    if (lo < prev || end > lim) break;
    prev = lo;
    hi = std::max(hi, end);
    bytes += lengths[j];
    ++j;
  }
  if (j == i || hi - first > bytes + bytes / 8 + (uint64_t(64) << 10)) return i;
  if (hi - first < kDmaMinBytes && !(tail && j == count)) return i;
  // the copy widened to the 256-byte grid inside the range: the copy engine
  // runs unaligned host copies at a fraction of its rate
  *a = std::max(rlo, first & ~uintptr_t(255));
  *b = std::min(rhi, (hi + 255) & ~uintptr_t(255));
  return j;
}

// The lane's copy stream and the slot's copy event, made on first use; false
// when the device cannot give them.
bool CopyStream(Lane* lane, Slot& s) {
  if (!lane->copy && hipStreamCreateWithFlags(&lane->copy, hipStreamNonBlocking) != hipSuccess) {
    lane->copy = nullptr;
    (void)hipGetLastError();
    return false;
  }
  if (!s.copied && hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) != hipSuccess) {
    s.copied = nullptr;
    (void)hipGetLastError();
    return false;
  }
  return true;
}

// The same and the slot's copy buffer, made on first use; false when the
// device cannot give them (nothing half-made is kept).
bool CopyBuffers(Lane* lane, Slot& s) {
  if (!CopyStream(lane, s)) return false;
  if (s.d_copy) return true;
  if (hipMalloc(reinterpret_cast<void**>(&s.d_copy), kDmaBytes) != hipSuccess) {
    s.d_copy = nullptr;
    (void)hipGetLastError();
    return false;
  }
  return true;
}

// Pinned batches: a dense piece (DensePiece) is copied into the slot's
// d_copy by the copy engine -- the PCIe bytes are the covering range once,
// at the copy engine's rate -- on the lane's copy stream, and the kernel
// reads it out of HBM on the lane's stream once the copy's event fires, so
// the next piece's copy runs under this piece's descriptors, kernel and
// results; any other piece runs zero-copy: the kernel reads the spans
// straight out of mapped host memory over PCIe (no device buffer; its read
// windows cross PCIe, so it trails the copy engine on unaligned spans).  The
// descriptors and the results cross through the slots either way.
int BatchZeroCopy(hcrc_ctx* ctx, LaneLease& lane, const uint8_t* dev_base,
                  const uint8_t* host_base, const uint64_t* offsets, const uint32_t* lengths,
                  const uint32_t* inits, uint32_t* out, size_t count, int flags) {
  const hipStream_t st = lane->stream;
  if (const int frc = lane.FaultsBefore()) return frc;
  size_t i = 0, piece = 0;
  int k = 0;
  bool copying = false;
  while (i < count) {
    Slot& s = lane->slots[k];
    int rc = s.Drain();
    if (rc) return rc;
    if (InjectedPieceFault(piece++)) return HCRC_ERR_LAUNCH;
    // (the last piece after a copied one has no floor: its copy queues
    // behind that one's)
    uintptr_t ca = 0, cb = 0;
    size_t j =
        HostDma() ? DensePiece(host_base, offsets, lengths, i, count, kDmaBytes, copying, &ca, &cb)
                  : i;
    // (no device memory or stream for the copy: the piece runs zero-copy)
    if (j > i && !CopyBuffers(lane.get(), s)) j = i;
    const bool dma = j > i;
    copying = dma;
    const size_t n = dma ? j - i : std::min(count - i, kStageSpans);
#ifdef WIPDB_HCRC_TEST_HOOKS
    ++(dma ? g_test_dma_pieces : g_test_zc_pieces);
#endif
    const uint8_t* kbase = dev_base;
    // a small zero-copy piece reads its descriptors and writes its results
    // in pinned memory: its data crosses PCIe anyway, and a copy each way
    // is ~10 us of a one-SST call
    const bool direct = !dma && n <= kDirectSpans;
    if (direct) s.DirectLayout(n);
    else s.Layout(n);
    if (dma) {
      // the covering range at its address mod 256 in the slot
      const uintptr_t at = ca & 255u;
      // (the slot's previous piece is drained: its kernel is done with d_copy;
      // the copy goes out first, the descriptors are written under it)
      HCRC_CHECK(hipMemcpyAsync(s.d_copy + at, reinterpret_cast<const void*>(ca), cb - ca,
                                hipMemcpyHostToDevice, lane->copy));
      HCRC_CHECK(hipEventRecord(s.copied, lane->copy));
      const uintptr_t rebase = ca - at - reinterpret_cast<uintptr_t>(host_base);
      for (size_t q = 0; q < n; ++q) s.h_off[q] = offsets[i + q] - rebase;
      kbase = s.d_copy;
    } else {
      memcpy(s.h_off, offsets + i, n * 8);
    }
    memcpy(s.h_len, lengths + i, n * 4);
    if (inits) memcpy(s.h_init, inits + i, n * 4);
    const int pflags = flags | AutoSplit(host_base, offsets + i, lengths + i, n) |
                       AutoLongHost(lengths + i, n);
    HostIndex hi;
    const HostIndex* hidx = SlotHostIndex(ctx, s, s.h_off, s.h_len, n, pflags, &hi);
    if (!direct)
      HCRC_CHECK(s.SendDesc(n, inits != nullptr, hidx ? lk::kPsMetaWords + hidx->C + 1 : 0, st));
    // the kernel waits for the piece's copy (its descriptors went ahead)
    if (dma) HCRC_CHECK(hipStreamWaitEvent(st, s.copied, 0));
    rc = LaunchSpans(ctx, kbase, s.d_off, s.d_len, inits ? s.d_init : nullptr,
                     direct ? s.hd_out : s.d_out, n, pflags, st, AutoLong::kNo, lane.FaultWord(),
                     hidx);
    if (rc) return rc;
    if (!direct) HCRC_CHECK(hipMemcpyAsync(s.h_out, s.d_out, n * 4, hipMemcpyDeviceToHost, st));
    HCRC_CHECK(hipEventRecord(s.done, st));
    s.user_out = out + i;
    s.n_out = n;
    i += n;
    k ^= 1;
  }
  for (Slot& s : lane->slots) {
    const int rc = s.Drain();
    if (rc) return rc;
  }
  return lane.CheckFaults();
}

int BatchHost(hcrc_ctx* ctx, const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
              const uint32_t* inits, uint32_t* out, size_t count, int flags) {
  LaneLease lane(ctx);
  int rc = lane.Staging();
  if (rc) return rc;
  if (const uint8_t* dev = MappedSpans(base, offsets, lengths, count))
    return BatchZeroCopy(ctx, lane, dev, base, offsets, lengths, inits, out, count, flags);
  const hipStream_t st = lane->stream;
  if (const int frc = lane.FaultsBefore()) return frc;
  size_t i = 0, piece = 0;
  int k = 0;
  while (i < count) {
    Slot& s = lane->slots[k];
    rc = s.Drain();
    if (rc) return rc;
    if (InjectedPieceFault(piece++)) return HCRC_ERR_LAUNCH;
    // piece = spans [i, j) fitting the slot (a single larger span grows it)
    size_t bytes = 0, j = i;
    while (j < count && j - i < kStageSpans) {
      const size_t b = size_t(lengths[j]) + 32;
      if (j > i && bytes + b > s.cap_bytes) break;
      bytes += b;
      ++j;
    }
    rc = s.Grow(bytes);
    if (rc) return rc;
    size_t used = 0;
    const size_t n = j - i;
    s.Layout(n);
    PackSpans(s, base, offsets, lengths, inits, i, j, &used);
    // a big piece's bytes go on the lane's copy stream, so the next piece's
    // copy runs under this piece's kernel and results (a small one stays on
    // the lane's stream: no cross-stream wait in a one-SST call)
    const bool ahead = used >= kDmaMinBytes && CopyStream(lane.get(), s);
    HCRC_CHECK(hipMemcpyAsync(s.d_data, s.h_data, used, hipMemcpyHostToDevice,
                              ahead ? lane->copy : st));
    if (ahead) HCRC_CHECK(hipEventRecord(s.copied, lane->copy));
    // (the staged layout is the slot's own: spans in order, 16-byte-aligned
    // cursor, gaps < 32 bytes -- packed whatever the caller's layout was)
    const int pflags = flags | AutoSplit(base, offsets + i, lengths + i, n) |
                       AutoLongHost(lengths + i, n);
    HostIndex hi;
    const HostIndex* hidx = SlotHostIndex(ctx, s, s.h_off, s.h_len, n, pflags, &hi);
    HCRC_CHECK(s.SendDesc(n, inits != nullptr, hidx ? lk::kPsMetaWords + hidx->C + 1 : 0, st));
    if (ahead) HCRC_CHECK(hipStreamWaitEvent(st, s.copied, 0));
    rc = LaunchSpans(ctx, s.d_data, s.d_off, s.d_len, inits ? s.d_init : nullptr, s.d_out, n,
                     pflags, st, AutoLong::kNo, lane.FaultWord(), hidx);
    if (rc) return rc;
    HCRC_CHECK(hipMemcpyAsync(s.h_out, s.d_out, n * 4, hipMemcpyDeviceToHost, st));
    HCRC_CHECK(hipEventRecord(s.done, st));
    s.user_out = out + i;
    s.n_out = n;
    i = j;
    k ^= 1;
  }
  for (Slot& s : lane->slots) {
    rc = s.Drain();
    if (rc) return rc;
  }
  return lane.CheckFaults();
}

// Long spans of a host batch (SURVEY 5's long-context analogue): a span of
// at least kLongSpan bytes runs as parts of kPartBytes (the first part takes
// the remainder), so its segments run on many waves at once instead of one
// chained wave; the parts' CRCs are combined on the host by linearity
// (gf2_crc32c.h): part 0 runs with the span's init, the others from init ~0
// (so they return ~feed(0, part)), and
//   feed(~init, span) = Horner over r = shift(r, kPartBytes) ^ feed(0, part j),
// the same identity crc32c_3way's CombineCRC uses (kv/src/util/crc32c.cc:640-657).
constexpr uint64_t kPartBytes = uint64_t(64) << 10;
constexpr uint64_t kLongSpan = 4 * kPartBytes;

struct PartShift {
  uint32_t t[4][256];
  PartShift() { wipdb::gf2::BuildShiftTable(kPartBytes, t); }
  uint32_t operator()(uint32_t r) const {
    return t[0][r & 0xffu] ^ t[1][(r >> 8) & 0xffu] ^ t[2][(r >> 16) & 0xffu] ^ t[3][r >> 24];
  }
};

int BatchHostLong(hcrc_ctx* ctx, const uint8_t* base, const uint64_t* offsets,
                  const uint32_t* lengths, const uint32_t* inits, uint32_t* out, size_t count,
                  int flags) {
  size_t parts = 0;
  bool any = false;
  for (size_t i = 0; i < count; ++i) {
    if (lengths[i] >= kLongSpan) {
      any = true;
      parts += (lengths[i] + kPartBytes - 1) / kPartBytes;
    } else {
      ++parts;
    }
  }
  if (!any) return BatchHost(ctx, base, offsets, lengths, inits, out, count, flags);
  std::vector<uint64_t> po(parts);
  std::vector<uint32_t> pl(parts), pi(parts), pr(parts);
  size_t k = 0;
  for (size_t i = 0; i < count; ++i) {
    const uint32_t init = inits ? inits[i] : 0u;
    const uint64_t n = lengths[i];
    if (n < kLongSpan) {
      po[k] = offsets[i];
      pl[k] = static_cast<uint32_t>(n);
      pi[k++] = init;
      continue;
    }
    const uint64_t m = (n + kPartBytes - 1) / kPartBytes;
    const uint64_t first = n - (m - 1) * kPartBytes;  // 1 .. kPartBytes
    po[k] = offsets[i];
    pl[k] = static_cast<uint32_t>(first);
    pi[k++] = init;
    for (uint64_t j = 1; j < m; ++j) {
      po[k] = offsets[i] + first + (j - 1) * kPartBytes;
      pl[k] = static_cast<uint32_t>(kPartBytes);
      pi[k++] = ~0u;
    }
  }
  const int rc = BatchHost(ctx, base, po.data(), pl.data(), pi.data(), pr.data(), parts,
                           flags & ~HCRC_MASK_OUTPUT);
  if (rc) return rc;
  static const PartShift shift;
  const bool mask = (flags & HCRC_MASK_OUTPUT) != 0;
  k = 0;
  for (size_t i = 0; i < count; ++i) {
    uint32_t v;
    if (lengths[i] < kLongSpan) {
      v = pr[k++];
    } else {
      const uint64_t m = (uint64_t(lengths[i]) + kPartBytes - 1) / kPartBytes;
      uint32_t r = ~pr[k++];
      for (uint64_t j = 1; j < m; ++j) r = shift(r) ^ ~pr[k++];
      v = ~r;
    }
    out[i] = mask ? wipdb::gf2::Mask(v) : v;
  }
  return HCRC_OK;
}

std::mutex g_ctx_mu;
std::map<int, hcrc_ctx*>& SharedCtxs() {
  static auto* m = new std::map<int, hcrc_ctx*>;
  return *m;
}

// One context per device shared by hcrc_batch_multi's threads (contexts are
// thread-safe: each synchronous call leases its own lane).
int SharedCtx(int device, hcrc_ctx** out) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto& m = SharedCtxs();
  auto it = m.find(device);
  if (it != m.end()) {
    *out = it->second;
    return HCRC_OK;
  }
  const int rc = hcrc_ctx_create(device, out);
  if (rc) return rc;
  m[device] = *out;
  return HCRC_OK;
}

}  // namespace

extern "C" {

int hcrc_abi_version(void) { return HCRC_ABI_VERSION; }

#ifdef WIPDB_HCRC_TEST_HOOKS
// Test build only (not in the header): the forced fault on (1) or off (0)
// for the launches that follow, whatever WIPDB_HCRC_FORCE_FAULT says.
__attribute__((visibility("default"))) void hcrc_test_force_fault(int on) {
  g_force_fault.store(on ? 1 : 0);
}
// The pre-pass words of the last HCRC_PACKED launch (n <= 8 copied).
// the host-built packed index of a piece (HostPsIndex), for the CPU test
// that checks it against a restatement of the device pre-pass
__attribute__((visibility("default"))) uint32_t hcrc_test_host_ps_index(const uint64_t* off,
                                                                        const uint32_t* len,
                                                                        size_t n, uint32_t C,
                                                                        uint32_t* ps) {
  return HostPsIndex(off, len, n, C, ps);
}
// The copy engine's piece choice (DensePiece) over a host range entered as
// pinned without pinning it (hcrc_test_fake_pinned_range; bytes 0 removes
// it), for the CPU test of the piece rules: returns j, and [a, b) as
// offsets from host_base.
__attribute__((visibility("default"))) void hcrc_test_fake_pinned_range(void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_host_mu);
  if (bytes) HostRanges()[reinterpret_cast<uintptr_t>(p)] = {bytes, static_cast<uint8_t*>(p)};
  else HostRanges().erase(reinterpret_cast<uintptr_t>(p));
}
__attribute__((visibility("default"))) size_t hcrc_test_dense_piece(const uint8_t* host_base,
                                                                   const uint64_t* offsets,
                                                                   const uint32_t* lengths,
                                                                   size_t i, size_t count, int tail,
                                                                   uint64_t* ab) {
  uintptr_t a = 0, b = 0;
  const size_t j = DensePiece(host_base, offsets, lengths, i, count, kDmaBytes, tail != 0, &a, &b);
  ab[0] = a - reinterpret_cast<uintptr_t>(host_base);
  ab[1] = b - reinterpret_cast<uintptr_t>(host_base);
  return j;
}
__attribute__((visibility("default"))) void hcrc_test_clear_packed_meta() {
  for (uint32_t k = 0; k < lk::kPsMetaWords; ++k) g_test_ps_meta[k] = 0xFFFFFFFFu;
}
__attribute__((visibility("default"))) void hcrc_test_packed_meta(uint32_t* out, int n) {
  for (int i = 0; i < n && i < static_cast<int>(lk::kPsMetaWords); ++i) out[i] = g_test_ps_meta[i];
}
// pinned-batch pieces since the last call: out[0] copy engine, out[1] zero-copy
__attribute__((visibility("default"))) void hcrc_test_pinned_pieces(uint64_t* out) {
  out[0] = g_test_dma_pieces.exchange(0);
  out[1] = g_test_zc_pieces.exchange(0);
}
#endif

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
    case HCRC_ERR_BOUNDS: return "span outside the base buffer";
    case HCRC_ERR_KERNEL: return "a kernel reported an internal fault (outputs incomplete)";
    default: return "unknown error";
  }
}

int hcrc_ctx_shared(int device, hcrc_ctx** out_ctx) {
  if (!out_ctx) return HCRC_ERR_INVALID;
  *out_ctx = nullptr;
  return SharedCtx(device, out_ctx);
}

int hcrc_ctx_create(int device, hcrc_ctx** out_ctx) {
  if (!out_ctx) return HCRC_ERR_INVALID;
  *out_ctx = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return HCRC_ERR_NO_DEVICE;
  DeviceGuard dg(device);
  if (!dg.ok()) return HCRC_ERR_HIP;
  std::unique_ptr<hcrc_ctx> ctx(new hcrc_ctx);
  ctx->device = device;
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
  const void* kernels[] = {
      reinterpret_cast<const void*>(lk::crc32c_lds_spans_kernel<0>),
      reinterpret_cast<const void*>(lk::crc32c_lds_spans_kernel<1>),
      reinterpret_cast<const void*>(lk::crc32c_lds_strided_kernel),
      reinterpret_cast<const void*>(lk::crc32c_lds_verify_kernel),
      reinterpret_cast<const void*>(lk::crc32c_lds_packed_kernel<0>),
      reinterpret_cast<const void*>(lk::crc32c_lds_packed_kernel<1>),
      reinterpret_cast<const void*>(lk::crc32c_dma_ceiling_kernel),
      reinterpret_cast<const void*>(lk::crc32c_lds_list_kernel<1, 0>),
      reinterpret_cast<const void*>(lk::crc32c_lds_list_kernel<2, 0>),
      reinterpret_cast<const void*>(lk::crc32c_lds_list_kernel<4, 0>),
      reinterpret_cast<const void*>(lk::crc32c_lds_list_kernel<1, 1>),
      reinterpret_cast<const void*>(lk::crc32c_lds_list_kernel<2, 1>),
      reinterpret_cast<const void*>(lk::crc32c_lds_list_kernel<4, 1>),
  };
  for (const void* k : kernels)
    HCRC_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lk::kLdsBytes));
  HCRC_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ctx->fault_words), 4 * kFaultWords,
                           hipHostMallocCoherent | hipHostMallocMapped));
  memset(ctx->fault_words, 0, 4 * kFaultWords);
  HCRC_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_fault_words),
                                     ctx->fault_words, 0));
  {
    std::vector<uint32_t> img(lk::kImageBytes / 4);
    lk::BuildLdsImage(img.data());
    HCRC_CHECK(hipMalloc(reinterpret_cast<void**>(&ctx->d_image), lk::kImageBytes));
    HCRC_CHECK(hipMemcpy(ctx->d_image, img.data(), lk::kImageBytes, hipMemcpyHostToDevice));
  }
  *out_ctx = ctx.release();
  return HCRC_OK;
}

int hcrc_ctx_destroy(hcrc_ctx* ctx) {
  if (!ctx) return HCRC_ERR_INVALID;
  {
    // a shared context (hcrc_ctx_shared) lives until the process ends: other
    // threads (ExtendBatch, hcrc_batch_multi) may hold it at any moment
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    for (const auto& kv : SharedCtxs())
      if (kv.second == ctx) return HCRC_ERR_INVALID;
  }
  delete ctx;
  return HCRC_OK;
}

hcrc_ctx::~hcrc_ctx() {
  if (device < 0) return;
  DeviceGuard dg(device);
  for (auto& lane : lanes) {
    if (lane->stream) (void)hipStreamSynchronize(lane->stream);
    if (lane->copy) (void)hipStreamSynchronize(lane->copy);
    for (Slot& s : lane->slots) s.Free();
    if (lane->stream) (void)hipStreamDestroy(lane->stream);
    if (lane->copy) (void)hipStreamDestroy(lane->copy);
  }
  if (stream) (void)hipStreamSynchronize(stream);
  if (d_image) (void)hipFree(d_image);
  if (stream) (void)hipStreamDestroy(stream);
  if (scratch_pool) {
    (void)hipDeviceSynchronize();
    (void)hipMemPoolDestroy(scratch_pool);
  }
  if (fault_words) (void)hipHostFree(fault_words);
  for (auto& kv : ps_scratch) {
    if (kv.second->d) (void)hipFree(kv.second->d);
    if (kv.second->h_hint) (void)hipHostFree(kv.second->h_hint);
  }
}

void* hcrc_ctx_stream(hcrc_ctx* ctx) { return ctx ? ctx->stream : nullptr; }
int hcrc_ctx_device(hcrc_ctx* ctx) { return ctx ? ctx->device : -1; }

int hcrc_batch(hcrc_ctx* ctx, const void* base, const uint64_t* offsets, const uint32_t* lengths,
               const uint32_t* init_crcs, uint32_t* out_crcs, size_t count, int flags) {
  if (!ctx || (count && (!base || !offsets || !lengths || !out_crcs))) return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_DEVICE_PTRS | HCRC_MASK_OUTPUT | HCRC_SPLIT_SMALL | HCRC_SPLIT_LONG |
                HCRC_BALANCE | HCRC_PACKED))
    return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  if (flags & HCRC_DEVICE_PTRS) {
    LaneLease lane(ctx);
    int rc = lane.Stream();
    if (rc == HCRC_OK) rc = lane.FaultsBefore();
    if (rc == HCRC_OK)
      rc = LaunchSpans(ctx, base, offsets, lengths, init_crcs, out_crcs, count, flags,
                       lane->stream, AutoLong::kDevice, lane.FaultWord());
    if (rc) return rc;
    return lane.CheckFaults();
  }
  // host pointers: HCRC_BALANCE is dropped (the header: the copy or the
  // zero-copy reads bound these batches, not the kernel's balance)
  return BatchHostLong(ctx, static_cast<const uint8_t*>(base), offsets, lengths, init_crcs,
                       out_crcs, count, flags & ~HCRC_BALANCE);
}

int hcrc_batch_async(hcrc_ctx* ctx, const void* d_base, const uint64_t* d_offsets,
                     const uint32_t* d_lengths, const uint32_t* d_init_crcs, uint32_t* d_out_crcs,
                     size_t count, int flags, void* stream) {
  if (!ctx || !(flags & HCRC_DEVICE_PTRS)) return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_DEVICE_PTRS | HCRC_MASK_OUTPUT | HCRC_SPLIT_SMALL | HCRC_SPLIT_LONG |
                HCRC_BALANCE | HCRC_PACKED))
    return HCRC_ERR_INVALID;
  if (count && (!d_base || !d_offsets || !d_lengths || !d_out_crcs)) return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  return LaunchSpans(ctx, d_base, d_offsets, d_lengths, d_init_crcs, d_out_crcs, count, flags, st,
                     AutoLong::kDevice, StreamFaultWord(ctx, st));
}

int hcrc_batch_strided_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride, uint32_t length,
                             uint32_t init_crc, uint32_t* d_out_crcs, size_t count, int flags,
                             void* stream) {
  if (!ctx || !(flags & HCRC_DEVICE_PTRS)) return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_DEVICE_PTRS | HCRC_MASK_OUTPUT)) return HCRC_ERR_INVALID;
  if (count && (!d_base || !d_out_crcs)) return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  unsigned int* const fault = StreamFaultWord(ctx, st);
  for (size_t pos = 0; pos < count; pos += kMaxLaunchSpans) {
    const size_t n = std::min(count - pos, kMaxLaunchSpans);
    hipLaunchKernelGGL(lk::crc32c_lds_strided_kernel, dim3(LdsGrid(ctx, n)), dim3(lk::kThreads),
                       lk::kLdsBytes, st, static_cast<const uint8_t*>(d_base) + pos * stride,
                       stride, length, init_crc, d_out_crcs + pos, static_cast<uint64_t>(n),
                       static_cast<uint32_t>(flags & HCRC_MASK_OUTPUT), ctx->d_image, fault);
    const int rc = LaunchedLp(st, fault);
    if (rc) return rc;
  }
  return HCRC_OK;
}

int hcrc_verify_async_ex(hcrc_ctx* ctx, const void* d_base, const uint64_t* d_offsets,
                         const uint32_t* d_lengths, uint8_t* d_status, size_t count, int flags,
                         void* stream) {
  if (!ctx) return HCRC_ERR_INVALID;
  if (flags & ~HCRC_SPLIT_SMALL) return HCRC_ERR_INVALID;
  if (count && (!d_base || !d_offsets || !d_lengths || !d_status)) return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const bool split = (flags & HCRC_SPLIT_SMALL) != 0;
  const size_t piece_max = split ? size_t(lk::kMaxListSpans) : kMaxLaunchSpans;
  unsigned int* const fault = split ? nullptr : StreamFaultWord(ctx, st);
  for (size_t pos = 0; pos < count; pos += piece_max) {
    const size_t n = std::min(count - pos, piece_max);
    int rc;
    if (split) {
      rc = LaunchClasses(ctx, static_cast<const uint8_t*>(d_base), d_offsets + pos,
                         d_lengths + pos, nullptr, d_status + pos, n, 1, false, st);
    } else {
      hipLaunchKernelGGL(lk::crc32c_lds_verify_kernel, dim3(LdsGrid(ctx, n)), dim3(lk::kThreads),
                         lk::kLdsBytes, st, static_cast<const uint8_t*>(d_base), d_offsets + pos,
                         d_lengths + pos, d_status + pos, static_cast<uint64_t>(n), ctx->d_image,
                         fault);
      rc = LaunchedLp(st, fault);
    }
    if (rc) return rc;
  }
  return HCRC_OK;
}

int hcrc_verify_async(hcrc_ctx* ctx, const void* d_base, const uint64_t* d_offsets,
                      const uint32_t* d_lengths, uint8_t* d_status, size_t count, void* stream) {
  return hcrc_verify_async_ex(ctx, d_base, d_offsets, d_lengths, d_status, count, 0, stream);
}

int hcrc_readstream_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride, uint32_t length,
                          uint32_t* d_out, size_t count, void* stream) {
  if (!ctx || (count && (!d_base || !d_out)) || (length & 15)) return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  hipLaunchKernelGGL(wipdb::util::readstream_kernel, dim3(ctx->num_cu), dim3(1024), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(d_base), stride,
                     length, d_out, static_cast<uint64_t>(count));
  return Launched();
}

int hcrc_dma_ceiling_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride, uint32_t length,
                           uint32_t* d_out, size_t count, void* stream) {
  if (!ctx || (count && (!d_base || !d_out)) || length != 4096u || stride < 4096u ||
      count > kMaxLaunchSpans)
    return HCRC_ERR_INVALID;
  if (count == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  hipLaunchKernelGGL(lk::crc32c_dma_ceiling_kernel, dim3(LdsGrid(ctx, count)), dim3(lk::kThreads),
                     lk::kLdsBytes, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(d_base), stride, d_out,
                     static_cast<uint64_t>(count), ctx->d_image);
  return Launched();
}

int hcrc_check_spans_async(hcrc_ctx* ctx, uint64_t base_bytes, const uint64_t* d_offsets,
                           const uint32_t* d_lengths, uint32_t extra, size_t count,
                           uint64_t* d_result, void* stream) {
  if (!ctx || !d_result || (count && (!d_offsets || !d_lengths))) return HCRC_ERR_INVALID;
  HCRC_DEVICE(ctx);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  // result words {0, ~0}: stream-ordered memsets, no host source in flight
  HCRC_CHECK(hipMemsetAsync(d_result, 0, 8, st));
  HCRC_CHECK(hipMemsetAsync(d_result + 1, 0xff, 8, st));
  if (count == 0) return HCRC_OK;
  const int grid =
      static_cast<int>(std::min<uint64_t>((count + 255) / 256, uint64_t(ctx->num_cu) * 8));
  hipLaunchKernelGGL(wipdb::util::check_spans_kernel, dim3(grid), dim3(256), 0, st, d_offsets,
                     d_lengths, static_cast<uint64_t>(count), base_bytes, extra,
                     reinterpret_cast<unsigned long long*>(d_result));
  return Launched();
}

int hcrc_check_spans(hcrc_ctx* ctx, uint64_t base_bytes, const uint64_t* d_offsets,
                     const uint32_t* d_lengths, uint32_t extra, size_t count,
                     uint64_t* first_bad) {
  if (!ctx) return HCRC_ERR_INVALID;
  HCRC_DEVICE(ctx);
  uint64_t* d_res = nullptr;
  const hipStream_t st = ctx->stream;
  HCRC_CHECK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&d_res), 16, ctx->scratch_pool, st));
  uint64_t res[2] = {0, ~uint64_t(0)};
  int rc = hcrc_check_spans_async(ctx, base_bytes, d_offsets, d_lengths, extra, count, d_res, st);
  if (rc == HCRC_OK &&
      hipMemcpyAsync(res, d_res, sizeof(res), hipMemcpyDeviceToHost, st) != hipSuccess)
    rc = HCRC_ERR_HIP;
  if (hipFreeAsync(d_res, st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
  if (hipStreamSynchronize(st) != hipSuccess && rc == HCRC_OK) rc = HCRC_ERR_HIP;
  if (rc) return rc;
  if (first_bad) *first_bad = res[1];
  return res[0] ? HCRC_ERR_BOUNDS : HCRC_OK;
}

int hcrc_fill_splitmix64_async(hcrc_ctx* ctx, void* d_dst, uint64_t nbytes, uint64_t seed,
                               uint64_t first_word, void* stream) {
  if (!ctx || (nbytes && !d_dst) || (nbytes & 7) || (reinterpret_cast<uintptr_t>(d_dst) & 7))
    return HCRC_ERR_INVALID;
  if (nbytes == 0) return HCRC_OK;
  HCRC_DEVICE(ctx);
  const uint64_t nwords = nbytes / 8;
  const int grid =
      static_cast<int>(std::min<uint64_t>((nwords + 255) / 256, uint64_t(ctx->num_cu) * 16));
  hipLaunchKernelGGL(wipdb::util::fill_splitmix64_kernel, dim3(grid), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<uint64_t*>(d_dst), nwords,
                     first_word, seed);
  return Launched();
}

int hcrc_ctx_check(hcrc_ctx* ctx) {
  if (!ctx) return HCRC_ERR_INVALID;
  // every caller stream's word (and the shared word 0), read and cleared:
  // the caller synchronised the streams it launched on, so their launches
  // are complete and their stores visible (coherent host memory)
  std::lock_guard<std::mutex> lk(ctx->faults_mu);
  unsigned int any = __atomic_exchange_n(ctx->fault_words, 0u, __ATOMIC_SEQ_CST);
  for (const auto& kv : ctx->stream_words)
    any |= __atomic_exchange_n(ctx->fault_words + kv.second, 0u, __ATOMIC_SEQ_CST);
  return any ? HCRC_ERR_KERNEL : HCRC_OK;
}

int hcrc_sync(hcrc_ctx* ctx, void* stream) {
  if (!ctx) return HCRC_ERR_INVALID;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  {
    HCRC_DEVICE(ctx);
    HCRC_CHECK(hipStreamSynchronize(st));
  }
  // this stream's word only (plus the shared word 0 of streams past the
  // table), read and cleared: another caller's fault stays with its stream
  std::lock_guard<std::mutex> lk(ctx->faults_mu);
  unsigned int any = 0;
  const auto it = ctx->stream_words.find(st);
  if (it != ctx->stream_words.end())
    any = __atomic_exchange_n(ctx->fault_words + it->second, 0u, __ATOMIC_SEQ_CST);
  else if (ctx->stream_words.size() >= kStreamFaultWords)
    any = __atomic_exchange_n(ctx->fault_words, 0u, __ATOMIC_SEQ_CST);
  return any ? HCRC_ERR_KERNEL : HCRC_OK;
}

int hcrc_stream_forget(hcrc_ctx* ctx, void* stream) {
  if (!ctx) return HCRC_ERR_INVALID;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  unsigned int any = 0;
  {
    std::lock_guard<std::mutex> lk(ctx->faults_mu);
    const auto it = ctx->stream_words.find(st);
    if (it != ctx->stream_words.end()) {
      any = __atomic_exchange_n(ctx->fault_words + it->second, 0u, __ATOMIC_SEQ_CST);
      ctx->free_stream_words.push_back(it->second);
      ctx->stream_words.erase(it);
    }
  }
  std::unique_ptr<hcrc_ctx::PsScratch> ps;
  {
    std::lock_guard<std::mutex> lk(ctx->ps_mu);
    const auto it = ctx->ps_scratch.find(st);
    if (it != ctx->ps_scratch.end()) {
      ps = std::move(it->second);
      ctx->ps_scratch.erase(it);
    }
  }
  if (ps && ps->d) {
    HCRC_DEVICE(ctx);
    // (the caller's launches on the stream are complete; hipFree waits for
    // the device anyway)
    if (hipFree(ps->d) != hipSuccess) return HCRC_ERR_HIP;
    if (ps->h_hint && hipHostFree(ps->h_hint) != hipSuccess) return HCRC_ERR_HIP;
  }
  return any ? HCRC_ERR_KERNEL : HCRC_OK;
}

int hcrc_batch_multi_ex(const int* devices, int ndev, const void* base, const uint64_t* offsets,
                        const uint32_t* lengths, const uint32_t* init_crcs, uint32_t* out_crcs,
                        size_t count, int flags, int* shard_rc) {
  if (!devices || ndev <= 0 || (flags & HCRC_DEVICE_PTRS)) return HCRC_ERR_INVALID;
  if (flags & ~(HCRC_MASK_OUTPUT | HCRC_SPLIT_SMALL)) return HCRC_ERR_INVALID;
  if (count && (!base || !offsets || !lengths || !out_crcs)) return HCRC_ERR_INVALID;
  if (shard_rc)
    for (int k = 0; k < ndev; ++k) shard_rc[k] = HCRC_OK;
  if (count == 0) return HCRC_OK;
  // byte-balanced contiguous shards (weight = length + 64 per span)
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
        rc = hcrc_batch(ctx, base, offsets + lo, lengths + lo, init_crcs ? init_crcs + lo : nullptr,
                        out_crcs + lo, hi - lo, flags);
      rcs[k] = rc;
    });
  }
  for (auto& th : pool) th.join();
  int first = HCRC_OK;
  for (int k = 0; k < ndev; ++k) {
    if (shard_rc) shard_rc[k] = rcs[k];
    if (first == HCRC_OK) first = rcs[k];
  }
  return first;
}

int hcrc_batch_multi(const int* devices, int ndev, const void* base, const uint64_t* offsets,
                     const uint32_t* lengths, const uint32_t* init_crcs, uint32_t* out_crcs,
                     size_t count, int flags) {
  return hcrc_batch_multi_ex(devices, ndev, base, offsets, lengths, init_crcs, out_crcs, count,
                             flags, nullptr);
}

int hcrc_host_alloc(size_t bytes, void** out_ptr) {
  if (!out_ptr || !bytes) return HCRC_ERR_INVALID;
  // portable + mapped: every device of a multi-GPU batch reads it zero-copy
  HCRC_CHECK(hipHostMalloc(out_ptr, bytes, hipHostMallocPortable | hipHostMallocMapped));
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, *out_ptr, 0) != hipSuccess) dev = *out_ptr;
  std::lock_guard<std::mutex> lk(g_host_mu);
  HostRanges()[reinterpret_cast<uintptr_t>(*out_ptr)] = {bytes, static_cast<uint8_t*>(dev)};
  return HCRC_OK;
}

int hcrc_host_free(void* ptr) {
  if (!ptr) return HCRC_ERR_INVALID;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    HostRanges().erase(reinterpret_cast<uintptr_t>(ptr));
  }
  HCRC_CHECK(hipHostFree(ptr));
  return HCRC_OK;
}

int hcrc_host_register(void* ptr, size_t bytes) {
  if (!ptr || !bytes) return HCRC_ERR_INVALID;
  HCRC_CHECK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess) dev = ptr;
  std::lock_guard<std::mutex> lk(g_host_mu);
  HostRanges()[reinterpret_cast<uintptr_t>(ptr)] = {bytes, static_cast<uint8_t*>(dev)};
  return HCRC_OK;
}

int hcrc_host_unregister(void* ptr) {
  if (!ptr) return HCRC_ERR_INVALID;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    HostRanges().erase(reinterpret_cast<uintptr_t>(ptr));
  }
  HCRC_CHECK(hipHostUnregister(ptr));
  return HCRC_OK;
}

}  // extern "C"
