// tests/cpp/lk_emu.h -- host SIMT emulation of the kernels' hardware
// primitives (wipdb_amd/csrc/crc32c_prim.h), for tests/cpp/test_lp_emu.cc:
// the LDS-staged kernels' OWN source (crc32c_lds.hip) compiled for the host,
// one std::thread per lane, 1024 per workgroup.  Cross-lane operations
// (DPP, ballot, readlane, ds_bpermute, readfirstlane) exchange through a
// per-wave buffer between two barriers; LDS is a per-workgroup array (the
// queue's atomics are host atomics); global_load_lds copies the 16 bytes at
// issue and checks that they lie in the range the test registered.  The
// hand-counted waits are no-ops (the copy is done at issue).  Test
// infrastructure only: the library never includes this file.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(x)
#define __restrict__ __restrict

namespace wipdb {
namespace lk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t g_u32;
typedef uint8_t g_u8;

namespace emu {

// A reusable barrier of n threads: an arrival count and a generation the
// waiters sleep on (futex-backed std::atomic wait: no mutex convoy when the
// last arrival wakes the other 63 lanes of a wave -- the emulation spends
// most of its time here)
struct Barrier {
  std::atomic<int> count{0};
  std::atomic<uint32_t> gen{0};
  int n;
  explicit Barrier(int n_) : n(n_) {}
  void wait() {
    const uint32_t g = gen.load(std::memory_order_acquire);
    if (count.fetch_add(1, std::memory_order_acq_rel) + 1 == n) {
      count.store(0, std::memory_order_relaxed);
      gen.fetch_add(1, std::memory_order_release);
      gen.notify_all();
    } else {
      for (int i = 0; i < 128; ++i) {
        if (gen.load(std::memory_order_acquire) != g) return;
        std::this_thread::yield();
      }
      while (gen.load(std::memory_order_acquire) == g) gen.wait(g, std::memory_order_acquire);
    }
  }
};
struct Wave {
  Barrier bar{64};
  uint64_t buf[64];
};
struct Group {
  std::vector<uint8_t> lds;
  Barrier bar{kThreads};
  Wave waves[kWaves];
  Group() : lds(163840, 0xCD) {}
};
// the DMA source range the test allows, and the first violation
inline uint64_t g_src_lo = 0, g_src_hi = ~uint64_t(0);
inline std::atomic<uint64_t> g_bad_src{0};
inline std::atomic<uint64_t> g_dma_chunks{0};

inline thread_local uint32_t t_tid = 0, t_bid = 0, t_grid = 1;
inline thread_local Group* t_group = nullptr;

inline uint32_t lane() { return t_tid & 63u; }
inline Wave& wave() { return t_group->waves[t_tid >> 6]; }
template <class F>
inline uint64_t xchg(uint64_t v, F f) {
  Wave& w = wave();
  w.buf[lane()] = v;
  w.bar.wait();
  const uint64_t r = f(w.buf);
  w.bar.wait();
  return r;
}
inline void copy16(uint32_t dst, uint64_t src) {
  if (src < g_src_lo || src + 16u > g_src_hi) {
    uint64_t z = 0;
    g_bad_src.compare_exchange_strong(z, src | 1u);
    return;
  }
  g_dma_chunks.fetch_add(1, std::memory_order_relaxed);
  memcpy(t_group->lds.data() + dst, reinterpret_cast<const void*>(src), 16);
}

// Runs kernel() on `grid` workgroups of kThreads lane threads (one workgroup at
// a time, as many as the device has CUs would run at once).
template <class F>
inline void launch_blocks(uint32_t grid, const std::vector<uint32_t>& blocks, F kernel) {
  for (uint32_t b : blocks) {
    Group g;
    std::vector<std::thread> th;
    th.reserve(kThreads);
    for (uint32_t t = 0; t < static_cast<uint32_t>(kThreads); ++t)
      th.emplace_back([&, t] {
        t_tid = t;
        t_bid = b;
        t_grid = grid;
        t_group = &g;
        kernel();
      });
    for (auto& x : th) x.join();
  }
}
template <class F>
inline void launch(uint32_t grid, F kernel) {
  for (uint32_t b = 0; b < grid; ++b) {
    Group g;
    std::vector<std::thread> th;
    th.reserve(kThreads);
    for (uint32_t t = 0; t < static_cast<uint32_t>(kThreads); ++t)
      th.emplace_back([&, t] {
        t_tid = t;
        t_bid = b;
        t_grid = grid;
        t_group = &g;
        kernel();
      });
    for (auto& x : th) x.join();
  }
}

}  // namespace emu

// ---- LDS ----
inline uint8_t* lds_base() { return emu::t_group->lds.data(); }
inline uint32_t lds_ld(uint32_t a) {
  uint32_t v;
  memcpy(&v, lds_base() + a, 4);
  return v;
}
inline u32x4 lds_ld4(uint32_t a) {
  uint32_t v[4];
  memcpy(v, lds_base() + a, 16);
  return u32x4{v[0], v[1], v[2], v[3]};
}
inline uint32_t* lds_w(uint32_t a) { return reinterpret_cast<uint32_t*>(lds_base() + a); }
inline uint32_t lds_add(uint32_t a, uint32_t v) { return __atomic_fetch_add(lds_w(a), v, __ATOMIC_SEQ_CST); }
inline uint32_t lds_cas(uint32_t a, uint32_t cmp, uint32_t v) {
  uint32_t c = cmp;
  __atomic_compare_exchange_n(lds_w(a), &c, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return c;
}
inline void lds_st(uint32_t a, uint32_t v) { memcpy(lds_base() + a, &v, 4); }
inline void lds_st4(uint32_t a, const u32x4& v) {
  if (a & 15u) abort();  // (ds_write_b128 needs 16-byte alignment here)
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  memcpy(lds_base() + a, w, 16);
}
inline uint32_t lds_ld_sync(uint32_t a) { return __atomic_load_n(lds_w(a), __ATOMIC_SEQ_CST); }
inline void lds_st_sync(uint32_t a, uint32_t v) { __atomic_store_n(lds_w(a), v, __ATOMIC_SEQ_CST); }
// the wave's LDS accesses are complete: the lanes meet (a lane thread must
// not overwrite a slot another lane has yet to read)
inline void lgkm_wait() { emu::wave().bar.wait(); }
inline void compiler_barrier() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
inline void lds_order() { emu::wave().bar.wait(); }
template <class T>
inline void loads_landed(T&) {}
inline uint32_t vzero() { return 0u; }

inline void global_or(uint32_t* a, uint32_t v) { __atomic_fetch_or(a, v, __ATOMIC_SEQ_CST); }
inline void global_max(uint32_t* a, uint32_t v) {
  uint32_t c = __atomic_load_n(a, __ATOMIC_SEQ_CST);
  while (c < v && !__atomic_compare_exchange_n(a, &c, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
}

// ---- faults ----
// the fault bits of the launches (the device counts faulting waves instead)
namespace emu {
inline std::atomic<uint32_t> g_faults{0};
}
inline void report_fault(unsigned int* word, uint32_t bits) {
  if (emu::lane() == 0u) {
    emu::g_faults.fetch_or(bits);
    if (word) __atomic_store_n(word, 1u, __ATOMIC_SEQ_CST);
  }
}
// queue record g_hide_marker's marker reads as 0 (never written): forces the
// popper's timeout (with a small WIPDB_LP_SPIN)
namespace emu {
inline std::atomic<uint32_t> g_hide_marker{~0u};
inline std::atomic<uint32_t> g_spin{1u << 22};  // WIPDB_LP_SPIN of the emulation
}
inline uint32_t queue_marker(uint32_t v, uint32_t idx) { return idx == emu::g_hide_marker.load() ? 0u : v; }
// the launches' pipeline choices (bit 0 run_ea, bit 1 run_lp); g_force_pipe
// >= 0 overrides the choice (1 = run_ea, 0 = run_lp)
namespace emu {
inline std::atomic<uint32_t> g_pipes{0};
inline std::atomic<int> g_force_pipe{-1};
}
inline bool pipeline_marker(bool ea) {
  const int f = emu::g_force_pipe.load();
  if (f >= 0) ea = f != 0;
  emu::g_pipes.fetch_or(ea ? 1u : 2u);
  return ea;
}

// ---- lanes ----
inline uint32_t lane_tid() { return emu::t_tid; }
inline uint32_t group_id() { return emu::t_bid; }
inline uint32_t group_count() { return emu::t_grid; }
inline void wg_sync() { emu::t_group->bar.wait(); }
inline void lk_sleep() { std::this_thread::yield(); }
template <int P>
inline void lk_prio() {}
inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
inline uint32_t vperm(uint32_t a, uint32_t b, uint32_t sel) {
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t s = (sel >> (8 * i)) & 0xffu;
    uint32_t byte;
    if (s < 4u) byte = (b >> (8 * s)) & 0xffu;
    else if (s < 8u) byte = (a >> (8 * (s - 4))) & 0xffu;
    else if (s == 0x0cu) byte = 0u;
    else abort();
    r |= byte << (8 * i);
  }
  return r;
}
template <int CTRL>
inline uint32_t dpp(uint32_t v) {
  return static_cast<uint32_t>(emu::xchg(v, [](const uint64_t* b) -> uint64_t {
    const int l = static_cast<int>(emu::lane());
    int src;
    if (CTRL < 0x100) {  // quad_perm
      src = (l & ~3) + ((CTRL >> (2 * (l & 3))) & 3);
    } else if (CTRL >= 0x101 && CTRL <= 0x10F) {  // row_shl: lane i reads i + n
      const int n = CTRL - 0x100;
      src = (l & 15) + n < 16 ? l + n : -1;
    } else if (CTRL >= 0x111 && CTRL <= 0x11F) {  // row_shr: lane i reads i - n
      const int n = CTRL - 0x110;
      src = (l & 15) >= n ? l - n : -1;
    } else {
      abort();
    }
    return src < 0 ? 0u : static_cast<uint32_t>(b[src]);
  }));
}
inline uint32_t bcast15(uint32_t v) {
  return static_cast<uint32_t>(emu::xchg(v, [](const uint64_t* b) -> uint64_t {
    const int l = static_cast<int>(emu::lane()), row = l >> 4;
    return (row == 1 || row == 3) ? static_cast<uint32_t>(b[16 * row - 1]) : 0u;
  }));
}
inline uint32_t bcast31(uint32_t v) {
  return static_cast<uint32_t>(emu::xchg(v, [](const uint64_t* b) -> uint64_t {
    const int row = static_cast<int>(emu::lane()) >> 4;
    return row >= 2 ? static_cast<uint32_t>(b[31]) : 0u;
  }));
}
inline uint32_t uni(uint32_t v) {
  return static_cast<uint32_t>(emu::xchg(v, [](const uint64_t* b) { return b[0]; }));
}
inline uint64_t uni64(uint64_t v) {
  return emu::xchg(v, [](const uint64_t* b) { return b[0]; });
}
inline uint32_t uni_act(uint32_t v) { return v; }  // (under a lane branch: no exchange)
inline uint64_t uni_act64(uint64_t v) { return v; }
inline uint32_t rdlane(uint32_t v, uint32_t k) {
  return static_cast<uint32_t>(emu::xchg(v, [k](const uint64_t* b) { return b[k & 63u]; }));
}
inline uint32_t wrlane(uint32_t old, uint32_t v, uint32_t k) { return emu::lane() == (k & 63u) ? v : old; }
inline uint64_t ballot(bool p) {
  return emu::xchg(p ? 1u : 0u, [](const uint64_t* b) {
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i) m |= (b[i] & 1u) << i;
    return m;
  });
}
inline uint32_t vsel(uint64_t m, uint32_t a, uint32_t b) {
  return ((m >> emu::lane()) & 1u) ? a : b;
}
inline uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t sh) {
  return static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | lo) >> (sh & 31u));
}
inline uint32_t mbcnt_lo(uint32_t m, uint32_t acc) {
  const uint32_t l = emu::lane();
  return acc + static_cast<uint32_t>(__builtin_popcount(l < 32u ? (m & ((1u << l) - 1u)) : m));
}
inline uint32_t mbcnt_hi(uint32_t m, uint32_t acc) {
  const uint32_t l = emu::lane();
  return acc + (l < 32u ? 0u : static_cast<uint32_t>(__builtin_popcount(m & ((1u << (l - 32u)) - 1u))));
}
inline uint32_t fperm(uint32_t v, uint32_t dst) {
  const uint64_t pk = static_cast<uint64_t>(v) | (static_cast<uint64_t>(dst & 63u) << 32);
  return static_cast<uint32_t>(emu::xchg(pk, [](const uint64_t* b) -> uint64_t {
    const uint32_t me = emu::lane();
    uint32_t r = 0;  // (the highest pusher wins; none: 0)
    for (uint32_t j = 0; j < 64; ++j)
      if ((b[j] >> 32) == me) r = static_cast<uint32_t>(b[j]);
    return r;
  }));
}
inline uint32_t bperm_raw(uint32_t v, uint32_t ln) {
  return static_cast<uint32_t>(emu::xchg(v, [ln](const uint64_t* b) { return b[ln & 63u]; }));
}

// ---- DMA: the LDS destination is M0 + 16 * lane ----
inline void dma4(uint64_t base, uint32_t slot, uint32_t o0, uint32_t o1, uint32_t o2, uint32_t o3) {
  const uint32_t l = emu::lane();
  emu::copy16(slot + 16u * l, base + o0);
  emu::copy16(slot + 1024u + 16u * l, base + o1);
  emu::copy16(slot + 2048u + 16u * l, base + o2);
  emu::copy16(slot + 3072u + 16u * l, base + o3);
}
inline void dma2(uint64_t base, uint32_t slot, uint32_t o0, uint32_t o1) {
  const uint32_t l = emu::lane();
  emu::copy16(slot + 16u * l, base + o0);
  emu::copy16(slot + 1024u + 16u * l, base + o1);
}
inline void dma1(uint64_t base, uint32_t dst, uint32_t off) {
  memcpy(lds_base() + dst + 16u * emu::lane(), reinterpret_cast<const void*>(base + off), 16);
}
inline void dma1nt(uint64_t base, uint32_t dst, uint32_t off) {
  emu::copy16(dst + 16u * emu::lane(), base + off);
}
inline void dma1v(uint64_t addr, uint32_t dst) { emu::copy16(dst + 16u * emu::lane(), addr); }
// the wave's DMAs have landed: the lanes meet (each copied its chunks at issue)
template <int N>
inline void wait_vm() {
  emu::wave().bar.wait();
}

}  // namespace lk
}  // namespace wipdb
