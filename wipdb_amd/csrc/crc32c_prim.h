// crc32c_prim.h -- the gfx950 hardware primitives the LDS-staged CRC32C
// kernels are written in (crc32c_dev.h, crc32c_lds.hip): LDS access and
// atomics, cross-lane operations (DPP, ballot, readlane, ds_bpermute),
// global_load_lds DMA and the hand-counted waits.  tests/cpp/lk_emu.h
// defines the same functions on the host (one thread per lane), so the
// kernels' own source runs there for the CPU test suite (tests/cpp/
// test_lp_emu.cc); nothing else differs between the two builds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wipdb {
namespace lk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t l_u32;
typedef __attribute__((address_space(3))) uint32_t l_u32w;
typedef __attribute__((address_space(3))) const u32x4 l_u32x4;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint8_t g_u8;

// ---- LDS (byte addresses) ----
__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {
  return *reinterpret_cast<l_u32*>(static_cast<uintptr_t>(a));
}
__device__ __forceinline__ u32x4 lds_ld4(uint32_t a) {
  return *reinterpret_cast<l_u32x4*>(static_cast<uintptr_t>(a));
}
__device__ __forceinline__ l_u32w* lds_p(uint32_t a) {
  return reinterpret_cast<l_u32w*>(static_cast<uintptr_t>(a));
}
__device__ __forceinline__ uint32_t lds_add(uint32_t a, uint32_t v) {
  return __atomic_fetch_add(lds_p(a), v, __ATOMIC_RELAXED);
}
__device__ __forceinline__ uint32_t lds_cas(uint32_t a, uint32_t cmp, uint32_t v) {
  uint32_t c = cmp;
  __atomic_compare_exchange_n(lds_p(a), &c, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
  return c;  // the old value
}
// a plain LDS store (the wave's own data; ordered by program order)
__device__ __forceinline__ void lds_st(uint32_t a, uint32_t v) { *lds_p(a) = v; }
// a 16-byte store (a 16-byte aligned address: ds_write_b128)
__device__ __forceinline__ void lds_st4(uint32_t a, const u32x4& v) {
  *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(static_cast<uintptr_t>(a)) = v;
}
// uncached (another wave may write it)
__device__ __forceinline__ uint32_t lds_ld_sync(uint32_t a) {
  return __atomic_load_n(lds_p(a), __ATOMIC_RELAXED);
}
__device__ __forceinline__ void lds_st_sync(uint32_t a, uint32_t v) {
  __atomic_store_n(lds_p(a), v, __ATOMIC_RELAXED);
}
// every LDS access of this wave has completed (and none moves across)
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void compiler_barrier() { asm volatile("" ::: "memory"); }
// LDS writes of some lanes, then reads of the same words by other lanes of
// the wave: the wave's DS instructions execute in order, so program order is
// enough here (the host emulation, a thread per lane, meets at a barrier)
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }
// v was loaded from global memory and that load is known to be complete
// (a wait on the DMA issued after it): an asm use makes the compiler place
// its own wait for the load here, where it costs nothing, and not at a later
// register copy -- where it would also wait for a DMA issued in between.
template <class T>
__device__ __forceinline__ void loads_landed(T& v) { asm volatile("" : "+v"(v)); }
// 0, but lane-varying to the compiler: a load from a uniform address made
// a vector load (its wait is a vmcnt one, ordered with the DMA, not an lgkmcnt
// one that every later LDS access would also wait for)
__device__ __forceinline__ uint32_t vzero() { return __builtin_amdgcn_mbcnt_lo(0u, 0u); }

// a |= v in global memory (agent scope; the pre-pass's verdict word)
__device__ __forceinline__ void global_or(uint32_t* a, uint32_t v) {
  __hip_atomic_fetch_or(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a = max(a, v) in global memory (agent scope; the epoch-tagged verdict)
__device__ __forceinline__ void global_max(uint32_t* a, uint32_t v) {
  __hip_atomic_fetch_max(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- faults ----
// A queue record's marker as read (the host emulation can hide one to force
// the timeout path; here the identity).
__device__ __forceinline__ uint32_t queue_marker(uint32_t v, uint32_t) { return v; }
// the pipeline a launch's waves chose (run_ea if true): identity here; the
// host emulation records it and can force either one
__device__ __forceinline__ bool pipeline_marker(bool ea) { return ea; }

// ---- lanes ----
__device__ __forceinline__ uint32_t lane_tid() { return threadIdx.x; }
__device__ __forceinline__ uint32_t group_id() { return blockIdx.x; }
__device__ __forceinline__ uint32_t group_count() { return gridDim.x; }
__device__ __forceinline__ void wg_sync() { __syncthreads(); }
__device__ __forceinline__ void lk_sleep() { __builtin_amdgcn_s_sleep(1); }
// wave issue priority (s_setprio): the stretch from a slot's arrival to the
// next DMA's issue runs above the other waves' compute
template <int P>
__device__ __forceinline__ void lk_prio() { __builtin_amdgcn_s_setprio(P); }
// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t vperm(uint32_t a, uint32_t b, uint32_t sel) {
  return __builtin_amdgcn_perm(a, b, sel);
}
// DPP move (lanes without a source read 0)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xF, 0xF, true));
}
// DPP row broadcasts: bcast15 gives rows 1 and 3 lane 15 of the row before
// (rows 0 and 2: 0), bcast31 gives rows 2 and 3 lane 31 (rows 0 and 1: 0) --
// the last two steps of a wave scan after the row_shr steps
__device__ __forceinline__ uint32_t bcast15(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xA, 0xF, false));
}
__device__ __forceinline__ uint32_t bcast31(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xC, 0xF, false));
}
// uniform value of the wave (all lanes active)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (static_cast<uint64_t>(uni(static_cast<uint32_t>(v >> 32))) << 32) |
         uni(static_cast<uint32_t>(v));
}
// a value the active lanes agree on, said to be uniform (any exec mask)
__device__ __forceinline__ uint32_t uni_act(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni_act64(uint64_t v) {
  return (static_cast<uint64_t>(uni_act(static_cast<uint32_t>(v >> 32))) << 32) |
         uni_act(static_cast<uint32_t>(v));
}
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t k) {
  return __builtin_amdgcn_readlane(v, k);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// v_writelane: lane k (uniform) takes the uniform value v, the others keep old
__device__ __forceinline__ uint32_t wrlane(uint32_t old, uint32_t v, uint32_t k) {
  uint32_t r = old;
  // (the lane select through M0: one SGPR operand per VALU on gfx9)
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(r) : "s"(v), "{m0}"(k));
  return r;
}
// Per-lane select by a wave mask: m's bit of the lane ? a : b, one
// v_cndmask_b32 with the mask in an SGPR pair (hipcc lowered some per-lane ?:
// chains of the batch path into exec-masked branches)
__device__ __forceinline__ uint32_t vsel(uint64_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
  return r;
}
// The low word of (hi:lo) >> (sh % 32) (v_alignbit_b32)
__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbit(hi, lo, sh);
}
__device__ __forceinline__ uint32_t mbcnt_lo(uint32_t m, uint32_t acc) {
  return __builtin_amdgcn_mbcnt_lo(m, acc);
}
__device__ __forceinline__ uint32_t mbcnt_hi(uint32_t m, uint32_t acc) {
  return __builtin_amdgcn_mbcnt_hi(m, acc);
}
// ds_permute_b32 (a push): lane `dst` receives v.  Every lane active and the
// dst a permutation of the lanes (gfx950: a lane that two lanes push to keeps
// the higher one's value; one that none pushes to reads 0)
__device__ __forceinline__ uint32_t fperm(uint32_t v, uint32_t dst) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_permute(static_cast<int>(dst << 2),
                                                           static_cast<int>(v)));
}
__device__ __forceinline__ uint32_t bperm_raw(uint32_t v, uint32_t lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(lane << 2),
                                                            static_cast<int>(v)));
}

// ---------------------------------------------------------------------------
// DMA.  The LDS destination of global_load_lds is M0 + 16 * lane (lane-
// linear); the source address is per lane (SGPR base + VGPR offset).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dma4(uint64_t base, uint32_t slot, uint32_t o0, uint32_t o1,
                                     uint32_t o2, uint32_t o3) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %6 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %6 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %6 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %4, %6 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(o0), "v"(o1), "v"(o2), "v"(o3), "s"(slot), "s"(base)
      : "memory", "scc");
}

__device__ __forceinline__ void dma1(uint64_t base, uint32_t dst, uint32_t off) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(dst), "s"(base)
      : "memory");
}

__device__ __forceinline__ void dma2(uint64_t base, uint32_t slot, uint32_t o0, uint32_t o1) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %4 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %4 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(o0), "v"(o1), "s"(slot), "s"(base)
      : "memory", "scc");
}

__device__ __forceinline__ void dma1nt(uint64_t base, uint32_t dst, uint32_t off) {
  uint32_t keep;
  // (callers' values are uniform; say so, so they stay in SGPRs under a lane branch)
  dst = uni_act(dst);
  base = uni_act64(base);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(dst), "s"(base)
      : "memory");
}

// One DMA with per-lane 64-bit source addresses (the lanes of one
// instruction may serve different spans).
__device__ __forceinline__ void dma1v(uint64_t addr, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(addr), "s"(dst)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
}


}  // namespace lk
}  // namespace wipdb
