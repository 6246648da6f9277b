// crc32c_device.h -- constants and table layout shared by the HIP kernels
// (crc32c_kernels.hip) and the host side that builds/uploads the tables
// (hcrc_api.cc).  See DESIGN.md "Data layout".
#pragma once
#include <stdint.h>

namespace wipdb {
namespace dev {

#ifndef WIPDB_WAVES
#define WIPDB_WAVES 16
#endif
constexpr int kWaves = WIPDB_WAVES;      // waves per workgroup (1 WG per CU)
constexpr int kThreads = kWaves * 64;    // 1024 threads
constexpr uint32_t kFlagMask = 0x2;      // == HCRC_MASK_OUTPUT
// spans kernel: leave spans of at most kSmallMax bytes to the small-span
// kernel (HCRC_SPLIT_SMALL, crc32c_small.inc)
constexpr uint32_t kFlagSkipSmall = 0x4;
constexpr uint32_t kSmallMax = 1024;
// spans kernel: a span whose rest after its first 4 KiB segment is at most
// kSmallMax bytes stops there (its unmasked partial CRC goes to out[i]) and
// the small-span kernel finishes it (SplitRemainder below)
constexpr uint32_t kFlagSplitRem = 0x8;
// small-span list entries that continue a span from out[id] (remainders)
constexpr uint32_t kSmallIdRem = 0x80000000u;
// small-span kernel, read-side verify: compare with the stored trailer
// (LE32 right after the span) and write a status byte instead of a CRC
constexpr uint32_t kFlagVerify = 0x10;

// The remainder rule, shared by the spans kernel's cursor and the partition
// kernel: a span of n bytes starting at address a is cut after its first
// segment (4096 - a % 16 bytes) when what follows is 16..kSmallMax bytes.
__host__ __device__ constexpr uint32_t SplitRemainder(uint64_t a, uint32_t n) {
  return (n > kSmallMax && n > 4096u - static_cast<uint32_t>(a & 15u) + 15u &&
          n - (4096u - static_cast<uint32_t>(a & 15u)) <= kSmallMax)
             ? 4096u - static_cast<uint32_t>(a & 15u)
             : 0u;
}

// Compacted descriptors of a batch's small spans (written by
// crc32c_partition_kernel, read by crc32c_small_kernel); count is a
// device counter.
struct SmallList {
  uint64_t* off;
  uint32_t* len;
  uint32_t* init;
  uint32_t* id;  // the span's index in the batch (its output slot)
  uint32_t* count;
};

// Spans in flight per wave: the wave is split into kGroups lane groups of
// kGroupLanes lanes; each group CRCs its own span, kChunksPerLane 16-byte
// chunks per lane, so one segment (one load group) is kGroupLanes *
// kChunksPerLane = 256 chunks = 4 KiB per group.
constexpr int kGroups = 2;
constexpr int kGroupLanes = 64 / kGroups;          // 32
constexpr int kChunksPerLane = 256 / kGroupLanes;  // 8
constexpr int kSpansPerWG = kWaves * kGroups;   // spans a workgroup starts at once

// Shift tables: multiply by x^(8 * 16 * 2^j) for j < kNumShift (16 B .. 2 KiB)
// in device memory; a kernel keeps the kLdsShiftTables of them it uses
// (j = log2(chunks per chain) + 0..5) in LDS.
constexpr uint32_t kNumShift = 8;
constexpr uint32_t kLdsShiftTables = 6;

// LDS map (bytes), 160 KiB = the whole CU:
//  [0, 24 KiB)    shift tables: 6 x [4 byte positions][256] u32 -- below
//                 64 KiB so a compile-time table base fits the 16-bit
//                 ds_read offset field.
//  [24 KiB, +1 KiB) inv_top (256 u32), then head0 (16 u32), then the
//                 workgroup's work counter (one u32).
//  [32 KiB, 160 KiB) slicing-by-4 tables T0..T3, 32 replicas: entry
//                 (t, b, lane) at 32 KiB + (t >> 1) * 64 KiB + b * 256 +
//                 (t & 1) * 128 + (lane & 31) * 4.  Lane l only ever reads
//                 replica l & 31 -> bank l & 31: no conflicts for any data.
//                 The address minus 32 KiB is one v_perm_b32 of
//                 [lane byte | table bit, data byte, table half, 0]; the
//                 32 KiB rides in the ds_read offset field.
constexpr uint32_t kLdsShift = 0;
constexpr uint32_t kLdsInvTop = kLdsShift + kLdsShiftTables * 4096;   // 24 KiB
constexpr uint32_t kLdsHead0 = kLdsInvTop + 1024;
constexpr uint32_t kLdsWork = kLdsHead0 + 64;  // the workgroup's work counter (u32)
constexpr uint32_t kLdsMain = 32768;
constexpr uint32_t kLdsBytes = kLdsMain + 4 * 32768;            // 160 KiB

// Device-global copy of the tables (built on the host by gf2::BuildTables /
// gf2::BuildShiftTable, uploaded once per context).
struct DevTables {
  uint32_t t[4][256];                 // t[k][b]: byte b followed by k zero bytes
  uint32_t shift[kNumShift][4][256];  // x^(8*16*2^j) multiply tables
  uint32_t inv_top[256];              // un-feed helper (see gf2_crc32c.h)
  uint32_t head0[16];                 // ~0 * x^(-8h)
};

}  // namespace dev
}  // namespace wipdb
