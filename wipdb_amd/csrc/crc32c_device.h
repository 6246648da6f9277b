// crc32c_device.h -- constants and table layout shared by the HIP kernels
// (crc32c_kernels.hip) and the host side that builds/uploads the tables
// (hcrc_api.cc).  See DESIGN.md "Data layout".
#pragma once
#include <stdint.h>

namespace wipdb {
namespace dev {

constexpr int kWaves = 16;               // waves per workgroup (1 WG per CU)
constexpr int kThreads = kWaves * 64;    // 1024 threads
constexpr uint32_t kNumShift = 8;        // shift tables for 16*2^j bytes, j<8
constexpr uint32_t kFlagMask = 0x2;      // == HCRC_MASK_OUTPUT
constexpr int kChains = 4;               // independent CRC chains per lane

// LDS map (bytes).
//  [0, 32 KiB)   shift tables: 8 x [4 byte positions][256] u32 -- below
//                64 KiB so a compile-time table base fits the 16-bit
//                ds_read offset field.
//  [32 KiB, +1 KiB) inv_top (256 u32), then head0 (16 u32).
//  [64 KiB, 128 KiB) slicing-by-2 tables, 32 replicas: entry (b, u, lane)
//                at 64 KiB + (b << 8) | (u << 7) | (lane & 31) << 2,
//                u=0: T1, u=1: T0.  Lane l only ever reads replica l&31 ->
//                bank l&31: no conflicts for any data.  The address is one
//                v_perm_b32: [lane byte, table byte, 0x01, 0x00].
constexpr uint32_t kLdsShift = 0;
constexpr uint32_t kLdsInvTop = kLdsShift + kNumShift * 4096;
constexpr uint32_t kLdsHead0 = kLdsInvTop + 1024;
constexpr uint32_t kLdsMain = 65536;
constexpr uint32_t kLdsBytes = kLdsMain + 65536;  // 128 KiB

// Device-global copy of the tables (built on the host by gf2::BuildTables /
// gf2::BuildShiftTable, uploaded once per context).
struct DevTables {
  uint32_t t0[256];                 // byte table (reference table0_)
  uint32_t t1[256];                 // byte followed by one zero byte
  uint32_t shift[kNumShift][4][256];  // x^(8*16*2^j) multiply tables
  uint32_t inv_top[256];            // un-feed helper (see gf2_crc32c.h)
  uint32_t head0[16];               // ~0 * x^(-8h)
};

}  // namespace dev
}  // namespace wipdb
