// crc32c_lds.h -- LDS layout of the LDS-staged CRC32C kernels
// (crc32c_lds.hip) and the host builder of the table image they load.
// Shared by the device code and hcrc_api.cc.  DESIGN.md section 3.
//
// One 1024-thread workgroup (16 waves) per CU owns all 160 KiB of LDS:
//
//   [0, 32 KiB)     fold level-2 tables, 256 rows of 128 B: row b holds
//                   entry (c, p) at (4c + p) * 4 = shift(b << 8p, 512c bytes)
//                   for c = 1..7; the c = 0 column (bytes 0..15 of each row,
//                   an identity shift nobody looks up) holds the misc words.
//   [32, 96 KiB)    main region, 256 rows of 256 B:
//                   bytes [0, 128): slicing-by-4 tables, slot t (0..3) x
//                   replica r (0..7) at 32t + 4r = T[3 - t][b] (the table of
//                   byte position t of a word);
//                   bytes [128, 256): fold level-1 tables, entry (a, p) at
//                   128 + (4a + p) * 4 = shift(b << 8p, 64a bytes), a = 1..7;
//                   the a = 0 column (bytes 128..143, an identity shift
//                   nobody looks up) of rows 16w .. 16w + 15 holds wave w's
//                   16-byte aux pieces: the tail chunks and trailer chunks
//                   of its segments, DMA'd in with the segment.
//   [96, 160 KiB)   16 wave slots of 4 KiB: the segment being DMA'd in.
//
// Bank rule (ds_read_b32: lanes 0-31 and 32-63 are serviced separately,
// bank = (address / 4) mod 32).  In lookup instruction j a lane reads the
// table slot t = (j + q) & 3, q = (lane >> 3) & 3, replica r = lane & 7:
// the 32 lanes of a half hit banks 8t + r -- all different, for any data.
// The level-1 fold reads column 4a + t with a = 7 - (lane & 7), the
// level-2 fold (lanes 8k only) column 4c + t: distinct banks again.
// Each lookup address is ONE v_perm_b32 of (lane constant, data word,
// per-lane selector): [const byte j, data byte t, 0, 0] = (byte << 8) | const.
#pragma once
#include <stdint.h>

#include "gf2_crc32c.h"

#if defined(__HIPCC__)
#define WIPDB_LK_HD __host__ __device__
#else
#define WIPDB_LK_HD
#endif

namespace wipdb {
namespace lk {

#ifndef WIPDB_LP_WAVES
#define WIPDB_LP_WAVES 16
#endif
constexpr int kWaves = WIPDB_LP_WAVES;  // waves per workgroup (one workgroup per CU)
constexpr int kThreads = kWaves * 64;
constexpr uint32_t kLdsL2 = 0;
constexpr uint32_t kLdsMain = 32768;
constexpr uint32_t kLdsSlots = 98304;
constexpr uint32_t kSlotBytes = 4096;
constexpr uint32_t kLdsBytes = kLdsSlots + kWaves * kSlotBytes;  // 160 KiB
constexpr uint32_t kImageBytes = kLdsSlots;                    // tables + misc
constexpr uint32_t kSegChunks = 256;                           // 16-B chunks per segment

// aux piece k (< 16) of wave w: 16 bytes in the a = 0 column of main row 16w + k
WIPDB_LK_HD constexpr uint32_t AuxAddr(uint32_t w, uint32_t k) {
  return kLdsMain + (16u * w + k) * 256u + 128u;
}
constexpr uint32_t kAuxTail = 0;   // + g (g < 8): group g's tail chunk
constexpr uint32_t kAuxNext = 8;   // + g: the chunk after it (verify trailers)

// misc word i (i < 1024) lives in the c = 0 column of level-2 row i / 4
WIPDB_LK_HD constexpr uint32_t MiscAddr(uint32_t i) {
  return (i >> 2) * 128u + (i & 3u) * 4u;
}
constexpr uint32_t kMiscInvTop = 0;    // 256 words: inv_top[v] (gf2::Tables)
constexpr uint32_t kMiscHead0 = 256;   // 16 words: ~0 * x^(-8h)
constexpr uint32_t kMiscUnit = 272;    // the workgroup's unit counter
constexpr uint32_t kMiscQHead = 273;   // the long-span queue's head / tail (run_lp)
constexpr uint32_t kMiscQTail = 274;
constexpr uint32_t kMiscDesks = 275;   // desks grabbed, not sorted yet (run_lp)
constexpr uint32_t kMiscIdle = 276;    // waves out of work, waiting for shared long spans
constexpr uint32_t kMiscHeld = 277;    // long spans held by a wave, not taken or shared yet
constexpr uint32_t kMiscQRes = 278;    // queue records pushed and not yet freed (<= kQSlots)
constexpr uint32_t kMiscFault = 279;   // kFault* bits of the workgroup (run_lp)
constexpr uint32_t kMiscFaultWord = 280;  // 2 words: the launch's fault word (run_lp)
constexpr uint32_t kMiscPsProgress = 512;  // 16 words: run_ps, wave w's pages done
constexpr uint32_t kMiscQInit = 576;   // 256 words: the init_crc of queue record k
constexpr uint32_t kMiscBytes = 1024 * 4;

// run_lp (the lane-packed spans / strided / verify kernels):
//   * the workgroup's long-span queue: 256 records of 16 bytes in the a = 0
//     column of the main rows (bytes 128..143 of row k; the list kernels
//     keep their aux pieces there instead): {a_lo, a_hi, n, span + 1}, a
//     last word of 0 = a free slot; record k's init_crc in misc word
//     kMiscQInit + k;
//   * wave w's aux chunk of a segment tail: the c = 0 column of level-2 row
//     128 + w (misc words 512 .. 575; run_ps, never in the same launch,
//     keeps its progress words in 512 .. 527).
constexpr uint32_t kQSlots = 256;
WIPDB_LK_HD constexpr uint32_t QRecAddr(uint32_t k) {
  return kLdsMain + (k & (kQSlots - 1u)) * 256u + 128u;
}
WIPDB_LK_HD constexpr uint32_t SegAuxAddr(uint32_t w) { return kLdsL2 + (128u + w) * 128u; }

// Flags of a launch (the HCRC_MASK_OUTPUT value is shared with the C-ABI).
constexpr uint32_t kFlagMask = 0x2;
// the packed kernel: run_ps even where run_ea suits the batch (tests, A/Bs)
constexpr uint32_t kFlagPsOnly = 0x200;
// Fault bits a launch ORs into its error word (a span was left uncomputed;
// the host returns HCRC_ERR_KERNEL): a queue record whose producer never
// wrote it, a queue slot never freed for its next record.
constexpr uint32_t kFaultQueuePop = 0x1;
constexpr uint32_t kFaultQueueSlot = 0x2;
// run_ps: a desk that could not advance (never in a batch its pre-pass
// passed: at most 63 spans meet a window)
constexpr uint32_t kFaultPsDesk = 0x4;

// HCRC_PACKED (crc32c_ps.h): the meta words of a packed launch (device,
// zeroed by the host, written by the pre-pass): [0] nonzero = the batch is
// not packed (kPsBad* bits); [1..2] chunk bytes (u64); [3..4] the first
// span's start offset (u64).  The chunk index first[C + 1] follows them.
constexpr uint32_t kPsMetaWords = 8;
constexpr uint32_t kPsBad = 1u, kPsBadDense = 2u;
// run_ps computes spans shorter than its stream minimum byte by byte from
// memory; a run of 8 of them, or 32 among a step's 64 spans (WAL records),
// sends the batch to the lane-packed pipeline instead
constexpr uint32_t kPsBadShort = 4u;
// not indexed: the batch suits run_ea (pick_ea), which the packed kernel takes
// without reading the index -- the pre-pass stops after its sample
constexpr uint32_t kPsEa = 8u;
// the pre-pass kernel's workgroup (16 waves: one verdict atomic per 1024
// threads) and its LDS (a word per wave)
constexpr uint32_t kPsIndexThreads = 1024;
constexpr uint32_t kPsIndexLds = kPsIndexThreads / 64u * 4u;
// steps of 64 spans a wave loads at once (memory-level parallelism)
constexpr uint32_t kPsIndexSteps = 4;

// Size classes (HCRC_SPLIT_SMALL).  A span of n bytes at address a covers
// f = (a % 16 + n) / 16 full chunks of its 16-byte grid.  Class 4 (16-lane
// groups, 4 spans per wave iteration): f <= 64; class 2 (32-lane groups):
// f <= 128; class 1: the rest, on the end-aligned pipeline of the spans
// kernel (table blocks as a main segment + a batched front piece).
constexpr uint32_t kClass4Chunks = 64;
constexpr uint32_t kClass2Chunks = 128;
constexpr uint64_t kMaxListSpans = uint64_t(1) << 31;  // list ids are 32 bits

// One size-class list (struct of arrays, device memory); `count` is a device
// counter the partition kernel fills.
struct SpanList {
  uint64_t* off;   // byte offset of the span's first byte from the batch base
  uint32_t* len;   // bytes (verify: including the type byte)
  uint32_t* init;  // init_crc
  uint32_t* id;    // output slot
  uint32_t* count;
};

// Builds the 96 KiB LDS image (tables + misc words; counters 0).
inline void BuildLdsImage(uint32_t* img) {
  using namespace wipdb::gf2;
  Tables T;  // ~9 KiB on the caller's stack, built once per context
  BuildTables(&T);
  for (uint32_t i = 0; i < kImageBytes / 4; ++i) img[i] = 0;
  uint32_t sh[4][256];
  for (int c = 1; c < 8; ++c) {
    BuildShiftTable(uint64_t(512) * c, sh);
    for (int p = 0; p < 4; ++p)
      for (int b = 0; b < 256; ++b) img[(kLdsL2 + b * 128 + (c * 4 + p) * 4) / 4] = sh[p][b];
  }
  for (int b = 0; b < 256; ++b)
    for (int t = 0; t < 4; ++t)
      for (int r = 0; r < 8; ++r) img[(kLdsMain + b * 256 + t * 32 + r * 4) / 4] = T.t[3 - t][b];
  for (int a = 1; a < 8; ++a) {
    BuildShiftTable(uint64_t(64) * a, sh);
    for (int p = 0; p < 4; ++p)
      for (int b = 0; b < 256; ++b)
        img[(kLdsMain + b * 256 + 128 + (a * 4 + p) * 4) / 4] = sh[p][b];
  }
  for (int v = 0; v < 256; ++v) img[MiscAddr(kMiscInvTop + v) / 4] = T.inv_top[v];
  for (int h = 0; h < 16; ++h) img[MiscAddr(kMiscHead0 + h) / 4] = T.head0[h];
}

}  // namespace lk
}  // namespace wipdb
