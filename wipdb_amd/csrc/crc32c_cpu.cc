// crc32c_cpu.cc -- the host C++ CRC32C path, written from scratch.
//
// This is the CPU side of the engine (not the oracle): it backs the
// per-span kv::crc32c::Extend / leveldb::crc32c::Extend surface
// (include/wipdb/crc32c.h) and the multi-threaded host batch entry point.
// Behaviour follows the reference surface kv/src/util/crc32c.h:24-47 and
// its dispatch (kv/src/util/crc32c.cc:1202-1227): SSE4.2+PCLMUL when the
// CPU has them, else a portable table path.
//
//  * Portable: slicing-by-8 over little-endian 64-bit words (8 tables of
//    256 entries from gf2::BuildTables).  Same algorithm class as the
//    reference's ExtendImpl<Slow_CRC32> (crc32c.cc:325-339, 355-397).
//  * SSE4.2: three independent crc32q streams over equal thirds of each
//    window, folded with two carry-less multiplies and one crc32q
//    (register = shift(c0,2B) ^ shift(c1,B) ^ c2, shift(a,L) =
//    crc32q(0, clmul(a, x^(8L-33)))).  Same class as the reference's
//    crc32c_3way/CombineCRC (crc32c.cc:640-1198), own derivation: the fold
//    constants are computed at start-up from gf2::XPowBits, not tabulated.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "gf2_crc32c.h"

#if defined(__x86_64__)
#include <immintrin.h>
#define WIPDB_X86 1
#endif

namespace wipdb {
namespace cpu {

namespace {

const gf2::Tables& Tab() {
  static const gf2::Tables* t = [] {
    auto* x = new gf2::Tables;
    gf2::BuildTables(x);
    return x;
  }();
  return *t;
}

inline uint64_t Load64LE(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;  // x86/little-endian hosts only (as the reference's coding.h)
}

uint32_t FeedPortable(uint32_t r, const uint8_t* p, size_t n) {
  const gf2::Tables& T = Tab();
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    r = T.t[0][(r ^ *p++) & 0xff] ^ (r >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t x = Load64LE(p) ^ r;
    r = T.t[7][x & 0xff] ^ T.t[6][(x >> 8) & 0xff] ^ T.t[5][(x >> 16) & 0xff] ^
        T.t[4][(x >> 24) & 0xff] ^ T.t[3][(x >> 32) & 0xff] ^
        T.t[2][(x >> 40) & 0xff] ^ T.t[1][(x >> 48) & 0xff] ^ T.t[0][x >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) r = T.t[0][(r ^ *p++) & 0xff] ^ (r >> 8);
  return r;
}

#ifdef WIPDB_X86
// Fold constants for stream length B = 8*k bytes, k = 1..kMaxK:
// kc[k][0] = x^(16B-33) (shifts stream 0 over streams 1 and 2),
// kc[k][1] = x^(8B-33)  (shifts stream 1 over stream 2).
constexpr int kMaxK = 512;  // B up to 4 KiB per stream (12 KiB windows)
struct Fold {
  uint64_t kc[kMaxK + 1][2];
};
const Fold& FoldTab() {
  static const Fold* f = [] {
    auto* x = new Fold;
    for (int k = 1; k <= kMaxK; ++k) {
      uint64_t b = 8ull * k;
      x->kc[k][0] = gf2::XPowBits(16 * b - 33);
      x->kc[k][1] = gf2::XPowBits(8 * b - 33);
    }
    return x;
  }();
  return *f;
}

bool HaveSse42Clmul() {
  static const bool ok = __builtin_cpu_supports("sse4.2") &&
                         __builtin_cpu_supports("pclmul");
  return ok;
}

__attribute__((target("sse4.2,pclmul"))) uint32_t FeedSse42(uint32_t r,
                                                           const uint8_t* p,
                                                           size_t n) {
  uint64_t c0 = r;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c0 = _mm_crc32_u8((uint32_t)c0, *p++);
    --n;
  }
  const Fold& F = FoldTab();
  while (n >= 24) {
    size_t k = n / 24;
    if (k > (size_t)kMaxK) k = kMaxK;
    const size_t B = 8 * k;
    const uint64_t* s0 = reinterpret_cast<const uint64_t*>(p);
    const uint64_t* s1 = reinterpret_cast<const uint64_t*>(p + B);
    const uint64_t* s2 = reinterpret_cast<const uint64_t*>(p + 2 * B);
    uint64_t c1 = 0, c2 = 0;
    for (size_t i = 0; i < k; ++i) {
      c0 = _mm_crc32_u64(c0, s0[i]);
      c1 = _mm_crc32_u64(c1, s1[i]);
      c2 = _mm_crc32_u64(c2, s2[i]);
    }
    __m128i k01 = _mm_set_epi64x((long long)F.kc[k][1], (long long)F.kc[k][0]);
    __m128i a = _mm_clmulepi64_si128(_mm_cvtsi64_si128((long long)c0), k01, 0x00);
    __m128i b = _mm_clmulepi64_si128(_mm_cvtsi64_si128((long long)c1), k01, 0x10);
    uint64_t folded = (uint64_t)_mm_cvtsi128_si64(_mm_xor_si128(a, b));
    c0 = _mm_crc32_u64(0, folded) ^ c2;
    p += 3 * B;
    n -= 3 * B;
  }
  while (n >= 8) {
    c0 = _mm_crc32_u64(c0, Load64LE(p));
    p += 8;
    n -= 8;
  }
  while (n--) c0 = _mm_crc32_u8((uint32_t)c0, *p++);
  return (uint32_t)c0;
}
#endif

// WIPDB_CRC_PORTABLE=1 in the environment forces the portable path on a
// host that has SSE4.2 + PCLMUL -- the reference's Choose_Extend falling to
// ExtendImpl<Slow_CRC32> (kv/src/util/crc32c.cc:1202-1222), made reachable
// so the portable path is exercised (tests/test_cpu_path.py).
bool ForcePortable() {
  static const bool force = [] {
    const char* e = getenv("WIPDB_CRC_PORTABLE");
    return e && *e && strcmp(e, "0") != 0;
  }();
  return force;
}

}  // namespace

// Raw register feed (no pre/post inversion).
uint32_t Feed(uint32_t reg, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
#ifdef WIPDB_X86
  if (HaveSse42Clmul() && !ForcePortable()) return FeedSse42(reg, p, n);
#endif
  return FeedPortable(reg, p, n);
}

uint32_t Extend(uint32_t init_crc, const void* data, size_t n) {
  return ~Feed(~init_crc, data, n);
}

uint32_t ExtendPortable(uint32_t init_crc, const void* data, size_t n) {
  return ~FeedPortable(~init_crc, static_cast<const uint8_t*>(data), n);
}

bool IsAccelerated() {
#ifdef WIPDB_X86
  return HaveSse42Clmul() && !ForcePortable();
#else
  return false;
#endif
}

void Batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
           const uint32_t* inits, uint32_t* out, size_t count, bool mask,
           int threads) {
  auto run = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      uint32_t c = Extend(inits ? inits[i] : 0u, base + offsets[i], lengths[i]);
      out[i] = mask ? gf2::Mask(c) : c;
    }
  };
  if (threads <= 1 || count < 64) {
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

}  // namespace cpu
}  // namespace wipdb
