// gf2_crc32c.h -- CRC-32C arithmetic in GF(2)[x] / P(x), host side.
//
// Representation (the one every table below uses): a 32-bit "register"
// value r is a polynomial in reflected bit order, bit 31 = coefficient of
// x^0 ... bit 0 = coefficient of x^31, reduced modulo the Castagnoli
// polynomial P (reflected constant 0x82F63B78, the entry table0_[0x80] of
// /root/reference/kv/src/util/crc32c.cc:82).
//
// The one identity the whole engine is built on (linearity of the raw CRC
// register, the same fact crc32c_3way's CombineCRC relies on,
// kv/src/util/crc32c.cc:640-657):
//
//   feed(r, M) = shift(r, |M|) XOR feed(0, M),   shift(r, n) = r * x^(8n) mod P
//   Extend(init, M) = ~feed(~init, M)            (crc32c.cc:360, :396)
//   Extend(c, B)    = Value(B) XOR shift(c, |B|) (combine of two Extends)
//
// Everything here is constexpr-free plain C++ so it compiles with g++ and
// hipcc alike; the device kernels consume the tables this file builds.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace wipdb {
namespace gf2 {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli
constexpr uint32_t kOne = 0x80000000u;   // x^0 in reflected order

// a * b mod P, both reflected.
inline uint32_t MulMod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (kOne >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);  // b *= x
  }
  return p;
}

// x^(8n) mod P by square-and-multiply.
inline uint32_t XPow8N(uint64_t n) {
  uint32_t result = kOne;
  uint32_t sq = 0x00800000u;  // x^8 (bit 31-8 = 23)
  while (n) {
    if (n & 1) result = MulMod(result, sq);
    sq = MulMod(sq, sq);
    n >>= 1;
  }
  return result;
}

// x^m mod P for an arbitrary bit exponent m (used for the clmul fold
// constants of the CPU path, which are x^(8L-33)).
inline uint32_t XPowBits(uint64_t m) {
  uint32_t result = kOne;
  uint32_t sq = kOne >> 1;  // x^1
  while (m) {
    if (m & 1) result = MulMod(result, sq);
    sq = MulMod(sq, sq);
    m >>= 1;
  }
  return result;
}

// Register after feeding n zero bytes into register r.
inline uint32_t Shift(uint32_t r, uint64_t nbytes) {
  return MulMod(r, XPow8N(nbytes));
}

// One byte of the raw register (Sarwate step); T0 = table of this step.
inline uint32_t ByteStepSlow(uint32_t r, uint8_t b) {
  r ^= b;
  for (int k = 0; k < 8; ++k) r = (r >> 1) ^ (kPoly & (0u - (r & 1u)));
  return r;
}

// All tables the engine uses, built once.
struct Tables {
  // Slicing-by-8: t[k][b] = contribution of byte b followed by k zero bytes.
  // t[0] is the classic byte table (reference table0_), t[1] is the second
  // table of the device's slicing-by-2 step.
  uint32_t t[8][256];
  // inv_top[v] = the byte i with (t[0][i] >> 24) == v.  The top byte of the
  // byte table is a bijection for CRC-32C (checked in Build()), so one zero
  // byte can be un-fed: r = ((r' ^ t0[i]) << 8) | i, i = inv_top[r' >> 24].
  uint8_t inv_top[256];
  // head0[h] = ~0 * x^(-8h): the register that, after h zero bytes, equals
  // ~0 -- the Value()/init==0 state placed h bytes before a span start.
  uint32_t head0[16];
  bool ok;
};

inline void BuildTables(Tables* T) {
  for (int i = 0; i < 256; ++i) T->t[0][i] = ByteStepSlow(0, (uint8_t)i);
  for (int k = 1; k < 8; ++k)
    for (int i = 0; i < 256; ++i) {
      uint32_t v = T->t[k - 1][i];
      T->t[k][i] = T->t[0][v & 0xff] ^ (v >> 8);
    }
  bool seen[256] = {false};
  T->ok = true;
  for (int i = 0; i < 256; ++i) {
    uint32_t top = T->t[0][i] >> 24;
    if (seen[top]) T->ok = false;
    seen[top] = true;
    T->inv_top[top] = (uint8_t)i;
  }
  for (int h = 0; h < 16; ++h) {
    uint32_t r = 0xffffffffu;
    for (int s = 0; s < h; ++s) {
      uint8_t i = T->inv_top[r >> 24];
      r = ((r ^ T->t[0][i]) << 8) | i;
    }
    T->head0[h] = r;
  }
}

// Un-feed h zero bytes: returns r0 with shift(r0, h) == r.
inline uint32_t Unshift(const Tables& T, uint32_t r, int h) {
  for (int s = 0; s < h; ++s) {
    uint8_t i = T.inv_top[r >> 24];
    r = ((r ^ T.t[0][i]) << 8) | i;
  }
  return r;
}

// 4 x 256 "multiply by x^(8n)" table: out[p][b] = shift(b << 8p, n).  Any
// register is then shifted by n bytes with 4 lookups.
inline void BuildShiftTable(uint64_t nbytes, uint32_t out[4][256]) {
  uint32_t k = XPow8N(nbytes);
  for (int p = 0; p < 4; ++p)
    for (int b = 0; b < 256; ++b) out[p][b] = MulMod((uint32_t)b << (8 * p), k);
}

inline uint32_t Mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}
inline uint32_t Unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

}  // namespace gf2
}  // namespace wipdb
