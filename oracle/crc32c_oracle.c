/*
 * oracle/crc32c_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference CRC32C used by WipDB's table layer,
 * kept as the parity checker for the MI355X batch engine.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product path (wipdb_amd/, include/) never links it.
 *
 * Parity pinning: the restatement is checked against (a) the RFC 3720 B.4
 * vectors and the folly 3-way vectors from rocksdb/util/crc32c_test.cc:21-100,
 * (b) leveldb/util/crc32c.cc:269-271 ("TestCRCBuffer" -> 0xdcbc59fa), and
 * (c) the reference kv/src/util/crc32c.cc itself, compiled from its own
 * sources into oracle/_ref/ (oracle/Makefile) -- see tests/test_oracle.py.
 *
 * What it restates (all citations relative to /root/reference):
 *   - polynomial: CRC-32C Castagnoli, reflected 0x82F63B78 -- entry 128 of
 *     table0_ in kv/src/util/crc32c.cc:49-82 (table0_[0x80] = 0x82f63b78).
 *   - ExtendImpl<Slow_CRC32> kv/src/util/crc32c.cc:355-397: the register
 *     starts at crc ^ 0xffffffff (:360), bytes are folded in one at a time
 *     with table0_ (STEP1, :365-368) and the result is l ^ 0xffffffff (:396).
 *     The reference's 4-byte slicing (Slow_CRC32 :325-339), 1-stream crc32q
 *     (Fast_CRC32 :341-353) and 3-way (crc32c_3way :667-1198) produce the same
 *     function; this restatement uses the byte-at-a-time form only, because
 *     it is the definition the others are optimisations of.
 *   - Mask / Unmask / kMaskDelta kv/src/util/crc32c.h:31-47.
 *   - the folly buffer fill, rocksdb/util/crc32c_test.cc:145-176 (FNV-64 of
 *     the previous 8 bytes, note the signed-char XOR at :155-156).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

static uint32_t g_table0[256];
static int g_init = 0;

/* Builds the byte table the reference lists literally as table0_
 * (kv/src/util/crc32c.cc:49-312): table0_[i] = CRC register after feeding
 * byte i into a zero register, reflected polynomial 0x82F63B78. */
static void oracle_init(void) {
  if (g_init) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    g_table0[i] = c;
  }
  g_init = 1;
}

uint32_t oracle_table0(int i) {
  oracle_init();
  return g_table0[i & 0xff];
}

/* kv::crc32c::Extend (kv/src/util/crc32c.h:24, crc32c.cc:1225) restated as
 * ExtendImpl with the byte step (crc32c.cc:355-397). */
uint32_t oracle_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  oracle_init();
  const uint8_t* p = (const uint8_t*)data;
  uint32_t l = init_crc ^ 0xffffffffu;           /* crc32c.cc:360 */
  for (size_t i = 0; i < n; ++i)                  /* STEP1, crc32c.cc:365 */
    l = g_table0[(l ^ p[i]) & 0xff] ^ (l >> 8);
  return l ^ 0xffffffffu;                         /* crc32c.cc:396 */
}

/* kv::crc32c::Value, crc32c.h:27-29. */
uint32_t oracle_crc32c_value(const void* data, size_t n) {
  return oracle_crc32c_extend(0, data, n);
}

/* crc32c.h:38-41 */
uint32_t oracle_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

/* crc32c.h:44-47 */
uint32_t oracle_unmask(uint32_t masked) {
  uint32_t rot = masked - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

/* Batch form used by the tests: out[i] = Extend(init[i] (or 0), base+off[i],
 * len[i]); with mask != 0 the stored form Mask(crc) is returned
 * (kv/src/table/table_builder.cc:194-196). */
void oracle_crc32c_batch(const uint8_t* base, const uint64_t* offsets,
                         const uint32_t* lengths, const uint32_t* inits,
                         uint32_t* out, size_t count, int mask) {
  for (size_t i = 0; i < count; ++i) {
    uint32_t c = oracle_crc32c_extend(inits ? inits[i] : 0u, base + offsets[i],
                                      lengths[i]);
    out[i] = mask ? oracle_mask(c) : c;
  }
}

/* rocksdb/util/crc32c_test.cc:145-176: buffer[0..8) = 0, then each 64-bit
 * little-endian word is FNV-64 (folly variant) of the previous 8 bytes. */
static uint64_t fnv64_buf(const uint8_t* buf, size_t n, uint64_t hash) {
  for (size_t i = 0; i < n; ++i) {
    hash += (hash << 1) + (hash << 4) + (hash << 5) + (hash << 7) +
            (hash << 8) + (hash << 40);
    hash ^= (uint64_t)(int64_t)(int8_t)buf[i];    /* signed char, :155 */
  }
  return hash;
}

void oracle_fill_folly_buffer(uint8_t* buf, size_t size) {
  const uint64_t start = 14695981039346656037ULL;
  memset(buf, 0, 8);
  for (size_t w = 1; w < size / 8; ++w) {
    uint64_t h = fnv64_buf(buf + 8 * (w - 1), 8, start);
    for (int b = 0; b < 8; ++b) buf[8 * w + b] = (uint8_t)(h >> (8 * b));
  }
}
