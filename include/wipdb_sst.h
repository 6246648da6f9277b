/* include/wipdb_sst.h -- C-ABI over the batched table / log layer
 * (include/wipdb/table.h, include/wipdb/log.h), for FFI callers (the
 * Python package binds it with ctypes, wipdb_amd/_lib.py).
 *
 * Status codes (the kv::Status a reference call returns for the same input):
 *   WSST_OK            0   OK
 *   WSST_CORRUPTION    1   Corruption other than a checksum mismatch
 *   WSST_CRC_MISMATCH  2   Corruption("block checksum mismatch") /
 *                          "checksum mismatch" (log records)
 *   WSST_OTHER         3   any other non-OK status
 *   WSST_ERR_*        <0   API errors (bad argument, buffer too small,
 *                          device error under WSST_CRC_BATCH_GPU)
 *
 * crc_mode: WSST_CRC_INLINE (per block on the host, the reference's
 * schedule), WSST_CRC_BATCH_CPU, WSST_CRC_BATCH_GPU (MI355X, errors are
 * reported), WSST_CRC_BATCH_AUTO (MI355X when usable).
 */
#ifndef WIPDB_SST_H_
#define WIPDB_SST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WSST_OK 0
#define WSST_CORRUPTION 1
#define WSST_CRC_MISMATCH 2
#define WSST_OTHER 3
#define WSST_ERR_INVALID (-1)
#define WSST_ERR_TOO_SMALL (-2)
#define WSST_ERR_DEVICE (-3)

#define WSST_CRC_INLINE 0
#define WSST_CRC_BATCH_CPU 1
#define WSST_CRC_BATCH_GPU 2
#define WSST_CRC_BATCH_AUTO 3

/* Builds ntables tables with wipdb::table::TableBuilder (the reference's
 * kv::TableBuilder format, kv/src/table/table_builder.cc): table t gets the
 * next entries[t] (key, value) pairs (keys sorted within a table; blobs are
 * concatenated, *_lens give the sizes).  The tables are finished together by
 * FinishTables (one CRC batch).  Table t's bytes go to out[out_offsets[t],
 * out_offsets[t] + sizes[t]) with tables packed back to back; cap bounds
 * the total.  batched_blocks (nullable) receives the number of block CRCs
 * computed in batches.  Returns a status code of the first failing table. */
int wsst_build_tables(size_t ntables, const size_t* entries, const char* keys,
                      const uint32_t* key_lens, const char* vals, const uint32_t* val_lens,
                      int block_size, int restart_interval, int bloom_bits,
                      size_t max_buffer_size, int crc_mode, int device, char* out,
                      size_t cap, uint64_t* out_offsets, uint64_t* sizes,
                      uint64_t* batched_blocks);

/* Key formats of wsst_build_tables_ex.
 *   WSST_KEYS_BYTEWISE  kv::Options defaults: BytewiseComparator, raw bloom keys
 *   WSST_KEYS_INTERNAL  WipDB's DB tables: InternalKeyComparator(Bytewise) and
 *                       InternalFilterPolicy (kv/src/db/db_impl.cc:141-144,
 *                       dbformat.cc:89-136); every key carries the 8-byte tag */
#define WSST_KEYS_BYTEWISE 0
#define WSST_KEYS_INTERNAL 1

/* wsst_build_tables with a key format: WSST_KEYS_INTERNAL writes the index
 * separators and bloom filters of the tables WipDB's flush (BuildTableKV,
 * kv/src/db/builder.cc:46-54) and compaction produce. */
int wsst_build_tables_ex(size_t ntables, const size_t* entries, const char* keys,
                         const uint32_t* key_lens, const char* vals, const uint32_t* val_lens,
                         int block_size, int restart_interval, int bloom_bits,
                         size_t max_buffer_size, int crc_mode, int device, int key_format,
                         char* out, size_t cap, uint64_t* out_offsets, uint64_t* sizes,
                         uint64_t* batched_blocks);

/* ReadBlock(verify_checksums) on a table image (kv/src/table/format.cc:66). */
int wsst_read_block(const char* image, size_t n, uint64_t offset, uint64_t size);

/* Table::Open(paranoid_checks) + a verified iteration over n table images,
 * the CRCs batched across all tables (kv/src/table/table.cc:37-138).
 * codes[i] = table i's status code; returns the first non-OK code.
 * bad_blocks (nullable) = blocks whose CRC failed, over all tables. */
int wsst_verify_tables(const char* const* images, const size_t* sizes, size_t n,
                       int bloom_bits, int crc_mode, int device, int* codes,
                       uint64_t* blocks_checked, uint64_t* bad_blocks);

/* The compaction input path (kv/src/db/version_set.cc:1348-1373): the merged
 * (InternalKeyComparator for WSST_KEYS_INTERNAL, else bytewise) entries of
 * n table images, data blocks checked ahead of the merge prefetch_blocks per
 * input per CRC batch (verify != 0: paranoid_checks).  Keys and values go
 * to key_out / val_out (concatenated, lengths in key_lens / val_lens) in
 * merge order, *nentries of them; *crc_batches (nullable) = CRC batches
 * issued.  Returns the iterator's final status code; WSST_ERR_TOO_SMALL
 * when a capacity is exceeded. */
int wsst_merge_tables(const char* const* images, const size_t* sizes, size_t n, int key_format,
                      int verify, size_t prefetch_blocks, int crc_mode, int device,
                      char* key_out, size_t key_cap, uint32_t* key_lens, char* val_out,
                      size_t val_cap, uint32_t* val_lens, size_t max_entries,
                      uint64_t* nentries, uint64_t* crc_batches);

/* kv::log::Writer::AddRecord for n records (concatenated + lengths) into a
 * fresh log (kv/src/db/log_writer.cc), every header CRC in one batch.
 * *out_size = image size; WSST_ERR_TOO_SMALL when it exceeds cap. */
int wsst_log_write(const char* records, const uint32_t* lens, size_t n, int recycle,
                   uint64_t log_number, int crc_mode, int device, char* out, size_t cap,
                   uint64_t* out_size);

/* kv::log::Reader::ReadRecord (checksum on, initial offset 0) over nlogs log
 * images, all record CRCs in one batch (kv/src/db/log_reader.cc).  Records of
 * all logs go to rec_out / rec_lens / rec_offsets (LastRecordOffset) in order,
 * nrecs[i] per log; corruption reports to drop_bytes and 64-byte
 * "Corruption: <reason>" slots of drop_reasons, ndrops[i] per log.
 * WSST_ERR_TOO_SMALL when a capacity is exceeded. */
int wsst_log_read(const char* const* images, const size_t* sizes, size_t nlogs, int crc_mode,
                  int device, char* rec_out, size_t rec_cap, uint32_t* rec_lens,
                  uint64_t* rec_offsets, size_t max_recs, uint64_t* nrecs,
                  uint64_t* drop_bytes, char* drop_reasons, size_t max_drops,
                  uint64_t* ndrops);

#ifdef __cplusplus
}
#endif
#endif /* WIPDB_SST_H_ */
