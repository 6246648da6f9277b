/*
 * hip_crc32c_batch.h -- C-ABI of the MI355X batched CRC32C engine.
 *
 * The boundary between WipDB's C++ table layer and the HIP kernels.  Plain
 * pointers and sizes only; no C++ or torch types cross it; nothing throws.
 *
 * What each entry point replaces in the reference (/root/reference):
 *
 *   hcrc_batch / hcrc_batch_async
 *       N calls of kv::crc32c::Extend(init_crc, data, n)
 *       (kv/src/util/crc32c.h:24, kv/src/util/crc32c.cc:1225-1227), as made
 *       one block at a time by TableBuilder::WriteRawBlock
 *       (kv/src/table/table_builder.cc:194-196) and ReadBlock
 *       (kv/src/table/format.cc:91-93).  With HCRC_MASK_OUTPUT the stored
 *       form kv::crc32c::Mask(crc) (kv/src/util/crc32c.h:38-41) is written.
 *       leveldb::crc32c::Extend (leveldb/util/crc32c.h:17,
 *       leveldb/util/crc32c.cc:275) is the same function.
 *   hcrc_batch_strided_async
 *       the same for fixed-size, fixed-stride blocks (no descriptor arrays).
 *   hcrc_verify_async, hcrc_verify_async_ex
 *       ReadBlock's check (kv/src/table/format.cc:91-99):
 *       Unmask(stored) == Value(data, n+1) for a batch of blocks.
 *   hcrc_batch_multi, hcrc_batch_multi_ex
 *       a batch sharded by bytes over several GPUs of one node (no
 *       collective: blocks are independent).
 *   hcrc_cpu_extend / hcrc_cpu_batch
 *       the host CPU path (from scratch, SSE4.2+PCLMUL or portable), i.e.
 *       what kv::crc32c::Extend itself does on the host.
 *
 * Semantics shared by every batch call (bit-exact with the reference):
 *   out[i] = Extend(inits ? inits[i] : 0, base + offsets[i], lengths[i])
 *   optionally Mask()-ed.  Any span alignment, any length >= 0 (a length
 *   of 0 returns the init value, as Extend does).
 *
 * Ownership: the caller owns base/offsets/lengths/inits/out and keeps them
 * valid until the call (sync) or the stream (async) completes.  The context
 * owns device tables, staging buffers and its stream.  No pointer is
 * retained after completion.
 *
 * Errors: 0 on success, a negative HCRC_ERR_* code otherwise.  The batch
 * entry points never fall back to the CPU silently; a caller that wants a
 * fallback (the C++ wrapper's AUTO policy) calls hcrc_cpu_batch itself.
 *
 * Threading (the reference's flush, compaction and split pools call
 * Extend concurrently, kv/tests/db/kv_bench.cc:2041-2043): a context may be
 * used from any number of threads at once.  The async entry points take no
 * lock (they only enqueue on the caller's stream); a synchronous call
 * (hcrc_batch, hcrc_batch_multi) leases one of up to 8 per-context lanes --
 * its own HIP stream and pinned staging slots -- so concurrent calls overlap
 * on the device.  Every entry point leaves the caller's current HIP device
 * as it found it.
 */
#ifndef HIP_CRC32C_BATCH_H_
#define HIP_CRC32C_BATCH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HCRC_ABI_VERSION 1

/* return codes */
#define HCRC_OK 0
#define HCRC_ERR_INVALID (-1)   /* bad argument (null pointer, bad flags) */
#define HCRC_ERR_NO_DEVICE (-2) /* no HIP device or bad device index     */
#define HCRC_ERR_NO_MEMORY (-3) /* device or pinned allocation failed    */
#define HCRC_ERR_HIP (-4)       /* other HIP runtime error               */
#define HCRC_ERR_LAUNCH (-5)    /* kernel launch failed                  */
#define HCRC_ERR_MISMATCH (-6)  /* hcrc_verify*: at least one bad block  */
#define HCRC_ERR_BOUNDS (-7)    /* hcrc_check_spans: a span leaves base   */
#define HCRC_ERR_KERNEL (-8)    /* a kernel reported an internal fault:   */
                                /* some outputs were not written          */

/* flags */
#define HCRC_HOST_PTRS 0x0    /* all array/data pointers are host memory    */
#define HCRC_DEVICE_PTRS 0x1  /* all array/data pointers are device memory  */
#define HCRC_MASK_OUTPUT 0x2  /* write Mask(crc) instead of crc             */
/* Size classes: a partition pass sorts the batch into spans of at most
 * ~1 KiB (checksummed 4 per wave iteration), at most ~2 KiB (2 per wave
 * iteration) and longer ones (round 2's end-aligned pipeline).  Same results.
 * An opt-in: the default kernel packs short spans by itself and is as fast or
 * faster on every measured shape, so no entry point
 * chooses it by itself any more.  Uses stream-ordered scratch (~60 bytes per
 * span). */
#define HCRC_SPLIT_SMALL 0x4
/* Long spans (device batches; host batches do it by themselves for spans of
 * >= 256 KiB): a span of >= 128 KiB is cut into 16 KiB parts checksummed on
 * many waves at once and combined by GF(2) linearity (crc32c_3way's
 * CombineCRC, kv/src/util/crc32c.cc:640-657) -- a lone span otherwise runs
 * its segments chained on one wave (~2.7 GiB/s).  Same results; four
 * launches instead of one and stream-ordered scratch (~36 bytes per span +
 * a pool of 64 Ki..1 Mi parts, past which spans stay whole).  A latency
 * tool for batches of few long spans (a lone 16 MiB span: 5.6 -> 0.14 ms);
 * batches of many short spans run slower with it.  Takes precedence over
 * HCRC_SPLIT_SMALL.  A device batch of at most 16 spans (without
 * HCRC_SPLIT_SMALL) takes it by itself: there one long span is the job. */
#define HCRC_SPLIT_LONG 0x8
/* Byte-balanced workgroups (device descriptor batches, hcrc_batch_async /
 * hcrc_batch with HCRC_DEVICE_PTRS): two small passes over the length
 * column cut the batch into one contiguous range per workgroup of equal
 * weight (bytes + 64 per span), instead of dealing every workgroup the same
 * NUMBER of spans.  For large batches of mixed sizes (config 3's Zipf mix:
 * the default deal leaves the busiest of 256 workgroups ~1.17x the mean);
 * same results, two extra launches and (G + 1) * 4 + 8 * n / 1024 bytes of
 * stream-ordered scratch.  Ignored with HCRC_SPLIT_SMALL / HCRC_SPLIT_LONG,
 * for batches of fewer than 64 spans per workgroup, and on host pointers
 * (hcrc_batch without HCRC_DEVICE_PTRS: those batches are bound by the
 * host-device copy or the zero-copy reads, not by the kernel's balance, and
 * the passes would only add two launches per staged piece). */
#define HCRC_BALANCE 0x10
/* SST-packed device batch (hcrc_batch_async / hcrc_batch with
 * HCRC_DEVICE_PTRS): the spans are sorted by offset, do not overlap and
 * leave gaps of less than 4 KiB -- what TableBuilder::WriteRawBlock leaves
 * in a write buffer (kv/src/table/table_builder.cc:183-202), a WAL block,
 * config 3's stream.  Such a batch is read as ONE byte stream, 4 KiB page by
 * page, fully coalesced, each workgroup an equal share of the bytes
 * (stream-tiled kernel).  A small pre-pass checks the
 * promise (and that no 4 KiB holds more than 62 span starts); a batch that
 * breaks it runs the default pipelines instead, and one the end-aligned
 * loop suits (aligned 4 KiB blocks, table blocks, spans of >= 16 KiB) runs
 * that loop, so the promise can cost speed, never a CRC.
 *   Since round 6 no flag is needed: every device batch of >= 32 Ki spans
 * takes this sequence, and a REPEATED batch (same base, columns and count on
 * the same stream) whose last verdict was "suits the end-aligned loop" or
 * "not packed" skips the pre-pass (the verdict comes back through a pinned
 * word the kernel stores; re-checked every 64 launches).  The flag lowers
 * the minimum (WIPDB_PS_MIN_SPANS, tests) and keeps HCRC_BALANCE batches on
 * this path.  Host batches build the check and the chunk index on the host
 * for every piece of >= 4096 spans (staged pieces are packed by
 * construction).  Scratch: (16 G + 9) * 4 bytes and a pinned word per
 * stream that launches one, allocated on its first and kept with the
 * context (hcrc_stream_forget releases them).  Ignored with
 * HCRC_SPLIT_SMALL / HCRC_SPLIT_LONG.  Below 32 Ki spans the default kernel
 * runs: there the stream's start (desk loads, a page a wave) is slower than
 * the default kernel (one 2 MiB SST of 488 spans: 15 vs 24 us). */
#define HCRC_PACKED 0x20

typedef struct hcrc_ctx hcrc_ctx;

/* Library / device queries. */
int hcrc_abi_version(void);
int hcrc_device_count(int* count);
const char* hcrc_strerror(int code);

/* A context per call of hcrc_ctx_create (its own tables, streams, staging),
 * released by hcrc_ctx_destroy.  hcrc_ctx_shared is idempotent per device
 * (SURVEY 8b): every call returns the same process-wide context for that
 * device, created on first use (the one the C++ ExtendBatch and
 * hcrc_batch_multi use); it lives until the process ends: hcrc_ctx_destroy
 * refuses it (HCRC_ERR_INVALID), since other threads may hold it at any
 * moment. */
int hcrc_ctx_create(int device, hcrc_ctx** out_ctx);
int hcrc_ctx_shared(int device, hcrc_ctx** out_ctx);
int hcrc_ctx_destroy(hcrc_ctx* ctx);
/* The context's own HIP stream (hipStream_t as void*). */
void* hcrc_ctx_stream(hcrc_ctx* ctx);
int hcrc_ctx_device(hcrc_ctx* ctx);

/* Synchronous batch.  HCRC_HOST_PTRS: data is staged through pinned
 * buffers (H2D + kernel + D2H, overlapped); HCRC_DEVICE_PTRS: all pointers
 * are device memory.  Returns after out[] is written. */
int hcrc_batch(hcrc_ctx* ctx, const void* base, const uint64_t* offsets,
               const uint32_t* lengths, const uint32_t* init_crcs,
               uint32_t* out_crcs, size_t count, int flags);

/* Asynchronous batch on device memory, enqueued on `stream` (a hipStream_t;
 * NULL = the HIP default stream, as in HIP itself; pass hcrc_ctx_stream(ctx)
 * for the context's own stream).  Requires HCRC_DEVICE_PTRS in flags. */
int hcrc_batch_async(hcrc_ctx* ctx, const void* d_base,
                     const uint64_t* d_offsets, const uint32_t* d_lengths,
                     const uint32_t* d_init_crcs, uint32_t* d_out_crcs,
                     size_t count, int flags, void* stream);

/* Fixed-size blocks: span i = d_base + i*stride, `length` bytes, all with
 * the same init_crc.  Device memory, asynchronous on `stream`. */
int hcrc_batch_strided_async(hcrc_ctx* ctx, const void* d_base,
                             uint64_t stride, uint32_t length,
                             uint32_t init_crc, uint32_t* d_out_crcs,
                             size_t count, int flags, void* stream);

/* Read-side verification (ReadBlock, kv/src/table/format.cc:91-99): block i
 * is d_base + offsets[i] with handle size lengths[i] = n; the checksum
 * covers n+1 bytes (contents + type byte) and is compared with the masked
 * crc stored little-endian at byte n+1.  d_status[i] = 1 if it matches,
 * 0 if not.  Asynchronous on `stream`, device memory. */
int hcrc_verify_async(hcrc_ctx* ctx, const void* d_base,
                      const uint64_t* d_offsets, const uint32_t* d_lengths,
                      uint8_t* d_status, size_t count, void* stream);
/* The same with flags: 0 or HCRC_SPLIT_SMALL (the size classes above:
 * small blocks -- meta-index, small filters -- several per wave iteration). */
int hcrc_verify_async_ex(hcrc_ctx* ctx, const void* d_base,
                         const uint64_t* d_offsets, const uint32_t* d_lengths,
                         uint8_t* d_status, size_t count, int flags, void* stream);

/* Bounds check of a device descriptor batch before it is handed to the
 * kernels, which trust it (a span outside the caller's buffer is a GPU page
 * fault).  Span i is out of bounds when offsets[i] + lengths[i] + extra >
 * base_bytes, computed without overflow; extra = 0 for a CRC batch, 5 for a
 * verify batch (type byte + stored crc).  The async form writes
 * d_result[0] = the number of such spans and d_result[1] = the lowest such
 * index (UINT64_MAX if none) on `stream`; the synchronous form returns
 * HCRC_OK or HCRC_ERR_BOUNDS (with *first_bad, nullable).  The reference's
 * equivalent is the size check ReadBlock makes on the pread result
 * (kv/src/table/format.cc:84-87). */
int hcrc_check_spans_async(hcrc_ctx* ctx, uint64_t base_bytes,
                           const uint64_t* d_offsets, const uint32_t* d_lengths,
                           uint32_t extra, size_t count, uint64_t* d_result,
                           void* stream);
int hcrc_check_spans(hcrc_ctx* ctx, uint64_t base_bytes,
                     const uint64_t* d_offsets, const uint32_t* d_lengths,
                     uint32_t extra, size_t count, uint64_t* first_bad);

/* In-kernel faults.  The lane-packed kernels never leave a span
 * uncomputed without saying so: a wait of the workgroup's long-span queue
 * that runs out of its bound (no schedule of a resident workgroup gets
 * there) sets the launch's fault word instead.  Every launch writes the word
 * of its owner only: a synchronous entry point (hcrc_batch,
 * hcrc_batch_multi*) checks its own and returns HCRC_ERR_KERNEL (outputs
 * incomplete; the C++ ExtendBatch(kAuto) then computes the batch on the
 * CPU); the *_async entry points use one word per caller stream, which
 * hcrc_sync(ctx, stream) reads and clears for that stream (a fault of a
 * launch on another stream, or of a synchronous call, is never reported
 * there).  hcrc_ctx_check reads and clears the words of every stream the
 * context has launched on -- call it after synchronising them.  The
 * reference's Extend is infallible (kv/src/util/crc32c.h:24); a wrong CRC
 * returned as success is the one failure a checksum must never have. */
int hcrc_ctx_check(hcrc_ctx* ctx);

/* Wait for all work on `stream` (NULL = the HIP default stream), then
 * HCRC_ERR_KERNEL if a launch of this context on `stream` reported a fault
 * since that stream's last check (the check clears it). */
int hcrc_sync(hcrc_ctx* ctx, void* stream);

/* Release what the context keeps for `stream`: its fault word (returned to
 * the free list -- a stream created later, even one HIP hands the same
 * handle, starts clean) and its HCRC_PACKED pre-pass scratch.  Call it once
 * the stream's launches are complete (after hcrc_sync or the caller's own
 * synchronisation) and before the stream is destroyed.  Returns
 * HCRC_ERR_KERNEL if the stream's word held an unread fault (read and
 * cleared here, as hcrc_sync would), else HCRC_OK; forgetting a stream the
 * context never launched on is a no-op.  Without it a context keeps one word
 * per stream it has seen: past 1024 streams the others share word 0 (a fault
 * is then reported to every stream past the table: conservative, never
 * silent) and their packed batches take the default path.
 * hipStreamPerThread stands for a different queue on every host thread: its
 * packed batches take the default path, and its threads share one word. */
int hcrc_stream_forget(hcrc_ctx* ctx, void* stream);

/* Host-memory batch sharded over `ndev` devices by bytes, one host thread
 * and context per device; results land in disjoint slices of out_crcs. */
int hcrc_batch_multi(const int* devices, int ndev, const void* base,
                     const uint64_t* offsets, const uint32_t* lengths,
                     const uint32_t* init_crcs, uint32_t* out_crcs,
                     size_t count, int flags);
/* The same, with each shard's own return code in shard_rc[ndev] (nullable):
 * a failing device fails its shard only; the return value is the first
 * non-zero shard code.  A device may be listed more than once (its shards
 * then run concurrently on one shared context). */
int hcrc_batch_multi_ex(const int* devices, int ndev, const void* base,
                        const uint64_t* offsets, const uint32_t* lengths,
                        const uint32_t* init_crcs, uint32_t* out_crcs,
                        size_t count, int flags, int* shard_rc);

/* Pinned host memory.  hcrc_batch over spans that each lie inside a range
 * allocated by hcrc_host_alloc or registered by hcrc_host_register (e.g.
 * mmap'd SST files, a long-lived memtable arena, a table builder's write
 * buffers -- one or several ranges) needs no staging copy: a dense,
 * in-order piece of >= 8 MiB inside one range (up to 128 MiB a piece; the
 * last piece of a batch after such a piece has no floor) is copied to the
 * device by the copy engine, the next piece's copy running under this
 * one's kernel, and checked out of HBM; any other piece (smaller batches,
 * sparse or shuffled spans) runs zero-copy: the kernel reads the spans over
 * PCIe directly.  Anything else (a span in pageable memory, memory pinned by
 * other means, a span straddling two ranges) sends the batch through the
 * pinned staging slots.  The copy-engine pieces use two 128 MiB device
 * buffers per concurrent caller, allocated on first use. */
int hcrc_host_alloc(size_t bytes, void** out_ptr);
int hcrc_host_free(void* ptr);
int hcrc_host_register(void* ptr, size_t bytes);
int hcrc_host_unregister(void* ptr);

/* Diagnostic: the measured read-stream ceiling.  Reads `count` fixed-size
 * blocks like hcrc_batch_strided_async but only XOR-reduces them (same
 * bytes in, 4 bytes out per block).  Used for the roofline denominator. */
int hcrc_readstream_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride,
                          uint32_t length, uint32_t* d_out, size_t count,
                          void* stream);

/* Diagnostic: the kernel's own memory ceiling.  The memory side of the
 * spans kernel's pipeline for aligned 4 KiB blocks alone -- the table image
 * into LDS, the same unit deal, the same four 1 KiB LDS-DMA loads per block
 * into the wave's slot, the same slot reads, 4 bytes stored per block -- with
 * no CRC work (out[i] = XOR of the first 64 bytes of block i).  length must be
 * 4096, stride >= 4096.  The bench line's roofline reports the CRC kernel
 * against this same-box ceiling (frac_of_ceiling). */
int hcrc_dma_ceiling_async(hcrc_ctx* ctx, const void* d_base, uint64_t stride,
                           uint32_t length, uint32_t* d_out, size_t count,
                           void* stream);

/* Test/bench data: fills nbytes (multiple of 8, 8-byte aligned) of device
 * memory with the seeded splitmix64 stream whose 64-bit word k is
 * mix(seed + (first_word + k + 1) * 0x9E3779B97F4A7C15), so the host can
 * regenerate any block for parity checks (tests/golden/common.py). */
int hcrc_fill_splitmix64_async(hcrc_ctx* ctx, void* d_dst, uint64_t nbytes,
                               uint64_t seed, uint64_t first_word,
                               void* stream);

/* Host CPU path (from-scratch SSE4.2+PCLMUL 3-stream, or portable
 * slicing-by-8); the function kv::crc32c::Extend is built on. */
uint32_t hcrc_cpu_extend(uint32_t init_crc, const void* data, size_t n);
/* The portable slicing-by-8 path alone, whatever the CPU supports (the
 * reference's ExtendImpl<Slow_CRC32>, kv/src/util/crc32c.cc:325-339,
 * 355-397).  WIPDB_CRC_PORTABLE=1 in the environment makes hcrc_cpu_extend,
 * hcrc_cpu_batch and the C++ surface use it too (and
 * hcrc_cpu_is_accelerated return 0), as on a host without SSE4.2. */
uint32_t hcrc_cpu_extend_portable(uint32_t init_crc, const void* data, size_t n);
int hcrc_cpu_batch(const void* base, const uint64_t* offsets,
                   const uint32_t* lengths, const uint32_t* init_crcs,
                   uint32_t* out_crcs, size_t count, int flags, int threads);
int hcrc_cpu_is_accelerated(void);

/* Mask / Unmask of kv/src/util/crc32c.h:38-47. */
uint32_t hcrc_mask(uint32_t crc);
uint32_t hcrc_unmask(uint32_t masked_crc);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* HIP_CRC32C_BATCH_H_ */
