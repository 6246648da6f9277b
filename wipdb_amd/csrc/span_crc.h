// span_crc.h -- one CRC32C batch over spans scattered in host memory, for
// the table and log layers (table_builder.cc, table_reader.cc, log_batch.cc).
// Internal header.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/wipdb/status.h"
#include "../../include/wipdb/table.h"

namespace wipdb {
namespace spancrc {

// out[i] = crc32c(ptrs[i][0, lens[i])) (Mask()-ed when mask), as ONE batch:
// kBatchGpu / kBatchAuto through ExtendBatch (the C-ABI's hcrc_batch),
// kInline / kBatchCpu on the host.  Only kBatchGpu can fail.
Status Compute(const char* const* ptrs, const uint32_t* lens, size_t n, bool mask,
               table::CrcMode mode, int device, uint32_t* out);

}  // namespace spancrc
}  // namespace wipdb
