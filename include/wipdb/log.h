// include/wipdb/log.h -- WipDB's write-ahead log with batched record CRCs
// (SURVEY.md 8f-3).
//
// Format (kv/src/db/log_format.h, log_writer.cc:38-154): 32 KiB blocks of
// physical records [masked crc32c : 4][length : 2][type : 1]([log number : 4]
// for the recyclable types 5..8)[payload], FULL / FIRST / MIDDLE / LAST
// fragments, a block tail shorter than a header zero-filled.  The CRC covers
// the type byte, the log number (recyclable) and the payload -- bytes that
// sit contiguously in the file, so each record is one span of a CRC batch.
//
// WriteLog lays out AddRecord's bytes for many records and computes every
// header CRC in ONE batch.  ReadLog / ReadLogs are kv::log::Reader::ReadRecord
// (log_reader.cc:62-279, checksum on, initial offset 0) over whole log images
// -- the bulk verify of recovery (RecoverLogFile, kv/src/db/kv.cc:117-148):
// every physical record's CRC in one batch, then the reader's state machine
// replayed over the results, so the records returned and the corruption
// reports (bytes dropped, reason) are the reference's.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <string_view>
#include <vector>

#include "wipdb/status.h"
#include "wipdb/table.h"

namespace wipdb {
namespace log {

constexpr size_t kBlockSize = 32768;
constexpr size_t kHeaderSize = 7;
constexpr size_t kRecyclableHeaderSize = 11;

struct Record {
  uint64_t offset;   // Reader::LastRecordOffset(): the first fragment's header
  std::string data;
};

struct Drop {
  uint64_t bytes;
  std::string reason;  // kv Status::ToString(): "Corruption: checksum mismatch", ...
};

// Appends AddRecord(records[i]) for every record to *out, as a kv::log::Writer
// (recycle_log_files, log_number) that starts at a block boundary would.
Status WriteLog(const std::vector<std::string_view>& records, bool recycle, uint64_t log_number,
                table::CrcMode mode, int device, std::string* out);
// WriteLog straight into a caller's buffer of cap bytes: *size = the image
// size; InvalidArgument (nothing written) when it exceeds cap.
Status WriteLogTo(const std::vector<std::string_view>& records, bool recycle, uint64_t log_number,
                  table::CrcMode mode, int device, char* out, size_t cap, size_t* size);

// Recovery read of one log image (checksum = true, initial offset 0).
Status ReadLog(const char* image, size_t n, table::CrcMode mode, int device,
               std::vector<Record>* records, std::vector<Drop>* drops);

// The same over many logs with one CRC batch for all of them.
Status ReadLogs(const char* const* images, const size_t* sizes, size_t nlogs,
                table::CrcMode mode, int device, std::vector<std::vector<Record>>* records,
                std::vector<std::vector<Drop>>* drops);

// ReadLogs handing each record to fn(ctx, log, LastRecordOffset, data, size)
// in order instead of copying it into a Record: a record of one fragment is
// a view of the image, a fragmented one a view of scratch valid during the
// call.
typedef void (*RecordFn)(void* ctx, size_t log, uint64_t offset, const char* data, size_t n);
Status ReadLogsEach(const char* const* images, const size_t* sizes, size_t nlogs,
                    table::CrcMode mode, int device, RecordFn fn, void* ctx,
                    std::vector<std::vector<Drop>>* drops);

}  // namespace log
}  // namespace wipdb
