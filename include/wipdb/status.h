// include/wipdb/status.h -- the result type of the table / log layer.
//
// Mirrors the codes and messages of kv::Status (kv/src/include/kv/status.h,
// kv/src/util/status.cc) that the block-checksum path produces, so callers
// can map them 1:1: Corruption("block checksum mismatch") from ReadBlock
// (kv/src/table/format.cc:96), "bad block handle" (format.cc:31),
// "not an sstable (bad magic number)" (format.cc:54), "truncated block
// read" (format.cc:83), "file is too short to be an sstable"
// (table.cc:46).
#pragma once
#include <string>
#include <utility>

namespace wipdb {

class Status {
 public:
  enum Code { kOk = 0, kNotFound = 1, kCorruption = 2, kNotSupported = 3,
              kInvalidArgument = 4, kIOError = 5 };

  Status() = default;
  static Status OK() { return Status(); }
  static Status Corruption(std::string m) { return Status(kCorruption, std::move(m)); }
  static Status InvalidArgument(std::string m) { return Status(kInvalidArgument, std::move(m)); }
  static Status IOError(std::string m) { return Status(kIOError, std::move(m)); }
  static Status NotSupported(std::string m) { return Status(kNotSupported, std::move(m)); }

  bool ok() const { return code_ == kOk; }
  bool IsCorruption() const { return code_ == kCorruption; }
  Code code() const { return code_; }
  const std::string& message() const { return msg_; }
  // kv::Status::ToString() style: "Corruption: block checksum mismatch"
  std::string ToString() const {
    static const char* const kName[] = {"OK", "NotFound: ", "Corruption: ", "Not implemented: ",
                                        "Invalid argument: ", "IO error: "};
    return code_ == kOk ? "OK" : std::string(kName[code_]) + msg_;
  }

 private:
  Status(Code c, std::string m) : code_(c), msg_(std::move(m)) {}
  Code code_ = kOk;
  std::string msg_;
};

}  // namespace wipdb
