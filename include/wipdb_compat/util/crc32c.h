// include/wipdb_compat/util/crc32c.h -- put include/wipdb_compat ahead of a
// source tree's own include path and every `#include "util/crc32c.h"` in
// kv/src, leveldb, pebblesdb/src and rocksdb resolves here: the same
// declarations (kv::crc32c, leveldb::crc32c, rocksdb::crc32c), served by
// libhip_crc32c_batch.so.
#pragma once
#include "../../wipdb/crc32c.h"
