"""wipdb_amd -- MI355X-native batched CRC32C for WipDB's table blocks.

The hot path of hansonzhao007/WipDB this package accelerates is the per-block
CRC32C that TableBuilder::WriteRawBlock stamps (kv/src/table/table_builder.cc:
183-202) and ReadBlock verifies (kv/src/table/format.cc:66-143).  The native
library (wipdb_amd/lib/libhip_crc32c_batch.so, sources in wipdb_amd/csrc/)
holds the gfx950 kernels, the C-ABI (include/hip_crc32c_batch.h) and the C++
surface (include/wipdb/crc32c.h); this package is its Python host mirror.
"""
from .crc32c import (  # noqa: F401
    MASK_DELTA,
    Engine,
    HcrcError,
    batch_multi,
    cpu_batch,
    device_count,
    extend,
    is_fast_crc32_supported,
    mask,
    unmask,
    value,
)

__version__ = "0.1.0"
