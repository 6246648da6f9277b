"""ctypes binding of the hip_crc32c_batch C-ABI (include/hip_crc32c_batch.h).

This is exactly the binding a Python caller of the reference's CRC would add
(see INTEGRATION.md).  It loads the in-tree ``wipdb_amd/lib/libhip_crc32c_batch.so``
and fails loudly when it is missing: there is no pure-Python or CPU fallback
for the batch entry points.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# WIPDB_HCRC_LIB: load another build of the same library (kernel experiments
# compare variants in one GPU session); the default is the in-tree build.
LIB_PATH = os.environ.get("WIPDB_HCRC_LIB") or os.path.join(_HERE, "lib", "libhip_crc32c_batch.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hip_crc32c_batch.h")

HCRC_OK = 0
HCRC_ERR_INVALID = -1
HCRC_ERR_NO_DEVICE = -2
HCRC_ERR_NO_MEMORY = -3
HCRC_ERR_HIP = -4
HCRC_ERR_LAUNCH = -5
HCRC_ERR_MISMATCH = -6
HCRC_ERR_BOUNDS = -7
HCRC_ERR_KERNEL = -8

HCRC_HOST_PTRS = 0x0
HCRC_DEVICE_PTRS = 0x1
HCRC_MASK_OUTPUT = 0x2
HCRC_SPLIT_SMALL = 0x4
HCRC_SPLIT_LONG = 0x8
HCRC_BALANCE = 0x10
HCRC_PACKED = 0x20

_c = ctypes
_u32p = _c.POINTER(_c.c_uint32)
_u64p = _c.POINTER(_c.c_uint64)
_vp = _c.c_void_p
_sz = _c.c_size_t

# name -> (restype, argtypes); mirrors include/hip_crc32c_batch.h one to one
_PROTOS = {
    "hcrc_abi_version": (_c.c_int, []),
    "hcrc_device_count": (_c.c_int, [_c.POINTER(_c.c_int)]),
    "hcrc_strerror": (_c.c_char_p, [_c.c_int]),
    "hcrc_ctx_create": (_c.c_int, [_c.c_int, _c.POINTER(_vp)]),
    "hcrc_ctx_shared": (_c.c_int, [_c.c_int, _c.POINTER(_vp)]),
    "hcrc_ctx_destroy": (_c.c_int, [_vp]),
    "hcrc_ctx_stream": (_vp, [_vp]),
    "hcrc_ctx_device": (_c.c_int, [_vp]),
    "hcrc_batch": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, _c.c_int]),
    "hcrc_batch_async": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, _c.c_int, _vp]),
    "hcrc_batch_strided_async": (
        _c.c_int, [_vp, _vp, _c.c_uint64, _c.c_uint32, _c.c_uint32, _vp, _sz, _c.c_int, _vp]),
    "hcrc_verify_async": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "hcrc_verify_async_ex": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _c.c_int, _vp]),
    "hcrc_sync": (_c.c_int, [_vp, _vp]),
    "hcrc_ctx_check": (_c.c_int, [_vp]),
    "hcrc_stream_forget": (_c.c_int, [_vp, _vp]),
    "hcrc_batch_multi": (
        _c.c_int, [_c.POINTER(_c.c_int), _c.c_int, _vp, _vp, _vp, _vp, _vp, _sz, _c.c_int]),
    "hcrc_batch_multi_ex": (
        _c.c_int, [_c.POINTER(_c.c_int), _c.c_int, _vp, _vp, _vp, _vp, _vp, _sz, _c.c_int,
                   _c.POINTER(_c.c_int)]),
    "hcrc_host_alloc": (_c.c_int, [_sz, _c.POINTER(_vp)]),
    "hcrc_host_free": (_c.c_int, [_vp]),
    "hcrc_host_register": (_c.c_int, [_vp, _sz]),
    "hcrc_host_unregister": (_c.c_int, [_vp]),
    "hcrc_readstream_async": (_c.c_int, [_vp, _vp, _c.c_uint64, _c.c_uint32, _vp, _sz, _vp]),
    "hcrc_dma_ceiling_async": (_c.c_int, [_vp, _vp, _c.c_uint64, _c.c_uint32, _vp, _sz, _vp]),
    "hcrc_check_spans_async": (
        _c.c_int, [_vp, _c.c_uint64, _vp, _vp, _c.c_uint32, _sz, _vp, _vp]),
    "hcrc_check_spans": (
        _c.c_int, [_vp, _c.c_uint64, _vp, _vp, _c.c_uint32, _sz, _c.POINTER(_c.c_uint64)]),
    "hcrc_fill_splitmix64_async": (
        _c.c_int, [_vp, _vp, _c.c_uint64, _c.c_uint64, _c.c_uint64, _vp]),
    "hcrc_cpu_extend": (_c.c_uint32, [_c.c_uint32, _vp, _sz]),
    "hcrc_cpu_extend_portable": (_c.c_uint32, [_c.c_uint32, _vp, _sz]),
    "hcrc_cpu_batch": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _c.c_int, _c.c_int]),
    "hcrc_cpu_is_accelerated": (_c.c_int, []),
    "hcrc_mask": (_c.c_uint32, [_c.c_uint32]),
    "hcrc_unmask": (_c.c_uint32, [_c.c_uint32]),
}

_lib = None


class HcrcError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = load().hcrc_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


def header_symbols() -> list[str]:
    """Function names declared in include/hip_crc32c_batch.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(hcrc_\w+)\s*\(", text, re.M)))


def load() -> ctypes.CDLL:
    """Load the native library (once).  Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C wipdb_amd/csrc` (there is no fallback implementation)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _PROTOS.items():
        if os.environ.get("WIPDB_HCRC_LIB") and not hasattr(lib, name):
            continue  # an older experiment build: bind what it has
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != HCRC_OK:
        raise HcrcError(rc, what)
