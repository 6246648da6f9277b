"""Python mirror of the batched table layer (include/wipdb/table.h) through
its C-ABI (include/wipdb_sst.h).

    build_tables(tables, ...)   kv::TableBuilder's SST bytes, block CRCs in one batch
    verify_tables(images, ...)  Table::Open(paranoid) + verified iteration, batched
    read_block(image, off, n)   ReadBlock(verify_checksums)
    log_write(records, ...)     kv::log::Writer::AddRecord bytes, record CRCs in one batch
    log_read(images, ...)       kv::log::Reader::ReadRecord over whole logs, CRCs batched

Status codes follow wipdb_sst.h: 0 OK, 1 corruption, 2 checksum mismatch,
3 other; negative = API / device error (raised as SstError).
"""
from __future__ import annotations

import ctypes
import os
import re
import time
from typing import Sequence

import numpy as np

from . import _lib

HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "include", "wipdb_sst.h")

OK, CORRUPTION, CRC_MISMATCH, OTHER = 0, 1, 2, 3
ERR_INVALID, ERR_TOO_SMALL, ERR_DEVICE = -1, -2, -3
CRC_INLINE, CRC_BATCH_CPU, CRC_BATCH_GPU, CRC_BATCH_AUTO = 0, 1, 2, 3
KEYS_BYTEWISE, KEYS_INTERNAL = 0, 1

_c = ctypes
_vp, _sz = _c.c_void_p, _c.c_size_t
_PROTOS = {
    "wsst_build_tables": (_c.c_int, [_sz, _vp, _vp, _vp, _vp, _vp, _c.c_int, _c.c_int, _c.c_int,
                                     _sz, _c.c_int, _c.c_int, _vp, _sz, _vp, _vp, _vp]),
    "wsst_build_tables_ex": (_c.c_int, [_sz, _vp, _vp, _vp, _vp, _vp, _c.c_int, _c.c_int,
                                        _c.c_int, _sz, _c.c_int, _c.c_int, _c.c_int, _vp, _sz,
                                        _vp, _vp, _vp]),
    "wsst_read_block": (_c.c_int, [_vp, _sz, _c.c_uint64, _c.c_uint64]),
    "wsst_merge_tables": (_c.c_int, [_vp, _vp, _sz, _c.c_int, _c.c_int, _sz, _c.c_int, _c.c_int,
                                     _vp, _sz, _vp, _vp, _sz, _vp, _sz, _vp, _vp]),
    "wsst_verify_tables": (_c.c_int, [_vp, _vp, _sz, _c.c_int, _c.c_int, _c.c_int, _vp, _vp,
                                      _vp]),
    "wsst_log_write": (_c.c_int, [_vp, _vp, _sz, _c.c_int, _c.c_uint64, _c.c_int, _c.c_int, _vp,
                                  _sz, _vp]),
    "wsst_log_read": (_c.c_int, [_vp, _vp, _sz, _c.c_int, _c.c_int, _vp, _sz, _vp, _vp, _sz, _vp,
                                 _vp, _vp, _sz, _vp]),
}
_bound = None
# wall time of the last native call (the C-ABI call alone, no Python packing)
last_call_seconds = 0.0


class SstError(RuntimeError):
    pass


def header_symbols() -> list[str]:
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(wsst_\w+)\s*\(", text, re.M)))


def _load():
    global _bound
    if _bound is None:
        lib = _lib.load()
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _bound = lib
    return _bound


def _blob(items: Sequence[bytes]):
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    return b"".join(items), lens


def build_tables(tables: Sequence[Sequence[tuple[bytes, bytes]]], block_size: int = 4096,
                 restart_interval: int = 16, bloom_bits: int = 0,
                 max_buffer_size: int = 4 << 20, crc_mode: int = CRC_BATCH_AUTO,
                 device: int = 0, key_format: int = KEYS_BYTEWISE) -> tuple[int, list[bytes], int]:
    """Builds every table (a sorted list of (key, value)) and finishes them
    together.  Returns (status code, table images, blocks CRC'd in batches).
    key_format=KEYS_INTERNAL: WipDB's DB tables (internal keys with their
    8-byte tag, InternalKeyComparator + InternalFilterPolicy)."""
    entries = np.array([len(t) for t in tables], dtype=np.uint64)
    flat = [kv for t in tables for kv in t]
    keys, klen = _blob([k for k, _ in flat])
    vals, vlen = _blob([v for _, v in flat])
    return build_tables_raw(entries, keys, klen, vals, vlen, block_size, restart_interval,
                            bloom_bits, max_buffer_size, crc_mode, device, key_format)


def build_tables_raw(entries, keys: bytes, klen, vals: bytes, vlen, block_size: int = 4096,
                     restart_interval: int = 16, bloom_bits: int = 0,
                     max_buffer_size: int = 4 << 20, crc_mode: int = CRC_BATCH_AUTO,
                     device: int = 0, key_format: int = KEYS_BYTEWISE) -> tuple[int, list[bytes], int]:
    """build_tables over pre-packed blobs: entries[t] pairs for table t, keys
    and values concatenated with their uint32 lengths."""
    lib = _load()
    entries = np.ascontiguousarray(entries, dtype=np.uint64)
    klen = np.ascontiguousarray(klen, dtype=np.uint32)
    vlen = np.ascontiguousarray(vlen, dtype=np.uint32)
    n = entries.size
    cap = 2 * (len(keys) + len(vals)) + 4096 * (n + 1) + 64 * int(klen.size)
    out = _c.create_string_buffer(cap)
    offs = np.zeros(max(n, 1), np.uint64)
    sizes = np.zeros(max(n, 1), np.uint64)
    batched = _c.c_uint64(0)
    kbuf = _c.create_string_buffer(keys, len(keys) or 1)
    vbuf = _c.create_string_buffer(vals, len(vals) or 1)
    global last_call_seconds
    t0 = time.perf_counter()
    rc = lib.wsst_build_tables_ex(n, entries.ctypes.data, kbuf, klen.ctypes.data, vbuf,
                                  vlen.ctypes.data, block_size, restart_interval, bloom_bits,
                                  max_buffer_size, crc_mode, device, key_format, out, cap,
                                  offs.ctypes.data, sizes.ctypes.data, _c.byref(batched))
    last_call_seconds = time.perf_counter() - t0
    if rc < 0:
        raise SstError(f"wsst_build_tables_ex: {rc}")
    raw = out.raw
    imgs = [raw[int(offs[i]):int(offs[i] + sizes[i])] for i in range(n)]
    return rc, imgs, int(batched.value)


def verify_tables(images: Sequence[bytes], bloom_bits: int = 0, crc_mode: int = CRC_BATCH_AUTO,
                  device: int = 0, count_blocks: bool = False):
    """Returns (first status code, per-table codes[, blocks checked, bad blocks])."""
    bufs = [_c.create_string_buffer(im, len(im) or 1) for im in images]
    return verify_tables_at([_c.addressof(b) for b in bufs], [len(im) for im in images],
                            bloom_bits, crc_mode, device, count_blocks)


def verify_tables_at(addrs: Sequence[int], sizes: Sequence[int], bloom_bits: int = 0,
                     crc_mode: int = CRC_BATCH_AUTO, device: int = 0,
                     count_blocks: bool = False):
    """verify_tables over images already in memory at the given addresses
    (e.g. in pinned memory from PinnedImages, which the MI355X reads
    zero-copy)."""
    lib = _load()
    n = len(addrs)
    ptrs = (_c.c_void_p * max(n, 1))(*addrs)
    sizes = np.array(list(sizes) or [0], dtype=np.uint64)
    codes = np.zeros(max(n, 1), np.int32)
    chk, bad = _c.c_uint64(0), _c.c_uint64(0)
    global last_call_seconds
    t0 = time.perf_counter()
    rc = lib.wsst_verify_tables(ptrs, sizes.ctypes.data, n, bloom_bits, crc_mode, device,
                                codes.ctypes.data, _c.byref(chk) if count_blocks else None,
                                _c.byref(bad) if count_blocks else None)
    last_call_seconds = time.perf_counter() - t0
    if rc < 0:
        raise SstError(f"wsst_verify_tables: {rc}")
    if count_blocks:
        return rc, codes[:n].tolist(), int(chk.value), int(bad.value)
    return rc, codes[:n].tolist()


def merge_tables(images: Sequence[bytes], key_format: int = KEYS_INTERNAL, verify: bool = True,
                 prefetch_blocks: int = 64, crc_mode: int = CRC_BATCH_AUTO, device: int = 0):
    """The compaction input path (MakeInputIteratorKV): the merged entries of
    the tables, data blocks checked ahead of the merge in batches.  Returns
    (status code, [(key, value), ...], CRC batches issued)."""
    lib = _load()
    n = len(images)
    bufs = [_c.create_string_buffer(im, len(im) or 1) for im in images]
    ptrs = (_c.c_void_p * max(n, 1))(*[_c.addressof(b) for b in bufs])
    sizes = np.array([len(im) for im in images] or [0], dtype=np.uint64)
    cap = sum(len(im) for im in images) * 4 + 4096
    kout, vout = _c.create_string_buffer(cap), _c.create_string_buffer(cap)
    maxe = cap // 4
    kl, vl = np.zeros(maxe, np.uint32), np.zeros(maxe, np.uint32)
    ne, nb = _c.c_uint64(0), _c.c_uint64(0)
    global last_call_seconds
    t0 = time.perf_counter()
    rc = lib.wsst_merge_tables(ptrs, sizes.ctypes.data, n, key_format, int(verify),
                               prefetch_blocks, crc_mode, device, kout, cap, kl.ctypes.data,
                               vout, cap, vl.ctypes.data, maxe, _c.byref(ne), _c.byref(nb))
    last_call_seconds = time.perf_counter() - t0
    if rc < 0:
        raise SstError(f"wsst_merge_tables: {rc}")
    k, v = kout.raw, vout.raw
    out, ko, vo = [], 0, 0
    for i in range(int(ne.value)):
        out.append((k[ko:ko + int(kl[i])], v[vo:vo + int(vl[i])]))
        ko += int(kl[i])
        vo += int(vl[i])
    return rc, out, int(nb.value)


class PinnedImages:
    """Table images copied into one pinned host allocation (hcrc_host_alloc),
    the way a store would keep SST pages it checksums often: hcrc_batch
    needs no staging copy there (dense pieces of >= 8 MiB go through the
    copy engine, the rest is read zero-copy over PCIe)."""

    def __init__(self, images: Sequence[bytes]):
        from wipdb_amd import _lib as hl
        self._hl = hl.load()
        total = sum(len(i) for i in images) + 64 * len(images) + 64
        ptr = _c.c_void_p()
        hl.check(self._hl.hcrc_host_alloc(total, _c.byref(ptr)), "hcrc_host_alloc")
        self.ptr = ptr.value
        self.addrs, self.sizes = [], []
        at = self.ptr
        for im in images:
            _c.memmove(at, im, len(im))
            self.addrs.append(at)
            self.sizes.append(len(im))
            at += (len(im) + 63) // 64 * 64
        self.nbytes = sum(self.sizes)

    def close(self):
        if self.ptr:
            self._hl.hcrc_host_free(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_block(image: bytes, offset: int, size: int) -> int:
    lib = _load()
    buf = _c.create_string_buffer(image, len(image) or 1)
    return int(lib.wsst_read_block(buf, len(image), offset, size))


def log_write(records: Sequence[bytes], recycle: bool = False, log_number: int = 0,
              crc_mode: int = CRC_BATCH_AUTO, device: int = 0) -> bytes:
    lib = _load()
    blob, lens = _blob(list(records))
    cap = len(blob) + 11 * (len(records) + len(blob) // 32000 + 2) + 32768
    out = _c.create_string_buffer(cap)
    size = _c.c_uint64(0)
    b = _c.create_string_buffer(blob, len(blob) or 1)
    global last_call_seconds
    t0 = time.perf_counter()
    rc = lib.wsst_log_write(b, lens.ctypes.data if len(records) else None, len(records),
                            int(recycle), log_number, crc_mode, device, out, cap, _c.byref(size))
    last_call_seconds = time.perf_counter() - t0
    if rc != OK:
        raise SstError(f"wsst_log_write: {rc}")
    return out.raw[:size.value]


def log_read(images: Sequence[bytes], crc_mode: int = CRC_BATCH_AUTO, device: int = 0):
    """Per log: (records [(LastRecordOffset, bytes)], drops [(bytes, reason)])."""
    lib = _load()
    n = len(images)
    bufs = [_c.create_string_buffer(im, len(im) or 1) for im in images]
    ptrs = (_c.c_void_p * max(n, 1))(*[_c.addressof(b) for b in bufs])
    sizes = np.array([len(im) for im in images] or [0], dtype=np.uint64)
    total = int(sizes.sum())
    max_recs = total // 7 + 16
    rec_out = _c.create_string_buffer(total + 16)
    rec_lens = np.zeros(max_recs, np.uint32)
    rec_offs = np.zeros(max_recs, np.uint64)
    nrecs = np.zeros(max(n, 1), np.uint64)
    max_drops = total // 7 + 16
    drop_bytes = np.zeros(max_drops, np.uint64)
    reasons = _c.create_string_buffer(64 * max_drops)
    ndrops = np.zeros(max(n, 1), np.uint64)
    global last_call_seconds
    t0 = time.perf_counter()
    rc = lib.wsst_log_read(ptrs, sizes.ctypes.data, n, crc_mode, device, rec_out, total + 16,
                           rec_lens.ctypes.data, rec_offs.ctypes.data, max_recs,
                           nrecs.ctypes.data, drop_bytes.ctypes.data, reasons, max_drops,
                           ndrops.ctypes.data)
    last_call_seconds = time.perf_counter() - t0
    if rc != OK:
        raise SstError(f"wsst_log_read: {rc}")
    raw, rraw = rec_out.raw, reasons.raw
    out, r, d, used = [], 0, 0, 0
    for i in range(n):
        recs, drops = [], []
        for _ in range(int(nrecs[i])):
            ln = int(rec_lens[r])
            recs.append((int(rec_offs[r]), raw[used:used + ln]))
            used += ln
            r += 1
        for _ in range(int(ndrops[i])):
            drops.append((int(drop_bytes[d]), rraw[64 * d:64 * d + 64].split(b"\0")[0].decode()))
            d += 1
        out.append((recs, drops))
    return out
