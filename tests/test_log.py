"""Write-ahead log with batched record CRCs against the
reference's own kv::log::Writer / kv::log::Reader (oracle/_ref/libref_table.so,
compiled from /root/reference/kv/src/db/log_{writer,reader}.cc).

Writer: byte-identical log images (legacy and recyclable records, records
spanning blocks, empty records, block-tail padding).  Reader: the batched
recovery read returns the reference's records, LastRecordOffsets and
corruption reports (bytes dropped + reason) for clean logs, truncated logs and
seeded single-byte damage.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from wipdb_amd import sst

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_table.so")


class RefLog:
    def __init__(self, path: str = REF_SO):
        lib = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.ref_log_write.restype = ctypes.c_long
        lib.ref_log_write.argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_uint64, vp, sz]
        lib.ref_log_read.restype = ctypes.c_int
        lib.ref_log_read.argtypes = [vp, sz, ctypes.c_int, vp, sz, vp, vp, sz,
                                     ctypes.POINTER(sz), vp, vp, sz, ctypes.POINTER(sz)]
        self.lib = lib

    def write(self, recs, recycle=False, log_number=0) -> bytes:
        blob = b"".join(recs)
        lens = np.array([len(r) for r in recs] or [0], np.uint32)
        cap = len(blob) + 11 * (len(recs) + len(blob) // 32000 + 2) + 32768
        out = ctypes.create_string_buffer(cap)
        b = ctypes.create_string_buffer(blob, len(blob) or 1)
        n = self.lib.ref_log_write(b, lens.ctypes.data, len(recs), int(recycle), log_number,
                                   out, cap)
        assert 0 <= n <= cap
        return out.raw[:n]

    def read(self, img: bytes):
        total = len(img)
        mr = total // 7 + 16
        rec_out = ctypes.create_string_buffer(total + 16)
        lens = np.zeros(mr, np.uint32)
        offs = np.zeros(mr, np.uint64)
        db = np.zeros(mr, np.uint64)
        reasons = ctypes.create_string_buffer(64 * mr)
        nr, nd = ctypes.c_size_t(0), ctypes.c_size_t(0)
        b = ctypes.create_string_buffer(img, len(img) or 1)
        rc = self.lib.ref_log_read(b, len(img), 1, rec_out, total + 16, lens.ctypes.data,
                                   offs.ctypes.data, mr, ctypes.byref(nr), db.ctypes.data,
                                   reasons, mr, ctypes.byref(nd))
        assert rc == 0
        raw, rr = rec_out.raw, reasons.raw
        recs, used = [], 0
        for i in range(nr.value):
            recs.append((int(offs[i]), raw[used:used + int(lens[i])]))
            used += int(lens[i])
        drops = [(int(db[i]), rr[64 * i:64 * i + 64].split(b"\0")[0].decode())
                 for i in range(nd.value)]
        return recs, drops


    def seconds(self, recs, img: bytes, reps=3):
        """best native times of the reference's writer and reader alone"""
        import time
        blob = b"".join(recs)
        lens = np.array([len(r) for r in recs], np.uint32)
        b = ctypes.create_string_buffer(blob, len(blob) or 1)
        out = ctypes.create_string_buffer(len(img) + 1024)
        ib = ctypes.create_string_buffer(img, len(img))
        ro = ctypes.create_string_buffer(len(img))
        rl, rof = np.zeros(len(recs) + 8, np.uint32), np.zeros(len(recs) + 8, np.uint64)
        db, dr = np.zeros(16, np.uint64), ctypes.create_string_buffer(64 * 16)
        nr, nd = ctypes.c_size_t(0), ctypes.c_size_t(0)
        tw = tr = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            n = self.lib.ref_log_write(b, lens.ctypes.data, len(recs), 0, 9, out, len(img) + 1024)
            tw = min(tw, time.perf_counter() - t0)
            assert n == len(img)
            t0 = time.perf_counter()
            self.lib.ref_log_read(ib, len(img), 1, ro, len(img), rl.ctypes.data, rof.ctypes.data,
                                  len(recs) + 8, ctypes.byref(nr), db.ctypes.data, dr, 16,
                                  ctypes.byref(nd))
            tr = min(tr, time.perf_counter() - t0)
            assert nr.value == len(recs)
        return tw, tr


# "dropin": the reference's log_writer.cc / log_reader.cc with util/crc32c.cc
# left out, their kv::crc32c::Extend / Value calls resolved from
# libhip_crc32c_batch.so (oracle/Makefile DROPIN_SO)
REF_DROPIN_SO = os.path.join(REPO, "oracle", "_ref", "libref_table_dropin.so")


@pytest.fixture(scope="module", params=["reference", "dropin"])
def ref_log(request):
    path = REF_SO if request.param == "reference" else REF_DROPIN_SO
    if not os.path.exists(path):
        pytest.skip(f"{os.path.relpath(path, REPO)} not built (reference absent, no prebuilt copy)")
    return RefLog(path)


def records(n: int, seed: int):
    """WriteBatch-sized records: mostly small, some spanning 32 KiB blocks,
    some empty, lengths that land headers on block tails."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.05:
            ln = 0
        elif r < 0.12:
            ln = int(rng.integers(32768 - 40, 100000))
        elif r < 0.2:
            ln = int(rng.integers(32760 - 14, 32768))
        else:
            ln = int(rng.integers(1, 400))
        out.append(bytes(rng.integers(0, 256, size=ln, dtype=np.uint8)))
    return out


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
@pytest.mark.parametrize("recycle", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_log_bytes_equal_reference(ref_log, seed, recycle, mode):
    recs = records(300, seed)
    want = ref_log.write(recs, recycle, 77 + seed)
    got = sst.log_write(recs, recycle, 77 + seed, mode)
    assert got == want


def test_log_empty_and_tiny(ref_log):
    for recs in ([], [b""], [b"x"], [b""] * 5000):
        assert sst.log_write(recs, crc_mode=sst.CRC_BATCH_CPU) == ref_log.write(recs)


@pytest.mark.parametrize("seed", [4, 5])
def test_log_read_clean_matches_reference(ref_log, seed):
    recs = records(400, seed)
    img = ref_log.write(recs)
    (got, drops), = sst.log_read([img], sst.CRC_BATCH_CPU)
    want, wdrops = ref_log.read(img)
    assert got == want and drops == wdrops == []
    assert [r for _, r in got] == recs


def test_log_read_damage_matches_reference(ref_log):
    recs = records(250, 6)
    img = ref_log.write(recs)
    rng = np.random.default_rng(11)
    imgs = []
    for _ in range(120):
        b = bytearray(img)
        for _ in range(int(rng.integers(1, 3))):
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
        imgs.append(bytes(b))
    # truncations (a crash mid-write), zeroed tails (preallocated files),
    # a legacy reader over recyclable records ("checksum mismatch" on each)
    for cut in (1, 7, 100, 32768, 32775, len(img) // 2):
        imgs.append(img[:-cut])
    z = bytearray(img)
    z[len(z) // 3:] = bytes(len(z) - len(z) // 3)
    imgs.append(bytes(z))
    imgs.append(ref_log.write(recs[:40], recycle=True, log_number=9))
    got = sst.log_read(imgs, sst.CRC_BATCH_CPU)
    n_drop = 0
    for im, (grec, gdrop) in zip(imgs, got):
        wrec, wdrop = ref_log.read(im)
        assert grec == wrec
        assert gdrop == wdrop
        n_drop += len(wdrop)
    assert n_drop > 50


@pytest.mark.gpu
def test_gpu_log_write_and_recover(ref_log, engine):
    recs = records(3000, 21)
    want = ref_log.write(recs)
    assert sst.log_write(recs, crc_mode=sst.CRC_BATCH_GPU) == want
    imgs = [want]
    rng = np.random.default_rng(2)
    for _ in range(16):
        b = bytearray(want)
        b[int(rng.integers(0, len(b)))] ^= 0x08
        imgs.append(bytes(b))
    got = sst.log_read(imgs, sst.CRC_BATCH_GPU)
    for im, g in zip(imgs, got):
        assert g == ref_log.read(im)


# (host write / recovery rates against the reference's Writer / Reader are
# measured by scripts/bench_host_rates.py, which prints them: wall-clock
# comparisons do not belong in a correctness suite)
