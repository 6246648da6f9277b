"""HCRC_PACKED's chunk index built on the host (hcrc_api.cc HostPsIndex, the
host pieces' path since round 6) against a numpy restatement of the device
pre-pass it replaces (crc32c_ps.h ps_index): the same verdict bits and, for a
packed piece, the same first[] -- on packed layouts (SST-like, aligned,
dense, WAL-like) and on every way to break the promise.  CPU only: the test
build of the library (build/testlib, WIPDB_HCRC_TEST_HOOKS) exports the
host function; no GPU call is made.
"""
import ctypes
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST_LIB = os.path.join(REPO, "build", "testlib", "libhip_crc32c_batch.so")

BAD, DENSE, SHORT = 1, 2, 4
META = 8


def ps_index_ref(off, ln, C):
    """crc32c_ps.h ps_index restated (verdict bits, first[C + 1], cb, lo)."""
    n = off.size
    lo = int(off[0])
    hi = int(off[-1]) + int(ln[-1])
    rng = max(hi - lo, 1)
    cb = -(-rng // C)
    cb = max(4096, (cb + 4095) & ~4095)
    bad = BAD if cb >> 44 else 0
    first = np.zeros(C + 1, np.int64)
    a = off.astype(np.int64)
    end = a + ln.astype(np.int64)
    c = (a - lo) // cb
    if (a < lo).any() or (c >= C).any():
        bad |= BAD
    if n > 1:
        gap = a[1:] - end[:-1]
        if (gap < 0).any() or (gap >= 4096).any():
            bad |= BAD
    if ((cb + ln.astype(np.int64) + 8192) >= 1 << 32).any():
        bad |= BAD
    if n > 62:
        d = a[62:] - a[:-62]
        if (d < 0).any():
            bad |= BAD
        elif (d < 4096).any():
            bad |= DENSE
    short = ln < 96
    for g in range(0, n, 64):
        m = short[g:g + 64]
        if m.sum() >= 32:
            bad |= SHORT
        run = 0
        for v in m:
            run = run + 1 if v else 0
            if run >= 8:
                bad |= SHORT
                break
    if bad == 0:
        # first[k] = the first span starting in chunk k (chunks without a start:
        # the next span that starts after them), first[C] = n
        for k in range(C + 1):
            first[k] = int(np.searchsorted(c, k, side="left"))
    return bad, first, cb, lo


@pytest.fixture(scope="module")
def host_index():
    if not os.path.exists(TEST_LIB):
        pytest.skip("the test build is made by make -C wipdb_amd/csrc (build/testlib)")
    lib = ctypes.CDLL(TEST_LIB)
    fn = lib.hcrc_test_host_ps_index
    fn.restype = ctypes.c_uint32
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                   ctypes.c_void_p]

    def call(off, ln, C):
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint32)
        ps = np.full(META + C + 1, 0xDEADBEEF, np.uint32)
        bits = fn(off.ctypes.data, ln.ctypes.data, off.size, C, ps.ctypes.data)
        return int(bits), ps
    return call


def lay(rng, n, lo, hi, gap, start=0):
    ln = rng.integers(lo, hi + 1, n).astype(np.uint64)
    off = start + np.concatenate([[0], np.cumsum(ln + gap)[:-1]]).astype(np.uint64)
    return off, ln.astype(np.uint32)


def cases(rng):
    yield "sst", lay(rng, 20000, 4097, 4225, 4)
    yield "512-2k", lay(rng, 20000, 512, 2200, 5, 3)
    yield "aligned4k", (np.arange(9000, dtype=np.uint64) * 4096, np.full(9000, 4096, np.uint32))
    yield "mixed_gaps", lay(rng, 9000, 0, 3000, 0, 11)
    yield "staged_like", lay(rng, 6000, 100, 9000, 17, 5)
    yield "long", lay(rng, 500, 1 << 16, 1 << 20, 3)
    yield "one", (np.array([7], np.uint64), np.array([300], np.uint32))
    o, ln = lay(rng, 5000, 300, 3000, 5)
    o2 = o.copy()
    o2[[10, 11]] = o2[[11, 10]]
    yield "unsorted", (o2, ln)
    o3 = o.copy()
    o3[500] -= 10
    yield "overlap", (o3, ln)
    o4 = o.copy()
    o4[700:] += 5000
    yield "gap5k", (o4, ln)
    yield "dense", lay(rng, 5000, 5, 60, 7)
    yield "wal", lay(rng, 5000, 40, 95, 7)
    yield "wal64", lay(rng, 5000, 64, 127, 7)
    o, ln = lay(rng, 20, 600, 800, 5)
    ln[10] = 2**32 - 64
    o[11:] += np.uint64(2**32)
    yield "huge", (o, ln)


@pytest.mark.parametrize("C", [16, 512, 4096])
def test_host_index_matches_device_prepass(host_index, C):
    rng = np.random.default_rng(C)
    for name, (off, ln) in cases(rng):
        bits, ps = host_index(off, ln, C)
        want_bits, want_first, cb, lo = ps_index_ref(off, ln, C)
        # (broken pieces: the host stops at the first broken span, the device
        # ORs the bits of whole steps -- the same verdict, a shared reason)
        assert (bits == 0) == (want_bits == 0), (name, C, bits, want_bits)
        assert bits == 0 or bits & want_bits, (name, C, bits, want_bits)
        assert ps[0] == (1 << 4 | bits), (name, ps[0])
        if bits == 0:
            assert ps[1] | (int(ps[2]) << 32) == cb, name
            assert ps[3] | (int(ps[4]) << 32) == lo, name
            np.testing.assert_array_equal(ps[META:META + C + 1].astype(np.int64), want_first,
                                          err_msg=f"{name} C={C}")
            # every span in exactly one chunk: first[] rises from 0 to n
            f = ps[META:META + C + 1].astype(np.int64)
            assert f[0] == 0 and f[-1] == off.size and (np.diff(f) >= 0).all(), name


def test_host_index_verdicts(host_index):
    rng = np.random.default_rng(4)
    got = {name: host_index(off, ln, 512)[0] for name, (off, ln) in cases(rng)}
    for k in ("sst", "512-2k", "aligned4k", "mixed_gaps", "staged_like", "long", "one"):
        assert got[k] == 0, (k, got[k])
    for k in ("unsorted", "overlap", "gap5k", "huge"):
        assert got[k] & BAD, (k, got[k])
    assert got["dense"] & (DENSE | SHORT), got["dense"]
    assert got["wal"] & SHORT and got["wal64"] & SHORT, got
