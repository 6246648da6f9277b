"""The copy engine's piece rules for pinned host batches (hcrc_api.cc
DensePiece, round 6) against a Python restatement, on the CPU: which spans
of a batch in pinned memory form a piece the copy engine moves (in address
order, inside one pinned range, at most 128 MiB of covering range, at most
an eighth + 64 KiB more than the span bytes, at least 8 MiB unless it ends
the batch behind a copied piece, at most 128 Ki spans) and which range it
copies (widened to the 256-byte grid inside the range).  The test build
(build/testlib) enters a host range as pinned without pinning it -- the
rules only do address arithmetic, so the ranges are fake addresses and no
memory is touched; no GPU call is made.
"""
import ctypes
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST_LIB = os.path.join(REPO, "build", "testlib", "libhip_crc32c_batch.so")

CAP = 128 << 20          # kDmaBytes
MIN = 8 << 20            # kDmaMinBytes
STAGE_SPANS = 1 << 17    # kStageSpans
BASE = 0x7A0000000000    # the fake ranges' addresses (never dereferenced)


def dense_ref(ranges, offs, lens, i, tail):
    """DensePiece restated: (j, a, b) with a, b offsets from BASE, or (i,)."""
    count = offs.size
    first = BASE + int(offs[i])
    rng = [(lo, hi) for lo, hi in ranges if lo <= first < hi]
    if not rng:
        return (i,)
    rlo, rhi = rng[0]
    lim = min(rhi, first - (first & 255) + CAP)
    hi = prev = first
    nbytes = 0
    j = i
    while j < count and j - i < STAGE_SPANS:
        lo = BASE + int(offs[j])
        end = lo + int(lens[j])
        if lo < prev or end > lim:
            break
        prev = lo
        hi = max(hi, end)
        nbytes += int(lens[j])
        j += 1
    if j == i or hi - first > nbytes + nbytes // 8 + (64 << 10):
        return (i,)
    if hi - first < MIN and not (tail and j == count):
        return (i,)
    a = max(rlo, first & ~255)
    b = min(rhi, (hi + 255) & ~255)
    return (j, a - BASE, b - BASE)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(TEST_LIB):
        pytest.skip("the test build is made by make -C wipdb_amd/csrc (build/testlib)")
    L = ctypes.CDLL(TEST_LIB)
    L.hcrc_test_fake_pinned_range.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.hcrc_test_dense_piece.restype = ctypes.c_size_t
    L.hcrc_test_dense_piece.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p]
    return L


class Ranges:
    def __init__(self, lib, spans):
        self.lib = lib
        self.spans = [(BASE + a, BASE + b) for a, b in spans]

    def __enter__(self):
        for lo, hi in self.spans:
            self.lib.hcrc_test_fake_pinned_range(lo, hi - lo)
        return self.spans

    def __exit__(self, *exc):
        for lo, _ in self.spans:
            self.lib.hcrc_test_fake_pinned_range(lo, 0)


def piece(lib, offs, lens, i, tail):
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    ab = (ctypes.c_uint64 * 2)()
    j = lib.hcrc_test_dense_piece(BASE, offs.ctypes.data, lens.ctypes.data, i, offs.size,
                                  int(tail), ab)
    return (j,) if j == i else (j, int(ab[0]), int(ab[1]))


def sst(rng, n, start=0, gap=4):
    lens = rng.integers(4097, 4226, n).astype(np.uint32)
    offs = (start + np.concatenate([[0], np.cumsum(lens.astype(np.int64) + gap)[:-1]])).astype(np.uint64)
    return offs, lens


def walk(lib, ranges, offs, lens):
    """Every piece of a batch as BatchZeroCopy cuts it (a zero-copy piece
    takes min(rest, 128 Ki) spans), the library against the restatement."""
    i, copying, out = 0, False, []
    while i < offs.size:
        got = piece(lib, offs, lens, i, copying)
        want = dense_ref(ranges, offs, lens, i, copying)
        assert got == want, (i, got, want)
        copying = len(got) > 1
        out.append(got)
        i = got[0] if copying else min(offs.size, i + STAGE_SPANS)
    return out


def test_sst_batches(lib):
    rng = np.random.default_rng(1)
    with Ranges(lib, [(0, 1 << 30)]) as rg:
        # one SST (~2 MiB): under the floor, zero-copy
        o, l = sst(rng, 500, 7)
        assert piece(lib, o, l, 0, False) == (0,)
        # ... but copied as the tail behind a copied piece
        assert piece(lib, o, l, 0, True)[0] == 500
        # 40 MiB: one piece to its end, the range widened to 256 bytes
        o, l = sst(rng, 10000, 77)
        j, a, b = piece(lib, o, l, 0, False)
        assert j == 10000 and a == 0 and b % 256 == 0 and b >= int(o[-1] + l[-1])
        # 600 MiB: 128 MiB pieces, the last one whatever is left
        o, l = sst(rng, 150000, 3)
        pieces = walk(lib, rg, o, l)
        assert all(len(p) == 3 for p in pieces) and len(pieces) == 5
        assert all(p[2] - p[1] <= CAP for p in pieces)


def test_order_density_and_ranges(lib):
    rng = np.random.default_rng(2)
    with Ranges(lib, [(0, 64 << 20), (64 << 20, 200 << 20), (300 << 20, (300 << 20) + 1000)]) as rg:
        o, l = sst(rng, 12000)            # ~50 MB inside the first range
        # an order break after 12 MiB: a piece up to it
        k = int(np.searchsorted(o, 12 << 20))
        o2 = o.copy()
        o2[[k, k + 1]] = o2[[k + 1, k]]
        assert piece(lib, o2, l, 0, False)[0] == k + 1
        # an order break after 1 MiB: no piece (zero-copy takes the rest)
        k = int(np.searchsorted(o, 1 << 20))
        o3 = o.copy()
        o3[[k, k + 1]] = o3[[k + 1, k]]
        assert piece(lib, o3, l, 0, False) == (0,)
        # sparse: 4 KiB spans 16 KiB apart
        o4 = np.arange(3000, dtype=np.uint64) * 16384
        assert piece(lib, o4, np.full(3000, 4096, np.uint32), 0, False) == (0,)
        # a batch across the boundary of two ranges: the piece stops at it
        o5, l5 = sst(rng, 12000, 40 << 20)
        got = piece(lib, o5, l5, 0, False)
        assert len(got) == 3 and got[2] <= 64 << 20
        assert int(o5[got[0]] + l5[got[0]]) > 64 << 20
        walk(lib, rg, o5, l5)
        # spans in no range, and a range too small for the floor
        assert piece(lib, np.array([250 << 20], np.uint64), np.array([100], np.uint32), 0, True) == (0,)
        assert piece(lib, np.array([(300 << 20) + 10], np.uint64), np.array([100], np.uint32), 0,
                     False) == (0,)
        # ... but a tail there is copied, clamped to the range
        assert piece(lib, np.array([(300 << 20) + 10], np.uint64), np.array([100], np.uint32), 0,
                     True) == (1, 300 << 20, (300 << 20) + 256)


def test_span_count_limit(lib):
    with Ranges(lib, [(0, 1 << 30)]):
        n = 200000                         # 100-byte spans back to back: 20 MB, 200 Ki spans
        o = np.arange(n, dtype=np.uint64) * 100
        l = np.full(n, 100, np.uint32)
        assert piece(lib, o, l, 0, False)[0] == STAGE_SPANS


def test_random_batches_match_the_restatement(lib):
    rng = np.random.default_rng(3)
    spans = [(0, 96 << 20), ((96 << 20) + 4096, 400 << 20)]
    with Ranges(lib, spans) as rg:
        for _ in range(40):
            n = int(rng.integers(1, 60000))
            lens = rng.integers(0, int(rng.choice([200, 5000, 70000])), n).astype(np.uint32)
            gaps = rng.integers(0, int(rng.choice([1, 64, 4096, 40000])), n)
            start = int(rng.integers(0, 300 << 20))
            offs = (start + np.concatenate([[0], np.cumsum(lens.astype(np.int64) + gaps)[:-1]]))
            keep = offs + lens < (400 << 20)
            offs, lens = offs[keep].astype(np.uint64), lens[keep]
            if offs.size == 0:
                continue
            if rng.random() < 0.3:         # a few order breaks
                for k in rng.integers(0, offs.size, 3):
                    if k + 1 < offs.size:
                        offs[[k, k + 1]] = offs[[k + 1, k]]
            walk(lib, rg, offs, lens)
