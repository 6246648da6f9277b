"""Batched table layer (SURVEY.md 8f-1 write side, 8f-2 read side) against the
reference's own table code (oracle/_ref/libref_table.so: kv::TableBuilder,
Table::Open, ReadBlock compiled from /root/reference/kv/src).

Write side: the SST bytes of wipdb::table::TableBuilder -- block CRCs
deferred and computed in batches -- equal kv::TableBuilder's bytes for the
same (key, value) stream, over block sizes, restart intervals, bloom filters,
mid-table buffer flushes and multi-table FinishTables.
Read side: the batched verifier returns the reference's status for clean
images and for seeded single-byte corruptions, and ReadBlock agrees block by
block.  CPU modes run here; the MI355X modes are the `gpu` tests at the end.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from wipdb_amd import sst

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_TABLE_SO = os.path.join(REPO, "oracle", "_ref", "libref_table.so")
KV_BUILDER_TEST = os.path.join(REPO, "oracle", "_ref", "test_kv_builder")


class RefTable:
    """ctypes view of oracle/_ref/libref_table.so (test infrastructure)."""

    def __init__(self, path: str = REF_TABLE_SO):
        lib = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.ref_build_table.restype = ctypes.c_long
        lib.ref_build_table.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, vp, sz]
        lib.ref_build_table_ex.restype = ctypes.c_long
        lib.ref_build_table_ex.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, vp, sz]
        lib.ref_internal_compare.restype = ctypes.c_int
        lib.ref_internal_compare.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        lib.ref_merge_tables.restype = ctypes.c_int
        lib.ref_merge_tables.argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_int, vp, sz, vp, vp,
                                         sz, vp, sz, ctypes.POINTER(sz)]
        lib.ref_filter_may_match.restype = ctypes.c_int
        lib.ref_filter_may_match.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz,
                                             ctypes.c_int, ctypes.c_int]
        lib.ref_verify_table.restype = ctypes.c_int
        lib.ref_verify_table.argtypes = [vp, sz, ctypes.c_int, ctypes.POINTER(sz)]
        lib.ref_read_block.restype = ctypes.c_int
        lib.ref_read_block.argtypes = [vp, sz, ctypes.c_uint64, ctypes.c_uint64]
        self.lib = lib

    def build(self, kvs, block_size=4096, restart=16, bloom=0, internal=False) -> bytes:
        keys = b"".join(k for k, _ in kvs)
        vals = b"".join(v for _, v in kvs)
        kl = np.array([len(k) for k, _ in kvs] or [0], np.uint32)
        vl = np.array([len(v) for _, v in kvs] or [0], np.uint32)
        cap = 2 * (len(keys) + len(vals)) + 8192 + 64 * len(kvs)
        out = ctypes.create_string_buffer(cap)
        kb = ctypes.create_string_buffer(keys, len(keys) or 1)
        vb = ctypes.create_string_buffer(vals, len(vals) or 1)
        n = self.lib.ref_build_table_ex(kb, kl.ctypes.data, vb, vl.ctypes.data, len(kvs),
                                        block_size, restart, bloom, int(internal), out, cap)
        assert 0 < n <= cap
        return out.raw[:n]

    def verify(self, img: bytes, bloom=0) -> int:
        b = ctypes.create_string_buffer(img, len(img) or 1)
        nb = ctypes.c_size_t(0)
        return int(self.lib.ref_verify_table(b, len(img), bloom, ctypes.byref(nb)))

    def merge(self, imgs, internal=True, verify=True):
        """MakeInputIteratorKV over the images: (status code, entries)."""
        bufs = [ctypes.create_string_buffer(i, len(i) or 1) for i in imgs]
        ptrs = (ctypes.c_void_p * max(len(imgs), 1))(*[ctypes.addressof(b) for b in bufs])
        sizes = np.array([len(i) for i in imgs] or [0], np.uint64)
        cap = sum(len(i) for i in imgs) * 4 + 4096
        ko, vo = ctypes.create_string_buffer(cap), ctypes.create_string_buffer(cap)
        kl, vl = np.zeros(cap // 4, np.uint32), np.zeros(cap // 4, np.uint32)
        ne = ctypes.c_size_t(0)
        rc = self.lib.ref_merge_tables(ptrs, sizes.ctypes.data, len(imgs), int(internal),
                                       int(verify), ko, cap, kl.ctypes.data, vo, cap,
                                       vl.ctypes.data, cap // 4, ctypes.byref(ne))
        assert rc >= 0
        k, v, out, a, b = ko.raw, vo.raw, [], 0, 0
        for i in range(ne.value):
            out.append((k[a:a + int(kl[i])], v[b:b + int(vl[i])]))
            a += int(kl[i])
            b += int(vl[i])
        return rc, out

    def merge_seconds(self, imgs, internal=True, reps=3) -> float:
        """best time of the native merge call alone (buffers prepared once)"""
        import time
        bufs = [ctypes.create_string_buffer(i, len(i) or 1) for i in imgs]
        ptrs = (ctypes.c_void_p * len(imgs))(*[ctypes.addressof(b) for b in bufs])
        sizes = np.array([len(i) for i in imgs], np.uint64)
        cap = sum(len(i) for i in imgs) * 4 + 4096
        ko, vo = ctypes.create_string_buffer(cap), ctypes.create_string_buffer(cap)
        kl, vl = np.zeros(cap // 4, np.uint32), np.zeros(cap // 4, np.uint32)
        ne = ctypes.c_size_t(0)
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            rc = self.lib.ref_merge_tables(ptrs, sizes.ctypes.data, len(imgs), int(internal), 1, ko,
                                           cap, kl.ctypes.data, vo, cap, vl.ctypes.data, cap // 4,
                                           ctypes.byref(ne))
            best = min(best, time.perf_counter() - t0)
            assert rc == 0
        return best

    def read_block(self, img: bytes, off: int, size: int) -> int:
        b = ctypes.create_string_buffer(img, len(img) or 1)
        return int(self.lib.ref_read_block(b, len(img), off, size))


# "reference": kv/src's table code with its own util/crc32c.cc;
# "dropin": the same unchanged sources with util/crc32c.cc left out, every
# kv::crc32c::Extend they make resolved from libhip_crc32c_batch.so
# (oracle/Makefile DROPIN_SO) -- VERDICT r3 item 5: the reference's own
# callers (table_builder.cc:194-196, format.cc:91-99) on the product's Extend
# must give the same bytes and statuses, in every test below.
REF_DROPIN_SO = os.path.join(REPO, "oracle", "_ref", "libref_table_dropin.so")


@pytest.fixture(scope="module", params=["reference", "dropin"])
def ref_table(request):
    path = REF_TABLE_SO if request.param == "reference" else REF_DROPIN_SO
    if not os.path.exists(path):
        pytest.skip(f"{os.path.relpath(path, REPO)} not built (reference absent, no prebuilt copy)")
    return RefTable(path)


# ---- seeded (key, value) streams -------------------------------------------

def kv_8binsert(n: int, seed: int):
    """test_bench/8Binsert.sh shape: 16-byte user keys + 8-byte tag, 100-byte
    printable values (CompressibleString-like, kv/src/util/testutil.cc:34-46)."""
    rng = np.random.default_rng(seed)
    user = np.unique(rng.integers(0, 2**63, size=n * 2, dtype=np.int64))[:n]
    out = []
    for i, u in enumerate(sorted(int(x) for x in user)):
        tag = ((i + 1) << 8 | 1).to_bytes(8, "little")
        key = b"%016x" % u + tag
        val = bytes(rng.integers(32, 127, size=100, dtype=np.uint8))
        out.append((key, val))
    return out


def kv_mixed(n: int, seed: int):
    """Variable key/value sizes, long shared prefixes, 0xff bytes (separator
    edge cases), empty values and values larger than a block."""
    rng = np.random.default_rng(seed)
    keys = set()
    while len(keys) < n:
        kind = rng.integers(0, 4)
        if kind == 0:
            k = bytes(rng.integers(0, 256, size=int(rng.integers(1, 40)), dtype=np.uint8))
        elif kind == 1:
            k = b"common/prefix/" + bytes(rng.integers(97, 100, size=int(rng.integers(1, 12)),
                                                       dtype=np.uint8))
        elif kind == 2:
            k = b"\xff" * int(rng.integers(1, 6)) + bytes([int(rng.integers(0, 256))])
        else:
            k = b"k%08d" % int(rng.integers(0, 10**8))
        keys.add(k)
    out = []
    for k in sorted(keys):
        r = rng.random()
        vl = 0 if r < 0.05 else (int(rng.integers(4200, 9000)) if r < 0.08 else int(rng.integers(1, 300)))
        out.append((k, bytes(rng.integers(0, 256, size=vl, dtype=np.uint8))))
    return out


def _tag(seq: int, typ: int) -> bytes:
    """PackSequenceAndType (kv/src/db/dbformat.cc:12-16), fixed64."""
    return ((seq << 8) | typ).to_bytes(8, "little")


def kv_internal(n: int, seed: int, dup: bool = True):
    """Internal keys as a flush / compaction writes them: user keys of every
    shape kv_mixed makes (0xff runs, shared prefixes, keys that are prefixes
    of others), each with 1..3 versions (sequence descending, puts and
    deletions), ordered by InternalKeyComparator(BytewiseComparator)."""
    rng = np.random.default_rng(seed)
    users = sorted({k for k, _ in kv_mixed(n, seed + 1000)} | {b"ab", b"abc", b"abd", b"b"})
    out, seq = [], 1 << 40
    for u in users:
        for _ in range(int(rng.integers(1, 4)) if dup else 1):
            seq -= int(rng.integers(1, 1000))
            typ = 0 if rng.random() < 0.1 else 1
            vl = 0 if typ == 0 else int(rng.integers(1, 300))
            out.append((u + _tag(seq, typ), bytes(rng.integers(0, 256, size=vl, dtype=np.uint8))))
    return out


def kv_8binsert_internal(n: int, seed: int):
    """8Binsert's DB tables: 16-byte hex user keys + tag, 100-byte values."""
    return kv_8binsert(n, seed)


CONFIGS = [
    # (stream, n, seed, block_size, restart, bloom, max_buffer)
    ("8binsert", 6000, 1, 4096, 16, 10, 4 << 20),
    ("8binsert", 6000, 2, 4096, 16, 0, 4 << 20),
    ("mixed", 3000, 3, 4096, 16, 10, 4 << 20),
    ("mixed", 3000, 4, 1024, 1, 10, 64 << 10),   # buffer flushes mid-table
    ("mixed", 2000, 5, 256, 4, 7, 4 << 20),
    ("8binsert", 1, 6, 4096, 16, 10, 4 << 20),   # a single entry
    ("8binsert", 0, 7, 4096, 16, 10, 4 << 20),   # an empty table
]


def _stream(kind, n, seed):
    return kv_8binsert(n, seed) if kind == "8binsert" else kv_mixed(n, seed)


# ---- write side -------------------------------------------------------------

@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
@pytest.mark.parametrize("cfg", CONFIGS, ids=[f"{c[0]}-{c[1]}-b{c[3]}-r{c[4]}-f{c[5]}" for c in CONFIGS])
def test_table_bytes_equal_reference(ref_table, cfg, mode):
    kind, n, seed, bs, rs, bloom, mb = cfg
    kvs = _stream(kind, n, seed)
    want = ref_table.build(kvs, bs, rs, bloom)
    rc, imgs, batched = sst.build_tables([kvs], bs, rs, bloom, mb, mode)
    assert rc == sst.OK
    assert imgs[0] == want
    if mode == sst.CRC_BATCH_CPU:
        assert batched > 0
    assert ref_table.verify(imgs[0], bloom) == 0


def test_finish_tables_matches_one_by_one(ref_table):
    """A compaction's outputs finished together (one CRC batch) are the same
    files the reference writes one at a time."""
    kvs = kv_8binsert(20000, 11)
    tables = [kvs[i:i + 2500] for i in range(0, len(kvs), 2500)]
    rc, imgs, batched = sst.build_tables(tables, bloom_bits=10, crc_mode=sst.CRC_BATCH_CPU)
    assert rc == sst.OK and len(imgs) == len(tables)
    for t, img in zip(tables, imgs):
        assert img == ref_table.build(t, bloom=10)
    assert batched == sum(len(_handles(img)) for img in imgs)


# ---- WipDB's DB tables: internal keys (db_impl.cc:141-144) -------------------

INTERNAL_CONFIGS = [
    # (stream, n, seed, block_size, restart, bloom)
    ("internal", 3000, 51, 4096, 16, 10),
    ("internal", 3000, 52, 1024, 4, 10),
    ("internal", 2000, 53, 256, 1, 7),
    ("8binsert", 6000, 54, 4096, 16, 10),
    ("8binsert", 6000, 55, 4096, 16, 0),
    ("internal", 1, 56, 4096, 16, 10),
]


def _istream(kind, n, seed):
    return kv_8binsert_internal(n, seed) if kind == "8binsert" else kv_internal(n, seed)


def test_internal_comparator_order_matches_reference(ref_table):
    """The streams are sorted the way the reference's InternalKeyComparator
    sorts them (user key ascending, sequence descending)."""
    kvs = kv_internal(1500, 50)
    for (a, _), (b, _) in zip(kvs, kvs[1:]):
        assert ref_table.lib.ref_internal_compare(a, len(a), b, len(b)) < 0


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
@pytest.mark.parametrize("cfg", INTERNAL_CONFIGS,
                         ids=[f"{c[0]}-{c[1]}-b{c[3]}-r{c[4]}-f{c[5]}" for c in INTERNAL_CONFIGS])
def test_internal_key_tables_equal_reference(ref_table, cfg, mode):
    """Byte parity with kv::TableBuilder under the DB's options:
    InternalKeyComparator separators / successors (the shortened user key +
    (kMaxSequenceNumber, kValueTypeForSeek)) and user-key bloom filters."""
    kind, n, seed, bs, rs, bloom = cfg
    kvs = _istream(kind, n, seed)
    want = ref_table.build(kvs, bs, rs, bloom, internal=True)
    rc, imgs, batched = sst.build_tables([kvs], bs, rs, bloom, crc_mode=mode,
                                         key_format=sst.KEYS_INTERNAL)
    assert rc == sst.OK
    assert imgs[0] == want
    assert ref_table.verify(imgs[0], bloom) == 0


def test_internal_key_format_changes_index_and_filter(ref_table):
    """The internal-key options are not the default ones: the same stream
    built bytewise has different index separators and filter bits (so a
    bytewise-only builder would not be a drop-in for the DB's tables).  The
    8Binsert shape (fixed-size unique user keys) is sorted in both orders."""
    kvs = kv_8binsert(3000, 57)
    a = ref_table.build(kvs, bloom=10, internal=True)
    b = ref_table.build(kvs, bloom=10, internal=False)
    assert a != b
    _, (ia,), _ = sst.build_tables([kvs], bloom_bits=10, crc_mode=sst.CRC_BATCH_CPU,
                                   key_format=sst.KEYS_INTERNAL)
    _, (ib,), _ = sst.build_tables([kvs], bloom_bits=10, crc_mode=sst.CRC_BATCH_CPU)
    assert ia == a and ib == b


def test_internal_key_filter_matches_user_keys(ref_table):
    """The filter block of an internal-key table answers KeyMayMatch for every
    user key under the reference's InternalFilterPolicy (any tag)."""
    kvs = kv_internal(800, 58)
    _, (img,), _ = sst.build_tables([kvs], bloom_bits=10, crc_mode=sst.CRC_BATCH_CPU,
                                    key_format=sst.KEYS_INTERNAL)
    hs = _handles(img)
    fo, fs = hs[-1]  # the filter block (last handle found in the meta-index)
    blob = img[fo:fo + fs]
    # one 2 KiB-granular filter per data block start; the first filter covers
    # the first block's keys -- check them with the policy directly
    nf = (len(blob) - int.from_bytes(blob[-5:-1], "little") - 1) // 4
    off0 = int.from_bytes(blob[-5:-1], "little")
    first = blob[int.from_bytes(blob[off0:off0 + 4], "little"):
                 int.from_bytes(blob[off0 + 4:off0 + 8], "little") if nf > 1 else off0]
    k0 = kvs[0][0]
    other_tag = k0[:-8] + _tag(1, 1)
    for key in (k0, other_tag):
        assert ref_table.lib.ref_filter_may_match(first, len(first), key, len(key), 10, 1) == 1


@pytest.mark.parametrize("mode", [sst.CRC_BATCH_CPU])
def test_internal_key_compaction_outputs_one_batch(ref_table, mode):
    kvs = kv_internal(6000, 59)
    tables = [kvs[i:i + 1100] for i in range(0, len(kvs), 1100)]
    rc, imgs, _ = sst.build_tables(tables, bloom_bits=10, crc_mode=mode,
                                   key_format=sst.KEYS_INTERNAL)
    assert rc == sst.OK
    for t, img in zip(tables, imgs):
        assert img == ref_table.build(t, bloom=10, internal=True)


def _run_kv_builder(mode: int):
    """tests/cpp/test_kv_builder.cc: the patched BuildTableKV / compaction
    (kvcompat::WritableFileWriterSink over kv::WritableFileWriter) against
    kv::TableBuilder under the DB's options, and kv::Table reading it back."""
    if not os.path.exists(KV_BUILDER_TEST):
        pytest.skip("oracle/_ref/test_kv_builder not built (reference absent)")
    r = subprocess.run([KV_BUILDER_TEST, str(mode)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "6 identical" in r.stdout and "identical" in r.stdout.splitlines()[0]


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
def test_kv_builder_integration(mode):
    _run_kv_builder(mode)


# ---- the leveldb/table adapter (include/wipdb_compat/leveldb_table_sink.h) --

LEVELDB_INCLUDE = "/root/reference/leveldb/include"
LEVELDB_ADAPTER_PREBUILT = os.path.join(REPO, "oracle", "_ref", "test_leveldb_adapter")


@pytest.fixture(scope="module")
def leveldb_adapter():
    """tests/cpp/test_leveldb_adapter.cc, built by oracle/Makefile against
    leveldb's headers, leveldb's table code compiled in place (its real
    comparators and bloom filter) and this library."""
    if not os.path.exists(LEVELDB_ADAPTER_PREBUILT):
        pytest.skip("oracle/_ref/test_leveldb_adapter not built (reference absent, no prebuilt copy)")
    return LEVELDB_ADAPTER_PREBUILT


LEVELDB_CONFIGS = [("8binsert", 3000, 4096, 16, 10, False), ("mixed", 1500, 1024, 4, 0, False),
                   ("internal", 2500, 4096, 16, 10, True), ("internal", 800, 256, 1, 7, True)]

# leveldb's own table code compiled in place (oracle/Makefile LDB_SO; VERDICT
# r4 item 5), and the same sources with util/crc32c.cc left out, linked to
# this library's leveldb::crc32c::Extend (LDB_DROPIN_SO)
REF_LEVELDB_SO = os.path.join(REPO, "oracle", "_ref", "libref_leveldb.so")
REF_LEVELDB_DROPIN_SO = os.path.join(REPO, "oracle", "_ref", "libref_leveldb_dropin.so")


class RefLevelDB:
    """ctypes view of oracle/_ref/libref_leveldb*.so: leveldb::TableBuilder
    (leveldb/table/table_builder.cc:185-187), Table::Open + a verified
    iteration, ReadBlock (format.cc:91-92).  Test infrastructure."""

    def __init__(self, path):
        lib = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.ldb_build_table_ex.restype = ctypes.c_long
        lib.ldb_build_table_ex.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, vp, sz]
        lib.ldb_verify_table.restype = ctypes.c_int
        lib.ldb_verify_table.argtypes = [vp, sz, ctypes.c_int, ctypes.c_int, ctypes.POINTER(sz)]
        lib.ldb_read_block.restype = ctypes.c_int
        lib.ldb_read_block.argtypes = [vp, sz, ctypes.c_uint64, ctypes.c_uint64]
        lib.ldb_crc32c_value.restype = ctypes.c_uint32
        lib.ldb_crc32c_value.argtypes = [ctypes.c_char_p, sz]
        self.lib = lib

    def build(self, kvs, block_size=4096, restart=16, bloom=0, internal=False) -> bytes:
        keys = b"".join(k for k, _ in kvs)
        vals = b"".join(v for _, v in kvs)
        kl = np.array([len(k) for k, _ in kvs] or [0], np.uint32)
        vl = np.array([len(v) for _, v in kvs] or [0], np.uint32)
        cap = 2 * (len(keys) + len(vals)) + 8192 + 64 * len(kvs)
        out = ctypes.create_string_buffer(cap)
        kb = ctypes.create_string_buffer(keys, len(keys) or 1)
        vb = ctypes.create_string_buffer(vals, len(vals) or 1)
        n = self.lib.ldb_build_table_ex(kb, kl.ctypes.data, vb, vl.ctypes.data, len(kvs),
                                        block_size, restart, bloom, int(internal), out, cap)
        assert 0 < n <= cap
        return out.raw[:n]

    def verify(self, img: bytes, bloom=0, internal=False) -> int:
        b = ctypes.create_string_buffer(img, len(img) or 1)
        nb = ctypes.c_size_t(0)
        return int(self.lib.ldb_verify_table(b, len(img), bloom, int(internal), ctypes.byref(nb)))

    def read_block(self, img: bytes, off: int, size: int) -> int:
        b = ctypes.create_string_buffer(img, len(img) or 1)
        return int(self.lib.ldb_read_block(b, len(img), off, size))


@pytest.fixture(scope="module", params=["leveldb", "leveldb-dropin"])
def ref_leveldb(request):
    path = REF_LEVELDB_SO if request.param == "leveldb" else REF_LEVELDB_DROPIN_SO
    if not os.path.exists(path):
        pytest.skip(f"{os.path.relpath(path, REPO)} not built (reference absent, no prebuilt copy)")
    return RefLevelDB(path)


def test_leveldb_reference_kat(ref_leveldb):
    """leveldb's crc32c compiled in place (and the product's, in the drop-in
    build) on the leveldb KAT (leveldb/util/crc32c_test.cc)."""
    assert ref_leveldb.lib.ldb_crc32c_value(b"123456789", 9) == 0xE3069283


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
@pytest.mark.parametrize("cfg", LEVELDB_CONFIGS, ids=[f"{c[0]}-b{c[2]}-r{c[3]}-f{c[4]}"
                                                       for c in LEVELDB_CONFIGS])
def test_leveldb_adapter_bytes_equal_reference(ref_table, leveldb_adapter, tmp_path, cfg, mode):
    _adapter_table(ref_table, leveldb_adapter, tmp_path, cfg, mode)


def _adapter_table(ref_table, leveldb_adapter, tmp_path, cfg, mode):
    """The leveldb/table call sites (leveldb/table/table_builder.cc:185-187
    write side, format.cc:91-92 read side) through the adapter: a table
    written with WritableFileSink + TableOptionsFrom(leveldb::Options-shaped
    options), read back through ReadImage and VerifyTable, equals the
    reference's kv::TableBuilder file for the same entries and options (the
    leveldb and kv table formats coincide; leveldb's own TableBuilder is not
    compiled here, so its byte identity is parity-unpinned beyond that)."""
    kind, n, bs, restart, bloom, internal = cfg
    kvs = kv_internal(n, 31) if internal else _stream(kind, n, 31)
    blob = bytearray(len(kvs).to_bytes(4, "little"))
    for k, v in kvs:
        blob += len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v
    ent, out = tmp_path / "entries.bin", tmp_path / "out.sst"
    ent.write_bytes(bytes(blob))
    r = subprocess.run([leveldb_adapter, str(ent), str(out), str(bs), str(restart), str(bloom),
                        str(int(internal)), str(mode)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = out.read_bytes()
    # kv's reader accepts it (the framing is kv's; the index separators are
    # leveldb's comparator's, so the bytes are leveldb's, not kv's builder's)
    assert ref_table.verify(got, bloom) == 0
    return got, kvs


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
@pytest.mark.parametrize("cfg", LEVELDB_CONFIGS, ids=[f"{c[0]}-b{c[2]}-r{c[3]}-f{c[4]}"
                                                       for c in LEVELDB_CONFIGS])
def test_leveldb_adapter_bytes_equal_leveldb_builder(ref_table, ref_leveldb, leveldb_adapter,
                                                     tmp_path, cfg, mode):
    """the adapter's table equals the file leveldb's OWN
    TableBuilder writes (leveldb/table/table_builder.cc:185-187, compiled in
    place, and again with its crc32c taken from this library), and leveldb's
    Table::Open + verified iteration accepts it."""
    got, kvs = _adapter_table(ref_table, leveldb_adapter, tmp_path, cfg, mode)
    kind, n, bs, restart, bloom, internal = cfg
    assert got == ref_leveldb.build(kvs, block_size=bs, restart=restart, bloom=bloom,
                                    internal=internal)
    assert ref_leveldb.verify(got, bloom, internal) == 0


def test_read_block_statuses_match_leveldb(ref_leveldb):
    """ReadBlock's verdicts (leveldb/table/format.cc:91-92) on every block of
    a leveldb-built table, clean and with seeded damage in the contents, the
    type byte and the trailer: the library's read_block (batched CRC path)
    returns leveldb's status for each."""
    kvs = kv_8binsert(4000, 23)
    img = ref_leveldb.build(kvs, bloom=10)
    rng = np.random.default_rng(24)
    for o, s in _handles(img):
        assert sst.read_block(img, o, s) == ref_leveldb.read_block(img, o, s) == sst.OK
        for where in (int(rng.integers(0, s)), s, s + 1, s + 4):  # contents, type, trailer
            b = bytearray(img)
            b[o + where] ^= 1 << int(rng.integers(0, 8))
            assert sst.read_block(bytes(b), o, s) == ref_leveldb.read_block(bytes(b), o, s)
    assert ref_leveldb.verify(img, 10) == 0
    # whole-table verification over seeded corruptions: the same verdicts
    for case in range(30):
        b = bytearray(img)
        b[int(rng.integers(0, len(b) - 48))] ^= 1 << int(rng.integers(0, 8))
        want = ref_leveldb.verify(bytes(b), 10)
        rc, codes = sst.verify_tables([bytes(b)], 10, sst.CRC_BATCH_CPU)
        assert codes[0] == want, case


# ---- the compaction input path (MakeInputIteratorKV) -----------------------

def _compaction_inputs(ntables: int, seed: int):
    """Overlapping input tables of one compaction: every table draws user
    keys from the whole range, some user keys appear in several tables with
    different sequence numbers (newer in lower-numbered tables), 1 KiB
    blocks so each table has many."""
    rng = np.random.default_rng(seed)
    users = sorted({b"user%010d" % int(x) for x in rng.integers(0, 10**9, 6000)})
    per = [[] for _ in range(ntables)]
    seq = 1 << 30
    for u in users:
        for t in sorted(rng.choice(ntables, size=int(rng.integers(1, 3)), replace=False)):
            seq -= int(rng.integers(1, 50))
            typ = 0 if rng.random() < 0.1 else 1
            val = b"" if typ == 0 else bytes(rng.integers(32, 127, size=int(rng.integers(8, 200)),
                                                          dtype=np.uint8))
            per[int(t)].append((u + _tag(seq, typ), val))
    ic = InternalOrder()
    for p in per:
        p.sort(key=ic)
    return per


class InternalOrder:
    """sort key of InternalKeyComparator(BytewiseComparator)"""
    def __call__(self, kv):
        k = kv[0]
        return (k[:-8], -int.from_bytes(k[-8:], "little"))


def _merge_inputs(ref_table, ntables, seed, block_size=1024):
    tables = _compaction_inputs(ntables, seed)
    return tables, [ref_table.build(t, block_size, 16, 10, internal=True) for t in tables]


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
@pytest.mark.parametrize("prefetch", [1, 7, 64])
def test_compaction_input_clean_matches_reference(ref_table, mode, prefetch):
    """Merged entries of 6 overlapping inputs equal the reference's merging
    iterator; the look-ahead checks batch many blocks per CRC call."""
    tables, imgs = _merge_inputs(ref_table, 6, 70)
    want_rc, want = ref_table.merge(imgs)
    rc, got, batches = sst.merge_tables(imgs, prefetch_blocks=prefetch, crc_mode=mode)
    assert rc == want_rc == sst.OK
    assert got == want and len(got) == sum(len(t) for t in tables)
    nblocks = sum(len(_handles(i)) - 2 for i in imgs)  # data blocks
    assert batches <= 1 + -(-nblocks // (prefetch * 6)) * 6 + 6


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
def test_compaction_input_corruptions_match_reference(ref_table, mode):
    """Seeded damage in data blocks, index blocks, footers and whole-image
    truncation: the same entries (failed blocks skipped) and the same
    status as the reference's merging iterator with paranoid_checks."""
    tables, imgs = _merge_inputs(ref_table, 4, 71)
    rng = np.random.default_rng(72)
    seen = set()
    for case in range(40):
        cur = list(imgs)
        for _ in range(int(rng.integers(1, 4))):
            t = int(rng.integers(0, len(cur)))
            b = bytearray(cur[t])
            kind = case % 4
            if kind == 0 or kind == 1:  # anywhere in the body (mostly data blocks)
                b[int(rng.integers(0, len(b) - 48))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 2:  # the index block
                io, isz = _handles(cur[t])[1]
                b[io + int(rng.integers(0, isz + 5))] ^= 0x04
            else:  # truncation or a footer byte
                if rng.random() < 0.5:
                    b = b[:int(rng.integers(0, len(b)))]
                else:
                    b[len(b) - 1 - int(rng.integers(0, 48))] ^= 0x80
            cur[t] = bytes(b)
        want_rc, want = ref_table.merge(cur)
        rc, got, _ = sst.merge_tables(cur, prefetch_blocks=int(rng.integers(1, 40)), crc_mode=mode)
        assert (rc, got) == (want_rc, want), case
        seen.add(want_rc)
    assert {sst.CRC_MISMATCH, sst.CORRUPTION} <= seen


def test_compaction_input_without_checksums_matches_reference(ref_table):
    """paranoid_checks off: no block CRC at all, the same merged stream."""
    _, imgs = _merge_inputs(ref_table, 5, 73)
    want_rc, want = ref_table.merge(imgs, verify=False)
    rc, got, batches = sst.merge_tables(imgs, verify=False, crc_mode=sst.CRC_BATCH_CPU)
    assert (rc, got) == (want_rc, want) and batches == 0


# (the merge rate against the reference's merging iterator is measured by
# scripts/bench_host_rates.py, which prints it)


def _sst_stream(tables: int, per_table: int, seed: int):
    """tables x per_table entries: 16-hex-digit user keys + an 8-byte tag,
    100-byte printable values (bench_layers' compaction stream)"""
    rng = np.random.default_rng(seed)
    n = tables * per_table
    user = np.sort(rng.choice(2**62, size=n, replace=False).astype(np.uint64))
    keys = bytearray()
    for i, u in enumerate(user.tolist()):
        keys += b"%016x" % u + ((i + 1) << 8 | 1).to_bytes(8, "little")
    vals = rng.integers(32, 127, size=n * 100, dtype=np.uint8).tobytes()
    return (np.full(tables, per_table, np.uint64), bytes(keys), np.full(n, 24, np.uint32), vals,
            np.full(n, 100, np.uint32))


# ---- read side --------------------------------------------------------------

def _handles(img: bytes):
    """(offset, size) of every block of a table image: data blocks from the
    index, plus index, meta-index and filter (parsed in Python)."""
    def varint(b, p):
        r = s = 0
        while True:
            x = b[p]
            p += 1
            r |= (x & 0x7F) << s
            s += 7
            if x < 0x80:
                return r, p

    def entries(block):
        nr = int.from_bytes(block[-4:], "little")
        lim = len(block) - 4 * (nr + 1)
        p, key, out = 0, b"", []
        while p < lim:
            sh, p = varint(block, p)
            ns, p = varint(block, p)
            vl, p = varint(block, p)
            key = key[:sh] + block[p:p + ns]
            out.append((key, block[p + ns:p + ns + vl]))
            p += ns + vl
        return out

    f = img[-48:]
    mo, p = varint(f, 0)
    ms, p = varint(f, p)
    io, p = varint(f, p)
    isz, p = varint(f, p)
    hs = [(mo, ms), (io, isz)]
    for _, v in entries(img[io:io + isz]):
        o, q = varint(v, 0)
        s, q = varint(v, q)
        hs.append((o, s))
    for k, v in entries(img[mo:mo + ms]):
        if k.startswith(b"filter."):
            o, q = varint(v, 0)
            s, q = varint(v, q)
            hs.append((o, s))
    return hs


@pytest.mark.parametrize("mode", [sst.CRC_INLINE, sst.CRC_BATCH_CPU])
def test_verify_clean_and_corrupted_match_reference(ref_table, mode):
    kvs = kv_mixed(2500, 21)
    img = ref_table.build(kvs, 1024, 16, 10)
    assert sst.verify_tables([img], 10, mode)[0] == sst.OK
    rng = np.random.default_rng(5)
    body = len(img) - 48  # footer corruptions are checked separately
    imgs, want = [], []
    for pos in rng.integers(0, body, size=150):
        b = bytearray(img)
        b[int(pos)] ^= 1 << int(rng.integers(0, 8))
        imgs.append(bytes(b))
        want.append(ref_table.verify(bytes(b), 10))
    # and inside every non-data block: index damage fails Open, meta-index
    # and filter damage is ignored (Table::ReadMeta, table.cc:84-138)
    for o, s in _handles(img)[:2] + _handles(img)[-1:]:
        for d in (0, s // 2, s, s + 1):
            b = bytearray(img)
            b[o + d] ^= 0x20
            imgs.append(bytes(b))
            want.append(ref_table.verify(bytes(b), 10))
    rc, codes = sst.verify_tables(imgs, 10, mode)
    assert codes == want
    assert sst.CRC_MISMATCH in want and sst.OK in want


def test_verify_footer_and_truncation(ref_table):
    img = ref_table.build(kv_8binsert(3000, 31), bloom=10)
    cases = [img[:40], img[:-1], img[:len(img) // 2] + img[-48:]]
    for pos in range(len(img) - 48, len(img)):
        b = bytearray(img)
        b[pos] ^= 0x40
        cases.append(bytes(b))
    _, codes = sst.verify_tables(cases, 10, sst.CRC_BATCH_CPU)
    for c, got in zip(cases, codes):
        want = ref_table.verify(c, 10)
        assert (got == sst.OK) == (want == sst.OK), (len(c), got, want)


def test_read_block_matches_reference(ref_table):
    img = ref_table.build(kv_mixed(1500, 41), 2048, 16, 10)
    hs = _handles(img)
    rng = np.random.default_rng(9)
    for o, s in hs:
        assert sst.read_block(img, o, s) == ref_table.read_block(img, o, s) == sst.OK
        for d in (-1, 1, 7):
            assert sst.read_block(img, o + d, s) == ref_table.read_block(img, o + d, s)
    for _ in range(200):
        o, s = int(rng.integers(0, len(img))), int(rng.integers(0, 5000))
        assert sst.read_block(img, o, s) == ref_table.read_block(img, o, s)


def test_verify_many_tables_one_batch(ref_table):
    tables = [kv_8binsert(1500, 100 + i) for i in range(12)]
    imgs = [ref_table.build(t, bloom=10) for t in tables]
    bad = bytearray(imgs[5])
    bad[1000] ^= 4
    imgs[5] = bytes(bad)
    rc, codes, checked, nbad = sst.verify_tables(imgs, 10, sst.CRC_BATCH_CPU, count_blocks=True)
    assert codes == [ref_table.verify(i, 10) for i in imgs]
    assert codes[5] == sst.CRC_MISMATCH and rc == sst.CRC_MISMATCH
    assert nbad == 1 and checked == sum(len(_handles(i)) for i in imgs)


def test_c_abi_header_symbols_exported():
    from wipdb_amd import _lib
    lib = _lib.load()
    syms = sst.header_symbols()
    assert set(syms) == set(sst._PROTOS)
    assert all(hasattr(lib, s) for s in syms)


# ---- MI355X ------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONFIGS[:5], ids=[f"{c[0]}-{c[1]}-b{c[3]}" for c in CONFIGS[:5]])
def test_gpu_table_bytes_equal_reference(ref_table, cfg, engine):
    kind, n, seed, bs, rs, bloom, mb = cfg
    kvs = _stream(kind, n, seed)
    rc, imgs, batched = sst.build_tables([kvs], bs, rs, bloom, mb, sst.CRC_BATCH_GPU)
    assert rc == sst.OK and batched > 0
    assert imgs[0] == ref_table.build(kvs, bs, rs, bloom)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", LEVELDB_CONFIGS, ids=[f"{c[0]}-b{c[2]}-r{c[3]}-f{c[4]}"
                                                       for c in LEVELDB_CONFIGS])
def test_gpu_leveldb_adapter_bytes_equal_reference(ref_table, ref_leveldb, leveldb_adapter,
                                                   tmp_path, cfg, engine):
    """The leveldb/table call sites through the adapter (leveldb/table/
    table_builder.cc:185-187, format.cc:91-92) with the block CRCs batched on
    the MI355X (CRC_BATCH_GPU, write and verify side): the same bytes as the
    reference's kv::TableBuilder and as leveldb's own TableBuilder (compiled
    in place, and with its crc32c from this library), which accepts them."""
    got, kvs = _adapter_table(ref_table, leveldb_adapter, tmp_path, cfg, sst.CRC_BATCH_GPU)
    kind, n, bs, restart, bloom, internal = cfg
    assert got == ref_leveldb.build(kvs, block_size=bs, restart=restart, bloom=bloom,
                                    internal=internal)
    assert ref_leveldb.verify(got, bloom, internal) == 0


@pytest.mark.gpu
def test_gpu_compaction_outputs_one_batch(ref_table, engine):
    """64 SSTs of ~2 MiB (8Binsert shape) finished in one MI355X batch."""
    kvs = kv_8binsert(64 * 1200, 77)
    tables = [kvs[i:i + 1200] for i in range(0, len(kvs), 1200)]
    rc, imgs, batched = sst.build_tables(tables, bloom_bits=10, crc_mode=sst.CRC_BATCH_GPU)
    assert rc == sst.OK
    rc2, cpu_imgs, _ = sst.build_tables(tables, bloom_bits=10, crc_mode=sst.CRC_INLINE)
    assert imgs == cpu_imgs
    for i in (0, 31, 63):
        assert imgs[i] == ref_table.build(tables[i], bloom=10)


@pytest.mark.gpu
def test_gpu_verify_matches_reference(ref_table, engine):
    tables = [kv_mixed(1200, 200 + i) for i in range(6)]
    imgs = [ref_table.build(t, 1024, 16, 10) for t in tables]
    rng = np.random.default_rng(3)
    for i in range(len(imgs)):
        for _ in range(8):
            b = bytearray(imgs[i])
            b[int(rng.integers(0, len(b) - 48))] ^= 0x10
            imgs.append(bytes(b))
    rc, codes = sst.verify_tables(imgs, 10, sst.CRC_BATCH_GPU)
    assert codes == [ref_table.verify(i, 10) for i in imgs]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", INTERNAL_CONFIGS[:4],
                         ids=[f"{c[0]}-{c[1]}-b{c[3]}" for c in INTERNAL_CONFIGS[:4]])
def test_gpu_internal_key_tables_equal_reference(ref_table, cfg, engine):
    """WipDB's DB tables (internal keys, InternalFilterPolicy) with every
    block CRC computed on the MI355X: bytes equal the reference's."""
    kind, n, seed, bs, rs, bloom = cfg
    kvs = _istream(kind, n, seed)
    rc, imgs, batched = sst.build_tables([kvs], bs, rs, bloom, crc_mode=sst.CRC_BATCH_GPU,
                                         key_format=sst.KEYS_INTERNAL)
    assert rc == sst.OK and batched > 0
    assert imgs[0] == ref_table.build(kvs, bs, rs, bloom, internal=True)


@pytest.mark.gpu
def test_gpu_internal_key_compaction_outputs(ref_table, engine):
    """A compaction's 16 internal-key output tables finished in one MI355X batch."""
    kvs = kv_internal(16 * 700, 60)
    tables = [kvs[i:i + 700] for i in range(0, len(kvs), 700)]
    rc, imgs, batched = sst.build_tables(tables, bloom_bits=10, crc_mode=sst.CRC_BATCH_GPU,
                                         key_format=sst.KEYS_INTERNAL)
    assert rc == sst.OK and batched > 0
    for t, img in zip(tables, imgs):
        assert img == ref_table.build(t, bloom=10, internal=True)


@pytest.mark.gpu
def test_gpu_kv_builder_integration(engine):
    """The reference-side integration with every block CRC on the MI355X."""
    _run_kv_builder(sst.CRC_BATCH_GPU)


@pytest.mark.gpu
def test_gpu_verify_pinned_images_zero_copy(ref_table, engine):
    """Table images in pinned memory (sst.PinnedImages): the verify batch
    reads them zero-copy; statuses equal the reference's for clean and
    corrupted images."""
    tables = [kv_8binsert(1500, 300 + i) for i in range(8)]
    imgs = [ref_table.build(t, bloom=10) for t in tables]
    bad = bytearray(imgs[3])
    bad[2000] ^= 8
    imgs[3] = bytes(bad)
    want = [ref_table.verify(i, 10) for i in imgs]
    with sst.PinnedImages(imgs) as pin:
        rc, codes = sst.verify_tables_at(pin.addrs, pin.sizes, 10, sst.CRC_BATCH_GPU)
    assert codes == want and want[3] == sst.CRC_MISMATCH


@pytest.mark.gpu
def test_gpu_compaction_input_matches_reference(ref_table, engine):
    """The compaction input path with every look-ahead CRC batch on the
    MI355X: clean and damaged inputs give the reference's entries and status."""
    _, imgs = _merge_inputs(ref_table, 8, 74)
    want = ref_table.merge(imgs)
    rc, got, batches = sst.merge_tables(imgs, prefetch_blocks=64, crc_mode=sst.CRC_BATCH_GPU)
    assert (rc, got) == want and batches > 1
    rng = np.random.default_rng(75)
    for case in range(6):
        cur = list(imgs)
        t = int(rng.integers(0, len(cur)))
        b = bytearray(cur[t])
        b[int(rng.integers(0, len(b) - 48))] ^= 0x10
        cur[t] = bytes(b)
        rc, got, _ = sst.merge_tables(cur, prefetch_blocks=16, crc_mode=sst.CRC_BATCH_GPU)
        assert (rc, got) == ref_table.merge(cur), case


def test_dropin_build_takes_extend_from_the_product():
    """The drop-in build is what INTEGRATION.md section 1 describes: the
    reference's table / format / log sources with util/crc32c.cc removed
    (kv/src/util/CMakeLists.txt:69-77) link against libhip_crc32c_batch.so
    alone for kv::crc32c::Extend -- it is undefined in the drop-in library,
    which needs the product library, while the reference build defines its
    own."""
    if not os.path.exists(REF_DROPIN_SO):
        pytest.skip("oracle/_ref/libref_table_dropin.so not built")
    sym = "_ZN2kv6crc32c6ExtendEjPKcm"

    def nm(path, *flags):
        r = subprocess.run(["nm", "-D", *flags, path], capture_output=True, text=True, check=True)
        return {ln.split()[-1] for ln in r.stdout.splitlines() if ln.strip()}

    assert sym in nm(REF_DROPIN_SO, "--undefined-only")
    assert sym not in nm(REF_DROPIN_SO, "--defined-only")
    assert sym in nm(REF_TABLE_SO, "--defined-only")
    r = subprocess.run(["readelf", "-d", REF_DROPIN_SO], capture_output=True, text=True, check=True)
    assert "[libhip_crc32c_batch.so]" in r.stdout
    product = os.path.join(REPO, "wipdb_amd", "lib", "libhip_crc32c_batch.so")
    assert sym in nm(product, "--defined-only")
