"""Pin the oracle (oracle/crc32c_oracle.c) before trusting it.

Checks the C restatement against every known-answer vector the reference's
own tests hold for this path (rocksdb/util/crc32c_test.cc,
leveldb/util/crc32c_test.cc, leveldb/util/crc32c.cc:269-271) and against the
golden spans produced by the compiled reference (tests/golden/make_golden.py),
and -- when oracle/_ref is present -- against the reference itself on fresh
random spans.
"""
import numpy as np


def test_rfc3720_and_leveldb_kats(oracle, kats):
    for v in kats["rfc"]:
        data = np.frombuffer(bytes.fromhex(v["data_hex"]), dtype=np.uint8).copy()
        assert oracle.extend(0, data) == v["crc"], v["name"]


def test_folly_vectors_and_stitching(oracle, kats):
    f = kats["folly"]
    buf = oracle.folly_buffer(f["buffer_size"])
    for v in f["vectors"]:
        off, n = v["offset"], v["length"]
        assert oracle.extend(0, buf, off, n) == v["crc"], (off, n)
        half = n // 2  # rocksdb/util/crc32c_test.cc:111-119
        first = oracle.extend(0, buf, off, half)
        assert oracle.extend(first, buf, off + half, n - half) == v["crc"]


def test_extend_and_mask(oracle, kats):
    e = kats["extend"]
    hello = np.frombuffer(b"hello ", dtype=np.uint8).copy()
    world = np.frombuffer(b"world", dtype=np.uint8).copy()
    assert oracle.extend(0, hello) == e["hello_"]
    assert oracle.extend(oracle.extend(0, hello), world) == e["hello_world"]
    m = kats["mask"]
    foo = np.frombuffer(b"foo", dtype=np.uint8).copy()
    crc = oracle.extend(0, foo)
    assert crc == m["foo_crc"]
    mk = int(oracle.lib.oracle_mask(crc))
    assert mk == m["foo_mask"] and mk != crc
    assert int(oracle.lib.oracle_mask(mk)) == m["foo_mask_mask"]
    assert int(oracle.lib.oracle_unmask(mk)) == crc
    assert int(oracle.lib.oracle_unmask(oracle.lib.oracle_unmask(m["foo_mask_mask"]))) == crc
    a = np.frombuffer(b"a", dtype=np.uint8).copy()
    assert oracle.extend(0, a) != crc  # CRC.Values, crc32c_test.cc:121-125


def test_survey_anchors(oracle, kats):
    pat = (np.arange(65536) & 0xFF).astype(np.uint8)
    a = kats["anchors"]
    assert oracle.extend(0, np.zeros(4096, np.uint8)) == a["zeros4096"]
    assert oracle.extend(0, np.full(4096, 0xFF, np.uint8)) == a["ones4096"]
    for n in (512, 1024, 2048, 4096, 8192, 16384, 32768, 65536):
        assert oracle.extend(0, pat, 0, n) == a[f"iota{n}"]
    blk = np.concatenate([pat[:4096], np.zeros(1, np.uint8)])
    assert oracle.extend(0, blk) == a["iota4096_type0"]
    assert int(oracle.lib.oracle_mask(a["iota4096_type0"])) == a["iota4096_type0_mask"]


def test_golden_spans(oracle, golden_spans):
    g = golden_spans
    got = oracle.batch(g["buf"], g["offsets"], g["lengths"], g["inits"])
    np.testing.assert_array_equal(got, g["crc"])
    got_m = oracle.batch(g["buf"], g["offsets"], g["lengths"], g["inits"], mask=True)
    np.testing.assert_array_equal(got_m, g["masked"])


def test_oracle_matches_compiled_reference(oracle, reference):
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 3000
    off = rng.integers(0, 1 << 19, n).astype(np.uint64)
    ln = np.where(rng.random(n) < 0.5, rng.integers(0, 64, n), rng.integers(0, 1 << 19, n)).astype(np.uint32)
    ini = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 2**32, n)).astype(np.uint32)
    np.testing.assert_array_equal(oracle.batch(buf, off, ln, ini), reference.batch(buf, off, ln, ini))
