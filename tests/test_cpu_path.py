"""The library's host CPU path (crc32c_cpu.cc) and the Python mirror of the
kv::crc32c surface, checked against the oracle and the golden vectors.
CPU only: no device is touched."""
import numpy as np
import pytest

import wipdb_amd as w


def test_surface_kats(kats):
    for v in kats["rfc"]:
        assert w.value(bytes.fromhex(v["data_hex"])) == v["crc"], v["name"]
    e = kats["extend"]
    assert w.extend(w.value(b"hello "), b"world") == e["hello_world"] == w.value(b"hello world")
    crc = w.value(b"foo")
    assert w.mask(crc) == kats["mask"]["foo_mask"]
    assert w.unmask(w.mask(crc)) == crc
    assert w.unmask(w.unmask(w.mask(w.mask(crc)))) == crc
    assert w.MASK_DELTA == 0xA282EAD8
    assert w.is_fast_crc32_supported() in ("Supported on x86", "Not supported on x86")


def test_python_mask_matches_c():
    lib = w._lib.load()
    rng = np.random.default_rng(3)
    for c in rng.integers(0, 2**32, 200):
        c = int(c)
        assert w.mask(c) == lib.hcrc_mask(c)
        assert w.unmask(c) == lib.hcrc_unmask(c)


def test_folly_vectors(oracle, kats):
    f = kats["folly"]
    buf = oracle.folly_buffer(f["buffer_size"])
    for v in f["vectors"]:
        off, n = v["offset"], v["length"]
        assert w.extend(0, buf[off:off + n]) == v["crc"]


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_batch_golden(golden_spans, threads):
    g = golden_spans
    got = w.cpu_batch(g["buf"], g["offsets"], g["lengths"], g["inits"], threads=threads)
    np.testing.assert_array_equal(got, g["crc"])
    got = w.cpu_batch(g["buf"], g["offsets"], g["lengths"], g["inits"], mask_output=True,
                      threads=threads)
    np.testing.assert_array_equal(got, g["masked"])


def test_cpu_path_random_vs_oracle(oracle):
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    for _ in range(400):
        off = int(rng.integers(0, 4096))
        n = int(rng.integers(0, 40000))
        init = int(rng.integers(0, 2**32)) if rng.random() < 0.5 else 0
        assert w.extend(init, buf[off:off + n]) == oracle.extend(init, buf, off, n)
