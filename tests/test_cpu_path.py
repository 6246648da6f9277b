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


# ---- the portable fallback (ExtendImpl<Slow_CRC32>, kv/src/util/crc32c.cc:
# 325-339, 355-397): slicing-by-8, reached on hosts without SSE4.2 + PCLMUL,
# or forced with WIPDB_CRC_PORTABLE=1 ----

def _portable(init, buf, off=0, n=None):
    import ctypes
    n = buf.size - off if n is None else n
    return int(w._lib.load().hcrc_cpu_extend_portable(init & 0xFFFFFFFF,
                                                       ctypes.c_void_p(buf.ctypes.data + off), n))


def test_portable_path_kats_and_golden(kats, golden_spans, oracle):
    for v in kats["rfc"]:
        b = np.frombuffer(bytes.fromhex(v["data_hex"]), np.uint8).copy()
        assert _portable(0, b) == v["crc"], v["name"]
    f = kats["folly"]
    buf = oracle.folly_buffer(f["buffer_size"])
    for v in f["vectors"]:
        assert _portable(0, buf, v["offset"], v["length"]) == v["crc"]
    g = golden_spans
    for o, n, i, c in zip(g["offsets"], g["lengths"], g["inits"], g["crc"]):
        assert _portable(int(i), g["buf"], int(o), int(n)) == int(c)


def test_portable_path_every_alignment_vs_oracle(oracle):
    """every start mod 8 and every length around the 8-byte word loop's edges"""
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 4096, dtype=np.uint8)
    for off in range(16):
        for n in list(range(0, 40)) + [63, 64, 65, 255, 256, 257, 1000, 2049]:
            init = int(rng.integers(0, 2**32)) if (off + n) % 3 == 0 else 0
            assert _portable(init, buf, off, n) == oracle.extend(init, buf, off, n), (off, n)


def test_forced_portable_surface_matches_golden(tmp_path):
    """WIPDB_CRC_PORTABLE=1: the whole host surface (hcrc_cpu_extend,
    hcrc_cpu_batch over threads, the kv::crc32c mirror) runs the portable
    path, reports no acceleration, and still matches the golden spans."""
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, wipdb_amd as w\n"
        "from tests.conftest import load_golden_spans\n"
        "g = load_golden_spans()\n"
        "assert w._lib.load().hcrc_cpu_is_accelerated() == 0\n"
        "assert w.is_fast_crc32_supported() == 'Not supported on x86'\n"
        "for t in (1, 4):\n"
        "    got = w.cpu_batch(g['buf'], g['offsets'], g['lengths'], g['inits'], threads=t)\n"
        "    assert (got == g['crc']).all()\n"
        "assert w.value(b'123456789') == 0xE3069283\n"
        "print('portable ok')\n")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WIPDB_CRC_PORTABLE="1", PYTHONPATH=repo)
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "portable ok" in r.stdout, r.stderr[-2000:]
