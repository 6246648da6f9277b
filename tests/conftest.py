"""Shared fixtures: build-on-demand, oracle bindings, golden data.

Markers: ``gpu`` = needs a real MI355X (run with ``-m gpu``); everything else
runs on the CPU-only build container.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# HCRC_PACKED hands batches of fewer than 32 Ki spans to the default path
# (the pre-pass costs more than it saves there); the suite's packed cases
# are smaller than that and must reach the stream-tiled kernel
os.environ.setdefault("WIPDB_PS_MIN_SPANS", "0")

GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "liboracle.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
LIB_SO = os.path.join(REPO, "wipdb_amd", "lib", "libhip_crc32c_batch.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(LIB_SO):
        subprocess.run(["make", "-C", os.path.join(REPO, "wipdb_amd", "csrc")], check=True,
                       stdout=subprocess.DEVNULL)


_ensure_built()


class Oracle:
    """ctypes view of oracle/_build/liboracle.so (test infrastructure)."""

    def __init__(self, path=ORACLE_SO):
        lib = ctypes.CDLL(path)
        vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
        lib.oracle_crc32c_extend.restype = u32
        lib.oracle_crc32c_extend.argtypes = [u32, vp, sz]
        lib.oracle_mask.restype = u32
        lib.oracle_mask.argtypes = [u32]
        lib.oracle_unmask.restype = u32
        lib.oracle_unmask.argtypes = [u32]
        lib.oracle_crc32c_batch.restype = None
        lib.oracle_crc32c_batch.argtypes = [vp, vp, vp, vp, vp, sz, ctypes.c_int]
        lib.oracle_fill_folly_buffer.argtypes = [vp, sz]
        self.lib = lib

    def extend(self, init, buf: np.ndarray, off=0, n=None) -> int:
        n = buf.size - off if n is None else n
        return int(self.lib.oracle_crc32c_extend(init & 0xFFFFFFFF, buf.ctypes.data + off, n))

    def batch(self, buf, offsets, lengths, inits=None, mask=False) -> np.ndarray:
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.empty(off.size, dtype=np.uint32)
        self.lib.oracle_crc32c_batch(buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                     None if ini is None else ini.ctypes.data,
                                     out.ctypes.data, off.size, int(mask))
        return out

    def folly_buffer(self, size) -> np.ndarray:
        buf = np.zeros(size, dtype=np.uint8)
        self.lib.oracle_fill_folly_buffer(buf.ctypes.data, size)
        return buf


class Reference:
    """ctypes view of oracle/_ref/libref_crc32c.so (the reference, compiled)."""

    def __init__(self, path=REF_SO):
        lib = ctypes.CDLL(path)
        vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
        lib.ref_crc32c_extend.restype = u32
        lib.ref_crc32c_extend.argtypes = [u32, vp, sz]
        lib.ref_crc32c_batch.restype = None
        lib.ref_crc32c_batch.argtypes = [vp, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int]
        self.lib = lib

    def extend(self, init, buf, off=0, n=None) -> int:
        n = buf.size - off if n is None else n
        return int(self.lib.ref_crc32c_extend(init & 0xFFFFFFFF, buf.ctypes.data + off, n))

    def batch(self, buf, offsets, lengths, inits=None, mask=False, threads=8) -> np.ndarray:
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.empty(off.size, dtype=np.uint32)
        self.lib.ref_crc32c_batch(buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                  None if ini is None else ini.ctypes.data, out.ctypes.data,
                                  off.size, int(mask), threads)
        return out


@pytest.fixture(scope="session")
def oracle() -> Oracle:
    return Oracle()


@pytest.fixture(scope="session")
def reference():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (reference absent and no prebuilt copy)")
    return Reference()


@pytest.fixture(scope="session")
def kats() -> dict:
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_spans():
    return load_golden_spans()


def load_golden_spans() -> dict:
    from tests.golden.common import splitmix64_bytes
    with open(os.path.join(GOLDEN, "spans.json")) as f:
        d = json.load(f)
    b = d["buffer"]
    buf = splitmix64_bytes(b["seed"], b["size"])
    rows = np.array(d["rows"], dtype=np.uint64)
    return {"buf": buf, "seed": b["seed"], "offsets": rows[:, 0], "lengths": rows[:, 1].astype(np.uint32),
            "inits": rows[:, 2].astype(np.uint32), "crc": rows[:, 3].astype(np.uint32),
            "masked": rows[:, 4].astype(np.uint32)}


def gpu_available() -> bool:
    try:
        from wipdb_amd import device_count
        return device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    import torch  # noqa: F401  (torch first: one HIP runtime in the process)
    from wipdb_amd import Engine
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but torch sees no HIP device")
    eng = Engine(0)
    yield eng
    eng.close()
