#!/usr/bin/env python3
"""BASELINE config 1: 1 M x 4 KiB random blocks (4 GiB, splitmix64 seed 42)
through the host CRC on one thread -- the reference's own kv::crc32c
(oracle/_ref/libref_crc32c.so, compiled from kv/src/util/crc32c.cc) and this
library's CPU path (crc32c_cpu.cc: SSE4.2 3-stream + PCLMUL combine, the
C++ drop-in's Extend), plus both on every host thread.  Bit-exact check of
the two over all blocks.  One JSON line.

    python scripts/bench_cpu.py [--blocks N] [--threads T]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from tests.golden.common import splitmix64_bytes  # noqa: E402
from wipdb_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    a = ap.parse_args()
    n, B = a.blocks, 4096
    t0 = time.time()
    buf = splitmix64_bytes(42, n * B)
    gen_s = time.time() - t0
    offs = np.arange(n, dtype=np.uint64) * B
    lens = np.full(n, B, np.uint32)
    res = {"config": "1: 1 M x 4 KiB random blocks, host CPU", "blocks": n, "bytes": n * B,
           "gen_s": round(gen_s, 1), "cpu": "", "threads_all": a.threads}
    try:
        with open("/proc/cpuinfo") as f:
            res["cpu"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    outs = {}
    ref_path = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
    if os.path.exists(ref_path):
        ref = ctypes.CDLL(ref_path)
        ref.ref_crc32c_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int,
                                                                   ctypes.c_int]
        for th in (1, a.threads):
            out = np.empty(n, np.uint32)
            t = time.perf_counter()
            ref.ref_crc32c_batch(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None,
                                 out.ctypes.data, n, 0, th)
            el = time.perf_counter() - t
            res[f"reference_{th}t_GiBps"] = round(n * B / el / 2**30, 2)
            outs["ref"] = out
    lib = _lib.load()
    for th in (1, a.threads):
        out = np.empty(n, np.uint32)
        t = time.perf_counter()
        _lib.check(lib.hcrc_cpu_batch(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None,
                                      out.ctypes.data, n, 0, th), "hcrc_cpu_batch")
        el = time.perf_counter() - t
        res[f"library_cpu_{th}t_GiBps"] = round(n * B / el / 2**30, 2)
        outs["lib"] = out
    if "ref" in outs:
        res["mismatches_library_vs_reference"] = int((outs["ref"] != outs["lib"]).sum())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
