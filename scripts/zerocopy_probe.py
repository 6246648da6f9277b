#!/usr/bin/env python3
"""Diagnostic: CRC of host-resident 4 KiB blocks three ways on one MI355X --
(a) hcrc_batch from pageable memory (pack into pinned staging, H2D, kernel,
D2H), (b) hcrc_batch from pinned memory (same path), (c) the spans kernel
reading pinned host memory directly over PCIe (zero-copy: base is the
pinned host pointer, descriptors and outputs on the device).  GiB/s each,
results checked against each other."""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wipdb_amd import Engine, _lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 262144  # 1 GiB
BLOCK = 4096
lib = _lib.load()
eng = Engine(0)
nbytes = N * BLOCK

rng = np.random.default_rng(7)
page = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
offs = np.arange(N, dtype=np.uint64) * BLOCK
lens = np.full(N, BLOCK, np.uint32)
res = {"blocks": N, "bytes": nbytes}

def timeit(fn, reps=5):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps

out_a = np.empty(N, np.uint32)
t = timeit(lambda: out_a.__setitem__(slice(None), eng.batch(page, offs, lens)))
res["pageable_staged_GiBps"] = round(nbytes / t / 2**30, 2)

pin = ctypes.c_void_p()
_lib.check(lib.hcrc_host_alloc(nbytes, ctypes.byref(pin)), "host_alloc")
pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(pin.value))
pinned[:] = page
t = timeit(lambda: eng.batch(pinned, offs, lens))
res["pinned_staged_GiBps"] = round(nbytes / t / 2**30, 2)

d_off = torch.from_numpy(offs.view(np.int64)).cuda()
d_len = torch.from_numpy(lens.view(np.int32)).cuda()
d_out = torch.empty(N, dtype=torch.int32, device="cuda")
stream = torch.cuda.current_stream()


def zc():
    _lib.check(lib.hcrc_batch_async(eng._ctx, pin.value, d_off.data_ptr(), d_len.data_ptr(), None,
                                    d_out.data_ptr(), N, _lib.HCRC_DEVICE_PTRS,
                                    stream.cuda_stream), "zero-copy")
    torch.cuda.synchronize()


t = timeit(zc)
res["pinned_zero_copy_GiBps"] = round(nbytes / t / 2**30, 2)
got = d_out.cpu().numpy().view(np.uint32)
res["zero_copy_matches_staged"] = bool((got == out_a).all())
print(json.dumps(res), flush=True)
lib.hcrc_host_free(pin)
eng.close()
