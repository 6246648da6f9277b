#!/usr/bin/env python3
"""AutoSplit A/B: for host batches of short spans, is the
size-class path (HCRC_SPLIT_SMALL: a partition pass + three list kernels)
still faster than the default lane-packed spans kernel?

Shapes: WAL record CRC spans (type byte + payload of 60..300 bytes, 7-byte
record headers between them, as log_batch.cc lays them out), meta / filter
block spans (200..2000 bytes + type byte, SST-packed), and the 512 B and
1 KiB buckets.  Paths: hcrc_batch on pageable host memory (staged),
hcrc_batch on pinned memory from hcrc_host_alloc (zero-copy), and the
device-resident entry point (kernel time).  Each host batch runs with the
choice forced both ways through the test build's WIPDB_HCRC_AUTOSPLIT hook
(0 = spans kernel, 1 = classes), alternating, same session; results are
checked against the CPU path.  One JSON line per (shape, batch size, path).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("WIPDB_HCRC_LIB", os.path.join(REPO, "build", "testlib",
                                                     "libhip_crc32c_batch.so"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wipdb_amd import Engine, _lib, cpu_batch  # noqa: E402


def layout(rng, kind, nbytes):
    if kind == "wal":
        lo, hi, gap, extra = 60, 300, 7, 1
    elif kind == "meta":
        lo, hi, gap, extra = 200, 2000, 5, 1
    elif kind == "512":
        lo, hi, gap, extra = 512, 576, 5, 0
    else:
        lo, hi, gap, extra = 1024, 1152, 5, 0
    est = nbytes // ((lo + hi) // 2 + gap) + 16
    n = rng.integers(lo, hi + 1, est).astype(np.uint64) + extra
    offs = 6 + np.concatenate([[0], np.cumsum(n + gap)[:-1]]).astype(np.uint64)
    keep = offs + n <= nbytes
    return offs[keep], n[keep].astype(np.uint32)


def host_rate(eng, host, offs, lens, mode, reps):
    os.environ["WIPDB_HCRC_AUTOSPLIT"] = mode
    eng.batch(host, offs, lens)  # warm (lanes, staging)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        got = eng.batch(host, offs, lens)
        ts.append(time.perf_counter() - t0)
    return float(lens.sum()) / float(np.median(ts)) / 2**30, got


def dev_rate(eng, d, do, dl, split, reps):
    st = torch.cuda.current_stream()
    eng.batch_device(d, do, dl, split_small=split)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(reps):
        out = eng.batch_device(d, do, dl, split_small=split)
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="wal,meta,512,1k")
    ap.add_argument("--sizes-mib", default="4,32")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    lib = _lib.load()
    rng = np.random.default_rng(11)
    with Engine(0) as eng:
        for kind in a.kinds.split(","):
            for mib in (int(x) for x in a.sizes_mib.split(",")):
                nbytes = mib << 20
                offs, lens = layout(rng, kind, nbytes)
                page = rng.integers(0, 256, nbytes, dtype=np.uint8)
                want = cpu_batch(page, offs, lens)
                pin = ctypes.c_void_p()
                _lib.check(lib.hcrc_host_alloc(nbytes, ctypes.byref(pin)), "hcrc_host_alloc")
                pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(pin.value))
                pinned[:] = page
                res = {"shape": kind, "batch_MiB": mib, "spans": int(offs.size),
                       "mean_span": round(float(lens.mean()), 1)}
                for path, host in (("staged", page), ("zero_copy", pinned)):
                    r = {"spans_kernel": [], "classes": []}
                    bad = 0
                    for _ in range(3):  # alternating rounds
                        for mode, key in (("0", "spans_kernel"), ("1", "classes")):
                            g, got = host_rate(eng, host, offs, lens, mode, a.reps)
                            r[key].append(g)
                            bad += int((got != want).sum())
                    res[path] = {k: round(float(np.median(v)), 2) for k, v in r.items()}
                    res[path]["mismatches"] = bad
                os.environ.pop("WIPDB_HCRC_AUTOSPLIT", None)
                d = torch.from_numpy(page).cuda()
                do = torch.from_numpy(offs.view(np.int64)).cuda()
                dl = torch.from_numpy(lens.view(np.int32)).cuda()
                ms = {}
                for split, key in ((False, "spans_kernel"), (True, "classes")):
                    t, out = dev_rate(eng, d, do, dl, split, 20)
                    ms[key] = round(float(lens.sum()) / t / 2**30, 1)
                    ms[key + "_ok"] = bool((out.cpu().numpy().view(np.uint32) == want).all())
                res["device_GiBps"] = ms
                lib.hcrc_host_free(pin)
                print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
