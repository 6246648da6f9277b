#!/usr/bin/env python3
"""Wall time of batches holding ONE long span (1..64 MiB) or 16 of them:
host batches through hcrc_batch (pinned memory: zero-copy, so PCIe -- not a
staging copy -- is the other bound; long spans are split by themselves), and
device batches through hcrc_batch_async with and without HCRC_SPLIT_LONG.
Without a split a span's segments run chained on a single wave; with it, in
parts on many waves.  One JSON line per case; checked against the library's
host CPU path."""
import json
import os
import sys
import time
import ctypes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from wipdb_amd import Engine, cpu_batch, _lib  # noqa: E402


def main():
    lib = _lib.load()
    total = 80 << 20
    p = ctypes.c_void_p()
    _lib.check(lib.hcrc_host_alloc(total, ctypes.byref(p)), "host_alloc")
    try:
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p.value))
        buf[:] = np.random.default_rng(5).integers(0, 256, total, dtype=np.uint8)
        with Engine(0) as eng:
            for mib, count in ((1, 1), (4, 1), (16, 1), (64, 1), (4, 16)):
                n = (mib << 20) + 3
                offs = (np.arange(count, dtype=np.uint64) * np.uint64(n + 13) + 7).astype(np.uint64)
                lens = np.full(count, n, np.uint32)
                got = eng.batch(buf, offs, lens)  # warm
                ts = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    got = eng.batch(buf, offs, lens)
                    ts.append(time.perf_counter() - t0)
                want = cpu_batch(buf, offs, lens)
                t = sorted(ts)[len(ts) // 2]
                print(json.dumps({"path": "host", "span_MiB": mib, "spans": count,
                                  "ms": round(t * 1e3, 3),
                                  "GiBps": round(count * n / t / 2**30, 2),
                                  "mismatches": int((got != want).sum())}), flush=True)
                if not hasattr(lib, "hcrc_check_spans"):
                    continue  # an older build (A/B): host path only
                import torch
                dbuf = torch.from_numpy(buf).to("cuda:0")
                do = torch.from_numpy(offs.view(np.int64)).to("cuda:0")
                dl = torch.from_numpy(lens.view(np.int32)).to("cuda:0")
                for split in (False, True):
                    out = eng.batch_device(dbuf, do, dl, split_long=split)
                    torch.cuda.synchronize()
                    ts = []
                    for _ in range(5):
                        t0 = time.perf_counter()
                        eng.batch_device(dbuf, do, dl, out_t=out, split_long=split)
                        torch.cuda.synchronize()
                        ts.append(time.perf_counter() - t0)
                    t = sorted(ts)[len(ts) // 2]
                    g = out.cpu().numpy().view(np.uint32)
                    print(json.dumps({"path": "device", "split_long": split, "span_MiB": mib,
                                      "spans": count, "ms": round(t * 1e3, 3),
                                      "GiBps": round(count * n / t / 2**30, 2),
                                      "mismatches": int((g != want).sum())}), flush=True)
                del dbuf
    finally:
        lib.hcrc_host_free(p)


if __name__ == "__main__":
    main()
