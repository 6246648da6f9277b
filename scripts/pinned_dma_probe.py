"""Diagnostic: GiB/s of one synchronous hcrc_batch over ~550 MB of pinned
host memory for several span layouts (the config-5 SST stream, the same
spans moved onto a 256-byte grid, aligned 4 KiB blocks, the SST stream's data
blocks alone), best of 3 calls each, so the copy-engine path's rate can be
told apart by layout.

  python scripts/pinned_dma_probe.py [layout,...]   (raw: also the copy engine's own rates)
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))


def main():
    import torch
    from bench_extra import sst_layout
    from wipdb_amd import Engine, _lib
    torch.cuda.init()
    rng = np.random.default_rng(0xC0F1)
    lib = _lib.load()
    offs, lens, nbytes = sst_layout(rng, 256)
    layouts = {"sst": (offs, lens)}
    step = (lens.astype(np.uint64) + 4 + 255) // 256 * 256
    g = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.uint64)
    keep = g + lens <= nbytes
    layouts["sst_on_256_grid"] = (g[keep], lens[keep])
    data = lens < 5000
    layouts["sst_data_blocks"] = (offs[data], lens[data])
    n4 = nbytes // 4096
    layouts["aligned_4k"] = (np.arange(n4, dtype=np.uint64) * 4096, np.full(n4, 4096, np.uint32))
    res = {}
    with Engine(0) as eng:
        pin = ctypes.c_void_p()
        _lib.check(lib.hcrc_host_alloc(nbytes, ctypes.byref(pin)), "hcrc_host_alloc")
        try:
            host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(pin.value))
            host[:] = 33
            eng.batch(host, offs[:1000], lens[:1000])
            only = sys.argv[1].split(",") if len(sys.argv) > 1 else list(layouts)
            for name, (o, ln) in layouts.items():
                if name not in only:
                    continue
                best = 1e9
                for _ in range(3):
                    t0 = time.perf_counter()
                    eng.batch(host, o, ln)
                    best = min(best, time.perf_counter() - t0)
                cover = int(o.max() + ln[np.argmax(o)]) - int(o.min())
                res[name] = {"spans": int(o.size), "GiBps_span_bytes": round(float(ln.sum()) / best / 2**30, 2),
                             "GiBps_covering": round(cover / best / 2**30, 2), "ms": round(best * 1e3, 2)}
                print(name, res[name], flush=True)
            if "raw" in only:
                res["raw_copy"] = raw_copies(pin.value, nbytes)
                print("raw", res["raw_copy"], flush=True)
        finally:
            lib.hcrc_host_free(pin)
    print(json.dumps(res))


def raw_copies(src, nbytes):
    """hipMemcpyAsync rates (GiB/s) straight from the hcrc_host_alloc buffer and
    from torch-pinned memory into HBM: 512 MiB as 1 copy, 4 x 128 MiB, 16 x 32 MiB."""
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    n = 512 << 20
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    tp = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for name, base in (("hcrc_host_alloc", src), ("torch_pinned", tp.data_ptr())):
        for chunk in (n, 128 << 20, 32 << 20):
            best = 1e9
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for off in range(0, n, chunk):
                    assert hip.hipMemcpyAsync(dst.data_ptr() + off, base + off, chunk, 1, st) == 0
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            out[f"{name}/{chunk >> 20}MiB"] = round(n / best / 2**30, 2)
    return out


if __name__ == "__main__":
    main()
