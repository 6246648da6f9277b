"""A/B of pinned host batches: dense pieces through the copy engine (the
default) against every piece zero-copy (WIPDB_HOST_DMA=0), alternating child
processes on one box.  Each child runs config 5 as bench.py does
(scripts/bench_configs.run_config5: 256 SSTs of the 8Binsert stream in
hcrc_host_alloc memory, hcrc_batch HOST_PTRS, PCIe-inclusive; one SST a call
for the latency) and a 1 GiB batch of aligned 4 KiB blocks, with a sample
of every result against bench.py's checker (oracle/_ref).

  python scripts/pinned_dma_ab.py [rounds]
"""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child():
    import torch
    from bench import _ref_batch
    from scripts.bench_configs import _ref_check, run_config5
    from wipdb_amd import Engine, _lib
    torch.cuda.init()
    ref_fn = _ref_batch()[0]
    rng = np.random.default_rng(0xC0F1)
    lib = _lib.load()
    with Engine(0) as eng:
        c5 = run_config5(eng, ref_fn, rng)
        n = 1 << 30
        pin = ctypes.c_void_p()
        _lib.check(lib.hcrc_host_alloc(n, ctypes.byref(pin)), "hcrc_host_alloc")
        try:
            host = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pin.value))
            host[:] = 7
            host[::4093] = rng.integers(0, 256, host[::4093].size, dtype=np.uint8)
            offs = np.arange(n // 4096, dtype=np.uint64) * 4096
            lens = np.full(offs.size, 4096, np.uint32)
            eng.batch(host, offs[:1000], lens[:1000])
            t0 = time.perf_counter()
            for _ in range(3):
                got = eng.batch(host, offs, lens)
            t = (time.perf_counter() - t0) / 3
            a4 = {"GiBps": round(n / t / 2**30, 2),
                  "parity": _ref_check(ref_fn, host, offs, lens, got, rng)}
        finally:
            lib.hcrc_host_free(pin)
    return {"config5": {k: c5[k] for k in ("GiBps_end_to_end", "pcie_h2d_ceiling_GiBps",
                                           "fraction_of_pcie_ceiling", "latency_2MiB_sst",
                                           "parity")},
            "aligned_4k_1GiB": a4}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        print("RES " + json.dumps(child()), flush=True)
        return
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for r in range(rounds):
        for dma in ("1", "0"):
            env = dict(os.environ, PYTHONPATH=REPO, WIPDB_HOST_DMA=dma)
            p = subprocess.run([sys.executable, __file__, "--child"], env=env, cwd=REPO,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            res = json.loads(p.stdout.split("RES ", 1)[1].splitlines()[0])
            print(json.dumps({"round": r, "WIPDB_HOST_DMA": dma, **res}), flush=True)


if __name__ == "__main__":
    main()
