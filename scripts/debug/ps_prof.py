#!/usr/bin/env python3
"""Where run_ps's time goes (HCRC_PACKED), per wave: the profiling build of
the library (make -C wipdb_amd/csrc LPFLAGS=-DWIPDB_LP_PROF
LIBDIR=$PWD/build/prof OBJDIR=$PWD/build/objprof) sums s_memtime cycles of
each part of the page loop -- the wait for the page, landed -> next DMA out,
the compute, the desk loads, the deferred span ends -- and the page counts.
With --default the same shapes through the default pipeline (run_ea's
markers: wait, issue, compute, pages; its shapes only -- a4k, tblocks,
b65536).  GPU box only:
  python scripts/debug/ps_prof.py [--default] [shape ...]  (packed_ab.py's shapes)"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PROF_LIB = os.environ.get("WIPDB_PROF_LIB") or os.path.join(REPO, "build", "prof",
                                                           "libhip_crc32c_batch.so")
os.environ["WIPDB_HCRC_LIB"] = PROF_LIB
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_extra import dev  # noqa: E402
from packed_ab import shape_of  # noqa: E402
from wipdb_amd import Engine  # noqa: E402

NAMES = ["wait", "issue", "compute", "desk", "pages", "cut_pages", "plan", "life", "finish",
         "chunks"]
NPROF = 16


def main():
    packed = "--default" not in sys.argv
    shapes = [a for a in sys.argv[1:] if not a.startswith("--")] or \
        ["b512", "b4096", "b65536", "tblocks", "a4k"]
    lib = ctypes.CDLL(PROF_LIB)
    fn = lib.hcrc_debug_lp_prof
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    host = np.zeros(4096 * NPROF, np.uint64)
    nbytes = 2 << 30
    d = torch.device("cuda", 0)
    buf = torch.randint(0, 256, (2 * nbytes,), dtype=torch.uint8, device=d)
    with Engine(0) as eng:
        for name in shapes:
            o, ln = shape_of(name, np.random.default_rng(42), nbytes)
            do, dl = dev(o, d), dev(ln, d)
            out = torch.empty(o.size, dtype=torch.int32, device=d)
            for _ in range(20):
                eng.batch_device(buf, do, dl, None, out, packed=packed)
            torch.cuda.synchronize()
            assert fn(None, 0, 1) == 0
            reps = 10
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                eng.batch_device(buf, do, dl, None, out, packed=packed)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            assert fn(host.ctypes.data, host.nbytes, 1) == 0
            p = host.reshape(4096, NPROF).astype(np.float64) / reps
            lifeg = p[:, 7].reshape(256, 16)
            wg = lifeg[(lifeg > 0).all(axis=1)]
            if len(wg):
                wmax, wmean, wmin = wg.max(axis=1), wg.mean(axis=1), wg.min(axis=1)
                print(f"  workgroups: last wave at {wmax.min():.0f} .. {wmax.max():.0f} cycles "
                      f"(mean {wmax.mean():.0f}); within a workgroup first / last wave "
                      f"{np.mean(wmin / wmax):.3f}, mean / last {np.mean(wmean / wmax):.3f}")
                # wave slot w of every workgroup: is a slot systematically slow?
                print("  life by wave slot (mean over workgroups / overall mean): " +
                      " ".join(f"{v:.2f}" for v in wg.mean(axis=0) / wg.mean()))
            live = p[:, 7] > 0
            p = p[live]
            pages = p[:, 4].sum()
            print(f"{name} ({'packed' if packed else 'default'}): {ms:.4f} ms/launch, {live.sum()} waves, "
                  f"{float(ln.sum()) / ms / 1e6 / 1.073741824:.0f} GiB/s", flush=True)
            print(f"  per wave: pages {p[:, 4].mean():.1f} (cut {p[:, 5].mean():.1f}), chunks "
                  f"{p[:, 9].mean():.1f}; life cycles mean {p[:, 7].mean():.0f} min "
                  f"{p[:, 7].min():.0f} max {p[:, 7].max():.0f}")
            per = {NAMES[k]: p[:, k].sum() / max(pages, 1) for k in (6, 0, 1, 2, 3, 8)}
            rest = p[:, 7].sum() / max(pages, 1) - sum(per.values())
            print("  cycles per page: " + ", ".join(f"{k} {v:.0f}" for k, v in per.items())
                  + f", rest {rest:.0f} (life {p[:, 7].sum() / max(pages, 1):.0f})", flush=True)
            del do, dl, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
