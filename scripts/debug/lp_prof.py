#!/usr/bin/env python3
"""Where run_lp's time goes, per wave: the profiling build of the library
(make -C wipdb_amd/csrc LPFLAGS=-DWIPDB_LP_PROF LIBDIR=$PWD/build/prof
OBJDIR=$PWD/build/objprof) sums s_memtime cycles of each part of the loop --
the wait for the iteration's bytes, decide (up to the next DMA's issue), the
compute, the tail (queue / desk work) -- and the iteration counts.  GPU box
only:  python scripts/debug/lp_prof.py [shape ...]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PROF_LIB = os.environ.get("WIPDB_PROF_LIB") or os.path.join(REPO, "build", "prof",
                                                           "libhip_crc32c_batch.so")
os.environ["WIPDB_HCRC_LIB"] = PROF_LIB
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wipdb_amd import Engine  # noqa: E402

NAMES = ["wait", "decide", "compute", "tail", "segs", "batches", "idle", "life",
         "s_checks", "s_wait", "s_read_desk", "s_issue", "s_compute", "s_iters"]
NPROF = 16


def shape(name):
    if name == "headline":
        n = 1 << 20
        return np.arange(n, dtype=np.int64) * 4096, np.full(n, 4096, np.int32), n * 4096
    if name == "tblocks":  # WriteRawBlock spans: 4097..4225 B (contents + type), SST-packed
        rng = np.random.default_rng(5)
        n = 1 << 20
        ln = rng.integers(4097, 4226, n).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(ln + 4)[:-1]])
        return offs.astype(np.int64), ln.astype(np.int32), int(offs[-1] + ln[-1] + 64)
    if name == "zipf":  # config 3's mix: Zipf(0.99) over 512 B .. 64 KiB (+0..L/8), SST-packed
        sys.path.insert(0, os.path.join(REPO, "scripts"))
        from bench_extra import BUCKETS, zipf_spans
        offs, lens, _ = zipf_spans(np.random.default_rng(42), 2 << 30, BUCKETS)
        return offs.astype(np.int64), lens.astype(np.int32), 2 << 30
    if name.startswith("bucket"):  # bucketN: SST-packed N-byte spans + 5-byte trailers
        b = int(name[6:])
        n = (4 << 30) // (b + 5)
        return np.arange(n, dtype=np.int64) * (b + 5), np.full(n, b, np.int32), n * (b + 5) + 64
    raise SystemExit(f"unknown shape {name}")


def main():
    shapes = sys.argv[1:] or ["headline", "tblocks", "bucket512", "bucket4096", "bucket65536"]
    lib = ctypes.CDLL(PROF_LIB)
    fn = lib.hcrc_debug_lp_prof
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    host = np.zeros(4096 * NPROF, np.uint64)
    with Engine(0) as eng:
        for name in shapes:
            offs, lens, size = shape(name)
            buf = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda")
            o = torch.from_numpy(offs).cuda()
            ln = torch.from_numpy(lens).cuda()
            out = torch.empty(offs.size, dtype=torch.int32, device="cuda")
            for _ in range(20):
                eng.batch_device(buf, o, ln, None, out)
            torch.cuda.synchronize()
            assert fn(None, 0, 1) == 0
            reps = 10
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                eng.batch_device(buf, o, ln, None, out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            assert fn(host.ctypes.data, host.nbytes, 1) == 0
            p = host.reshape(4096, NPROF).astype(np.float64) / reps
            # wave lifetimes per workgroup (slot = workgroup * 16 + wave):
            # the spread across workgroups vs within them
            lifeg = p[:, 7].reshape(256, 16)
            wg = lifeg[(lifeg > 0).all(axis=1)]
            if len(wg):
                wmax, wmean = wg.max(axis=1), wg.mean(axis=1)
                print(f"  workgroups: last wave at {wmax.min():.0f} .. {wmax.max():.0f} cycles "
                      f"(mean {wmax.mean():.0f}, max/mean {wmax.max() / wmax.mean():.3f}); "
                      f"within a workgroup mean wave / last wave {np.mean(wmean / wmax):.3f}")
            live = p[:, 7] > 0
            p = p[live]
            it = p[:, 4] + p[:, 5] + p[:, 6]
            tot = p[:, :4].sum(axis=1)
            print(f"{name}: {ms:.4f} ms/launch, {live.sum()} waves, "
                  f"{size / ms / 1e6 / 1.073741824:.0f} GiB/s", flush=True)
            print(f"  per wave: iterations {it.mean():.1f} (min {it.min():.0f} max {it.max():.0f}), "
                  f"segs {p[:, 4].mean():.1f} batches {p[:, 5].mean():.1f} idle {p[:, 6].mean():.1f}")
            print(f"  life cycles: mean {p[:, 7].mean():.0f} min {p[:, 7].min():.0f} "
                  f"max {p[:, 7].max():.0f}; loop share {tot.mean() / p[:, 7].mean():.3f}")
            per = p[:, :4].sum(axis=0) / max(it.sum(), 1)
            print("  cycles per iteration: " + ", ".join(
                f"{NAMES[k]} {per[k]:.0f}" for k in range(4)) + f" (sum {per.sum():.0f})", flush=True)
            si = p[:, 13].sum()
            if si:
                sp = p[:, 8:13].sum(axis=0) / si
                print(f"  segment loop: {si / live.sum():.1f} iterations per wave; cycles per "
                      "iteration: " + ", ".join(f"{NAMES[8 + k][2:]} {sp[k]:.0f}" for k in range(5))
                      + f" (sum {sp.sum():.0f})", flush=True)
            del buf, o, ln, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
