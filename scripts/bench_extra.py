#!/usr/bin/env python3
"""Secondary measurements (BASELINE.json configs 3 and 5, and the
PCIe-inclusive host path) -- one JSON line each, for DESIGN.md.

  mixed      config 3: Zipf(0.99) sizes over {512 .. 64 Ki} (+0..L/8 jitter),
             SST-packed at unaligned offsets (prev + L + 5), device-resident:
             per-bucket GiB/s, the mixed batch's GiB/s, and p50/p99 latency of
             SST-sized batches (one ~2 MiB SST per launch, synchronised).
  sst        config 5: 8Binsert-shaped SSTs (~500 data blocks of 4097..4225
             bytes incl. the type byte, one ~18 KiB index block, one ~25 KiB
             filter block, one metaindex block) in HOST memory, checksummed
             through hcrc_batch(HOST_PTRS): pinned staging + H2D + kernel +
             D2H, overlapped -- the PCIe-inclusive end-to-end rate.
  sstpin     config 5 from PINNED host memory (the table builder's write
             buffers): copy engine / zero-copy, as a fraction of the measured
             PCIe ceiling.
  host4k     the headline 1 M x 4 KiB blocks from host memory (PCIe-inclusive).

Every batch is checked against the library's host CPU path on a sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wipdb_amd import Engine, cpu_batch  # noqa: E402

BUCKETS = [512, 1024, 2048, 4096, 8192, 16384, 32768, 65536]


def zipf_spans(rng, nbytes, buckets, theta=0.99, start=3):
    p = 1.0 / np.arange(1, len(buckets) + 1) ** theta
    p /= p.sum()
    est = int(nbytes / (np.dot(p, buckets) * 1.07 + 5)) + 16
    L = np.asarray(buckets)[rng.choice(len(buckets), est, p=p)]
    n = L + rng.integers(0, L // 8 + 1)
    offs = start + np.concatenate([[0], np.cumsum(n + 5)[:-1]])
    keep = offs + n <= nbytes
    return offs[keep].astype(np.uint64), n[keep].astype(np.uint32), L[keep]


def dev(a, d):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(d)


PRECONDITION_S = 0.08  # bench.py's power-transient preconditioning


def time_kernel(fn, stream, reps, windows=2):
    """Average launch time of fn on `stream` over `reps` back-to-back
    launches, the best of `windows` such windows, after untimed launches
    worth >= PRECONDITION_S of GPU time (the first ~30-60 ms of back-to-back
    launches after idle run slow while the SMU raises the clocks, bench.py;
    a single window right after a large allocation and fill once read 26 %
    slow on a box that timed the same batch at its usual rate again a minute
    later, profiles/r05z_bench.log vs r05z_tbl.log).  The preconditioning
    launches and the windows are queued back to back with no host wait
    between them: a host pause of >= 2 ms lets the memory clocks drop again
    and the next ~20 launches run 5-18 % slow (profiles/r06a_gap_*.log)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record(stream)
    fn()
    e.record(stream)
    torch.cuda.synchronize()
    one = max(s.elapsed_time(e) / 1e3, 1e-6)
    n = int(min(4096, max(8, PRECONDITION_S / one + 1)))
    for _ in range(n):
        fn()
    ev = []
    for _ in range(max(1, windows)):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(reps):
            fn()
        e.record(stream)
        ev.append((s, e))
    torch.cuda.synchronize()
    return min(s.elapsed_time(e) / reps / 1e3 for s, e in ev)


def usable_cpus() -> int:
    """CPUs this job may use (affinity, capped by OMP_NUM_THREADS: the GPU
    box gives a one-GPU job 16 of its 256 CPUs)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, share) if share > 0 else n


def cpu_rates(host, offs, lens):
    """BASELINE config 3's CPU side: the library's host CRC path (SSE4.2
    3-stream + PCLMUL combine, the reference's crc32c_3way class) over the
    same spans from host memory, 1 thread and all usable CPUs, GiB/s."""
    if NO_CPU:
        return [None, None]
    nbytes = float(lens.sum())
    out = []
    for threads in (1, usable_cpus()):
        cpu_batch(host, offs, lens, threads=threads)  # warm
        t0 = time.perf_counter()
        cpu_batch(host, offs, lens, threads=threads)
        out.append(round(nbytes / (time.perf_counter() - t0) / 2**30, 1))
    return out


def check_sample(host, offs, lens, got, rng, k=4000):
    idx = rng.choice(offs.size, min(k, offs.size), replace=False)
    want = cpu_batch(host, offs[idx], lens[idx])
    return int((want != got[idx]).sum())


SPLIT = False  # --split: HCRC_SPLIT_SMALL on the device batches
SPLIT_LONG = False  # --split-long: HCRC_SPLIT_LONG on config 3's device batches
NO_CPU = False  # --no-cpu: skip the CPU rates (same-session A/B runs)


def batch_latency(eng, dbuf, do, dl, stream, nbatch_bytes=2 << 20, reps=200):
    """p50 / p99 of synchronised SST-sized batches (~2 MiB of these spans per
    launch, consecutive slices of the batch), host wall time from the launch
    call to the synchronize's return.  The launch goes through the C-ABI
    (hcrc_batch_async by ctypes, as a C++ caller would make it; the Python
    wrapper's argument checks cost ~10 us a call, profiles/r06g_latency.log)."""
    from wipdb_amd import _lib
    lens = dl.cpu().numpy().view(np.uint32).astype(np.int64)
    per = max(1, int(np.searchsorted(np.cumsum(lens + 5), nbatch_bytes)))
    n = lens.size
    outs = torch.empty(per, dtype=torch.int32, device=dbuf.device)
    flags = (_lib.HCRC_DEVICE_PTRS | (_lib.HCRC_SPLIT_SMALL if SPLIT else 0)
             | (_lib.HCRC_SPLIT_LONG if SPLIT_LONG else 0))
    lib, ctx, sp = eng._lib, eng._ctx, stream.cuda_stream
    lat = []
    for i in range(reps + 20):
        lo = (i * per) % max(1, n - per)
        cnt = min(per, n - lo)
        a_off, a_len = do.data_ptr() + 8 * lo, dl.data_ptr() + 4 * lo
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib.hcrc_batch_async(ctx, dbuf.data_ptr(), a_off, a_len, None, outs.data_ptr(), cnt,
                                  flags, sp)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
        _lib.check(rc, "hcrc_batch_async")
    lat = np.array(lat[20:]) * 1e6
    return {"spans_per_batch": int(min(per, n)), "p50_us": round(float(np.percentile(lat, 50)), 1),
            "p99_us": round(float(np.percentile(lat, 99)), 1)}


def host_batch_latency(eng, host_ptr, offs, lens, nbatch_bytes=2 << 20, reps=200):
    """The same for the product's own per-SST call: hcrc_batch on host
    pointers (a TableBuilder write buffer in pinned memory: zero-copy), ~2 MiB
    of spans a call, synchronous."""
    from wipdb_amd import _lib
    per = max(1, int(np.searchsorted(np.cumsum(lens.astype(np.int64) + 5), nbatch_bytes)))
    n = offs.size
    out = np.empty(per, np.uint32)
    lib, ctx = eng._lib, eng._ctx
    lat = []
    for i in range(reps + 20):
        lo = (i * per) % max(1, n - per)
        cnt = min(per, n - lo)
        o = offs[lo:lo + cnt]
        ln = lens[lo:lo + cnt]
        t0 = time.perf_counter()
        rc = lib.hcrc_batch(ctx, host_ptr, o.ctypes.data, ln.ctypes.data, None, out.ctypes.data,
                            cnt, _lib.HCRC_MASK_OUTPUT)
        lat.append(time.perf_counter() - t0)
        _lib.check(rc, "hcrc_batch")
    lat = np.array(lat[20:]) * 1e6
    return {"spans_per_batch": int(min(per, n)), "p50_us": round(float(np.percentile(lat, 50)), 1),
            "p99_us": round(float(np.percentile(lat, 99)), 1)}


def run_mixed(eng, d, stream, rng, gib):
    nbytes = int(gib * 2**30)
    host = rng.integers(0, 256, nbytes, dtype=np.uint8)
    dbuf = torch.from_numpy(host).to(d)
    res = {"config": "3 mixed (Zipf 0.99, SST-packed, unaligned)", "split_small": SPLIT,
           "split_long": SPLIT_LONG,
           "buckets": {}}
    offs, lens, L = zipf_spans(rng, nbytes, BUCKETS)
    do, dl = dev(offs, d), dev(lens, d)
    out = torch.empty(offs.size, dtype=torch.int32, device=d)
    t = time_kernel(lambda: eng.batch_device(dbuf, do, dl, None, out, stream=stream.cuda_stream,
                                                 split_small=SPLIT, split_long=SPLIT_LONG),
                    stream, 10)
    got = out.cpu().numpy().view(np.uint32)
    cpu = cpu_rates(host, offs, lens)
    res["cpu_threads"] = usable_cpus()
    res["mixed"] = {"spans": int(offs.size), "bytes": int(lens.sum()),
                    "GiBps": round(float(lens.sum()) / t / 2**30, 1),
                    "cpu_1t_GiBps": cpu[0], "cpu_all_GiBps": cpu[1],
                    "mismatches_in_sample": check_sample(host, offs, lens, got, rng),
                    "sst_batch_latency": batch_latency(eng, dbuf, do, dl, stream)}
    for b in BUCKETS:  # one batch per bucket: same packing, only this size
        ob, lb, _ = zipf_spans(rng, nbytes, [b])
        dob, dlb = dev(ob, d), dev(lb, d)
        outb = torch.empty(ob.size, dtype=torch.int32, device=d)
        tb = time_kernel(lambda: eng.batch_device(dbuf, dob, dlb, None, outb,
                                                  stream=stream.cuda_stream, split_small=SPLIT,
                                                  split_long=SPLIT_LONG),
                         stream, 10)
        gotb = outb.cpu().numpy().view(np.uint32)
        cpu = cpu_rates(host, ob, lb)
        res["buckets"][str(b)] = {"spans": int(ob.size),
                                  "GiBps": round(float(lb.sum()) / tb / 2**30, 1),
                                  "cpu_1t_GiBps": cpu[0], "cpu_all_GiBps": cpu[1],
                                  "mismatches_in_sample": check_sample(host, ob, lb, gotb, rng,
                                                                       1000),
                                  "batch_latency": batch_latency(eng, dbuf, dob, dlb, stream,
                                                                 reps=100)}
    del dbuf
    return res


def run_tblocks(eng, d, stream, rng, gib=4.0):
    """Table-block-shaped device batch: data blocks as TableBuilder cuts them
    (4096 + the last entry: 4097..4225 bytes with the type byte), packed like
    an SST (contents + type, then the 4-byte crc), device-resident; spans
    kernel alone and with HCRC_SPLIT_SMALL (remainders to the small kernel)."""
    nbytes = int(gib * 2**30)
    dbuf = torch.empty(nbytes + 8192, dtype=torch.uint8, device=d)
    eng.fill_splitmix64_device(dbuf, 11, stream=stream.cuda_stream)
    n = nbytes // 4165
    lens = rng.integers(4097, 4226, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 4)[:-1]]).astype(np.uint64)
    do, dl = dev(offs, d), dev(lens, d)
    res = {"config": "table blocks 4097..4225 B (contents + type), SST-packed, device-resident",
           "spans": int(n), "bytes": int(lens.sum())}
    ref = None
    for split in (False, True):
        out = torch.empty(n, dtype=torch.int32, device=d)
        t = time_kernel(lambda: eng.batch_device(dbuf, do, dl, None, out, stream=stream.cuda_stream,
                                                     split_small=split), stream, 10)
        got = out.cpu().numpy()
        if ref is None:
            ref = got
        res["split" if split else "spans_kernel"] = {
            "GiBps": round(float(lens.sum()) / t / 2**30, 1), "ms": round(t * 1e3, 4),
            "same_as_unsplit": bool((got == ref).all())}
    del dbuf
    return res


def run_verify(eng, d, stream, rng, nblk=1 << 20):
    """Read side, device-resident (hcrc_verify_async, ReadBlock's check):
    1 M blocks of 4096 bytes on disk = 4091 contents + type byte + masked
    crc, every trailer stamped with the right crc, a few corrupted."""
    B, n = 4096, 4091
    data = torch.empty(nblk * B, dtype=torch.uint8, device=d)
    eng.fill_splitmix64_device(data, 7, stream=stream.cuda_stream)
    offs = torch.arange(nblk, dtype=torch.int64, device=d) * B
    lens = torch.full((nblk,), n + 1, dtype=torch.int32, device=d)
    crc = eng.batch_device(data, offs, lens, mask_output=True, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    trailer = data.view(nblk, B)[:, n + 1:n + 5]
    trailer.copy_(crc.view(torch.uint8).view(nblk, 4))
    bad = torch.from_numpy(rng.choice(nblk, 64, replace=False)).to(d)
    data.view(nblk, B)[bad, 100] ^= 1
    hl = torch.full((nblk,), n, dtype=torch.int32, device=d)
    st = torch.empty(nblk, dtype=torch.uint8, device=d)
    t = time_kernel(lambda: eng.verify_device(data, offs, hl, st, stream=stream.cuda_stream),
                    stream, 10)
    flagged = int((st == 0).sum())
    return {"config": "read side: ReadBlock verify of 1 M x 4 KiB device-resident blocks",
            "blocks": nblk, "GiBps": round(nblk * (n + 1) / t / 2**30, 1),
            "kernel_ms": round(t * 1e3, 4), "corrupted": 64, "flagged": flagged}


def run_vtblocks(eng, d, stream, rng, gib=4.0):
    """Read side on table-block-shaped data: 4096..4224-byte blocks + type
    byte + masked crc, SST-packed, device-resident; verify without and with
    HCRC_SPLIT_SMALL."""
    nbytes = int(gib * 2**30)
    n = nbytes // 4165
    lens = rng.integers(4096, 4225, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 5)[:-1]]).astype(np.uint64)
    size = (int(offs[-1]) + int(lens[-1]) + 5 + 8191) // 4096 * 4096
    data = torch.empty(size, dtype=torch.uint8, device=d)
    eng.fill_splitmix64_device(data, 13, stream=stream.cuda_stream)
    do, dl = dev(offs, d), dev(lens, d)
    crc = eng.batch_device(data, do, dev(lens + 1, d), mask_output=True, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    # stamp the trailers (byte n+1..n+4 of every block)
    pos = torch.from_numpy((offs + lens + 1).astype(np.int64)).to(d)
    cb = crc.view(torch.uint8).view(n, 4)
    for k in range(4):
        data[pos + k] = cb[:, k]
    torch.cuda.synchronize()
    res = {"config": "read side: verify of table blocks 4096..4224 B + type + crc, SST-packed",
           "blocks": int(n), "bytes": int((lens + 1).sum())}
    for split in (False, True):
        st = torch.empty(n, dtype=torch.uint8, device=d)
        t = time_kernel(lambda: eng.verify_device(data, do, dl, st, stream=stream.cuda_stream,
                                                  split_small=split), stream, 10)
        res["split" if split else "verify_kernel"] = {
            "GiBps": round(float((lens + 1).sum()) / t / 2**30, 1), "ms": round(t * 1e3, 4),
            "all_ok": bool((st == 1).all())}
    del data
    return res


def sst_layout(rng, n_sst):
    """8Binsert-shaped SSTs (test_bench/8Binsert.sh): spans cover contents +
    type byte; every block is followed by its 4-byte crc slot."""
    offs, lens, cur = [], [], 0
    for _ in range(n_sst):
        for _ in range(int(rng.integers(480, 520))):   # data blocks
            n = int(rng.integers(4096, 4225)) + 1
            offs.append(cur)
            lens.append(n)
            cur += n + 4
        for n in (int(rng.integers(15000, 20000)), int(rng.integers(24000, 26000)),
                  int(rng.integers(40, 100))):          # index, filter, metaindex
            offs.append(cur)
            lens.append(n + 1)
            cur += n + 5
        cur += 48  # footer
    return np.array(offs, np.uint64), np.array(lens, np.uint32), cur


def run_sst(eng, rng, n_sst):
    offs, lens, nbytes = sst_layout(rng, n_sst)
    host = rng.integers(32, 127, nbytes, dtype=np.uint8)  # printable, like CompressibleString
    eng.batch(host, offs, lens)  # warm: staging, copy stream and buffers allocated
    t0 = time.perf_counter()
    got = eng.batch(host, offs, lens, mask_output=True)
    t = time.perf_counter() - t0
    idx = rng.choice(offs.size, 4000, replace=False)
    want = cpu_batch(host, offs[idx], lens[idx], mask_output=True)
    tc0 = time.perf_counter()
    cpu_batch(host, offs, lens, mask_output=True, threads=16)
    tc = time.perf_counter() - tc0
    return {"config": "5 8Binsert SST stream, host memory, PCIe-inclusive (hcrc_batch HOST_PTRS)",
            "ssts": n_sst, "spans": int(offs.size), "bytes": int(lens.sum()),
            "GiBps_end_to_end": round(float(lens.sum()) / t / 2**30, 2),
            "cpu_16_threads_GiBps": round(float(lens.sum()) / tc / 2**30, 2),
            "mismatches_in_sample": int((want != got[idx]).sum())}


def pcie_h2d_ceiling(nbytes=1 << 30, reps=5):
    """The measured PCIe host-to-device ceiling: a pinned (torch
    pin_memory) -> HBM copy of nbytes by the copy engine, GiB/s."""
    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    del src, dst
    return round(nbytes / t / 2**30, 2)


def run_sst_pinned(eng, rng, n_sst):
    """Config 5 through the product path the table layer takes: the SST
    stream in pinned host memory (hcrc_host_alloc -- TableBuilder's pooled
    write buffers are such memory), hcrc_batch(HOST_PTRS) finds every span
    in it and needs no staging copy (dense pieces by the copy engine, the
    rest zero-copy), as a fraction of the measured PCIe H2D ceiling."""
    import ctypes
    from wipdb_amd import _lib
    lib = _lib.load()
    offs, lens, nbytes = sst_layout(rng, n_sst)
    pin = ctypes.c_void_p()
    _lib.check(lib.hcrc_host_alloc(nbytes, ctypes.byref(pin)), "hcrc_host_alloc")
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(pin.value))
        host[:] = rng.integers(32, 127, nbytes, dtype=np.uint8)
        eng.batch(host, offs, lens)  # warm: the slots and the copy-engine buffers allocated
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            got = eng.batch(host, offs, lens, mask_output=True)
        t = (time.perf_counter() - t0) / reps
        idx = rng.choice(offs.size, 4000, replace=False)
        want = cpu_batch(host, offs[idx], lens[idx], mask_output=True)
        ceiling = pcie_h2d_ceiling()
        rate = float(lens.sum()) / t / 2**30
        return {"config": "5 8Binsert SST stream in PINNED host memory (TableBuilder's write "
                          "buffers), hcrc_batch HOST_PTRS -> copy engine / zero-copy, PCIe-inclusive",
                "ssts": n_sst, "spans": int(offs.size), "bytes": int(lens.sum()),
                "GiBps_end_to_end": round(rate, 2), "pcie_h2d_ceiling_GiBps": ceiling,
                "fraction_of_pcie_ceiling": round(rate / ceiling, 3),
                "mismatches_in_sample": int((want != got[idx]).sum())}
    finally:
        lib.hcrc_host_free(pin)


def run_host4k(eng, rng, nblk):
    host = rng.integers(0, 256, nblk * 4096, dtype=np.uint8)
    offs = np.arange(nblk, dtype=np.uint64) * 4096
    lens = np.full(nblk, 4096, np.uint32)
    eng.batch(host, offs, lens)  # warm: staging, copy stream and buffers allocated
    t0 = time.perf_counter()
    got = eng.batch(host, offs, lens)
    t = time.perf_counter() - t0
    idx = rng.choice(nblk, 4000, replace=False)
    return {"config": "headline blocks from host memory (PCIe-inclusive, pageable source)",
            "blocks": nblk, "GiBps_end_to_end": round(nblk * 4096 / t / 2**30, 2),
            "mismatches_in_sample": int((cpu_batch(host, offs[idx], lens[idx]) != got[idx]).sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="mixed,sst,host4k")
    ap.add_argument("--split", action="store_true", help="HCRC_SPLIT_SMALL on device batches")
    ap.add_argument("--split-long", action="store_true",
                    help="HCRC_SPLIT_LONG on config 3's device batches")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU rates of config 3")
    ap.add_argument("--mixed-gib", type=float, default=2.0)
    ap.add_argument("--ssts", type=int, default=256)
    ap.add_argument("--host-blocks", type=int, default=1 << 18)
    a = ap.parse_args()
    global SPLIT, SPLIT_LONG, NO_CPU
    SPLIT = a.split
    NO_CPU = a.no_cpu
    SPLIT_LONG = a.split_long
    rng = np.random.default_rng(42)
    d = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(d)
    with Engine(0) as eng:
        for w in a.what.split(","):
            if w == "mixed":
                r = run_mixed(eng, d, stream, rng, a.mixed_gib)
            elif w == "verify":
                r = run_verify(eng, d, stream, rng)
            elif w == "tblocks":
                r = run_tblocks(eng, d, stream, rng)
            elif w == "vtblocks":
                r = run_vtblocks(eng, d, stream, rng)
            elif w == "sst":
                r = run_sst(eng, rng, a.ssts)
            elif w == "sstpin":
                r = run_sst_pinned(eng, rng, a.ssts)
            elif w == "host4k":
                r = run_host4k(eng, rng, a.host_blocks)
            else:
                raise SystemExit(f"unknown {w}")
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
