#!/usr/bin/env python3
"""Headline benchmark: device-resident GiB/s of batched CRC32C over 4 KiB
blocks on 1..8 MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A "step" is one launch of the batch entry point (hcrc_batch_async, the
descriptor path a table builder would use) over this rank's whole shard of
4 KiB blocks already resident in HBM, generated on device with a seeded
splitmix64 stream.  N = 1: 1 M blocks (4 GiB, BASELINE configs[1]);
N > 1: 8 M blocks (32 GiB) per rank, i.e. configs[3]'s 64 M x 4 KiB over 8
GPUs.  Weak scaling: every rank has its own shard; there is no data-path
collective (blocks are independent) -- only the barrier and the max-time
reduction of the contract.  value = total bytes of all ranks / max time.

Before the W warmup steps the bench preconditions the card with untimed
launches of the same step (at least --precondition-ms of GPU time, 250 by
default) and checks that every one of them returns the same CRCs: right
after idle, back-to-back launches of this kernel run up to 1.5x slower for
the first ~30-60 ms while the SMU settles the power-capped clocks
(profiles/r02_launch_series.json); the timed steps measure the steady state.
The compare kernels torch uses for the check are loaded before the window
(their first use cost ~250 ms of GPU idle inside it), so the
window is continuous GPU work; the line reports the mean kernel time of the
window's first and last 10 launches, so the settling is visible
("precondition").  The W warmup steps are queued right behind the window
and its per-launch times are read only after the timed region: a host pause
of >= 2 ms between the window and the timed steps (round 5 read 382 event
pairs there) let the memory clocks drop and cost the timed launches 4-6 %
(profiles/r06a_gap_*.log, scripts/gap_probe.py).

Also printed in the same JSON line:
  roofline      the CRC kernel's average launch time from HIP events on the
                launch stream -- by default one event pair around the K
                timed launches (time / K: the ~1.5 us dispatch gaps count
                against the kernel); --events step puts a pair around every
                launch instead (per-launch times and their minimum, but
                ~5 us of event packets between launches inside the timed
                region: profiles/r04x_events.log); achieved = algorithmic
                bytes per launch (4096 + 4 per block) / that time, vs the
                8 TB/s HBM peak;
                traffic = PMC HBM bytes per launch from the committed rocprof
                profile of this config (profiles/traffic.json), or null.
  cpu_baseline  the reference kv::crc32c (oracle/_ref, compiled from the
                reference's own sources) on this host, 1 thread, over the
                shard's blocks copied back from HBM (config 1's 4 GiB from
                DRAM), and on every CPU this process may use; rank 0, N=1.
  parity        the reference CRCs vs the GPU's for every block of the shard
                (N = 1) or a 64 Ki-block sample per rank (N > 1).
  ceiling       this box's ceiling for the kernel: the spans kernel's own
                memory side alone (hcrc_dma_ceiling_async -- the table image,
                the unit deal, the same LDS-DMAs and slot reads, 4 B stored
                per block, no CRC) over the same shard, after the timed
                region; roofline frac_of_ceiling = ceiling time / kernel
                time with both timed alternating back to back in runs of
                K / 2 (frac_of_ceiling_alternating; the same power and
                clock state for both).  roofline.timed_dispatch_first
                = the index of the first timed launch among this process's
                CRC-kernel dispatches (spans or packed kernel, one a
                step; scripts/trace_timed.py picks the K timed ones out of
                a rocprofv3 kernel trace).
  config3_mixed, table_blocks, verified_table_blocks, config5_pcie
                (rank 0, N = 1, after the headline; --no-extra skips them)
                BASELINE configs[2] and [4] under the same clock: config 3's
                Zipf-mixed SST-packed batch and its per-bucket GiB/s and p99
                batch latency, WriteRawBlock-shaped table blocks and their
                ReadBlock verify (device-resident), and config 5's 8Binsert
                SST stream from pinned host memory (copy engine, PCIe-inclusive)
                against a measured PCIe H2D ceiling; every one sample-checked
                against the reference's kv::crc32c (oracle/_ref).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BLOCK = 4096
ALGO_BYTES_PER_BLOCK = BLOCK + 4  # L bytes read + 4 bytes written
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md: 8.0 TB/s spec
SEED = 0x4B10C5


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)  # >= 50 back-to-back launches
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--precondition-ms", type=float, default=250.0,
                   help="untimed GPU time of same-step launches before the warmup (power "
                        "transient, see the docstring); 0 disables")
    p.add_argument("--blocks", type=int, default=0,
                   help="blocks per GPU (default: 1 M at N = 1, 8 M per rank at N > 1)")
    p.add_argument("--mode", choices=["spans", "strided"], default="spans")
    p.add_argument("--events", choices=["step", "bracket"], default="bracket",
                   help="HIP events around every timed launch (per-launch kernel times) or "
                        "only around the timed region (no event between launches)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--poll-events", action="store_true",
                   help="diagnostic: poll the timed region's events before the synchronize")
    p.add_argument("--cpu-seconds", type=float, default=5.0,
                   help="minimum time of the 1-thread reference baseline (whole passes)")
    p.add_argument("--no-ceiling", "--no-readstream", dest="no_ceiling", action="store_true",
                   help="skip the same-box ceiling kernel (timed after the headline)")
    p.add_argument("--no-extra", action="store_true",
                   help="skip configs 3 / 5 and the table-block shapes after the headline")
    return p.parse_args()


def _ref_batch():
    """The reference kv::crc32c batch driver (oracle/_ref, compiled from the
    reference's own sources), or the oracle restatement (a port)."""
    ref_path = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
    if os.path.exists(ref_path):
        lib = ctypes.CDLL(ref_path)
        fn = lib.ref_crc32c_batch
        fn.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        return fn, "reference"
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    ofn = lib.oracle_crc32c_batch
    ofn.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int]

    def fn(b, o, l, i, out, n, m, t):  # noqa: E741
        ofn(b, o, l, i, out, n, m)
    return fn, "port"


def usable_cpus() -> int:
    """CPUs this process may use: the affinity mask, capped by the job's CPU
    share when the launcher states one (OMP_NUM_THREADS; the GPU box gives a
    one-GPU job 16 of the host's 256 CPUs)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        share = 0
    return min(n, share) if share > 0 else n


def cpu_check(host_blocks, gpu_crc, target_s, baseline: bool):
    """Reference CRCs of every given block (all usable CPUs) vs the GPU's;
    with `baseline`, also the reference's rate on 1 thread (whole passes
    over the blocks, at least target_s) and on all usable CPUs."""
    import numpy as np
    fn, kind = _ref_batch()
    nblk = host_blocks.size // BLOCK
    offs = np.arange(nblk, dtype=np.uint64) * BLOCK
    lens = np.full(nblk, BLOCK, np.uint32)
    out = np.empty(nblk, np.uint32)
    args = (host_blocks.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, out.ctypes.data)
    ncpu = usable_cpus()
    fn(*args, nblk, 0, ncpu)
    mism = int((out != gpu_crc[:nblk]).sum())
    parity = {"blocks_checked": int(nblk), "mismatches": mism}
    if not baseline:
        return None, parity
    passes, t0 = 0, time.perf_counter()
    while True:
        fn(*args, nblk, 0, 1)
        passes += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    gib_s = passes * nblk * BLOCK / el / 2**30
    # all usable CPUs, timed the same way (whole passes for >= target_s; the
    # parity pass above was the warm one)
    apasses, t0 = 0, time.perf_counter()
    while True:
        fn(*args, nblk, 0, ncpu)
        apasses += 1
        ael = time.perf_counter() - t0
        if ael >= target_s:
            break
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(gib_s, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
        "sample": f"all {nblk} x 4 KiB blocks of rank 0's shard ({nblk * BLOCK >> 20} MiB, "
                  f"copied back from HBM, read from DRAM), {passes} pass(es) in {el:.1f} s, "
                  f"ref kv::crc32c::Extend per block",
        "all_cores": {"value": round(apasses * nblk * BLOCK / ael / 2**30, 3), "cores": ncpu,
                      "sample": f"{apasses} whole passes over the same blocks in {ael:.1f} s "
                                f"after a warm pass, on every CPU this job may use (affinity "
                                f"mask capped by OMP_NUM_THREADS)"},
        "host": {"cpu": cpu_model, "nproc": os.cpu_count(), "usable_cpus": ncpu,
                 "hostname": socket.gethostname()},
    }, parity


def committed_traffic(mode: str, blocks: int):
    """HBM bytes per launch from the committed PMC profile, if one matches."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(f"{mode}_{blocks}")
        return None if e is None else e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


KERNEL = {"spans": "crc32c_lds_spans_kernel", "strided": "crc32c_lds_strided_kernel"}


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    from wipdb_amd import Engine
    from wipdb_amd.shard import block_shard, max_over_ranks

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # WIPDB_BENCH_REHEARSAL=1 (tests only): more ranks than GPUs share the
    # visible ones and talk over gloo -- rehearses the N > 1 path on a one-GPU
    # box (RCCL refuses two ranks on one device); the driver's runs are one
    # rank per GPU over RCCL
    rehearsal = os.environ.get("WIPDB_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local %= max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    blocks = a.blocks or ((1 << 20) if world == 1 else (8 << 20))

    eng = Engine(local)
    first, nblk = block_shard(rank, world, blocks)  # weak scaling, no collective
    data = torch.empty(nblk * BLOCK, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    eng.fill_splitmix64_device(data, SEED, first_word=first * BLOCK // 8, stream=stream.cuda_stream)
    offs = torch.arange(nblk, dtype=torch.int64, device=dev) * BLOCK
    lens = torch.full((nblk,), BLOCK, dtype=torch.int32, device=dev)
    out = torch.empty(nblk, dtype=torch.int32, device=dev)

    def step(dst=out):
        if a.mode == "spans":
            eng.batch_device(data, offs, lens, None, dst, stream=stream.cuda_stream)
        else:
            eng.batch_strided_device(data, BLOCK, BLOCK, nblk, 0, dst, stream=stream.cuda_stream)

    # precondition: untimed back-to-back launches of the step (at least
    # precondition_ms of GPU time), every output compared with the first.
    # The warmup steps follow on the stream with no host wait in between, and
    # the per-launch times are read only after the timed region: a host-side
    # pause of even 2 ms lets the memory clocks drop, and the next ~20
    # launches then run 5-18 % slower (profiles/r06a_gap_*.log,
    # scripts/gap_probe.py) -- the timed steps must start from the settled
    # state the precondition reached, not from an idle card.
    pre = {"launches": 0, "gpu_ms": 0.0, "identical_outputs": True}
    pev = []
    if a.precondition_ms > 0:
        ref = torch.empty_like(out)
        scratch = torch.empty_like(out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        step(ref)
        e0.record(stream)
        step(scratch)
        e1.record(stream)
        mism = torch.zeros((), dtype=torch.int64, device=dev)
        mism += (scratch != ref).sum()  # torch's compare / reduce kernels loaded here
        torch.cuda.synchronize(dev)
        n = max(16, min(4096, int(a.precondition_ms / max(e0.elapsed_time(e1), 1e-3)) + 1))
        pev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(n)]
        e0.record(stream)
        for ps, pe in pev:
            ps.record(stream)
            step(scratch)
            pe.record(stream)
            mism += (scratch != ref).sum()
        e1.record(stream)
        pre["launches"] = n + 2

    nev = a.steps if a.events == "step" else 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(nev)]
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    # One marker on the stream and a second synchronize before the timed
    # region: the HIP runtime releases the completed commands of the stream
    # (here the precondition's ~1500 launches and markers) at the next enqueue,
    # which cost the timed region's first event record 0.2-0.4 ms of host time
    # (timed_region_host_ms.event_recorded, profiles/r06f_host.log); it also
    # creates the timed events (torch creates a HIP event at its first record).
    for es, ee in ev:
        es.record(stream)
        ee.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if a.events == "step":
        for s, e in ev:
            s.record(stream)
            step()
            e.record(stream)
    else:
        ev[0][0].record(stream)
        t_rec = time.perf_counter()
        for i in range(a.steps):
            step()
            if i == 0:
                t_first = time.perf_counter()
        ev[0][1].record(stream)
    t_queued = time.perf_counter()
    t_started = None
    if a.poll_events and a.events != "step":  # (diagnostic: when did the GPU reach the bracket?)
        while not ev[0][0].query():
            pass
        t_started = time.perf_counter()
        while not ev[0][1].query():
            pass
    torch.cuda.synchronize(dev)
    t_synced = time.perf_counter()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    host_ms = {"event_recorded": round((t_rec - t0) * 1e3, 3) if a.events != "step" else None,
               "first_launch_returned": round((t_first - t0) * 1e3, 3) if a.events != "step" else None,
               "all_queued": round((t_queued - t0) * 1e3, 3),
               "gpu_started_seen": None if t_started is None else round((t_started - t0) * 1e3, 3),
               "synced": round((t_synced - t0) * 1e3, 3), "elapsed": round(elapsed * 1e3, 3)}
    kern_ms = [s.elapsed_time(e) * nev / a.steps for s, e in ev]
    kern_avg_ms = sum(kern_ms) / len(kern_ms)

    elapsed_max = max_over_ranks(elapsed, dev)
    kern_avg_ms = max_over_ranks(kern_avg_ms, dev)

    if pev:
        pk = [ps.elapsed_time(pe) for ps, pe in pev]
        pre.update({"gpu_ms": round(e0.elapsed_time(e1), 2),
                    "kernel_ms_sum": round(sum(pk), 2),
                    "first10_kernel_ms": round(sum(pk[:10]) / 10, 4),
                    "last10_kernel_ms": round(sum(pk[-10:]) / 10, 4),
                    "identical_outputs": int(mism.item()) == 0,
                    "why": "after idle, back-to-back launches run up to 1.5x slower for ~30-60 ms "
                           "while the SMU raises the clocks again (profiles/r02_launch_series.json, "
                           "r06a_gap_*.log); the warmup and timed steps follow with no host pause"})
        del ref, scratch, pev

    ceil = None
    if not a.no_ceiling and a.mode == "spans":
        # The same-box ceiling: the spans kernel's memory side alone on the
        # same shard (hcrc_dma_ceiling_async: the image load, the unit deal,
        # the same LDS-DMAs and slot reads, 4 B stored per block, no CRC).
        # Warmed back to back for >= 100 ms from the timed region's end, then
        # K ceiling launches and K more CRC launches alternating in rounds of
        # K / 2, one event pair per run, nothing between them on the stream.
        c_out = torch.empty(nblk, dtype=torch.int32, device=dev)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        eng.dma_ceiling_device(data, BLOCK, nblk, c_out, stream=stream.cuda_stream)
        s1.record(stream)
        torch.cuda.synchronize(dev)
        nw = max(16, int(100.0 / max(s0.elapsed_time(s1), 1e-3)))
        for _ in range(nw):
            eng.dma_ceiling_device(data, BLOCK, nblk, c_out, stream=stream.cuda_stream)
        half = max(1, a.steps // 2)
        runs = []
        for r in range(4):
            b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b0.record(stream)
            for _ in range(half):
                if r % 2 == 0:
                    eng.dma_ceiling_device(data, BLOCK, nblk, c_out, stream=stream.cuda_stream)
                else:
                    step()
            b1.record(stream)
            runs.append((r % 2, b0, b1))
        torch.cuda.synchronize(dev)
        cms = [b0.elapsed_time(b1) / half for k, b0, b1 in runs if k == 0]
        kms = [b0.elapsed_time(b1) / half for k, b0, b1 in runs if k == 1]
        c_ms, k_ms = sum(cms) / len(cms), sum(kms) / len(kms)
        heads = data.view(nblk, BLOCK)[:, :64].contiguous().view(torch.int32)
        want = heads[:, 0]
        for j in range(1, 16):
            want = torch.bitwise_xor(want, heads[:, j])
        ceil = {"kernel": "crc32c_dma_ceiling_kernel", "avg_ms": round(c_ms, 4),
                "GBps": round(nblk * ALGO_BYTES_PER_BLOCK / c_ms / 1e6, 1),
                "crc_kernel_ms_alternating": round(k_ms, 4),
                "frac_of_ceiling_alternating": round(c_ms / k_ms, 4),
                "words_checked": int(nblk), "word_mismatches": int((c_out != want).sum().item()),
                "what": "the spans kernel's memory side alone (table image, unit deal, the same "
                        "LDS-DMAs and slot reads, 4 B stored per block, no CRC) over the same "
                        "shard on this box, after the timed region; alternating with the CRC "
                        "kernel in runs of K/2 back to back"}
        del c_out, heads, want

    # parity (and, rank 0 at N = 1, the CPU baseline) on the host
    gpu_crc = out.cpu().numpy().view(np.uint32)
    full = world == 1
    nchk = nblk if full else min(nblk, 1 << 16)
    host_blocks = data[: nchk * BLOCK].cpu().numpy()
    cb, par = cpu_check(host_blocks, gpu_crc, a.cpu_seconds,
                        baseline=(rank == 0 and world == 1 and not a.no_cpu_baseline))
    del host_blocks
    if world > 1:
        t = torch.tensor([par["mismatches"], par["blocks_checked"]], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        par = {"blocks_checked": int(t[1].item()), "mismatches": int(t[0].item()),
               "scope": "64 Ki-block sample per rank"}

    extra = {}
    if rank == 0 and world == 1 and not a.no_extra:
        from scripts.bench_configs import run_all
        extra = run_all(eng, dev, stream, _ref_batch()[0])

    if rank == 0:
        total_bytes = world * nblk * BLOCK
        value = total_bytes * a.steps / elapsed_max / 2**30
        achieved = nblk * ALGO_BYTES_PER_BLOCK / (kern_avg_ms * 1e-3) / 1e9
        if nblk == 1 << 20 and world == 1:
            cfg = "BASELINE configs[1]"
        elif nblk == 8 << 20:
            cfg = "BASELINE configs[3]: its 8 M-block per-GPU shard" + (
                " (one GPU)" if world == 1 else "")
        else:
            cfg = "custom size (--blocks)"
        line = {
            "metric": "device-resident GiB/s, batched CRC32C of 4 KiB blocks, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device-generated splitmix64, seed 0x4B10C5)",
            "config": {"workload": f"{nblk} x 4 KiB blocks per GPU, device-resident "
                                   f"({cfg}); {a.mode} entry point",
                       "blocks_per_gpu": nblk, "block_bytes": BLOCK,
                       "parallelism": f"shard{world} (independent blocks, no collective)"},
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": committed_traffic(a.mode, nblk),
                "kernel": KERNEL[a.mode],
                "kernel_avg_ms": round(kern_avg_ms, 4),
                "kernel_min_ms": round(min(kern_ms), 4) if a.events == "step" else None,
                "kernel_timing": ("HIP events around each timed launch" if a.events == "step" else
                                  "HIP events around the timed launches / K"),
                "algorithmic_bytes_per_launch": nblk * ALGO_BYTES_PER_BLOCK,
                "timed_dispatch_first": pre["launches"] + a.warmup,
            },
            "timed_region_host_ms": host_ms,
            "precondition": pre,
        }
        if ceil:
            # the ceiling and the CRC kernel timed alternating, back to back
            # (the same power / clock state): the timed region itself runs
            # right after the precondition and reads 1-2 % faster than
            # anything measured after it (profiles/r06g_bench.log), so the
            # ratio to the timed kernel is listed beside it, not used
            line["ceiling"] = ceil
            line["roofline"]["frac_of_ceiling"] = ceil["frac_of_ceiling_alternating"]
            line["roofline"]["ceiling_ms_over_timed_kernel_ms"] = round(ceil["avg_ms"] / kern_avg_ms, 4)
        if cb:
            line["cpu_baseline"] = cb
        line["parity"] = par
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
