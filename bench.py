#!/usr/bin/env python3
"""Headline benchmark: device-resident GiB/s of batched CRC32C over 4 KiB
blocks on 1..8 MI355X (BASELINE.json metric, configs[1] per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A "step" is one launch of the batch entry point (hcrc_batch_async, the
descriptor path a table builder would use) over this rank's whole shard:
1 M blocks x 4 KiB (4 GiB) already resident in HBM, generated on device with
a seeded splitmix64 stream (so the host can regenerate any block).  Weak
scaling: every rank has its own 1 M-block shard; there is no data-path
collective (blocks are independent) -- only the barrier and the max-time
reduction of the contract.  value = total bytes of all ranks / max time.

Also printed in the same JSON line:
  roofline      the CRC kernel's average launch time from HIP events on the
                launch stream; achieved = algorithmic bytes per launch
                (4096 + 4 per block) / that time, vs the 8 TB/s HBM peak;
                traffic = PMC HBM bytes per launch from the committed rocprof
                profile of this config (profiles/), or null.
  cpu_baseline  the reference kv::crc32c (oracle/_ref, compiled from the
                reference's own sources) on this host, 1 thread, over a
                bounded sample of the same blocks; rank 0, N=1 only.
  parity        the sample's reference CRCs vs the GPU's for the same blocks.
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
    # the first ~20 back-to-back launches of a fresh process run 5-15 % slow
    # while the card's clocks settle under sustained load
    # (scripts/launch_series.py): the default warmup
    # covers them, so the timed steps see the steady state
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--blocks", type=int, default=1 << 20, help="blocks per GPU")
    p.add_argument("--mode", choices=["spans", "strided"], default="spans")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="target CPU time of the reference baseline sample")
    p.add_argument("--readstream", action="store_true",
                   help="also time the read-stream ceiling kernel")
    p.add_argument("--stride", type=int, default=BLOCK,
                   help="diagnostic: block stride (0 = every block reads the same 4 KiB, "
                        "i.e. cache-resident compute ceiling); the headline uses 4096")
    p.add_argument("--len", type=int, default=BLOCK, choices=range(0, 65537), metavar="0..65536",
                   help="diagnostic: bytes CRC'd per block (<= stride; e.g. 4092 = a 4 KiB "
                        "on-disk block minus its 5-byte trailer, plus the type byte)")
    p.add_argument("--fill", choices=["splitmix", "zero"], default="splitmix",
                   help="diagnostic: block contents (zero = low-toggle data, to probe "
                        "the power/clock limit); the headline uses splitmix")
    p.add_argument("--order", choices=["natural", "group", "cu"], default="natural",
                   help="diagnostic: which block each descriptor names (natural: block i; "
                        "group: every lane group sweeps its own contiguous run; cu: every "
                        "workgroup sweeps its own contiguous region)")
    return p.parse_args()


def cpu_baseline(seed, blocks_on_gpu_crc, first_block, target_s):
    """Reference kv::crc32c on this host over a bounded sample of rank 0's
    blocks (regenerated from the seed), 1 thread; plus the parity check of
    those CRCs against the GPU's."""
    import numpy as np
    from tests.golden.common import splitmix64_bytes
    ref_path = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
    kind = "reference"
    if os.path.exists(ref_path):
        lib = ctypes.CDLL(ref_path)
        fn = lib.ref_crc32c_batch
        fn.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    else:  # fall back to the oracle restatement (a port), still a CPU baseline
        kind = "port"
        lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
        ofn = lib.oracle_crc32c_batch
        ofn.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int]

        def fn(b, o, l, i, out, n, m, t):  # noqa: E741
            ofn(b, o, l, i, out, n, m)
    nblk = 1 << 16  # 64 Ki blocks = 256 MiB sample
    buf = splitmix64_bytes(seed, nblk * BLOCK, start=first_block * BLOCK)
    offs = (np.arange(nblk, dtype=np.uint64) * BLOCK)
    lens = np.full(nblk, BLOCK, np.uint32)
    out = np.empty(nblk, np.uint32)
    args = (buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, out.ctypes.data)
    fn(*args, nblk, 0, 1)  # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        fn(*args, nblk, 0, 1)
        passes += 1
        el = time.perf_counter() - t0
        if el >= target_s or passes >= 400:
            break
    gib_s = passes * nblk * BLOCK / el / 2**30
    mism = int((out != blocks_on_gpu_crc[:nblk]).sum())
    t16, tt0 = 16, time.perf_counter()
    fn(*args, nblk, 0, t16)
    fn(*args, nblk, 0, t16)
    all_gib = 2 * nblk * BLOCK / (time.perf_counter() - tt0) / 2**30
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
        "sample": f"{nblk} x 4 KiB blocks (256 MiB) of rank 0's shard regenerated on the host, "
                  f"{passes} passes ({el:.1f} s), ref kv::crc32c::Extend per block",
        "all_cores": {"value": round(all_gib, 3), "cores": t16},
        "host": {"cpu": cpu_model, "nproc": os.cpu_count(), "hostname": socket.gethostname()},
    }, {"blocks_checked": nblk, "mismatches": mism}


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
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    eng = Engine(local)
    first, nblk = block_shard(rank, world, a.blocks)  # weak scaling, no collective
    # diagnostic spans longer than the 4 KiB pitch (--len > 4096) or a wider
    # --stride run past nblk * 4 KiB: size the buffer so every span stays
    # inside the allocation
    need = max(nblk * BLOCK, (nblk - 1) * max(a.stride, 0) + a.len)
    data = torch.empty((need + 4095) // 4096 * 4096, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    if a.fill == "zero":
        data.zero_()
    else:
        eng.fill_splitmix64_device(data, SEED, first_word=first * BLOCK // 8,
                                   stream=stream.cuda_stream)
    idx = torch.arange(nblk, dtype=torch.int64, device=dev)
    if a.order != "natural":
        # span s is taken by lane group q = s % G at step k = s // G of the
        # persistent grid (G = groups in the grid)
        G = torch.cuda.get_device_properties(dev).multi_processor_count * 16 * 2
        assert nblk % G == 0, "diagnostic orders need blocks divisible by the grid's groups"
        q, k = idx % G, idx // G
        if a.order == "group":
            idx = q * (nblk // G) + k
        else:
            per_wg = 2 * 16  # groups per workgroup
            idx = (q // per_wg) * (nblk // (G // per_wg)) + k * per_wg + q % per_wg
    offs = idx * a.stride
    lens = torch.full((nblk,), a.len, dtype=torch.int32, device=dev)
    out = torch.empty(nblk, dtype=torch.int32, device=dev)

    def step():
        if a.mode == "spans":
            eng.batch_device(data, offs, lens, None, out, stream=stream.cuda_stream)
        else:
            eng.batch_strided_device(data, a.stride, BLOCK, nblk, 0, out, stream=stream.cuda_stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = sorted(s.elapsed_time(e) for s, e in ev)
    kern_avg_ms = sum(kern_ms) / len(kern_ms)

    elapsed_max = max_over_ranks(elapsed, dev)
    kern_avg_ms = max_over_ranks(kern_avg_ms, dev)

    rs = None
    if a.readstream:
        rs_out = torch.empty(nblk, dtype=torch.int32, device=dev)
        for _ in range(2):
            eng.readstream_device(data, BLOCK, BLOCK, nblk, rs_out, stream=stream.cuda_stream)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        for _ in range(a.steps):
            eng.readstream_device(data, BLOCK, BLOCK, nblk, rs_out, stream=stream.cuda_stream)
        s1.record(stream)
        torch.cuda.synchronize(dev)
        rs_ms = s0.elapsed_time(s1) / a.steps
        rs = {"kernel": "readstream_kernel", "avg_ms": round(rs_ms, 4),
              "read_GBps": round(nblk * BLOCK / rs_ms / 1e6, 1)}

    if rank == 0:
        total_bytes = world * nblk * BLOCK
        value = total_bytes * a.steps / elapsed_max / 2**30
        achieved = nblk * ALGO_BYTES_PER_BLOCK / (kern_avg_ms * 1e-3) / 1e9
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
                                   f"(BASELINE configs[1]); {a.mode} entry point",
                       "blocks_per_gpu": nblk, "block_bytes": BLOCK,
                       "parallelism": f"shard{world} (independent blocks, no collective)"},
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": committed_traffic(a.mode, nblk),
                "kernel": "crc32c_spans_kernel" if a.mode == "spans" else "crc32c_strided_kernel",
                "kernel_avg_ms": round(kern_avg_ms, 4),
                "algorithmic_bytes_per_launch": nblk * ALGO_BYTES_PER_BLOCK,
            },
        }
        if rs:
            line["readstream_ceiling"] = rs
        if a.len != BLOCK:
            line["config"]["diagnostic_len"] = a.len
            line["metric"] += " [DIAGNOSTIC len]"
        if a.fill != "splitmix":
            line["config"]["diagnostic_fill"] = a.fill
            line["metric"] += " [DIAGNOSTIC fill]"
        if a.order != "natural":
            line["config"]["diagnostic_order"] = a.order
            line["metric"] += " [DIAGNOSTIC order]"
        if a.stride != BLOCK:
            line["config"]["diagnostic_stride"] = a.stride
            line["metric"] += " [DIAGNOSTIC stride, not the headline]"
        if (world == 1 and not a.no_cpu_baseline and a.stride == BLOCK and a.fill == "splitmix"
                and a.len == BLOCK):
            gpu_crc = out.cpu().numpy().view(np.uint32)
            cb, par = cpu_baseline(SEED, gpu_crc, first, a.cpu_seconds)
            line["cpu_baseline"] = cb
            line["parity"] = par
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
