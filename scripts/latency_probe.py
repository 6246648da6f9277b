"""Where a synchronised SST-sized batch's microseconds go (VERDICT r5 item 6:
p50 31-54 us for ~2 MiB device-resident batches, the shape BuildTableKV
hands the CRC per flushed SST, kv/src/db/builder.cc:18-109).

For one ~2 MiB batch of WriteRawBlock table blocks (and of config 3's 512 B
spans), `reps` times each:
  launch_us    host time of the launch call (Python + ctypes + hipLaunch)
  kernel_us    HIP events around the launch (GPU time, incl. dispatch)
  wall_us      host wall time launch -> completion seen, per wait method:
               torch.cuda.synchronize (the bench's batch_latency), hcrc_sync
               on the stream, and a spin on hipStreamQuery (torch query)
Prints medians / p99 as one JSON line; run it under rocprofv3 --kernel-trace
to split the kernel's own duration from the dispatch.

  python scripts/latency_probe.py [--reps 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wipdb_amd.crc32c import Engine  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=300)
    p.add_argument("--mib", type=float, default=2.0)
    a = p.parse_args()
    from bench_configs import table_layout
    from bench_extra import zipf_spans
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    st = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(5)
    shapes = {}
    offs, lens = table_layout(rng, a.mib / 1024)
    shapes["table_blocks"] = (offs, lens)
    o5, l5, _ = zipf_spans(rng, int(a.mib * 2**20), [512])
    shapes["spans_512"] = (o5, l5)
    res = {}
    for name, (offs, lens) in shapes.items():
        size = int(offs[-1]) + int(lens[-1]) + 8
        buf = torch.empty((size + 7) // 8 * 8, dtype=torch.uint8, device=dev)
        eng.fill_splitmix64_device(buf, 9, stream=st.cuda_stream)
        do = torch.from_numpy(offs.astype(np.int64)).to(dev)
        dl = torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(offs.size, dtype=torch.int32, device=dev)
        lib, ctx = eng._lib, eng._ctx
        args = (ctx, buf.data_ptr(), do.data_ptr(), dl.data_ptr(), None, out.data_ptr(),
                offs.size, 1, st.cuda_stream)
        r = {"spans": int(offs.size), "bytes": int(lens.sum())}
        for method in ["torch_sync", "hcrc_sync", "query_spin"]:
            launch, kern, wall = [], [], []
            for i in range(a.reps + 20):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                s.record(st)
                lib.hcrc_batch_async(*args)
                e.record(st)
                t1 = time.perf_counter()
                if method == "torch_sync":
                    torch.cuda.synchronize(dev)
                elif method == "hcrc_sync":
                    lib.hcrc_sync(ctx, st.cuda_stream)
                else:
                    while not st.query():
                        pass
                t2 = time.perf_counter()
                if i >= 20:
                    launch.append((t1 - t0) * 1e6)
                    wall.append((t2 - t0) * 1e6)
                    kern.append(s.elapsed_time(e) * 1e3)
            r[method] = {k: {"p50": round(float(np.percentile(v, 50)), 1),
                             "p99": round(float(np.percentile(v, 99)), 1)}
                         for k, v in (("launch_us", launch), ("kernel_us", kern), ("wall_us", wall))}
        res[name] = r
        del buf, do, dl, out
    print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
