"""Per-launch kernel time of the headline batch (1 M x 4 KiB, spans entry
point) over a long back-to-back series: does the rate settle after the
first launches (clocks, TLB), and how much do launches vary?

  python scripts/launch_series.py [--launches 200] [--blocks N] [--idle-ms 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wipdb_amd.crc32c import Engine  # noqa: E402


def span_order(order, n, dev):
    idx = torch.arange(n, dtype=torch.int64, device=dev)
    if order == "natural":
        return idx
    if order == "random":
        g = torch.Generator(device="cpu").manual_seed(7)
        return torch.randperm(n, generator=g).to(dev)
    G = torch.cuda.get_device_properties(dev).multi_processor_count * 16 * 2
    assert n % G == 0
    q, k = idx % G, idx // G
    if order == "group":
        return q * (n // G) + k
    per_wg = 32
    return (q // per_wg) * (n // (G // per_wg)) + k * per_wg + q % per_wg


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--launches", type=int, default=200)
    p.add_argument("--blocks", type=int, default=1 << 20)
    p.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between launches")
    p.add_argument("--buffers", type=int, default=1,
                   help="allocate this many copies of the batch and run them round robin "
                        "(is the rate a property of the allocation?)")
    p.add_argument("--pre-alloc-gib", type=float, default=0.0,
                   help="allocate (and keep) this much device memory before the batches")
    p.add_argument("--desc-first", action="store_true",
                   help="allocate the descriptor and output columns before the batches")
    p.add_argument("--order", choices=["natural", "group", "cu", "random"], default="natural",
                   help="span order of the descriptor columns (bench.py --order; random: a "
                        "seeded permutation)")
    p.add_argument("--what", choices=["spans", "strided", "readstream"], default="spans",
                   help="readstream: the same blocks through readstream_kernel (no CRC work)")
    p.add_argument("--pre-what", choices=["spans", "strided", "readstream"], default=None,
                   help="run this many untimed launches of another kernel first (--pre-launches)")
    p.add_argument("--pre-launches", type=int, default=0)
    p.add_argument("--series", action="store_true", help="print every launch time")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    n = a.blocks
    st = torch.cuda.current_stream(dev)
    pre = (torch.empty(int(a.pre_alloc_gib * 2**30), dtype=torch.uint8, device=dev)
           if a.pre_alloc_gib else None)
    if a.desc_first:
        offs = span_order(a.order, n, dev) * 4096
        lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
    bufs = []
    for _ in range(a.buffers):
        bufs.append(torch.empty(n * 4096, dtype=torch.uint8, device=dev))
        eng.fill_splitmix64_device(bufs[-1], 0x4B10C5, stream=st.cuda_stream)
    if not a.desc_first:
        offs = span_order(a.order, n, dev) * 4096
        lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    def launch(what, data):
        if what == "spans":
            eng.batch_device(data, offs, lens, None, out, stream=st.cuda_stream)
        elif what == "strided":
            eng.batch_strided_device(data, 4096, 4096, n, 0, out, stream=st.cuda_stream)
        else:
            eng.readstream_device(data, 4096, 4096, n, out, stream=st.cuda_stream)

    for i in range(a.pre_launches):
        launch(a.pre_what, bufs[i % a.buffers])
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.launches)]
    for i, (s, e) in enumerate(ev):
        data = bufs[i % a.buffers]
        s.record(st)
        launch(a.what, data)
        e.record(st)
        if a.idle_ms:
            torch.cuda.synchronize(dev)
            time.sleep(a.idle_ms / 1e3)
    torch.cuda.synchronize(dev)
    ms = np.array([s.elapsed_time(e) for s, e in ev])
    res = {"what": a.what, "blocks": n, "idle_ms": a.idle_ms, "first10": [round(float(x), 4) for x in ms[:10]]}
    for lo, hi in [(0, 3), (3, 23), (3, 53), (20, 70), (50, 100), (100, 200)]:
        if hi <= len(ms):
            res[f"mean[{lo}:{hi}]"] = round(float(ms[lo:hi].mean()), 4)
    if len(ms) >= 1000:
        res["per500"] = [round(float(ms[i:i + 500].mean()), 4) for i in range(0, len(ms) - 499, 500)]
    if a.buffers > 1:
        res["per_buffer"] = [round(float(ms[b::a.buffers][10:].mean()), 4) for b in range(a.buffers)]
        res["buffer_addr_MiB"] = [b.data_ptr() >> 20 for b in bufs]
    if a.series:
        res["series"] = [round(float(x), 3) for x in ms]
    res["pct(5,50,95)"] = [round(float(x), 4) for x in np.percentile(ms, [5, 50, 95])]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
