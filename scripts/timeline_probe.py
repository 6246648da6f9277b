"""Where does a spans launch spend its time?  Runs the headline batch
(1 M x 4 KiB, device-resident) through a WIPDB_TIMELINE variant build and
prints, per workgroup, the wall-clock stamps the kernel wrote: entry,
tables in LDS, and each wave's end -- the prologue cost, the spread of
workgroup start times and the tail (first wave done -> last wave done).

  scripts/build_variant.sh timeline -DWIPDB_TIMELINE=1
  WIPDB_HCRC_LIB=build/variants/timeline/libhip_crc32c_batch.so \\
      python scripts/timeline_probe.py [--blocks N]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wipdb_amd import _lib  # noqa: E402
from wipdb_amd.crc32c import Engine  # noqa: E402

WAVES = 16
STRIDE = 2 + WAVES
TICK_NS = 10.0  # s_memrealtime: 100 MHz constant clock


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--blocks", type=int, default=1 << 20)
    p.add_argument("--len", type=int, default=4096)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    fn = lib.hcrc_debug_timeline
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    n = a.blocks
    data = torch.empty(n * 4096 + 4096, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    eng.fill_splitmix64_device(data, 0x4B10C5, stream=st.cuda_stream)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    lens = torch.full((n,), a.len, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    for r in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        eng.batch_device(data, offs, lens, None, out, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize(dev)
        ev_ms = e0.elapsed_time(e1)
        buf = np.zeros(ncu * STRIDE, np.uint64)
        got = fn(buf.ctypes.data, buf.size)
        assert got == buf.size, got
        t = buf.reshape(ncu, STRIDE).astype(np.int64)
        t0 = t[:, 0].min()
        rel = (t - t0) * TICK_NS / 1000.0  # us
        entry, tables, done = rel[:, 0], rel[:, 1], rel[:, 2:]
        wg_done = done.max(axis=1)
        xcd = np.arange(ncu) % 8
        res = {
            "rep": r, "event_ms": round(ev_ms, 4),
            "span_us": round(float(done.max()), 1),
            "entry_us": [round(float(x), 1) for x in np.percentile(entry, [0, 50, 100])],
            "tables_us(after entry)": [round(float(x), 1) for x in
                                       np.percentile(tables - entry, [0, 50, 100])],
            "wave_done_us": [round(float(x), 1) for x in np.percentile(done, [0, 1, 10, 50, 90, 99, 100])],
            "wg_done_by_xcd_us": [round(float(wg_done[xcd == x].mean()), 1) for x in range(8)],
            "idle_tail_frac": round(float(1.0 - done.mean() / done.max()), 4),
            "done_by_wave_us": [round(float(x), 1) for x in done.mean(axis=0)],
            "wg_spread_us": [round(float(x), 1) for x in
                             np.percentile(done.max(axis=1) - done.min(axis=1), [0, 50, 100])],
            "wg_done_us": [round(float(x), 1) for x in np.percentile(wg_done, [0, 10, 50, 90, 100])],
        }
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
