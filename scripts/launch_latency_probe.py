"""Host time of the first launches after a device synchronize (the bench's
timed region starts that way): event record, first and second headline
launch, each timed on the host, medians over repetitions.

  python scripts/launch_latency_probe.py [--reps 15]
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--blocks", type=int, default=1 << 20)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    n = a.blocks
    st = torch.cuda.current_stream(dev)
    data = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    eng.fill_splitmix64_device(data, 1, stream=st.cuda_stream)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    lib, ctx = eng._lib, eng._ctx
    args = (ctx, data.data_ptr(), offs.data_ptr(), lens.data_ptr(), None, out.data_ptr(), n, 1,
            st.cuda_stream)

    def step_py():
        eng.batch_device(data, offs, lens, None, out, stream=st.cuda_stream)

    def step_c():
        lib.hcrc_batch_async(*args)

    for _ in range(30):
        step_py()
    torch.cuda.synchronize(dev)
    res = {}
    for name in ["event_then_step", "step_only", "c_step_only", "event_then_c_step",
                 "after_query_spin", "after_long_queue", "after_long_queue_c",
                 "after_events_queue"]:
        t = []
        for _ in range(a.reps if "queue" not in name else max(3, a.reps // 4)):
            if name == "after_events_queue":  # the precondition's form
                pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                         for _ in range(200)]
                for s0, s1 in pairs:
                    s0.record(st)
                    step_py()
                    s1.record(st)
            for _ in range(200 if "long_queue" in name else 4):
                step_py()
            torch.cuda.synchronize(dev)
            e = torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            if name == "after_query_spin":
                while not torch.cuda.current_stream(dev).query():
                    pass
            if name.startswith("event") or "queue" in name:
                e.record(st)
            t1 = time.perf_counter()
            (step_c if "c_step" in name else step_py)()
            t2 = time.perf_counter()
            (step_c if "c_step" in name else step_py)()
            t3 = time.perf_counter()
            t.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6))
        torch.cuda.synchronize(dev)
        m = np.median(np.array(t), axis=0)
        res[name] = {"pre_us": round(float(m[0]), 1), "first_launch_us": round(float(m[1]), 1),
                     "second_launch_us": round(float(m[2]), 1)}
    print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
