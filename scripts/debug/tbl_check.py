import sys, os, json
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/scripts')
import numpy as np, torch
from bench_extra import dev, time_kernel
from bench_configs import table_layout
from wipdb_amd import Engine
d = torch.device('cuda', 0); stream = torch.cuda.current_stream(d)
rng = np.random.default_rng(5)
for gib in (2.0, 4.0):
    offs, lens = table_layout(rng, gib)
    n = offs.size; size = int(offs[-1]) + int(lens[-1]) + 4
    data = torch.empty(size, dtype=torch.uint8, device=d)
    with Engine(0) as eng:
        eng.fill_splitmix64_device(data[: size // 8 * 8], 0x7AB1E5, stream=stream.cuda_stream)
        do, dl = dev(offs, d), dev(lens, d)
        out = torch.empty(n, dtype=torch.int32, device=d)
        for r in range(3):
            for m in ('default', 'packed', 'balance'):
                t = time_kernel(lambda: eng.batch_device(data, do, dl, None, out, stream=stream.cuda_stream,
                                packed=(m == 'packed'), balance=(m == 'balance')), stream, 10)
                print(gib, r, m, round(t * 1e3, 4), round(float(lens.sum()) / t / 2**30, 1), flush=True)
    del data
