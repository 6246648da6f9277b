#!/usr/bin/env python3
"""Kernel time of the descriptor batch on synthetic span shapes (1 M spans
each unless noted): which part of a span's shape costs time -- the head
(unaligned start), the tail (length % 16), the piece (chunks past 256).
Prints one JSON line per shape; checks a sample against the CPU path.
--verify: the same byte footprints through the verify kernel (handle size
n = length - 5: contents + type byte + stored crc = length bytes read)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wipdb_amd import Engine, cpu_batch  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "scripts"))
from bench_extra import dev, time_kernel  # noqa: E402

SHAPES = [  # name, start offset in slot, length, slot stride
    ("aligned 4096", 0, 4096, 4096),
    ("aligned 4080 (f 255, no tail; window at -16)", 0, 4080, 4096),
    ("aligned 4064 (window at -32)", 0, 4064, 4096),
    ("aligned 4032 (window at -64)", 0, 4032, 4096),
    ("aligned 3968 (window at -128)", 0, 3968, 4096),
    ("head 64, 4032 (window at 0)", 64, 4032, 4096),
    ("aligned 4092 (f 255, tail 12)", 0, 4092, 4096),
    ("head 16, 4080 (f 255 at +16)", 16, 4080, 4096),
    ("head 3, 4093 (f 256, no tail)", 3, 4093, 4096),
    ("aligned 4099 (tail 3)", 0, 4099, 4112),
    ("head 3, 4096 (tail 3)", 3, 4096, 4112),
    ("aligned 4112 (piece 1)", 0, 4112, 4112),
    ("aligned 4208 (piece 7)", 0, 4208, 4208),
    ("head 5, 4200 (piece 6 + tail)", 5, 4200, 4224),
]


def main():
    args = [a for a in sys.argv[1:] if a != "--verify"]
    verify = "--verify" in sys.argv[1:]
    only = args[0] if args else ""
    d = torch.device("cuda", 0)
    st = torch.cuda.current_stream(d)
    n = 1 << 20
    rng = np.random.default_rng(1)
    with Engine(0) as eng:
        buf = torch.empty(n * 4224 + 4096, dtype=torch.uint8, device=d)
        eng.fill_splitmix64_device(buf, 5, stream=st.cuda_stream)
        host = None
        for name, h, ln, stride in SHAPES:
            if only and only not in name:
                continue
            offs = (np.arange(n, dtype=np.uint64) * stride + h).astype(np.uint64)
            lens = np.full(n, ln, np.uint32)
            if verify:
                # timing only: the trailers are random, so the statuses are too
                dl = dev(np.full(n, ln - 5, np.uint32), d)
                do = dev(offs, d)
                st8 = torch.empty(n, dtype=torch.uint8, device=d)
                t = time_kernel(lambda: eng.verify_device(buf, do, dl, st8, stream=st.cuda_stream),
                                st, 20)
                print(json.dumps({"shape": name, "verify": True, "ms": round(t * 1e3, 4),
                                  "GiBps": round(float(lens.sum()) / t / 2**30, 1)}), flush=True)
                continue
            do, dl = dev(offs, d), dev(lens, d)
            out = torch.empty(n, dtype=torch.int32, device=d)
            t = time_kernel(lambda: eng.batch_device(buf, do, dl, None, out, stream=st.cuda_stream), st, 20)
            if host is None:
                host = buf.cpu().numpy()
            idx = rng.choice(n, 2000, replace=False)
            got = out.cpu().numpy().view(np.uint32)[idx]
            bad = int((cpu_batch(host, offs[idx], lens[idx]) != got).sum())
            print(json.dumps({"shape": name, "ms": round(t * 1e3, 4),
                              "GiBps": round(float(lens.sum()) / t / 2**30, 1), "mismatches": bad}),
                  flush=True)


if __name__ == "__main__":
    main()
