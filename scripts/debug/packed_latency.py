#!/usr/bin/env python3
"""Per-call latency of HCRC_PACKED against the default path on small
SST-packed device batches (one SST of 2 MiB .. 32 MiB): the pre-pass's two
extra stream operations (a memset and the index kernel) against the
kernel's own time.  p50 of 200 synchronised calls each.
  python scripts/debug/packed_latency.py [MiB,...] [span,...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_extra import dev  # noqa: E402
from wipdb_amd import Engine  # noqa: E402


def main():
    d = torch.device("cuda", 0)
    s = torch.cuda.current_stream(d)
    rng = np.random.default_rng(3)
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,8,32").split(",")]
    spans = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1024,4096").split(",")]
    buf = torch.randint(0, 256, ((max(sizes) + 1) << 20,), dtype=torch.uint8, device=d)
    with Engine(0) as eng:
        for mib in sizes:
            for span in spans:
                n = (mib << 20) // (span + 5)
                lens = rng.integers(span, span + span // 8 + 1, n).astype(np.uint32)
                offs = 3 + np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 5)[:-1]])
                keep = offs + lens <= buf.numel()
                do, dl = dev(offs[keep].astype(np.uint64), d), dev(lens[keep], d)
                out = torch.empty(int(keep.sum()), dtype=torch.int32, device=d)
                res = {}
                for mode in ("default", "packed", "default", "packed"):
                    ts = []
                    for _ in range(200 if mib <= 64 else 40):
                        t0 = time.perf_counter()
                        eng.batch_device(buf, do, dl, None, out, stream=s.cuda_stream, packed=(mode == "packed"))
                        s.synchronize()
                        ts.append(time.perf_counter() - t0)
                    res[mode] = round(float(np.percentile(ts, 50)) * 1e6, 1)
                print(f"{mib} MiB of {span} B spans ({int(keep.sum())} spans): p50 us {res}", flush=True)


if __name__ == "__main__":
    main()
