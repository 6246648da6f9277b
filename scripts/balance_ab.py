"""HCRC_BALANCE A/B on the GPU: config 3's Zipf mix (2 GiB, SST-packed,
bench_extra.zipf_spans), single buckets, table blocks and the 1 M x 4 KiB
headline shape, each timed with and without byte-balanced workgroup ranges
in alternating rounds (same session); the balanced outputs are compared with
the default ones over the whole batch, and a sample with the CPU path.
  python scripts/balance_ab.py [rounds]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_extra import BUCKETS, dev, time_kernel, zipf_spans  # noqa: E402
from wipdb_amd import Engine  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    d = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(d)
    rng = np.random.default_rng(42)
    nbytes = 2 << 30
    shapes = {}
    o, l, _ = zipf_spans(rng, nbytes, BUCKETS)
    shapes["mix"] = (o, l)
    for b in (1024, 8192, 65536):
        ob, lb, _ = zipf_spans(rng, nbytes, [b])
        shapes[f"b{b}"] = (ob, lb)
    lt = rng.integers(4097, 4226, nbytes // 4230).astype(np.uint32)
    ot = np.concatenate([[0], np.cumsum(lt.astype(np.uint64) + 5)[:-1]]).astype(np.uint64) + 3
    shapes["tblocks"] = (ot, lt)
    n4 = nbytes // 4096  # 512 Ki aligned 4 KiB blocks, and the headline's 1 Mi over 4 GiB
    shapes["4k"] = (np.arange(n4, dtype=np.uint64) * 4096, np.full(n4, 4096, np.uint32))
    shapes["4k_1M"] = (np.arange(2 * n4, dtype=np.uint64) * 4096, np.full(2 * n4, 4096, np.uint32))
    # the buffer the shapes need, to the byte (the 1 Mi-block shape covers 4
    # GiB); every shape's spans are checked against it once before timing
    need = max(int(o[-1]) + int(l[-1]) for o, l in shapes.values())
    dbuf = torch.empty(need, dtype=torch.uint8, device=d)
    res = {}
    with Engine(0) as eng:
        eng.fill_splitmix64_device(dbuf, 11, stream=stream.cuda_stream)
        for name, (o, l) in shapes.items():
            do, dl = dev(o, d), dev(l, d)
            eng.check_spans(dbuf.numel(), do, dl)  # raises on a span past the buffer
            out0 = torch.empty(o.size, dtype=torch.int32, device=d)
            out1 = torch.empty(o.size, dtype=torch.int32, device=d)
            t = {"default": [], "balance": []}
            arg = {"default": False, "balance": True}
            for _ in range(rounds):
                for mode, out in (("default", out0), ("balance", out1)):
                    out.fill_(0x5A5A5A5A)
                    t[mode].append(time_kernel(
                        lambda: eng.batch_device(dbuf, do, dl, None, out, stream=stream.cuda_stream,
                                                 balance=arg[mode]), stream, 10))
            torch.cuda.synchronize()
            diff = int((out0 != out1).sum().item())
            idx = rng.choice(o.size, 512, replace=False)
            host = None
            hb = dbuf.cpu().numpy() if name == "mix" else None
            if hb is not None:
                host = eng.batch(hb, o[idx], l[idx])
                ok = int((host != out1.cpu().numpy().view(np.uint32)[idx]).sum())
            else:
                ok = None
            byt = float(l.sum())
            r = {"spans": int(o.size), "bytes": int(byt), "mismatch_vs_default": diff,
                 "mismatch_sample_vs_host_path": ok}
            for mode in t:
                ms = [x * 1e3 for x in t[mode]]
                r[mode + "_ms"] = [round(x, 4) for x in ms]
                r[mode + "_GiBps"] = round(byt / (min(ms) / 1e3) / 2**30, 1)
            r["gain"] = round(r["balance_GiBps"] / r["default_GiBps"] - 1.0, 4)
            res[name] = r
            print(name, json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
