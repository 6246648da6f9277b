#!/usr/bin/env python3
"""HCRC_PACKED (the stream-tiled kernel) against the default pipeline on
config 3's shapes, same session: per shape, the default batch and the same
batch declared packed, alternating rounds, min of the rounds; outputs
compared over the whole batch.

  python scripts/packed_ab.py [rounds] [shape,...] [--only default|packed]

Shapes: b512 b1024 b2048 b4096 b8192 b65536 (one Zipf bucket, SST-packed,
gap 5, 2 GiB), mix (config 3's Zipf mix), tblocks (WriteRawBlock spans
4097..4225 + 4-byte trailer), a4k (1 Mi aligned 4 KiB blocks, the
headline's), walN (WAL-record-like spans of N..2N-1 bytes behind 7-byte
headers).  --only runs one mode (for rocprofv3 --pmc passes)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_extra import BUCKETS, dev, time_kernel, zipf_spans  # noqa: E402
from wipdb_amd import Engine  # noqa: E402


def shape_of(name, rng, nbytes):
    if name == "mix":
        o, l, _ = zipf_spans(rng, nbytes, BUCKETS)
    elif name.startswith("b"):
        o, l, _ = zipf_spans(rng, nbytes, [int(name[1:])])
    elif name == "tblocks":
        l = rng.integers(4097, 4226, nbytes // 4230).astype(np.uint32)
        o = np.concatenate([[0], np.cumsum(l.astype(np.uint64) + 4)[:-1]]).astype(np.uint64) + 3
    elif name.startswith("wal"):  # walN: WAL-record-like spans N..2N-1 B, 7-byte headers between
        b = int(name[3:])
        l = rng.integers(b, 2 * b, int(nbytes // (1.5 * b + 7))).astype(np.uint32)
        o = np.concatenate([[0], np.cumsum(l.astype(np.uint64) + 7)[:-1]]).astype(np.uint64) + 7
    elif name == "a4k":
        n = 2 * nbytes // 4096
        o, l = np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096, np.uint32)
    else:
        raise SystemExit(f"unknown shape {name}")
    return o.astype(np.uint64), l.astype(np.uint32)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    only = None
    if "--only" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1]
        args = [a for a in args if a != only]
    rounds = int(args[0]) if args else 3
    shapes = (args[1] if len(args) > 1 else "b512,b1024,b2048,b4096,b8192,b65536,mix,tblocks,a4k").split(",")
    d = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(d)
    rng = np.random.default_rng(42)
    nbytes = 2 << 30
    dbuf = torch.empty(2 * nbytes, dtype=torch.uint8, device=d)
    res = {}
    with Engine(0) as eng:
        eng.fill_splitmix64_device(dbuf, 11, stream=stream.cuda_stream)
        for name in shapes:
            o, l = shape_of(name, rng, nbytes)
            do, dl = dev(o, d), dev(l, d)
            eng.check_spans(dbuf.numel(), do, dl)
            outs = {"default": torch.empty(o.size, dtype=torch.int32, device=d),
                    "packed": torch.empty(o.size, dtype=torch.int32, device=d)}
            modes = [only] if only else ["default", "packed"]
            t = {m: [] for m in modes}
            for _ in range(rounds):
                for m in modes:
                    t[m].append(time_kernel(
                        lambda: eng.batch_device(dbuf, do, dl, None, outs[m], stream=stream.cuda_stream,
                                                 packed=(m == "packed")), stream, 10))
            torch.cuda.synchronize()
            byt = float(l.sum())
            r = {"spans": int(o.size), "bytes": int(byt)}
            for m in modes:
                r[m + "_GiBps"] = round(byt / min(t[m]) / 2**30, 1)
                r[m + "_ms"] = [round(x * 1e3, 4) for x in t[m]]
            if not only:
                r["same"] = bool((outs["default"] == outs["packed"]).all())
                r["gain"] = round(r["packed_GiBps"] / r["default_GiBps"] - 1.0, 4)
            res[name] = r
            print(name, json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
