#!/usr/bin/env python3
"""Debug probe of the spans kernel: several shaped batches, each checked
against the oracle; prints mismatch counts and the first mismatching spans
(index, offset, length, got, want).  GPU box only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.conftest import Oracle  # noqa: E402
from wipdb_amd import Engine  # noqa: E402


def t(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


def run(eng, oracle, name, buf, offs, lens, inits=None, verify=False):
    offs = np.asarray(offs, np.uint64)
    lens = np.asarray(lens, np.uint32)
    want = oracle.batch(buf, offs, lens, inits)
    out = torch.full((offs.size,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    eng.batch_device(t(buf), t(offs), t(lens), None if inits is None else t(np.asarray(inits, np.uint32)),
                     out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != want)[0]
    unwritten = int((got[bad] == 0x5A5A5A5A).sum())
    print(f"{name}: {bad.size}/{offs.size} bad ({unwritten} unwritten)", flush=True)
    for i in bad[:8]:
        print(f"   i={i} off={int(offs[i])} len={int(lens[i])} got={int(got[i]):08x} want={int(want[i]):08x}")
    if bad.size:
        lb = lens[bad]
        print("   bad lengths: min", int(lb.min()), "max", int(lb.max()),
              "hist", np.histogram(lb, bins=[0, 1, 4, 16, 64, 256, 1024, 4096, 4097, 8192, 1 << 30])[0].tolist())


def main():
    rng = np.random.default_rng(1)
    oracle = Oracle()
    buf = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    with Engine(0) as eng:
        run(eng, oracle, "one 100B", buf, [64], [100])
        run(eng, oracle, "one 4096 aligned", buf, [4096], [4096])
        run(eng, oracle, "one 8192", buf, [4096], [8192])
        run(eng, oracle, "one 5000", buf, [4096 + 3], [5000])
        run(eng, oracle, "16 x 100B", buf, np.arange(16) * 128, [100] * 16)
        run(eng, oracle, "17 x 100B", buf, np.arange(17) * 128, [100] * 17)
        run(eng, oracle, "64 x 512B aligned", buf, np.arange(64) * 512, [512] * 64)
        run(eng, oracle, "200 x 512B", buf, np.arange(200) * 600 + 3, [512] * 200)
        run(eng, oracle, "16 x 4096", buf, np.arange(16) * 4096, [4096] * 16)
        run(eng, oracle, "1000 x 4096", buf, np.arange(1000) * 4096, [4096] * 1000)
        run(eng, oracle, "100 x 8192", buf, np.arange(100) * 8192, [8192] * 100)
        n = 2000
        lens = rng.integers(0, 300, n)
        run(eng, oracle, "2000 x 0..300", buf, np.arange(n) * 400 + 5, lens)
        lens = rng.integers(4097, 4226, n)
        run(eng, oracle, "2000 table blocks", buf, np.concatenate([[0], np.cumsum(lens + 4)[:-1]]), lens)
        lens = rng.choice([100, 600, 4096, 5000, 9000], n)
        run(eng, oracle, "2000 mixed", buf, np.concatenate([[0], np.cumsum(lens + 4)[:-1]]), lens)


if __name__ == "__main__":
    main()
