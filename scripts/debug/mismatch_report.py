"""Debug aid: run the golden spans through the device path and print which
(h = start % 16, length, init) classes mismatch the oracle."""
import collections
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.conftest import Oracle, load_golden_spans  # noqa: E402
from wipdb_amd import Engine  # noqa: E402


def t(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to("cuda:0")


def main():
    g = load_golden_spans()
    with Engine(0) as eng:
        dbuf = t(g["buf"])
        out = eng.batch_device(dbuf, t(g["offsets"]), t(g["lengths"]), t(g["inits"]))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        base = dbuf.data_ptr()
    bad = np.nonzero(got != g["crc"])[0]
    print("bad", bad.size, "of", got.size, "base%16", base % 16)
    cls = collections.Counter()
    for i in bad:
        n = int(g["lengths"][i]); h = int(g["offsets"][i] + base) % 16
        f = (h + n) >> 4
        cls[(h != 0, "nc<256" if 0 < f % 256 else "full", (h + n) % 16 != 0, int(g["inits"][i]) != 0, (f + 255) // 256)] += 1
    for k, v in sorted(cls.items(), key=lambda kv: -kv[1])[:30]:
        print(k, v)
    ok = np.nonzero(got == g["crc"])[0]
    cls2 = collections.Counter()
    for i in ok:
        n = int(g["lengths"][i]); h = int(g["offsets"][i] + base) % 16
        f = (h + n) >> 4
        cls2[(h != 0, "nc<256" if 0 < f % 256 else "full", (h + n) % 16 != 0, int(g["inits"][i]) != 0, (f + 255) // 256)] += 1
    print("ok classes:")
    for k, v in sorted(cls2.items(), key=lambda kv: -kv[1])[:30]:
        print(k, v)
    for i in bad[:12]:
        print(i, int(g["offsets"][i]), int(g["lengths"][i]), hex(int(g["inits"][i])), hex(int(got[i])), hex(int(g["crc"][i])))


if __name__ == "__main__":
    main()
