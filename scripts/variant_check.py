"""Parity spot-check of the kernel for per-wave slot patterns (which ring
slot processes which kind of segment).  Run with WIPDB_HCRC_LIB pointing at a
variant build.  Exits 1 on any mismatch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from tests.conftest import Oracle
from wipdb_amd import Engine

o = Oracle()
rng = np.random.default_rng(1)
W = 4096          # waves of the persistent grid (256 CUs x 16)
PITCH = 8192
MAXK = 4
buf = rng.integers(0, 256, W * MAXK * PITCH + 65536, dtype=np.uint8)
eng = Engine(0)
dbuf = torch.from_numpy(buf).cuda()
LEN = {"F": (0, 4096), "P": (0, 160), "N": (3, 1), "T": (0, 4100), "U": (5, 4090),
       "S": (7, 8000)}
fails = 0
for kinds in (["P"], ["F", "P"], ["P", "F"], ["P", "P"], ["P", "P", "P"], ["F", "F", "P"],
              ["N", "N"], ["F", "N"], ["T"], ["T", "T"], ["F", "F", "F", "P"],
              ["P", "F", "F", "F"], ["U", "S", "U"], ["S", "S", "S", "S"]):
    n = W * len(kinds)
    offs = np.zeros(n, np.uint64)
    lens = np.zeros(n, np.uint32)
    for k, kind in enumerate(kinds):
        i = np.arange(k * W, (k + 1) * W, dtype=np.uint64)
        offs[k * W:(k + 1) * W] = i * PITCH + LEN[kind][0]
        lens[k * W:(k + 1) * W] = LEN[kind][1]
    assert int((offs + lens).max()) <= buf.size
    out = eng.batch_device(dbuf, torch.from_numpy(offs.view(np.int64)).cuda(),
                           torch.from_numpy(lens.view(np.int32)).cuda())
    torch.cuda.synchronize()
    g = out.cpu().numpy().view(np.uint32)
    want = o.batch(buf, offs, lens)
    bad = (g != want).reshape(len(kinds), W).sum(axis=1)
    fails += int(bad.sum())
    print(f"{''.join(kinds):6s} bad per slot: {bad.tolist()}", flush=True)
    if bad[1:].any():  # how wrong: compare with plausible mix-ups
        G = g.reshape(len(kinds), W)
        Wt = want.reshape(len(kinds), W)
        k = int(np.nonzero(bad)[0][-1])
        ext = o.batch(buf, offs[k * W:(k + 1) * W], lens[k * W:(k + 1) * W], Wt[k - 1].copy())
        print("   slot", k, "got==want[slot-1]:", int((G[k] == Wt[k - 1]).sum()),
              "got==Extend(want[slot-1], span):", int((G[k] == ext).sum()),
              "got==0:", int((G[k] == 0).sum()),
              "got==want shifted by one wave:", int((G[k][1:] == Wt[k][:-1]).sum()),
              "sample", [hex(int(x)) for x in G[k][:2]], [hex(int(x)) for x in Wt[k][:2]],
              flush=True)
# many short spans per wave (pitch 256): which output lanes go wrong
kinds = 40
n = W * kinds
offs = np.arange(n, dtype=np.uint64) * 256
lens = np.full(n, 160, np.uint32)
out = eng.batch_device(dbuf, torch.from_numpy(offs.view(np.int64)).cuda(),
                       torch.from_numpy(lens.view(np.int32)).cuda())
torch.cuda.synchronize()
g = out.cpu().numpy().view(np.uint32)
want = o.batch(buf, offs, lens)
bad = (g != want).reshape(kinds, W).sum(axis=1)
fails += int(bad.sum())
print("P x40 bad per slot:", bad.tolist(), flush=True)
print("VARIANT", os.environ.get("WIPDB_HCRC_LIB", "default"), "OK" if fails == 0 else "FAIL")
sys.exit(1 if fails else 0)
