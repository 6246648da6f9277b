#!/usr/bin/env python3
"""Per-shape mean of each PMC counter (per span) from gpu_shapes_pmc.sh output:
dispatches of the spans kernel are grouped in shape order."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
kern = sys.argv[2] if len(sys.argv) > 2 else "spans_kernel"
rows = []
for f in glob.glob(f"{d}/shapes_pmc/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = collections.defaultdict(dict)
for r in rows:
    if kern in r["Kernel_Name"]:
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(by)
shapes = [json.loads(x) for x in open(f"{d}/shapes.log") if x.startswith("{")]
per = len(ids) // max(1, len(shapes))
n = 1 << 20
for i, sh in enumerate(shapes):
    grp = ids[i * per:(i + 1) * per]
    cs = sorted(by[grp[0]])
    vals = {c: sum(by[g].get(c, 0) for g in grp) / len(grp) / n for c in cs}
    print(f"{sh['shape'][:34]:34s} {sh['ms']:.4f} ms " +
          " ".join(f"{c.replace('SQ_INSTS_', '').replace('SQ_', '')}={v:.4g}" for c, v in vals.items()))
