#!/usr/bin/env python3
"""Per-kernel mean of each PMC counter in rocprofv3 counter_collection CSVs.
  python scripts/pmc_summary.py DIR [DIR...] [--kernel SUBSTR]"""
import csv
import glob
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = "spans_kernel"
if "--kernel" in sys.argv:
    ksub = sys.argv[sys.argv.index("--kernel") + 1]
    args = [a for a in args if a != ksub]
for d in args:
    acc = defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
