"""Average SQ/GRBM counters per launch of crc32c_*_kernel from rocprofv3
--pmc output directories (gpurun_out/<prefix>*), per stride, with derived
per-span instruction counts and busy fractions.

    python scripts/pmc_summary.py ROOT PREFIX
"""
import collections
import csv
import glob
import json
import os
import sys

root, prefix = sys.argv[1], sys.argv[2]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(root, prefix + "*", "**", "*counter_collection.csv"),
                      recursive=True):
    stride = path.split(prefix)[1].split("_")[0]
    with open(path) as f:
        for row in csv.DictReader(f):
            if "crc32c_" in row["Kernel_Name"] and "_kernel" in row["Kernel_Name"]:
                by[stride][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for stride, cs in sorted(by.items()):
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    spans = 1 << 20
    d = {k: round(v) for k, v in avg.items()}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
        if k in avg:
            d[k + "_per_span"] = round(avg[k] / spans, 1)
    if "SQ_WAVE_CYCLES" in avg:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                d[k + "_frac_of_wave_cycles"] = round(avg[k] / avg["SQ_WAVE_CYCLES"], 3)
    out[stride] = d
print(json.dumps(out, indent=1))
