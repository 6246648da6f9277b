#!/usr/bin/env python3
"""Per-dispatch clock of the spans kernel from a rocprofv3 --pmc CSV:
SQ_CYCLES / (dispatch ns) summed over the SQs, GRBM_GUI_ACTIVE / ns, and the
instruction counts; the mean over the timed dispatches (the last half)."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    rows = defaultdict(dict)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "spans_kernel" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[k]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    ks = sorted(rows)[len(rows) // 2:]
    if not ks:
        print(d, "no dispatches")
        continue
    m = {c: sum(rows[k][c] for k in ks) / len(ks) for c in rows[ks[0]]}
    print(d, {"dispatches": len(ks), "kernel_ms": round(m["ns"] / 1e6, 4),
              "grbm_GHz": round(m.get("GRBM_GUI_ACTIVE", 0) / m["ns"], 3),
              "sq_cycles_per_ns": round(m.get("SQ_CYCLES", 0) / m["ns"], 2),
              "valu": int(m.get("SQ_INSTS_VALU", 0)), "salu": int(m.get("SQ_INSTS_SALU", 0)),
              "wave_cycles": int(m.get("SQ_WAVE_CYCLES", 0)), "busy": int(m.get("SQ_BUSY_CYCLES", 0))})
