"""Average duration of a kernel's last K dispatches in a rocprofv3
--kernel-trace CSV (the timed launches of a bench run; the stats file
averages the warmup launches too).

  python scripts/trace_tail.py <rocprof output dir> <kernel name> <K>
"""
import csv
import glob
import json
import sys


def main():
    root, name, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    paths = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)
    assert paths, f"no kernel_trace.csv under {root}"
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if name in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    dur = [(e - s) / 1e6 for s, e in rows]
    tail = dur[-k:]
    print(json.dumps({"kernel": name, "dispatches": len(dur), "timed": len(tail),
                      "avg_ms_timed": round(sum(tail) / len(tail), 4),
                      "avg_ms_all": round(sum(dur) / len(dur), 4),
                      "min_ms": round(min(tail), 4), "max_ms": round(max(tail), 4)}))


if __name__ == "__main__":
    main()
