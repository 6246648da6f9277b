"""Summary of a rocprofv3 --kernel-trace --memory-copy-trace run of
scripts/pinned_dma_probe.py (one layout): the last call's timeline -- each
host-to-device copy of >= 1 MiB (the copy engine's pieces) with its
duration, rate and the gap since the previous one, and the CRC kernels
between them.

  python scripts/copy_trace_summary.py <rocprof output dir> > summary.log
"""
import csv
import glob
import json
import sys


def main():
    root = sys.argv[1]
    ev = []
    for p in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel",
                       r["Kernel_Name"].split("(")[0].replace("void ", "")[:60], 0))
    for p in glob.glob(f"{root}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            n = int(r.get("Bytes", r.get("Size", 0)) or 0)
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", r["Direction"], n))
    ev.sort()
    big = [e for e in ev if e[2] == "copy" and e[3].endswith("HOST_TO_DEVICE") and (e[4] >= 1 << 20 or e[1] - e[0] > 500_000)]
    # the last call: the big copies after the last gap of > 150 us between them (17 us within a call)
    calls, cur = [], [big[0]]
    for a, b in zip(big, big[1:]):
        if b[0] - a[1] > 150_000:
            calls.append(cur)
            cur = []
        cur.append(b)
    calls.append(cur)
    last = calls[-1]
    t0, t1 = last[0][0], max(e[1] for e in ev if e[0] >= last[0][0])
    out = {"calls_seen": len(calls), "copies": []}
    prev = None
    for e in last:
        d = {"start_us": round((e[0] - t0) / 1e3, 1), "ms": round((e[1] - e[0]) / 1e6, 3)}
        if e[4]:
            d["MiB"] = round(e[4] / 2**20, 1)
            d["GiBps"] = round(e[4] / ((e[1] - e[0]) / 1e9) / 2**30, 2)
        if prev is not None:
            d["gap_us"] = round((e[0] - prev[1]) / 1e3, 1)
        out["copies"].append(d)
        prev = e
    ks = [e for e in ev if e[2] == "kernel" and t0 <= e[0] <= t1]
    out["kernels"] = [{"start_us": round((e[0] - t0) / 1e3, 1), "us": round((e[1] - e[0]) / 1e3, 1),
                       "name": e[3]} for e in ks if "crc32c" in e[3]]
    out["call_span_ms"] = round((t1 - t0) / 1e6, 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
