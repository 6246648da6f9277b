"""The K timed dispatches of a bench.py run out of its rocprofv3
--kernel-trace CSV: the CRC-kernel dispatches (spans or packed kernel: one
per step) [first, first + K) of the process, first = the line's
roofline.timed_dispatch_first (the precondition's launches + the warmup).  Prints their average / min / max duration, the gaps
between them, and the average over every dispatch of the kernel (what the
--stats summary averages) for comparison.

  python scripts/trace_timed.py <rocprof output dir> <bench log with the JSON line>
"""
import csv
import glob
import json
import sys


def main():
    root, log = sys.argv[1], sys.argv[2]
    line = None
    with open(log) as f:
        for t in f:
            if t.startswith("{") and '"metric"' in t:
                line = json.loads(t)
    assert line, f"no bench line in {log}"
    first = int(line["roofline"]["timed_dispatch_first"])
    k = int(line["steps"])
    name = line["roofline"]["kernel"]
    # every step is ONE launch of the spans kernel or of the packed kernel
    # (device batches of >= 32 Ki spans take the packed sequence until the
    # stream's verdict for the batch -- "suits run_ea" -- is back on the
    # host; the precondition's first launches do), so both count
    names = (name, "crc32c_lds_packed_kernel")
    paths = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)
    assert paths, f"no kernel_trace.csv under {root}"
    rows, kinds = [], []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if any(k in r["Kernel_Name"] for k in names):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                 name in r["Kernel_Name"]))
    rows.sort()
    timed = rows[first:first + k]
    assert len(timed) == k, f"{len(rows)} dispatches, wanted [{first}, {first + k})"
    kinds = sorted({("spans" if t[2] else "packed") for t in timed})
    dur = [(e - s) / 1e6 for s, e, _ in timed]
    gaps = [(timed[i + 1][0] - timed[i][1]) / 1e3 for i in range(k - 1)]
    alld = [(e - s) / 1e6 for s, e, sp in rows if sp]
    span_ms = (timed[-1][1] - timed[0][0]) / 1e6
    out = {"kernel": name, "timed_kernels": kinds, "dispatches": len(rows), "timed_first": first,
           "timed": k,
           "avg_ms_timed": round(sum(dur) / k, 4), "min_ms": round(min(dur), 4),
           "max_ms": round(max(dur), 4), "gap_us_avg": round(sum(gaps) / max(1, len(gaps)), 2),
           "first_start_to_last_end_ms_per_launch": round(span_ms / k, 4),
           "line_kernel_avg_ms": line["roofline"]["kernel_avg_ms"],
           "avg_ms_all_dispatches": round(sum(alld) / len(alld), 4),
           "achieved_GBps_trace": round(line["roofline"]["algorithmic_bytes_per_launch"]
                                         / (sum(dur) / k) / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
