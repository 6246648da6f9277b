"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py into
profiles/traffic.json (HBM bytes per launch of the CRC kernel) and a short
markdown summary.  Corrections per /opt/skills/guides/MI355X_MICROARCH.md
(HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a 16-B/lane streaming read, so it is doubled.

    python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR KEY OUT_PREFIX
"""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter, kernel_sub):
    vals = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter and kernel_sub in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, key, prefix = sys.argv[1:5]
    kern = "crc32c_lds_spans_kernel" if key.startswith("spans") else "crc32c_lds_strided_kernel"
    f = per_kernel(fdir, "FETCH_SIZE", kern)
    w = per_kernel(wdir, "WRITE_SIZE", kern)
    if not f or not w:
        sys.exit(f"no {kern} samples (fetch {len(f)}, write {len(w)})")
    fetch_b = 2 * 1024 * sum(f) / len(f)
    write_b = 1024 * sum(w) / len(w)
    nblk = int(key.split("_")[1])
    algo = nblk * (4096 + 4)
    entry = {"hbm_bytes_per_launch": round(fetch_b + write_b),
             "fetch_bytes_per_launch": round(fetch_b), "write_bytes_per_launch": round(write_b),
             "algorithmic_bytes_per_launch": algo,
             "traffic_over_algorithmic": round((fetch_b + write_b) / algo, 4),
             "launches_sampled": [len(f), len(w)],
             "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 half-count) + WRITE_SIZE(KiB)*1024",
             "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes ({prefix})"}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        d = {}
    d[key] = entry
    with open(path, "w") as fh:
        json.dump(d, fh, indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
