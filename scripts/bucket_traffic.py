#!/usr/bin/env python3
"""HBM traffic per config-3 bucket (BASELINE config 3: Zipf sizes over
512 B .. 64 KiB, SST-packed at unaligned offsets, device-resident): each
bucket's batch is launched LAUNCHES times through the default
hcrc_batch_async entry point (no flags), in bucket order, so a rocprofv3
--pmc pass over this script can be split per bucket.

  python scripts/bucket_traffic.py run            # the launches (under rocprofv3)
  python scripts/bucket_traffic.py summarize FETCH_DIR WRITE_DIR > out.json
  python scripts/bucket_traffic.py summarize_sq SQ_DIR > out.json  # SQ_* pass

Algorithmic bytes per launch: the spans' bytes read + 4 bytes
written per span; the descriptor columns (8 + 4 bytes per span) are listed
beside it.  Corrections per MI355X_MICROARCH.md (HBM section): FETCH_SIZE
and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a
16-B/lane streaming read (the segment / piece DMAs), so it is doubled."""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

BUCKETS = [512, 1024, 2048, 4096, 8192, 16384, 32768, 65536, "mix"]
LAUNCHES = 3
KERNEL = "crc32c_lds_spans_kernel"


def run():
    import numpy as np
    import torch

    from bench_extra import BUCKETS as B, dev, zipf_spans
    from wipdb_amd import Engine

    d = torch.device("cuda", 0)
    st = torch.cuda.current_stream(d)
    rng = np.random.default_rng(42)
    nbytes = 2 << 30
    meta = []
    with Engine(0) as eng:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=d)
        eng.fill_splitmix64_device(buf, 3, stream=st.cuda_stream)
        for b in BUCKETS:
            offs, lens, _ = zipf_spans(rng, nbytes, B if b == "mix" else [b])
            do, dl = dev(offs, d), dev(lens, d)
            out = torch.empty(offs.size, dtype=torch.int32, device=d)
            torch.cuda.synchronize()
            for _ in range(LAUNCHES):
                eng.batch_device(buf, do, dl, None, out, stream=st.cuda_stream)
            torch.cuda.synchronize()
            meta.append({"bucket": b, "spans": int(offs.size), "span_bytes": int(lens.sum())})
            del do, dl, out
    with open(os.path.join(REPO, "gpurun_out", "bucket_traffic_meta.json"), "w") as f:
        json.dump(meta, f)
    print(json.dumps(meta))


def counters_of(d):
    names = set()
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            names.update(r["Counter_Name"] for r in csv.DictReader(f) if KERNEL in r["Kernel_Name"])
    return sorted(names)


def summarize_sq(sdir):
    """Per-bucket SQ counters per span and per wave (mean of the launches)."""
    with open(os.path.join(REPO, "gpurun_out", "bucket_traffic_meta.json")) as f:
        meta = json.load(f)
    need = LAUNCHES * len(meta)
    cols = {}
    for c in counters_of(sdir):
        v = per_dispatch(sdir, c)
        if len(v) != need:
            sys.exit(f"{c}: expected {need} dispatches, got {len(v)}")
        cols[c] = v
    out = []
    for k, m in enumerate(meta):
        row = dict(m)
        for c, v in cols.items():
            row[c] = round(sum(v[k * LAUNCHES:(k + 1) * LAUNCHES]) / LAUNCHES)
        if "SQ_WAVE_CYCLES" in row and row.get("SQ_WAVES"):
            row["wave_cycles_per_wave"] = round(row["SQ_WAVE_CYCLES"] / row["SQ_WAVES"])
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_INST_ANY"):
            if c in row:
                row[c + "_per_span"] = round(row[c] / m["spans"], 2)
        out.append(row)
    print(json.dumps({"source": "rocprofv3 --pmc SQ_* (one pass), "
                                f"mean of {LAUNCHES} launches per bucket, default entry point",
                      "buckets": out}, indent=1))


def per_dispatch(d, counter):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]:
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    acc = {}
    for i, v in rows:  # (a counter may be reported per XCD / instance: summed)
        acc[i] = acc.get(i, 0.0) + v
    return [acc[i] for i in sorted(acc)]


def summarize(fdir, wdir):
    with open(os.path.join(REPO, "gpurun_out", "bucket_traffic_meta.json")) as f:
        meta = json.load(f)
    fv, wv = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    need = LAUNCHES * len(meta)
    if len(fv) != need or len(wv) != need:
        sys.exit(f"expected {need} dispatches, got fetch {len(fv)} write {len(wv)}")
    out = []
    for k, m in enumerate(meta):
        fs = fv[k * LAUNCHES:(k + 1) * LAUNCHES]
        ws = wv[k * LAUNCHES:(k + 1) * LAUNCHES]
        fetch = 2 * 1024 * sum(fs) / len(fs)
        write = 1024 * sum(ws) / len(ws)
        algo = m["span_bytes"] + 4 * m["spans"]
        desc = 12 * m["spans"]
        out.append({**m, "fetch_bytes": round(fetch), "write_bytes": round(write),
                    "algorithmic_bytes": algo, "descriptor_bytes": desc,
                    "traffic_over_algorithmic": round((fetch + write) / algo, 4),
                    "traffic_over_algorithmic_plus_descriptors": round((fetch + write) / (algo + desc), 4)})
    print(json.dumps({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                                "FETCH_SIZE(KiB)*1024*2 (gfx950 half count) + WRITE_SIZE(KiB)*1024; "
                                f"mean of {LAUNCHES} launches per bucket, default entry point",
                      "buckets": out}, indent=1))


if __name__ == "__main__":
    if sys.argv[1:2] == ["run"]:
        run()
    elif sys.argv[1:2] == ["summarize"]:
        summarize(sys.argv[2], sys.argv[3])
    elif sys.argv[1:2] == ["summarize_sq"]:
        summarize_sq(sys.argv[2])
    else:
        sys.exit(__doc__)
