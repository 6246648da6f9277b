#!/usr/bin/env python3
"""HBM traffic per launch of the current tree's kernels on the shapes the
bench line reports: the headline (1 M aligned 4 KiB
blocks, spans kernel), its same-box ceiling (hcrc_dma_ceiling_async),
WriteRawBlock table blocks (default and HCRC_PACKED) and their ReadBlock
verify, and config 3's 512 B / 2 KiB buckets and Zipf mix (default and
HCRC_PACKED).  Every shape is launched LAUNCHES times, and shapes are
separated by an 8-byte fill_splitmix64_kernel launch, so a rocprofv3 --pmc
pass over `run` splits per shape (every dispatch between two separators
counts: the packed path's pre-pass too).

  python scripts/shape_traffic.py run       # the launches (under rocprofv3 --pmc ...)
  python scripts/shape_traffic.py summarize FETCH_DIR WRITE_DIR [OUT_JSON]

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes of a 16-B/lane streaming read, so it is doubled.  Algorithmic bytes
(SURVEY 8d): span bytes read + 4 bytes written per span (verify: + the
4-byte trailer read, 1 byte written); descriptors (12 B per span) are
listed beside it.
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

LAUNCHES = 3
META = os.path.join(REPO, "gpurun_out", "shape_traffic_meta.json")


def run():
    import numpy as np
    import torch

    from bench_configs import table_layout
    from bench_extra import BUCKETS, dev, zipf_spans
    from wipdb_amd import Engine

    d = torch.device("cuda", 0)
    st = torch.cuda.current_stream(d)
    rng = np.random.default_rng(42)
    meta = []
    with Engine(0) as eng:
        sep = torch.empty(8, dtype=torch.uint8, device=d)

        def separator():
            eng.fill_splitmix64_device(sep, 0, stream=st.cuda_stream)

        n = 1 << 20
        blocks = torch.empty(n * 4096, dtype=torch.uint8, device=d)
        eng.fill_splitmix64_device(blocks, 1, stream=st.cuda_stream)
        offs = torch.arange(n, dtype=torch.int64, device=d) * 4096
        lens = torch.full((n,), 4096, dtype=torch.int32, device=d)
        out = torch.empty(n, dtype=torch.int32, device=d)
        tb_offs, tb_lens = table_layout(rng, 2.0)
        tb_size = int(tb_offs[-1]) + int(tb_lens[-1]) + 4
        tb = torch.empty((tb_size + 7) // 8 * 8, dtype=torch.uint8, device=d)
        eng.fill_splitmix64_device(tb, 2, stream=st.cuda_stream)
        tdo, tdl = dev(tb_offs, d), dev(tb_lens, d)
        thl = dev(tb_lens - 1, d)
        tout = torch.empty(tb_offs.size, dtype=torch.int32, device=d)
        tst = torch.empty(tb_offs.size, dtype=torch.uint8, device=d)
        mix = torch.empty(2 << 30, dtype=torch.uint8, device=d)
        eng.fill_splitmix64_device(mix, 3, stream=st.cuda_stream)
        torch.cuda.synchronize()

        def shape(name, fn, spans, span_bytes, algo):
            separator()
            for _ in range(LAUNCHES):
                fn()
            torch.cuda.synchronize()
            meta.append({"shape": name, "spans": int(spans), "span_bytes": int(span_bytes),
                         "algorithmic_bytes": int(algo), "descriptor_bytes": int(12 * spans)})

        shape("headline_4k_spans", lambda: eng.batch_device(blocks, offs, lens, None, out,
                                                            stream=st.cuda_stream),
              n, n * 4096, n * 4100)
        shape("dma_ceiling_4k", lambda: eng.dma_ceiling_device(blocks, 4096, n, out,
                                                               stream=st.cuda_stream),
              n, n * 4096, n * 4100)
        tsum = int(tb_lens.sum())
        shape("table_blocks", lambda: eng.batch_device(tb, tdo, tdl, None, tout,
                                                       stream=st.cuda_stream),
              tb_offs.size, tsum, tsum + 4 * tb_offs.size)
        shape("table_blocks_packed", lambda: eng.batch_device(tb, tdo, tdl, None, tout,
                                                              stream=st.cuda_stream, packed=True),
              tb_offs.size, tsum, tsum + 4 * tb_offs.size)
        shape("table_blocks_verify", lambda: eng.verify_device(tb, tdo, thl, tst,
                                                               stream=st.cuda_stream),
              tb_offs.size, tsum, tsum + 5 * tb_offs.size)
        for b in [512, 2048, "mix"]:
            o, ln, _ = zipf_spans(rng, 2 << 30, BUCKETS if b == "mix" else [b])
            do, dl = dev(o, d), dev(ln, d)
            mo = torch.empty(o.size, dtype=torch.int32, device=d)
            s = int(ln.sum())
            shape(f"config3_{b}", lambda: eng.batch_device(mix, do, dl, None, mo,
                                                           stream=st.cuda_stream),
                  o.size, s, s + 4 * o.size)
            shape(f"config3_{b}_packed", lambda: eng.batch_device(mix, do, dl, None, mo,
                                                                  stream=st.cuda_stream,
                                                                  packed=True),
                  o.size, s, s + 4 * o.size)
            del do, dl, mo
        separator()
        torch.cuda.synchronize()
    os.makedirs(os.path.dirname(META), exist_ok=True)
    with open(META, "w") as f:
        json.dump(meta, f)
    print(json.dumps(meta))


def _per_shape(d, counter, nshapes):
    """[{kernel: [value per dispatch]}] per shape: the dispatches split at
    every fill_splitmix64_kernel; the shapes are the nshapes segments right
    before the last (trailing) separator."""
    per = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter:
                    kk = per.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0])
                    kk[1] += float(r["Counter_Value"])  # (summed over dimensions, if listed so)
    segs = [{}]
    for did in sorted(per):
        k, v = per[did]
        if "fill_splitmix64" in k:
            segs.append({})
            continue
        name = k.split("(")[0].split("<")[0].split("::")[-1]
        segs[-1].setdefault(name, []).append(v)
    assert len(segs) >= nshapes + 1, f"{len(segs)} segments for {nshapes} shapes"
    return segs[-1 - nshapes:-1]


def summarize(fdir, wdir, out_json=None):
    with open(META) as f:
        meta = json.load(f)
    fs = _per_shape(fdir, "FETCH_SIZE", len(meta))
    ws = _per_shape(wdir, "WRITE_SIZE", len(meta))
    res = {}
    for i, m in enumerate(meta):
        f, w = fs[i], ws[i]
        fetch = 2 * 1024 * sum(sum(v) for v in f.values()) / LAUNCHES
        write = 1024 * sum(sum(v) for v in w.values()) / LAUNCHES
        main = max(f, key=lambda k: sum(f[k]))
        fm = 2 * 1024 * sum(f[main]) / LAUNCHES
        wm = 1024 * sum(w.get(main, [0.0])) / LAUNCHES
        res[m["shape"]] = {
            "hbm_bytes_per_launch": round(fetch + write),
            "fetch_bytes": round(fetch), "write_bytes": round(write),
            "algorithmic_bytes": m["algorithmic_bytes"],
            "traffic_over_algorithmic": round((fetch + write) / m["algorithmic_bytes"], 4),
            "with_descriptors_over_algorithmic": round(
                (fetch + write) / (m["algorithmic_bytes"] + m["descriptor_bytes"]), 4),
            "main_kernel": main, "main_kernel_bytes": round(fm + wm),
            "kernels": {k: len(v) // LAUNCHES for k, v in f.items()},
            "spans": m["spans"], "span_bytes": m["span_bytes"]}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes over "
                     "scripts/shape_traffic.py run",
           "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 half-count) + WRITE_SIZE(KiB)*1024",
           "launches_per_shape": LAUNCHES, "shapes": res}
    txt = json.dumps(doc, indent=1)
    if out_json:
        with open(out_json, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(*sys.argv[2:5])
