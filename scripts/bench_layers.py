#!/usr/bin/env python3
"""Rates of the widened rows per CRC schedule, one JSON
line per workload.  Times are the native C-ABI call alone (sst.last_call_seconds).

  compaction  T SSTs of the 8Binsert shape (16-byte key + 8-byte tag, 100-byte
              printable value, 4 KiB blocks, bloom 10) built and finished
              together: table MB/s for kInline (the reference's schedule:
              CRC per block on the host), kBatchCpu, kBatchGpu.
  verify      the same tables through the batched Table::Open + verified
              iteration: MB/s per schedule (and, on the MI355X, with the
              images in pinned memory: zero-copy).
  merge       the compaction input path (MakeInputIteratorKV): the merged
              entries of the same tables read with paranoid checks, data
              blocks checked 64 per input per CRC batch: MB/s per schedule.
  wal         a log of R WriteBatch-sized records (100-400 B): AddRecord
              layout + CRCs (write) and the recovery read, MB/s per schedule.

    python scripts/bench_layers.py [--tables 64] [--records 1000000] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from wipdb_amd import sst  # noqa: E402

MODES = {"inline": sst.CRC_INLINE, "batch_cpu": sst.CRC_BATCH_CPU, "batch_gpu": sst.CRC_BATCH_GPU}


def sst_stream(tables: int, per_table: int, seed: int):
    rng = np.random.default_rng(seed)
    n = tables * per_table
    user = np.sort(rng.choice(2**62, size=n, replace=False).astype(np.uint64))
    keys = bytearray()
    for i, u in enumerate(user.tolist()):
        keys += b"%016x" % u + ((i + 1) << 8 | 1).to_bytes(8, "little")
    vals = rng.integers(32, 127, size=n * 100, dtype=np.uint8).tobytes()
    return (np.full(tables, per_table, np.uint64), bytes(keys), np.full(n, 24, np.uint32), vals,
            np.full(n, 100, np.uint32))


def best(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        out = fn()
        ts.append(sst.last_call_seconds)
    return min(ts), out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tables", type=int, default=64)
    p.add_argument("--per-table", type=int, default=16000)  # ~2 MiB SSTs
    p.add_argument("--records", type=int, default=1_000_000)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--modes", default="inline,batch_cpu,batch_gpu")
    a = p.parse_args()
    modes = [m for m in a.modes.split(",") if m]
    if "batch_gpu" in modes:
        import torch  # noqa: F401  (one HIP runtime in the process)

    t0 = time.time()
    ent, keys, klen, vals, vlen = sst_stream(a.tables, a.per_table, 1)
    res = {"workload": "compaction", "tables": a.tables, "entries": int(ent.sum()),
           "gen_s": round(time.time() - t0, 1)}
    imgs_ref = None
    for m in modes:
        t, (rc, imgs, batched) = best(lambda: sst.build_tables_raw(
            ent, keys, klen, vals, vlen, bloom_bits=10, crc_mode=MODES[m]), a.reps)
        assert rc == sst.OK
        if imgs_ref is None:
            imgs_ref = imgs
        assert imgs == imgs_ref, f"{m}: table bytes differ between CRC schedules"
        mb = sum(len(i) for i in imgs) / 1e6
        res[m] = {"s": round(t, 4), "MB_per_s": round(mb / t, 1), "batched_blocks": batched}
    res["table_MB"] = round(sum(len(i) for i in imgs_ref) / 1e6, 1)
    print(json.dumps(res), flush=True)

    res = {"workload": "verify", "tables": len(imgs_ref)}
    for m in modes:
        t, (rc, codes) = best(lambda: sst.verify_tables(imgs_ref, 10, MODES[m]), a.reps)
        assert rc == sst.OK
        res[m] = {"s": round(t, 4), "MB_per_s": round(sum(len(i) for i in imgs_ref) / 1e6 / t, 1)}
    if "batch_gpu" in modes:
        # the images in pinned memory (as a store keeps SST pages it reads):
        # the block CRC batch reads them zero-copy
        with sst.PinnedImages(imgs_ref) as pin:
            t, (rc, codes) = best(lambda: sst.verify_tables_at(pin.addrs, pin.sizes, 10,
                                                               sst.CRC_BATCH_GPU), a.reps)
            assert rc == sst.OK
            res["batch_gpu_pinned_images"] = {"s": round(t, 4),
                                              "MB_per_s": round(pin.nbytes / 1e6 / t, 1)}
    print(json.dumps(res), flush=True)

    res = {"workload": "merge", "tables": len(imgs_ref)}
    want = None
    for m in modes:
        t, (rc, ents, batches) = best(lambda: sst.merge_tables(
            imgs_ref, key_format=sst.KEYS_BYTEWISE, prefetch_blocks=64, crc_mode=MODES[m]), a.reps)
        assert rc == sst.OK
        if want is None:
            want = ents
        assert ents == want, f"{m}: merged entries differ between CRC schedules"
        res[m] = {"s": round(t, 4), "MB_per_s": round(sum(len(i) for i in imgs_ref) / 1e6 / t, 1),
                  "crc_batches": batches}
    res["entries"] = len(want)
    print(json.dumps(res), flush=True)
    del want

    rng = np.random.default_rng(2)
    lens = rng.integers(100, 400, size=a.records)
    blob = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)])
    recs = [blob[offs[i]:offs[i + 1]] for i in range(a.records)]
    res = {"workload": "wal", "records": a.records, "payload_MB": round(len(blob) / 1e6, 1)}
    img_ref = None
    for m in modes:
        t, img = best(lambda: sst.log_write(recs, crc_mode=MODES[m]), a.reps)
        if img_ref is None:
            img_ref = img
        assert img == img_ref
        tr, out = best(lambda: sst.log_read([img_ref], MODES[m]), a.reps)
        assert len(out[0][0]) == a.records and not out[0][1]
        res[m] = {"write_s": round(t, 4), "write_MB_per_s": round(len(img) / 1e6 / t, 1),
                  "recover_s": round(tr, 4), "recover_MB_per_s": round(len(img) / 1e6 / tr, 1)}
    res["log_MB"] = round(len(img_ref) / 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
