#!/usr/bin/env python3
"""Host-side layer rates against the compiled reference (oracle/_ref), printed
as one JSON line each -- the wall-clock comparisons that used to sit inside
the CPU correctness suite (tests/test_table.py, tests/test_log.py), where a
noisy host slice could cut off a ``pytest -x`` run.  No assertions: this is a
measurement, run by hand or on the GPU box.

  merge   CompactionInput's merging iterator (16 x ~2 MiB internal-key SSTs,
          paranoid checks, host CRC path) vs the reference's
          NewMergingIterator over the same images
  log     log::Writer / log::Reader layouts (300 k WriteBatch-sized records)
          on the inline and batched-CPU CRC schedules vs the reference
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from wipdb_amd import sst  # noqa: E402


def run_merge(reps: int) -> dict:
    from tests.test_table import REF_TABLE_SO, RefTable, _sst_stream
    if not os.path.exists(REF_TABLE_SO):
        return {"what": "merge", "skipped": "oracle/_ref/libref_table.so not built"}
    ref_table = RefTable()
    ent, keys, klen, vals, vlen = _sst_stream(16, 16000, 5)
    rc, imgs, _ = sst.build_tables_raw(ent, keys, klen, vals, vlen, bloom_bits=10,
                                       crc_mode=sst.CRC_INLINE, key_format=sst.KEYS_INTERNAL)
    assert rc == sst.OK
    mb = sum(len(i) for i in imgs) / 1e6
    ours = ref = float("inf")
    for _ in range(reps):  # interleaved, best of each
        rc, got, _ = sst.merge_tables(imgs, prefetch_blocks=64, crc_mode=sst.CRC_INLINE)
        assert rc == sst.OK and len(got) == int(ent.sum())
        ours = min(ours, sst.last_call_seconds)
        ref = min(ref, ref_table.merge_seconds(imgs, reps=1))
    return {"what": "merge (CompactionInput vs reference NewMergingIterator)", "MB": round(mb, 1),
            "ours_MBps": round(mb / ours), "reference_MBps": round(mb / ref),
            "ratio": round(ref / ours, 2)}


def run_log(reps: int) -> list:
    from tests.test_log import REF_SO, RefLog
    if not os.path.exists(REF_SO):
        return [{"what": "log", "skipped": "oracle/_ref/libref_table.so not built"}]
    ref_log = RefLog()
    rng = np.random.default_rng(2)
    lens = rng.integers(100, 400, size=300_000)
    blob = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)])
    recs = [blob[offs[i]:offs[i + 1]] for i in range(lens.size)]
    out = []
    for name, mode in (("inline", sst.CRC_INLINE), ("batch_cpu", sst.CRC_BATCH_CPU)):
        tw = tr = float("inf")
        for _ in range(reps):
            img = sst.log_write(recs, log_number=9, crc_mode=mode)
            tw = min(tw, sst.last_call_seconds)
            got = sst.log_read([img], mode)
            tr = min(tr, sst.last_call_seconds)
            assert len(got[0][0]) == len(recs) and not got[0][1]
        rw, rr = ref_log.seconds(recs, img)
        mb = len(img) / 1e6
        out.append({"what": f"log ({name} CRC schedule vs reference Writer/Reader)",
                    "MB": round(mb, 1), "write_MBps": round(mb / tw),
                    "reference_write_MBps": round(mb / rw), "recover_MBps": round(mb / tr),
                    "reference_recover_MBps": round(mb / rr)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="merge,log")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for w in a.what.split(","):
        if w == "merge":
            print(json.dumps(run_merge(a.reps)), flush=True)
        elif w == "log":
            for r in run_log(a.reps):
                print(json.dumps(r), flush=True)
        else:
            raise SystemExit(f"unknown {w}")


if __name__ == "__main__":
    main()
