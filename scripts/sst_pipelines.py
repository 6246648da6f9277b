"""Which pipeline serves WipDB's own batches?  The
8Binsert SST stream (BASELINE configs[4]: per SST ~500 data blocks of
4097..4225 B, an index block, a filter block and a metaindex block, each
followed by its 4-byte trailer, kv/src/table/table_builder.cc:183-202) and a
WAL stream (kv/src/db/log_writer.cc: 7-byte headers, records of 16 B keys +
100 B values, 32 KiB blocks), device-resident, through the default entry
point, HCRC_PACKED, and HCRC_PACKED with run_ps forced (WIPDB_PS_ONLY set in
a child process): GiB/s of the same batch, one SST (~2 MiB) and 1024 SSTs
(~2 GiB), every result compared with the default pipeline's.

  python scripts/sst_pipelines.py
"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))


def wal_layout(rng, nbytes):
    """Physical WAL records as log::Writer::EmitPhysicalRecord lays them out:
    each CRC span is type byte + payload (log_writer.cc:108-130), records of
    one 8-byte-key Put batch (~130 B), 7-byte headers, 32 KiB blocks."""
    offs, lens, cur = [], [], 0
    while cur < nbytes:
        n = int(rng.integers(110, 160))
        left = 32768 - cur % 32768
        if left < 7 + 1:
            cur += left
            continue
        n = min(n, left - 7)
        offs.append(cur + 6)   # the CRC covers the type byte (header byte 6) + payload
        lens.append(n + 1)
        cur += 7 + n
    return np.array(offs, np.uint64), np.array(lens, np.uint32)


def measure(mode):
    import torch
    from bench_extra import sst_layout, time_kernel
    from wipdb_amd import Engine
    d = torch.device("cuda", 0)
    st = torch.cuda.current_stream(d)
    rng = np.random.default_rng(11)
    res = {}
    with Engine(0) as eng:
        shapes = {}
        o, l, n = sst_layout(rng, 1)
        shapes["sst_1"] = (o, l, n)
        o, l, n = sst_layout(rng, 1024)
        shapes["sst_1024"] = (o, l, n)
        o, l = wal_layout(rng, 2 << 30)
        shapes["wal_2GiB"] = (o, l, int(o[-1]) + int(l[-1]) + 8)
        for name, (o, l, n) in shapes.items():
            buf = torch.empty((n + 64 + 7) // 8 * 8, dtype=torch.uint8, device=d)
            eng.fill_splitmix64_device(buf, 5, stream=st.cuda_stream)
            do = torch.from_numpy(o.astype(np.int64)).to(d)
            dl = torch.from_numpy(l.astype(np.int32)).to(d)
            out = torch.empty(o.size, dtype=torch.int32, device=d)
            ref = eng.batch_device(buf, do, dl, stream=st.cuda_stream)
            packed = mode != "default"
            t = time_kernel(lambda: eng.batch_device(buf, do, dl, None, out, stream=st.cuda_stream,
                                                     packed=packed), st, 10)
            res[name] = {"spans": int(o.size), "bytes": int(l.sum()),
                         "GiBps": round(float(l.sum()) / t / 2**30, 1), "us": round(t * 1e6, 1),
                         "same_as_default": bool((out == ref).all())}
            del buf, do, dl, out, ref
    return res


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        print("RES " + json.dumps(measure(sys.argv[2])), flush=True)
        return
    out = {}
    for mode in ("default", "packed", "ps_only"):
        env = dict(os.environ, PYTHONPATH=REPO, WIPDB_PS_MIN_SPANS="0")
        if mode == "ps_only":
            env["WIPDB_PS_ONLY"] = "1"
        r = subprocess.run([sys.executable, __file__, "--child", mode], env=env, cwd=REPO,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-2000:])
            sys.exit(r.returncode)
        out[mode] = json.loads(r.stdout.split("RES ", 1)[1].splitlines()[0])
    print(json.dumps({"note": "WIPDB_PS_MIN_SPANS=0: packed batches of any count take the "
                              "packed kernel (the product's floor is 32 Ki spans)", **out}))


if __name__ == "__main__":
    main()
