"""Diagnostic: the read-stream kernel (readstream_kernel, a wave per block)
over the same 4 GiB as the headline, cut into blocks of 4, 8 or 16 KiB --
with a WIPDB_RS_UNROLL build, how HBM throughput depends on the loads a
wave keeps in flight (1 KiB each).

  WIPDB_HCRC_LIB=build/variants/rs8/libhip_crc32c_batch.so python scripts/stream_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wipdb_amd.crc32c import Engine  # noqa: E402


def main():
    d = torch.device("cuda", 0)
    eng = Engine(0)
    total = 4 << 30
    data = torch.empty(total, dtype=torch.uint8, device=d)
    st = torch.cuda.current_stream(d)
    eng.fill_splitmix64_device(data, 5, stream=st.cuda_stream)
    res = {}
    for blk in [int(x) for x in os.environ.get("PROBE_BLOCKS", "4096,8192,16384").split(",")]:
        n = total // blk
        out = torch.empty(n, dtype=torch.int32, device=d)
        for _ in range(3):
            eng.readstream_device(data, blk, blk, n, out, stream=st.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(20):
            eng.readstream_device(data, blk, blk, n, out, stream=st.cuda_stream)
        b.record(st)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        res[blk] = {"ms": round(ms, 4), "TBps": round(total / ms / 1e9, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
