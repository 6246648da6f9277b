"""Why do back-to-back headline launches run slower than gapped ones?
(BENCH_r05's precondition.last10_kernel_ms 0.627 ms,
launches separated by torch compare kernels, against 0.666 ms for the timed
back-to-back launches.)

Runs the headline step (1 M x 4 KiB, spans entry point) in several regimes
on one context and prints one JSON line:

  warm        >= --warm-ms of back-to-back launches, one event pair
  idle_<x>    after a host idle of x ms: 40 launches with an event pair
              around each (per-launch times by position) and then 20 with
              one pair around them all (the bench's timed form)
  gapped      40 launches, each followed by the precondition's compare and
              sum kernels (per-launch event pairs, as bench.py's precondition)
  clocks      a host thread samples torch.cuda.clock_rate / power_draw
              (amdsmi) every ~2 ms; mean MHz / W per phase

  python scripts/gap_probe.py [--warm-ms 300] [--idles 0,0.2,2,10,50]
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wipdb_amd.crc32c import Engine  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--warm-ms", type=float, default=300.0)
    p.add_argument("--idles", default="0,0.2,2,10,50")
    p.add_argument("--blocks", type=int, default=1 << 20)
    p.add_argument("--no-clock", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    n = a.blocks
    st = torch.cuda.current_stream(dev)
    data = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    eng.fill_splitmix64_device(data, 0x4B10C5, stream=st.cuda_stream)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ref = torch.empty_like(out)

    def step(dst=out):
        eng.batch_device(data, offs, lens, None, dst, stream=st.cuda_stream)

    step(ref)
    mism = torch.zeros((), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)

    samples = []  # (t, phase, MHz, W)
    phase = ["setup"]
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            try:
                mhz = torch.cuda.clock_rate(dev)
                w = torch.cuda.power_draw(dev)
            except Exception as e:  # amdsmi missing or refused: no clocks
                samples.append((time.perf_counter(), "error", str(e), 0))
                return
            samples.append((time.perf_counter(), phase[0], mhz, w))
            time.sleep(0.002)

    th = None
    if not a.no_clock:
        th = threading.Thread(target=sampler, daemon=True)
        th.start()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    res = {"blocks": n}
    # warm: back-to-back, one pair
    phase[0] = "warm"
    e0, e1 = ev(), ev()
    e0.record(st)
    step()
    e1.record(st)
    torch.cuda.synchronize(dev)
    k = max(20, int(a.warm_ms / max(e0.elapsed_time(e1), 1e-3)))
    e0.record(st)
    for _ in range(k):
        step()
    e1.record(st)
    torch.cuda.synchronize(dev)
    res["warm"] = {"launches": k, "ms_per_launch": round(e0.elapsed_time(e1) / k, 4)}

    for idle in [float(x) for x in a.idles.split(",")]:
        phase[0] = f"idle_{idle}"
        # keep the card busy right up to the idle, as the warm phase did
        for _ in range(20):
            step()
        torch.cuda.synchronize(dev)
        if idle > 0:
            time.sleep(idle / 1e3)
        phase[0] = f"after_idle_{idle}"
        pairs = [(ev(), ev()) for _ in range(40)]
        for s, e in pairs:
            s.record(st)
            step()
            e.record(st)
        b0, b1 = ev(), ev()
        b0.record(st)
        for _ in range(20):
            step()
        b1.record(st)
        torch.cuda.synchronize(dev)
        ms = [s.elapsed_time(e) for s, e in pairs]
        res[f"idle_{idle}"] = {
            "per_launch[0:5]": round(sum(ms[:5]) / 5, 4),
            "per_launch[5:20]": round(sum(ms[5:20]) / 15, 4),
            "per_launch[20:40]": round(sum(ms[20:40]) / 20, 4),
            "then_20_bracketed": round(b0.elapsed_time(b1) / 20, 4),
        }
        # the same 20 bracketed launches right after the idle, no per-launch pairs
        for _ in range(20):
            step()
        torch.cuda.synchronize(dev)
        if idle > 0:
            time.sleep(idle / 1e3)
        b0, b1 = ev(), ev()
        b0.record(st)
        for _ in range(20):
            step()
        b1.record(st)
        torch.cuda.synchronize(dev)
        res[f"idle_{idle}"]["bracketed_20_right_after"] = round(b0.elapsed_time(b1) / 20, 4)

    # gapped: the precondition's form
    phase[0] = "gapped"
    scratch = torch.empty_like(out)
    pairs = [(ev(), ev()) for _ in range(60)]
    for s, e in pairs:
        s.record(st)
        step(scratch)
        e.record(st)
        mism += (scratch != ref).sum()
    torch.cuda.synchronize(dev)
    ms = [s.elapsed_time(e) for s, e in pairs]
    res["gapped"] = {"per_launch[0:20]": round(sum(ms[:20]) / 20, 4),
                     "per_launch[20:60]": round(sum(ms[20:]) / 40, 4)}
    # gapped, then immediately back-to-back with no host sync in between
    phase[0] = "gapped_then_b2b"
    b0, b1 = ev(), ev()
    b0.record(st)
    for _ in range(20):
        step()
    b1.record(st)
    torch.cuda.synchronize(dev)
    res["gapped_then_b2b_20"] = round(b0.elapsed_time(b1) / 20, 4)
    res["identical_outputs"] = int(mism.item()) == 0 and bool((out == ref).all().item())

    stop.set()
    if th is not None:
        th.join(timeout=1)
    if samples and samples[0][1] == "error":
        res["clocks"] = {"error": samples[0][2]}
    elif samples:
        agg = {}
        for _, ph, mhz, w in samples:
            d = agg.setdefault(ph, [0, 0.0, 0.0])
            d[0] += 1
            d[1] += mhz
            d[2] += w
        res["clocks"] = {ph: {"samples": c, "MHz": round(m / c, 1), "W": round(w / c, 1)}
                         for ph, (c, m, w) in agg.items()}
    res["lib"] = os.environ.get("WIPDB_HCRC_LIB", "tree")
    print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
