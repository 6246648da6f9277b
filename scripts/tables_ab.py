"""Same-session A/B of library builds on the table-block shapes of the bench
line: WriteRawBlock spans and their ReadBlock verify, device-resident
(scripts/bench_configs.run_tables: the line's own workload, timing and
parity sample against bench.py's checker), one child process per build and
round, builds alternating.

  python scripts/tables_ab.py ROUNDS tree build/ab/lib_x.so ...
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    from bench import _ref_batch
    from scripts.bench_configs import run_tables
    from wipdb_amd import Engine
    d = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(d)
    rng = np.random.default_rng(0xC0F1)
    with Engine(0) as eng:
        tb, vt = run_tables(eng, d, stream, _ref_batch()[0], rng)
    return {"table_blocks": tb["GiBps"], "packed": tb["packed"]["GiBps"],
            "verified": vt["GiBps"], "parity_mismatches": tb["parity"]["mismatches"],
            "verify_status_mismatches": vt["status_mismatches"],
            "latency_2MiB_p50_us": tb["latency_2MiB_device"]["p50_us"]}


def main():
    if sys.argv[1] == "--child":
        print("RES " + json.dumps(child()), flush=True)
        return
    rounds = int(sys.argv[1])
    for r in range(rounds):
        for v in sys.argv[2:]:
            env = dict(os.environ, PYTHONPATH=REPO)
            if v == "tree":
                env.pop("WIPDB_HCRC_LIB", None)
            else:
                env["WIPDB_HCRC_LIB"] = os.path.join(REPO, v)
            p = subprocess.run([sys.executable, __file__, "--child"], env=env, cwd=REPO,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            res = json.loads(p.stdout.split("RES ", 1)[1].splitlines()[0])
            print(json.dumps({"round": r, "lib": v, **res}), flush=True)


if __name__ == "__main__":
    main()
