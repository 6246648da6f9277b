#!/bin/bash
# GPU box: effective shader clock (GRBM_GUI_ACTIVE / 8 / kernel time) of the
# CRC kernel for each variant in $VARIANTS ("default" = in-tree build), in
# the headline (stride 4096) and compute-only (stride 0) modes, plus the
# read-stream kernel.  One PMC pass + one kernel-trace pass per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; fi
  for stride in 4096 0; do
    d=gpurun_out/clk_${v}_$stride
    timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE -d ${d}_pmc -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --readstream --stride $stride > ${d}_pmc.log 2>&1 || exit $?
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${d}_trace -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --readstream --stride $stride > ${d}_trace.log 2>&1 || exit $?
    python3 - "$d" "$v" "$stride" <<'PY'
import csv, glob, collections, sys
d, v, stride = sys.argv[1:4]
g = collections.defaultdict(list)
for p in glob.glob(d + "_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        g[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
t = {}
for p in glob.glob(d + "_trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        t[r["Name"].split("(")[0]] = float(r["AverageNs"])
for k, vals in g.items():
    if ("crc32c" in k or "readstream" in k) and k in t:
        cyc = sum(vals) / len(vals) / 8
        print(f"{v:8s} stride {stride:5s} {k.split('::')[-1]:22s} cycles/XCD {cyc:10.0f} avg {t[k]/1e3:7.1f} us clock {cyc / t[k]:.3f} GHz")
PY
  done
done
