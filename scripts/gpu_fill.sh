#!/bin/bash
# GPU box: headline kernel time and clock on random vs zero block contents
# (is the kernel power/clock-limited?), for the in-tree build and loadonly.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; fi
  for f in splitmix zero; do
    d=gpurun_out/fill_${v}_$f
    timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE -d ${d}_pmc -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --fill $f > ${d}_pmc.log 2>&1 || exit $?
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --fill $f > ${d}.log 2>&1 || exit $?
    ms=$(grep -o '"kernel_avg_ms": [0-9.]*' ${d}.log | grep -o '[0-9.]*$')
    cyc=$(python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for p in glob.glob('${d}_pmc/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(p)) if 'crc32c_spans' in r['Kernel_Name']]
print(sum(v)/len(v)/8 if v else 0)")
    echo "$v $f kernel_ms $ms cycles/XCD $cyc GHz $(python3 -c "print(round($cyc/($ms*1e6),3))")"
  done
done
echo ALLDONE
