#!/bin/bash
# GPU box: headline kernel time under the diagnostic block orders (which
# block each descriptor names), for each variant in $VARIANTS.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so
  for o in natural group cu; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --order $o > gpurun_out/o_${v}_$o.log 2>&1 || { echo "ABORT $v $o"; tail -5 gpurun_out/o_${v}_$o.log; exit 3; }
    echo "$v $o $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/o_${v}_$o.log)"
  done
done
echo ALLDONE
