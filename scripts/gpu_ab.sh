#!/bin/bash
# GPU box: same-session A/B of the in-tree library against another build
# (WIPDB_HCRC_LIB): headline kernel ms and the table-block / verify shapes,
# alternating builds for ROUNDS rounds.
#   bash scripts/gpu_ab.sh build/ab/lib_head.so [ROUNDS] [bench_extra --what list]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=$1
ROUNDS=${2:-2}
WHAT=${3:-tblocks,verify}
for r in $(seq 1 "$ROUNDS"); do
  for v in new alt; do
    if [ $v = alt ]; then export WIPDB_HCRC_LIB=$PWD/$ALT; else unset WIPDB_HCRC_LIB; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/ab_bench.log 2>&1 || exit $?
    b=$(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/ab_bench.log)
    timeout -k 10 200 python scripts/bench_extra.py --what "$WHAT" > gpurun_out/ab_extra.log 2>&1 || exit $?
    e=$(grep -o '"ms": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/ab_extra.log | tr '\n' ' ')
    echo "round $r $v: headline $b | $e"
  done
done
