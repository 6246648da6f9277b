#!/bin/bash
# GPU box: same-session A/B of library builds on the headline line (driver
# arguments, no extras, no CPU baseline), builds alternating within rounds.
#   bash scripts/gpu_headline_ab.sh ROUNDS tree build/ab/lib_x.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=$1
shift
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
    timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/hab.log 2>&1 || exit $?
    echo "round $r $v: $(grep -o '"value": [0-9.]*\|"kernel_avg_ms": [0-9.]*\|"frac_of_ceiling": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/hab.log | tr '\n' ' ')"
  done
done
