#!/bin/bash
# GPU box: same-session A/B of library builds on the headline (bench.py, the
# driver's --steps 20 --warmup 5, no extras) and the launch-gap probe
# (scripts/gap_probe.py), builds alternating within each round.
#   bash scripts/gpu_gap_ab.sh ROUNDS PREFIX tree build/ab/lib_r04.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=$1
P=$2
shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    tag=$(basename "$v" .so)
    if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
    timeout -k 10 180 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > gpurun_out/${P}_bench_${r}_${tag}.log 2>&1 || exit $?
    b=$(grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*\|"last10_kernel_ms": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/${P}_bench_${r}_${tag}.log | tr '\n' ' ')
    echo "round $r $v: bench $b"
    timeout -k 10 180 python scripts/gap_probe.py > gpurun_out/${P}_gap_${r}_${tag}.log 2>&1 || exit $?
    tail -1 gpurun_out/${P}_gap_${r}_${tag}.log
  done
done
