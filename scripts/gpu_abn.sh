#!/bin/bash
# GPU box: same-session comparison of several builds of the library --
# headline kernel ms and the bench_extra shapes, the builds alternating
# within each round.  "tree" = the in-tree library, anything else a path to
# another build (loaded through WIPDB_HCRC_LIB).
#   bash scripts/gpu_abn.sh ROUNDS WHAT tree build/ab/lib_head.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=$1
WHAT=$2
shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    tag=$(basename "$v" .so)
    if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/ab_bench.log 2>&1 || exit $?
    b=$(grep -o '"kernel_avg_ms": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/ab_bench.log | tr '\n' ' ')
    e=""
    if [ -n "$WHAT" ] && [ "$WHAT" != none ]; then
      timeout -k 10 300 python scripts/bench_extra.py --no-cpu --what "$WHAT" > gpurun_out/ab_extra_${r}_${tag}.log 2>&1 || exit $?
      e=$(grep -o '"GiBps": [0-9.]*\|"GiBps_end_to_end": [0-9.]*' gpurun_out/ab_extra_${r}_${tag}.log | tr '\n' ' ')
    fi
    echo "round $r $v: headline $b | $e"
  done
done
