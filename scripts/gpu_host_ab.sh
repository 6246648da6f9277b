#!/bin/bash
# GPU box: where the timed region's host time goes (bench.py's
# timed_region_host_ms), with and without Python's GC in the timed region.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in --keep-gc ""; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-ceiling $v > gpurun_out/host_ab.log 2>&1 || exit $?
    echo "round $r $v: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*\|"timed_region_host_ms": {[^}]*}' gpurun_out/host_ab.log | tr '\n' ' ')"
  done
done
