#!/bin/bash
# GPU box: the bench line's host overhead (ms_per_step - kernel_avg_ms) under
# HIP runtime wait settings, alternating (driver arguments, no extras).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in default 50 1000 100000; do
    if [ "$v" = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$v; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-ceiling > gpurun_out/sync_ab.log 2>&1 || exit $?
    echo "round $r wait=$v: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*' gpurun_out/sync_ab.log | tr '\n' ' ')"
  done
done
