#!/bin/bash
# GPU box: slot-pattern parity check, GPU tests, headline bench and the
# compute-only diagnostic of the in-tree build.  Stops at the first fault.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # log timeout cmd...
  local log=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "=== $log rc=$rc"; grep -v amdgpu.ids "gpurun_out/$log" | tail -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $log (rc=$rc)"; exit $rc; fi
  return $rc
}
step q_check.log 240 python scripts/variant_check.py || exit 1
step q_tests.log 600 python -m pytest tests -m gpu -x -q || exit 1
step q_bench.log 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --readstream
step q_s0.log 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --stride 0
step q_strided.log 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --mode strided
echo ALLDONE
