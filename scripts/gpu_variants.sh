#!/bin/bash
# GPU box: for each variant in $VARIANTS (build/variants/NAME), run the
# slot-pattern parity check, then the headline bench and the compute-only
# diagnostic (stride 0).  Stops at the first faulting/aborting step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # log timeout cmd...
  local log=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "=== $log rc=$rc"; tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $log (rc=$rc)"; exit $rc; fi
  return $rc
}
for v in $VARIANTS; do
  export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so
  case $v in
    lo*) ;;  # diagnostic builds that skip the CRC work: no parity check
    *) step "v_${v}_check.log" 240 python scripts/variant_check.py || continue ;;
  esac
  step "v_${v}_bench.log" 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
  step "v_${v}_s0.log" 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --stride 0
  [ -n "$STRIDED" ] && step "v_${v}_strided.log" 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --mode strided
done
echo ALLDONE
