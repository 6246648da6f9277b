#!/bin/bash
# Runs on the GPU box (via gpurun): smoke, short bench, GPU tests, rocprof.
# Stops at the first GPU step that faults/aborts/times out (rc not in {0,1}).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-"smoke bench tests prof"}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 --readstream ;;
    bench_strided) run bench_strided 300 python bench.py --steps 10 --warmup 2 --mode strided --no-cpu-baseline --readstream ;;
    tests) run tests 900 python -m pytest tests -m gpu -x -q ;;
    testsall) run testsall 900 python -m pytest tests -m gpu -q ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc_fetch) run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmc_write) run pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    diag) run diag_s0 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --stride 0 &&
          run diag_s0_strided 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --stride 0 --mode strided &&
          run diag_small 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --blocks 16384 ;;
    pmc_sq) run pmc_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_sq2) run pmc_sq2 400 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s" ;;
  esac
done
echo ALLDONE
