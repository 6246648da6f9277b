#!/bin/bash
# GPU box: one call's worth of checks and measurements, each step under its
# own time limit, stopping at the first step that faults / aborts / times out.
#   STEPS="probe tests bench extra ab" PREFIX=r03a bash scripts/gpu_round.sh
# Logs: gpurun_out/${PREFIX}_<step>.log (+ a summary in gpurun_out/steps.log).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r03}
STEPS=${STEPS:-"probe tests bench extra"}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "gpurun_out/${P}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a gpurun_out/steps.log
  grep -v "amdgpu.ids" "gpurun_out/${P}_$name.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  # a Python exception from a GPU fault exits 1: nothing more on the GPU
  if grep -q -E "illegal memory access|hipErrorIllegalAddress|Memory access fault" "gpurun_out/${P}_$name.log"; then
    echo "ABORT after $name (GPU fault)"; exit 3
  fi
  return 0
}
for s in $STEPS; do
  case $s in
    probe) run probe 200 python -u scripts/debug/lp_probe.py ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    testsall) run testsall 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py --steps 20 --warmup 5 ;;
    benchq) run benchq 200 python bench.py --steps 50 --no-cpu-baseline ;;
    extra) run extra 400 python scripts/bench_extra.py --what mixed,tblocks,vtblocks,verify ;;
    mixed) run mixed 300 python scripts/bench_extra.py --what mixed ;;
    host) run host 400 python scripts/bench_extra.py --what sst,sstpin,host4k ;;
    long) run long 300 python scripts/long_span_probe.py ;;
    lpprof) run lpprof 300 python -u scripts/debug/lp_prof.py ${LPPROF_SHAPES:-headline tblocks bucket512 bucket1024 bucket2048 bucket65536} ;;
    autosplit) run autosplit 500 python -u scripts/autosplit_ab.py ;;
    balance) run balance 500 python -u scripts/balance_ab.py ${BAL_ROUNDS:-3} ;;
    balance_prof) run balance_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_balprof -o run --output-format csv -- python scripts/balance_ab.py 1 ;;
    cfg4) run cfg4 400 python bench.py --blocks 8388608 --steps 10 --warmup 5 ;;
    ab) run ab 900 bash scripts/gpu_abn.sh ${AB_ROUNDS:-2} ${AB_WHAT:-mixed,tblocks,vtblocks,verify} tree ${AB_LIBS:-build/ab/lib_r02.so} ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    pmc_fetch) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${P}_pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmc_write) run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${P}_pmc_write -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    bucket_pmc) run bucket_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${P}_bfetch -o run --output-format csv -- python3 scripts/bucket_traffic.py run &&
                run bucket_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${P}_bwrite -o run --output-format csv -- python3 scripts/bucket_traffic.py run &&
                python3 scripts/bucket_traffic.py summarize gpurun_out/${P}_bfetch gpurun_out/${P}_bwrite > gpurun_out/${P}_bucket_traffic.json; tail -40 gpurun_out/${P}_bucket_traffic.json ;;
    bucket_sq) run bucket_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d gpurun_out/${P}_bsq -o run --output-format csv -- python3 scripts/bucket_traffic.py run &&
                python3 scripts/bucket_traffic.py summarize_sq gpurun_out/${P}_bsq > gpurun_out/${P}_bucket_sq.json; tail -30 gpurun_out/${P}_bucket_sq.json ;;
    shape_sq) run shape_sq 600 bash scripts/pmc_shape_ab.sh tblocks tree &&
              run shape_sq_v 600 env KERNEL=verify bash scripts/pmc_shape_ab.sh vtblocks tree ;;
    pmc_sq) run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d gpurun_out/${P}_pmc_sq -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s" ;;
  esac
done
echo ALLDONE
