#!/bin/bash
# GPU box: the round's evidence for the in-tree build -- headline bench with
# the CPU baseline (driver arguments and the default), rocprofv3 kernel-trace
# stats of the same command, the HBM traffic counters in separate passes
# (FETCH_SIZE, WRITE_SIZE), and the config-4 per-GPU shard (8 M x 4 KiB =
# 32 GiB).  Stops at the first failing GPU step.
#   PREFIX=r02 bash scripts/gpu_profile.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r02}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -2 | cut -c1-600
  if [ $rc -ne 0 ]; then echo "ABORT after $name"; exit $rc; fi
}
run ${P}_bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
run ${P}_bench 300 python bench.py --readstream --no-cpu-baseline
run ${P}_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline
run ${P}_pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${P}_pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --precondition-ms 0 --no-cpu-baseline
run ${P}_pmc_write 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${P}_pmc_write -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --precondition-ms 0 --no-cpu-baseline
# the stats average every dispatch (precondition and warmup too); this is
# the average of the 50 timed ones, as bench.py reports
run ${P}_prof_timed 60 python scripts/trace_tail.py gpurun_out/${P}_prof crc32c_lds_spans_kernel 50
run ${P}_cfg4_shard 300 python bench.py --blocks 8388608 --steps 10 --no-cpu-baseline
echo ALLDONE
