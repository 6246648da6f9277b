#!/bin/bash
# GPU box: the bench line as the driver runs it (twice), the ceiling test,
# and a rocprofv3 kernel trace of the driver's command with its K timed
# dispatches picked out (scripts/trace_timed.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r06b}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -2 | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "ABORT after $name"; exit $rc; fi
}
run ${P}_test_ceiling 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "dma_ceiling or readstream or full_size_4k" -m gpu
run ${P}_bench_a 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra
run ${P}_bench_b 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline
run ${P}_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline
run ${P}_prof_timed 60 python scripts/trace_timed.py gpurun_out/${P}_prof gpurun_out/${P}_prof.log
echo ALLDONE
