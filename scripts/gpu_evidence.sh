#!/bin/bash
# GPU box: the round's evidence for the in-tree build -- the bench line as
# the driver runs it, a rocprofv3 kernel trace of the same command with its
# K timed dispatches picked out, and the HBM traffic of every reported shape
# (separate FETCH_SIZE / WRITE_SIZE passes over scripts/shape_traffic.py).
#   PREFIX=r06g bash scripts/gpu_evidence.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r06g}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -2 | cut -c1-3000
  if [ $rc -ne 0 ]; then echo "ABORT after $name"; exit $rc; fi
}
run ${P}_bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run ${P}_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline
run ${P}_prof_timed 60 python scripts/trace_timed.py gpurun_out/${P}_prof gpurun_out/${P}_prof.log
run ${P}_pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${P}_pmc_fetch -o run --output-format csv -- python scripts/shape_traffic.py run
run ${P}_pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${P}_pmc_write -o run --output-format csv -- python scripts/shape_traffic.py run
run ${P}_traffic 60 python scripts/shape_traffic.py summarize gpurun_out/${P}_pmc_fetch gpurun_out/${P}_pmc_write gpurun_out/${P}_traffic.json
echo ALLDONE
