#!/bin/bash
# GPU box: every secondary workload of scripts/bench_extra.py into
# gpurun_out/${PREFIX}_extra*.log (config 3 with and without the split,
# table blocks, read-side verify, config 5 SST stream, host 4 KiB blocks).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
P=${PREFIX:-r01}
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" python scripts/bench_extra.py "$@" > "gpurun_out/${P}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/${P}_$name.log"; exit $rc; fi
}
run extra 400 --what mixed,sst,host4k
run extra_split 300 --what mixed --split
run extra_blocks 300 --what tblocks,vtblocks,verify
echo ALLDONE
