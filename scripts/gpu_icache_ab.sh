#!/bin/bash
# GPU box: instruction-cache counters (SQC) of the headline bench for several
# builds ("tree" = the in-tree library, else a path), one --pmc pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
SET=${SET:-"SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH"}
for v in "$@"; do
  tag=$(basename "$v" .so)
  if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
  d=gpurun_out/ic_${tag}
  timeout -s KILL 120 rocprofv3 --pmc $SET -d $d -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  rc=$?
  echo "icache $v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
  python3 scripts/pmc_summary.py $d
done
