#!/bin/bash
# GPU box: SQ instruction / wait counters of the headline bench for several
# builds (one rocprofv3 --pmc pass per build), summarised per launch of the
# spans kernel.  "tree" = the in-tree library, else a path to another build.
#   bash scripts/gpu_sq_ab.sh tree build/ab/lib_r02.so
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
SET="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for v in "$@"; do
  tag=$(basename "$v" .so)
  if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
  d=gpurun_out/sq_${tag}
  timeout -s KILL 120 rocprofv3 --pmc $SET -d $d -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  rc=$?
  echo "sq $v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
  python3 scripts/pmc_summary.py $d
done
