#!/bin/bash
# GPU box: per-shape instruction counters (scripts/probe_shapes.py under one
# rocprofv3 --pmc pass) for several builds, summarised per span.
#   PMC="SQ_INSTS_SALU ..." [VERIFY=1] bash scripts/gpu_shapes_pmc_ab.sh tree build/ab/lib_head.so
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${PMC:-SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES}
i=0
V=""; K=spans_kernel
if [ -n "$VERIFY" ]; then V=--verify; K=verify_kernel; fi
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
  D=gpurun_out/pmc_ab_$i
  mkdir -p $D
  timeout -k 10 300 python scripts/probe_shapes.py $V > $D/shapes.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc $C -d $D/shapes_pmc -o run --output-format csv -- python3 scripts/probe_shapes.py $V > $D/pmc.log 2>&1 || exit $?
  echo "== $v"
  python scripts/shapes_pmc_summary.py $D $K
done
