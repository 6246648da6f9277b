#!/bin/bash
# GPU box: SQ instruction / wait counters of the headline kernel for the
# in-tree library and an alternative one (A/B of a kernel change).
#   bash scripts/pmc_ab.sh <alt .so> [counters...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=$1; shift
C=${*:-SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY}
for v in new alt; do
  if [ $v = alt ]; then export WIPDB_HCRC_LIB=$PWD/$ALT; else unset WIPDB_HCRC_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --precondition-ms 0 --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
