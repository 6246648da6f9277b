#!/bin/bash
# GPU box: one rocprofv3 --pmc pass over a command, counters from $PMC.
#   PMC="SQ_WAVES SQ_INSTS_VALU" bash scripts/pmc_run.sh NAME python3 scripts/bench_extra.py --what tblocks
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
NAME=$1; shift
C=${PMC:-SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY}
timeout -s KILL 150 rocprofv3 --pmc $C -d gpurun_out/$NAME -o run --output-format csv -- "$@" > gpurun_out/$NAME.log 2>&1
rc=$?; echo "$NAME rc=$rc"; exit $rc
