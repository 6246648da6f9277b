#!/bin/bash
# GPU box: wave-state and LDS counters of the spans kernel (two --pmc passes
# of 8 SQ counters each) on the headline and on SST-packed table blocks.
#   PREFIX=r04f bash scripts/pmc_state.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r04f}
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
B="SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS"
for set in A B; do
  ctr=${!set}
  for shape in head tblocks; do
    d=gpurun_out/${P}_pmc_${set}_${shape}
    if [ $shape = head ]; then
      timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $d.log 2>&1 || exit $?
    else
      timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d -o run --output-format csv -- python3 scripts/bench_extra.py --no-cpu --what tblocks > $d.log 2>&1 || exit $?
    fi
    python3 scripts/pmc_summary.py $d
  done
done
