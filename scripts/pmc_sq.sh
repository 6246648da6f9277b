#!/bin/bash
# GPU box: SQ/LDS counter passes (one rocprofv3 --pmc pass per set) of the
# headline bench and of the compute-only diagnostic (stride 0), summarised
# per launch of the CRC kernel by scripts/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-sq}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
n=0
for stride in 4096 0; do
  for set in "$P1" "$P2"; do
    n=$((n+1))
    d=gpurun_out/pmc_${TAG}_s${stride}_$n
    timeout -k 10 300 rocprofv3 --pmc $set -d $d -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --stride $stride > $d.log 2>&1
    rc=$?
    echo "pass $n stride $stride rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
  done
done
python3 scripts/pmc_summary.py gpurun_out pmc_${TAG}_
