#!/bin/bash
# GPU box: LDS occupancy counters of the packed (stream-tiled) kernel vs the
# default spans kernel (scripts/packed_ab.py --only MODE): LDS-array cycles
# and bank-conflict cycles against the kernel's busy cycles, one rocprofv3
# --pmc pass per shape and mode.
#   PREFIX=r05j SHAPES="a4k tblocks b512" bash scripts/gpu_lds_pmc.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r05}
for s in ${SHAPES:-a4k tblocks b512}; do
  for m in default packed; do
    d=gpurun_out/${P}_lds_${s}_${m}
    timeout -k 10 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE -d $d -o run --output-format csv -- python3 scripts/packed_ab.py 1 $s --only $m > $d.log 2>&1
    rc=$?
    echo "== $s $m rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    k=$([ $m = packed ] && echo packed_kernel || echo spans_kernel)
    python3 scripts/pmc_summary.py $d --kernel $k
  done
done
echo ALLDONE
