#!/bin/bash
# GPU box: SQ counters of the packed (stream-tiled) kernel vs the default
# spans kernel on a few shapes (scripts/packed_ab.py --only MODE), one
# rocprofv3 --pmc pass per shape and mode, then the per-kernel means.
#   PREFIX=r05d SHAPES="b65536 tblocks b1024" bash scripts/gpu_packed_pmc.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r05}
for s in ${SHAPES:-b65536 tblocks b1024}; do
  for m in default packed; do
    d=gpurun_out/${P}_pmc_${s}_${m}
    timeout -k 10 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d $d -o run --output-format csv -- python3 scripts/packed_ab.py 1 $s --only $m > $d.log 2>&1
    rc=$?
    echo "== $s $m rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    k=$([ $m = packed ] && echo packed_kernel || echo spans_kernel)
    python3 scripts/pmc_summary.py $d --kernel $k
  done
done
echo ALLDONE
