#!/bin/bash
# GPU box: PMC counters of the spans / verify kernel on one bench_extra shape
# for several builds (one --pmc pass per counter set and build).
#   KERNEL=spans_kernel bash scripts/pmc_shape_ab.sh tblocks tree build/ab/x/libhip_crc32c_batch.so
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
WHAT=$1
shift
K=${KERNEL:-spans_kernel}
A="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVES"
B="FETCH_SIZE"
C="WRITE_SIZE"
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
  for set in A B C; do
    d=gpurun_out/pmcshape_${WHAT}_${i}_${set}
    timeout -s KILL 150 rocprofv3 --pmc ${!set} -d $d -o run --output-format csv -- python3 scripts/bench_extra.py --no-cpu --what $WHAT > $d.log 2>&1 || exit $?
    echo "$v $set: $(python3 scripts/pmc_summary.py $d --kernel $K)"
  done
done
