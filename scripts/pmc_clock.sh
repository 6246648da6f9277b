#!/bin/bash
# GPU box: effective shader clock of the spans kernel for several builds
# ("tree" or a library path): SQ_CYCLES / SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE
# and instruction counts in one --pmc pass per build; the dispatch times are
# in the same CSV (scripts/pmc_clock.py divides).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PREFIX:-r04k}
for v in "$@"; do
  tag=$(basename "$(dirname "$v")")
  [ "$v" = tree ] && tag=tree
  if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
  d=gpurun_out/${P}_clk_${tag}
  timeout -s KILL 120 rocprofv3 --pmc SQ_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $d -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $d.log 2>&1 || exit $?
  python3 scripts/pmc_clock.py $d
done
