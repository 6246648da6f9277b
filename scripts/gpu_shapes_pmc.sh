#!/bin/bash
# GPU box: span-shape probe (scripts/probe_shapes.py) timings, then one
# rocprofv3 --pmc pass over the same probe (dispatches are in shape order).
#   PMC="SQ_INSTS_VALU SQ_INSTS_SALU" bash scripts/gpu_shapes_pmc.sh [shape-substring]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${PMC:-FETCH_SIZE TCP_TCC_READ_REQ_sum}
timeout -k 10 300 python scripts/probe_shapes.py "$@" > gpurun_out/shapes.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/shapes_pmc -o run --output-format csv -- python3 scripts/probe_shapes.py "$@" > gpurun_out/shapes_pmc.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/shapes.log
