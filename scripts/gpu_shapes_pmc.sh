#!/bin/bash
# GPU box: span-shape probe (scripts/probe_shapes.py) timings, then the HBM
# fetch counter per shape (dispatches are in shape order, 21 per shape).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/probe_shapes.py "$@" > gpurun_out/shapes.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum -d gpurun_out/shapes_pmc -o run --output-format csv -- python3 scripts/probe_shapes.py "$@" > gpurun_out/shapes_pmc.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/shapes.log
