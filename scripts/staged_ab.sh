#!/bin/bash
# GPU box: same-session A/B of library builds on host batches from PAGEABLE
# memory (staged through the pinned slots): 1 GiB of aligned 4 KiB blocks and
# 256 SSTs of the 8Binsert stream (scripts/bench_extra.py host4k, sst),
# builds alternating, order flipped every round.
#   bash scripts/staged_ab.sh ROUNDS tree build/ab/lib_x.so
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
ROUNDS=$1
shift
for r in $(seq 1 "$ROUNDS"); do
  if [ $((r % 2)) -eq 0 ]; then ORDER=$(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' '); else ORDER="$*"; fi
  for v in $ORDER; do
    if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
    timeout -k 10 120 python scripts/bench_extra.py --what host4k,sst --ssts 256 > gpurun_out/staged_ab.log 2>&1 || exit $?
    echo "round $r $v: $(grep -o '"GiBps_end_to_end": [0-9.]*\|"mismatches_in_sample": [0-9]*' gpurun_out/staged_ab.log | tr '\n' ' ')"
  done
done
