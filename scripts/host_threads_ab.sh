#!/bin/bash
# GPU box: host batches from PAGEABLE memory (staged through the pinned
# slots, the pack on the copy pool) with the pool's helper count varied
# (WIPDB_COPY_THREADS), orders rotated over rounds.
#   bash scripts/host_threads_ab.sh "3 7 15" ROUNDS
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
COUNTS=${1:-"3 7 15"}
ROUNDS=${2:-2}
for r in $(seq 1 "$ROUNDS"); do
  set -- $COUNTS
  if [ $((r % 2)) -eq 0 ]; then COUNTS_R=$(echo $COUNTS | tr ' ' '\n' | tac | tr '\n' ' '); else COUNTS_R=$COUNTS; fi
  for t in $COUNTS_R; do
    WIPDB_COPY_THREADS=$t timeout -k 10 120 python scripts/bench_extra.py --what host4k,sst --ssts 256 > gpurun_out/w_host.log 2>&1 || exit $?
    echo "round $r threads $t: $(grep -o '"GiBps_end_to_end": [0-9.]*' gpurun_out/w_host.log | tr '\n' ' ')"
  done
done
