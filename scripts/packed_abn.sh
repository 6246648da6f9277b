#!/bin/bash
# GPU box: same-session A/B of library builds on the packed shapes
# (scripts/packed_ab.py --only packed, WIPDB_PS_ONLY=1), builds alternating
# within each round.  "tree" = the in-tree library, else a path to a build.
#   bash scripts/packed_abn.sh ROUNDS SHAPES tree build/ab/ps_prev/libhip_crc32c_batch.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
ROUNDS=$1
SHAPES=$2
shift 2
export WIPDB_PS_ONLY=1
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
    out=$(timeout -k 10 200 python3 scripts/packed_ab.py 1 "$SHAPES" --only packed 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "round $r $v: $(echo "$out" | grep -v '^{' | grep -o '^[a-z0-9]* {[^}]*packed_GiBps": [0-9.]*' | sed 's/ {.*packed_GiBps"://' | tr '\n' ' ')"
  done
done
