cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in tree build/ab/lib_long48.so build/ab/lib_long32.so; do
  n=$(basename $v .so)
  if [ "$v" = tree ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/$v; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "split_long" -x -q --timeout 150 --timeout-method thread > gpurun_out/slt_$n.log 2>&1 || { tail -20 gpurun_out/slt_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/slt_$n.log)"
  timeout -k 10 300 python -u scripts/bench_extra.py --what mixed --split-long > gpurun_out/sl_$n.log 2>&1 || { tail -5 gpurun_out/sl_$n.log; exit 1; }
done
