# GPU box: where does the spans kernel's per-launch overhead go?  Kernel ms
# per 1 M spans at 1 M / 4 M / 8 M blocks for the in-tree build and the
# load-only skeleton, plus the WIPDB_TIMELINE stamps at 1 M and 8 M.
#   scripts/build_variant.sh timeline -DWIPDB_TIMELINE=1
#   scripts/build_variant.sh loadonly -DWIPDB_LOADONLY=1
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-default loadonly}; do
  if [ $v = default ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; fi
  for B in ${BLOCKS:-1048576 4194304 8388608}; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --blocks $B ${BENCH_ARGS:-} > gpurun_out/lo.log 2>&1 || { tail -5 gpurun_out/lo.log; exit 1; }
    echo "$v blocks $B $(grep -o "\"kernel_avg_ms\": [0-9.]*" gpurun_out/lo.log)"
  done
done
if [ -z "${NO_TIMELINE:-}" ]; then
  export WIPDB_HCRC_LIB=$PWD/build/variants/timeline/libhip_crc32c_batch.so
  for B in 1048576 8388608; do
    timeout -k 10 200 python scripts/timeline_probe.py --blocks $B --reps 3 > gpurun_out/tl_$B.log 2>&1 || { tail -5 gpurun_out/tl_$B.log; exit 1; }
    echo "timeline $B"; grep '^{' gpurun_out/tl_$B.log | tail -1 | cut -c1-900
  done
fi
