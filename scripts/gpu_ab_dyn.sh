set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
for r in 1 2; do for v in default static; do
  if [ $v = default ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; fi
  for L in 4096 4092; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --len $L > gpurun_out/bl.log 2>&1 || { tail -5 gpurun_out/bl.log; exit 1; }
    echo "$v len $L $(grep -o "\"kernel_avg_ms\": [0-9.]*" gpurun_out/bl.log)"
  done
done; done
unset WIPDB_HCRC_LIB
timeout -k 10 300 python scripts/bench_extra.py --what verify > gpurun_out/vf3.txt 2>&1 || exit 1; echo "verify $(tail -1 gpurun_out/vf3.txt | cut -c1-200)"
WIPDB_HCRC_LIB=$PWD/build/variants/timeline/libhip_crc32c_batch.so timeout -k 10 200 python scripts/timeline_probe.py --reps 3 > gpurun_out/tl.txt 2>&1 || exit 1
cut -c1-900 gpurun_out/tl.txt | grep rep
