# Same-session A/B of kernel variants without the test suite (diagnostic
# builds that give wrong results on purpose):
#   VARIANTS="default NAME" BLOCKS=1048576 ROUNDS=3 bash scripts/gpu_ab_quick.sh
set -o pipefail
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; fi
  timeout -k 10 200 python bench.py --blocks ${BLOCKS:-1048576} --steps 50 --warmup 30 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abq.log 2>&1 || { tail -5 gpurun_out/abq.log; exit 1; }
  echo "$v $(grep -o "\"kernel_avg_ms\": [0-9.]*" gpurun_out/abq.log)"
done; done
