# Same-session A/B of kernel variants (build/variants/NAME, scripts/build_variant.sh):
#   bash scripts/gpu_ab.sh "default NAME ..." "4096 4092 ..."   [EXTRA=verify,mixed]
set -o pipefail
VARIANTS=${1:-default}
LENS=${2:-4096}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
for r in 1 2; do for v in $VARIANTS; do
  if [ $v = default ]; then unset WIPDB_HCRC_LIB; else export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; fi
  for L in $LENS; do
    timeout -k 10 200 python bench.py --steps 50 --warmup 30 --no-cpu-baseline --len $L > gpurun_out/bl.log 2>&1 || { tail -5 gpurun_out/bl.log; exit 1; }
    echo "$v len $L $(grep -o "\"kernel_avg_ms\": [0-9.]*" gpurun_out/bl.log)"
  done
  case ",$EXTRA," in *,verify,*)
    timeout -k 10 300 python scripts/bench_extra.py --what verify > gpurun_out/vf.txt 2>&1 || exit 1
    echo "$v verify $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/vf.txt)";; esac
  case ",$EXTRA," in *,tblocks,*)
    timeout -k 10 300 python scripts/bench_extra.py --what tblocks > gpurun_out/tb.txt 2>&1 || exit 1
    echo "$v tblocks $(grep '^{' gpurun_out/tb.txt | cut -c1-400)";; esac
  case ",$EXTRA," in *,vtblocks,*)
    timeout -k 10 300 python scripts/bench_extra.py --what vtblocks > gpurun_out/vtb.txt 2>&1 || exit 1
    echo "$v vtblocks $(grep '^{' gpurun_out/vtb.txt | cut -c1-400)";; esac
  case ",$EXTRA," in *,mixed,*)
    timeout -k 10 300 python scripts/bench_extra.py --what mixed > gpurun_out/mx.txt 2>&1 || exit 1
    echo "$v mixed $(python - <<'PY'
import json
for l in open("gpurun_out/mx.txt"):
    if l.startswith("{"):
        d = json.loads(l); print({k: v["GiBps"] for k, v in d["buckets"].items()}, d["mixed"]["GiBps"])
PY
)";; esac
done; done
