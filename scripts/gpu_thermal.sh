# Does the headline kernel slow down as the card warms?  Long launch series
# back to back, with the card's temperature / clocks / power sampled by
# rocm-smi while each series runs.
set -o pipefail
mkdir -p gpurun_out
for i in ${SERIES:-1 2 3 4}; do
  # rN: the read stream; NAME or NAME.k: the spans kernel of build/variants/NAME
  # (default: the in-tree build)
  v=${i%%.*}
  case $i in r*) W=readstream;; *) W=spans;; esac
  if [ $W = spans ] && [ -d build/variants/$v ]; then export WIPDB_HCRC_LIB=$PWD/build/variants/$v/libhip_crc32c_batch.so; else unset WIPDB_HCRC_LIB; fi
  timeout -k 10 120 python scripts/launch_series.py --launches ${LAUNCHES:-6000} --what $W > gpurun_out/th_$i.log 2>&1 &
  pid=$!
  : > gpurun_out/th_smi_$i.log
  for t in ${SAMPLES:-3 1 1 1 1}; do
    sleep $t
    (rocm-smi --showclocks --showpower 2>&1 || true) | grep -iE "sclk|fclk|mclk|Package Power" | grep -o '([0-9]*Mhz)\|: [0-9.]*$' | tr -d ' :()\n' >> gpurun_out/th_smi_$i.log
    echo -n " | " >> gpurun_out/th_smi_$i.log
  done
  wait $pid || { tail -5 gpurun_out/th_$i.log; exit 1; }
  echo "series $i ($W): $(grep -v amdgpu.ids gpurun_out/th_$i.log | grep -o '"per500": \[[0-9., ]*\]' | tr '\n' ' ')"
  echo "  smi: $(cat gpurun_out/th_smi_$i.log)"
done
