#!/bin/bash
# Build an experimental variant of the product library with extra kernel
# defines:  scripts/build_variant.sh NAME -DFOO=1 ...
# -> build/variants/NAME/libhip_crc32c_batch.so  (load it with WIPDB_HCRC_LIB)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
make -s -C "$ROOT/wipdb_amd/csrc" >/dev/null
OUT="$ROOT/build/variants/$NAME"
mkdir -p "$OUT"
# KSRC: another kernel source (e.g. a committed version) built against the
# in-tree headers
KSRC=${KSRC:-$ROOT/wipdb_amd/csrc/crc32c_kernels.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 "$@" \
  -I"$ROOT/wipdb_amd/csrc" -c -o "$OUT/crc32c_kernels.o" "$KSRC"
O="$ROOT/build/obj"
# the launcher sees the same knobs (block size, table window)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 "$@" \
  -I"$ROOT/wipdb_amd/csrc" -x hip -c -o "$OUT/hcrc_api.o" "$ROOT/wipdb_amd/csrc/hcrc_api.cc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libhip_crc32c_batch.so" \
  "$OUT/crc32c_kernels.o" "$OUT/hcrc_api.o" "$O/crc32c_api.o" "$O/crc32c_cpu.o" -lpthread
echo "$OUT/libhip_crc32c_batch.so"
