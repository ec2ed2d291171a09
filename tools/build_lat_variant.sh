#!/bin/bash
# A/B variant of lib/libouro_verify.so that differs only in the latency-mode
# translation unit (kernels_lat.hip): the main build's kernels.o and pack.o
# (and host_path.o, numa.o, task_pool.o) are reused, kernels_lat.hip is compiled with the extra -D flags.
#   tools/build_lat_variant.sh NAME [-DFLAG=VALUE ...]
set -euo pipefail
cd "$(dirname "$0")/../ouroboros-network_amd"
NAME=$1; shift
B=build/variant_$NAME
mkdir -p "$B" lib/variants
test -f build/kernels.o -a -f build/pack.o -a -f build/host_path.o -a -f build/numa.o -a -f build/task_pool.o -a -f build/knobs.o -a -f build/byron_dlg.o || { echo "build the library first (make)"; exit 1; }
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" \
  -c -o "$B/kernels_lat.o" csrc/kernels_lat.hip
/opt/rocm/bin/hipcc --hip-link -shared -fPIC -o "lib/variants/$NAME.so" build/kernels.o "$B/kernels_lat.o" build/pack.o build/host_path.o build/numa.o build/task_pool.o build/knobs.o build/byron_dlg.o -lpthread
echo "lib/variants/$NAME.so"
