#!/bin/bash
# Build an A/B variant of lib/libouro_verify.so with extra -D flags into
# lib/variants/NAME.so (tools/ab_variants.py, tools/ab_latency.py --libs).
#   tools/build_variant.sh NAME [-DFLAG=VALUE ...]
set -euo pipefail
cd "$(dirname "$0")/../ouroboros-network_amd"
NAME=$1; shift
B=build/variant_$NAME
mkdir -p "$B" lib/variants
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -c -o "$B/pack.o" csrc/pack.cpp
/opt/rocm/bin/hipcc $F -c -o "$B/kernels.o" csrc/kernels.hip &
/opt/rocm/bin/hipcc $F -c -o "$B/kernels_lat.o" csrc/kernels_lat.hip &
/opt/rocm/bin/hipcc --offload-host-only -O3 -std=c++17 -fPIC $* -c -o "$B/host_path.o" csrc/host_path.hip &
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c -o "$B/numa.o" csrc/numa.cpp &
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c -o "$B/task_pool.o" csrc/task_pool.cpp &
wait
/opt/rocm/bin/hipcc --hip-link -shared -fPIC -o "lib/variants/$NAME.so" "$B/kernels.o" "$B/kernels_lat.o" "$B/pack.o" "$B/host_path.o" "$B/numa.o" "$B/task_pool.o" build/knobs.o build/byron_dlg.o -lpthread
echo "lib/variants/$NAME.so"
