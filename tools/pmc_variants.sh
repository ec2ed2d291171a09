#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE; separate passes) of the standalone and
# header kernels for each build variant given (OURO_VERIFY_LIB swaps the
# product library), via bench.py --components-only.  Run under gpurun.
#   tools/pmc_variants.sh TAG lib1.so lib2.so ...
set -euo pipefail
TAG=$1; shift
ITEMS=${ITEMS:-262144}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    OURO_VERIFY_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --pmc $ctr --output-format csv \
      -d gpurun_out/vpmc_${TAG}_${name}_$ctr -o run \
      -- python3 bench.py --components-only --no-cpu --headers $ITEMS --steps 1 > /dev/null
  done
done
echo pmc-variants-done
