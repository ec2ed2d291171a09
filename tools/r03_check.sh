#!/bin/bash
# One GPU-box pass of this round's development loop (run under gpurun from the
# repo root): the GPU test suite, then the component profile (TAG), then a
# short default bench.  Every step has its own time limit; the chain stops at
# the first failure.
set -euo pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
echo tests-done
if [ "${PROFILE:-1}" = 1 ]; then
  bash tools/profile_components.sh "$TAG" > gpurun_out/cprof_$TAG.log 2>&1
  echo profile-done
fi
timeout -k 10 600 python bench.py --steps 5 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench-done
