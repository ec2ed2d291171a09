#!/bin/bash
# Round-3 GPU pass (run under gpurun from the repo root).  Part "a": the GPU
# test suite, then the default bench.  Part "b": header-kernel and component
# rocprofv3 traces + PMC (tools/profile.sh, tools/profile_components.sh) and
# a kernel trace of the configs[4] plan.  Each step has its own time limit;
# the chain stops at the first failure.
set -euo pipefail
PART=$1
TAG=${2:-r03s}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$PART" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests-done
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  echo bench-done
else
  bash tools/profile.sh "$TAG" > gpurun_out/prof_$TAG.log 2>&1
  echo profile-done
  bash tools/profile_components.sh "$TAG" > gpurun_out/cprof_$TAG.log 2>&1
  echo components-done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof_$TAG -o run \
    -- python3 tools/ab_latency.py --libs ouroboros-network_amd/lib/libouro_verify.so --iters 2000 --rounds 1 \
    > gpurun_out/lprof_$TAG.json 2> gpurun_out/lprof_$TAG.err
  echo latency-profile-done
fi
