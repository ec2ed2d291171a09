#!/bin/bash
# Round-3 GPU pass A (run under gpurun from the repo root): the GPU test
# suite, a 2-rank strong-scaling rehearsal of bench.py on the one GPU (gloo:
# the ranks share the device), then the default bench.  Each step has its own
# time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
echo tests-done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  --dist-backend gloo --no-extras --no-latency --no-e2e --no-cpu \
  > gpurun_out/bench_2rank_$TAG.json 2> gpurun_out/bench_2rank_$TAG.err
echo rehearsal-done
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench-done
