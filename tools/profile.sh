#!/bin/bash
# Profile the header kernel on the GPU box (run under gpurun from the repo root).
#   1. kernel trace + stats (per-kernel durations)           -> gpurun_out/prof_$TAG
#   2. HBM traffic counters, one pass each (FETCH_SIZE, WRITE_SIZE), per the
#      MI355X_MICROARCH.md HBM/rocprofv3 recipe                -> gpurun_out/pmc_*_$TAG
#   3. SQ instruction/cycle counters                          -> gpurun_out/pmc_sq_$TAG
#   4. SQ wait/issue-stall shares                             -> gpurun_out/pmc_wait_$TAG
# Every step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
HEADERS=${HEADERS:-262144}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --no-cpu --no-extras --no-latency --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- $B --steps 3 > gpurun_out/prof_$TAG.bench.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run \
  -- $B --steps 1 --warmup 0 --headers $HEADERS > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$TAG -o run \
  -- $B --steps 1 --warmup 0 --headers $HEADERS > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq_$TAG -o run \
  -- $B --steps 1 --warmup 0 --headers $HEADERS > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_wait_$TAG -o run \
  -- $B --steps 1 --warmup 0 --headers $HEADERS > /dev/null
echo profile-done
